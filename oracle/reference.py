"""fp64 naive attention and the reference's accuracy gate.  TEST INFRASTRUCTURE ONLY.

Restates common/reference.py (tyler-utah/exploring_flash_attention):
  naive_attention  common/reference.py:7-21
  check_accuracy   common/reference.py:24-78
  print_comparison common/reference.py:81-96
"""
import numpy as np


def naive_attention(Q, K, V):
    """softmax(Q K^T / sqrt(d)) V with the row max subtracted (common/reference.py:7-21).

    The reference computes in the input dtype; this restatement upcasts to fp64 so it is
    an oracle for every storage type (for fp64 inputs the two are identical up to BLAS
    summation order).
    """
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    L, d = Q.shape
    scale = 1.0 / np.sqrt(d)
    scores = (Q @ K.T) * scale
    scores = scores - scores.max(axis=1, keepdims=True)
    probs = np.exp(scores)
    probs = probs / probs.sum(axis=1, keepdims=True)
    return probs @ V


def accuracy_metrics(output, reference):
    """The three metrics of check_accuracy (common/reference.py:42-69), as a dict."""
    output = np.asarray(output, dtype=np.float64)
    reference = np.asarray(reference, dtype=np.float64)
    diff = np.abs(output - reference)
    out = {"max_abs": float(diff.max()) if diff.size else 0.0,
           "max_rel": None, "mean_rel": None}
    mask = np.abs(reference) > 1e-3
    if mask.any():
        rel = diff[mask] / np.abs(reference[mask])
        out["max_rel"] = float(rel.max())
        out["mean_rel"] = float(rel.mean())
    return out


def check_accuracy(output, reference, config_str="", max_abs_tol=1e-2, max_rel_tol=0.5,
                   mean_rel_tol=0.05, verbose=False):
    """Raise AssertionError when any metric exceeds its tolerance (common/reference.py:24-78).

    Same defaults and the same three metrics as the reference: max |out - ref|; max and
    mean relative error over |ref| > 1e-3.  Returns the metrics dict.
    """
    m = accuracy_metrics(output, reference)
    errors = []
    if m["max_abs"] > max_abs_tol:
        errors.append(f"Max absolute difference {m['max_abs']:.6f} exceeds tolerance {max_abs_tol}")
    if m["max_rel"] is not None:
        if m["max_rel"] > max_rel_tol:
            errors.append(f"Max relative difference {m['max_rel']:.6f} exceeds tolerance {max_rel_tol}")
        if m["mean_rel"] > mean_rel_tol:
            errors.append(f"Mean relative error {m['mean_rel']:.6f} exceeds tolerance {mean_rel_tol}")
    if verbose:
        print(f"[{config_str}] {m}")
    if errors:
        raise AssertionError(f"Accuracy check failed: {'; '.join(errors)}")
    return m


def print_comparison(output, reference, num_rows=3, num_cols=5):
    """common/reference.py:81-96."""
    print("Output shape:", output.shape)
    print(f"First {num_rows} rows (output):")
    print(output[:num_rows, :num_cols])
    print(f"\nFirst {num_rows} rows (reference):")
    print(reference[:num_rows, :num_cols])
