"""Host-array plumbing for the reference's NumPy call surfaces.

The reference's Python functions take host ``[L, d]`` (or flat ``[L*d]``) NumPy arrays.  The
drop-in versions accept those too: the arrays are copied to the current ROCm device as
``[1, 1, L, d]``, the gfx950 kernel runs, and the result is copied back in the caller's
dtype.  torch device tensors pass through without copies.

Compute dtype for host arrays, following the reference, whose NumPy functions compute in
the input dtype: float16 inputs run the fp16 kernels (fp32 accumulation); float32 and
float64 inputs run the fp64 kernels (the reference's USE_FP64 build: fp64 MFMA and softmax),
so the host surfaces reproduce the reference's fp64 outputs to ~1e-15.  The PCIe copies
are part of these host surfaces only; bench.py times device-resident bf16 tensors.
"""
import numpy as np
import torch



def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("exploring_flash_attention_amd needs a ROCm GPU (MI355X / gfx950); "
                           "there is no CPU fallback")


def compute_dtype(*arrays):
    if all(a.dtype == np.float16 for a in arrays):
        return torch.float16
    return torch.float64


def to_device(arrays, dtype):
    """Host [L, d] (or [B, H, L, d]) arrays -> contiguous [B, H, L, d] device tensors."""
    require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    out = []
    for a in arrays:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64 if dtype == torch.float64
                                                  else np.float32))
        t = t.to(device=dev, dtype=dtype, non_blocking=False)
        out.append((t[None, None] if t.dim() == 2 else t).contiguous())
    return out


def to_host(t, like_dtype, ndim=2):
    """[B, H, L, d] device tensor -> host array of like_dtype ([L, d] when ndim == 2)."""
    t = t[0, 0] if ndim == 2 else t
    t = t if t.dtype == torch.float64 else t.float()
    return t.cpu().numpy().astype(like_dtype, copy=False)


def run_qkv(fn, Q, K, V):
    """Apply ``fn(q, k, v) -> o`` (device [B, H, L, d] tensors) to any of the accepted forms:

    * torch device tensors, [B, H, L, d] or [L, d] (zero-copy; result on the device);
    * host NumPy arrays (or anything ``np.asarray`` takes), [L, d] or [B, H, L, d]
      (copied in and out; result in Q's dtype, float64 for non-float input).
    """
    if is_device_tensor(Q):
        if Q.dim() == 2:
            return fn(Q[None, None].contiguous(), K[None, None].contiguous(),
                      V[None, None].contiguous())[0, 0]
        return fn(Q, K, V)
    Q, K, V = (np.asarray(x) for x in (Q, K, V))
    assert Q.ndim in (2, 4), f"Q must be [L, d] or [B, H, L, d], got shape {Q.shape}"
    assert K.ndim == Q.ndim and V.ndim == Q.ndim, "Q, K, V must have the same rank"
    like = Q.dtype if np.issubdtype(Q.dtype, np.floating) else np.float64
    q, k, v = to_device((Q, K, V), compute_dtype(Q, K, V))
    return to_host(fn(q, k, v), like, Q.ndim)


def is_device_tensor(x):
    return isinstance(x, torch.Tensor) and x.device.type == "cuda"
