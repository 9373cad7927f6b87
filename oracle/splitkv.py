"""FA-v2 split-KV forward on the CPU.  TEST INFRASTRUCTURE ONLY.

``flash_attention_tiled_v2`` restates flash_attention_v2/numpy_gpu_like.py:
  partial_attention_kernel  :174-226  (per (q_tile, kv_block): online softmax over
                                       kv_tiles_per_block KV tiles -> unnormalised O, m, l)
  reduction_kernel          :229-288  (M = max_k m_k; s_k = e^(m_k - M);
                                       O = sum s_k O_k / sum s_k l_k; scales are float32 :277)
  flash_attention_tiled_v2  :343-405  (workspaces are dicts keyed (q_tile, kv_block))

``partial_lse`` / ``combine_lse`` are the vectorised fp64 equivalents in the form the
GPU library uses (normalised partial O plus base-2 log-sum-exp of the scaled scores),
used to check ``fa_fwd_partial`` / ``fa_combine`` and the multi-GPU exchange.
"""
import numpy as np

from .tiled_d import _step


def _partial(Q, K, V, qt, kb, L, d, Bq, Bk, dtq, dtv, t0, t1, wO, wm, wl):
    q0 = qt * Bq
    q_len = min(Bq, L - q0)
    m = np.full(q_len, -np.inf, dtype=Q.dtype)
    l = np.zeros(q_len, dtype=Q.dtype)
    O_acc = np.zeros((q_len, d), dtype=Q.dtype)
    for t in range(t0, t1):
        k0 = t * Bk
        m, l, O_acc = _step(Q, K, V, q0, q_len, k0, min(Bk, L - k0), m, l, O_acc, dtq, dtv)
    wO[(qt, kb)] = O_acc.reshape(-1).copy()
    wm[(qt, kb)] = m.copy()
    wl[(qt, kb)] = l.copy()


def _reduce(wO, wm, wl, O, qt, nkb, L, d, Bq):
    q0 = qt * Bq
    q_len = min(Bq, L - q0)
    for i in range(q_len):
        M = max(wm[(qt, k)][i] for k in range(nkb))
        scales = np.array([np.exp(wm[(qt, k)][i] - M) for k in range(nkb)], dtype=np.float32)
        den = sum(wl[(qt, k)][i] * scales[k] for k in range(nkb))
        num = sum(wO[(qt, k)].reshape(q_len, d)[i] * scales[k] for k in range(nkb))
        O[(q0 + i) * d:(q0 + i + 1) * d] = num / den


def flash_attention_tiled_v2(Q, K, V, O, workspace_O, workspace_m, workspace_l, L, d,
                             Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16, kv_tiles_per_block=1):
    """Two-phase split-KV forward on flat [L*d] buffers, O written in place."""
    Q2, K2, V2 = (np.asarray(x).reshape(L, d) for x in (Q, K, V))
    nq = (L + Bq - 1) // Bq
    nkv = (L + Bk - 1) // Bk
    nkb = (nkv + kv_tiles_per_block - 1) // kv_tiles_per_block
    for qt in range(nq):
        for kb in range(nkb):
            t0 = kb * kv_tiles_per_block
            _partial(Q2, K2, V2, qt, kb, L, d, Bq, Bk, d_tile_qk, d_tile_v,
                     t0, min(t0 + kv_tiles_per_block, nkv), workspace_O, workspace_m, workspace_l)
    for qt in range(nq):
        _reduce(workspace_O, workspace_m, workspace_l, O, qt, nkb, L, d, Bq)


LOG2E = 1.4426950408889634


def partial_lse(Q, K, V):
    """One key range: (O_part [.., Lq, d] normalised, lse [.., Lq] base 2 of scaled scores).

    Q [..., Lq, d], K/V [..., Lk, d]; computed in fp64.
    """
    Q = np.asarray(Q, np.float64)
    K = np.asarray(K, np.float64)
    V = np.asarray(V, np.float64)
    d = Q.shape[-1]
    s = np.einsum("...qd,...kd->...qk", Q, K) * (LOG2E / np.sqrt(d))
    mx = s.max(axis=-1, keepdims=True)
    p = np.exp2(s - mx)
    den = p.sum(axis=-1, keepdims=True)
    O = np.einsum("...qk,...kd->...qd", p, V) / den
    return O, (mx + np.log2(den))[..., 0]


def combine_lse(O_parts, lses):
    """Combine partials [S, ..., L, d] / [S, ..., L] -> O [..., L, d] (fp64)."""
    O_parts = np.asarray(O_parts, np.float64)
    lses = np.asarray(lses, np.float64)
    M = lses.max(axis=0)
    w = np.exp2(lses - M)
    return (w[..., None] * O_parts).sum(axis=0) / w.sum(axis=0)[..., None]
