"""Vectorised fp64 attention over [B, H, L, d].  TEST INFRASTRUCTURE ONLY.

The same maths as naive_attention (common/reference.py:7-21) applied per (b, h), with the
score matrix built in query chunks so large L fits in host memory.  Used to check the GPU
kernels on full tensors.
"""
import numpy as np


def attention_fp64(Q, K, V, q_chunk=1024):
    """Q [..., Lq, d], K/V [..., Lk, d] -> O [..., Lq, d] in fp64."""
    Q = np.asarray(Q, np.float64)
    K = np.asarray(K, np.float64)
    V = np.asarray(V, np.float64)
    d = Q.shape[-1]
    out = np.empty(Q.shape, np.float64)
    scale = 1.0 / np.sqrt(d)
    Kt = np.swapaxes(K, -1, -2)
    for q0 in range(0, Q.shape[-2], q_chunk):
        s = (Q[..., q0:q0 + q_chunk, :] @ Kt) * scale
        s -= s.max(axis=-1, keepdims=True)
        p = np.exp(s)
        p /= p.sum(axis=-1, keepdims=True)
        out[..., q0:q0 + q_chunk, :] = p @ V
    return out
