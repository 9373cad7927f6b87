"""d-tiled FA-v1 forward on the CPU.  TEST INFRASTRUCTURE ONLY.

Restates flash_attention_v1_tiled_d/numpy_basic.py:
  process_kv_tile_global       :13-96   (S accumulated over d_tile_qk column chunks,
                                         P@V accumulated per d_tile_v column chunk)
  flash_attention_tiled_global :99-151  (argument asserts :112-120)
"""
import numpy as np


def _step(Q, K, V, q0, q_len, k0, k_len, m, l, O_acc, d_tile_qk, d_tile_v):
    d = Q.shape[1]
    S = np.zeros((q_len, k_len), dtype=Q.dtype)
    for c0 in range(0, d, d_tile_qk):
        c1 = min(c0 + d_tile_qk, d)
        S += Q[q0:q0 + q_len, c0:c1] @ K[k0:k0 + k_len, c0:c1].T
    S *= 1.0 / np.sqrt(d)
    m_new = np.maximum(m, S.max(axis=1))
    alpha = np.exp(m - m_new)
    P = np.exp(S - m_new[:, None])
    l_new = l * alpha + P.sum(axis=1)
    O_acc = O_acc * alpha[:, None]
    for c0 in range(0, d, d_tile_v):
        c1 = min(c0 + d_tile_v, d)
        O_acc[:, c0:c1] += P @ V[k0:k0 + k_len, c0:c1]
    return m_new, l_new, O_acc


def flash_attention_tiled_global(Q, K, V, Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16):
    """Q,K,V [L,d] -> O [L,d] (flash_attention_v1_tiled_d/numpy_basic.py:99-151)."""
    assert Q.shape == K.shape == V.shape, "Q, K, V must have the same shape [L, d]"
    L, d = Q.shape
    assert L > 0 and d > 0
    for name, val in (("Bq", Bq), ("Bk", Bk), ("d_tile_qk", d_tile_qk), ("d_tile_v", d_tile_v)):
        assert isinstance(val, int) and val > 0, name
    assert d_tile_qk <= d and d_tile_v <= d
    O = np.zeros((L, d), dtype=Q.dtype)
    for q0 in range(0, L, Bq):
        q_len = min(Bq, L - q0)
        m = np.full(q_len, -np.inf, dtype=Q.dtype)
        l = np.zeros(q_len, dtype=Q.dtype)
        O_acc = np.zeros((q_len, d), dtype=Q.dtype)
        for k0 in range(0, L, Bk):
            m, l, O_acc = _step(Q, K, V, q0, q_len, k0, min(Bk, L - k0), m, l, O_acc,
                                d_tile_qk, d_tile_v)
        O[q0:q0 + q_len] = O_acc / l[:, None]
    return O
