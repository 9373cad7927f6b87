"""FA-v1 tiled forward on the CPU.  TEST INFRASTRUCTURE ONLY (checker + CPU baseline).

Two restatements of the reference's FA-v1 algorithm:

* ``flash_attention_tiled`` -- the high-level NumPy form,
  flash_attention_v1/numpy_basic.py:69-105 (tile step :7-66).
* ``flash_attention_tiled_flat`` -- the fused, C-style form with flat row-major buffers
  and explicit element loops, flash_attention_v1/numpy_gpu_like_opt2.py:198-241
  (tile step :135-195, helpers :7-133).  It keeps the reference's loop structure on
  purpose: bench.py times it as the CPU baseline the north_star names ("the repo's own
  numpy_gpu_like_opt2.py CPU path"), so it must cost what that path costs.
"""
import numpy as np


# ---------------------------------------------------------------------------
# numpy_basic.py form
# ---------------------------------------------------------------------------

def _process_kv_tile(Q_tile, K_tile, V_tile, m, l, O_acc):
    """flash_attention_v1/numpy_basic.py:7-66: one online-softmax step."""
    d = Q_tile.shape[1]
    S = (Q_tile @ K_tile.T) / np.sqrt(d)
    m_new = np.maximum(m, S.max(axis=1))
    alpha = np.exp(m - m_new)
    P = np.exp(S - m_new[:, None])
    l_new = l * alpha + P.sum(axis=1)
    O_new = O_acc * alpha[:, None] + P @ V_tile
    return m_new, l_new, O_new


def flash_attention_tiled(Q, K, V, Bq=8, Bk=8):
    """FA-v1 forward, Q,K,V [L,d] -> O [L,d] in the input dtype
    (flash_attention_v1/numpy_basic.py:69-105)."""
    L, d = Q.shape
    O = np.zeros((L, d), dtype=Q.dtype)
    for q_start in range(0, L, Bq):
        q_end = min(q_start + Bq, L)
        Q_tile = Q[q_start:q_end]
        q_len = q_end - q_start
        m = np.full(q_len, -np.inf, dtype=Q.dtype)
        l = np.zeros(q_len, dtype=Q.dtype)
        O_acc = np.zeros((q_len, d), dtype=Q.dtype)
        for k_start in range(0, L, Bk):
            k_end = min(k_start + Bk, L)
            m, l, O_acc = _process_kv_tile(Q_tile, K[k_start:k_end], V[k_start:k_end], m, l, O_acc)
        O[q_start:q_end] = O_acc / l[:, None]
    return O


# ---------------------------------------------------------------------------
# numpy_gpu_like_opt2.py form (flat buffers, fused in-place steps, element loops)
# ---------------------------------------------------------------------------

def _idx2d(i, j, cols):
    return i * cols + j


def _mat_mul_scaled(A, B, C, b, m, n, k):
    """C = A @ B^T * b on flat buffers (numpy_gpu_like_opt2.py:14-33)."""
    C[:m * n] = ((A[:m * k].reshape(m, k) @ B[:n * k].reshape(n, k).T) * b).ravel()


def _mat_scale_rows_mul_add(A, v, B, C, m, n, k):
    """A = A * v[:, None] + B @ C (numpy_gpu_like_opt2.py:35-63), same loop order."""
    for i in range(m):
        for j in range(n):
            A[_idx2d(i, j, n)] = A[_idx2d(i, j, n)] * v[i]
    result = B[:m * k].reshape(m, k) @ C[:k * n].reshape(k, n)
    for i in range(m):
        for j in range(n):
            A[_idx2d(i, j, n)] += result[i, j]


def _mat_sub_vec_exp(S, v, out, m, n):
    """out[i,j] = exp(S[i,j] - v[i]) (numpy_gpu_like_opt2.py:65-80)."""
    for i in range(m):
        for j in range(n):
            idx = _idx2d(i, j, n)
            out[idx] = np.exp(S[idx] - v[i])


def _mat_div_vec_store(A, v, out, out_row_offset, m, n):
    """out[row0+i, j] = A[i,j] / v[i] (numpy_gpu_like_opt2.py:82-97)."""
    for i in range(m):
        for j in range(n):
            out[_idx2d(out_row_offset + i, j, n)] = A[_idx2d(i, j, n)] / v[i]


def _row_sum_mul_add_inplace(S, l, alpha, m, n):
    """l[i] = l[i]*alpha[i] + sum_j S[i,j] (numpy_gpu_like_opt2.py:99-116)."""
    for i in range(m):
        acc = 0.0
        for j in range(n):
            acc += S[_idx2d(i, j, n)]
        l[i] = l[i] * alpha[i] + acc


def _load_tile(src, tile, start, end, d):
    """Row copy into a flat tile buffer (numpy_gpu_like_opt2.py:118-133)."""
    for i in range(end - start):
        for j in range(d):
            tile[_idx2d(i, j, d)] = src[_idx2d(start + i, j, d)]


def _process_kv_tile_flat(Q_tile, K_tile, V_tile, m, l, O_acc, bq, bk, d):
    """numpy_gpu_like_opt2.py:135-195: scores -> max/alpha -> exp -> l -> O, in place."""
    inv_sqrt_d = 1.0 / np.sqrt(d)
    S = np.empty(bq * bk, dtype=Q_tile.dtype)
    alpha = np.empty(bq, dtype=Q_tile.dtype)
    _mat_mul_scaled(Q_tile, K_tile, S, inv_sqrt_d, bq, bk, d)
    for i in range(bq):
        new_max = m[i]
        for j in range(bk):
            if S[_idx2d(i, j, bk)] > new_max:
                new_max = S[_idx2d(i, j, bk)]
        alpha[i] = np.exp(m[i] - new_max)
        m[i] = new_max
    _mat_sub_vec_exp(S, m, S, bq, bk)
    _row_sum_mul_add_inplace(S, l, alpha, bq, bk)
    _mat_scale_rows_mul_add(O_acc, alpha, S, V_tile, bq, d, bk)


def flash_attention_tiled_flat(Q, K, V, O, L, d, Bq=8, Bk=8):
    """FA-v1 forward on flat [L*d] buffers, writing O in place
    (flash_attention_v1/numpy_gpu_like_opt2.py:198-241)."""
    for q_start in range(0, L, Bq):
        q_end = min(q_start + Bq, L)
        q_len = q_end - q_start
        Q_tile = np.empty(Bq * d, dtype=Q.dtype)
        _load_tile(Q, Q_tile, q_start, q_end, d)
        m = np.full(Bq, -np.inf, dtype=Q.dtype)
        l = np.zeros(Bq, dtype=Q.dtype)
        O_acc = np.zeros(Bq * d, dtype=Q.dtype)
        for k_start in range(0, L, Bk):
            k_end = min(k_start + Bk, L)
            K_tile = np.empty(Bk * d, dtype=K.dtype)
            V_tile = np.empty(Bk * d, dtype=V.dtype)
            _load_tile(K, K_tile, k_start, k_end, d)
            _load_tile(V, V_tile, k_start, k_end, d)
            _process_kv_tile_flat(Q_tile, K_tile, V_tile, m, l, O_acc, q_len, k_end - k_start, d)
        _mat_div_vec_store(O_acc, l, O, q_start, q_len, d)
