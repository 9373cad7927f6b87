"""FA-v1 d-tiled forward -- drop-in surfaces of the reference's flash_attention_v1_tiled_d.

Reference surfaces mirrored (tyler-utah/exploring_flash_attention):

* ``flash_attention_tiled_global(Q, K, V, Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16) -> O``
      flash_attention_v1_tiled_d/numpy_basic.py:99, with its argument asserts (:112-120)
      raising AssertionError exactly as the reference does
* ``flash_attention_tiled(Q, K, V, O, L, d, Bq, Bk, d_tile_qk, d_tile_v)``
      flash_attention_v1_tiled_d/numpy_gpu_like.py:224 (flat buffers, O in place)
* ``flash_attention_v1_tiled_d(Q, K, V, O, B, H, L, d, d_tile_qk, d_tile_v)`` (alias
  ``flash_attention_v1_opt``)
      flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:312, flash_attention_v1_opt.h:448

The d-tile arguments are validated like the reference's (0 < d_tile <= d).  For d <= 256 one
LDS tile holds a whole row and the fused kernel runs (its QK^T accumulates 32-column MFMA
k-steps, O_acc stays in VGPRs), the tiles not changing the result; for 256 < d <= 512 the
d-tiled kernel (csrc/fa_fwd_dtiled.hip) streams K and V through LDS in d_tile-wide column
chunks (rounded down to 32, 64 or 128 columns), O_acc in VGPRs for all d columns -- the case
the reference's variant exists for.
"""
import numpy as np

from . import _host, ops


def _check_args(Q, K, V, Bq, Bk, d_tile_qk, d_tile_v):
    assert Q.shape == K.shape == V.shape, "Q, K, V must have the same shape [L, d]"
    L, d = Q.shape[-2], Q.shape[-1]
    assert L > 0 and d > 0
    assert isinstance(Bq, (int, np.integer)) and Bq > 0
    assert isinstance(Bk, (int, np.integer)) and Bk > 0
    assert isinstance(d_tile_qk, (int, np.integer)) and d_tile_qk > 0
    assert isinstance(d_tile_v, (int, np.integer)) and d_tile_v > 0
    assert d_tile_qk <= d and d_tile_v <= d


def flash_attention_tiled_global(Q, K, V, Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16):
    """Q,K,V [L, d] (host arrays or device tensors) -> O [L, d]."""
    if _host.is_device_tensor(Q):
        _check_args(Q, K, V, Bq, Bk, d_tile_qk, d_tile_v)
        if Q.dim() == 2:
            return ops.attention_tiled_d(Q[None, None], K[None, None], V[None, None],
                                         d_tile_qk, d_tile_v)[0, 0]
        return ops.attention_tiled_d(Q, K, V, d_tile_qk, d_tile_v)
    Q, K, V = (np.asarray(x) for x in (Q, K, V))
    _check_args(Q, K, V, Bq, Bk, d_tile_qk, d_tile_v)
    dt = _host.compute_dtype(Q, K, V)
    q, k, v = _host.to_device((Q, K, V), dt)
    return _host.to_host(ops.attention_tiled_d(q, k, v, d_tile_qk, d_tile_v), Q.dtype)


def flash_attention_tiled(Q, K, V, O, L, d, Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16):
    """Flat-buffer surface: O[:L*d] = attention(Q, K, V) (reshaped [L, d])."""
    q2, k2, v2 = (np.asarray(x).reshape(L, d) for x in (Q, K, V))
    O[:L * d] = flash_attention_tiled_global(q2, k2, v2, Bq, Bk, d_tile_qk, d_tile_v).reshape(-1)


def flash_attention_v1_tiled_d(Q, K, V, O=None, B=None, H=None, L=None, d=None, d_tile_qk=32,
                               d_tile_v=32):
    """``flash_attention_v1_tiled_d(Q, K, V, d_tile_qk=32, d_tile_v=32) -> O`` (host or
    device), or the launcher form ``(Q, K, V, O, B, H, L, d, d_tile_qk, d_tile_v)``
    (asynchronous on the current stream)."""
    if O is None:
        dd = int(Q.shape[-1])
        assert 0 < d_tile_qk <= dd and 0 < d_tile_v <= dd, "d_tile must be valid"
        return _host.run_qkv(lambda q, k, v: ops.attention_tiled_d(q, k, v, d_tile_qk, d_tile_v),
                             Q, K, V)
    assert B > 0 and H > 0 and L > 0 and d > 0, "All dimensions must be positive"
    assert tuple(Q.shape) == (B, H, L, d), f"Q shape {tuple(Q.shape)} != {(B, H, L, d)}"
    assert 0 < d_tile_qk <= d and 0 < d_tile_v <= d, "d_tile must be valid"
    ops.attention_tiled_d(Q, K, V, d_tile_qk, d_tile_v, out=O)


flash_attention_v1_opt = flash_attention_v1_tiled_d
