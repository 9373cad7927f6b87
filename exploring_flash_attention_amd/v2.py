"""FA-v2 split-KV forward -- drop-in surfaces of the reference's flash_attention_v2.

Reference surfaces mirrored (tyler-utah/exploring_flash_attention):

* ``flash_attention_tiled_v2(Q, K, V, O, workspace_O, workspace_m, workspace_l, L, d,
  Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16, kv_tiles_per_block=1)``
      flash_attention_v2/numpy_gpu_like.py:343 (flat [L*d] buffers, O in place)
* ``flash_attention_v2(Q, K, V, O, B, H, L, d, d_tile_qk, d_tile_v, kv_tiles_per_block)``
  (alias ``flash_attention_v2_opt``)
      flash_attention_v2/CUDA/flash_attention_v2.h:438, flash_attention_v2_opt.h:559

Split size: the reference splits the keys into blocks of ``kv_tiles_per_block x Bk``
keys; the gfx950 kernel's KV tile is 64 keys, so a split here is
``kv_tiles_per_block x 64`` keys (KV_TILES_PER_BLOCK keeps its meaning: KV tiles per
partial workgroup).  The host workspace dicts of the NumPy surface are accepted for
signature compatibility and left untouched: the device workspace (normalised partial O
+ log-sum-exp per split) is owned by this call.
"""
import numpy as np

from . import _host, ops


def flash_attention_tiled_v2(Q, K, V, O, workspace_O, workspace_m, workspace_l, L, d, Bq=8, Bk=8,
                             d_tile_qk=16, d_tile_v=16, kv_tiles_per_block=1):
    assert kv_tiles_per_block > 0, "kv_tiles_per_block must be positive"
    assert Bq > 0 and Bk > 0 and 0 < d_tile_qk <= d and 0 < d_tile_v <= d
    q2, k2, v2 = (np.asarray(x).reshape(L, d) for x in (Q, K, V))
    dt = _host.compute_dtype(q2, k2, v2)
    q, k, v = _host.to_device((q2, k2, v2), dt)
    o = ops.attention_v2(q, k, v, kv_tiles_per_block, d_tile_qk, d_tile_v)
    O[:L * d] = _host.to_host(o, O.dtype).reshape(-1)


def flash_attention_v2(Q, K, V, O, B, H, L, d, d_tile_qk=32, d_tile_v=32, kv_tiles_per_block=4,
                       partial_dtype=None, workspace=None):
    """Device launcher surface (asynchronous; workspace from torch's caching allocator)."""
    assert B > 0 and H > 0 and L > 0 and d > 0, "All dimensions must be positive"
    assert tuple(Q.shape) == (B, H, L, d), f"Q shape {tuple(Q.shape)} != {(B, H, L, d)}"
    assert kv_tiles_per_block > 0, "kv_tiles_per_block must be positive"
    ops.attention_v2(Q, K, V, kv_tiles_per_block, d_tile_qk, d_tile_v, partial_dtype, out=O,
                     workspace=workspace)


flash_attention_v2_opt = flash_attention_v2
