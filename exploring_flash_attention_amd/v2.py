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


def flash_attention_v2(Q, K, V, O=None, B=None, H=None, L=None, d=None, d_tile_qk=32,
                       d_tile_v=32, kv_tiles_per_block=4, partial_dtype=None, workspace=None,
                       world_size=1, group=None):
    """``flash_attention_v2(Q, K, V, kv_tiles_per_block=4, world_size=1) -> O`` (host or
    device), or the launcher form ``(Q, K, V, O, B, H, L, d, d_tile_qk, d_tile_v,
    kv_tiles_per_block)`` (asynchronous; workspace from torch's caching allocator).

    ``world_size > 1`` (device tensors, torch.distributed initialised, one process per GPU):
    every rank passes the full Q, K, V; rank r keeps keys [r*L/W, (r+1)*L/W) and the
    split-KV partials are combined across ranks (dist.splitkv_attention); every rank
    returns the full O.
    """
    assert kv_tiles_per_block > 0, "kv_tiles_per_block must be positive"
    if O is None:
        if world_size > 1:
            return _v2_dist(Q, K, V, world_size, group, partial_dtype)
        return _host.run_qkv(lambda q, k, v: ops.attention_v2(q, k, v, kv_tiles_per_block, d_tile_qk,
                                                              d_tile_v, partial_dtype),
                             Q, K, V)
    assert B > 0 and H > 0 and L > 0 and d > 0, "All dimensions must be positive"
    assert tuple(Q.shape) == (B, H, L, d), f"Q shape {tuple(Q.shape)} != {(B, H, L, d)}"
    assert kv_tiles_per_block > 0, "kv_tiles_per_block must be positive"
    ops.attention_v2(Q, K, V, kv_tiles_per_block, d_tile_qk, d_tile_v, partial_dtype, out=O,
                     workspace=workspace)


def _v2_dist(Q, K, V, world_size, group, partial_dtype):
    import torch.distributed as tdist

    from . import dist as fadist
    import torch
    assert isinstance(Q, torch.Tensor) and Q.dim() == 4, \
        "world_size > 1 takes [B, H, L, d] device tensors (one process per GPU)"
    W = tdist.get_world_size(group)
    assert W == world_size, f"world_size={world_size} but the process group has {W} ranks"
    rank = tdist.get_rank(group)
    lo, hi = fadist.shard_bounds(Q.shape[2], W, rank)
    # partial_dtype None: splitkv_attention's default (per-row scaled fp16, fp64 for fp64
    # inputs) -- the same exchange format as every other multi-GPU entry point
    return fadist.splitkv_attention(Q, K[:, :, lo:hi].contiguous(), V[:, :, lo:hi].contiguous(),
                                    group=group, gather=True, partial_dtype=partial_dtype)


flash_attention_v2_opt = flash_attention_v2
