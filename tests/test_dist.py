"""Multi-rank split-KV exchange on CPU: world_size 2 and 4 over gloo.

The per-rank kernels need a GPU, so here dist._partial_fn / dist._combine_fn are replaced
by the fp64 oracle (oracle.splitkv) computing the SAME layouts the HIP kernels write:
o_part [W, B*H, L/W, d] (send layout: chunk j goes to rank j) and lse [W, B*H, L/W].
What is under test is the product's exchange logic: chunking, the all_to_all_single
pairing, the combine of the received partials and the final all_gather.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.batched import attention_fp64
from oracle.splitkv import combine_lse, partial_lse


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_partial(q, k, v, chunk_rows, partial_dtype):
    """The kernel's layouts; for ops.PARTIAL_FP16_SCALED (include/fa_mi355x.h) the rows are
    fp16 O * 2^-e with e = frexp exponent of the row's max |O|, lse [..., 2] = {lse, e}."""
    B, H, Lq, d = q.shape
    O, lse = partial_lse(q.double().numpy(), k.double().numpy(), v.double().numpy())
    nch = Lq // chunk_rows
    O = O.reshape(B * H, nch, chunk_rows, d).transpose(1, 0, 2, 3)
    lse = lse.reshape(B * H, nch, chunk_rows).transpose(1, 0, 2)
    if partial_dtype == "fp16_scaled":
        e = np.frexp(np.abs(O).max(axis=-1))[1].astype(np.float64)
        O = np.ldexp(O, -e[..., None].astype(np.int64)).astype(np.float16)
        lse = np.stack([lse, e], axis=-1)
        return torch.from_numpy(np.ascontiguousarray(O)), torch.from_numpy(np.ascontiguousarray(lse)).float()
    return (torch.from_numpy(np.ascontiguousarray(O)).to(partial_dtype),
            torch.from_numpy(np.ascontiguousarray(lse)).float())


def _oracle_combine(o_part, lse, B, H, dtype):
    S, BH, L, d = o_part.shape
    O, lse = o_part.double().numpy(), lse.double().numpy()
    if lse.ndim == 4:  # scaled fp16 partials: undo 2^-e
        O = np.ldexp(O, lse[..., 1:].astype(np.int64))
        lse = lse[..., 0]
    O = combine_lse(O, lse)
    return torch.from_numpy(O.reshape(B, H, L, d)).to(dtype)


def _oracle_partial_chunk(q_rows, k, v, o_out, lse_out, partial_dtype):
    """The chunked partial of the overlapped path: same layouts as the kernel writes."""
    assert not q_rows.is_contiguous() or q_rows.shape[2] == q_rows.stride(1) // q_rows.shape[3]
    o, lse = _oracle_partial(q_rows.contiguous(), k, v, q_rows.shape[2], partial_dtype)
    o_out.copy_(o[0])
    lse_out.copy_(lse[0].to(lse_out.dtype))


def _worker(rank, world, port, result_path, overlap, pdtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exploring_flash_attention_amd import dist as fdist
    fdist._partial_fn = _oracle_partial
    fdist._combine_fn = _oracle_combine
    fdist._partial_chunk_fn = _oracle_partial_chunk
    g = torch.Generator().manual_seed(0)
    B, H, L, d = 2, 3, 64, 32
    q, k, v = (torch.randn(B, H, L, d, generator=g, dtype=torch.float64) for _ in range(3))
    lo, hi = fdist.shard_bounds(L, world, rank)
    local = fdist.splitkv_attention(q, k[:, :, lo:hi].contiguous(), v[:, :, lo:hi].contiguous(),
                                    partial_dtype=pdtype, overlap=overlap)
    full = fdist.splitkv_attention(q, k[:, :, lo:hi].contiguous(), v[:, :, lo:hi].contiguous(),
                                   partial_dtype=pdtype, gather=True, overlap=overlap)
    ref = attention_fp64(q.numpy(), k.numpy(), v.numpy())
    err_local = np.abs(local.numpy() - ref[:, :, lo:hi]).max()
    err_full = np.abs(full.numpy() - ref).max()
    with open(f"{result_path}.{rank}", "w") as f:
        f.write(f"{err_local} {err_full} {tuple(local.shape)} {tuple(full.shape)}")
    dist.destroy_process_group()


@pytest.mark.parametrize("pdtype", [torch.float64, "fp16_scaled"], ids=["p64", "pf16s"])
@pytest.mark.parametrize("overlap", [False, True], ids=["all_to_all", "overlapped"])
@pytest.mark.parametrize("world", [2, 4])
def test_splitkv_exchange_gloo(tmp_path, world, overlap, pdtype):
    port = _free_port()
    path = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, port, path, overlap, pdtype), nprocs=world, join=True,
                       start_method="spawn")
    # fp32 lse as on the GPU; scaled fp16 rows: 2^-11 relative to each row's max (|O| < 4 here)
    tol = 1e-6 if pdtype == torch.float64 else 4 * 2.0 ** -11
    for r in range(world):
        err_local, err_full, *_ = open(f"{path}.{r}").read().split(" ", 2)
        assert float(err_local) < tol and float(err_full) < tol


def test_shard_bounds():
    from exploring_flash_attention_amd.dist import shard_bounds
    assert [shard_bounds(16384, 8, r) for r in (0, 7)] == [(0, 2048), (14336, 16384)]
    with pytest.raises(ValueError):
        shard_bounds(100, 8, 0)


def _surface_worker(rank, world, port, result_path):
    """The public surface flash_attention_v2(Q, K, V, world_size=W) (v2.py): every rank passes
    the full Q, K, V and gets the full O; kernels replaced by the oracle as above."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exploring_flash_attention_amd import dist as fdist
    from exploring_flash_attention_amd import v2
    fdist._partial_fn = _oracle_partial
    fdist._combine_fn = _oracle_combine
    fdist._partial_chunk_fn = _oracle_partial_chunk
    seen = []
    orig = fdist.splitkv_attention

    def spy(*a, **kw):
        seen.append(kw.get("partial_dtype"))
        return orig(*a, **kw)
    fdist.splitkv_attention = spy
    g = torch.Generator().manual_seed(5)
    B, H, L, d = 2, 2, 96, 32
    errs = []
    for dtype in (torch.float64, torch.float32):
        q, k, v = (torch.randn(B, H, L, d, generator=g, dtype=dtype) for _ in range(3))
        o = v2.flash_attention_v2(q, k, v, world_size=world)
        ref = attention_fp64(q.double().numpy(), k.double().numpy(), v.double().numpy())
        assert tuple(o.shape) == (B, H, L, d)
        errs.append(float(np.abs(o.double().numpy() - ref).max()))
    with open(f"{result_path}.{rank}", "w") as f:
        f.write(f"{errs[0]} {errs[1]} {seen[0]} {seen[1]}")
    dist.destroy_process_group()


def test_v2_surface_world_size_2(tmp_path):
    """flash_attention_v2(..., world_size=2) over gloo: full O on every rank, and the
    partial format left to splitkv_attention's default (fp64 for fp64 inputs, per-row scaled
    fp16 otherwise) -- the same exchange format as every other multi-GPU entry point."""
    port = _free_port()
    path = str(tmp_path / "res")
    mp.start_processes(_surface_worker, args=(2, port, path), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        e64, e32, p64, p32 = open(f"{path}.{r}").read().split(" ")
        assert float(e64) < 1e-6 and float(e32) < 4 * 2.0 ** -11
        assert p64 == "None" and p32 == "None"
