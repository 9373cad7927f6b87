"""Split-KV over ranks with the real HIP kernels: world size 2, 4 and 8 on ONE GPU.

The driver's multi-GPU runs need an 8-GPU node; a 1-GPU box can still run two or four ranks
that share the card.  RCCL expects one device per rank, so here the exchange goes over gloo,
whose all_to_all_single / all_gather take device tensors.  What runs on the GPU is the
product's whole per-rank sequence (dist.splitkv_attention, overlap=False): the partial
kernel writing the all-to-all send layout [W][B*H][L/W][d] with per-row scaled fp16 rows and
{lse, e} pairs, the exchange, the combine kernel and the all_gather -- checked against the
fp64 oracle over all rows on every rank.  (The overlapped send/recv pipeline and the native
RCCL library need one device per rank: tests/test_dist.py covers their exchange logic on CPU.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.batched import attention_fp64

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rows_ref(q, k, v, rows):
    """fp64 attention of the given query rows of every head (the oracle's maths on a row
    subset: the full L x L oracle at L = 16384 would not fit the test's time)."""
    qs = q[:, :, rows].double().numpy()
    kk, vv = k.double().numpy(), v.double().numpy()
    d = qs.shape[-1]
    s = np.einsum("bhqd,bhkd->bhqk", qs, kk) / np.sqrt(d)
    s -= s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(axis=-1, keepdims=True)
    return np.einsum("bhqk,bhkd->bhqd", p, vv)


def _worker(rank, world, port, path, dtype_name, shape, sampled):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exploring_flash_attention_amd import dist as fdist
    dtype = getattr(torch, dtype_name)
    g = torch.Generator().manual_seed(0)
    B, H, L, d = shape
    q, k, v = (torch.randn(B, H, L, d, generator=g).to(dtype) for _ in range(3))
    Lc = L // world
    lo, hi = fdist.shard_bounds(L, world, rank)
    own = np.arange(rank * Lc, (rank + 1) * Lc)
    if sampled:  # every rank's first and last row and 30 between, of every head
        pick = np.unique(np.linspace(0, Lc - 1, 32).round().astype(int))
        ref_local = _rows_ref(q, k, v, own[pick])
        ref_full = _rows_ref(q, k, v, np.concatenate([np.arange(r * Lc, (r + 1) * Lc)[pick] for r in range(world)]))
    else:
        pick = np.arange(Lc)
        ref = attention_fp64(q.double().numpy(), k.double().numpy(), v.double().numpy())
        ref_local, ref_full = ref[:, :, own], ref
    dev = torch.device("cuda", 0)
    qg = q.to(dev)
    ks, vs = k[:, :, lo:hi].contiguous().to(dev), v[:, :, lo:hi].contiguous().to(dev)
    local = fdist.splitkv_attention(qg, ks, vs)  # default overlap: a gloo group takes all-to-all
    full = fdist.splitkv_attention(qg, ks, vs, overlap=False, gather=True)
    torch.cuda.synchronize()
    full_rows = full if not sampled else full[:, :, torch.from_numpy(np.concatenate(
        [np.arange(r * Lc, (r + 1) * Lc)[pick] for r in range(world)])).to(dev)]
    err_local = np.abs(local[:, :, torch.from_numpy(pick).to(dev)].double().cpu().numpy() - ref_local).max()
    err_full = np.abs(full_rows.double().cpu().numpy() - ref_full).max()
    finite = bool(torch.isfinite(local).all()) and bool(torch.isfinite(full).all())
    with open(f"{path}.{rank}", "w") as f:
        f.write(f"{err_local}|{err_full}|{tuple(local.shape)}|{tuple(full.shape)}|{finite}")
    dist.destroy_process_group()


def _run(tmp_path, world, dtype_name, shape, sampled):
    port, path = _free_port(), str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, port, path, dtype_name, shape, sampled), nprocs=world, join=True,
                       start_method="spawn")
    tol = 6e-3 if dtype_name == "bfloat16" else 2e-3  # the single-GPU build gates (test_gpu.py)
    B, H, L, d = shape
    for r in range(world):
        err_local, err_full, local_shape, full_shape, finite = open(f"{path}.{r}").read().split("|")
        assert float(err_local) < tol and float(err_full) < tol, (r, err_local, err_full)
        assert local_shape == str((B, H, L // world, d)) and full_shape == str((B, H, L, d))
        assert finite == "True"


@pytest.mark.timeout(300, method="thread")  # a stuck rendezvous fails the test instead of hanging the run
@pytest.mark.parametrize("dtype_name", ["bfloat16", "float16"])
@pytest.mark.parametrize("world", [2, 4])
def test_splitkv_ranks_share_one_gpu(tmp_path, world, dtype_name):
    _run(tmp_path, world, dtype_name, (2, 4, 1024, 128), sampled=False)


@pytest.mark.timeout(400, method="thread")
def test_splitkv_eight_ranks_c5_length(tmp_path):
    """C5's sequence length and rank count: L = 16384 keys sharded over W = 8 ranks (2048 each),
    with B*H cut to 1 x 2 so that eight ranks fit one card; every rank's partial kernel over
    all 16384 query rows, the exchange, the combine and the all-gather, checked against the
    fp64 oracle on 32 sampled rows of every rank's chunk (first and last included)."""
    _run(tmp_path, 8, "bfloat16", (1, 2, 16384, 128), sampled=True)


def _native_worker(rank, world, port, path):
    """One rank per GPU over RCCL: the native C-ABI forward (fa_fwd_v2_dist: pipelined
    per-destination partial launches, the shifted send/recv steps, combine, all-gather) against
    the Python paths (all-to-all and pipelined send/recv) over the same RCCL group, bit for bit,
    and against the fp64 oracle on sampled rows."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    from exploring_flash_attention_amd import dist as fdist
    g = torch.Generator().manual_seed(0)
    B, H, L, d = 2, 4, 2048, 128
    q, k, v = (torch.randn(B, H, L, d, generator=g).to(torch.bfloat16) for _ in range(3))
    lo, hi = fdist.shard_bounds(L, world, rank)
    dev = torch.device("cuda", rank)
    qg = q.to(dev)
    ks, vs = k[:, :, lo:hi].contiguous().to(dev), v[:, :, lo:hi].contiguous().to(dev)
    comm = fdist.RcclComm()
    nat_local = fdist.splitkv_attention_native(qg, ks, vs, comm)
    nat_full = fdist.splitkv_attention_native(qg, ks, vs, comm, gather=True)
    py_full = fdist.splitkv_attention(qg, ks, vs, overlap=False, gather=True)
    py_ovl = fdist.splitkv_attention(qg, ks, vs, gather=True)  # pipelined send/recv over RCCL
    torch.cuda.synchronize()
    comm.close()
    rows = np.unique(np.linspace(0, L - 1, 64).round().astype(int))
    ref = _rows_ref(q, k, v, rows)
    err = np.abs(nat_full[:, :, torch.from_numpy(rows).to(dev)].double().cpu().numpy() - ref).max()
    same = bool(torch.equal(nat_full, py_full)) and bool(torch.equal(nat_full, py_ovl))
    own = bool(torch.equal(nat_local, nat_full[:, :, rank * (L // world):(rank + 1) * (L // world)]))
    with open(f"{path}.{rank}", "w") as f:
        f.write(f"{err}|{same}|{own}")
    dist.destroy_process_group()


@pytest.mark.timeout(300, method="thread")
@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_rccl_exchange_one_gpu_per_rank(tmp_path, world):
    """The native RCCL exchange at W > 1 (include/fa_mi355x_dist.h), which needs one device per
    rank: skipped on boxes with fewer GPUs (the CPU schedule test, tests/test_dist_schedule.py,
    covers its step pairing, offsets and failure latch everywhere)."""
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs, {torch.cuda.device_count()} visible")
    port, path = _free_port(), str(tmp_path / "res")
    mp.start_processes(_native_worker, args=(world, port, path), nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        err, same, own = open(f"{path}.{r}").read().split("|")
        assert float(err) < 6e-3, (r, err)
        assert same == "True", f"rank {r}: native and Python split-KV differ"
        assert own == "True", f"rank {r}: the local rows are not the gathered ones"
