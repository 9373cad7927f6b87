"""Split-KV over ranks with the real HIP kernels: world size 2 and 4 on ONE GPU.

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


def _worker(rank, world, port, path, dtype_name):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from exploring_flash_attention_amd import dist as fdist
    dtype = getattr(torch, dtype_name)
    g = torch.Generator().manual_seed(0)
    B, H, L, d = 2, 4, 1024, 128
    q, k, v = (torch.randn(B, H, L, d, generator=g).to(dtype) for _ in range(3))
    ref = attention_fp64(q.double().numpy(), k.double().numpy(), v.double().numpy())
    lo, hi = fdist.shard_bounds(L, world, rank)
    dev = torch.device("cuda", 0)
    qg = q.to(dev)
    ks, vs = k[:, :, lo:hi].contiguous().to(dev), v[:, :, lo:hi].contiguous().to(dev)
    local = fdist.splitkv_attention(qg, ks, vs)  # default overlap: a gloo group takes all-to-all
    full = fdist.splitkv_attention(qg, ks, vs, overlap=False, gather=True)
    torch.cuda.synchronize()
    rows = slice(rank * (L // world), (rank + 1) * (L // world))
    err_local = np.abs(local.double().cpu().numpy() - ref[:, :, rows]).max()
    err_full = np.abs(full.double().cpu().numpy() - ref).max()
    with open(f"{path}.{rank}", "w") as f:
        f.write(f"{err_local}|{err_full}|{tuple(local.shape)}|{tuple(full.shape)}")
    dist.destroy_process_group()


@pytest.mark.timeout(300, method="thread")  # a stuck rendezvous fails the test instead of hanging the run
@pytest.mark.parametrize("dtype_name", ["bfloat16", "float16"])
@pytest.mark.parametrize("world", [2, 4])
def test_splitkv_ranks_share_one_gpu(tmp_path, world, dtype_name):
    port, path = _free_port(), str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, port, path, dtype_name), nprocs=world, join=True,
                       start_method="spawn")
    tol = 6e-3 if dtype_name == "bfloat16" else 2e-3  # the single-GPU build gates (test_gpu.py)
    for r in range(world):
        err_local, err_full, local_shape, full_shape = open(f"{path}.{r}").read().split("|")
        assert float(err_local) < tol and float(err_full) < tol, (r, err_local, err_full)
        assert local_shape == f"(2, 4, {1024 // world}, 128)" and full_shape == "(2, 4, 1024, 128)"
