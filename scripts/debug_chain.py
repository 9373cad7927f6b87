"""Where a chained-kernel build differs from the one-shot kernel at a given shape: max |diff|
per query tile, grouped by the tile's position j in its workgroup's item list
(fa_fwd16_chain.hpp schedule) and by the rows of the tile.

    python scripts/debug_chain.py base.so chain.so [--shape B,H,L]
"""
import argparse
import ctypes

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--shape", default="32,8,1024")
    ap.add_argument("--cus", type=int, default=256)
    args = ap.parse_args()
    B, H, L = (int(x) for x in args.shape.split(","))
    d = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    outs = []
    for p in args.libs:
        h = ctypes.CDLL(p)
        h.fa_fwd_v1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int, ctypes.c_void_p]
        o = torch.full_like(q, float("nan"))
        st = h.fa_fwd_v1(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, 1,
                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        assert st == 0
        outs.append(o)
    ref = torch.softmax(q.float() @ k.float().transpose(-1, -2) / d ** 0.5, -1) @ v.float()
    nqt = L // 128
    nitems = B * H * nqt
    grid = 2 * args.cus // 8 * 8
    nl, iq, ir = grid >> 3, nitems >> 3, nitems & 7
    pos = {}
    for b in range(grid):
        x, l = b & 7, b >> 3
        gs = x * (iq + 1) if x < ir else ir * (iq + 1) + (x - ir) * iq
        gc = iq + (1 if x < ir else 0)
        n = (gc - l + nl - 1) // nl if l < gc else 0
        for j in range(n):
            pos[gs + l + nl * j] = (b, j)
    for p, o in zip(args.libs, outs):
        err = (o.float() - ref).abs().reshape(B * H, nqt, 128, d)
        per_tile = err.amax(dim=(2, 3)).flatten()  # item = bh * nqt + qt
        nan = torch.isnan(o).reshape(B * H, nqt, 128, d).any(dim=3).any(dim=2).flatten()
        byj = {}
        for w in range(nitems):
            j = pos.get(w, (None, -1))[1]
            byj.setdefault(j, []).append((float(per_tile[w]), bool(nan[w])))
        print(p, "max err", float(per_tile.max()), "nan tiles", int(nan.sum()))
        for j in sorted(byj):
            e = [x for x, _ in byj[j]]
            print(f"   j={j}: tiles {len(e)} max {max(e):.3e} bad(>1e-2) {sum(x > 1e-2 for x in e)} nan {sum(n for _, n in byj[j])}")
        rows = err.amax(dim=(0, 1, 3))  # per row within the tile
        print("   rows with err > 1e-2:", [i for i in range(128) if rows[i] > 1e-2][:40])


if __name__ == "__main__":
    main()
