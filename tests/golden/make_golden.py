"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own Python.

Run in the build container only (it needs /root/reference, which does not exist on the
GPU box; the committed .npz files travel instead):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [wide]

Every fixture stores its inputs, the reference function's output(s) and the reference
naive_attention output, plus a ``call`` string naming the reference function and
arguments that produced them.  Reference files used (tyler-utah/exploring_flash_attention):
  common/reference.py                          naive_attention
  flash_attention_v1/numpy_basic.py            flash_attention_tiled(Q,K,V,Bq,Bk)
  flash_attention_v1/numpy_gpu_like_opt2.py    flash_attention_tiled(Q,K,V,O,L,d,Bq,Bk)
  flash_attention_v1_tiled_d/numpy_basic.py    flash_attention_tiled_global(...)
  flash_attention_v2/numpy_gpu_like.py         flash_attention_tiled_v2(...)
"""
import importlib.util
import os
import sys

import numpy as np

REF = os.environ.get("FA_REFERENCE_ROOT", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


def _load(rel, name):
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _rng_inputs(L, d, dtype, seed=0):
    rng = np.random.default_rng(seed)
    return tuple(rng.standard_normal((L, d)).astype(dtype) for _ in range(3))


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


def wide(ref, tdb):
    """g6: tiled-d at a head dim past one tile (d = 384), the case the reference's tiled-d variant
    exists for: L=16, ragged d tiles (100 / 96 columns: chunks 100,100,100,84 and 4 x 96); inputs are multiples of 1/16 in [-2, 2) stored as int8 (exact in every
    float type), computed in fp64."""
    rng = np.random.default_rng(6)
    qi, ki, vi = (rng.integers(-32, 32, (16, 384)).astype(np.int8) for _ in range(3))
    Q, K, V = (x.astype(np.float64) / 16 for x in (qi, ki, vi))
    outs = {}
    for (dq, dv) in ((100, 96),):
        outs[f"O_{dq}_{dv}"] = tdb.flash_attention_tiled_global(Q, K, V, Bq=8, Bk=8, d_tile_qk=dq, d_tile_v=dv)
    _save("g6_tiled_d_d384.npz", Q16=qi, K16=ki, V16=vi, O_naive=ref.naive_attention(Q, K, V), **outs,
          call=np.array("flash_attention_v1_tiled_d/numpy_basic.py flash_attention_tiled_global(Q,K,V,Bq=8,Bk=8,"
                        "d_tile_qk,d_tile_v) with Q = Q16 / 16 etc."))


def main():
    ref = _load("common/reference.py", "ref_common")
    if sys.argv[1:] == ["wide"]:  # only g6 (the others unchanged)
        wide(ref, _load("flash_attention_v1_tiled_d/numpy_basic.py", "ref_td_basic"))
        return
    v1b = _load("flash_attention_v1/numpy_basic.py", "ref_v1_basic")
    v1o = _load("flash_attention_v1/numpy_gpu_like_opt2.py", "ref_v1_opt2")
    tdb = _load("flash_attention_v1_tiled_d/numpy_basic.py", "ref_td_basic")
    v2 = _load("flash_attention_v2/numpy_gpu_like.py", "ref_v2")

    # g1: config C1 plumbing -- numpy_basic FA-v1, L=64 d=32, rng(0) N(0,1), fp64 and fp16.
    for tag, dt in (("f64", np.float64), ("f16", np.float16)):
        Q, K, V = _rng_inputs(64, 32, dt)
        O = v1b.flash_attention_tiled(Q, K, V, Bq=8, Bk=8)
        _save(f"g1_v1_basic_{tag}.npz", Q=Q, K=K, V=V, O=O, O_naive=ref.naive_attention(Q, K, V),
              call=np.array("flash_attention_v1/numpy_basic.py flash_attention_tiled(Q,K,V,Bq=8,Bk=8)"))

    # g1r: ragged tail (L not a multiple of the tiles), numpy_basic, fp64.
    Q, K, V = _rng_inputs(50, 32, np.float64, seed=1)
    _save("g1_v1_basic_ragged.npz", Q=Q, K=K, V=V, O=v1b.flash_attention_tiled(Q, K, V, Bq=8, Bk=16),
          O_naive=ref.naive_attention(Q, K, V),
          call=np.array("flash_attention_v1/numpy_basic.py flash_attention_tiled(Q,K,V,Bq=8,Bk=16) L=50"))

    # g2: opt2 fused C-style form (the CPU baseline), flat buffers, fp64.
    for (L, d, bq, bk, seed) in ((64, 32, 8, 8, 0), (40, 16, 8, 16, 2)):
        Q, K, V = _rng_inputs(L, d, np.float64, seed=seed)
        O = np.zeros(L * d, dtype=np.float64)
        v1o.flash_attention_tiled(Q.ravel(), K.ravel(), V.ravel(), O, L, d, Bq=bq, Bk=bk)
        _save(f"g2_v1_opt2_L{L}_d{d}.npz", Q=Q, K=K, V=V, O=O.reshape(L, d),
              O_naive=ref.naive_attention(Q, K, V), Bq=bq, Bk=bk,
              call=np.array(f"flash_attention_v1/numpy_gpu_like_opt2.py flash_attention_tiled(Q,K,V,O,{L},{d},Bq={bq},Bk={bk})"))

    # g3: tiled-d, L=64 d=128, two tile settings, fp64; plus fp16.
    for tag, dt in (("f64", np.float64), ("f16", np.float16)):
        Q, K, V = _rng_inputs(64, 128, dt)
        outs = {}
        for (bq, bk, dq, dv) in ((8, 8, 16, 16), (16, 16, 32, 32)):
            outs[f"O_{bq}_{bk}_{dq}_{dv}"] = tdb.flash_attention_tiled_global(
                Q, K, V, Bq=bq, Bk=bk, d_tile_qk=dq, d_tile_v=dv)
        _save(f"g3_tiled_d_{tag}.npz", Q=Q, K=K, V=V, O_naive=ref.naive_attention(Q, K, V), **outs,
              call=np.array("flash_attention_v1_tiled_d/numpy_basic.py flash_attention_tiled_global(Q,K,V,Bq,Bk,d_tile_qk,d_tile_v)"))

    # g4: split-KV v2, L=64, d in {32, 128}, KVTPB in {1, 4}, Bq=Bk=8, d_tiles 16 -- output,
    # and for d=32 KVTPB=4 also the per-(q_tile, kv_block) workspace (O_acc, m, l).
    for d in (32, 128):
        Q, K, V = _rng_inputs(64, d, np.float64, seed=3)
        rec = {"Q": Q, "K": K, "V": V, "O_naive": ref.naive_attention(Q, K, V)}
        for kvtpb in (1, 4):
            O = np.zeros(64 * d)
            wO, wm, wl = {}, {}, {}
            v2.flash_attention_tiled_v2(Q.ravel(), K.ravel(), V.ravel(), O, wO, wm, wl, 64, d,
                                        Bq=8, Bk=8, d_tile_qk=16, d_tile_v=16,
                                        kv_tiles_per_block=kvtpb)
            rec[f"O_kvtpb{kvtpb}"] = O.reshape(64, d)
            if d == 32 and kvtpb == 4:
                keys = sorted(wO)
                nq = 1 + max(k[0] for k in keys)
                nkb = 1 + max(k[1] for k in keys)
                rec["ws_O"] = np.stack([np.stack([wO[(q, b)] for b in range(nkb)]) for q in range(nq)])
                rec["ws_m"] = np.stack([np.stack([wm[(q, b)] for b in range(nkb)]) for q in range(nq)])
                rec["ws_l"] = np.stack([np.stack([wl[(q, b)] for b in range(nkb)]) for q in range(nq)])
        _save(f"g4_v2_d{d}.npz", **rec,
              call=np.array("flash_attention_v2/numpy_gpu_like.py flash_attention_tiled_v2(...,Bq=8,Bk=8,d_tile_qk=16,d_tile_v=16,kv_tiles_per_block=K)"))

    # g5: CUDA-driver style batch (srand(42) U[-1,1], flash_attention_v1/CUDA/driver.cu:71-75,
    # rounded to fp16), B=1 H=2 L=128; O (stored fp32) = reference naive_attention per head on the
    # fp16-rounded values in fp64.  The rand() stream is glibc's; the C oracle restates it.
    import ctypes
    lib = ctypes.CDLL(os.path.join(HERE, "..", "..", "oracle", "_build", "liboracle.so"))
    for d in (32, 128):
        n = 1 * 2 * 128 * d
        buf = np.empty(3 * n, np.float32)
        lib.oracle_driver_random(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(3 * n),
                                 ctypes.c_uint(42), ctypes.c_int(1))
        x = buf.astype(np.float16).reshape(3, 1, 2, 128, d)
        O = np.stack([np.stack([ref.naive_attention(*(x[i, b, h].astype(np.float64) for i in range(3)))
                                for h in range(2)]) for b in range(1)]).astype(np.float32)
        _save(f"g5_driver_d{d}.npz", Q=x[0], K=x[1], V=x[2], O=O,
              call=np.array("common/reference.py naive_attention per (b,h) on driver.cu srand(42) inputs"))
    wide(ref, tdb)


if __name__ == "__main__":
    main()
