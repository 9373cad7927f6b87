"""Every global access of the forward kernels stays inside its allocation (CPU replay).

VERDICT round 3, item 1: a full-size C3 run of fa_fwd16_kernel aborted once (gpurun_out/one.log,
round 3, uncommitted state between 300255a and 949eaba; DESIGN.md section 9 records what is and
is not known about it).  A GPU memory fault needs a global address outside an allocation, so
this test replays, for whole BASELINE-size grids, the address arithmetic of
csrc/fa_fwd16_kernel.hpp (d = 128, whole 64-key tiles: final, row-layout partial incl. the
multi-GPU row-range chunks (QSTR), fused split-KV) and of csrc/fa_fwd_kernel.hpp (other head
dims, key tails, strided views) with the C ABI's own launch arguments (split plans from
fa_fwd_v2_split_plan, workspace sizes from fa_fwd_v2_workspace_size_ex, both called through
ctypes -- no GPU needed), and asserts for every workgroup:

* the block -> (query tile, split, b*h) decode after xcd_remap is a bijection onto the grid;
* the Q buffer descriptor [base, base + num_records) lies inside q's allocation (the hardware
  clamps lane offsets to num_records, so the descriptor's extent bounds every Q load);
* every K / V tile descriptor the prologue and the steps build (tiles 0 .. ntiles-1 of the
  split) lies inside k / v;
* every output row store (final O, row-layout partials, lse / {lse, e} pairs) and every fused
  workspace descriptor (fragment-order partials, lse, scale exponents, the counter) lies inside
  its buffer.
"""
import ctypes

import numpy as np
import pytest

from exploring_flash_attention_amd import _lib

KBQ = 128          # query rows per workgroup (fa_internal.hpp kBQ)
ALIGN = 256


def bk_for(d):
    return 64 if d <= 128 else 32


def xcd_remap(b, n):
    q, r = n >> 3, n & 7
    x, i = b & 7, b >> 3
    return np.where(x < r, x * (q + 1), r * (q + 1) + (x - r) * q) + i


def a256(x):
    return (x + 255) & ~255


class Alloc:
    """A buffer [lo, hi) in bytes; the kernel pointer sits at byte 0 unless a view offset."""

    def __init__(self, name, nbytes, ptr_off=0):
        self.name, self.lo, self.hi = name, -ptr_off, nbytes - ptr_off

    def check(self, start, length, what):
        start = np.asarray(start, dtype=np.int64)
        length = np.broadcast_to(np.asarray(length, dtype=np.int64), start.shape)
        live = length > 0
        bad = live & ((start < self.lo) | (start + length > self.hi))
        assert not bad.any(), (f"{what}: {int(bad.sum())} accesses leave {self.name} "
                               f"[{self.lo}, {self.hi}); first at {int(start[bad].flat[0])}+{int(length[bad].flat[0])}")


def replay(args, allocs, kernel16, strided=None, qstr=None, mode="final", pt_bytes=2, scaled=False,
           flat_decode=False, tile_group=0):
    """Replay one launch.  args: the FwdArgs fields the kernels read; allocs: q, k, v, o (and
    for fused: ws_o, ws_lse, ws_esc, counters, o_final)."""
    BH, Lq, Lk, D = args["BH"], args["Lq"], args["Lk"], args["D"]
    nqt, nsplit, kvps = args["nqt"], args["nsplit"], args["kv_per_split"]
    nblk = nqt * nsplit * BH
    assert nblk <= 0x7fffffff
    b = np.arange(nblk, dtype=np.int64)
    w = xcd_remap(b, nblk)
    assert np.array_equal(np.sort(w), b), "xcd_remap is not a bijection onto the grid"
    qt, rest = w % nqt, w // nqt
    split, bh = rest % nsplit, rest // nsplit
    if tile_group == 1:  # fa_internal.hpp decode_item, FwdArgs::tile_group
        split, rest = w % nsplit, w // nsplit
        qt, bh = rest % nqt, rest // nqt
    elif 1 < tile_group < nqt:
        assert nqt % tile_group == 0
        qi, rest = w % tile_group, w // tile_group
        split, rest = rest % nsplit, rest // nsplit
        ng = nqt // tile_group
        qt, bh = (rest % ng) * tile_group + qi, rest // ng
    if flat_decode:  # (test_replay_catches_a_bad_decode: the split index ignored)
        split, bh = np.zeros_like(rest), rest
    assert bh.max() < BH and bh.min() >= 0, f"b*h decoded up to {int(bh.max())} of {BH}"
    ROWB, bk = 2 * D, bk_for(D)
    kv_begin = split * kvps
    kv_end = np.minimum(kv_begin + kvps, Lk)
    nkv = kv_end - kv_begin
    assert (nkv > 0).all(), "an empty split"
    ntiles = (nkv + bk - 1) // bk
    if kernel16:  # fa_fwd16_kernel: whole 64-key tiles (strided views too, round 4)
        assert D == 128 and (nkv % 64 == 0).all()
    H = args.get("H", 1)
    # ---- Q descriptor
    q_tile0 = qt * KBQ
    q_rows = np.minimum(Lq - q_tile0, KBQ)
    assert (q_rows > 0).all()
    if strided:
        qs, ks, os_ = strided
        qrb, krb = 2 * qs[2], 2 * ks[2]
        q_head = (bh // H) * qs[0] + (bh % H) * qs[1]
        k_head = (bh // H) * ks[0] + (bh % H) * ks[1]
        o_head, orow = (bh // H) * os_[0] + (bh % H) * os_[1], os_[2]
        q_base = 2 * q_head + q_tile0 * qrb
        q_len = (q_rows - 1) * qrb + ROWB
    else:
        qrb = krb = ROWB
        q_head = ((bh // H) * qstr[0] + (bh % H) * qstr[1]) if qstr else bh * Lq * D
        k_head = bh * Lk * D
        o_head, orow = bh * Lq * D, D
        q_base = 2 * q_head + q_tile0 * ROWB
        q_len = q_rows * ROWB
    allocs["q"].check(q_base, q_len, "Q descriptor")
    # ---- K / V tile descriptors, tiles 0 .. ntiles-1 of the split
    kbase = 2 * k_head + kv_begin * krb
    for t in range(int(ntiles.max())):
        live = t < ntiles
        valid = np.clip(nkv - t * bk, 0, bk)
        tstride = bk * krb
        length = np.where(live, (valid - 1) * krb + ROWB if strided else valid * ROWB, 0)
        for name in ("k", "v"):
            allocs[name].check(kbase + t * tstride, length, f"{name.upper()} tile {t} descriptor")
    # ---- stores
    rows = q_tile0[:, None] + np.arange(KBQ)[None, :]
    live = rows < Lq
    if mode == "final":
        allocs["o"].check(np.where(live, 2 * (o_head[:, None] + rows * orow), 0), np.where(live, ROWB, 0), "O row store")
    elif mode == "partial":
        cr = args["chunk_rows"]
        row_lin = (rows // cr) * BH * cr + bh[:, None] * cr + rows % cr
        ostart = pt_bytes * (split[:, None] * args["split_stride"] + row_lin * D)
        allocs["o"].check(np.where(live, ostart, 0), np.where(live, pt_bytes * D, 0), "partial row store")
        lidx = split[:, None] * BH * Lq + row_lin
        lb = 8 if scaled else 4
        allocs["lse"].check(np.where(live, lb * lidx, 0), np.where(live, lb, 0), "lse store")
    else:  # fused
        grp = bh * nqt + qt
        blk = split * BH * nqt + grp
        BLK = KBQ * D
        allocs["ws_o"].check(blk * BLK * pt_bytes, BLK * pt_bytes, "fragment-order partial descriptor")
        allocs["ws_lse"].check(blk * KBQ * 4, KBQ * 4, "lse descriptor")
        if scaled:
            allocs["ws_esc"].check(blk * KBQ * 4, KBQ * 4, "scale-exponent descriptor")
        allocs["counters"].check(grp * 4, 4, "counter")
        allocs["o_final"].check(np.where(live, 2 * (o_head[:, None] + rows * orow), 0), np.where(live, ROWB, 0),
                                "combined O row store")
    return nblk


def _plan(B, H, L, d, kvt, group):
    lib = _lib.lib()
    kb, per, ppt = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _lib.check(lib.fa_fwd_v2_split_plan(B, H, L, d, kvt, group, _lib.FA_DTYPE_BF16, ctypes.byref(kb),
                                        ctypes.byref(per), ctypes.byref(ppt)))
    nb, ns = ctypes.c_size_t(), ctypes.c_int()
    _lib.check(lib.fa_fwd_v2_workspace_size_ex(B, H, L, d, kvt, group, _lib.FA_DTYPE_BF16, _lib.FA_DTYPE_FP16_SCALED,
                                               ctypes.byref(nb), ctypes.byref(ns)))
    return kb.value, per.value, ppt.value, nb.value


def _final_args(B, H, L, d):
    return dict(BH=B * H, H=H, Lq=L, Lk=L, D=d, nqt=-(-L // KBQ), nsplit=1, kv_per_split=L)


def _tensor(name, B, H, L, d):
    return Alloc(name, 2 * B * H * L * d)


@pytest.mark.parametrize("B,H,L,d", [(32, 8, 1024, 32), (32, 8, 1024, 128), (32, 8, 4096, 128), (32, 8, 1024, 64),
                                     (32, 8, 1024, 256), (2, 3, 1000, 128), (1, 1, 200, 256), (4, 2, 77, 32)],
                         ids=["C2", "C3", "C4-unsplit", "d64", "d256", "tail-d128", "tail-d256", "tail-d32"])
def test_final_mode_in_bounds(B, H, L, d):
    a = _final_args(B, H, L, d)
    allocs = {n: _tensor(n, B, H, L, d) for n in "qkvo"}
    k16 = d == 128 and L % 64 == 0  # the dispatch of fa_fwd.hip launch_one
    replay(a, allocs, k16)


def test_c3_decode_of_the_aborting_commit_equals_the_fixed_one():
    """At 300255a the final-mode kernel decoded bh = w / nqt (one split); 949eaba decodes
    split = (w / nqt) % nsplit, bh = (w / nqt) / nsplit.  With nsplit = 1 both give the same
    (query tile, b*h) for all 2048 workgroups of C3, so that decode could not have faulted."""
    nblk, nqt = 2048, 8
    w = xcd_remap(np.arange(nblk), nblk)
    old_bh = w // nqt
    new_bh = (w // nqt) // 1
    assert np.array_equal(old_bh, new_bh) and old_bh.max() == 255


@pytest.mark.parametrize("order", ["qtile-fastest", "split-fastest", "tile-group-4"])
@pytest.mark.parametrize("group", [0, 1, 4, 16], ids=["auto", "1-per-wg", "4-per-wg", "16-per-wg"])
@pytest.mark.parametrize("B,H,L", [(32, 8, 4096), (1, 1, 16384), (1, 2, 4096), (2, 2, 1000)],
                         ids=["C4", "b1h1-l16k", "b1h2-l4k", "tail"])
def test_fused_split_in_bounds(B, H, L, group, order):
    d, kvt = 128, 4
    kb, per, ppt, nbytes = _plan(B, H, L, d, kvt, group)
    if ppt == 1:
        a = _final_args(B, H, L, d)
        replay(a, {n: _tensor(n, B, H, L, d) for n in "qkvo"}, L % 64 == 0)
        return
    BH, nqt = B * H, -(-L // KBQ)
    rows = ppt * BH * nqt * KBQ
    o_bytes = a256(rows * d * 2)
    lse_off = o_bytes
    esc_off = lse_off + a256(rows * 4)
    cnt_off = esc_off + a256(rows * 4)
    assert cnt_off + a256(BH * nqt * 4) == nbytes  # the layout fa_capi.cpp v2_layout gives
    a = dict(BH=BH, H=H, Lq=L, Lk=L, D=d, nqt=nqt, nsplit=ppt, kv_per_split=min(kvt * 64 * per, L))
    allocs = {n: _tensor(n, B, H, L, d) for n in "qkv"}
    allocs.update(ws_o=Alloc("ws partials", nbytes), ws_lse=Alloc("ws lse", nbytes - lse_off),
                  ws_esc=Alloc("ws esc", nbytes - esc_off), counters=Alloc("ws counters", nbytes - cnt_off),
                  o_final=_tensor("o", B, H, L, d))
    replay(a, allocs, L % 64 == 0, mode="fused", scaled=True,
           tile_group={"qtile-fastest": 0, "split-fastest": 1, "tile-group-4": 4}[order])


@pytest.mark.parametrize("cus", [256, 80])
@pytest.mark.parametrize("B,H,L,group", [(32, 8, 4096, 1), (32, 8, 4096, 4), (2, 2, 16384, 4), (1, 8, 16384, 16),
                                         (3, 5, 2048, 2)],
                         ids=["C4-16-partials", "C4-4-partials", "b2h2-l16k", "b1h8-l16k", "odd-heads"])
def test_chain_walk_in_bounds(B, H, L, group, cus):
    """The fused chain (fa_fwd16_chain.hpp, MODE kFused -- the walk): under fa_fwd.hip's
    conditions (keys per block a multiple of 128 and >= 256, whole query tiles, at least one
    query tile per workgroup of the 2-per-CU grid) every query tile is walked by exactly one
    workgroup, over key blocks 0..ns-1; every K / V tile of every block, every partial block
    (all but the last, stored; every one, read by the combine) and every O row lies inside its
    buffer."""
    d, kvt = 128, 4
    kb, per, ppt, nbytes = _plan(B, H, L, d, kvt, group)
    BH, nqt = B * H, L // KBQ
    tiles, grid = BH * nqt, 2 * cus // 8 * 8
    kvps = min(kvt * 64 * per, L)
    if not (ppt > 1 and kvps % 128 == 0 and kvps >= 256 and L % kvps == 0 and L % KBQ == 0 and tiles >= grid):
        pytest.skip("the launcher runs the one-shot kernel for this shape")
    assert ppt * kvps == L
    lists = chain_items(tiles, grid)
    flat = np.array([w for lst in lists for w in lst], dtype=np.int64)
    assert sorted(flat.tolist()) == list(range(tiles)) and all(len(lst) > 0 for lst in lists)
    rows = ppt * BH * nqt * KBQ
    o_bytes = a256(rows * d * 2)
    ws_o = Alloc("ws partials", o_bytes)
    ws_lse = Alloc("ws lse", a256(rows * 4))
    q, k, v, o = (_tensor(n, B, H, L, d) for n in "qkvo")
    qt, bh = flat % nqt, flat // nqt
    grp = bh * nqt + qt
    q.check(2 * (bh * L + qt * KBQ) * d, KBQ * 256, "walk Q tile")
    o.check(2 * (bh * L + qt * KBQ) * d, KBQ * 256, "walk O tile (combine)")
    BLK, TILEB = KBQ * d, 64 * 256
    for sp in range(ppt):
        kv0 = 2 * (bh * L + sp * kvps) * d
        for t in range(kvps // 64):
            k.check(kv0 + t * TILEB, TILEB, "walk K tile")
            v.check(kv0 + t * TILEB, TILEB, "walk V tile")
        blk = sp * BH * nqt + grp
        ws_o.check(blk * BLK * 2, BLK * 2, "walk partial block")
        ws_lse.check(blk * KBQ * 4, KBQ * 4, "walk lse / e block")
    # every block of every tile is written by exactly one workgroup (the tile's walker)
    blks = (np.arange(ppt)[:, None] * BH * nqt + grp[None, :]).ravel()
    assert len(np.unique(blks)) == ppt * tiles


@pytest.mark.parametrize("W", [2, 8])
@pytest.mark.parametrize("L", [16384, 2048])
def test_multi_gpu_partials_in_bounds(W, L):
    """C5's per-rank partials: the one-launch all-to-all layout (chunk_rows = L / W) and the
    pipelined per-destination chunks (q row-range views, fa_fwd16_kernel's QSTR form)."""
    B, H, d = 32 if L == 2048 else 2, 8 if L == 2048 else 2, 128
    BH, Lc = B * H, L // W
    kv = {n: _tensor(n, B, H, Lc, d) for n in "kv"}
    # one launch over all L rows
    a = dict(BH=BH, H=H, Lq=L, Lk=Lc, D=d, nqt=-(-L // KBQ), nsplit=1, kv_per_split=Lc, chunk_rows=Lc, split_stride=0)
    allocs = dict(kv, q=_tensor("q", B, H, L, d), o=Alloc("o_part", 2 * BH * L * d), lse=Alloc("lse", 8 * BH * L))
    replay(a, allocs, True, mode="partial", scaled=True)
    # chunk p: q is the row range [p*Lc, (p+1)*Lc) of the [B, H, L, d] tensor
    for p in range(W):
        a = dict(BH=BH, H=H, Lq=Lc, Lk=Lc, D=d, nqt=-(-Lc // KBQ), nsplit=1, kv_per_split=Lc, chunk_rows=Lc,
                 split_stride=0)
        allocs = dict(kv, q=Alloc("q", 2 * BH * L * d, ptr_off=2 * p * Lc * d), o=Alloc("chunk", 2 * BH * Lc * d),
                      lse=Alloc("chunk lse", 8 * BH * Lc))
        replay(a, allocs, True, qstr=(H * L * d, L * d, d), mode="partial", scaled=True)


@pytest.mark.parametrize("d", [32, 128, 256])
@pytest.mark.parametrize("L", [1000, 1024])
def test_strided_blhd_views_in_bounds(d, L):
    """[B, L, H, d] tensors viewed as [B, H, L, d] (fa_fwd_v1_ex strides {L*H*d, d, H*d}); d = 128
    with whole 64-key tiles runs fa_fwd16_kernel's strided form."""
    B, H = 2, 4
    st = (L * H * d, d, H * d)
    allocs = {n: _tensor(n, B, H, L, d) for n in "qkvo"}
    replay(dict(_final_args(B, H, L, d)), allocs, d == 128 and L % 64 == 0, strided=(st, st, st))


def test_replay_catches_a_bad_decode():
    """The replay is not vacuous: a fused launch (4 splits) decoded as if it had one split
    addresses heads past B*H -- the kind of index error a GPU memory fault needs."""
    B, H, L, d = 2, 2, 4096, 128
    a = dict(BH=B * H, H=H, Lq=L, Lk=L, D=d, nqt=L // KBQ, nsplit=4, kv_per_split=1024)
    allocs = {n: _tensor(n, B, H, L, d) for n in "qkvo"}
    replay(a, allocs, True)  # the real decode: in bounds
    with pytest.raises(AssertionError, match="decoded up to"):
        replay(a, allocs, True, flat_decode=True)


@pytest.mark.parametrize("B,H,L,d", [(32, 8, 1024, 512), (2, 3, 200, 384), (1, 1, 1, 512), (1, 2, 77, 384)])
@pytest.mark.parametrize("dq,dv", [(32, 32), (128, 64), (64, 128)])
def test_dtiled_kernel_in_bounds(B, H, L, d, dq, dv):
    """csrc/fa_fwd_dtiled.hip (d = 384 / 512): 64-row query tiles; per 64-key tile the K and V
    column chunks [64][dt] are DMA'd through descriptors that start at the chunk's first column
    and end at the last valid key's chunk end."""
    BH, D, ROWD = B * H, d, 2 * d
    nqt = -(-L // 64)
    nblk = nqt * BH
    w = xcd_remap(np.arange(nblk, dtype=np.int64), nblk)
    assert np.array_equal(np.sort(w), np.arange(nblk))
    qt, bh = w % nqt, w // nqt
    q, k, v, o = (_tensor(n, B, H, L, d) for n in "qkvo")
    q_tile0 = qt * 64
    q_rows = np.minimum(L - q_tile0, 64)
    q.check(2 * (bh * L * D + q_tile0 * D), q_rows * ROWD, "Q descriptor")
    ntiles = -(-L // 64)
    pshare = d == 512  # the paired form of fa_fwd_dt_kernel: V chunk c holds dv/2 columns of each half of d
    for t in range(ntiles):
        valid = min(64, L - t * 64)
        for c in range(D // dq):
            k.check(bh * L * ROWD + t * 64 * ROWD + c * 2 * dq, (valid - 1) * ROWD + 2 * dq, f"K chunk t={t} c={c}")
        for c in range(D // dv):
            if pshare:
                base, span = bh * L * ROWD + t * 64 * ROWD + c * dv, (valid - 1) * ROWD + 2 * (D // 2 + dv // 2)
            else:
                base, span = bh * L * ROWD + t * 64 * ROWD + c * 2 * dv, (valid - 1) * ROWD + 2 * dv
            v.check(base, span, f"V chunk t={t} c={c}")
    rows = q_tile0[:, None] + np.arange(64)[None, :]
    live = rows < L
    o.check(np.where(live, 2 * (bh[:, None] * L * D + rows * D), 0), np.where(live, ROWD, 0), "O row store")


@pytest.mark.parametrize("dv", [32, 64, 128])
def test_dtiled_pair_columns(dv):
    """fa_fwd_dt_kernel, paired (d = 512): V chunk c's image takes its first dv/2 columns from the first
    half of d and the rest from the second (the DMA source offsets of src_off); wave h of a pair
    reads image column blocks h * dv/32 .. and stores them as its O^T blocks c * dv/32 + j of
    half h.  Every column of V is read once per tile, into the O^T block that owns it, and the
    two waves of a pair store every column of both of its query blocks once."""
    D = 512
    seen = {}
    for c in range(D // dv):
        for ch in range(dv // 8):  # 16-byte chunks of the image row
            col = 8 * ch + (D // 2 - dv // 2 if 8 * ch >= dv // 2 else 0)
            gcol = c * dv // 2 + col  # the descriptor starts at column c * dv/2
            for x in range(8):
                assert gcol + x not in seen
                seen[gcol + x] = (c, ch)
    assert sorted(seen) == list(range(D))
    bph = dv // 32  # 16-column blocks per half of a chunk
    for h in (0, 1):
        for c in range(D // dv):
            for j in range(bph):
                jj = h * bph + j  # image column block
                b = c * bph + j  # O^T block of this half
                image_cols = [seen_c for seen_c, (cc, ch) in seen.items() if cc == c and ch // 2 == jj]
                assert sorted(image_cols) == list(range(h * D // 2 + 16 * b, h * D // 2 + 16 * b + 16))


def chain_items(nitems, grid):
    """fa_fwd16_chain.hpp's static schedule: block b serves XCD group b % 8 and takes items
    l, l + G/8, ... (l = b / 8) of the contiguous range xcd_remap gives the group."""
    nl = grid >> 3
    iq, ir = nitems >> 3, nitems & 7
    out = []
    for b in range(grid):
        x, l = b & 7, b >> 3
        gstart = x * (iq + 1) if x < ir else ir * (iq + 1) + (x - ir) * iq
        gcnt = iq + (1 if x < ir else 0)
        nmine = (gcnt - l + nl - 1) // nl if l < gcnt else 0
        out.append([gstart + l + nl * j for j in range(nmine)])
    return out


@pytest.mark.parametrize("cus", [256, 304, 80])
@pytest.mark.parametrize("B,H,L", [(32, 8, 1024), (32, 8, 2048), (32, 8, 4096), (4, 32, 1024), (64, 2, 256),
                                   (3, 7, 1408)],
                         ids=["C3", "L2048", "C4-unsplit", "b4h32", "l256", "odd-heads"])
def test_chain_kernel_items_and_bounds(B, H, L, cus):
    """The chained persistent kernel (d = 128 final mode, fa_fwd16_chain.hpp): under the
    launcher's conditions (fa_fwd.hip launch_one: Lk % 128 == 0, Lk >= 256, Lq % 128 == 0, a
    grid of 2 workgroups per CU rounded down to a multiple of 8, at most one workgroup per
    query tile) every query tile is run by exactly one workgroup, no workgroup runs none (the
    kernel returns early only then), and every descriptor it builds -- Q, the K / V tiles
    0..ntiles-1 of the item and K(0), K(1), V(0) of the next, the O tile -- lies inside its
    tensor."""
    D, ROWB, BK, TILEB = 128, 256, 64, 64 * 256
    nqt, BH = L // KBQ, B * H
    nitems = nqt * BH
    grid = 2 * cus // 8 * 8
    if not (L % 128 == 0 and L >= 256 and L % KBQ == 0 and nitems >= grid):
        pytest.skip("the launcher runs the one-shot kernel for this shape")
    lists = chain_items(nitems, grid)
    flat = [w for lst in lists for w in lst]
    assert sorted(flat) == list(range(nitems)), "items not covered exactly once"
    assert all(len(lst) > 0 for lst in lists)
    assert max(map(len, lists)) - min(map(len, lists)) <= 1 + (nitems % grid != 0)
    q, k, v, o = (_tensor(n, B, H, L, D) for n in "qkvo")
    ntiles = L // BK
    w = np.array(flat, dtype=np.int64)
    qt, bh = w % nqt, w // nqt
    qoff = 2 * (bh * L + qt * KBQ) * D
    q.check(qoff, KBQ * ROWB, "chain Q tile")
    o.check(qoff, KBQ * ROWB, "chain O tile")
    kv0 = 2 * bh * L * D
    for t in range(ntiles):
        k.check(kv0 + t * TILEB, TILEB, "chain K tile")
        v.check(kv0 + t * TILEB, TILEB, "chain V tile")
