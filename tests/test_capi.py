"""The C-ABI library loads, exports every symbol include/fa_mi355x.h declares, and
validates arguments -- CPU only, no kernel launches."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
import exploring_flash_attention_amd._lib as L

HEADER = os.path.join(ROOT, "include", "fa_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(fa_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ("fa_fwd_v1", "fa_fwd_v1_tiled_d", "fa_fwd_v2", "fa_fwd_v2_workspace_size",
                 "fa_fwd_partial", "fa_combine", "fa_last_error", "fa_version", "fa_kernel_geometry"):
        assert must in names


def test_library_exports_every_declared_symbol():
    h = L.lib()
    for name in declared_functions():
        assert hasattr(h, name), f"{name} declared in fa_mi355x.h but not exported"
    assert set(declared_functions()) == set(L.SIGNATURES), "ctypes SIGNATURES out of sync with header"


def test_exports_are_c_symbols_not_mangled():
    out = os.popen(f"nm -D --defined-only {L.LIB_PATH}").read()
    for name in declared_functions():
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_version_and_geometry():
    # ABI 0.4 (include/fa_mi355x.h FA_MI355X_VERSION_*): blocks_per_workgroup in 0.2, d = 384 / 512
    # in 0.3, fa_last_kernels in 0.4
    hdr = open(os.path.join(ROOT, "include", "fa_mi355x.h")).read()
    major = int(re.search(r"#define FA_MI355X_VERSION_MAJOR (\d+)", hdr).group(1))
    minor = int(re.search(r"#define FA_MI355X_VERSION_MINOR (\d+)", hdr).group(1))
    assert L.lib().fa_version() == (major << 16) | (minor << 8) == 0x000400
    bq, bk, threads, lds = L.geometry(128)
    assert (bq, bk, threads) == (128, 64, 256)
    assert lds == 2 * 2 * 64 * 128 * 2
    bq, bk, threads, lds = L.geometry(128, L.FA_DTYPE_FP64)  # fp64 mode: 64 rows x 16 keys
    assert (bq, bk, threads) == (64, 16, 256)
    bq, bk, threads, lds = L.geometry(256)  # one wave per SIMD, 32-key tiles
    assert (bq, bk, threads, lds) == (128, 32, 256, 2 * 2 * 32 * 256 * 2)
    with pytest.raises(L.FaArgumentError):
        L.geometry(96)
    # the d-tiled kernels: 64 query rows, 64-key tiles, a ring of 16 KiB chunk images (8 slots
    # at d = 512: one workgroup per CU; 4 at d = 384: two)
    assert L.geometry(512) == (64, 64, 256, 4 * 16384 + 4 * 2048 + 4 * 64 + 64) and L.geometry(384) == (64, 64, 256, 3 * 16384)
    assert L.geometry(384, L.FA_DTYPE_FP64)[:3] == (64, 16, 256)


NULL = ctypes.c_void_p(0)


def _status(fn, *args):
    return getattr(L.lib(), fn)(*args)


def test_invalid_arguments_rejected_before_any_launch():
    lib = L.lib()
    st = lib.fa_fwd_v1(NULL, NULL, NULL, NULL, 1, 1, 64, 128, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"null" in lib.fa_last_error()
    st = lib.fa_fwd_v1(NULL, NULL, NULL, NULL, 0, 1, 64, 128, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"positive" in lib.fa_last_error()
    st = lib.fa_fwd_v1(NULL, NULL, NULL, NULL, 1, 1, 64, 96, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_UNSUPPORTED and b"d=96" in lib.fa_last_error()
    st = lib.fa_fwd_v1(NULL, NULL, NULL, NULL, 1, 1, 64, 128, 7, NULL)
    assert st == L.FA_ERR_UNSUPPORTED
    fake = ctypes.c_void_p(0x10000)
    st = lib.fa_fwd_v1_tiled_d(fake, fake, fake, fake, 1, 1, 64, 128, 256, 32, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"d_tile" in lib.fa_last_error()
    st = lib.fa_fwd_v1_tiled_d(fake, fake, fake, fake, 1, 1, 64, 128, 32, 0, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_INVALID_ARG
    st = lib.fa_fwd_v1(ctypes.c_void_p(0x10002), fake, fake, fake, 1, 1, 64, 128, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"aligned" in lib.fa_last_error()


def test_scaled_entry_points_validate_scale():
    lib = L.lib()
    fake = ctypes.c_void_p(0x10000)
    for bad in (0.0, -1.0, float("inf"), float("nan")):
        st = lib.fa_fwd_v1_scaled(fake, fake, fake, fake, 1, 1, 64, 128, bad, L.FA_DTYPE_BF16, NULL)
        assert st == L.FA_ERR_INVALID_ARG and b"softmax_scale" in lib.fa_last_error()
    st = lib.fa_fwd_v1_scaled(fake, fake, fake, fake, 1, 1, 64, 48, 0.1, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_UNSUPPORTED  # the scaled entry still needs a kernel head dim
    st = lib.fa_fwd_v2_scaled(fake, fake, fake, fake, 1, 1, 64, 128, 32, 32, 1, NULL, 0, -2.0,
                              L.FA_DTYPE_BF16, L.FA_DTYPE_FP32, NULL)
    assert st != L.FA_OK


def test_strided_entry_points_validate_strides():
    lib = L.lib()
    fake = ctypes.c_void_p(0x10000)
    S = ctypes.c_int64 * 3
    good = S(4 * 64 * 128, 128, 4 * 128)  # [B, L=64, H=4, d=128] viewed as [B, H, L, d]
    args = (fake, fake, fake, fake, 1, 4, 64, 128)
    for bad in (S(0, 128, 512), S(32768, 128, 100), S(32768, 128, 64), S(-8, 128, 512)):
        st = lib.fa_fwd_v1_ex(*args, bad, good, good, 0.1, L.FA_DTYPE_BF16, NULL)
        assert st == L.FA_ERR_INVALID_ARG and b"stride" in lib.fa_last_error(), bytes(lib.fa_last_error())
    st = lib.fa_fwd_v1_ex(*args, good, good, good, 0.1, L.FA_DTYPE_FP64, NULL)
    assert st == L.FA_ERR_UNSUPPORTED
    huge = S(1 << 40, 128, 1 << 25)  # rows of one head span > 2 GiB
    st = lib.fa_fwd_v1_ex(*args, huge, good, good, 0.1, L.FA_DTYPE_BF16, NULL)
    assert st == L.FA_ERR_UNSUPPORTED


def test_kernel_head_dim_padding_map():
    from exploring_flash_attention_amd import ops
    assert [ops.kernel_head_dim(d) for d in (1, 16, 32, 33, 48, 64, 80, 96, 128, 129, 200, 256)] == \
        [32, 32, 32, 64, 64, 64, 128, 128, 128, 256, 256, 256]
    assert [ops.kernel_head_dim(d) for d in (257, 300, 384, 385, 500, 512)] == [384, 384, 384, 512, 512, 512]
    for bad in (0, -4, 513, 1024):
        with pytest.raises(ValueError):
            ops.kernel_head_dim(bad)


def test_workspace_size_and_v2_checks():
    lib = L.lib()
    nbytes, ns = ctypes.c_size_t(), ctypes.c_int()
    # C4: B32 H8 L4096 d128, KVTPB=4 -> 256-key blocks -> 16 blocks; the 8192 query tiles fill
    # the device (no device here: the MI355X's 256 CUs assumed), so all 16 blocks of a tile go
    # to one workgroup and no partial crosses HBM
    assert lib.fa_fwd_v2_workspace_size(32, 8, 4096, 128, 4, L.FA_DTYPE_BF16, L.FA_DTYPE_BF16,
                                        ctypes.byref(nbytes), ctypes.byref(ns)) == 0
    assert ns.value == 16 and nbytes.value == 256
    kb, g, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    AUTO = L.FA_BLOCKS_PER_WG_AUTO
    assert lib.fa_fwd_v2_split_plan(32, 8, 4096, 128, 4, AUTO, L.FA_DTYPE_BF16, ctypes.byref(kb), ctypes.byref(g),
                                    ctypes.byref(p)) == 0
    assert (kb.value, g.value, p.value) == (16, 16, 1)
    # blocks_per_workgroup = 1: one workgroup and one HBM partial per key block (the reference's
    # layout), fixed by an argument -- the same call gives the same plan whatever the environment
    os.environ["FA_SPLIT_GROUP"] = "7"  # (round 2's environment knob: must be ignored now)
    try:
        assert lib.fa_fwd_v2_workspace_size_ex(32, 8, 4096, 128, 4, 1, L.FA_DTYPE_BF16, L.FA_DTYPE_BF16,
                                               ctypes.byref(nbytes), ctypes.byref(ns)) == 0
        assert lib.fa_fwd_v2_split_plan(32, 8, 4096, 128, 4, 1, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                        ctypes.byref(p)) == 0
        assert (g.value, p.value) == (1, 16)
        n_auto = ctypes.c_size_t()
        assert lib.fa_fwd_v2_workspace_size(32, 8, 4096, 128, 4, L.FA_DTYPE_BF16, L.FA_DTYPE_BF16,
                                            ctypes.byref(n_auto), None) == 0
        assert n_auto.value == 256
    finally:
        del os.environ["FA_SPLIT_GROUP"]
    # a group larger than the block count is clamped; negative is refused
    assert lib.fa_fwd_v2_split_plan(32, 8, 4096, 128, 4, 99, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                    ctypes.byref(p)) == 0 and (g.value, p.value) == (16, 1)
    assert lib.fa_fwd_v2_split_plan(32, 8, 4096, 128, 4, -1, L.FA_DTYPE_BF16, None, None,
                                    None) == L.FA_ERR_INVALID_ARG
    rows = 16 * 32 * 8 * 4096
    # partial O + lse (fragment order, 128-row tiles: 4096 = 32 x 128) + one counter per tile
    assert nbytes.value == rows * 128 * 2 + rows * 4 + 32 * 8 * 32 * 4
    assert nbytes.value > 2 ** 32  # 64-bit sizes (the reference overflows int32 here)
    # a short batch of long sequences: 64 query tiles, so 4 equal groups of the 32 key blocks
    # give each of the 256 CUs a workgroup
    assert lib.fa_fwd_v2_split_plan(1, 1, 8192, 128, 4, AUTO, L.FA_DTYPE_BF16, ctypes.byref(kb), ctypes.byref(g),
                                    ctypes.byref(p)) == 0
    assert (kb.value, g.value, p.value) == (32, 8, 4)
    # 256 query tiles already occupy every CU once; a second workgroup per CU pays when each
    # partial keeps >= 4096 keys (measured round 4, profiles/r04/split_sweep.txt): 2 partials
    # of 8192 keys here, 4 of 4096 at 128 query tiles
    assert lib.fa_fwd_v2_split_plan(1, 2, 16384, 128, 4, AUTO, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                    ctypes.byref(p)) == 0 and (g.value, p.value) == (32, 2)
    assert lib.fa_fwd_v2_split_plan(1, 1, 16384, 128, 4, AUTO, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                    ctypes.byref(p)) == 0 and (g.value, p.value) == (16, 4)
    # ... but not below 4096 keys: 100 query tiles: ceil(256 / 100) = 3 (its 50 key blocks in
    # groups of ceil(50 / 3) = 17; 6 partials would hold 2133 keys); B4 H2 L16384: 1024 tiles
    assert lib.fa_fwd_v2_split_plan(4, 2, 16384, 128, 4, AUTO, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                    ctypes.byref(p)) == 0 and p.value == 1
    assert lib.fa_fwd_v2_split_plan(1, 1, 12800, 128, 4, AUTO, L.FA_DTYPE_BF16, None, ctypes.byref(g),
                                    ctypes.byref(p)) == 0 and (g.value, p.value) == (17, 3)
    assert lib.fa_fwd_v2_workspace_size(1, 1, 100, 64, 1, L.FA_DTYPE_FP16, L.FA_DTYPE_FP32,
                                        ctypes.byref(nbytes), ctypes.byref(ns)) == 0
    assert ns.value == 2
    assert lib.fa_fwd_v2_workspace_size(1, 1, 100, 64, 0, L.FA_DTYPE_FP16, L.FA_DTYPE_FP32,
                                        ctypes.byref(nbytes), None) == L.FA_ERR_INVALID_ARG
    assert lib.fa_fwd_v2_workspace_size(1, 1, 100, 64, 1, L.FA_DTYPE_FP16, L.FA_DTYPE_BF16,
                                        ctypes.byref(nbytes), None) == L.FA_ERR_UNSUPPORTED
    # fp64: 16-key tiles (KVTPB=4 -> 64-key splits, the reference's own), fp64 partials only
    assert lib.fa_fwd_v2_workspace_size(1, 1, 100, 64, 4, L.FA_DTYPE_FP64, L.FA_DTYPE_FP64,
                                        ctypes.byref(nbytes), ctypes.byref(ns)) == 0
    assert ns.value == 2 and nbytes.value == 2 * 100 * 64 * 8 + 1792  # + lse (1600 B, 256-aligned)
    assert lib.fa_fwd_v2_workspace_size(1, 1, 100, 64, 4, L.FA_DTYPE_FP64, L.FA_DTYPE_FP32,
                                        ctypes.byref(nbytes), None) == L.FA_ERR_UNSUPPORTED
    # automatic split (FA_KV_TILES_AUTO; no device here -> the MI355X's 256 CUs assumed)
    assert lib.fa_fwd_v2_workspace_size(32, 8, 4096, 128, L.FA_KV_TILES_AUTO, L.FA_DTYPE_BF16,
                                        L.FA_DTYPE_FP32, ctypes.byref(nbytes), ctypes.byref(ns)) == 0
    assert ns.value == 1  # 8192 query tiles already fill the device
    assert lib.fa_fwd_v2_workspace_size(1, 1, 4096, 128, L.FA_KV_TILES_AUTO, L.FA_DTYPE_BF16,
                                        L.FA_DTYPE_FP32, ctypes.byref(nbytes), ctypes.byref(ns)) == 0
    assert ns.value == 8  # 32 query tiles x 8 splits of 8 KV tiles: one workgroup per CU
    fake = ctypes.c_void_p(0x10000)
    st = lib.fa_fwd_v2(fake, fake, fake, fake, 1, 1, 100, 64, 32, 32, 1, fake, 16, L.FA_DTYPE_FP16,
                       L.FA_DTYPE_FP32, NULL)
    assert st == L.FA_ERR_WORKSPACE and b"workspace" in lib.fa_last_error()


def test_partial_and_combine_checks():
    lib = L.lib()
    fake = ctypes.c_void_p(0x10000)
    st = lib.fa_fwd_partial(fake, fake, fake, fake, fake, 1, 1, 100, 50, 64, 30, L.FA_DTYPE_BF16,
                            L.FA_DTYPE_FP32, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"chunk_rows" in lib.fa_last_error()
    st = lib.fa_combine(fake, fake, fake, 0, 1, 1, 100, 64, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32, NULL)
    assert st == L.FA_ERR_INVALID_ARG


def test_partial_and_combine_alignment():
    """fa_combine moves 16 B per lane through o_part / o; lse is read per element (float,
    {lse, e} float pairs for scaled fp16, double for fp64): misaligned buffers are refused."""
    lib = L.lib()
    a16, a8, a4 = ctypes.c_void_p(0x10000), ctypes.c_void_p(0x10008), ctypes.c_void_p(0x10004)
    S = L.FA_DTYPE_FP16_SCALED
    for o_part, o in ((a8, a16), (a16, a4)):
        st = lib.fa_combine(o_part, a16, o, 2, 1, 1, 64, 64, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32, NULL)
        assert st == L.FA_ERR_INVALID_ARG and b"16-byte" in lib.fa_last_error()
    st = lib.fa_combine(a16, a4, a16, 2, 1, 1, 64, 64, L.FA_DTYPE_BF16, S, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"lse" in lib.fa_last_error()
    st = lib.fa_combine(a16, ctypes.c_void_p(0x10002), a16, 2, 1, 1, 64, 64, L.FA_DTYPE_BF16,
                        L.FA_DTYPE_FP32, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"lse" in lib.fa_last_error()
    st = lib.fa_fwd_partial(a16, a16, a16, a16, a4, 1, 1, 64, 64, 64, 64, L.FA_DTYPE_BF16, S, NULL)
    assert st == L.FA_ERR_INVALID_ARG and b"lse" in lib.fa_last_error()
    st = lib.fa_fwd_partial(a16, a16, a16, a16, a4, 1, 1, 64, 64, 64, 64, L.FA_DTYPE_FP64, L.FA_DTYPE_FP64, NULL)
    assert st == L.FA_ERR_INVALID_ARG


def test_split_grid_bound():
    """One workgroup per (query tile, split, b*h): a grid past 2^31-1 is refused with
    FA_ERR_UNSUPPORTED (never truncated to 32 bits), before any launch."""
    lib = L.lib()
    nbytes, ns = ctypes.c_size_t(), ctypes.c_int()
    # B*H = 2^16, L = 2^20, one workgroup per key block (blocks_per_workgroup = 1):
    # 8192 query tiles x 16384 one-tile splits x 65536 heads
    st = lib.fa_fwd_v2_workspace_size_ex(256, 256, 1 << 20, 64, 1, 1, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32,
                                         ctypes.byref(nbytes), ctypes.byref(ns))
    assert st == L.FA_ERR_UNSUPPORTED and b"2^31-1" in lib.fa_last_error()
    fake = ctypes.c_void_p(0x10000)
    st = lib.fa_fwd_v2_ex(fake, fake, fake, fake, 256, 256, 1 << 20, 64, 32, 32, 1, 1, fake, 1 << 40,
                          None, None, None, 0.125, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32, NULL)
    assert st == L.FA_ERR_UNSUPPORTED
    # the same shape with long splits fits: 8192 x 1 x 65536 < 2^31
    st = lib.fa_fwd_v2_workspace_size_ex(256, 256, 1 << 20, 64, 1 << 14, 1, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32,
                                         ctypes.byref(nbytes), ctypes.byref(ns))
    assert st == 0 and ns.value == 1
    # scheduled normally, the blocks of a query tile share workgroups and the grid fits
    st = lib.fa_fwd_v2_workspace_size(256, 256, 1 << 20, 64, 1, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32,
                                      ctypes.byref(nbytes), ctypes.byref(ns))
    assert st == 0 and ns.value == 16384


def test_python_check_raises_typed_errors():
    lib = L.lib()
    with pytest.raises(L.FaArgumentError) as ei:
        L.check(lib.fa_fwd_v1(NULL, NULL, NULL, NULL, 1, 1, 64, 64, L.FA_DTYPE_BF16, NULL))
    assert isinstance(ei.value, ValueError) and ei.value.status == L.FA_ERR_INVALID_ARG


def test_ops_reject_host_tensors():
    import torch
    from exploring_flash_attention_amd import ops
    q = torch.zeros(1, 1, 64, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.attention_v1(q, q, q)


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        L.lib()


def test_dist_library_exports():
    """libfa_mi355x_dist.so (RCCL path) exports every function of include/fa_mi355x_dist.h."""
    import ctypes
    path = os.path.join(os.path.dirname(L.LIB_PATH), "libfa_mi355x_dist.so")
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "fa_mi355x_dist.h")).read()
    names = re.findall(r"^(?:int|const char\*)\s+(fa_\w+)\(", hdr, flags=re.M)
    assert len(names) == 6, names
    out = os.popen(f"nm -D --defined-only {path}").read()
    for name in names:
        assert re.search(rf"\bT {name}$", out, flags=re.M), name
    from exploring_flash_attention_amd import dist as fadist
    lib = fadist.dist_lib()
    nbytes = ctypes.c_size_t()
    assert lib.fa_fwd_v2_dist_workspace_size(2, 2, 100, 64, 3, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32,
                                             ctypes.byref(nbytes)) == L.FA_ERR_INVALID_ARG  # 100 % 3
    assert b"divisible" in lib.fa_dist_last_error()
    assert lib.fa_fwd_v2_dist_workspace_size(2, 2, 96, 64, 4, L.FA_DTYPE_BF16, L.FA_DTYPE_FP32,
                                             ctypes.byref(nbytes)) == 0
    rows = 4 * 96
    assert nbytes.value == 2 * (rows * 64 * 4 + rows * 4) + rows * 64 * 2


def test_product_build_carries_no_experiments():
    """The product library is the shipped kernels only: no experiment or ablation knobs in the
    kernel sources it is built from, no experimental entry points, and the split schedule
    depends on arguments only (no environment lookups in the C ABI)."""
    csrc = os.path.join(ROOT, "exploring_flash_attention_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    srcs = re.search(r"^SRCS\s*=\s*(.*)$", mk, flags=re.M).group(1).split()
    assert "fa_fwd_w64.hip" not in srcs
    for f in srcs + ["fa_fwd_kernel.hpp", "fa_fwd16_kernel.hpp", "fa_device.hpp", "fa_internal.hpp"]:
        text = open(os.path.join(csrc, f)).read()
        for knob in ("FA_ABL_", "FA_PP", "FA_SGB", "FA_QSPLIT", "FA_QSCALE", "FA_IGLP", "FA_W64", "FA16_",
                     "FA_SHAPE16", "getenv"):
            assert knob not in text, (f, knob)
    out = os.popen(f"nm -D --defined-only {L.LIB_PATH}").read()
    assert "fa_fwd_v1_w64" not in out and "fa_fwd_v2_ex" in out


def test_dist_argument_and_error_paths():
    """fa_fwd_v2_dist / fa_dist_comm_* refuse bad arguments before any RCCL or HIP work (CPU:
    no device, so a communicator cannot be made and says so)."""
    from exploring_flash_attention_amd import dist as fadist
    lib = fadist.dist_lib()
    fake = ctypes.c_void_p(0x10000)
    st = lib.fa_fwd_v2_dist(fake, fake, fake, fake, 1, 1, 64, 128, None, 0, fake, 1 << 20,
                            L.FA_DTYPE_BF16, L.FA_DTYPE_FP16_SCALED, None)
    assert st == L.FA_ERR_INVALID_ARG and b"comm" in lib.fa_dist_last_error()
    assert lib.fa_dist_get_unique_id(None) == L.FA_ERR_INVALID_ARG
    comm = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(128)
    assert lib.fa_dist_comm_init(ctypes.byref(comm), 2, 2, uid) == L.FA_ERR_INVALID_ARG
    assert lib.fa_dist_comm_init(ctypes.byref(comm), 0, 0, uid) == L.FA_ERR_INVALID_ARG
    assert lib.fa_dist_comm_init(None, 1, 0, uid) == L.FA_ERR_INVALID_ARG
    st = lib.fa_dist_comm_init(ctypes.byref(comm), 1, 0, uid)
    assert st != L.FA_OK and not comm.value  # no device here: an error, never a half-made handle
    assert lib.fa_dist_comm_destroy(None) == L.FA_OK
    nbytes = ctypes.c_size_t()
    assert lib.fa_fwd_v2_dist_workspace_size(1, 1, 64, 128, 2, L.FA_DTYPE_FP64, L.FA_DTYPE_FP32,
                                             ctypes.byref(nbytes)) == L.FA_ERR_UNSUPPORTED


def test_d_tile_defaults():
    """None d tiles: min(32, d) up to d = 256 (the reference's D_TILE), 128 for the d-tiled
    kernel's wide head dims (24 vs 6 chunk waits per key tile; the result is the same)."""
    from exploring_flash_attention_amd import ops
    assert ops._d_tiles(16, None, None) == (16, 16)
    assert ops._d_tiles(128, None, None) == (32, 32)
    assert ops._d_tiles(256, None, 64) == (32, 64)
    assert ops._d_tiles(384, None, None) == (128, 128)
    assert ops._d_tiles(512, 32, None) == (32, 128)


def test_v2_ex2_flags_validated():
    """fa_fwd_v2_ex2 (ABI 0.4): an unknown flag bit is refused before anything is checked or
    launched; FA_V2_COUNTERS_ZERO is the only flag."""
    lib = L.lib()
    st = lib.fa_fwd_v2_ex2(None, None, None, None, 1, 1, 256, 128, 32, 32, 4, 0, None, 0, None, None, None,
                           1.0 / 128 ** 0.5, L.FA_DTYPE_BF16, L.FA_DTYPE_FP16_SCALED, 2, None)
    assert st == L.FA_ERR_INVALID_ARG and b"flags" in lib.fa_last_error()
    st = lib.fa_fwd_v2_ex2(None, None, None, None, 1, 1, 256, 128, 32, 32, 4, 0, None, 0, None, None, None,
                           1.0 / 128 ** 0.5, L.FA_DTYPE_BF16, L.FA_DTYPE_FP16_SCALED, L.FA_V2_COUNTERS_ZERO, None)
    assert st == L.FA_ERR_INVALID_ARG and b"null" in lib.fa_last_error()  # the flag itself is accepted
