"""Pin the CPU oracle against the reference's own outputs (golden fixtures).

The fixtures were produced by importing the reference's Python in the build container
(tests/golden/make_golden.py); these tests need neither the reference nor a GPU.
"""
import ctypes

import numpy as np
import pytest

from conftest import golden
from oracle import fa_v1, reference, splitkv, tiled_d
from oracle.batched import attention_fp64

TIGHT = 1e-12  # fp64 restatement vs fp64 reference: only summation order differs


def test_naive_attention_matches_reference_naive():
    for name in ("g1_v1_basic_f64.npz", "g1_v1_basic_ragged.npz", "g3_tiled_d_f64.npz",
                 "g4_v2_d128.npz"):
        g = golden(name)
        np.testing.assert_allclose(reference.naive_attention(g["Q"], g["K"], g["V"]), g["O_naive"],
                                   rtol=0, atol=TIGHT)


def test_v1_basic_restatement_matches_reference():
    for name in ("g1_v1_basic_f64.npz", "g1_v1_basic_ragged.npz"):
        g = golden(name)
        bk = 16 if "ragged" in name else 8
        O = fa_v1.flash_attention_tiled(g["Q"], g["K"], g["V"], Bq=8, Bk=bk)
        np.testing.assert_allclose(O, g["O"], rtol=0, atol=TIGHT)


def test_v1_basic_restatement_fp16_matches_reference():
    g = golden("g1_v1_basic_f16.npz")
    O = fa_v1.flash_attention_tiled(g["Q"], g["K"], g["V"], Bq=8, Bk=8)
    assert O.dtype == np.float16
    # same fp16 arithmetic sequence; allow a couple of fp16 ulps for BLAS order
    np.testing.assert_allclose(O.astype(np.float64), g["O"].astype(np.float64), rtol=0, atol=4e-3)


@pytest.mark.parametrize("name", ["g2_v1_opt2_L64_d32.npz", "g2_v1_opt2_L40_d16.npz"])
def test_opt2_restatement_matches_reference(name):
    g = golden(name)
    L, d = g["Q"].shape
    O = np.zeros(L * d)
    fa_v1.flash_attention_tiled_flat(g["Q"].ravel(), g["K"].ravel(), g["V"].ravel(), O, L, d,
                                     Bq=int(g["Bq"]), Bk=int(g["Bk"]))
    np.testing.assert_allclose(O.reshape(L, d), g["O"], rtol=0, atol=TIGHT)


def test_tiled_d_restatement_matches_reference():
    g = golden("g3_tiled_d_f64.npz")
    for (bq, bk, dq, dv) in ((8, 8, 16, 16), (16, 16, 32, 32)):
        O = tiled_d.flash_attention_tiled_global(g["Q"], g["K"], g["V"], bq, bk, dq, dv)
        np.testing.assert_allclose(O, g[f"O_{bq}_{bk}_{dq}_{dv}"], rtol=0, atol=TIGHT)


def test_tiled_d_asserts_like_reference():
    g = golden("g3_tiled_d_f64.npz")
    with pytest.raises(AssertionError):
        tiled_d.flash_attention_tiled_global(g["Q"], g["K"], g["V"], 8, 8, 256, 16)
    with pytest.raises(AssertionError):
        tiled_d.flash_attention_tiled_global(g["Q"], g["K"][:10], g["V"], 8, 8, 16, 16)


@pytest.mark.parametrize("d", [32, 128])
def test_splitkv_restatement_matches_reference(d):
    g = golden(f"g4_v2_d{d}.npz")
    L = g["Q"].shape[0]
    for kvtpb in (1, 4):
        O = np.zeros(L * d)
        wO, wm, wl = {}, {}, {}
        splitkv.flash_attention_tiled_v2(g["Q"].ravel(), g["K"].ravel(), g["V"].ravel(), O, wO, wm, wl,
                                         L, d, 8, 8, 16, 16, kvtpb)
        # the reference's float32 combine scales (numpy_gpu_like.py:277) bound agreement at ~1e-7
        np.testing.assert_allclose(O.reshape(L, d), g[f"O_kvtpb{kvtpb}"], rtol=0, atol=1e-12)
        if d == 32 and kvtpb == 4:
            nq, nkb = g["ws_O"].shape[:2]
            for q in range(nq):
                for b in range(nkb):
                    np.testing.assert_allclose(wO[(q, b)], g["ws_O"][q, b], rtol=0, atol=TIGHT)
                    np.testing.assert_allclose(wm[(q, b)], g["ws_m"][q, b], rtol=0, atol=TIGHT)
                    np.testing.assert_allclose(wl[(q, b)], g["ws_l"][q, b], rtol=0, atol=TIGHT)


def test_lse_form_equals_reference_workspace_combine():
    """The (normalised O, base-2 lse) partial form of the GPU library combines to the same O
    as the reference's (O_acc, m, l) workspace; lse_k = log2(l_k) + m_k * log2(e)."""
    g = golden("g4_v2_d32.npz")
    wsO, wsm, wsl = g["ws_O"], g["ws_m"], g["ws_l"]  # [nq][nkb][Bq*d], [nq][nkb][Bq]
    nq, nkb, bq = wsm.shape
    d = g["Q"].shape[1]
    O_parts = (wsO.reshape(nq, nkb, bq, d) / wsl[..., None]).transpose(1, 0, 2, 3).reshape(nkb, nq * bq, d)
    lses = (wsm * splitkv.LOG2E + np.log2(wsl)).transpose(1, 0, 2).reshape(nkb, nq * bq)
    np.testing.assert_allclose(splitkv.combine_lse(O_parts, lses), g["O_naive"], rtol=0, atol=1e-12)


def test_partial_lse_combine_equals_naive():
    rng = np.random.default_rng(5)
    Q, K, V = (rng.standard_normal((2, 3, 48, 32)) for _ in range(3))
    parts = [splitkv.partial_lse(Q, K[..., s:s + 16, :], V[..., s:s + 16, :]) for s in (0, 16, 32)]
    O = splitkv.combine_lse([p[0] for p in parts], [p[1] for p in parts])
    np.testing.assert_allclose(O, attention_fp64(Q, K, V), rtol=0, atol=1e-12)


def test_batched_matches_naive():
    g = golden("g4_v2_d128.npz")
    np.testing.assert_allclose(attention_fp64(g["Q"], g["K"], g["V"], q_chunk=16), g["O_naive"],
                               rtol=0, atol=TIGHT)


def test_check_accuracy_restatement():
    ref = np.ones((4, 4))
    assert reference.check_accuracy(ref + 1e-3, ref)["max_abs"] == pytest.approx(1e-3)
    with pytest.raises(AssertionError, match="Max absolute difference"):
        reference.check_accuracy(ref + 0.02, ref)
    with pytest.raises(AssertionError, match="Mean relative error"):
        reference.check_accuracy(ref * 1.06, ref, max_abs_tol=1.0)


def test_driver_random_reproduces_fixture(oracle_lib):
    """oracle_driver_random == driver.cu initialize_random after srand(42) (glibc rand)."""
    for d in (32, 128):
        g = golden(f"g5_driver_d{d}.npz")
        n = g["Q"].size
        buf = np.empty(3 * n, np.float32)
        oracle_lib.oracle_driver_random(buf.ctypes.data, 3 * n, 42, 1)
        x = buf.astype(np.float16)
        np.testing.assert_array_equal(x[:n].reshape(g["Q"].shape), g["Q"])
        np.testing.assert_array_equal(x[2 * n:].reshape(g["V"].shape), g["V"])


def test_standard_attention_c_restatement(oracle_lib):
    """C restatement of standard_attention_cpu vs the reference naive_attention fixtures."""
    for d in (32, 128):
        g = golden(f"g5_driver_d{d}.npz")
        Q, K, V = g["Q"], g["K"], g["V"]  # keep the arrays alive across the C call
        B, H, L, _ = Q.shape
        O = np.empty_like(Q)
        oracle_lib.oracle_standard_attention(Q.ctypes.data, K.ctypes.data, V.ctypes.data,
                                             O.ctypes.data, B, H, L, d, 0)
        err = np.abs(O.astype(np.float64) - g["O"]).max()
        assert err < 1e-3, err  # fp32 math + fp16 output rounding


def test_half_bfloat_conversions(oracle_lib):
    x = np.array([0.0, -0.0, 1.0, -2.5, 1e-6, 6.1e-5, 65504.0, 70000.0, 3.14159265, 1e-8],
                 dtype=np.float32)
    h = np.empty(x.size, np.uint16)
    oracle_lib.oracle_to_storage(x.ctypes.data, h.ctypes.data, x.size, 0)
    np.testing.assert_array_equal(h, x.astype(np.float16).view(np.uint16))
    back = np.empty_like(x)
    oracle_lib.oracle_from_storage(h.ctypes.data, back.ctypes.data, x.size, 0)
    np.testing.assert_array_equal(back, x.astype(np.float16).astype(np.float32))
    import torch
    b = np.empty(x.size, np.uint16)
    oracle_lib.oracle_to_storage(x.ctypes.data, b.ctypes.data, x.size, 1)
    ref = torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(b, ref)
    _ = ctypes  # keep import used


def test_tiled_d_restatement_at_a_wide_head_dim():
    """g6 (d = 384, ragged d tiles 100 / 96): the reference's own tiled-d output at a head dim
    past one tile, the case the d-tiled kernels (csrc/fa_fwd_dtiled.hip) serve."""
    g = golden("g6_tiled_d_d384.npz")
    Q, K, V = (g[n].astype(np.float64) / 16 for n in ("Q16", "K16", "V16"))
    O = tiled_d.flash_attention_tiled_global(Q, K, V, 8, 8, 100, 96)
    np.testing.assert_allclose(O, g["O_100_96"], rtol=0, atol=TIGHT)
    np.testing.assert_allclose(g["O_naive"], g["O_100_96"], rtol=0, atol=TIGHT)
