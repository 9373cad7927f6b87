// fa_fwd.hip -- launchers of the forward kernel (fa_fwd_kernel.hpp) on contiguous
// [B, H, L, d] tensors; strided tensors go to fa_fwd_strided.hip (a separate translation
// unit, so the two instantiation sets compile in parallel).
#define FA_FWD_MAIN_TU
#include "fa_fwd_kernel.hpp"
#include "fa_fwd16_kernel.hpp"
#include "fa_fwd16_chain.hpp"

#ifndef FA_CHAIN
#define FA_CHAIN 1  // d = 128 final mode: the chained persistent grid (fa_fwd16_chain.hpp)
#endif


namespace fa {

int fwd_lds_bytes(int d) { return 2 * 2 * bk_for(d) * d * 2; }

template <typename T, typename PT, int D, int MODE>
static hipError_t launch_one(const FwdArgs& a, hipStream_t s) {
    const int64_t nblk = (int64_t)a.nqt * a.nsplit * a.BH;
    const int lds = fwd_lds_bytes(D);
    // d = 128 without a key tail: the 16x16x32 kernel (fa_fwd16_kernel.hpp; C3 +5 %, C4 +3.4 %,
    // the C5 partial pass +9 % over this file's 32x32x16 kernel)
    if constexpr (D == 128) {
        if constexpr ((MODE == kFinal && std::is_same_v<T, PT>) || (MODE == kFused && std::is_same_v<PT, f16s_t>)) {
            // whole chains of query tiles (final), or of the key blocks of query tiles (fused,
            // scaled fp16 partials, each tile combined by its own workgroup): an even number >= 4
            // of 64-key tiles per key block, whole query tiles, and at least one query tile per
            // workgroup of a 2-per-CU grid
            const int64_t grid = 2 * (int64_t)device_cus(s) / 8 * 8;
            const int64_t kvi = MODE == kFused ? a.kv_per_split : a.Lk;
            const int64_t tiles = (int64_t)a.nqt * a.BH;
            if (FA_CHAIN && kvi % 128 == 0 && kvi >= 256 && a.Lk % kvi == 0 && a.Lq % kBQ == 0 &&
                (MODE == kFused || a.nsplit == 1) && tiles >= grid && grid >= 8 && nblk < (int64_t)1 << 31) {
                note_kernel(MODE == kFinal ? "fa_fwd16_chain_kernel<final>" : "fa_fwd16_chain_kernel<fused walk>", grid);
                hipLaunchKernelGGL((fa_fwd16_chain_kernel<T, MODE>), dim3((unsigned)grid), dim3(kThreads),
                                   lds, s, a, (int)tiles);
                return hipGetLastError();
            }
        }
        if (a.Lk % bk_for(D) == 0 && a.kv_per_split % bk_for(D) == 0) {  // no key tail in any split
            note_kernel(kernel_label(true, MODE, false), nblk);
            hipLaunchKernelGGL((fa_fwd16_kernel<T, PT, D, MODE>), dim3((unsigned)nblk), dim3(kThreads), lds, s, a);
            return hipGetLastError();
        }
    }
    note_kernel(kernel_label(false, MODE, false), nblk);
    if (a.Lk % bk_for(D) || !(kNoTailMask & d_bit(D)))
        hipLaunchKernelGGL((fa_fwd_kernel<T, PT, D, MODE, true>), dim3((unsigned)nblk), dim3(kThreads),
                           lds, s, a);
    else
        hipLaunchKernelGGL((fa_fwd_kernel<T, PT, D, MODE, false>), dim3((unsigned)nblk), dim3(kThreads),
                           lds, s, a);
    return hipGetLastError();
}

template <typename T, typename PT, int MODE>
static hipError_t launch_d(int d, const FwdArgs& a, hipStream_t s) {
#ifdef FA_LITE_D  // (scripts/build_lite.sh: one head dim, bf16 only, for fast A/B builds)
    if constexpr (std::is_same_v<T, __bf16>)
        return d == FA_LITE_D ? launch_one<T, PT, FA_LITE_D, MODE>(a, s) : hipErrorInvalidValue;
    return hipErrorInvalidValue;
#else
    switch (d) {
        case 32: return launch_one<T, PT, 32, MODE>(a, s);
        case 64: return launch_one<T, PT, 64, MODE>(a, s);
        case 128: return launch_one<T, PT, 128, MODE>(a, s);
        case 256: return launch_one<T, PT, 256, MODE>(a, s);
        default: return hipErrorInvalidValue;
    }
#endif
}

hipError_t launch_fwd(Elem t, Elem pt, int d, Mode mode, const FwdArgs& a, hipStream_t s) {
    if (a.strided) return launch_fwd_strided(t, pt, d, mode, a, s);
    if (mode == kFinal) {
        if (t == Elem::BF16) return launch_d<__bf16, __bf16, kFinal>(d, a, s);
        if (t == Elem::F16) return launch_d<_Float16, _Float16, kFinal>(d, a, s);
        return hipErrorInvalidValue;
    }
    auto pick = [&](auto mode_c) -> hipError_t {
        constexpr int M = decltype(mode_c)::value;
        if (t == Elem::BF16 && pt == Elem::BF16) return launch_d<__bf16, __bf16, M>(d, a, s);
        if (t == Elem::BF16 && pt == Elem::F32) return launch_d<__bf16, float, M>(d, a, s);
        if (t == Elem::F16 && pt == Elem::F16) return launch_d<_Float16, _Float16, M>(d, a, s);
        if (t == Elem::F16 && pt == Elem::F32) return launch_d<_Float16, float, M>(d, a, s);
        {  // per-row scaled fp16 partials
            if (t == Elem::BF16 && pt == Elem::F16S) return launch_d<__bf16, f16s_t, M>(d, a, s);
            if (t == Elem::F16 && pt == Elem::F16S) return launch_d<_Float16, f16s_t, M>(d, a, s);
        }
        return hipErrorInvalidValue;
    };
    if (mode == kPartial) return pick(std::integral_constant<int, kPartial>{});
    if (mode == kFused) return pick(std::integral_constant<int, kFused>{});
    return hipErrorInvalidValue;
}

}  // namespace fa
