// fa_fwd_strided.hip -- launchers of the forward kernel (fa_fwd_kernel.hpp) on strided
// tensors: [B, H, L, d] views with arbitrary (batch, head, row) element strides and a
// contiguous d, e.g. the [B, L, H, d] layout most frameworks keep, with no copy.  Final mode
// (FA-v1 fused / d-tiled), the fused split-KV mode (FA-v2) and the row-layout partial mode
// (fa_fwd_partial_ex: one chunk of query rows per launch in the multi-GPU path).  d = 128
// with whole 64-key tiles runs fa_fwd16_kernel's strided form, every other case
// fa_fwd_kernel's.
#include "fa_fwd_kernel.hpp"
#include "fa_fwd16_kernel.hpp"

namespace fa {

template <typename T, typename PT, int D, int MODE>
static hipError_t launch_strided_one(const FwdArgs& a, hipStream_t s) {
    const int64_t nblk = (int64_t)a.nqt * a.nsplit * a.BH;
    const int lds = fwd_lds_bytes(D);
    // d = 128 with whole 64-key tiles in every split (the multi-GPU q row ranges, [B, L, H, d]
    // views, ...): the 16x16x32 kernel with strided addressing -- the same bits as the
    // contiguous launch (round 4; the 32x32x16 kernel below sums in another order)
    if constexpr (D == 128) {
        if (a.Lk % bk_for(D) == 0 && a.kv_per_split % bk_for(D) == 0) {
            note_kernel(kernel_label(true, MODE, true), nblk);
            hipLaunchKernelGGL((fa_fwd16_kernel<T, PT, D, MODE, true>), dim3((unsigned)nblk), dim3(kThreads), lds, s, a);
            return hipGetLastError();
        }
    }
    note_kernel(kernel_label(false, MODE, true), nblk);
    if (a.Lk % bk_for(D))
        hipLaunchKernelGGL((fa_fwd_kernel<T, PT, D, MODE, true, true>), dim3((unsigned)nblk), dim3(kThreads),
                           lds, s, a);
    else
        hipLaunchKernelGGL((fa_fwd_kernel<T, PT, D, MODE, false, true>), dim3((unsigned)nblk), dim3(kThreads),
                           lds, s, a);
    return hipGetLastError();
}

template <typename T, typename PT, int MODE>
static hipError_t launch_strided_d(int d, const FwdArgs& a, hipStream_t s) {
    switch (d) {
        case 32: return launch_strided_one<T, PT, 32, MODE>(a, s);
        case 64: return launch_strided_one<T, PT, 64, MODE>(a, s);
        case 128: return launch_strided_one<T, PT, 128, MODE>(a, s);
        case 256: return launch_strided_one<T, PT, 256, MODE>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fwd_strided(Elem t, Elem pt, int d, Mode mode, const FwdArgs& a, hipStream_t s) {
    if (mode == kFinal) {
        if (t == Elem::BF16) return launch_strided_d<__bf16, __bf16, kFinal>(d, a, s);
        if (t == Elem::F16) return launch_strided_d<_Float16, _Float16, kFinal>(d, a, s);
        return hipErrorInvalidValue;
    }
    auto pick = [&](auto mode_c) -> hipError_t {
        constexpr int M = decltype(mode_c)::value;
        if (t == Elem::BF16 && pt == Elem::BF16) return launch_strided_d<__bf16, __bf16, M>(d, a, s);
        if (t == Elem::BF16 && pt == Elem::F32) return launch_strided_d<__bf16, float, M>(d, a, s);
        if (t == Elem::F16 && pt == Elem::F16) return launch_strided_d<_Float16, _Float16, M>(d, a, s);
        if (t == Elem::F16 && pt == Elem::F32) return launch_strided_d<_Float16, float, M>(d, a, s);
        {  // per-row scaled fp16 partials
            if (t == Elem::BF16 && pt == Elem::F16S) return launch_strided_d<__bf16, f16s_t, M>(d, a, s);
            if (t == Elem::F16 && pt == Elem::F16S) return launch_strided_d<_Float16, f16s_t, M>(d, a, s);
        }
        return hipErrorInvalidValue;
    };
    if (mode == kFused) return pick(std::integral_constant<int, kFused>{});
    if (mode == kPartial) return pick(std::integral_constant<int, kPartial>{});
    return hipErrorInvalidValue;
}

}  // namespace fa
