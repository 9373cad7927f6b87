// fa_combine.hip -- split-KV combine for MI355X (gfx950).
//
// <- reduction_kernel  flash_attention_v2/CUDA/flash_attention_v2.h:356-435
// <- reduction_kernel  flash_attention_v2/numpy_gpu_like.py:229-288
// The reference combines UNnormalised partials with their (m_k, l_k):
//   M = max_k m_k;  s_k = e^(m_k - M);  O = sum_k s_k O_k / sum_k s_k l_k.
// The partial kernel here stores O_k / l_k and lse_k = m_k + log l_k (base 2), so the
// same quantity is  O = sum_k 2^(lse_k - M') (O_k/l_k) / sum_k 2^(lse_k - M').
//
// HBM-bound streaming kernel: one thread owns 8 consecutive columns of one row
// (16-byte loads for 16-bit partials, 2 x 16 bytes for fp32), rows are contiguous.
#include "fa_internal.hpp"

namespace fa {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ float to_f(unsigned short u) {
    return (float)__builtin_bit_cast(T, u);
}
template <typename T>
__device__ __forceinline__ unsigned short from_f(float f) {
    return __builtin_bit_cast(unsigned short, static_cast<T>(f));
}

template <typename T, typename PT, int D>
__global__ __launch_bounds__(256) void fa_combine_kernel(CombineArgs a) {
    constexpr int TPR = D / 8;  // threads per row
    using PH = std::conditional_t<std::is_same_v<PT, f16s_t>, _Float16, T>;  // 16-bit element
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = gid / TPR;
    const int c8 = (int)(gid % TPR) * 8;
    if (row >= a.rows) return;

    // scaled fp16 partials: {lse, e} per row, values stored as O/l * 2^-e
    constexpr bool SCALED = std::is_same_v<PT, f16s_t>;
    constexpr int LS = SCALED ? 2 : 1;
    float mx = -INFINITY;
    // scaled partials: the weights carry 2^(e_s - E), E = the largest exponent, and 2^E is
    // applied after the division (2^e_s itself overflows fp32 for rows near the bf16 maximum)
    int emax = -1000;
    for (int s = 0; s < a.nsplit; ++s) {
        mx = fmaxf(mx, a.lse[LS * (s * a.rows + row)]);
        if constexpr (SCALED) emax = max(emax, (int)a.lse[2 * (s * a.rows + row) + 1]);
    }

    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float wsum = 0.f;
    for (int s = 0; s < a.nsplit; ++s) {
        float wgt = __builtin_amdgcn_exp2f(a.lse[LS * (s * a.rows + row)] - mx);
        wsum += wgt;
        if constexpr (SCALED) wgt = __builtin_amdgcn_ldexpf(wgt, (int)a.lse[2 * (s * a.rows + row) + 1] - emax);
        const int64_t base = ((int64_t)s * a.rows + row) * D + c8;
        if constexpr (sizeof(PT) == 4) {
            const f32x4 x0 = *(const f32x4*)((const float*)a.o_part + base);
            const f32x4 x1 = *(const f32x4*)((const float*)a.o_part + base + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j] += wgt * x0[j];
                acc[4 + j] += wgt * x1[j];
            }
        } else {
            const u32x4 x = *(const u32x4*)((const unsigned short*)a.o_part + base);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[2 * j] += wgt * to_f<PH>((unsigned short)(x[j] & 0xffff));
                acc[2 * j + 1] += wgt * to_f<PH>((unsigned short)(x[j] >> 16));
            }
        }
    }
    const float inv = 1.f / wsum;
    auto fin = [&](float x) { return SCALED ? __builtin_amdgcn_ldexpf(x * inv, emax) : x * inv; };
    u32x4 out;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        out[j] = (unsigned)from_f<T>(fin(acc[2 * j])) | ((unsigned)from_f<T>(fin(acc[2 * j + 1])) << 16);
    *(u32x4*)((unsigned short*)a.o + row * D + c8) = out;
}

template <typename T, typename PT>
static hipError_t launch_c(int d, const CombineArgs& a, hipStream_t s) {
    const int64_t threads = a.rows * (d / 8);
    const dim3 grid((unsigned)((threads + 255) / 256));
    note_kernel("fa_combine_kernel", grid.x);
    switch (d) {
        case 32: hipLaunchKernelGGL((fa_combine_kernel<T, PT, 32>), grid, dim3(256), 0, s, a); break;
        case 64: hipLaunchKernelGGL((fa_combine_kernel<T, PT, 64>), grid, dim3(256), 0, s, a); break;
        case 128: hipLaunchKernelGGL((fa_combine_kernel<T, PT, 128>), grid, dim3(256), 0, s, a); break;
        case 256: hipLaunchKernelGGL((fa_combine_kernel<T, PT, 256>), grid, dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_combine(Elem t, Elem pt, int d, const CombineArgs& a, hipStream_t s) {
    if (t == Elem::BF16 && pt == Elem::BF16) return launch_c<__bf16, __bf16>(d, a, s);
    if (t == Elem::BF16 && pt == Elem::F32) return launch_c<__bf16, float>(d, a, s);
    if (t == Elem::F16 && pt == Elem::F16) return launch_c<_Float16, _Float16>(d, a, s);
    if (t == Elem::F16 && pt == Elem::F32) return launch_c<_Float16, float>(d, a, s);
    if (t == Elem::BF16 && pt == Elem::F16S) return launch_c<__bf16, f16s_t>(d, a, s);
    if (t == Elem::F16 && pt == Elem::F16S) return launch_c<_Float16, f16s_t>(d, a, s);
    return hipErrorInvalidValue;
}

}  // namespace fa
