// fa_probe.hip -- libfa_probe.so: the MFMA ceiling the forward kernels are measured against.
// Not part of the forward's C ABI (include/fa_mi355x.h): bench.py loads it to report, beside
// roofline.frac against the 2.5 PF datasheet figure, the fraction of what the chip sustains on
// the MFMA shape the d = 128 kernel issues (v_mfma_f32_16x16x32_bf16) when the operands are
// random data, as attention operands are (MI355X_MICROARCH.md, DVFS give-back: the operand
// values set the MFMA array's power, hence the clock the chip holds).  SURVEY.md section 8(d).
//
// One kernel per (shape, operand pattern): 4 independent accumulation chains per wave, nothing
// else in the loop, `waves_per_simd` x 4 waves per CU.  Operand patterns (fragments are 8 random
// bf16 in [-2, 2) per lane, 8 A and 8 B fragments; MFMA k of a group of 8 reads A[ia(k)],
// B[ib(k)]):
//   0  constant small positive values (the datasheet-style loop: the chip holds ~2.1 GHz)
//   1  random, a new (A, B) pair every MFMA
//   2  random, A repeated in pairs -- the QK^T order of fa_fwd16_kernel (one K fragment feeds
//      the wave's two query blocks) and of its P.V (one V^T operand, two P^T blocks)
//   3  random values, both operands constant
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int SHAPE> struct Acc;
template <> struct Acc<0> { using T = f32x16; };  // v_mfma_f32_32x32x16_bf16
template <> struct Acc<1> { using T = f32x4; };   // v_mfma_f32_16x16x32_bf16

template <int SHAPE>
__device__ __forceinline__ typename Acc<SHAPE>::T mma(bf16x8 a, bf16x8 b, typename Acc<SHAPE>::T c) {
    if constexpr (SHAPE == 0)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int SHAPE, int PAT>
__global__ __launch_bounds__(256) void mfma_ceiling(float* sink, unsigned long long* clk, int iters) {
    using A = typename Acc<SHAPE>::T;
    bf16x8 a[8], b[8];
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (PAT == 0) {
                a[f][j] = (__bf16)(0.001f * (threadIdx.x + j));
                b[f][j] = (__bf16)(0.002f * (threadIdx.x - j));
            } else {
                const unsigned h = hash32(threadIdx.x * 977u + blockIdx.x * 7919u + f * 131u + j);
                a[f][j] = (__bf16)((float)(h & 0xffff) / 16384.f - 2.f);
                b[f][j] = (__bf16)((float)(h >> 16) / 16384.f - 2.f);
            }
        }
    A c0 = {}, c1 = {}, c2 = {}, c3 = {};
    constexpr bool CONST = PAT == 0 || PAT == 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i += 8) {
        // MFMA k of 8: A[ia(k)], B[ib(k)], accumulator k % 4
#define FA_PROBE_MMA(K, C)                                                              \
        C = mma<SHAPE>(a[PAT == 2 ? ((K) & ~1) : CONST ? 0 : (K)], b[CONST ? 0 : (K)], C);
        FA_PROBE_MMA(0, c0) FA_PROBE_MMA(1, c1) FA_PROBE_MMA(2, c2) FA_PROBE_MMA(3, c3)
        FA_PROBE_MMA(4, c0) FA_PROBE_MMA(5, c1) FA_PROBE_MMA(6, c2) FA_PROBE_MMA(7, c3)
#undef FA_PROBE_MMA
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < (int)(sizeof(A) / 4); ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
    if (s == 12345.678f) sink[threadIdx.x] = s;  // keeps the chains live
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int SHAPE>
void* pick(int pat) {
    switch (pat) {
        case 0: return (void*)&mfma_ceiling<SHAPE, 0>;
        case 1: return (void*)&mfma_ceiling<SHAPE, 1>;
        case 2: return (void*)&mfma_ceiling<SHAPE, 2>;
        case 3: return (void*)&mfma_ceiling<SHAPE, 3>;
        default: return nullptr;
    }
}

}  // namespace

extern "C" {

// Runs the ceiling loop `reps` times back to back (after `warm` untimed launches that let the
// clock settle) on the current device and stream 0.  out[0] = bf16 TFLOP/s (HIP events over
// the timed launches), out[1] = the shader clock held (MHz: s_memtime over s_memrealtime's
// 100 MHz, mean over workgroups of the last launch), out[2] = FLOPs per launch.
// shape: 0 = v_mfma_f32_32x32x16_bf16, 1 = v_mfma_f32_16x16x32_bf16; pattern: see above.
// Returns 0, or 1 on a bad argument, 2 on a HIP error.
int fa_probe_mfma_ceiling(int shape, int pattern, int waves_per_simd, int iters, int warm, int reps,
                          double* out) {
    if ((shape != 0 && shape != 1) || pattern < 0 || pattern > 3 || waves_per_simd < 1 || waves_per_simd > 2 ||
        iters < 8 || iters % 8 || warm < 0 || reps < 1 || !out)
        return 1;
    void* fn = shape == 0 ? pick<0>(pattern) : pick<1>(pattern);
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 2;
    const int blocks = ncu * waves_per_simd;  // 4 waves per block: waves_per_simd waves per SIMD
    float* sink = nullptr;
    unsigned long long* clk = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    if (hipMalloc(&sink, 256 * sizeof(float)) != hipSuccess ||
        hipMalloc(&clk, 2 * (size_t)blocks * sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
        rc = 2;
    } else {
        void* args[] = {&sink, &clk, &iters};
        for (int w = 0; w < warm && rc == 0; ++w)
            if (hipLaunchKernel(fn, dim3(blocks), dim3(256), args, 0, 0) != hipSuccess) rc = 2;
        if (rc == 0 && hipEventRecord(e0, 0) != hipSuccess) rc = 2;
        for (int r = 0; r < reps && rc == 0; ++r)
            if (hipLaunchKernel(fn, dim3(blocks), dim3(256), args, 0, 0) != hipSuccess) rc = 2;
        float ms = 0.f;
        if (rc == 0 && (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                        hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
            rc = 2;
        if (rc == 0) {
            unsigned long long* h = new unsigned long long[2 * (size_t)blocks];
            if (hipMemcpy(h, clk, 2 * (size_t)blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) {
                rc = 2;
            } else {
                double mhz = 0.0;
                for (int i = 0; i < blocks; ++i) mhz += (double)h[2 * i] / ((double)h[2 * i + 1] / 100.0);
                const double per_mfma = shape == 0 ? 2.0 * 32 * 32 * 16 : 2.0 * 16 * 16 * 32;
                const double launch_flops = per_mfma * iters * 4.0 * blocks;  // 4 waves per block
                out[0] = launch_flops * reps / (ms * 1e-3) / 1e12;
                out[1] = mhz / blocks;
                out[2] = launch_flops;
            }
            delete[] h;
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (sink) (void)hipFree(sink);
    if (clk) (void)hipFree(clk);
    return rc;
}

}  // extern "C"
