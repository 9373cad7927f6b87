// MFMA peak microbenchmark (confirm the bf16 dense peak on the box).
// Every wave issues back-to-back v_mfma_f32_32x32x16_bf16 on 4 independent accumulators
// (no VALU, no memory in the loop), 2 waves per SIMD on every CU.  Reports the achieved
// TFLOP/s, the shader clock the chip held (s_memtime cycles over s_memrealtime's 100 MHz
// wall clock, per workgroup) and the peak those imply (4096 FLOP / clk / CU x CUs x clock).
//   hipcc -O3 --offload-arch=gfx950 scripts/mfma_peak.hip -o scripts/bin/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* sink, unsigned long long* clk, int iters) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (threadIdx.x + j));
        b[j] = (__bf16)(0.002f * (threadIdx.x - j));
    }
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
    if (s == 12345.678f) sink[threadIdx.x] = s;  // keeps the chain live
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// The same loop on RANDOM operands: 8 A and 8 B fragments per lane (hash-generated bf16 in
// [-2, 2)), a different (A, B) pair for every MFMA, as an attention or GEMM inner loop feeds
// them.  Constant operands let the chip hold a higher clock (MI355X_MICROARCH.md, DVFS
// give-back): this is the ceiling a random-data kernel can approach at the clock it holds.
__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__global__ __launch_bounds__(256) void mfma_loop_rand(float* sink, unsigned long long* clk, int iters) {
    bf16x8 a[8], b[8];
    for (int f = 0; f < 8; ++f)
        for (int j = 0; j < 8; ++j) {
            const unsigned h = hash32(threadIdx.x * 977u + blockIdx.x * 7919u + f * 131u + j);
            a[f][j] = (__bf16)((float)(h & 0xffff) / 16384.f - 2.f);
            b[f][j] = (__bf16)((float)(h >> 16) / 16384.f - 2.f);
        }
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i += 2) {
#pragma unroll
        for (int f = 0; f < 8; f += 4) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f], b[f], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 1], b[f + 1], c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 2], b[f + 2], c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[f + 3], b[f + 3], c3, 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
    if (s == 12345.678f) sink[threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// Operand patterns on the same random fragments (which operand changes from one MFMA to the
// next): MFMA k of a group of 8 reads A fragment ia(k) and B fragment ib(k).
//   0 both change every MFMA (= mfma_loop_rand)       1 A repeats in pairs (k, k+1), B changes
//   2 B repeats in pairs, A changes (the QK^T order)  3 A constant, B changes
//   4 B constant, A changes                           5 both constant (random values)
template <int MODE>
__global__ __launch_bounds__(256) void mfma_loop_pattern(float* sink, unsigned long long* clk, int iters) {
    bf16x8 a[8], b[8];
    for (int f = 0; f < 8; ++f)
        for (int j = 0; j < 8; ++j) {
            const unsigned h = hash32(threadIdx.x * 977u + blockIdx.x * 7919u + f * 131u + j);
            a[f][j] = (__bf16)((float)(h & 0xffff) / 16384.f - 2.f);
            b[f][j] = (__bf16)((float)(h >> 16) / 16384.f - 2.f);
        }
    f32x16 c[4] = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i += 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int ia = MODE == 1 ? (k & ~1) : MODE == 3 || MODE == 5 ? 0 : k;
            const int ib = MODE == 2 ? (k & ~1) : MODE == 4 || MODE == 5 ? 0 : k;
            c[k & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ia], b[ib], c[k & 3], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += c[0][j] + c[1][j] + c[2][j] + c[3][j];
    if (s == 12345.678f) sink[threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <typename K>
static int run(K kernel, const char* label, int ncu, int khz) {
    const int blocks = ncu * 2;  // 2 x 4 waves per CU = 2 waves per SIMD
    const int iters = 20000;
    float* sink;
    unsigned long long* clk;
    (void)hipMalloc(&sink, 256 * sizeof(float));
    (void)hipMalloc(&clk, 2 * blocks * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) kernel<<<blocks, 256>>>(sink, clk, iters);  // clock ramp
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) kernel<<<blocks, 256>>>(sink, clk, iters);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) return 1;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long* h = new unsigned long long[2 * blocks];
    (void)hipMemcpy(h, clk, 2 * blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mhz_sum = 0.0;
    for (int i = 0; i < blocks; ++i) mhz_sum += (double)h[2 * i] / ((double)h[2 * i + 1] / 100.0);
    const double mhz = mhz_sum / blocks;  // s_memrealtime ticks at 100 MHz
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * 4.0) * reps;
    const double tflops = flops / (ms * 1e-3) / 1e12;
    printf("{\"operands\": \"%s\", \"cus\": %d, \"rated_clock_mhz\": %.0f, \"held_clock_mhz\": %.0f, "
           "\"mfma_bf16_tflops\": %.1f, \"peak_at_rated_clock_tflops\": %.1f, \"peak_at_held_clock_tflops\": %.1f, "
           "\"kernel\": \"4 independent v_mfma_f32_32x32x16_bf16 chains per wave, 2 waves per SIMD\"}\n",
           label, ncu, khz / 1000.0, mhz, tflops, 4096.0 * ncu * khz * 1e3 / 1e12, 4096.0 * ncu * mhz * 1e6 / 1e12);
    delete[] h;
    return 0;
}

int main_rand_and_const() {
    int dev = 0, ncu = 0, khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev);
    if (run(mfma_loop, "constant", ncu, khz)) return 1;
    if (run(mfma_loop_rand, "random", ncu, khz)) return 1;
    if (run(mfma_loop_pattern<1>, "random, A repeated in pairs", ncu, khz)) return 1;
    if (run(mfma_loop_pattern<2>, "random, B repeated in pairs", ncu, khz)) return 1;
    if (run(mfma_loop_pattern<3>, "random, A constant", ncu, khz)) return 1;
    if (run(mfma_loop_pattern<4>, "random, B constant", ncu, khz)) return 1;
    return run(mfma_loop_pattern<5>, "random values, both constant", ncu, khz);
}

int main() { return main_rand_and_const(); }

int main_constant_only() {
    int dev = 0, ncu = 0, khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev);
    const int blocks = ncu * 2;  // 2 x 4 waves per CU = 2 waves per SIMD
    const int iters = 20000;
    float* sink;
    unsigned long long* clk;
    (void)hipMalloc(&sink, 256 * sizeof(float));
    (void)hipMalloc(&clk, 2 * blocks * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) mfma_loop<<<blocks, 256>>>(sink, clk, iters);  // clock ramp
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) mfma_loop<<<blocks, 256>>>(sink, clk, iters);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) return 1;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long* h = new unsigned long long[2 * blocks];
    (void)hipMemcpy(h, clk, 2 * blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mhz_sum = 0.0;
    for (int i = 0; i < blocks; ++i) mhz_sum += (double)h[2 * i] / ((double)h[2 * i + 1] / 100.0);
    const double mhz = mhz_sum / blocks;  // s_memrealtime ticks at 100 MHz
    const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * 4.0) * reps;
    const double tflops = flops / (ms * 1e-3) / 1e12;
    printf("{\"cus\": %d, \"rated_clock_mhz\": %.0f, \"held_clock_mhz\": %.0f, \"mfma_bf16_tflops\": %.1f, "
           "\"peak_at_rated_clock_tflops\": %.1f, \"peak_at_held_clock_tflops\": %.1f, "
           "\"kernel\": \"4 independent v_mfma_f32_32x32x16_bf16 chains per wave, 2 waves per SIMD\"}\n",
           ncu, khz / 1000.0, mhz, tflops, 4096.0 * ncu * khz * 1e3 / 1e12, 4096.0 * ncu * mhz * 1e6 / 1e12);
    return 0;
}
