// fa_internal.hpp -- shared definitions between the gfx950 kernels (fa_fwd.hip,
// fa_combine.hip) and the C-ABI dispatch layer (fa_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>

namespace fa {

// Keys per KV tile and query rows per wave of the forward kernel.  A wave owns kRB
// blocks of 32 query rows (one 32x32x16 MFMA column block each) and every K / V
// fragment it reads from LDS feeds kRB MFMAs; a workgroup has kWaves waves.
//   kRB = 1: 32 rows per wave, <= 256 registers, two waves per SIMD (default);
//   kRB = 2: 64 rows per wave, ~460 registers, ONE wave per SIMD -- halves the LDS
//            fragment traffic per MFMA, but hipcc's schedule for it (AGPR shuffling, no
//            second wave to hide latency) measured 1.6x slower at C3 (profiles/).
#ifndef FA_WAVES
#define FA_WAVES 4
#endif
#ifndef FA_RB
#define FA_RB 1
#endif
// Keys per KV tile, per head dim (a multiple of 32).  Small d has registers to spare and
// is bound by per-tile overheads, so it takes longer tiles.
#ifndef FA_BK32
#define FA_BK32 (FA_RB == 1 ? 64 : 32)
#endif
#ifndef FA_BK64
#define FA_BK64 (FA_RB == 1 ? 64 : 32)
#endif
#ifndef FA_BK128
#define FA_BK128 (FA_RB == 1 ? 64 : 32)
#endif
#ifndef FA_BK256
#define FA_BK256 32
#endif
constexpr int bk_for(int d) {
    return d <= 32 ? FA_BK32 : d <= 64 ? FA_BK64 : d <= 128 ? FA_BK128 : FA_BK256;
}
constexpr int kRB = FA_RB;
constexpr int kRowsPerWave = 32 * kRB;
constexpr int kWaves = FA_WAVES;
constexpr int kThreads = kWaves * 64;
constexpr int kBQ = kWaves * kRowsPerWave;
constexpr int kWavesPerSimd = kRB == 1 ? 2 : 1;  // occupancy the register budget is sized for
// d = 256 holds 64 Q and 128 O registers per lane: one wave per SIMD, AGPRs in use
constexpr int waves_per_simd(int d) { return d > 128 ? 1 : kWavesPerSimd; }

enum class Elem : int { F16 = 0, BF16 = 1, F32 = 2, F64 = 3, F16S = 4 };
// F16S (split-KV partials only): fp16 values scaled per row by a power of two 2^-e so that the
// row's largest |value| is below 1, e stored beside the lse -- half the bytes of fp32 with
// 11 significant bits relative to the row maximum and no fp16 range limit
struct f16s_t {
    _Float16 x;
};

// Arguments of the forward kernel (final and partial modes share one struct).
struct FwdArgs {
    const void* q;           // [BH][Lq][D]
    const void* k;           // [BH][Lk][D]
    const void* v;           // [BH][Lk][D]
    void* o;                 // final: [BH][Lq][D] (T); partial: o_part (PT), see below
    float* lse;              // partial only: log2-sum-exp per row
    int64_t BH;
    int64_t Lq;
    int64_t Lk;
    int nqt;                 // query tiles per head = ceil(Lq / kBQ)
    int nsplit;              // key splits per head
    int kv_per_split;        // keys per split, multiple of bk_for(d) (Lk for a single split)
    int64_t chunk_rows;      // partial: output row chunking (divides Lq)
    int64_t split_stride;    // partial: elements between splits of o_part
    float scale_log2;        // log2(e) / sqrt(d)
    // fused split mode only: the last workgroup of each (query tile, b*h) to finish combines
    // the splits (see fa_fwd.hip); o / lse then hold the workspace in fragment order
    unsigned* counters;      // [BH][nqt], zero before the launch; left zero after it
    float* esc;              // F16S partials: per-row scale exponents, laid out as lse
    void* o_final;           // [BH][Lq][D] (T)
    // fp64 mode (fa_fwd64.hip)
    double scale_log2_64;    // log2(e) / sqrt(d) in double
    double* lse64;           // partial only: log2-sum-exp per row (double)
    // strided tensors (final and fused split modes of fa_fwd_kernel): element strides of
    // (batch, head, row); d is contiguous and V shares K's strides.  strided == 0: contiguous
    // [B, H, L, d] and these are unused.
    int strided;
    int64_t H;
    int64_t q_stride[3], k_stride[3], o_stride[3];
};

// Kernel modes: one workgroup per (query tile, split, b*h) in all three.
enum Mode : int {
    kFinal = 0,    // single split, writes O
    kPartial = 1,  // writes normalised partial O + lse in row layout (fa_combine reads them)
    kFused = 2,    // writes partials in fragment order; the last split to finish combines
};

struct CombineArgs {
    const void* o_part;      // [nsplit][rows][D] (PT)
    const float* lse;        // [nsplit][rows]
    void* o;                 // [rows][D] (T)
    int64_t rows;            // BH * L
    int nsplit;
    const double* lse64;     // fp64 mode: [nsplit][rows] (double)
};

// Launchers (defined in the .hip files).  Return hipSuccess or the launch error.
hipError_t launch_fwd(Elem t, Elem pt, int d, Mode mode, const FwdArgs& a, hipStream_t s);
hipError_t launch_combine(Elem t, Elem pt, int d, const CombineArgs& a, hipStream_t s);
// the strided instantiations (fa_fwd_strided.hip); launch_fwd forwards there when a.strided
hipError_t launch_fwd_strided(Elem t, Elem pt, int d, Mode mode, const FwdArgs& a, hipStream_t s);
int fwd_lds_bytes(int d);
// d = 128 final mode with 64 rows per wave (fa_fwd_w64.hip); FA_W64 selects it
#ifndef FA_W64
#define FA_W64 0  // measured: steady state equal to fa_fwd_kernel, per-item seam 1.5x
#endif
hipError_t launch_fwd_w64(Elem t, const FwdArgs& a, hipStream_t s);
int w64_rows_per_block();
// fp64 mode (fa_fwd64.hip): 64 query rows x 16-key tiles; final or row-layout partial
hipError_t launch_fwd64(int d, Mode mode, const FwdArgs& a, hipStream_t s);
hipError_t launch_combine64(int d, const CombineArgs& a, hipStream_t s);
int fwd64_rows_per_block();
int fwd64_keys_per_tile();

}  // namespace fa
