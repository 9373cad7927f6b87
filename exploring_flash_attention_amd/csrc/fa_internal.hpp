// fa_internal.hpp -- shared definitions between the gfx950 kernels (fa_fwd.hip,
// fa_combine.hip) and the C-ABI dispatch layer (fa_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>

namespace fa {

// Geometry of the forward kernel: a wave owns one block of 32 query rows (one 32x32x16 MFMA
// column block), a workgroup 4 waves = 128 rows, KV tiles of 64 keys (32 at d = 256).
// (64 rows per wave -- one wave per SIMD, every K / V fragment feeding two MFMAs -- and 8-wave
// workgroups were measured slower; they live in git history.)
constexpr int bk_for(int d) { return d <= 128 ? 64 : 32; }
constexpr int kRB = 1;
constexpr int kRowsPerWave = 32 * kRB;
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kBQ = kWaves * kRowsPerWave;
// waves per SIMD the register budget is sized for (d = 256 holds 64 Q and 128 O registers
// per lane: one wave per SIMD)
constexpr int waves_per_simd(int d) { return d > 128 ? 1 : 2; }
// Row sums on the 16x16x32 MFMA (fa_fwd_kernel.hpp) at d = 32 / 64 / 128; at d = 32 only in
// the final no-tail contiguous kernel.  Those kernels are held to the occupancy the VALU-sum
// kernels reach (d = 32: four waves per SIMD, d = 64: three); kernel_wps = the launch bound
// of an instantiation = workgroups per CU (4 waves per workgroup, one per SIMD).
constexpr int d_bit(int d) { return d == 32 ? 1 : d == 64 ? 2 : d == 128 ? 4 : 8; }
constexpr int kRowsum16Mask = 0x7;
constexpr bool rs16_on(int d, int mode, bool tail, bool strided) {
    return (kRowsum16Mask & d_bit(d)) != 0 && (d > 32 || (mode == 0 && !tail && !strided));
}
// (d = 32 at three waves per SIMD: 147 VGPRs, no scratch, C2 49.8 -> 50.4 us -- the 60 B of
// scratch at four are spilled around the last KV step only; profiles/r06/ab_c2_wps3_noscratch.txt)
constexpr int kernel_wps(int d, int mode, bool tail, bool strided) {
    return rs16_on(d, mode, tail, strided) && d <= 32 ? 4
           : rs16_on(d, mode, tail, strided) && d == 64 ? 3
                                                        : waves_per_simd(d);
}

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
    // d-tiled kernels (d = 384 / 512): effective column chunks of K and V (32, 64 or 128)
    int d_tile_qk, d_tile_v;
    // fused split mode: the order of the work items in the (remapped) block index, as groups of
    // tile_group query tiles (dividing nqt) whose splits are consecutive -- 0 or nqt: query tile
    // fastest (the tiles of one key block share its K / V in L2), 1: split fastest (the splits
    // of one query tile run together: Q re-read from L2, partials combined while hot), between:
    // both, for a group of tiles
    int tile_group;
    // fused split mode, fa_fwd16_kernel: arrival counted before the partial stores, so that the
    // last arriver never stores its own (fa_fwd16_kernel.hpp); 0: stores first
    int arrive_first;
};

// (query tile, split, b*h) of work item w (after xcd_remap)
__device__ __forceinline__ void decode_item(const FwdArgs& a, int w, int& qt, int& split, int64_t& bh) {
    const int G = a.tile_group;
    if (G <= 0 || G >= a.nqt) {  // (b*h, split, query tile)
        qt = w % a.nqt;
        const int rest = w / a.nqt;
        split = rest % a.nsplit;
        bh = rest / a.nsplit;
    } else if (G == 1) {  // (b*h, query tile, split)
        split = w % a.nsplit;
        const int rest = w / a.nsplit;
        qt = rest % a.nqt;
        bh = rest / a.nqt;
    } else {  // (b*h, tile group, split, tile in group)
        const int qi = w % G;
        int rest = w / G;
        split = rest % a.nsplit;
        rest /= a.nsplit;
        const int ng = a.nqt / G;
        qt = (rest % ng) * G + qi;
        bh = rest / ng;
    }
}

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
// compute units of the device that owns `s` (the current device for the null stream;
// fa_capi.cpp; 256 without a device)
int device_cus(hipStream_t s = nullptr);
// The kernels a C-ABI call enqueued, for fa_last_kernels() (fa_capi.cpp): every launcher
// names the kernel it picked and its grid, so callers (bench.py) report what ran instead of
// restating the launch rules.
void note_kernel(const char* name, int64_t grid);
// the forward kernels' labels (string literals: nothing allocated on the launch path)
inline const char* kernel_label(bool k16, int mode, bool strided) {
    static const char* const names[2][3][2] = {
        {{"fa_fwd_kernel<final>", "fa_fwd_kernel<final, strided>"},
         {"fa_fwd_kernel<partial>", "fa_fwd_kernel<partial, strided>"},
         {"fa_fwd_kernel<fused split, in-kernel combine>", "fa_fwd_kernel<fused split, in-kernel combine, strided>"}},
        {{"fa_fwd16_kernel<final>", "fa_fwd16_kernel<final, strided>"},
         {"fa_fwd16_kernel<partial>", "fa_fwd16_kernel<partial, strided>"},
         {"fa_fwd16_kernel<fused split, in-kernel combine>",
          "fa_fwd16_kernel<fused split, in-kernel combine, strided>"}}};
    return names[k16 ? 1 : 0][mode < 0 || mode > 2 ? 0 : mode][strided ? 1 : 0];
}
// fp64 mode (fa_fwd64.hip): 64 query rows x 16-key tiles; final or row-layout partial
hipError_t launch_fwd64(int d, Mode mode, const FwdArgs& a, hipStream_t s);
hipError_t launch_combine64(int d, const CombineArgs& a, hipStream_t s);
int fwd64_rows_per_block();
int fwd64_keys_per_tile();
// d-tiled forward for d = 384 / 512 (fa_fwd_dtiled.hip; fp64: fa_fwd64.hip), final mode,
// contiguous [B, H, L, d]; FwdArgs::nqt counts dtiled_rows_per_block() rows per query tile
hipError_t launch_fwd_dtiled(Elem t, int d, const FwdArgs& a, hipStream_t s);
hipError_t launch_fwd64_dtiled(int d, const FwdArgs& a, hipStream_t s);
int dtiled_rows_per_block();
int dtiled_lds_bytes(int d);
// the wide-d kernel serving (dtype, d): query rows per workgroup, threads, dynamic LDS bytes
void dtiled_geometry(Elem e, int d, int* rows, int* threads, int* lds);

}  // namespace fa
