// fa_capi.cpp -- the C ABI (include/fa_mi355x.h): argument validation, workspace
// arithmetic and dispatch to the gfx950 kernels.  No allocation, no device sync.
//
// Validation mirrors the reference launchers' asserts, turned into status codes:
//   B,H,L,d > 0                    flash_attention_v1/CUDA/flash_attention_v1.h:263
//   0 < d_tile_qk, d_tile_v <= d   flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:326-327
//   kv_tiles_per_block > 0         flash_attention_v2/CUDA/flash_attention_v2.h:447
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <atomic>

#include "../../include/fa_mi355x.h"
#include "fa_internal.hpp"

namespace fa {
// Compute units of the device that owns `s` (the current device for the null stream), queried
// once per device (the split planner runs on every fa_fwd_v2 call).  No device (CPU-only
// tests): the MI355X's 256.
int device_cus(hipStream_t s) {
    static std::atomic<int> cached[64];
    int dev = 0;
    hipError_t he = s ? hipStreamGetDevice(s, &dev) : hipGetDevice(&dev);
    if (he != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 256;
    }
    int n = cached[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = 256;
    }
    cached[dev].store(n, std::memory_order_relaxed);
    return n;
}

// fa_last_kernels(): what the last launching call of this thread enqueued
thread_local std::string g_kernels;
void kernels_begin() { g_kernels.clear(); }
void note_kernel(const char* name, int64_t grid) {
    if (!g_kernels.empty()) g_kernels += " + ";
    g_kernels += name;
    g_kernels += " [grid " + std::to_string(grid) + "]";
}
}  // namespace fa

namespace {

using fa::device_cus;
using fa::kernels_begin;

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int ok() {
    g_err.clear();
    return FA_OK;
}

bool supported_d(int64_t d) { return d == 32 || d == 64 || d == 128 || d == 256; }
// head dims past one tile: the d-tiled kernels (fa_fwd_dtiled.hip, fa_fwd64.hip), final mode only
bool wide_d(int64_t d) { return d == 384 || d == 512; }
// a d tile as the d-tiled kernels take it: 32, 64 or 128 columns (the request rounded down to
// one of them, at least 32: a QK^T k-step is 32 columns; all three divide 384 and 512)
int dtile_eff(int dt) { return dt >= 128 ? 128 : dt >= 64 ? 64 : 32; }

int check_dtype(int dtype, fa::Elem* e) {
    if (dtype == FA_DTYPE_BF16) { *e = fa::Elem::BF16; return FA_OK; }
    if (dtype == FA_DTYPE_FP16) { *e = fa::Elem::F16; return FA_OK; }
    if (dtype == FA_DTYPE_FP64) { *e = fa::Elem::F64; return FA_OK; }
    return fail(FA_ERR_UNSUPPORTED,
                "dtype %d has no kernel (use FA_DTYPE_BF16, FA_DTYPE_FP16 or FA_DTYPE_FP64)", dtype);
}

int check_partial_dtype(int pdtype, int dtype, fa::Elem* e) {
    if (dtype == FA_DTYPE_FP64) {
        if (pdtype == FA_DTYPE_FP64) { *e = fa::Elem::F64; return FA_OK; }
        return fail(FA_ERR_UNSUPPORTED, "fp64 inputs take fp64 partials (got partial dtype %d)", pdtype);
    }
    if (pdtype == FA_DTYPE_FP32) { *e = fa::Elem::F32; return FA_OK; }
    if (pdtype == FA_DTYPE_FP16_SCALED) { *e = fa::Elem::F16S; return FA_OK; }
    if (pdtype == dtype) return check_dtype(dtype, e);
    return fail(FA_ERR_UNSUPPORTED,
                "partial dtype %d must be FA_DTYPE_FP32, FA_DTYPE_FP16_SCALED or the input dtype %d", pdtype, dtype);
}

int check_shape(int64_t B, int64_t H, int64_t L, int64_t d, bool wide = false) {
    if (B <= 0 || H <= 0 || L <= 0 || d <= 0)
        return fail(FA_ERR_INVALID_ARG, "all dimensions must be positive (B=%lld H=%lld L=%lld d=%lld)",
                    (long long)B, (long long)H, (long long)L, (long long)d);
    if (!supported_d(d) && !(wide && wide_d(d)))
        return fail(FA_ERR_UNSUPPORTED, "head dim d=%lld has no kernel here (supported: 32, 64, 128, 256%s)",
                    (long long)d, wide ? ", 384, 512" : "; 384 and 512 through the FA-v1 / tiled-d / unsplit v2 paths");
    if (L > (int64_t)1 << 30)
        return fail(FA_ERR_UNSUPPORTED, "L=%lld exceeds 2^30", (long long)L);
    const int64_t nqt = (L + 63) / 64;  // the smallest query tile of any kernel
    if (B * H * nqt > (int64_t)0x7fffffff)
        return fail(FA_ERR_UNSUPPORTED, "grid of %lld workgroups exceeds 2^31-1", (long long)(B * H * nqt));
    return FA_OK;
}

int check_ptrs(const void* q, const void* k, const void* v, const void* o) {
    if (!q || !k || !v || !o) return fail(FA_ERR_INVALID_ARG, "null tensor pointer");
    if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15)
        return fail(FA_ERR_INVALID_ARG, "tensor pointers must be 16-byte aligned");
    return FA_OK;
}

int check_d_tiles(int64_t d, int d_tile_qk, int d_tile_v) {
    if (d_tile_qk <= 0 || d_tile_qk > d || d_tile_v <= 0 || d_tile_v > d)
        return fail(FA_ERR_INVALID_ARG, "need 0 < d_tile_qk, d_tile_v <= d (got %d, %d, d=%lld)",
                    d_tile_qk, d_tile_v, (long long)d);
    return FA_OK;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(FA_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

// query rows per workgroup and keys per KV tile of the kernel serving dtype e (and head dim d)
int rows_per_block(fa::Elem e, int64_t d = 128) {
    if (e == fa::Elem::F64) return fa::fwd64_rows_per_block();  // (its d-tiled kernel's too)
    return wide_d(d) ? fa::dtiled_rows_per_block() : fa::kBQ;
}
int keys_per_tile(fa::Elem e, int64_t d) {
    if (e == fa::Elem::F64) return fa::fwd64_keys_per_tile();
    return wide_d(d) ? 64 : fa::bk_for((int)d);
}

fa::FwdArgs base_args(const void* q, const void* k, const void* v, void* o, int64_t BH,
                      int64_t Lq, int64_t Lk, int64_t d, fa::Elem e) {
    fa::FwdArgs a{};
    a.q = q; a.k = k; a.v = v; a.o = o; a.lse = nullptr;
    a.BH = BH; a.Lq = Lq; a.Lk = Lk;
    a.nqt = (int)((Lq + rows_per_block(e, d) - 1) / rows_per_block(e, d));
    a.scale_log2_64 = 1.4426950408889634 / std::sqrt((double)d);
    a.nsplit = 1;
    a.kv_per_split = (int)Lk;
    a.chunk_rows = Lq;
    a.split_stride = 0;
    a.scale_log2 = (float)(1.4426950408889634 / std::sqrt((double)d));
    return a;
}

// Strided views ([B, H, L, d] with element strides {batch, head, row}, d contiguous; NULL =
// contiguous).  Every row start must stay 16-byte aligned (the kernel loads 16 B per lane)
// and one head's rows must span < 2 GiB (32-bit buffer offsets).
int apply_strides(fa::FwdArgs& a, fa::Elem e, int64_t B, int64_t H, int64_t L, int64_t d,
                  const int64_t* qs, const int64_t* kvs, const int64_t* os, int64_t Lk = -1) {
    a.H = H;
    if (!qs && !kvs && !os) return FA_OK;
    if (e == fa::Elem::F64) return fail(FA_ERR_UNSUPPORTED, "strided tensors: bf16 / fp16 only");
    if (Lk < 0) Lk = L;
    const int64_t contig[3] = {H * L * d, L * d, d}, contig_k[3] = {H * Lk * d, Lk * d, d};
    const int64_t* st[3] = {qs ? qs : contig, kvs ? kvs : contig_k, os ? os : contig};
    const char* names[3] = {"q", "k/v", "o"};
    const int64_t rows[3] = {L, Lk, L};
    for (int t = 0; t < 3; ++t) {
        for (int i = 0; i < 3; ++i) {
            if (st[t][i] <= 0 || (st[t][i] * 2) % 16)
                return fail(FA_ERR_INVALID_ARG, "%s stride[%d]=%lld must be positive and a multiple of 8 elements",
                            names[t], i, (long long)st[t][i]);
        }
        if (st[t][2] < d)
            return fail(FA_ERR_INVALID_ARG, "%s row stride %lld < d=%lld", names[t], (long long)st[t][2], (long long)d);
        if (st[t][2] > (int64_t)1 << 28 || (rows[t] - 1) * st[t][2] * 2 + d * 2 > 0x7fffffffLL)
            return fail(FA_ERR_UNSUPPORTED, "%s: one head's rows span more than 2 GiB", names[t]);
        (void)B;
    }
    a.strided = 1;
    for (int i = 0; i < 3; ++i) {
        a.q_stride[i] = st[0][i];
        a.k_stride[i] = st[1][i];
        a.o_stride[i] = st[2][i];
    }
    return FA_OK;
}

// softmax_scale > 0 replaces 1/sqrt(d) (the scaled entry points: a caller that zero-pads the
// head dim to a kernel's d keeps the scale of the unpadded one)
int apply_scale(fa::FwdArgs& a, double softmax_scale) {
    if (!(softmax_scale > 0.0) || !std::isfinite(softmax_scale))
        return fail(FA_ERR_INVALID_ARG, "softmax_scale must be positive and finite (got %g)", softmax_scale);
    a.scale_log2_64 = 1.4426950408889634 * softmax_scale;
    a.scale_log2 = (float)a.scale_log2_64;
    return FA_OK;
}

// d = 384 / 512: the d-tiled kernels with the given (requested) d tiles; their query tile is
// rows_per_block(e, d) rows (dtiled_rows_per_block; the fp64 kernel's 64)
hipError_t launch_wide(fa::Elem e, int d, fa::FwdArgs a, int d_tile_qk, int d_tile_v, hipStream_t s) {
    a.nqt = (int)((a.Lq + rows_per_block(e, d) - 1) / rows_per_block(e, d));
    a.d_tile_qk = dtile_eff(d_tile_qk);
    a.d_tile_v = dtile_eff(d_tile_v);
    return e == fa::Elem::F64 ? fa::launch_fwd64_dtiled(d, a, s) : fa::launch_fwd_dtiled(e, d, a, s);
}

// final mode; wide head dims take the d-tiled kernels with their largest tiles
hipError_t launch_final(fa::Elem e, int d, const fa::FwdArgs& a, hipStream_t s) {
    if (wide_d(d)) return launch_wide(e, d, a, 128, 128, s);
    return e == fa::Elem::F64 ? fa::launch_fwd64(d, fa::kFinal, a, s) : fa::launch_fwd(e, e, d, fa::kFinal, a, s);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split-KV workspace (fused split mode): normalised partial O [S][BH][nqt][BQ*d] (PT) and
// lse [S][BH][nqt][BQ] (fp32), both in the kernel's fragment order, then one uint32
// counter per (b*h, query tile).  Every part 256-byte aligned.
struct V2Layout {
    size_t o_bytes, lse_off, esc_off, cnt_off, total;
    int64_t ngroups;
};
V2Layout v2_layout(int64_t BH, int64_t L, int64_t d, int ns, fa::Elem pe) {
    V2Layout w{};
    if (pe == fa::Elem::F64) {  // fp64: row-major partials + double lse, separate combine
        const size_t rows = (size_t)ns * BH * L;
        w.o_bytes = align256(rows * d * 8);
        w.lse_off = w.o_bytes;
        w.cnt_off = w.lse_off + align256(rows * 8);
        w.total = w.cnt_off;
        return w;
    }
    const int64_t nqt = (L + fa::kBQ - 1) / fa::kBQ;
    const size_t esz = pe == fa::Elem::F32 ? 4 : 2;
    const size_t rows = (size_t)ns * BH * nqt * fa::kBQ;
    w.ngroups = BH * nqt;
    w.o_bytes = align256(rows * d * esz);
    w.lse_off = w.o_bytes;
    w.esc_off = w.lse_off + align256(rows * sizeof(float));
    w.cnt_off = w.esc_off + (pe == fa::Elem::F16S ? align256(rows * sizeof(float)) : 0);
    w.total = w.cnt_off + align256((size_t)w.ngroups * sizeof(unsigned));
    return w;
}


// How many partial workgroups per query tile the split-KV schedule wants: none beyond the
// first when the query tiles alone give every CU a workgroup, otherwise enough for one per CU.
// (Measured, round 3: a single workgroup per CU -- one wave per SIMD -- already runs the d = 128
// loop at 0.88x the throughput of two; splitting B1 H2 L16384 (256 query tiles) into 8 partials
// per tile to reach two per CU lost 10 %, B2 H2 L16384 into 4 lost 13 %: every partial pays a
// prologue, an epilogue and its round trip through the workspace.  Splits pay when CUs idle.)
// Measured again in round 4 (scripts/split_sweep.py, profiles/r04/split_sweep.txt, d = 128
// bf16): once every partial still runs >= 4096 keys its overheads amortise and the second
// workgroup per CU pays after all -- B1 H1 L16384 4 partials per tile 121.8 us vs 2: 128.8;
// B1 H2 L16384 2 vs 1: 225.8 vs 238.5 us -- while shorter partials do not (B1 H1 L8192 8 vs 4:
// 49.1 vs 44.3 us; B1 H4 L4096 4 vs 2: 42.0 vs 41.5).  So for the d = 128 16-bit kernel: two
// workgroups per CU when the partials stay that long, one per CU otherwise.
int64_t wanted_partials(int64_t items, int64_t cap, int64_t L, int64_t d, fa::Elem e) {
    const int64_t ncu = device_cus();
    int64_t ns = items >= ncu ? 1 : (ncu + items - 1) / items;
    if (d == 128 && (e == fa::Elem::BF16 || e == fa::Elem::F16)) {
        const int64_t ns2 = items >= 2 * ncu ? 1 : (2 * ncu + items - 1) / items;
        if (ns2 > ns && L / ns2 >= 4096) ns = ns2;
    }
    return ns < cap ? ns : cap;
}

// FA_KV_TILES_AUTO: pick the split from occupancy: the KV tiles of a head
// cut into wanted_partials() equal splits.
int auto_kv_tiles(int64_t BH, int64_t L, int64_t d, fa::Elem e) {
    if (BH <= 0 || L <= 0 || !(supported_d(d) || wide_d(d))) return 1;  // the shape checks report these
    const int64_t bk = keys_per_tile(e, d);
    const int64_t ntiles = (L + bk - 1) / bk;
    const int64_t items = BH * ((L + rows_per_block(e, d) - 1) / rows_per_block(e, d));
    const int64_t ns = wanted_partials(items, ntiles, L, d, e);
    return (int)((ntiles + ns - 1) / ns);
}

// Split-KV scheduling.  The reference splits each head's keys into blocks of
// kv_tiles_per_block tiles, one partial per block, and reduces the partials
// (flash_attention_v2/CUDA/flash_attention_v2.h:243, :356).  Here consecutive blocks of a
// query tile are grouped onto one workgroup: the blocks of a group are combined on chip (the
// online softmax carried across them -- algebraically the reduction's formula, split after
// split), the groups' partials through the workspace and the in-kernel reduction.  By default
// (blocks_per_workgroup = FA_BLOCKS_PER_WG_AUTO) the blocks of a query tile are cut into
// wanted_partials() equal groups: a problem whose query tiles already give every CU a
// workgroup moves no partials through HBM at all, a short batch of long sequences gets just
// enough partials to occupy every CU; a positive blocks_per_workgroup fixes the group (1 =
// the reference's layout: one workgroup and one HBM partial per block).  Planned once per call: the workspace size, the
// grid and the split length all come from the same SplitPlan.
struct SplitPlan {
    int kvtpb;       // KV tiles per key block (FA_KV_TILES_AUTO resolved)
    int units;       // the reference's key blocks: ceil(L / (kv_tiles_per_block * bk))
    int group;       // blocks per workgroup
    int launched;    // partial workgroups per query tile: ceil(units / group)
    int kv_per_wg;   // keys per workgroup (group * block keys, at most L)
};
int plan_splits(int64_t BH, int64_t L, int64_t d, int kvtpb, int blocks_per_wg, fa::Elem e, SplitPlan* out) {
    if (kvtpb == FA_KV_TILES_AUTO) kvtpb = auto_kv_tiles(BH, L, d, e);
    if (kvtpb <= 0) return fail(FA_ERR_INVALID_ARG, "kv_tiles_per_block must be positive (got %d)", kvtpb);
    if (blocks_per_wg < 0)
        return fail(FA_ERR_INVALID_ARG, "blocks_per_workgroup must be >= 0 (0 = library schedule), got %d",
                    blocks_per_wg);
    SplitPlan p{};
    p.kvtpb = kvtpb;
    const int64_t keys = (int64_t)kvtpb * keys_per_tile(e, d);
    p.units = (int)((L + keys - 1) / keys);
    const int64_t items = BH * ((L + rows_per_block(e, d) - 1) / rows_per_block(e, d));
    p.group = 1;
    if (wide_d(d)) {
        p.group = p.units;  // d = 384 / 512: no split kernel -- every key block on one workgroup
    } else if (blocks_per_wg > 0) {
        p.group = blocks_per_wg < p.units ? blocks_per_wg : p.units;
    } else {
        const int64_t ns = wanted_partials(items, p.units, L, d, e);
        p.group = (int)((p.units + ns - 1) / ns);  // equal groups (the last one may be shorter)
    }
    p.launched = (p.units + p.group - 1) / p.group;
    const int64_t kw = keys * p.group;
    p.kv_per_wg = (int)(kw < L ? kw : L);
    *out = p;
    return FA_OK;
}

// Work order of the fused split launch (FwdArgs::tile_group): split fastest when the whole
// grid is one workgroup per CU and a query tile has at least 4 partials, query tile fastest
// otherwise.
// Measured (round 4, A/B in one process, profiles/r04/ab_split_order.log; outputs bitwise
// equal): B1 H2 L4096 (4 partials, 256 workgroups) 30.9 -> 28.9 us; B1 H1 L16384 (2 partials,
// 256) 132.2 -> 131.5 us; but B2 H2 L16384 (4 partials, 2048) -1.6 %, C4 with 4 partials per
// tile -4 %, C4 with 16 (the reference's one block per workgroup) -18 %: once workgroups queue,
// the 32 query tiles of one key block sharing its K / V in L2 matter more than the splits of
// one tile finishing together.
#ifndef FA_SPLIT_ORDER_RULE
#define FA_SPLIT_ORDER_RULE 2  // 0: query tile fastest always; 1: split fastest always; 2: the rule
#endif
// At >= 8 partials per tile (the reference's one-block-per-workgroup layout) groups of 4 query
// tiles with their splits consecutive: C4 at blocks_per_workgroup = 1 3448 -> 3334 us (groups
// of 8: 3361; profiles/r04/ab_tile_group.txt, outputs bitwise equal) -- a group's partials are
// combined while still in L2, and each key block's K / V still serves 4 tiles.  Groups of 2
// lost 9 % there; at 4 partials per tile the groups measured +0.9 % (C4, 4 blocks per
// workgroup) and -1.4 % (B2 H2 L16384) and stay off (profiles/r04/ab_tile_group_2.txt).
#ifndef FA_TILE_GROUP
#define FA_TILE_GROUP 4  // 0: off
#endif
#ifndef FA_TG_MIN
#define FA_TG_MIN 8  // partials per tile from which queued grids take the tile groups
#endif
int tile_group(int64_t nblk, int ns, int nqt) {
    if (FA_SPLIT_ORDER_RULE != 2) return FA_SPLIT_ORDER_RULE == 1 ? 1 : 0;
    // Split fastest only when the whole grid is ONE workgroup per CU (B1 H2 L4096: 256): at two
    // per CU (B1 H1 L16384, 4 partials, 512 workgroups) the two orders measured within 0.5 %
    // (122.4 vs 122.9 us, profiles/r04/ab_split_order_g.log) but split fastest puts every key
    // on every XCD -- 110 MB of L2 egress per launch against ~68 MB query tile fastest
    // (round 5: VERDICT r4 item 6)
    if (ns >= 4 && nblk <= (int64_t)device_cus()) return 1;
    if (FA_TILE_GROUP > 1 && ns >= FA_TG_MIN && nqt % FA_TILE_GROUP == 0) return FA_TILE_GROUP;
    return 0;
}

// workspace bytes for a plan (the grid bound checked too)
int v2_workspace(int64_t B, int64_t H, int64_t L, int64_t d, const SplitPlan& sp, fa::Elem e, fa::Elem pe,
                 size_t* bytes) {
    const int ns = sp.launched;
    // one workgroup per (query tile, split group, b*h): the grid and the kernel's block index
    // are 32-bit (dim3, xcd_remap), so a grid past 2^31-1 is refused instead of truncated
    const int64_t nqt = (L + rows_per_block(e, d) - 1) / rows_per_block(e, d);
    if (B * H * nqt > (int64_t)0x7fffffff / ns)
        return fail(FA_ERR_UNSUPPORTED, "split-KV grid of %lld x %d workgroups exceeds 2^31-1 "
                    "(raise kv_tiles_per_block)", (long long)(B * H * nqt), ns);
    // the in-kernel combine counts arrivals and completions in 16-bit halves of one counter
    if (ns > 0xffff)
        return fail(FA_ERR_UNSUPPORTED, "split-KV with %d partials per query tile exceeds 65535 "
                    "(raise kv_tiles_per_block)", ns);
    // one partial workgroup per query tile: the FA-v1 kernel, no workspace needed
    *bytes = ns == 1 ? 256 : v2_layout(B * H, L, d, ns, pe).total;
    return FA_OK;
}

}  // namespace

extern "C" {

int fa_version(void) { return (FA_MI355X_VERSION_MAJOR << 16) | (FA_MI355X_VERSION_MINOR << 8) | 0; }

const char* fa_last_error(void) { return g_err.c_str(); }

const char* fa_last_kernels(void) { return fa::g_kernels.c_str(); }

int fa_kernel_geometry(int64_t d, int dtype, int* bq, int* bk, int* threads, int* lds_bytes) {
    fa::Elem e;
    if (int st = check_dtype(dtype, &e)) return st;
    if (!supported_d(d) && !wide_d(d))
        return fail(FA_ERR_UNSUPPORTED, "head dim d=%lld has no kernel", (long long)d);
    if (wide_d(d)) {  // the d-tiled kernels: 64 query rows, K / V chunks of at most 128 columns
        if (e == fa::Elem::F64) {
            if (bq) *bq = fa::fwd64_rows_per_block();
            if (threads) *threads = fa::kThreads;
            if (lds_bytes) *lds_bytes = (64 + 2 * 16) * 129 * 8 + 4 * 16 * 17 * 8;
        } else {
            int r = 0, th = 0, lds = 0;
            fa::dtiled_geometry(e, (int)d, &r, &th, &lds);
            if (bq) *bq = r;
            if (threads) *threads = th;
            if (lds_bytes) *lds_bytes = lds;
        }
        if (bk) *bk = keys_per_tile(e, d);
        return ok();
    }
    if (bq) *bq = fa::kBQ;
    if (bk) *bk = fa::bk_for((int)d);
    if (threads) *threads = fa::kThreads;
    if (e == fa::Elem::F64) {  // fp64 mode: 64 rows x 16-key tiles, padded LDS rows
        if (bq) *bq = fa::fwd64_rows_per_block();
        if (bk) *bk = fa::fwd64_keys_per_tile();
        if (lds_bytes) *lds_bytes = (int)(2 * 16 * (d + 1) * 8 + 4 * 16 * 17 * 8);
        return ok();
    }
    if (lds_bytes) *lds_bytes = fa::fwd_lds_bytes((int)d);
    return ok();
}

int fa_fwd_v1(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
              int64_t L, int64_t d, int dtype, void* stream) {
    return fa_fwd_v1_scaled(q, k, v, o, B, H, L, d, 1.0 / std::sqrt((double)(d > 0 ? d : 1)), dtype, stream);
}

int fa_fwd_v1_scaled(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
                     int64_t L, int64_t d, double softmax_scale, int dtype, void* stream) {
    return fa_fwd_v1_ex(q, k, v, o, B, H, L, d, nullptr, nullptr, nullptr, softmax_scale, dtype, stream);
}

int fa_fwd_v1_ex(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H, int64_t L,
                 int64_t d, const int64_t* q_strides, const int64_t* kv_strides, const int64_t* o_strides,
                 double softmax_scale, int dtype, void* stream) {
    fa::Elem e;
    if (int st = check_shape(B, H, L, d, true)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    if (wide_d(d) && (q_strides || kv_strides || o_strides))
        return fail(FA_ERR_UNSUPPORTED, "d=%lld: strided tensors not supported (contiguous [B, H, L, d] only)",
                    (long long)d);
    fa::FwdArgs a = base_args(q, k, v, o, B * H, L, L, d, e);
    if (int st = apply_scale(a, softmax_scale)) return st;
    if (int st = apply_strides(a, e, B, H, L, d, q_strides, kv_strides, o_strides)) return st;
    kernels_begin();
    if (hipError_t he = launch_final(e, (int)d, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v1 launch");
    return ok();
}

int fa_fwd_v1_tiled_d(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
                      int64_t L, int64_t d, int d_tile_qk, int d_tile_v, int dtype, void* stream) {
    return fa_fwd_v1_tiled_d_scaled(q, k, v, o, B, H, L, d, d_tile_qk, d_tile_v,
                                    1.0 / std::sqrt((double)(d > 0 ? d : 1)), dtype, stream);
}

int fa_fwd_v1_tiled_d_scaled(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
                             int64_t L, int64_t d, int d_tile_qk, int d_tile_v, double softmax_scale, int dtype,
                             void* stream) {
    fa::Elem e;
    if (int st = check_shape(B, H, L, d, true)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    if (int st = check_d_tiles(d, d_tile_qk, d_tile_v)) return st;
    fa::FwdArgs a = base_args(q, k, v, o, B * H, L, L, d, e);
    if (int st = apply_scale(a, softmax_scale)) return st;
    // d <= 256: one tile holds a whole row -- the fused kernel (its QK^T accumulates 32-column
    // k-steps, its O^T stays in VGPRs); d = 384 / 512: the d-tiled kernels, tiles honoured
    kernels_begin();
    const hipError_t he = wide_d(d) ? launch_wide(e, (int)d, a, d_tile_qk, d_tile_v, (hipStream_t)stream)
                                    : launch_final(e, (int)d, a, (hipStream_t)stream);
    if (he) return hip_fail(he, "fa_fwd_v1_tiled_d launch");
    return ok();
}

int fa_fwd_v2_workspace_size(int64_t B, int64_t H, int64_t L, int64_t d, int kv_tiles_per_block,
                             int dtype, int partial_dtype, size_t* bytes, int* num_splits) {
    return fa_fwd_v2_workspace_size_ex(B, H, L, d, kv_tiles_per_block, FA_BLOCKS_PER_WG_AUTO, dtype,
                                       partial_dtype, bytes, num_splits);
}

int fa_fwd_v2_workspace_size_ex(int64_t B, int64_t H, int64_t L, int64_t d, int kv_tiles_per_block,
                                int blocks_per_workgroup, int dtype, int partial_dtype, size_t* bytes,
                                int* num_splits) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, L, d, true)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (!bytes) return fail(FA_ERR_INVALID_ARG, "bytes is NULL");
    SplitPlan sp;
    if (int st = plan_splits(B * H, L, d, kv_tiles_per_block, blocks_per_workgroup, e, &sp)) return st;
    if (int st = v2_workspace(B, H, L, d, sp, e, pe, bytes)) return st;
    if (num_splits) *num_splits = sp.units;
    return ok();
}

int fa_fwd_v2_split_plan(int64_t B, int64_t H, int64_t L, int64_t d, int kv_tiles_per_block,
                         int blocks_per_workgroup, int dtype, int* key_blocks, int* blocks_per_wg_out,
                         int* partials_per_tile) {
    fa::Elem e;
    if (int st = check_shape(B, H, L, d, true)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    SplitPlan p;
    if (int st = plan_splits(B * H, L, d, kv_tiles_per_block, blocks_per_workgroup, e, &p)) return st;
    if (key_blocks) *key_blocks = p.units;
    if (blocks_per_wg_out) *blocks_per_wg_out = p.group;
    if (partials_per_tile) *partials_per_tile = p.launched;
    return ok();
}

int fa_fwd_v2(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H, int64_t L,
              int64_t d, int d_tile_qk, int d_tile_v, int kv_tiles_per_block, void* workspace,
              size_t workspace_bytes, int dtype, int partial_dtype, void* stream) {
    return fa_fwd_v2_scaled(q, k, v, o, B, H, L, d, d_tile_qk, d_tile_v, kv_tiles_per_block, workspace,
                            workspace_bytes, 1.0 / std::sqrt((double)(d > 0 ? d : 1)), dtype, partial_dtype,
                            stream);
}

int fa_fwd_v2_scaled(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
                     int64_t L, int64_t d, int d_tile_qk, int d_tile_v, int kv_tiles_per_block,
                     void* workspace, size_t workspace_bytes, double softmax_scale, int dtype,
                     int partial_dtype, void* stream) {
    return fa_fwd_v2_ex(q, k, v, o, B, H, L, d, d_tile_qk, d_tile_v, kv_tiles_per_block, FA_BLOCKS_PER_WG_AUTO,
                        workspace, workspace_bytes, nullptr, nullptr, nullptr, softmax_scale, dtype, partial_dtype,
                        stream);
}

int fa_fwd_v2_ex(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H, int64_t L,
                 int64_t d, int d_tile_qk, int d_tile_v, int kv_tiles_per_block, int blocks_per_workgroup,
                 void* workspace, size_t workspace_bytes, const int64_t* q_strides, const int64_t* kv_strides,
                 const int64_t* o_strides, double softmax_scale, int dtype, int partial_dtype, void* stream) {
    return fa_fwd_v2_ex2(q, k, v, o, B, H, L, d, d_tile_qk, d_tile_v, kv_tiles_per_block, blocks_per_workgroup,
                         workspace, workspace_bytes, q_strides, kv_strides, o_strides, softmax_scale, dtype,
                         partial_dtype, 0u, stream);
}

int fa_fwd_v2_ex2(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H, int64_t L,
                  int64_t d, int d_tile_qk, int d_tile_v, int kv_tiles_per_block, int blocks_per_workgroup,
                  void* workspace, size_t workspace_bytes, const int64_t* q_strides, const int64_t* kv_strides,
                  const int64_t* o_strides, double softmax_scale, int dtype, int partial_dtype, unsigned flags,
                  void* stream) {
    if (flags & ~(unsigned)FA_V2_COUNTERS_ZERO) return fail(FA_ERR_INVALID_ARG, "unknown flags 0x%x", flags);
    fa::Elem e, pe;
    if (int st = check_shape(B, H, L, d, true)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    if (int st = check_d_tiles(d, d_tile_qk, d_tile_v)) return st;
    if (wide_d(d) && (q_strides || kv_strides || o_strides))
        return fail(FA_ERR_UNSUPPORTED, "d=%lld: strided tensors not supported (contiguous [B, H, L, d] only)",
                    (long long)d);
    const int64_t BH = B * H;
    // one plan for the workspace check, the grid and the split length
    SplitPlan sp;
    if (int st = plan_splits(BH, L, d, kv_tiles_per_block, blocks_per_workgroup, e, &sp)) return st;
    size_t need = 0;
    if (int st = v2_workspace(B, H, L, d, sp, e, pe, &need)) return st;
    if (!workspace || workspace_bytes < need)
        return fail(FA_ERR_WORKSPACE, "workspace of %zu bytes needed, got %zu%s", need, workspace_bytes,
                    workspace ? "" : " (NULL)");
    if ((uintptr_t)workspace & 255) return fail(FA_ERR_WORKSPACE, "workspace must be 256-byte aligned");

    const int ns = sp.launched;
    fa::FwdArgs a = base_args(q, k, v, o, BH, L, L, d, e);
    if (int st = apply_scale(a, softmax_scale)) return st;
    if (int st = apply_strides(a, e, B, H, L, d, q_strides, kv_strides, o_strides)) return st;
    kernels_begin();
    if (ns == 1) {  // one partial workgroup per query tile: nothing to combine
        const hipError_t he = wide_d(d) ? launch_wide(e, (int)d, a, d_tile_qk, d_tile_v, (hipStream_t)stream)
                                        : launch_final(e, (int)d, a, (hipStream_t)stream);
        if (he) return hip_fail(he, "fa_fwd_v2 launch");
        return ok();
    }
    const V2Layout w = v2_layout(BH, L, d, ns, pe);
    a.nsplit = ns;
    a.kv_per_split = sp.kv_per_wg;
    if (e == fa::Elem::F64) {  // fp64: the reference's two kernels (partial, then reduction)
        a.o = workspace;
        a.lse64 = (double*)((char*)workspace + w.lse_off);
        a.chunk_rows = L;
        a.split_stride = BH * L * d;
        if (hipError_t he = fa::launch_fwd64((int)d, fa::kPartial, a, (hipStream_t)stream))
            return hip_fail(he, "fa_fwd_v2 partial launch");
        fa::CombineArgs c{};
        c.o_part = workspace; c.lse64 = a.lse64; c.o = o; c.rows = BH * L; c.nsplit = ns;
        if (hipError_t he = fa::launch_combine64((int)d, c, (hipStream_t)stream))
            return hip_fail(he, "fa_fwd_v2 combine launch");
        return ok();
    }
    a.o = workspace;
    a.lse = (float*)((char*)workspace + w.lse_off);
    a.esc = (float*)((char*)workspace + w.esc_off);
    a.tile_group = tile_group((int64_t)a.nqt * ns * BH, ns, a.nqt);
    // Hand-off order of fa_fwd16_kernel's combine (fa_fwd16_kernel.hpp): arrival first -- the
    // last arriver's partial never stored, 1/S of the partial bytes saved twice -- costs a
    // memory round trip on the tile's critical path when its workgroups finish together, so
    // only for key blocks of >= 4096 keys.  Round 5, d = 128 bf16 (profiles/r05/ab,
    // profiles/r05/hbm_traffic_r05.json): B1 H1 L16384 (4 blocks of 4096) 127.5 -> 127.2 us and
    // 72.7 -> 64.1 MB per launch; B1 H2 L4096 (4 of 1024) 28.7 -> 31.0 us (round 6 again:
    // 27.4 -> 30.0 us, B1 H4 L4096 with 2 of 2048 42.1 -> 43.1 us; profiles/r06/ab_b1h*_af.txt).
    a.arrive_first = a.kv_per_split >= 4096;
    a.counters = (unsigned*)((char*)workspace + w.cnt_off);
    a.o_final = o;
    // the kernel leaves every counter at zero; clearing them here makes a call that follows
    // an aborted one (or a fresh workspace) safe
    // ... unless the caller vouches for them (FA_V2_COUNTERS_ZERO: a zeroed workspace, or one
    // only this function has used since): the reset is a dispatch of its own, 1.6-1.8 us per
    // call (B1 H2 L4096: 27.1 -> 25.3 us, B1 H1 L16384: 127.1 -> 125.5 us; profiles/r06/ab_*_memset.txt)
    if (!(flags & FA_V2_COUNTERS_ZERO))
        if (hipError_t he = hipMemsetAsync(a.counters, 0, (size_t)w.ngroups * sizeof(unsigned),
                                           (hipStream_t)stream))
            return hip_fail(he, "fa_fwd_v2 counter reset");
    if (hipError_t he = fa::launch_fwd(e, pe, (int)d, fa::kFused, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v2 launch");
    return ok();
}

int fa_fwd_partial(const void* q, const void* k, const void* v, void* o_part, void* lse,
                   int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t d, int64_t chunk_rows,
                   int dtype, int partial_dtype, void* stream) {
    return fa_fwd_partial_ex(q, k, v, o_part, lse, B, H, Lq, Lk, d, chunk_rows, nullptr, dtype, partial_dtype,
                             stream);
}

int fa_fwd_partial_ex(const void* q, const void* k, const void* v, void* o_part, void* lse,
                      int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t d, int64_t chunk_rows,
                      const int64_t* q_strides, int dtype, int partial_dtype, void* stream) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, Lq, d)) return st;
    if (Lk <= 0 || Lk > (int64_t)1 << 30)
        return fail(FA_ERR_INVALID_ARG, "Lk=%lld out of range", (long long)Lk);
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (int st = check_ptrs(q, k, v, o_part)) return st;
    if (!lse) return fail(FA_ERR_INVALID_ARG, "lse is NULL");
    // lse element: fp32, {lse, e} float pairs for scaled fp16 partials, fp64 for fp64 inputs
    if ((uintptr_t)lse & (pe == fa::Elem::F16S || e == fa::Elem::F64 ? 7 : 3))
        return fail(FA_ERR_INVALID_ARG, "lse must be aligned to its element (%d bytes)",
                    pe == fa::Elem::F16S || e == fa::Elem::F64 ? 8 : 4);
    if (chunk_rows <= 0 || Lq % chunk_rows)
        return fail(FA_ERR_INVALID_ARG, "chunk_rows=%lld must divide Lq=%lld", (long long)chunk_rows,
                    (long long)Lq);
    fa::FwdArgs a = base_args(q, k, v, o_part, B * H, Lq, Lk, d, e);
    a.lse = (float*)lse;
    a.lse64 = (double*)lse;
    a.chunk_rows = chunk_rows;
    a.split_stride = 0;
    if (int st = apply_strides(a, e, B, H, Lq, d, q_strides, nullptr, nullptr, Lk)) return st;
    kernels_begin();
    if (hipError_t he = e == fa::Elem::F64
                            ? fa::launch_fwd64((int)d, fa::kPartial, a, (hipStream_t)stream)
                            : fa::launch_fwd(e, pe, (int)d, fa::kPartial, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_partial launch");
    return ok();
}

int fa_combine(const void* o_part, const void* lse, void* o, int64_t num_splits, int64_t B,
               int64_t H, int64_t L, int64_t d, int dtype, int partial_dtype, void* stream) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, L, d)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (!o_part || !lse || !o) return fail(FA_ERR_INVALID_ARG, "null pointer");
    // the combine kernel moves 16 bytes per lane through o_part and o
    if (((uintptr_t)o_part | (uintptr_t)o) & 15)
        return fail(FA_ERR_INVALID_ARG, "o_part and o must be 16-byte aligned");
    if ((uintptr_t)lse & (pe == fa::Elem::F16S || e == fa::Elem::F64 ? 7 : 3))
        return fail(FA_ERR_INVALID_ARG, "lse must be aligned to its element (%d bytes)",
                    pe == fa::Elem::F16S || e == fa::Elem::F64 ? 8 : 4);
    if (num_splits <= 0 || num_splits > 65536)
        return fail(FA_ERR_INVALID_ARG, "num_splits=%lld out of range", (long long)num_splits);
    fa::CombineArgs c{};
    c.o_part = o_part; c.lse = (const float*)lse; c.lse64 = (const double*)lse; c.o = o;
    c.rows = B * H * L; c.nsplit = (int)num_splits;
    kernels_begin();
    if (hipError_t he = e == fa::Elem::F64 ? fa::launch_combine64((int)d, c, (hipStream_t)stream)
                                           : fa::launch_combine(e, pe, (int)d, c, (hipStream_t)stream))
        return hip_fail(he, "fa_combine launch");
    return ok();
}

}  // extern "C"
