// fa_capi.cpp -- the C ABI (include/fa_mi355x.h): argument validation, workspace
// arithmetic and dispatch to the gfx950 kernels.  No allocation, no device sync.
//
// Validation mirrors the reference launchers' asserts, turned into status codes:
//   B,H,L,d > 0                    flash_attention_v1/CUDA/flash_attention_v1.h:263
//   0 < d_tile_qk, d_tile_v <= d   flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:326-327
//   kv_tiles_per_block > 0         flash_attention_v2/CUDA/flash_attention_v2.h:447
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/fa_mi355x.h"
#include "fa_internal.hpp"

namespace {

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

int check_dtype(int dtype, fa::Elem* e) {
    if (dtype == FA_DTYPE_BF16) { *e = fa::Elem::BF16; return FA_OK; }
    if (dtype == FA_DTYPE_FP16) { *e = fa::Elem::F16; return FA_OK; }
    return fail(FA_ERR_UNSUPPORTED, "dtype %d has no kernel (use FA_DTYPE_BF16 or FA_DTYPE_FP16)", dtype);
}

int check_partial_dtype(int pdtype, int dtype, fa::Elem* e) {
    if (pdtype == FA_DTYPE_FP32) { *e = fa::Elem::F32; return FA_OK; }
    if (pdtype == dtype) return check_dtype(dtype, e);
    return fail(FA_ERR_UNSUPPORTED, "partial dtype %d must be FA_DTYPE_FP32 or the input dtype %d",
                pdtype, dtype);
}

int check_shape(int64_t B, int64_t H, int64_t L, int64_t d) {
    if (B <= 0 || H <= 0 || L <= 0 || d <= 0)
        return fail(FA_ERR_INVALID_ARG, "all dimensions must be positive (B=%lld H=%lld L=%lld d=%lld)",
                    (long long)B, (long long)H, (long long)L, (long long)d);
    if (!supported_d(d))
        return fail(FA_ERR_UNSUPPORTED, "head dim d=%lld has no kernel (supported: 32, 64, 128, 256)",
                    (long long)d);
    if (L > (int64_t)1 << 30)
        return fail(FA_ERR_UNSUPPORTED, "L=%lld exceeds 2^30", (long long)L);
    const int64_t nqt = (L + fa::kBQ - 1) / fa::kBQ;
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

fa::FwdArgs base_args(const void* q, const void* k, const void* v, void* o, int64_t BH,
                      int64_t Lq, int64_t Lk, int64_t d) {
    fa::FwdArgs a{};
    a.q = q; a.k = k; a.v = v; a.o = o; a.lse = nullptr;
    a.BH = BH; a.Lq = Lq; a.Lk = Lk;
    a.nqt = (int)((Lq + fa::kBQ - 1) / fa::kBQ);
    a.nsplit = 1;
    a.kv_per_split = (int)Lk;
    a.chunk_rows = Lq;
    a.split_stride = 0;
    a.scale_log2 = (float)(1.4426950408889634 / std::sqrt((double)d));
    return a;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int splits_for(int64_t L, int64_t d, int kvtpb, int* kv_per_split) {
    const int64_t keys = (int64_t)kvtpb * fa::bk_for((int)d);
    *kv_per_split = (int)(keys < L ? keys : L);
    return (int)((L + keys - 1) / keys);
}

}  // namespace

extern "C" {

int fa_version(void) { return (0 << 16) | (1 << 8) | 0; }

const char* fa_last_error(void) { return g_err.c_str(); }

int fa_kernel_geometry(int64_t d, int dtype, int* bq, int* bk, int* threads, int* lds_bytes) {
    fa::Elem e;
    if (int st = check_dtype(dtype, &e)) return st;
    if (!supported_d(d))
        return fail(FA_ERR_UNSUPPORTED, "head dim d=%lld has no kernel", (long long)d);
    if (bq) *bq = fa::kBQ;
    if (bk) *bk = fa::bk_for((int)d);
    if (threads) *threads = fa::kThreads;
    if (lds_bytes) *lds_bytes = fa::fwd_lds_bytes((int)d);
    return ok();
}

int fa_fwd_v1(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
              int64_t L, int64_t d, int dtype, void* stream) {
    fa::Elem e;
    if (int st = check_shape(B, H, L, d)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    fa::FwdArgs a = base_args(q, k, v, o, B * H, L, L, d);
    if (hipError_t he = fa::launch_fwd(e, e, (int)d, false, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v1 launch");
    return ok();
}

int fa_fwd_v1_tiled_d(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H,
                      int64_t L, int64_t d, int d_tile_qk, int d_tile_v, int dtype, void* stream) {
    fa::Elem e;
    if (int st = check_shape(B, H, L, d)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    if (int st = check_d_tiles(d, d_tile_qk, d_tile_v)) return st;
    fa::FwdArgs a = base_args(q, k, v, o, B * H, L, L, d);
    if (hipError_t he = fa::launch_fwd(e, e, (int)d, false, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v1_tiled_d launch");
    return ok();
}

int fa_fwd_v2_workspace_size(int64_t B, int64_t H, int64_t L, int64_t d, int kv_tiles_per_block,
                             int dtype, int partial_dtype, size_t* bytes, int* num_splits) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, L, d)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (kv_tiles_per_block <= 0)
        return fail(FA_ERR_INVALID_ARG, "kv_tiles_per_block must be positive (got %d)", kv_tiles_per_block);
    if (!bytes) return fail(FA_ERR_INVALID_ARG, "bytes is NULL");
    int kvps;
    const int ns = splits_for(L, d, kv_tiles_per_block, &kvps);
    const size_t esz = pe == fa::Elem::F32 ? 4 : 2;
    const size_t rows = (size_t)ns * B * H * L;
    *bytes = align256(rows * d * esz) + align256(rows * sizeof(float));
    if (num_splits) *num_splits = ns;
    return ok();
}

int fa_fwd_v2(const void* q, const void* k, const void* v, void* o, int64_t B, int64_t H, int64_t L,
              int64_t d, int d_tile_qk, int d_tile_v, int kv_tiles_per_block, void* workspace,
              size_t workspace_bytes, int dtype, int partial_dtype, void* stream) {
    fa::Elem e, pe;
    size_t need = 0;
    int ns = 0;
    if (int st = fa_fwd_v2_workspace_size(B, H, L, d, kv_tiles_per_block, dtype, partial_dtype,
                                          &need, &ns))
        return st;
    if (int st = check_ptrs(q, k, v, o)) return st;
    if (int st = check_d_tiles(d, d_tile_qk, d_tile_v)) return st;
    check_dtype(dtype, &e);
    check_partial_dtype(partial_dtype, dtype, &pe);
    if (!workspace || workspace_bytes < need)
        return fail(FA_ERR_WORKSPACE, "workspace of %zu bytes needed, got %zu%s", need, workspace_bytes,
                    workspace ? "" : " (NULL)");
    if ((uintptr_t)workspace & 255) return fail(FA_ERR_WORKSPACE, "workspace must be 256-byte aligned");

    const int64_t BH = B * H;
    const size_t esz = pe == fa::Elem::F32 ? 4 : 2;
    const size_t rows = (size_t)ns * BH * L;
    void* o_part = workspace;
    float* lse = (float*)((char*)workspace + align256(rows * d * esz));

    fa::FwdArgs a = base_args(q, k, v, o_part, BH, L, L, d);
    int kvps;
    a.nsplit = splits_for(L, d, kv_tiles_per_block, &kvps);
    a.kv_per_split = kvps;
    a.lse = lse;
    a.chunk_rows = L;
    a.split_stride = BH * L * d;
    if (hipError_t he = fa::launch_fwd(e, pe, (int)d, true, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v2 partial launch");

    fa::CombineArgs c{};
    c.o_part = o_part; c.lse = lse; c.o = o; c.rows = BH * L; c.nsplit = ns;
    if (hipError_t he = fa::launch_combine(e, pe, (int)d, c, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_v2 combine launch");
    return ok();
}

int fa_fwd_partial(const void* q, const void* k, const void* v, void* o_part, float* lse,
                   int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t d, int64_t chunk_rows,
                   int dtype, int partial_dtype, void* stream) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, Lq, d)) return st;
    if (Lk <= 0 || Lk > (int64_t)1 << 30)
        return fail(FA_ERR_INVALID_ARG, "Lk=%lld out of range", (long long)Lk);
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (int st = check_ptrs(q, k, v, o_part)) return st;
    if (!lse) return fail(FA_ERR_INVALID_ARG, "lse is NULL");
    if (chunk_rows <= 0 || Lq % chunk_rows)
        return fail(FA_ERR_INVALID_ARG, "chunk_rows=%lld must divide Lq=%lld", (long long)chunk_rows,
                    (long long)Lq);
    fa::FwdArgs a = base_args(q, k, v, o_part, B * H, Lq, Lk, d);
    a.lse = lse;
    a.chunk_rows = chunk_rows;
    a.split_stride = 0;
    if (hipError_t he = fa::launch_fwd(e, pe, (int)d, true, a, (hipStream_t)stream))
        return hip_fail(he, "fa_fwd_partial launch");
    return ok();
}

int fa_combine(const void* o_part, const float* lse, void* o, int64_t num_splits, int64_t B,
               int64_t H, int64_t L, int64_t d, int dtype, int partial_dtype, void* stream) {
    fa::Elem e, pe;
    if (int st = check_shape(B, H, L, d)) return st;
    if (int st = check_dtype(dtype, &e)) return st;
    if (int st = check_partial_dtype(partial_dtype, dtype, &pe)) return st;
    if (!o_part || !lse || !o) return fail(FA_ERR_INVALID_ARG, "null pointer");
    if (num_splits <= 0 || num_splits > 65536)
        return fail(FA_ERR_INVALID_ARG, "num_splits=%lld out of range", (long long)num_splits);
    fa::CombineArgs c{};
    c.o_part = o_part; c.lse = lse; c.o = o; c.rows = B * H * L; c.nsplit = (int)num_splits;
    if (hipError_t he = fa::launch_combine(e, pe, (int)d, c, (hipStream_t)stream))
        return hip_fail(he, "fa_combine launch");
    return ok();
}

}  // extern "C"
