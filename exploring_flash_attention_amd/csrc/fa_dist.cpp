// fa_dist.cpp -- multi-GPU split-KV forward over RCCL (include/fa_mi355x_dist.h).
// Host orchestration only: the kernels are libfa_mi355x.so's fa_fwd_partial / fa_combine,
// the exchange is one grouped RCCL send/recv round over xGMI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/fa_mi355x_dist.h"

static_assert(sizeof(ncclUniqueId) == FA_DIST_UNIQUE_ID_BYTES, "ncclUniqueId size");

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
int rccl_fail(ncclResult_t r, const char* what) {
    return fail(FA_ERR_RCCL, "%s: %s", what, ncclGetErrorString(r));
}
int core_fail(int st, const char* what) { return fail(st, "%s: %s", what, fa_last_error()); }

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t esize(int dtype) { return dtype == FA_DTYPE_FP64 ? 8 : dtype == FA_DTYPE_FP32 ? 4 : 2; }
// lse bytes per row: fp64 for fp64 inputs; {lse, e} for scaled fp16 partials
size_t lsize(int dtype, int pdtype) {
    return dtype == FA_DTYPE_FP64 ? 8 : pdtype == FA_DTYPE_FP16_SCALED ? 8 : 4;
}

struct Layout {
    size_t part_bytes, lse_bytes;  // one side (send or receive)
    size_t send_o, send_lse, recv_o, recv_lse, gather, total;
};

Layout layout(int64_t BH, int64_t L, int64_t d, int dtype, int pdtype) {
    Layout w{};
    const size_t rows = (size_t)BH * L;  // W chunks of BH * L/W rows
    w.part_bytes = align256(rows * d * esize(pdtype));
    w.lse_bytes = align256(rows * lsize(dtype, pdtype));
    w.send_o = 0;
    w.send_lse = w.send_o + w.part_bytes;
    w.recv_o = w.send_lse + w.lse_bytes;
    w.recv_lse = w.recv_o + w.part_bytes;
    w.gather = w.recv_lse + w.lse_bytes;
    w.total = w.gather + align256(rows * d * esize(dtype));
    return w;
}

}  // namespace

extern "C" {

const char* fa_dist_last_error(void) { return g_err.c_str(); }

int fa_dist_get_unique_id(void* id) {
    if (!id) return fail(FA_ERR_INVALID_ARG, "id is NULL");
    ncclUniqueId u;
    if (ncclResult_t r = ncclGetUniqueId(&u)) return rccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return ok();
}

int fa_dist_comm_init(void** comm, int world, int rank, const void* id) {
    if (!comm || !id) return fail(FA_ERR_INVALID_ARG, "null argument");
    if (world <= 0 || rank < 0 || rank >= world)
        return fail(FA_ERR_INVALID_ARG, "bad rank %d / world %d", rank, world);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    if (ncclResult_t r = ncclCommInitRank(&c, world, u, rank)) return rccl_fail(r, "ncclCommInitRank");
    *comm = c;
    return ok();
}

int fa_dist_comm_destroy(void* comm) {
    if (!comm) return ok();
    if (ncclResult_t r = ncclCommDestroy((ncclComm_t)comm)) return rccl_fail(r, "ncclCommDestroy");
    return ok();
}

int fa_fwd_v2_dist_workspace_size(int64_t B, int64_t H, int64_t L, int64_t d, int world, int dtype,
                                  int partial_dtype, size_t* bytes) {
    if (!bytes) return fail(FA_ERR_INVALID_ARG, "bytes is NULL");
    if (B <= 0 || H <= 0 || L <= 0 || d <= 0 || world <= 0)
        return fail(FA_ERR_INVALID_ARG, "dimensions and world must be positive");
    if (L % world) return fail(FA_ERR_INVALID_ARG, "L=%lld must be divisible by world=%d", (long long)L, world);
    if (dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_FP16 && dtype != FA_DTYPE_FP64)
        return fail(FA_ERR_UNSUPPORTED, "dtype %d has no kernel", dtype);
    if (partial_dtype != dtype && !((partial_dtype == FA_DTYPE_FP32 || partial_dtype == FA_DTYPE_FP16_SCALED) &&
                                    dtype != FA_DTYPE_FP64))
        return fail(FA_ERR_UNSUPPORTED, "partial dtype %d not valid for dtype %d", partial_dtype, dtype);
    *bytes = layout(B * H, L, d, dtype, partial_dtype).total;
    return ok();
}

int fa_fwd_v2_dist(const void* q, const void* k_shard, const void* v_shard, void* o, int64_t B,
                   int64_t H, int64_t L, int64_t d, void* comm, int gather, void* workspace,
                   size_t workspace_bytes, int dtype, int partial_dtype, void* stream) {
    if (!comm) return fail(FA_ERR_INVALID_ARG, "comm is NULL");
    int world = 0, rank = 0;
    if (ncclResult_t r = ncclCommCount((ncclComm_t)comm, &world)) return rccl_fail(r, "ncclCommCount");
    if (ncclResult_t r = ncclCommUserRank((ncclComm_t)comm, &rank)) return rccl_fail(r, "ncclCommUserRank");
    size_t need = 0;
    if (int st = fa_fwd_v2_dist_workspace_size(B, H, L, d, world, dtype, partial_dtype, &need)) return st;
    if (!workspace || workspace_bytes < need)
        return fail(FA_ERR_WORKSPACE, "workspace of %zu bytes needed, got %zu", need, workspace_bytes);
    if ((uintptr_t)workspace & 255) return fail(FA_ERR_WORKSPACE, "workspace must be 256-byte aligned");
    const int64_t BH = B * H, Lc = L / world;
    const Layout w = layout(BH, L, d, dtype, partial_dtype);
    char* ws = (char*)workspace;
    hipStream_t s = (hipStream_t)stream;

    // 1. partials of all L query rows over this rank's keys, in the send layout
    if (int st = fa_fwd_partial(q, k_shard, v_shard, ws + w.send_o, ws + w.send_lse, B, H, L, Lc, d, Lc,
                                dtype, partial_dtype, stream))
        return core_fail(st, "fa_fwd_partial");
    // 2. chunk p -> rank p (one grouped send/recv round)
    const size_t chunk_o = (size_t)BH * Lc * d * esize(partial_dtype);
    const size_t chunk_l = (size_t)BH * Lc * lsize(dtype, partial_dtype);
    if (world > 1) {
        if (ncclResult_t r = ncclGroupStart()) return rccl_fail(r, "ncclGroupStart");
        const ncclComm_t c = (ncclComm_t)comm;
        for (int p = 0; p < world; ++p) {
            ncclResult_t r = ncclSend(ws + w.send_o + p * chunk_o, chunk_o, ncclUint8, p, c, s);
            if (r == ncclSuccess) r = ncclRecv(ws + w.recv_o + p * chunk_o, chunk_o, ncclUint8, p, c, s);
            if (r == ncclSuccess) r = ncclSend(ws + w.send_lse + p * chunk_l, chunk_l, ncclUint8, p, c, s);
            if (r == ncclSuccess) r = ncclRecv(ws + w.recv_lse + p * chunk_l, chunk_l, ncclUint8, p, c, s);
            if (r != ncclSuccess) {
                // close the group before reporting: an open group would swallow the next call
                (void)ncclGroupEnd();
                char what[64];
                snprintf(what, sizeof what, "send/recv with rank %d", p);
                return rccl_fail(r, what);
            }
        }
        if (ncclResult_t r = ncclGroupEnd()) return rccl_fail(r, "send/recv exchange");
    }
    const char* ro = world > 1 ? ws + w.recv_o : ws + w.send_o;
    const char* rl = world > 1 ? ws + w.recv_lse : ws + w.send_lse;
    // 3. combine the W partials of this rank's rows
    void* rows_out = gather && world > 1 ? (void*)(ws + w.gather + rank * (size_t)BH * Lc * d * esize(dtype)) : o;
    if (int st = fa_combine(ro, rl, rows_out, world, B, H, Lc, d, dtype, partial_dtype, stream))
        return core_fail(st, "fa_combine");
    if (!gather || world == 1) return ok();
    // 4. all-gather [W][B*H][Lc][d] then the strided copy to [B*H][W*Lc][d]
    const size_t part = (size_t)BH * Lc * d * esize(dtype);
    if (ncclResult_t r = ncclAllGather(ws + w.gather + rank * part, ws + w.gather, part, ncclUint8,
                                       (ncclComm_t)comm, s))
        return rccl_fail(r, "ncclAllGather");
    const size_t row_bytes = (size_t)Lc * d * esize(dtype);
    for (int p = 0; p < world; ++p)
        if (hipError_t he = hipMemcpy2DAsync((char*)o + p * row_bytes, (size_t)L * d * esize(dtype),
                                             ws + w.gather + p * part, row_bytes, row_bytes, BH,
                                             hipMemcpyDeviceToDevice, s))
            return fail(FA_ERR_HIP, "gather copy: %s", hipGetErrorString(he));
    return ok();
}

}  // extern "C"
