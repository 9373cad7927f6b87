// fa_dist.cpp -- multi-GPU split-KV forward over RCCL (include/fa_mi355x_dist.h).
// Host orchestration only: the kernels are libfa_mi355x.so's fa_fwd_partial_ex / fa_combine,
// the exchange is RCCL send/recv over xGMI on the communicator's own stream, so that the
// transfer of one destination's partials overlaps the next destination's partial kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fa_mi355x_dist.h"
#include "fa_dist_schedule.hpp"

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
int hip_fail(hipError_t e, const char* what) { return fail(FA_ERR_HIP, "%s: %s", what, hipGetErrorString(e)); }
int core_fail(int st, const char* what) { return fail(st, "%s: %s", what, fa_last_error()); }

// The communicator handle: the RCCL communicator plus what the pipelined exchange needs,
// all created once at fa_dist_comm_init (the forward itself never allocates): a stream for
// the RCCL operations and one event per destination step (+ one for "exchange done").
struct Comm {
    ncclComm_t nccl = nullptr;
    int world = 0, rank = 0, device = 0;
    hipStream_t xstream = nullptr;
    std::vector<hipEvent_t> ev;  // ev[s], s = 1..world-1: partial of step s queued; ev[0]: exchange done
    bool broken = false;         // a call failed after its first exchange step was posted
};

void destroy(Comm* c) {
    for (hipEvent_t e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->xstream) (void)hipStreamDestroy(c->xstream);
    delete c;
}

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


// The HIP / RCCL operations of fa_dist_schedule.hpp's run_exchange for one call.
struct RcclOps {
    Comm* c;
    char* ws;
    const void *q, *k, *v;
    int64_t B, H, L, Lc, d;
    int dtype, pdtype;
    hipStream_t s;
    int partial_chunk(int p, size_t o_off, size_t l_off) {
        // a q row-range view in place: rows [p*Lc, (p+1)*Lc) of every head
        const int64_t qst[3] = {H * L * d, L * d, d};
        const char* qp = (const char*)q + (size_t)p * Lc * d * esize(dtype);
        if (int st = fa_fwd_partial_ex(qp, k, v, ws + o_off, ws + l_off, B, H, Lc, Lc, d, Lc, qst, dtype, pdtype, s))
            return core_fail(st, "fa_fwd_partial_ex");
        return FA_OK;
    }
    int partial_all(size_t o_off, size_t l_off) {
        if (int st = fa_fwd_partial(q, k, v, ws + o_off, ws + l_off, B, H, L, Lc, d, Lc, dtype, pdtype, s))
            return core_fail(st, "fa_fwd_partial");
        return FA_OK;
    }
    int fence_to_exchange(int ev) {
        if (hipError_t he = hipEventRecord(c->ev[ev], s)) return hip_fail(he, "hipEventRecord");
        if (hipError_t he = hipStreamWaitEvent(c->xstream, c->ev[ev], 0)) return hip_fail(he, "hipStreamWaitEvent");
        return FA_OK;
    }
    int fence_to_compute() {
        if (hipError_t he = hipEventRecord(c->ev[0], c->xstream)) return hip_fail(he, "hipEventRecord");
        if (hipError_t he = hipStreamWaitEvent(s, c->ev[0], 0)) return hip_fail(he, "hipStreamWaitEvent");
        return FA_OK;
    }
    // one step of the shifted exchange on the exchange stream: send chunk rank+st to rank+st,
    // receive chunk rank from rank-st (all ranks' links busy at once, every step a matching)
    int post_step(int st, int dst, int src, size_t so, size_t ro, size_t sl, size_t rl) {
        const size_t chunk_o = (size_t)B * H * Lc * d * esize(pdtype);
        const size_t chunk_l = (size_t)B * H * Lc * lsize(dtype, pdtype);
        ncclResult_t r = ncclGroupStart();
        if (r == ncclSuccess) {
            // (inside a group RCCL only queues; an error here discards the whole group at
            // ncclGroupEnd, nothing of it is posted)
            ncclResult_t e = ncclSend(ws + so, chunk_o, ncclUint8, dst, c->nccl, c->xstream);
            if (e == ncclSuccess) e = ncclRecv(ws + ro, chunk_o, ncclUint8, src, c->nccl, c->xstream);
            if (e == ncclSuccess) e = ncclSend(ws + sl, chunk_l, ncclUint8, dst, c->nccl, c->xstream);
            if (e == ncclSuccess) e = ncclRecv(ws + rl, chunk_l, ncclUint8, src, c->nccl, c->xstream);
            r = ncclGroupEnd();
            if (e != ncclSuccess) r = e;
        }
        if (r != ncclSuccess) {
            char what[96];
            snprintf(what, sizeof what, "exchange step %d (to rank %d, from rank %d)", st, dst, src);
            return rccl_fail(r, what);
        }
        return FA_OK;
    }
    int local_copy(size_t dst_off, size_t src_off, size_t bytes) {
        if (hipError_t he = hipMemcpyAsync(ws + dst_off, ws + src_off, bytes, hipMemcpyDeviceToDevice, s))
            return hip_fail(he, "own chunk copy");
        return FA_OK;
    }
};

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
    Comm* c = new Comm;
    c->world = world;
    c->rank = rank;
    if (hipError_t he = hipGetDevice(&c->device)) {
        destroy(c);
        return hip_fail(he, "hipGetDevice");
    }
    if (hipError_t he = hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking)) {
        destroy(c);
        return hip_fail(he, "exchange stream");
    }
    c->ev.assign(world, nullptr);
    for (int i = 0; i < world; ++i)
        if (hipError_t he = hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming)) {
            destroy(c);
            return hip_fail(he, "exchange events");
        }
    if (ncclResult_t r = ncclCommInitRank(&c->nccl, world, u, rank)) {
        destroy(c);
        return rccl_fail(r, "ncclCommInitRank");
    }
    *comm = c;
    return ok();
}

int fa_dist_comm_destroy(void* comm) {
    if (!comm) return ok();
    Comm* c = (Comm*)comm;
    ncclResult_t r = c->nccl ? ncclCommDestroy(c->nccl) : ncclSuccess;
    destroy(c);
    if (r) return rccl_fail(r, "ncclCommDestroy");
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
    // ---- every check before anything is enqueued (a failure past the first RCCL post would
    // leave the peers in a half-posted exchange)
    if (!comm) return fail(FA_ERR_INVALID_ARG, "comm is NULL");
    Comm* c = (Comm*)comm;
    if (c->broken)
        return fail(FA_ERR_RCCL, "communicator unusable: an earlier exchange failed part-way (destroy it)");
    const int world = c->world, rank = c->rank;
    size_t need = 0;
    if (int st = fa_fwd_v2_dist_workspace_size(B, H, L, d, world, dtype, partial_dtype, &need)) return st;
    if (!q || !k_shard || !v_shard || !o) return fail(FA_ERR_INVALID_ARG, "null tensor pointer");
    if (!workspace || workspace_bytes < need)
        return fail(FA_ERR_WORKSPACE, "workspace of %zu bytes needed, got %zu", need, workspace_bytes);
    if ((uintptr_t)workspace & 255) return fail(FA_ERR_WORKSPACE, "workspace must be 256-byte aligned");
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != c->device)
        return fail(FA_ERR_INVALID_ARG, "current device %d is not the communicator's device %d", dev, c->device);
    const int64_t BH = B * H, Lc = L / world;
    const Layout w = layout(BH, L, d, dtype, partial_dtype);
    char* ws = (char*)workspace;
    hipStream_t s = (hipStream_t)stream;
    const size_t chunk_o = (size_t)BH * Lc * d * esize(partial_dtype);
    const size_t chunk_l = (size_t)BH * Lc * lsize(dtype, partial_dtype);
    // pipelined (one partial launch per destination chunk, a q row-range view in place) for
    // bf16 / fp16; fp64 (no strided kernels) computes all chunks in one launch first
    const bool pipelined = dtype != FA_DTYPE_FP64 && world > 1 && d % 8 == 0;
    // The schedule (step pairing, chunk offsets, own-chunk path, failure latch) is
    // fa_dist_schedule.hpp's run_exchange, exercised on the CPU with an in-process transport
    // (tests/test_dist_schedule.py); these are its HIP / RCCL operations.
    fa::dist::Plan plan;
    plan.world = world;
    plan.rank = rank;
    plan.pipelined = pipelined;
    plan.send_o = w.send_o;
    plan.send_lse = w.send_lse;
    plan.recv_o = w.recv_o;
    plan.recv_lse = w.recv_lse;
    plan.chunk_o = chunk_o;
    plan.chunk_l = chunk_l;
    RcclOps ops{c, ws, q, k_shard, v_shard, B, H, L, Lc, d, dtype, partial_dtype, s};
    if (int st = fa::dist::run_exchange(plan, ops, c->broken)) return st;
    // combine the W partials of this rank's rows
    void* rows_out = gather && world > 1 ? (void*)(ws + w.gather + rank * (size_t)BH * Lc * d * esize(dtype)) : o;
    const bool gathering = gather && world > 1;  // peers will post the all-gather: a failure
                                                   // from here on leaves them waiting on it
    if (int st = fa_combine(ws + w.recv_o, ws + w.recv_lse, rows_out, world, B, H, Lc, d, dtype, partial_dtype,
                            stream)) {
        if (gathering) c->broken = true;
        return core_fail(st, "fa_combine");
    }
    if (!gathering) return ok();
    // all-gather [W][B*H][Lc][d] then the strided copy to [B*H][W*Lc][d]
    const size_t part = (size_t)BH * Lc * d * esize(dtype);
    if (ncclResult_t r = ncclAllGather(ws + w.gather + rank * part, ws + w.gather, part, ncclUint8, c->nccl, s)) {
        c->broken = true;
        return rccl_fail(r, "ncclAllGather");
    }
    const size_t row_bytes = (size_t)Lc * d * esize(dtype);
    for (int p = 0; p < world; ++p)
        if (hipError_t he = hipMemcpy2DAsync((char*)o + p * row_bytes, (size_t)L * d * esize(dtype),
                                             ws + w.gather + p * part, row_bytes, row_bytes, BH,
                                             hipMemcpyDeviceToDevice, s))
            return hip_fail(he, "gather copy");
    return ok();
}

}  // extern "C"
