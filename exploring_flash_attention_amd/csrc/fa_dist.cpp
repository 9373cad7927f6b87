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
#include "fa_dist_ops.hpp"

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

using fa::dist::esize;
using fa::dist::Layout;
using fa::dist::layout;
using fa::dist::lsize;

// The HIP / RCCL primitives under fa_dist_ops.hpp's ExchangeOps (its Api): each maps the
// library's error to a status code with the message in g_err.
struct HipRcclApi {
    using Stream = hipStream_t;
    using Event = hipEvent_t;
    ncclComm_t nccl;
    int fwd_partial_ex(const void* q, const void* k, const void* v, void* o, void* lse, int64_t B, int64_t H,
                       int64_t Lq, int64_t Lk, int64_t d, int64_t chunk_rows, const int64_t* qst, int dtype,
                       int pdtype, Stream s) {
        if (int st = fa_fwd_partial_ex(q, k, v, o, lse, B, H, Lq, Lk, d, chunk_rows, qst, dtype, pdtype, s))
            return core_fail(st, "fa_fwd_partial_ex");
        return FA_OK;
    }
    int fwd_partial(const void* q, const void* k, const void* v, void* o, void* lse, int64_t B, int64_t H,
                    int64_t Lq, int64_t Lk, int64_t d, int64_t chunk_rows, int dtype, int pdtype, Stream s) {
        if (int st = fa_fwd_partial(q, k, v, o, lse, B, H, Lq, Lk, d, chunk_rows, dtype, pdtype, s))
            return core_fail(st, "fa_fwd_partial");
        return FA_OK;
    }
    int record(Event e, Stream s) {
        if (hipError_t he = hipEventRecord(e, s)) return hip_fail(he, "hipEventRecord");
        return FA_OK;
    }
    int wait(Stream s, Event e) {
        if (hipError_t he = hipStreamWaitEvent(s, e, 0)) return hip_fail(he, "hipStreamWaitEvent");
        return FA_OK;
    }
    // (inside a group RCCL only queues; an error there discards the whole group at
    // ncclGroupEnd, nothing of it is posted -- so the group is always closed)
    int group_start() {
        if (ncclResult_t r = ncclGroupStart()) return rccl_fail(r, "ncclGroupStart");
        return FA_OK;
    }
    int group_end(int first_error, int st, int dst, int src) {
        const ncclResult_t r = ncclGroupEnd();
        if (first_error) return first_error;
        if (r != ncclSuccess) {
            char what[96];
            snprintf(what, sizeof what, "exchange step %d (to rank %d, from rank %d)", st, dst, src);
            return rccl_fail(r, what);
        }
        return FA_OK;
    }
    int send(const void* p, size_t bytes, int peer, Stream s) {
        if (ncclResult_t r = ncclSend(p, bytes, ncclUint8, peer, nccl, s)) return rccl_fail(r, "ncclSend");
        return FA_OK;
    }
    int recv(void* p, size_t bytes, int peer, Stream s) {
        if (ncclResult_t r = ncclRecv(p, bytes, ncclUint8, peer, nccl, s)) return rccl_fail(r, "ncclRecv");
        return FA_OK;
    }
    int copy(void* dst, const void* src, size_t bytes, Stream s) {
        if (hipError_t he = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s))
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
    // pipelined (one partial launch per destination chunk, a q row-range view in place) for
    // bf16 / fp16; fp64 (no strided kernels) computes all chunks in one launch first
    const bool pipelined = dtype != FA_DTYPE_FP64 && world > 1 && d % 8 == 0;
    // The schedule (step pairing, chunk offsets, own-chunk path, failure latch) is
    // fa_dist_schedule.hpp's run_exchange; its operations (kernels, events, sends / receives)
    // are fa_dist_ops.hpp's ExchangeOps over this file's HIP / RCCL primitives.  Both run on
    // the CPU against simulated ranks (tests/test_dist_schedule.py, tests/test_dist_ops.py).
    const fa::dist::Plan plan = fa::dist::make_plan(world, rank, pipelined, w, BH, Lc, d, dtype, partial_dtype);
    HipRcclApi api{c->nccl};
    fa::dist::ExchangeOps<HipRcclApi> ops{api, c->ev.data(), s, c->xstream, ws, q, k_shard, v_shard,
                                          B, H, L, Lc, d, dtype, partial_dtype};
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
