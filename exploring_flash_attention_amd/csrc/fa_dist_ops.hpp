// fa_dist_ops.hpp -- the device operations of the multi-GPU split-KV exchange
// (fa_dist_schedule.hpp's Ops) over a primitive API: which kernel writes which workspace bytes,
// which stream waits for which event, what each RCCL send / receive moves and to whom.
//
// fa_dist.cpp instantiates ExchangeOps with its HIP / RCCL primitives (HipRcclApi there); the
// CPU test (tests/native/dist_ops_test.cpp, tests/test_dist_ops.py) instantiates the same code
// with a simulated multi-rank device: in-order streams, HIP event semantics (a wait binds to
// the event's most recent record at enqueue time), point-to-point FIFOs per rank pair, and
// fake partial kernels that check their arguments and write bytes naming (producer rank, chunk,
// call).  Every offset, size, peer, stream and event of this file is therefore executed
// without a GPU; the test also mutates this file and requires each mutation to be caught.
//
// Api (members; each returns 0 on success, else an FA_ERR_* status with the message set):
//   types Stream, Event
//   fwd_partial_ex(q, k, v, o, lse, B, H, Lq, Lk, d, chunk_rows, q_strides, dtype, pdtype, s)
//   fwd_partial(q, k, v, o, lse, B, H, Lq, Lk, d, chunk_rows, dtype, pdtype, s)
//   record(Event, Stream)              wait(Stream, Event)
//   group_start()                      group_end(int first_error, int step, int dst, int src)
//   send(const void*, bytes, peer, Stream)   recv(void*, bytes, peer, Stream)
//   copy(void* dst, const void* src, bytes, Stream)
// Reference: none (the reference is single-GPU); the combine it distributes is
// flash_attention_v2/CUDA/flash_attention_v2.h:356-435.
#pragma once
#include <cstddef>
#include <cstdint>

#include "../../include/fa_mi355x.h"
#include "fa_dist_schedule.hpp"

namespace fa {
namespace dist {

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
inline size_t esize(int dtype) { return dtype == FA_DTYPE_FP64 ? 8 : dtype == FA_DTYPE_FP32 ? 4 : 2; }
// lse bytes per row: fp64 for fp64 inputs; {lse, e} for scaled fp16 partials
inline size_t lsize(int dtype, int pdtype) {
    return dtype == FA_DTYPE_FP64 ? 8 : pdtype == FA_DTYPE_FP16_SCALED ? 8 : 4;
}

// workspace of fa_fwd_v2_dist: send partials + lse, receive partials + lse, all-gather staging
struct Layout {
    size_t part_bytes, lse_bytes;  // one side (send or receive)
    size_t send_o, send_lse, recv_o, recv_lse, gather, total;
};

inline Layout layout(int64_t BH, int64_t L, int64_t d, int dtype, int pdtype) {
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

// The schedule's plan for one call (fa_dist_schedule.hpp): offsets from layout(), chunk sizes
inline Plan make_plan(int world, int rank, bool pipelined, const Layout& w, int64_t BH, int64_t Lc, int64_t d,
                      int dtype, int pdtype) {
    Plan p;
    p.world = world;
    p.rank = rank;
    p.pipelined = pipelined;
    p.send_o = w.send_o;
    p.send_lse = w.send_lse;
    p.recv_o = w.recv_o;
    p.recv_lse = w.recv_lse;
    p.chunk_o = (size_t)BH * Lc * d * esize(pdtype);
    p.chunk_l = (size_t)BH * Lc * lsize(dtype, pdtype);
    return p;
}

template <class Api>
struct ExchangeOps {
    Api& api;
    const typename Api::Event* ev;  // ev[0]: exchange done; ev[s]: step s's partial queued
    typename Api::Stream s;         // the caller's (compute) stream
    typename Api::Stream xs;        // the communicator's exchange stream
    char* ws;
    const void *q, *k, *v;          // q [B, H, L, d]; k, v: this rank's shard [B, H, Lc, d]
    int64_t B, H, L, Lc, d;
    int dtype, pdtype;

    // chunk p of the partials (the rows rank p will own): a q row-range view in place, rows
    // [p*Lc, (p+1)*Lc) of every head, against this rank's Lc keys
    int partial_chunk(int p, size_t o_off, size_t l_off) {
        const int64_t qst[3] = {H * L * d, L * d, d};
        const char* qp = (const char*)q + (size_t)p * Lc * d * esize(dtype);
        return api.fwd_partial_ex(qp, k, v, ws + o_off, ws + l_off, B, H, Lc, Lc, d, Lc, qst, dtype, pdtype, s);
    }
    // all W chunks in one launch, in the send layout [W][B*H][Lc][d]
    int partial_all(size_t o_off, size_t l_off) {
        return api.fwd_partial(q, k, v, ws + o_off, ws + l_off, B, H, L, Lc, d, Lc, dtype, pdtype, s);
    }
    int fence_to_exchange(int e) {
        if (int st = api.record(ev[e], s)) return st;
        return api.wait(xs, ev[e]);
    }
    int fence_to_compute() {
        if (int st = api.record(ev[0], xs)) return st;
        return api.wait(s, ev[0]);
    }
    // one step of the shifted exchange on the exchange stream: send chunk dst to dst, receive
    // this rank's chunk from src -- O and lse, one group (RCCL posts a group whole or not at all)
    int post_step(int st, int dst, int src, size_t so, size_t ro, size_t sl, size_t rl) {
        const size_t chunk_o = (size_t)B * H * Lc * d * esize(pdtype);
        const size_t chunk_l = (size_t)B * H * Lc * lsize(dtype, pdtype);
        if (int e = api.group_start()) return e;
        int e = api.send(ws + so, chunk_o, dst, xs);
        if (!e) e = api.recv(ws + ro, chunk_o, src, xs);
        if (!e) e = api.send(ws + sl, chunk_l, dst, xs);
        if (!e) e = api.recv(ws + rl, chunk_l, src, xs);
        return api.group_end(e, st, dst, src);
    }
    int local_copy(size_t dst_off, size_t src_off, size_t bytes) {
        return api.copy(ws + dst_off, ws + src_off, bytes, s);
    }
};

}  // namespace dist
}  // namespace fa
