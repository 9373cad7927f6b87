// fa_dist_schedule.hpp -- the exchange schedule of the multi-GPU split-KV forward
// (fa_dist.cpp, include/fa_mi355x_dist.h), as host code with no HIP or RCCL in it, so that the
// step pairing, the chunk offsets, the own-chunk path and the part-way-failure latch can be
// exercised on the CPU with an in-process transport that moves the bytes
// (tests/native/dist_schedule_test.cpp, tests/test_dist_schedule.py).
//
// Per rank r of W, the key shard's partials for all L query rows are cut into W row chunks;
// chunk p belongs to rank p.  The schedule (the reference has no multi-GPU
// code -- its single-GPU split-KV is flash_attention_v2/CUDA/flash_attention_v2.h:243-435):
//   pipelined:  for s = 1 .. W-1: compute chunk dst = (r+s) % W into the send buffer; fence
//               (compute -> exchange stream, event s); post step s = one group of
//               {send chunk dst to dst, receive chunk r from src = (r-s) % W} for O and lse.
//               Every step is a perfect matching (rank r sends to r+s while r+s receives from
//               (r+s)-s = r), so all ranks' links are busy at once.  Then the own chunk r,
//               computed last straight into the receive buffer (it never crosses a link).
//   one launch: compute all W chunks into the send buffer; fence (event 1); post steps
//               1 .. W-1; copy the own chunk send -> receive on the compute stream.
//   world 1:    the partial straight into the receive buffer.
// then (W > 1) fence exchange -> compute (event 0) before the combine.
//
// Failure latch: once step 1 is posted, the peers are mid-exchange; any failure after that
// point -- a kernel launch, an event record or wait, a later step's post -- leaves them
// waiting for sends this rank will never post, so the communicator is marked broken (later
// calls refuse) and the error returned.  A failure before the first post leaves nothing
// posted and the handle usable.
#pragma once
#include <cstddef>
#include <cstdint>

namespace fa {
namespace dist {

// Byte offsets into the workspace (fa_dist.cpp layout()) and the per-chunk sizes.
struct Plan {
    int world = 1, rank = 0;
    bool pipelined = false;        // one partial launch per destination chunk
    size_t send_o = 0, send_lse = 0, recv_o = 0, recv_lse = 0;
    size_t chunk_o = 0, chunk_l = 0;  // bytes of one chunk of partial O / lse
};

inline int step_dst(const Plan& p, int s) { return (p.rank + s) % p.world; }
inline int step_src(const Plan& p, int s) { return (p.rank - s % p.world + p.world) % p.world; }

// Ops (a class with these members, each returning 0 on success or a status code):
//   partial_chunk(int chunk, size_t o_off, size_t l_off)  compute chunk `chunk` of the rows
//   partial_all(size_t o_off, size_t l_off)                all W chunks in one launch
//   fence_to_exchange(int ev)                              exchange stream waits for compute
//   fence_to_compute()                                     compute stream waits for exchange
//   post_step(int s, int dst, int src, size_t send_o, size_t recv_o, size_t send_l,
//             size_t recv_l)                               one grouped send/recv step
//   local_copy(size_t dst_off, size_t src_off, size_t bytes)
// `broken` is the communicator's latch (set here, never cleared).
template <class Ops>
int run_exchange(const Plan& p, Ops& ops, bool& broken) {
    bool posted = false;  // step 1 is out: from here on a failure breaks the communicator
    auto fail = [&](int st) {
        if (posted) broken = true;
        return st;
    };
    auto post = [&](int s) {
        const int dst = step_dst(p, s), src = step_src(p, s);
        const int st = ops.post_step(s, dst, src, p.send_o + dst * p.chunk_o, p.recv_o + src * p.chunk_o,
                                     p.send_lse + dst * p.chunk_l, p.recv_lse + src * p.chunk_l);
        if (st) return fail(st);
        posted = true;
        return 0;
    };
    if (p.world == 1) {
        if (int st = ops.partial_all(p.recv_o, p.recv_lse)) return st;
        return 0;
    }
    if (p.pipelined) {
        for (int s = 1; s < p.world; ++s) {
            const int dst = step_dst(p, s);
            if (int st = ops.partial_chunk(dst, p.send_o + dst * p.chunk_o, p.send_lse + dst * p.chunk_l)) return fail(st);
            if (int st = ops.fence_to_exchange(s)) return fail(st);
            if (int st = post(s)) return st;
        }
        if (int st = ops.partial_chunk(p.rank, p.recv_o + p.rank * p.chunk_o, p.recv_lse + p.rank * p.chunk_l))
            return fail(st);
    } else {
        if (int st = ops.partial_all(p.send_o, p.send_lse)) return st;
        if (int st = ops.fence_to_exchange(1)) return st;
        for (int s = 1; s < p.world; ++s)
            if (int st = post(s)) return st;
        if (int st = ops.local_copy(p.recv_o + p.rank * p.chunk_o, p.send_o + p.rank * p.chunk_o, p.chunk_o))
            return fail(st);
        if (int st = ops.local_copy(p.recv_lse + p.rank * p.chunk_l, p.send_lse + p.rank * p.chunk_l, p.chunk_l))
            return fail(st);
    }
    if (int st = ops.fence_to_compute()) return fail(st);
    return 0;
}

}  // namespace dist
}  // namespace fa
