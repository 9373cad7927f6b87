// CPU test of the multi-GPU split-KV exchange's device operations: fa_dist_ops.hpp's
// ExchangeOps -- the code fa_fwd_v2_dist runs over HIP and RCCL -- instantiated over a
// simulated node of W ranks instead of HipRcclApi (exploring_flash_attention_amd/csrc/fa_dist.cpp).
//
// The simulated device:
//   * streams are in-order queues; rank r owns a compute stream and an exchange stream;
//   * events follow HIP: a record makes a new instance, completed when the record executes in
//     its stream; a wait binds to the event's most recent record at the time it is enqueued;
//   * a send / receive group runs on one stream: when it reaches the head, its sends copy the
//     source bytes (as they are at that moment) into the (me -> peer) FIFO; it completes once
//     each receive has found its message in the (peer -> me) FIFO, in posting order;
//   * the partial kernels are fakes that check every argument ExchangeOps passes (the q row
//     view, shard pointers, row counts, strides, output ranges) and, when they execute, write
//     bytes naming (producer rank, chunk, call) into their outputs;
//   * the combine (fa_combine in fa_dist.cpp) is a check op on the compute stream: when it
//     executes, receive slot p of rank r must hold chunk r of rank p of this call.
// Scheduling policies: exchange streams first (transfers as early as the events allow),
// compute streams first, and seeded random picks; each case runs two calls back to back on
// the same workspace, so stale bytes of the first call are caught in the second.
//
// Prints one JSON line per case; exits non-zero on the first failed check.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <random>
#include <string>
#include <vector>

#ifndef FA_DIST_OPS_HEADER
#define FA_DIST_OPS_HEADER "../../exploring_flash_attention_amd/csrc/fa_dist_ops.hpp"
#endif
#include FA_DIST_OPS_HEADER
#include "../../include/fa_mi355x_dist.h"

using fa::dist::ExchangeOps;
using fa::dist::Layout;
using fa::dist::Plan;

static int g_fail = 0;
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            if (!g_fail) {                                        \
                std::fprintf(stderr, "CHECK failed: %s -- ", #cond); \
                std::fprintf(stderr, __VA_ARGS__);                \
                std::fprintf(stderr, "\n");                       \
            }                                                     \
            g_fail = 1;                                           \
        }                                                         \
    } while (0)

static unsigned char pat(int producer, int chunk, int call, size_t i, int lse) {
    const unsigned h = (unsigned)producer * 1000003u ^ (unsigned)chunk * 10007u ^ (unsigned)call * 101u ^ (unsigned)lse * 7u;
    return (unsigned char)((h + i * 131u) % 251u);
}

struct Sim;

struct Op {
    enum Kind { KERNEL, RECORD, WAIT, GROUP, COPY, CHECKPOINT } kind;
    std::function<void()> effect;  // KERNEL, COPY, CHECKPOINT
    int instance = -1;             // RECORD: the instance it completes; WAIT: the one it waits for
    struct Xfer {
        int peer;
        unsigned char* ptr;
        size_t bytes;
    };
    std::vector<Xfer> sends, recvs;  // GROUP
    bool deposited = false;
    int rank = -1;
};

struct Sim {
    int world;
    std::vector<std::deque<Op>> streams;  // 2r: compute, 2r+1: exchange
    std::vector<int> last_record;         // per event id: its most recent instance (-1: none)
    std::vector<char> done;               // per instance
    std::map<std::pair<int, int>, std::deque<std::vector<unsigned char>>> fifo;  // (src, dst)
    explicit Sim(int w) : world(w), streams(2 * w), last_record(w * w, -1) {}

    bool runnable(Op& op) {
        switch (op.kind) {
            case Op::WAIT: return op.instance < 0 || done[op.instance];
            case Op::GROUP: {
                if (!op.deposited) return true;
                std::map<int, int> need;
                for (auto& r : op.recvs) need[r.peer]++;
                for (auto& kv : need)
                    if ((int)fifo[{kv.first, op.rank}].size() < kv.second) return false;
                return true;
            }
            default: return true;
        }
    }
    // run the head op of stream i; returns true when it left the queue
    bool step(int i) {
        Op& op = streams[i].front();
        switch (op.kind) {
            case Op::KERNEL:
            case Op::COPY:
            case Op::CHECKPOINT: op.effect(); break;
            case Op::RECORD: done[op.instance] = 1; break;
            case Op::WAIT: break;
            case Op::GROUP:
                if (!op.deposited) {
                    for (auto& s : op.sends) fifo[{op.rank, s.peer}].emplace_back(s.ptr, s.ptr + s.bytes);
                    op.deposited = true;
                    if (!op.recvs.empty()) return false;
                    break;
                }
                for (auto& r : op.recvs) {
                    auto& q = fifo[{r.peer, op.rank}];
                    auto msg = std::move(q.front());
                    q.pop_front();
                    CHECK(msg.size() == r.bytes, "rank %d receives %zu bytes from %d, %zu were sent", op.rank, r.bytes,
                          r.peer, msg.size());
                    std::memcpy(r.ptr, msg.data(), std::min(msg.size(), r.bytes));
                }
                break;
        }
        streams[i].pop_front();
        return true;
    }
    // policy 0: exchange streams first; 1: compute streams first; 2+: random (seeded)
    void run(int policy) {
        std::mt19937 rng(policy);
        for (int guard = 0; guard < 1000000; ++guard) {
            std::vector<int> order;
            for (int i = 0; i < (int)streams.size(); ++i)
                if (!streams[i].empty() && runnable(streams[i].front())) order.push_back(i);
            if (order.empty()) {
                bool left = false;
                for (auto& s : streams) left |= !s.empty();
                CHECK(!left, "deadlock: queued operations can never run");
                return;
            }
            if (policy == 0)
                std::stable_partition(order.begin(), order.end(), [](int i) { return i & 1; });
            else if (policy == 1)
                std::stable_partition(order.begin(), order.end(), [](int i) { return !(i & 1); });
            else
                std::shuffle(order.begin(), order.end(), rng);
            step(order[0]);
        }
        CHECK(false, "simulation did not finish");
    }
};

struct Rank {
    int rank;
    std::vector<unsigned char> ws, q, k, v;
};

// The primitive API of fa_dist_ops.hpp over the simulated node, for one rank.
struct SimApi {
    using Stream = int;
    using Event = int;
    Sim* sim;
    Rank* r;
    int64_t B, H, L, Lc, d;
    int dtype, pdtype, call;
    const char* fail_op = "";  // failure injection: this primitive fails at its fail_at-th call
    int fail_at = -1, calls = 0;
    bool in_group = false, group_closed = true;
    Op group;
    int group_stream = -1;

    int compute() const { return 2 * r->rank; }
    int exchange() const { return 2 * r->rank + 1; }
    bool inject(const char* op) { return std::strcmp(op, fail_op) == 0 && calls++ == fail_at; }
    bool own_stream(Stream s) const { return s == compute() || s == exchange(); }
    bool own_event(Event e) const { return e >= r->rank * sim->world && e < (r->rank + 1) * sim->world; }
    bool in_ws(const void* p, size_t bytes) const {
        const unsigned char* b = (const unsigned char*)p;
        return b >= r->ws.data() && b + bytes <= r->ws.data() + r->ws.size();
    }
    void enqueue(Stream s, Op op) { sim->streams[s].push_back(std::move(op)); }

    void kernel(Stream s, unsigned char* o, unsigned char* lse, int nchunks, int first_chunk) {
        const size_t co = (size_t)B * H * Lc * d * fa::dist::esize(pdtype);
        const size_t cl = (size_t)B * H * Lc * fa::dist::lsize(dtype, pdtype);
        CHECK(in_ws(o, nchunks * co) && in_ws(lse, nchunks * cl), "rank %d: partial output outside the workspace",
              r->rank);
        CHECK(s == compute(), "rank %d: partial kernel on stream %d, not the compute stream", r->rank, s);
        if (g_fail) return;
        const int rank = r->rank, c = call;
        Op op{Op::KERNEL};
        op.effect = [=] {
            for (int j = 0; j < nchunks; ++j) {
                for (size_t i = 0; i < co; ++i) o[j * co + i] = pat(rank, first_chunk + j, c, i, 0);
                for (size_t i = 0; i < cl; ++i) lse[j * cl + i] = pat(rank, first_chunk + j, c, i, 1);
            }
        };
        enqueue(s, std::move(op));
    }
    int fwd_partial_ex(const void* q, const void* k, const void* v, void* o, void* lse, int64_t b, int64_t h,
                       int64_t Lq, int64_t Lk, int64_t dd, int64_t chunk_rows, const int64_t* qst, int dt, int pdt,
                       Stream s) {
        if (inject("partial")) return FA_ERR_HIP;
        CHECK(k == r->k.data() && v == r->v.data(), "rank %d: partial not on this rank's key shard", r->rank);
        CHECK(b == B && h == H && dd == d && dt == dtype && pdt == pdtype, "rank %d: shape / dtype", r->rank);
        CHECK(Lq == Lc && Lk == Lc && chunk_rows == Lq, "rank %d: chunk launch rows Lq %lld Lk %lld chunk %lld", r->rank,
              (long long)Lq, (long long)Lk, (long long)chunk_rows);
        CHECK(qst && qst[0] == H * L * d && qst[1] == L * d && qst[2] == d, "rank %d: q strides of the row view",
              r->rank);
        const ptrdiff_t off = (const unsigned char*)q - r->q.data();
        const ptrdiff_t per = (ptrdiff_t)(Lc * d * fa::dist::esize(dtype));
        CHECK(off >= 0 && off % per == 0 && off / per < sim->world, "rank %d: q view at byte %lld is no chunk start",
              r->rank, (long long)off);
        kernel(s, (unsigned char*)o, (unsigned char*)lse, 1, (int)(off / per));
        return 0;
    }
    int fwd_partial(const void* q, const void* k, const void* v, void* o, void* lse, int64_t b, int64_t h, int64_t Lq,
                    int64_t Lk, int64_t dd, int64_t chunk_rows, int dt, int pdt, Stream s) {
        if (inject("partial")) return FA_ERR_HIP;
        CHECK(q == r->q.data() && k == r->k.data() && v == r->v.data(), "rank %d: one-launch partial pointers",
              r->rank);
        CHECK(b == B && h == H && dd == d && dt == dtype && pdt == pdtype, "rank %d: shape / dtype", r->rank);
        CHECK(Lq == L && Lk == Lc && chunk_rows == Lc, "rank %d: one-launch rows Lq %lld Lk %lld chunk %lld", r->rank,
              (long long)Lq, (long long)Lk, (long long)chunk_rows);
        kernel(s, (unsigned char*)o, (unsigned char*)lse, sim->world, 0);
        return 0;
    }
    int record(Event e, Stream s) {
        if (inject("record")) return FA_ERR_HIP;
        CHECK(own_event(e) && own_stream(s), "rank %d: record of event %d on stream %d", r->rank, e, s);
        if (g_fail) return 0;
        Op op{Op::RECORD};
        op.instance = (int)sim->done.size();
        sim->done.push_back(0);
        sim->last_record[e] = op.instance;
        enqueue(s, std::move(op));
        return 0;
    }
    int wait(Stream s, Event e) {
        if (inject("wait")) return FA_ERR_HIP;
        CHECK(own_event(e) && own_stream(s), "rank %d: wait for event %d on stream %d", r->rank, e, s);
        if (g_fail) return 0;
        Op op{Op::WAIT};
        op.instance = sim->last_record[e];
        enqueue(s, std::move(op));
        return 0;
    }
    int group_start() {
        CHECK(!in_group, "rank %d: nested group", r->rank);
        in_group = true;
        group_closed = false;
        group = Op{Op::GROUP};
        group.rank = r->rank;
        group_stream = -1;
        return 0;
    }
    int xfer(std::vector<Op::Xfer>& list, const void* p, size_t bytes, int peer, Stream s, const char* what) {
        if (inject(what)) return FA_ERR_RCCL;
        CHECK(in_group, "rank %d: %s outside a group", r->rank, what);
        CHECK(s == exchange(), "rank %d: %s on stream %d, not the exchange stream", r->rank, what, s);
        CHECK(peer >= 0 && peer < sim->world && peer != r->rank, "rank %d: %s peer %d", r->rank, what, peer);
        CHECK(in_ws(p, bytes), "rank %d: %s buffer outside the workspace", r->rank, what);
        CHECK(group_stream < 0 || group_stream == s, "rank %d: one group on two streams", r->rank);
        group_stream = s;
        list.push_back({peer, (unsigned char*)p, bytes});
        return 0;
    }
    int send(const void* p, size_t bytes, int peer, Stream s) { return xfer(group.sends, p, bytes, peer, s, "send"); }
    int recv(void* p, size_t bytes, int peer, Stream s) { return xfer(group.recvs, p, bytes, peer, s, "recv"); }
    int group_end(int first_error, int, int, int) {
        CHECK(in_group, "rank %d: group_end without group_start", r->rank);
        in_group = false;
        group_closed = true;
        if (first_error) return first_error;  // RCCL discards a group with a failed member whole
        if (inject("group_end")) return FA_ERR_RCCL;
        if (!g_fail && group_stream >= 0) enqueue(group_stream, std::move(group));
        return 0;
    }
    int copy(void* dst, const void* src, size_t bytes, Stream s) {
        if (inject("copy")) return FA_ERR_HIP;
        CHECK(in_ws(dst, bytes) && in_ws(src, bytes), "rank %d: copy outside the workspace", r->rank);
        CHECK(own_stream(s), "rank %d: copy on stream %d", r->rank, s);
        if (g_fail) return 0;
        Op op{Op::COPY};
        unsigned char* dp = (unsigned char*)dst;
        const unsigned char* sp = (const unsigned char*)src;
        op.effect = [=] { std::memmove(dp, sp, bytes); };
        enqueue(s, std::move(op));
        return 0;
    }
};

struct Case {
    int world, dtype, pdtype;
    const char* name;
};

static const char* dname(int t) {
    return t == FA_DTYPE_BF16 ? "bf16" : t == FA_DTYPE_FP16 ? "fp16" : t == FA_DTYPE_FP32 ? "fp32"
                                      : t == FA_DTYPE_FP64 ? "fp64" : "fp16_scaled";
}

// Two calls of the exchange on W simulated ranks under one scheduling policy.
static void run_case(int world, int dtype, int pdtype, int policy) {
    const int64_t B = 2, H = 3, Lc = 4, d = 8, L = Lc * world, BH = B * H;
    const bool pipelined = dtype != FA_DTYPE_FP64 && world > 1 && d % 8 == 0;  // fa_fwd_v2_dist's rule
    const Layout w = fa::dist::layout(BH, L, d, dtype, pdtype);
    Sim sim(world);
    std::vector<Rank> ranks(world);
    for (int r = 0; r < world; ++r) {
        ranks[r].rank = r;
        ranks[r].ws.assign(w.total, 0xEE);
        ranks[r].q.assign((size_t)BH * L * d * fa::dist::esize(dtype), 0);
        ranks[r].k.assign((size_t)BH * Lc * d * fa::dist::esize(dtype), 0);
        ranks[r].v.assign(ranks[r].k.size(), 0);
    }
    // per rank: W events, ids rank*W + i, and one id past them that is no event of the rank
    std::vector<std::vector<int>> evs(world);
    for (int r = 0; r < world; ++r) {
        for (int i = 0; i < world; ++i) evs[r].push_back(r * world + i);
        evs[r].push_back(-777);
    }
    for (int call = 0; call < 2; ++call) {
        for (int r = 0; r < world; ++r) {
            SimApi api{&sim, &ranks[r], B, H, L, Lc, d, dtype, pdtype, call};
            ExchangeOps<SimApi> ops{api, evs[r].data(), api.compute(), api.exchange(), (char*)ranks[r].ws.data(),
                                    ranks[r].q.data(), ranks[r].k.data(), ranks[r].v.data(), B, H, L, Lc, d,
                                    dtype, pdtype};
            const Plan p = fa::dist::make_plan(world, r, pipelined, w, BH, Lc, d, dtype, pdtype);
            bool broken = false;
            const int st = fa::dist::run_exchange(p, ops, broken);
            CHECK(st == 0 && !broken, "world %d rank %d call %d: status %d", world, r, call, st);
            CHECK(api.group_closed, "rank %d: a group left open", r);
            // fa_combine of this call: at the time it runs, receive slot p holds chunk r of rank p
            Op chk{Op::CHECKPOINT};
            Rank* rk = &ranks[r];
            const size_t co = p.chunk_o, cl = p.chunk_l;
            chk.effect = [=] {
                for (int pr = 0; pr < world; ++pr) {
                    bool ok = true;
                    for (size_t i = 0; i < co; ++i) ok &= rk->ws[w.recv_o + pr * co + i] == pat(pr, r, call, i, 0);
                    for (size_t i = 0; i < cl; ++i) ok &= rk->ws[w.recv_lse + pr * cl + i] == pat(pr, r, call, i, 1);
                    CHECK(ok, "world %d call %d: rank %d slot %d does not hold chunk %d of rank %d when the combine runs",
                          world, call, r, pr, r, pr);
                }
            };
            sim.streams[2 * r].push_back(std::move(chk));
        }
        // the second call is enqueued while the first may still be in flight: run after both
    }
    sim.run(policy);
    for (auto& kv : sim.fifo) CHECK(kv.second.empty(), "unreceived sends %d -> %d", kv.first.first, kv.first.second);
    std::printf("{\"case\": \"ops\", \"world\": %d, \"dtype\": \"%s\", \"partial\": \"%s\", \"pipelined\": %d, "
                "\"policy\": %d, \"ok\": %d}\n",
                world, dname(dtype), dname(pdtype), pipelined, policy, !g_fail);
}

// A primitive failing inside ExchangeOps: the status comes back, a group is never left open,
// and the communicator latch follows the schedule's rule (broken iff step 1 was posted).
static void run_failure(int world, const char* op, int at, bool expect_broken) {
    const int64_t B = 1, H = 2, Lc = 4, d = 8, L = Lc * world, BH = B * H;
    const int dtype = FA_DTYPE_BF16, pdtype = FA_DTYPE_FP16_SCALED;
    const Layout w = fa::dist::layout(BH, L, d, dtype, pdtype);
    Sim sim(world);
    Rank rk{1 % world};
    rk.ws.assign(w.total, 0);
    rk.q.assign((size_t)BH * L * d * 2, 0);
    rk.k.assign((size_t)BH * Lc * d * 2, 0);
    rk.v.assign(rk.k.size(), 0);
    std::vector<int> ev;
    for (int i = 0; i < world; ++i) ev.push_back(rk.rank * world + i);
    SimApi api{&sim, &rk, B, H, L, Lc, d, dtype, pdtype, 0, op, at};
    ExchangeOps<SimApi> ops{api, ev.data(), api.compute(), api.exchange(), (char*)rk.ws.data(), rk.q.data(),
                            rk.k.data(), rk.v.data(), B, H, L, Lc, d, dtype, pdtype};
    const Plan p = fa::dist::make_plan(world, rk.rank, true, w, BH, Lc, d, dtype, pdtype);
    bool broken = false;
    const int st = fa::dist::run_exchange(p, ops, broken);
    CHECK(st != 0, "%s failing at call %d returned success", op, at);
    CHECK(api.group_closed, "%s failing at call %d left a group open", op, at);
    CHECK(broken == expect_broken, "world %d %s at call %d: broken=%d, expected %d", world, op, at, broken,
          expect_broken);
    std::printf("{\"case\": \"failure\", \"world\": %d, \"op\": \"%s\", \"at\": %d, \"status\": %d, \"broken\": %d, "
                "\"ok\": %d}\n",
                world, op, at, st, broken, !g_fail);
}

int main(int argc, char** argv) {
    const bool quick = argc > 1 && std::strcmp(argv[1], "--quick") == 0;
    const int pairs[][2] = {{FA_DTYPE_BF16, FA_DTYPE_FP16_SCALED},
                            {FA_DTYPE_BF16, FA_DTYPE_FP32},
                            {FA_DTYPE_FP16, FA_DTYPE_FP16},
                            {FA_DTYPE_FP64, FA_DTYPE_FP64}};
    const int policies = quick ? 4 : 8;
    for (int world : {1, 2, 3, 4, 8})
        for (auto& pr : pairs)
            for (int pol = 0; pol < policies; ++pol) run_case(world, pr[0], pr[1], pol);
    for (int world : {2, 4, 8}) {
        run_failure(world, "partial", 0, false);    // chunk of step 1: nothing posted yet
        run_failure(world, "record", 0, false);     // step 1's fence
        run_failure(world, "send", 0, false);       // inside step 1's group: the group is discarded
        run_failure(world, "recv", 0, false);
        run_failure(world, "group_end", 0, false);
        run_failure(world, "partial", 1, true);  // step 2's chunk (world 2: the own chunk, after the post)
        if (world > 2) {
            run_failure(world, "send", 2, true);  // step 2's O send (two sends per group)
            run_failure(world, "recv", 3, true);  // step 2's lse receive
        }
        run_failure(world, "record", world - 1, true);  // fence_to_compute's record
        run_failure(world, "wait", world - 1, true);
    }
    return g_fail;
}
