// CPU test of the multi-GPU split-KV exchange schedule (exploring_flash_attention_amd/csrc/
// fa_dist_schedule.hpp, the schedule fa_fwd_v2_dist runs over RCCL).  W in-process "ranks",
// each with its own host workspace, run run_exchange against a fake transport that moves the
// bytes:
//   * partial_chunk / partial_all fill a chunk with a pattern naming (producer rank, chunk);
//   * post_step records the step's grouped send and receive; a send deposits a copy of its
//     bytes in the (src -> dst) FIFO; receives are matched per (src -> dst) pair in posting
//     order (RCCL's point-to-point ordering) when the exchange is "done";
//   * every step must be a perfect matching: the send rank r posts at step s to d is the
//     receive d posts at the same step s from r, with the same byte counts.
// At the end every rank must hold, in its receive buffer, chunk r of every rank p at slot p.
// A failure injected at a given operation and step checks the communicator latch: broken
// exactly when the failure strikes after step 1 was posted.
//
// Prints one JSON line per case; exits non-zero on the first failed check.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../exploring_flash_attention_amd/csrc/fa_dist_schedule.hpp"

using fa::dist::Plan;

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            std::fprintf(stderr, "CHECK failed: %s -- ", #cond); \
            std::fprintf(stderr, __VA_ARGS__);             \
            std::fprintf(stderr, "\n");                    \
            g_fail = 1;                                    \
        }                                                  \
    } while (0)

struct Msg {
    int step;
    std::vector<unsigned char> bytes;
};

struct Net {
    int world;
    std::map<std::pair<int, int>, std::deque<Msg>> fifo;  // (src, dst) -> sends in order
    struct Recv {
        int rank, src, step;
        size_t off, bytes;
    };
    std::vector<Recv> recvs;  // in posting order
};

struct Rank {
    int rank;
    std::vector<unsigned char> ws;
    size_t chunk_o, chunk_l;
    int world;
};

static unsigned char pat(int producer, int chunk, size_t i, int lse) {
    return (unsigned char)(17 * producer + 5 * chunk + (i * 7) % 13 + 101 * lse);
}

struct FakeOps {
    Rank* r;
    Net* net;
    const Plan* p;
    // failure injection: fail when op == fail_op at step == fail_step (or any step if -1)
    std::string fail_op;
    int fail_step = -2;
    int cur_step = 0;  // the step whose partial/fence/post is being issued
    std::vector<std::string> log;

    bool inject(const char* op, int step) {
        if (fail_op == op && (fail_step == -1 || fail_step == step)) return true;
        return false;
    }
    void fill(size_t o_off, size_t l_off, int chunk) {
        for (size_t i = 0; i < r->chunk_o; ++i) r->ws[o_off + i] = pat(r->rank, chunk, i, 0);
        for (size_t i = 0; i < r->chunk_l; ++i) r->ws[l_off + i] = pat(r->rank, chunk, i, 1);
    }
    int partial_chunk(int chunk, size_t o_off, size_t l_off) {
        log.push_back("chunk" + std::to_string(chunk));
        if (inject("partial_chunk", chunk == r->rank ? r->world : cur_step + 1)) return 3;
        fill(o_off, l_off, chunk);
        return 0;
    }
    int partial_all(size_t o_off, size_t l_off) {
        log.push_back("all");
        if (inject("partial_all", 0)) return 3;
        for (int c = 0; c < r->world; ++c) fill(o_off + c * r->chunk_o, l_off + c * r->chunk_l, c);
        return 0;
    }
    int fence_to_exchange(int ev) {
        log.push_back("fence" + std::to_string(ev));
        if (inject("fence_to_exchange", ev)) return 4;
        return 0;
    }
    int fence_to_compute() {
        log.push_back("done");
        if (inject("fence_to_compute", -1)) return 4;
        return 0;
    }
    int post_step(int s, int dst, int src, size_t so, size_t ro, size_t sl, size_t rl) {
        cur_step = s;
        log.push_back("post" + std::to_string(s));
        if (inject("post_step", s)) return 5;
        CHECK(dst == (r->rank + s) % r->world && src == (r->rank - s + r->world) % r->world, "rank %d step %d pairing",
              r->rank, s);
        // the chunk sent must be the destination's, and it must already be computed
        bool computed = false;
        for (auto& e : log)
            if (e == "chunk" + std::to_string(dst) || e == "all") computed = true;
        CHECK(computed, "rank %d step %d sends chunk %d before computing it", r->rank, s, dst);
        net->fifo[{r->rank, dst}].push_back({s, std::vector<unsigned char>(r->ws.begin() + so, r->ws.begin() + so + r->chunk_o)});
        net->fifo[{r->rank, dst}].push_back({s, std::vector<unsigned char>(r->ws.begin() + sl, r->ws.begin() + sl + r->chunk_l)});
        net->recvs.push_back({r->rank, src, s, ro, r->chunk_o});
        net->recvs.push_back({r->rank, src, s, rl, r->chunk_l});
        return 0;
    }
    int local_copy(size_t dst_off, size_t src_off, size_t bytes) {
        log.push_back("copy");
        if (inject("local_copy", -1)) return 4;
        std::memmove(&r->ws[dst_off], &r->ws[src_off], bytes);
        return 0;
    }
};

static Plan make_plan(int world, int rank, bool pipelined, size_t chunk_o, size_t chunk_l) {
    Plan p;
    p.world = world;
    p.rank = rank;
    p.pipelined = pipelined;
    const size_t part = world * chunk_o, lse = world * chunk_l;
    p.send_o = 0;
    p.send_lse = part;
    p.recv_o = part + lse;
    p.recv_lse = 2 * part + lse;
    p.chunk_o = chunk_o;
    p.chunk_l = chunk_l;
    return p;
}

// One full exchange over W fake ranks; returns 0 when every rank holds the right chunks.
static void run_case(int world, bool pipelined) {
    const size_t chunk_o = 96 + 8 * world, chunk_l = 12;
    Net net{world, {}, {}};
    std::vector<Rank> ranks(world);
    std::vector<Plan> plans(world);
    for (int r = 0; r < world; ++r) {
        plans[r] = make_plan(world, r, pipelined, chunk_o, chunk_l);
        ranks[r] = {r, std::vector<unsigned char>(2 * world * (chunk_o + chunk_l), 0xEE), chunk_o, chunk_l, world};
    }
    int posts = 0;
    for (int r = 0; r < world; ++r) {
        FakeOps ops{&ranks[r], &net, &plans[r]};
        bool broken = false;
        const int st = fa::dist::run_exchange(plans[r], ops, broken);
        CHECK(st == 0 && !broken, "world %d rank %d status %d", world, r, st);
        for (auto& e : ops.log) posts += e.rfind("post", 0) == 0;
        if (world > 1) CHECK(ops.log.back() == "done", "rank %d: the combine fence is last", r);
        // the own chunk never crosses the network: computed last (pipelined) or copied
        if (world > 1 && pipelined)
            CHECK(ops.log[ops.log.size() - 2] == "chunk" + std::to_string(r), "rank %d own chunk last", r);
    }
    CHECK(posts == world * (world - 1), "world %d: %d steps posted", world, posts);
    // the exchange completes: match receives against the per-pair FIFOs in posting order
    for (auto& rv : net.recvs) {
        auto& q = net.fifo[{rv.src, rv.rank}];
        CHECK(!q.empty(), "rank %d step %d: nothing sent by %d", rv.rank, rv.step, rv.src);
        if (q.empty()) continue;
        Msg m = q.front();
        q.pop_front();
        CHECK(m.step == rv.step, "rank %d receives step %d from %d but it sent at step %d", rv.rank, rv.step, rv.src,
              m.step);
        CHECK(m.bytes.size() == rv.bytes, "size mismatch");
        std::memcpy(&ranks[rv.rank].ws[rv.off], m.bytes.data(), std::min(m.bytes.size(), rv.bytes));
    }
    for (auto& kv : net.fifo) CHECK(kv.second.empty(), "unreceived sends %d -> %d", kv.first.first, kv.first.second);
    // every rank r holds chunk r of every producer p at receive slot p
    for (int r = 0; r < world; ++r)
        for (int p = 0; p < world; ++p) {
            bool ok = true;
            for (size_t i = 0; i < chunk_o; ++i) ok &= ranks[r].ws[plans[r].recv_o + p * chunk_o + i] == pat(p, r, i, 0);
            for (size_t i = 0; i < chunk_l; ++i) ok &= ranks[r].ws[plans[r].recv_lse + p * chunk_l + i] == pat(p, r, i, 1);
            CHECK(ok, "world %d rank %d slot %d does not hold chunk %d of rank %d", world, r, p, r, p);
        }
    std::printf("{\"case\": \"exchange\", \"world\": %d, \"pipelined\": %d, \"steps_posted\": %d, \"ok\": %d}\n", world,
                pipelined, posts, !g_fail);
}

// Failure injection on rank `rank`: the status comes back and the latch is set iff step 1 was
// already posted when the failure struck.
static void run_failure(int world, bool pipelined, const char* op, int step, bool expect_broken) {
    const size_t chunk_o = 64, chunk_l = 8;
    Net net{world, {}, {}};
    const int rank = world > 2 ? 1 : 0;
    Rank rk{rank, std::vector<unsigned char>(2 * world * (chunk_o + chunk_l)), chunk_o, chunk_l, world};
    Plan p = make_plan(world, rank, pipelined, chunk_o, chunk_l);
    FakeOps ops{&rk, &net, &p, op, step};
    bool broken = false;
    const int st = fa::dist::run_exchange(p, ops, broken);
    CHECK(st != 0, "injected %s at step %d returned success", op, step);
    CHECK(broken == expect_broken, "world %d %s %s at step %d: broken=%d, expected %d", world,
          pipelined ? "pipelined" : "one-launch", op, step, broken, expect_broken);
    // and a broken communicator stays broken: nothing clears it
    std::printf("{\"case\": \"failure\", \"world\": %d, \"pipelined\": %d, \"op\": \"%s\", \"step\": %d, "
                "\"status\": %d, \"broken\": %d, \"ok\": %d}\n",
                world, pipelined, op, step, st, broken, !g_fail);
}

int main() {
    for (int world : {1, 2, 3, 4, 8})
        for (bool pip : {true, false}) run_case(world, pip);
    for (int world : {2, 4, 8}) {
        // pipelined: partial chunk of step s (s = 1 .. W-1), the fence of step s, the post of step s
        run_failure(world, true, "partial_chunk", 1, false);  // nothing posted yet
        run_failure(world, true, "fence_to_exchange", 1, false);
        run_failure(world, true, "post_step", 1, false);      // the group is discarded whole
        if (world > 2) {
            run_failure(world, true, "partial_chunk", 2, true);
            run_failure(world, true, "fence_to_exchange", 2, true);
            run_failure(world, true, "post_step", 2, true);
            run_failure(world, true, "post_step", world - 1, true);
        }
        run_failure(world, true, "partial_chunk", world, true);  // the own chunk, after every post
        run_failure(world, true, "fence_to_compute", -1, true);
        // one launch: the partial and the fence precede every post
        run_failure(world, false, "partial_all", 0, false);
        run_failure(world, false, "fence_to_exchange", 1, false);
        run_failure(world, false, "post_step", 1, false);
        if (world > 2) run_failure(world, false, "post_step", 2, true);
        run_failure(world, false, "local_copy", -1, true);
        run_failure(world, false, "fence_to_compute", -1, true);
    }
    return g_fail;
}
