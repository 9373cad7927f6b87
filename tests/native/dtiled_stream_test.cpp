// CPU replay of the d-tiled kernel's LDS ring protocol (exploring_flash_attention_amd/csrc/
// fa_dtiled_stream.hpp, the constants fa_fwd_dt_kernel is built from) for every instantiation
// (d = 384 / 512, d_tile_qk / d_tile_v = 32 / 64 / 128) and the ring variants (3-8 slots, chunks
// made readable one at a time or in pairs), at stream lengths of 1-9 tiles.
//
// One wave's view: each DMA piece is counted in issue order; `s_waitcnt vmcnt(N)` completes
// every piece but the N issued last.  Checked at every chunk the kernel consumes:
//   * every piece of the chunk has completed (the wait before it, or its pair's, covered it);
//   * its slot holds it (chunk c in slot c % NSLOT, through the kernel's slot arithmetic);
// and at every issue: the slot's previous chunk was consumed before the barrier that precedes
// the issue (no DMA lands in a slot a wave may still read).
// Prints one JSON line per configuration; exits non-zero on the first failed check.
#include <cstdio>
#include <deque>
#include <vector>

#include "../../exploring_flash_attention_amd/csrc/fa_dtiled_stream.hpp"

static int g_fail = 0;
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            std::fprintf(stderr, "CHECK failed: %s -- ", #cond);  \
            std::fprintf(stderr, __VA_ARGS__);                    \
            std::fprintf(stderr, "\n");                           \
            g_fail = 1;                                           \
        }                                                         \
    } while (0)

template <int D, int DQ, int DV, int NSLOT, int GRP>
static void run(int ntiles) {
    using S = fa::DtStream<D, DQ, DV, NSLOT, GRP>;
    const long total = (long)ntiles * S::PER_TILE;
    std::deque<long> inflight;                   // chunk id of each piece not yet completed
    std::vector<int> left(total, 0);             // pieces of a chunk not yet completed
    std::vector<int> issued(total, 0);
    std::vector<long> owner(NSLOT, -1);          // chunk written into each slot last
    long consumed = -1;                          // last chunk consumed
    long barrier_at = -1;                        // chunks < barrier_at were consumed at the last barrier
    int waits = 0, steady = 0, max_inflight = 0;
    auto issue = [&](long c, int slot) {
        CHECK(c < total, "chunk %ld past the stream", c);
        CHECK(slot == c % NSLOT, "chunk %ld into slot %d", c, slot);
        const long prev = owner[slot];
        CHECK(prev < 0 || prev < barrier_at, "chunk %ld overwrites chunk %ld (barrier at %ld)", c, prev, barrier_at);
        owner[slot] = c;
        const int pos = (int)(c % S::PER_TILE);
        for (int p = 0; p < S::pieces(pos); ++p) inflight.push_back(c);
        left[c] = S::pieces(pos);
        issued[c] = 1;
        if ((int)inflight.size() > max_inflight) max_inflight = (int)inflight.size();
    };
    auto wait = [&](int n) {
        ++waits;
        while ((int)inflight.size() > n) {
            --left[inflight.front()];
            inflight.pop_front();
        }
    };
    for (int i = 0; i < S::FILL && i < total; ++i) issue(i, i);
    int cslot = 0;
    for (long gi = 0; gi < total; ++gi) {
        const int pos = (int)(gi % S::PER_TILE);
        if (S::syncs(pos)) {
            if (S::steady(gi, total)) {
                wait(S::after(pos));
                ++steady;
            } else {
                wait(0);
            }
            barrier_at = gi;  // every wave has consumed the chunks before gi
            CHECK(consumed == gi - 1, "barrier before chunk %ld after consuming %ld", gi, consumed);
            for (int j = 0; j < S::GRP; ++j)
                if (gi + S::LEAD + j < total) issue(gi + S::LEAD + j, S::slot_after(cslot, S::LEAD + j));
        }
        CHECK(issued[gi] && left[gi] == 0, "chunk %ld (pos %d) read before it landed (%d pieces out)", gi, pos,
              left[gi]);
        CHECK(owner[cslot] == gi, "chunk %ld read from slot %d holding %ld", gi, cslot, owner[cslot]);
        consumed = gi;
        cslot = cslot == NSLOT - 1 ? 0 : cslot + 1;
    }
    std::printf("{\"d\": %d, \"dq\": %d, \"dv\": %d, \"slots\": %d, \"grp\": %d, \"tiles\": %d, \"waits\": %d, "
                "\"steady\": %d, \"max_inflight\": %d, \"ok\": %d}\n",
                D, DQ, DV, NSLOT, S::GRP, ntiles, waits, steady, max_inflight, !g_fail);
}

template <int D, int DQ, int DV>
static void all_rings() {
    for (int nt : {1, 2, 3, 9}) {
        run<D, DQ, DV, 3, 1>(nt);
        run<D, DQ, DV, 4, 1>(nt);  // the shipped ring
        run<D, DQ, DV, 5, 1>(nt);
        run<D, DQ, DV, 4, 2>(nt);
        if constexpr (D / DQ + D / DV >= 7) run<D, DQ, DV, 8, 1>(nt);
    }
}

template <int D>
static void all_tiles() {
    all_rings<D, 32, 32>();
    all_rings<D, 32, 64>();
    all_rings<D, 32, 128>();
    all_rings<D, 64, 32>();
    all_rings<D, 64, 64>();
    all_rings<D, 64, 128>();
    all_rings<D, 128, 32>();
    all_rings<D, 128, 64>();
    all_rings<D, 128, 128>();
}

int main() {
    all_tiles<384>();
    all_tiles<512>();
    return g_fail;
}
