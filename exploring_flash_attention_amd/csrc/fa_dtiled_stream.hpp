// fa_dtiled_stream.hpp -- the LDS ring protocol of the d-tiled kernel (fa_fwd_dtiled.hip) as
// constexpr C++ with no HIP in it, so that tests/native/dtiled_stream_test.cpp can replay it on
// the CPU for every instantiation: which chunk each wait makes readable, how many DMA pieces
// may stay in flight at it, which chunks go out after each barrier and into which slot.
//
// Per 64-key tile the stream holds NQC K chunks of DQ columns, then NVC V chunks of DV columns;
// a chunk is DQ / 32 (DV / 32) 1 KiB pieces per wave.  Chunk c lives in ring slot c % NSLOT.
//   GRP 1: before chunk gi: wait (pieces of the chunks issued after gi may stay in flight),
//          barrier, issue chunk gi + NSLOT - 1 into the slot chunk gi - 1 just left.
//   GRP 2: (4 slots) before the first chunk gi of each pair: wait until nothing is in flight,
//          barrier, issue the next pair gi + 2, gi + 3 into the slots of gi - 2, gi - 1.
#pragma once

namespace fa {

template <int D, int DQ, int DV, int NSLOT, int GRP_REQ>
struct DtStream {
    static constexpr int NQC = D / DQ, NVC = D / DV, PER_TILE = NQC + NVC;
    static constexpr int KPW = DQ / 32, VPW = DV / 32;
    static constexpr int GRP = (GRP_REQ == 2 && PER_TILE % 2 == 0 && NSLOT == 4) ? 2 : 1;
    static constexpr int LEAD = GRP == 2 ? 2 : NSLOT - 1;  // chunks between a consumer and the issue
    static constexpr int FILL = GRP == 2 ? 2 : NSLOT - 1;  // chunks issued before the loop
    static_assert(FILL <= PER_TILE, "the first ring fill lies within tile 0");
    static_assert(LEAD + GRP - 1 <= NSLOT - 1, "the chunks issued after a barrier fit the ring");

    static constexpr int pieces(int pos) { return pos < NQC ? KPW : VPW; }
    // a wait and a barrier come before the chunk at this position
    static constexpr bool syncs(int pos) { return GRP == 1 || pos % 2 == 0; }
    // pieces that may stay in flight at that wait in the steady state: those of the NSLOT - 2
    // chunks issued after chunk gi (GRP 1); nothing (GRP 2: only the pair itself is out)
    static constexpr int after(int pos) {
        int n = 0;
        if (GRP == 1)
            for (int i = 1; i <= NSLOT - 2; ++i) n += pieces((pos + i) % PER_TILE);
        return n;
    }
    // steady state: all NSLOT - 2 chunks after gi were issued (near the end of the stream fewer
    // were, and the wait drains everything)
    static constexpr bool steady(long gi, long total) { return GRP == 1 && gi + NSLOT - 1 <= total; }
    // ring slot of the chunk `ahead` chunks after the one in slot `cur`
    static constexpr int slot_after(int cur, int ahead) { return cur + ahead < NSLOT ? cur + ahead : cur + ahead - NSLOT; }
};

}  // namespace fa
