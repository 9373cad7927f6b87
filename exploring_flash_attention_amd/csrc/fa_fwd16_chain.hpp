// fa_fwd16_chain.hpp -- the d = 128 final-mode forward as a persistent grid whose workgroups run
// a fixed list of query tiles back to back with no seam between them (round 5).
//   <- flash_attention_kernel    flash_attention_v1/CUDA/flash_attention_v1.h:161
//   <- flash_attention_kernel (tiled-d) flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230
//
// Why: in the one-shot grid (fa_fwd16_kernel.hpp) every 128-row query tile is a workgroup that
// pays a prologue (Q, K0, V0, K1 landing: 4.6 k cycles), a first QK^T outside the software
// pipeline (1.7 k) and an epilogue (2.6 k + 1 k of store retirement) -- 20 % of its life at C3
// (B32 H8 L1024: 16 KV steps per tile), covered only in part by the CU's other workgroup
// (DESIGN.md section 5, round 4 stamps).  Here the KV step stream runs across tiles: the step
// that finishes tile i's P.V also computes QK^T(0) of tile i+1 -- its K(0), K(1), V(0) were
// DMA'd into the ring by the two preceding steps exactly as within a tile, and its Q^T was
// loaded into the (then dead) Q registers during the P.V half of the step before -- so the
// only work between two tiles is tile i's O normalisation and stores.
//
// Schedule: a grid of exactly 2 workgroups per CU (one wave per SIMD each, as the one-shot
// kernel); workgroup b serves XCD group x = b % 8 (blocks b and b+8 share an XCD, observed
// dispatch -- speed only) and takes the group's items l, l + G/8, l + 2G/8, ... (l = b / 8), of
// the contiguous item range xcd_remap gives the group: at any time an XCD runs consecutive
// items, i.e. all query tiles of a few heads, which share their K / V in that XCD's L2.
// Every item runs the same step sequence, with no branch between step variants (a diamond of
// whole steps made the register allocator spill the Q^T fragments, 500+ bytes of scratch):
// step 0 stores the previous item's O (the first item's step 0 into an empty range, so its
// stores are dropped) and starts O and the row sums from zero; the last pair of steps fetches
// the next item's K(0), K(1), V(0) and Q^T and computes its S(0) -- after the workgroup's last
// item from empty ranges (zero tiles, an S(0) nobody reads).
//
// Measured (A/B in one process against the one-shot kernel, outputs
// bitwise equal -- the same steps in the same order): C3 +1 ... +2 %, L = 2048 +0.6 ... +1.2 %,
// C4 +0.3 %.  Tried and dropped: issue priority alternating between the CU's two workgroups
// with the real-time clock (a persistent grid loses the one-shot grid's alternating age
// priority; it measured within noise), the next Q pulled toward L2 a few steps before the
// seam (within noise), a lazy row max tested on the packed P bits (spilled, 3x slower).
//
// Requirements (checked by the launcher): contiguous [B, H, L, d], d = 128, Lk (fused: keys per
// block) a multiple of 128 of at least 256 (an even number >= 4 of 64-key tiles, so every item
// starts on ring parity 0 and its first and last step pairs differ), Lq a multiple of 128 (every O row of a
// tile exists: the stores need no row test), at least as many query tiles as workgroups.
#pragma once
#include "fa_fwd16_kernel.hpp"

// schedule switch kept for A/B builds (scripts/build_lite.sh); the default is the measured
// choice
#ifndef FA_EPI_LATE
#define FA_EPI_LATE 1  // EPI step: DMA pieces first, the previous item's stores behind them
#endif

namespace fa {

// MODE kFinal: items are query tiles, O stored.  MODE kFused (split-KV, scaled fp16 partials in
// fragment order, fa_fwd16_kernel.hpp's workspace): items are query tiles too, and a workgroup
// walks an item's key blocks in order as one chain (block s's normalised partial and {lse, e}
// stored during block s+1's step 0), then combines the tile's partials itself -- no counters,
// no hand-off, the combine with the registers free.  Measured against the one-shot fused
// kernel (outputs bitwise equal; profiles/r05/ab): B2 H2 L16384 at 16 partials 545 -> 503 us,
// B1 H8 L16384 1061 -> 991 us, C4 at 4 partials 2120 -> 2044 us, C4 at 16 (the reference's one
// block per workgroup) 3285 -> 3002 us.  The first version -- (tile, block) items chained in
// decode order with the last arriver combining in the middle of its chain -- lost 4-10x: the
// combine's serial loads under full register pressure.
template <typename T, int MODE>
__global__ __launch_bounds__(kThreads, 2) void fa_fwd16_chain_kernel(FwdArgs a, int nitems) {
    static_assert(MODE == kFinal || MODE == kFused, "chain modes");
    constexpr bool FUSED = MODE == kFused;
    using M = Mma<T>;
    using v8 = typename M::v8;
    constexpr int D = 128;
    constexpr int ROWB = D * 2;
    constexpr int kBK = 64;
    constexpr int TILEB = kBK * ROWB;
    constexpr int NKS = D / 32;
    constexpr int NKB = kBK / 16;
    constexpr int NQB = 2;
    constexpr int NDB = D / 16;
    constexpr int NKK = kBK / 32;
    constexpr float kThr = 4.f;
    constexpr int KA = 3, VA = 2;
    constexpr int EXPA = 28;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const kring = smem;
    char* const vring = smem + 2 * TILEB;

    // this workgroup's items: group x = blockIdx % 8 owns xcd_remap's contiguous range
    const int x = blockIdx.x & 7;
    const int iq = nitems >> 3, ir = nitems & 7;
    const int nl = gridDim.x >> 3, l = blockIdx.x >> 3;
    const int gstart = x < ir ? x * (iq + 1) : ir * (iq + 1) + (x - ir) * iq;
    const int gcnt = iq + (x < ir ? 1 : 0);
    const int nmine = l < gcnt ? (gcnt - l + nl - 1) / nl : 0;
    if (nmine == 0) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n16 = lane & 15, g = lane >> 4;
    const int ntiles = (int)((FUSED ? (int64_t)a.kv_per_split : a.Lk) / kBK);

    // per-item addressing: (query tile, b*h) of item j of this workgroup
    struct Item {
        const unsigned short* k;
        const unsigned short* v;
        const unsigned short* q;  // first row of the query tile
        int64_t o_row0;           // element offset of the tile's first O row
        int64_t q_rows;
        int64_t grp;              // bh * nqt + qt (fused: the tile's counter)
        int64_t blk;              // fused: the partial block (split, b*h, query tile)
    };
    // (every field wave-uniform: readfirstlane keeps the loop-carried item in SGPRs -- a
    // descriptor the compiler cannot prove uniform becomes a waterfall loop around each DMA)
    auto uni = [](const unsigned short* p) {
        const uint64_t u = (uint64_t)(size_t)p;
        const uint64_t lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)u);
        const uint64_t hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
        return (const unsigned short*)(size_t)(lo | (hi << 32));
    };
    auto item = [&](int j) {  // query tile w of this workgroup's list (fused: its split 0)
        const int w = __builtin_amdgcn_readfirstlane(gstart + l + nl * j);
        const int qt = w % a.nqt;
        const int64_t bh = w / a.nqt;
        const int64_t q0 = (int64_t)qt * kBQ;
        Item it;
        it.k = uni((const unsigned short*)a.k + bh * a.Lk * D);
        it.v = uni((const unsigned short*)a.v + bh * a.Lk * D);
        it.grp = bh * a.nqt + qt;
        it.blk = it.grp;
        it.q = uni((const unsigned short*)a.q + (bh * a.Lq + q0) * D);
        it.o_row0 = (bh * a.Lq + q0) * D;
        it.q_rows = a.Lq - q0 < kBQ ? a.Lq - q0 : kBQ;
        return it;
    };
    auto split_of = [&](const Item& t0, int sp) {  // fused: key block sp of the same query tile
        Item it = t0;
        const int64_t kv0 = (int64_t)sp * a.kv_per_split * D;
        it.k = uni(t0.k + kv0);
        it.v = uni(t0.v + kv0);
        it.blk = (int64_t)sp * a.BH * a.nqt + t0.grp;
        return it;
    };

    const int pg = (0x2130 >> (4 * g)) & 3;
    v8 qf[NQB][NKS];
    auto load_q = [&](const Item& it) {
        const __amdgpu_buffer_rsrc_t qrs = make_rsrc(uni(it.q), (it.q_rows - 1) * ROWB + ROWB);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks)
                qf[qb][ks] = __builtin_bit_cast(
                    v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, (wid * 32 + 16 * qb + n16) * ROWB + ks * 64 + pg * 16, 0, 0));
    };

    // LDS-DMA source offsets of this lane's pieces (fa_fwd16_kernel.hpp): the swizzled image is
    // produced by giving each lane the SOURCE chunk that lands at its destination
    constexpr int DPW = TILEB / 1024 / kWaves;
    int dma_src[DPW];
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
        const int b = (wid * DPW + i) * 1024 + lane * 16;
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        dma_src[i] = row * ROWB + ch * 16;
    }
    auto tile_rsrc = [&](const unsigned short* base, int t) {
        return make_rsrc32(uni(base + (int64_t)t * (TILEB / 2)), TILEB);
    };
    auto dma_tile = [&](const unsigned short* base, char* slot, int t) {
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(base, t);
#pragma unroll
        for (int i = 0; i < DPW; ++i) dma16(rs, slot + (wid * DPW + i) * 1024, dma_src[i], 0);
    };

    const int rho = 8 * ((n16 >> 2) & 1) + 4 * (n16 >> 3) + (n16 & 3);
    const unsigned kaddr = (unsigned)(size_t)kring + (rho >> 3) * (8 * ROWB) + 64 * (rho & 7) + 16 * (pg ^ ((rho >> 2) & 3));
    const int r0 = 8 * (g & 1) + 4 * (g >> 1) + (n16 >> 2);
    const int sw = (r0 >> 2) & 3, c0 = (n16 >> 1) & 1;
    const unsigned vrow = (unsigned)(size_t)vring + (r0 >> 3) * (8 * ROWB) + 64 * (r0 & 7) + 8 * (n16 & 1);
    const unsigned vb_e = vrow + 16 * (c0 ^ sw);
    const unsigned vb_o = vrow + 16 * ((2 + c0) ^ sw);

    f32x4 o[NDB][NQB];
    f32x4 rs[NQB];
    float m[NQB];
    v8 ones;
    {
        constexpr unsigned kOne = std::is_same_v<T, __bf16> ? 0x3F80u : 0x3C00u;
        ones = __builtin_bit_cast(v8, u32x4{kOne | (kOne << 16), kOne | (kOne << 16), kOne | (kOne << 16),
                                            kOne | (kOne << 16)});
    }
    const float c = a.scale_log2;

    auto kread_ = [](auto r_c, auto slot_c, u32x4 (&kf)[KA + 1], unsigned ka) {
        constexpr int R = decltype(r_c)::value, KS = R / NKB, KB = R % NKB, SL = decltype(slot_c)::value;
        constexpr int OFF = SL * TILEB + KB * 16 * ROWB + KS * 512;
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[R % (KA + 1)]) : "v"(ka), "i"(OFF) : "memory");
    };
    auto vread_ = [](auto p_c, auto slot_c, u32x2 (&vf)[VA + 1][2], unsigned ve, unsigned vo) {
        constexpr int PP = decltype(p_c)::value, KK = PP / NDB, DB = PP % NDB, SL = decltype(slot_c)::value;
        constexpr int OFF = SL * TILEB + KK * 32 * ROWB + 512 * (DB >> 1);
        if constexpr (DB & 1) {
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][0]) : "v"(vo), "i"(OFF) : "memory");
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][1]) : "v"(vo), "i"(OFF + 16 * ROWB) : "memory");
        } else {
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][0]) : "v"(ve), "i"(OFF) : "memory");
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][1]) : "v"(ve), "i"(OFF + 16 * ROWB) : "memory");
        }
    };
    auto lwait = [](auto n_c, u32x4& reg) {
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(reg) : "i"(decltype(n_c)::value) : "memory");
    };
    auto lwait2 = [](auto n_c, u32x2 (&reg)[2]) {
        asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(reg[0]), "+v"(reg[1]) : "i"(decltype(n_c)::value) : "memory");
    };
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };

    auto qk_all = [&](auto slot_c, f32x4 (&s)[NKB][NQB]) {
        u32x4 kf[KA + 1];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) s[kb][qb] = f32x4{};
        static_for<KA>([&](auto r_c) { kread_(r_c, slot_c, kf, kaddr); });
        static_for<NKS * NKB>([&](auto s_c) {
            constexpr int S = decltype(s_c)::value;
            if constexpr (S + KA < NKS * NKB) kread_(std::integral_constant<int, S + KA>{}, slot_c, kf, kaddr);
            constexpr int AFTER = (S + KA < NKS * NKB ? S + KA : NKS * NKB - 1) - S;
            lwait(std::integral_constant<int, AFTER>{}, kf[S % (KA + 1)]);
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb)
                s[S % NKB][qb] = M::mma16(__builtin_bit_cast(v8, kf[S % (KA + 1)]), qf[qb][S / NKB], s[S % NKB][qb]);
        });
    };
    auto chain_max = [](const f32x4 (&s)[NKB][NQB], auto ch_c, auto h_c, float& acc) {
        constexpr int CH = decltype(ch_c)::value, H = decltype(h_c)::value;
        constexpr int QB = CH / 2, KB = 2 * (CH % 2) + H;
        if constexpr (H == 0)
            acc = fmax_nc(fmax_nc(fmax_nc(s[KB][QB][0], s[KB][QB][1]), s[KB][QB][2]), s[KB][QB][3]);
        else
            acc = fmax_nc(fmax_nc(fmax_nc(fmax_nc(acc, s[KB][QB][0]), s[KB][QB][1]), s[KB][QB][2]), s[KB][QB][3]);
    };
    auto rowmax_all = [&](const f32x4 (&s)[NKB][NQB], float (&mx)[NQB]) {
        float m4[4];
        static_for<8>([&](auto i_c) {
            constexpr int I = decltype(i_c)::value;
            chain_max(s, std::integral_constant<int, I / 2>{}, std::integral_constant<int, I % 2>{}, m4[I / 2]);
        });
        quad_max2(fmax_nc(m4[0], m4[1]), fmax_nc(m4[2], m4[3]), mx[0], mx[1]);
        mx[0] *= c;
        mx[1] *= c;
    };

    // O rows of the previous item, normalised and stored while the next item's first step runs
    // (EPI): lane (g, n) holds O^T[16*db + 4*g + i][query 16*qb + n]; dv blocks 2e and 2e+1 are
    // paired by one v_permlane16_swap per dword into a 16-byte row store (fa_fwd16_kernel.hpp)
    const int o_lane = (wid * 32 + n16) * ROWB + 2 * (16 * (g & 1) + 8 * (g >> 1));
    float einv[NQB] = {0.f, 0.f};  // 1 / row sum (fused: times 2^-e) of the item whose O is still in the registers
    float elsev[NQB] = {0.f, 0.f};  // fused: its lse (log2 units) and per-row scale exponent e
    float eesc[NQB] = {0.f, 0.f};
    // row group G = (query block G / 4, dv blocks 2 (G % 4), +1) of v * inv as 16-bit rows
    auto store_rows = [&](auto g_c, const f32x4 (&v)[NDB], float inv, __amdgpu_buffer_rsrc_t ors) {
        constexpr int G = decltype(g_c)::value, QB = G / 4, E = G % 4;
        const unsigned x0 = pack2<T>(v[2 * E][0] * inv, v[2 * E][1] * inv);
        const unsigned x1 = pack2<T>(v[2 * E][2] * inv, v[2 * E][3] * inv);
        const unsigned y0 = pack2<T>(v[2 * E + 1][0] * inv, v[2 * E + 1][1] * inv);
        const unsigned y1 = pack2<T>(v[2 * E + 1][2] * inv, v[2 * E + 1][3] * inv);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{s0[0], s1[0], s0[1], s1[1]}, ors,
                                               o_lane + QB * 16 * ROWB + E * 64, 0, 0);
    };
    auto store_group = [&](auto g_c, __amdgpu_buffer_rsrc_t ors) {
        constexpr int QB = decltype(g_c)::value / 4;
        f32x4 v[NDB];
#pragma unroll
        for (int db = 0; db < NDB; ++db) v[db] = o[db][QB];
        store_rows(g_c, v, einv[QB], ors);
    };
    auto o_rsrc = [&](const Item& it) { return make_rsrc(uni((const unsigned short*)a.o + it.o_row0), kBQ * ROWB); };

    // fused: the workspace of fa_fwd16_kernel.hpp's kFused mode -- per (split, b*h, query tile)
    // block the normalised partial (scaled fp16) in fragment order, lse and e per row
    constexpr int SC1 = 16;      // cache-policy bit: sc1
    constexpr int NF = NDB * NQB;  // fragments (4 values) per lane
    constexpr int BLK = kBQ * D;   // partial elements per block
    struct Epi {
        __amdgpu_buffer_rsrc_t o, l, e;
    };
    auto epi_of = [&](int64_t blk) {
        Epi ep;
        ep.o = make_rsrc(uni((const unsigned short*)a.o + blk * BLK), (int64_t)BLK * 2);
        ep.l = make_rsrc(a.lse + blk * kBQ, (int64_t)kBQ * 4);
        ep.e = make_rsrc(a.esc + blk * kBQ, (int64_t)kBQ * 4);
        return ep;
    };
    auto frag_off = [&](int f) { return ((wid * NF + f) * 64 + lane) * 8; };
    auto lse_off = [&](int qb) { return (wid * 32 + 16 * qb + n16) * 4; };
    auto part_store = [&](auto f_c, const Epi& ep) {  // fragment f = db * NQB + qb
        constexpr int F = decltype(f_c)::value, DB = F / NQB, QB = F % NQB;
        const f32x4 x = o[DB][QB] * einv[QB];
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2<_Float16>(x[0], x[1]), pack2<_Float16>(x[2], x[3])}, ep.o,
                                              frag_off(F), 0, SC1);
    };
    auto lse_store = [&](const Epi& ep) {  // (the 4 lanes of a row store the same value)
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(elsev[qb]), ep.l, lse_off(qb), 0, SC1);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(eesc[qb]), ep.e, lse_off(qb), 0, SC1);
        }
    };
    // fused: the item's partial is complete (O, row sums, m): its scale and lse
    auto finish_partial = [&]() {
        float mxa[NQB];
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            float mv = 0.f;
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int i = 0; i < 4; ++i) mv = fmax_nc(mv, __builtin_fabsf(o[db][qb][i]));
            mxa[qb] = mv;
        }
        quad_max2(mxa[0], mxa[1], mxa[0], mxa[1]);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            const float lsum = rs[qb][0];
            const float inv = 1.f / lsum;
            const int e = __builtin_amdgcn_frexp_expf(mxa[qb] * inv);
            eesc[qb] = (float)e;
            einv[qb] = __builtin_amdgcn_ldexpf(inv, -e);
            elsev[qb] = m[qb] + __builtin_amdgcn_logf(lsum);  // lse in log2 units: m + log2(l)
        }
    };
    // fused: the tile's partials summed in split order 0, 1, ... (fa_fwd16_kernel.hpp's combine,
    // the same order and arithmetic: bitwise the one-shot kernel's O) and O written
    // The last block's partial is never stored: it is still in the registers (o, einv, elsev,
    // eesc), rounded here exactly as part_store would round it; its ranges are empty (loads
    // return 0 and move no bytes).
    auto combine = [&](int64_t grp, int64_t o_row0) {
        const int ns = a.nsplit;
        const int own = ns - 1;
        auto blk_of = [&](int sp) { return (int64_t)sp * a.BH * a.nqt + grp; };
        auto epi_c = [&](int sp) {
            Epi ep = epi_of(blk_of(sp));
            if (sp == own) ep = Epi{make_rsrc(a.lse, 0), make_rsrc(a.lse, 0), make_rsrc(a.lse, 0)};
            return ep;
        };
        const __amdgpu_buffer_rsrc_t ofin = make_rsrc(uni((const unsigned short*)a.o_final + o_row0), kBQ * ROWB);
        // (U key blocks' loads in flight at a time: the walk schedule runs this between tiles,
        // where nothing hides its latency; an index past the last block re-reads the last one,
        // harmless to the maxima and given weight 0 in the sums -- the same sums in the same
        // order, as acc never holds -0)
        constexpr int U = 4;
        // (at most U blocks: everything loaded in one batch, one memory round trip, not two)
        static_for<NQB>([&](auto qb_c) {
            constexpr int QB = decltype(qb_c)::value;
            auto load_batch = [&](int sp0, float (&lv)[U], float (&ev)[U], u32x2 (&pv)[U][NDB]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int sp = sp0 + u < ns ? sp0 + u : ns - 1;
                    const Epi ep = epi_c(sp);
                    lv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ep.l, lse_off(QB), 0, SC1));
                    ev[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ep.e, lse_off(QB), 0, SC1));
#pragma unroll
                    for (int db = 0; db < NDB; ++db)
                        pv[u][db] = __builtin_bit_cast(
                            u32x2, __builtin_amdgcn_raw_buffer_load_b64(ep.o, frag_off(db * NQB + QB), 0, SC1));
                    if (sp == own) {
                        lv[u] = elsev[QB];
                        ev[u] = eesc[QB];
#pragma unroll
                        for (int db = 0; db < NDB; ++db) {
                            const f32x4 x = o[db][QB] * einv[QB];
                            pv[u][db] = u32x2{pack2<_Float16>(x[0], x[1]), pack2<_Float16>(x[2], x[3])};
                        }
                    }
                }
            };
            float Mx = -INFINITY, E = -1000.f;
            f32x4 acc[NDB];
#pragma unroll
            for (int db = 0; db < NDB; ++db) acc[db] = f32x4{};
            float wsum = 0.f;
            auto accumulate = [&](int sp0, const float (&lv)[U], const float (&ev)[U], const u32x2 (&pv)[U][NDB]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float wgt = sp0 + u < ns ? __builtin_amdgcn_exp2f(lv[u] - Mx) : 0.f;
                    const float wv = __builtin_amdgcn_ldexpf(wgt, (int)(ev[u] - E));
#pragma unroll
                    for (int db = 0; db < NDB; ++db) {
                        f32x4 r;
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            const unsigned wd = pv[u][db][jj >> 1];
                            r[jj] = (float)__builtin_bit_cast(_Float16, (unsigned short)((jj & 1) ? (wd >> 16) : (wd & 0xffff)));
                        }
                        acc[db] += wv * r;
                    }
                    wsum += wgt;
                }
            };
            if (ns <= U) {
                float lv[U], ev[U];
                u32x2 pv[U][NDB];
                load_batch(0, lv, ev, pv);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    Mx = fmaxf(Mx, lv[u]);
                    E = fmaxf(E, ev[u]);
                }
                accumulate(0, lv, ev, pv);
            } else {
                for (int sp0 = 0; sp0 < ns; sp0 += U) {
                    float lv[U], ev[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int sp = sp0 + u < ns ? sp0 + u : ns - 1;
                        const Epi ep = epi_c(sp);
                        lv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ep.l, lse_off(QB), 0, SC1));
                        ev[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ep.e, lse_off(QB), 0, SC1));
                        if (sp == own) {
                            lv[u] = elsev[QB];
                            ev[u] = eesc[QB];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        Mx = fmaxf(Mx, lv[u]);
                        E = fmaxf(E, ev[u]);
                    }
                }
                for (int sp0 = 0; sp0 < ns; sp0 += U) {
                    float lv[U], ev[U];
                    u32x2 pv[U][NDB];
                    load_batch(sp0, lv, ev, pv);
                    accumulate(sp0, lv, ev, pv);
                }
            }
            const float inv_w = 1.f / wsum;
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[db][i] = __builtin_amdgcn_ldexpf(acc[db][i] * inv_w, (int)E);
            static_for<4>([&](auto e_c) { store_rows(std::integral_constant<int, 4 * QB + decltype(e_c)::value>{}, acc, 1.f, ofin); });
        });
    };

    // One step of fa_fwd16_kernel.hpp (see there); what differs is only where the tiles come
    // from: krs / vrs describe the K tile fetched now (t+2, possibly the next item's 0 or 1)
    // and the V tile (t+1, possibly the next item's 0), and QK^T(t+1) reads whatever Q^T the
    // registers hold -- the next item's during the last step of an item.  Flags: 1 MORE (a tile
    // t+1 exists: QK^T, row max, V DMA), 4 DMAK (a K tile is fetched), 8 QNEXT (the next item's
    // Q^T is loaded in phase B, after phase A's last read of the current one, and the closing
    // barrier leaves those loads in flight), 32 EPI (step 0 of an item whose predecessor's O is
    // still in the registers: phase A stores it -- final: one 16-byte row store per even slot,
    // fused: one partial fragment per slot and the {lse, e} pairs -- and phase B's first P.V /
    // row-sum MFMAs start from zero instead of accumulating).
#if FA_STAMPS
    int stampv = 0, stamp_k = 0;
    const unsigned long long stamp_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    auto step = [&](auto par_c, auto flags_c, f32x4 (&sc)[NKB][NQB], f32x4 (&sn)[NKB][NQB], float (&mx)[NQB],
                    __amdgpu_buffer_rsrc_t krs, __amdgpu_buffer_rsrc_t vrs, const Item& nxt, const Epi& ep) {
        constexpr int P = decltype(par_c)::value;
        constexpr int F = decltype(flags_c)::value;
#if FA_STAMPS
        // (diagnostic builds: the start of each of the first 64 steps, lane k of a VGPR -- no
        // memory operation inside the loop; written out after it)
        if (stamp_k < 64)
        {
            const int tnow = (int)(unsigned)__builtin_amdgcn_s_memtime();
            stampv = lane == stamp_k ? tnow : stampv;
        }
        ++stamp_k;
#endif
        constexpr bool MORE = F & 1;
        constexpr bool DMAK = F & 4;
        constexpr bool QNEXT = F & 8;
        constexpr bool EPI = F & 32;
        using SLN = std::integral_constant<int, 1 - P>;
        using SLC = std::integral_constant<int, P>;
        if (!EPI && __builtin_amdgcn_ballot_w64(mx[0] > m[0] + kThr || mx[1] > m[1] + kThr)) {
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) {
                const float m_new = fmaxf(m[qb], mx[qb]);
                const float alpha = __builtin_amdgcn_exp2f(m[qb] - m_new);
                m[qb] = m_new;
                rs[qb] *= alpha;
#pragma unroll
                for (int db = 0; db < NDB; ++db) o[db][qb] *= alpha;
            }
        }
        const float nm0 = -m[0], nm1 = -m[1];
        char* const kdst = kring + P * TILEB + wid * DPW * 1024;
        char* const vdst = vring + (1 - P) * TILEB + wid * DPW * 1024;

        // score e of tile t: key step e / 16, query block (e / 8) & 1, key block 2*(e/16) + (e/4)&1, reg e&3
        auto ex = [&](auto e_c) {
            constexpr int E = decltype(e_c)::value, KK = E / 16, QB = (E / 8) & 1, KB = 2 * KK + ((E / 4) & 1), I = E & 3;
            sc[KB][QB][I] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[KB][QB][I], c, QB ? nm1 : nm0));
        };
        u32x4 pbu[NKK][NQB];  // packed P^T fragments
        auto cvt = [&](auto k_c) {  // pair k: key step k / 8, query block (k / 4) & 1, dword k % 4
            constexpr int K = decltype(k_c)::value, KK = K / 8, QB = (K / 4) & 1, J = K % 4;
            constexpr int KB = 2 * KK + (J >> 1), I = 2 * (J & 1);
            pbu[KK][QB][J] = pack2<T>(sc[KB][QB][I], sc[KB][QB][I + 1]);
        };
        auto dma = [&](auto i_c) {
            constexpr int I = decltype(i_c)::value;
            if constexpr (I < DPW) {
                if constexpr (DMAK) dma16(krs, kdst + I * 1024, dma_src[I], 0);
            } else if constexpr (MORE) {
                dma16(vrs, vdst + (I - DPW) * 1024, dma_src[I - DPW], 0);
            }
        };

        // ---- phase A: QK^T(t+1) || exponentials of t (and, EPI, the previous item's O stores)
        if constexpr (MORE) __builtin_amdgcn_s_setprio(1);
        u32x4 kf[KA + 1];
        if constexpr (MORE) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int qb = 0; qb < NQB; ++qb) sn[kb][qb] = f32x4{};
            static_for<KA>([&](auto r_c) { kread_(r_c, SLN{}, kf, kaddr); });
        }
        static_for<16>([&](auto s_c) {
            constexpr int S = decltype(s_c)::value;
            if constexpr (MORE) {
                if constexpr (S + KA < 16) kread_(std::integral_constant<int, S + KA>{}, SLN{}, kf, kaddr);
                constexpr int AFTER = (S + KA < 16 ? S + KA : 15) - S;
                lwait(std::integral_constant<int, AFTER>{}, kf[S % (KA + 1)]);
#pragma unroll
                for (int qb = 0; qb < NQB; ++qb)
                    sn[S % NKB][qb] = M::mma16(__builtin_bit_cast(v8, kf[S % (KA + 1)]), qf[qb][S / NKB], sn[S % NKB][qb]);
            }
            constexpr int E0 = S * EXPA / 16, E1 = (S + 1) * EXPA / 16;
            static_for<E1 - E0>([&](auto j_c) { ex(std::integral_constant<int, E0 + decltype(j_c)::value>{}); });
            if constexpr (S >= 6 && S < 14) cvt(std::integral_constant<int, S - 6>{});  // key step 0 packs
            if constexpr (EPI && FA_EPI_LATE) {
                // the DMA pieces in slots 0..7, the previous item's stores behind them in 8..15,
                // so that the closing barrier waits for the pieces only (vmcnt counts stores too,
                // in issue order; __syncthreads' fence would drain the stores: their write
                // latency, 1-2 us, at every item boundary)
                if constexpr (S < 8) dma(std::integral_constant<int, S>{});
                if constexpr (!FUSED && S >= 8) store_group(std::integral_constant<int, S - 8>{}, ep.o);
                if constexpr (FUSED && S >= 8) {
                    part_store(std::integral_constant<int, 2 * (S - 8)>{}, ep);
                    part_store(std::integral_constant<int, 2 * (S - 8) + 1>{}, ep);
                    if constexpr (S == 8) lse_store(ep);
                }
            } else {
                if constexpr (S % 2 == 1) dma(std::integral_constant<int, S / 2>{});
                if constexpr (EPI && !FUSED && S % 2 == 0) store_group(std::integral_constant<int, S / 2>{}, ep.o);
                if constexpr (EPI && FUSED) {
                    part_store(std::integral_constant<int, S>{}, ep);
                    if constexpr (S == 0) lse_store(ep);
                }
            }
            if constexpr (MORE) fence();
        });

        // ---- phase B: P.V(t) || exponentials of t (rest), row max of t+1
        __builtin_amdgcn_s_setprio(0);
        if constexpr (QNEXT) {  // phase A read the current Q^T for the last time
            load_q(nxt);
            fence();
        }
        u32x2 vf[VA + 1][2];
        float m4[4];
        static_for<VA>([&](auto p_c) { vread_(p_c, SLC{}, vf, vb_e, vb_o); });
        static_for<18>([&](auto j_c) {
            constexpr int J = decltype(j_c)::value;
            constexpr int KK = J / 9, JJ = J % 9;
            if constexpr (JJ < 8) {
                constexpr int PP = KK * NDB + JJ;
                if constexpr (PP + VA < NKK * NDB) vread_(std::integral_constant<int, PP + VA>{}, SLC{}, vf, vb_e, vb_o);
                constexpr int AFTER = 2 * ((PP + VA < NKK * NDB ? PP + VA : NKK * NDB - 1) - PP);
                lwait2(std::integral_constant<int, AFTER>{}, vf[PP % (VA + 1)]);
                const u32x4 vv = {vf[PP % (VA + 1)][0][0], vf[PP % (VA + 1)][0][1], vf[PP % (VA + 1)][1][0],
                                  vf[PP % (VA + 1)][1][1]};
#pragma unroll
                for (int qb = 0; qb < NQB; ++qb)
                    o[JJ][qb] = M::mma16(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbu[KK][qb]),
                                         EPI && KK == 0 ? f32x4{} : o[JJ][qb]);
            } else {
#pragma unroll
                for (int qb = 0; qb < NQB; ++qb)
                    rs[qb] = M::mma16(ones, __builtin_bit_cast(v8, pbu[KK][qb]), EPI && KK == 0 ? f32x4{} : rs[qb]);
            }
            // exponentials EXPA..31, two per slot; key step 1 packs in slots 1..8
            if constexpr (EXPA + 2 * J < 32) ex(std::integral_constant<int, EXPA + 2 * J>{});
            if constexpr (EXPA + 2 * J + 1 < 32) ex(std::integral_constant<int, EXPA + 2 * J + 1>{});
            if constexpr (J >= 1 && J <= 8) cvt(std::integral_constant<int, 8 + J - 1>{});
            if constexpr (MORE) {
                // row max of tile t+1: chain (J - 8) / 2, half (J - 8) % 2 in slots 8..15
                if constexpr (J >= 8 && J < 16)
                    chain_max(sn, std::integral_constant<int, (J - 8) / 2>{}, std::integral_constant<int, (J - 8) % 2>{},
                              m4[(J - 8) / 2]);
                if constexpr (J == 16) {
                    quad_max2(fmax_nc(m4[0], m4[1]), fmax_nc(m4[2], m4[3]), mx[0], mx[1]);
                    mx[0] *= c;
                    mx[1] *= c;
                }
            }
            fence();
        });
        if constexpr (QNEXT) {
            // the K / V pieces issued before the Q loads have landed (their 2 * DPW pieces are
            // older than the 8 Q loads); the Q loads stay in flight into the next step, whose
            // first QK^T MFMA the compiler makes wait for them
            static_assert(NQB * NKS == 8, "vmcnt count of the Q loads");
            asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        } else if constexpr (EPI && FA_EPI_LATE) {
            // every DMA piece landed; the stores (the youngest NST operations) stay in flight
            // (slots 8..15 issue them: final 8 store_group, one 16-byte row store each; fused 2
            // part_store per slot plus lse_store's 2 x NQB -- the ISA check of tests/test_vmcnt.py
            // verifies the emitted order)
            constexpr int NST = FUSED ? NF + 2 * NQB : 8;
            static_assert(NQB * (NDB / 2) == 16 - 8, "final EPI: one row store per slot 8..15");
            static_assert(NF == 2 * (16 - 8), "fused EPI: two partial fragments per slot 8..15");
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(NST) : "memory");
        } else {
            __syncthreads();  // hipcc drains the DMA (vmcnt(0)) here: K(t+2), V(t+1) landed
        }
    };

    // prologue of an item's first tile (fa_fwd16_kernel.hpp's): Q, K(0), V(0), K(1); S(0)
    f32x4 sa[NKB][NQB], sb[NKB][NQB];
    float mx[NQB];
    // (in two halves: the walk issues a tile's loads before the previous tile's combine)
    auto prologue_issue = [&](const Item& it) {
        load_q(it);
        dma_tile(it.k, kring, 0);
        dma_tile(it.v, vring, 0);
        dma_tile(it.k, kring + TILEB, 1);
    };
    auto prologue_finish = [&]() {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[qb][ks]));
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * DPW) : "memory");
        qk_all(std::integral_constant<int, 0>{}, sa);
        rowmax_all(sa, mx);
        m[0] = mx[0];  // the reference max starts at tile 0's row max (no step-0 rescale)
        m[1] = mx[1];
        __syncthreads();
    };
    auto prologue = [&](const Item& it) {
        prologue_issue(it);
        prologue_finish();
    };

    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using STEADY = std::integral_constant<int, 1 | 4>;
    Item cur = item(0);
    const __amdgpu_buffer_rsrc_t none = make_rsrc32(cur.k, 0);
    const Epi enone = {none, none, none};

    if constexpr (!FUSED) {
        prologue(cur);
        Epi prev_ep = enone;  // where the previous item's O goes
        for (int j = 0;; ++j) {
            const bool more = j + 1 < nmine;
            // after the last item the "next" Q^T load is an empty range too (q_rows = 0: the
            // loads return zeros and move no bytes) -- reloading the current tile's Q^T there
            // cost 32 KiB of L2 misses per workgroup, +17 MB (+6 %) of reads at C3 in the round-5
            // kernel (profiles/r06/pmc_fetch.txt), and its latency sat on the workgroup's tail
            Item nxt = item(more ? j + 1 : j);
            nxt.q_rows = more ? nxt.q_rows : 0;
            // t = 0, 1 (step 0 stores the previous item's O)
            step(C0{}, std::integral_constant<int, 1 | 4 | 32>{}, sa, sb, mx, tile_rsrc(cur.k, 2), tile_rsrc(cur.v, 1),
                 nxt, prev_ep);
            step(C1{}, STEADY{}, sb, sa, mx, tile_rsrc(cur.k, 3), tile_rsrc(cur.v, 2), nxt, enone);
            int t = 2;
            for (; t + 2 < ntiles; t += 2) {
                step(C0{}, STEADY{}, sa, sb, mx, tile_rsrc(cur.k, t + 2), tile_rsrc(cur.v, t + 1), nxt, enone);
                step(C1{}, STEADY{}, sb, sa, mx, tile_rsrc(cur.k, t + 3), tile_rsrc(cur.v, t + 2), nxt, enone);
            }
            // t = ntiles - 2: K(t+2) = the next item's K(0) into K slot 0, V(t+1) ours; the next
            // Q^T loaded in phase B.  t = ntiles - 1: K(t+2) = next K(1) into slot 1, V(t+1) =
            // next V(0) into slot 0; QK^T(next 0) -> sa and its row max -> mx
            step(C0{}, std::integral_constant<int, 1 | 4 | 8>{}, sa, sb, mx, more ? tile_rsrc(nxt.k, 0) : none,
                 tile_rsrc(cur.v, t + 1), nxt, enone);
            step(C1{}, STEADY{}, sb, sa, mx, more ? tile_rsrc(nxt.k, 1) : none, more ? tile_rsrc(nxt.v, 0) : none,
                 nxt, enone);
            // this item's O stays in the registers until the next item's step 0 stores it
            einv[0] = 1.f / rs[0][0];
            einv[1] = 1.f / rs[1][0];
            prev_ep = Epi{o_rsrc(cur), none, none};
            m[0] = mx[0];
            m[1] = mx[1];
            if (!more) break;
            cur = nxt;
        }
        static_for<8>([&](auto g_c) { store_group(g_c, prev_ep.o); });
#if FA_STAMPS
        // slots per workgroup (80): 0..63 step starts (s_memtime, low 32 bits), 64 loop end,
        // 65 / 66 s_memrealtime at entry / loop end, 67 HW_ID, 68 XCC_ID (scripts/chain_stamps.py)
        {
            const unsigned long long t_end = __builtin_amdgcn_s_memtime();
            const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
            if (tid < 64) g_fa_stamps[blockIdx.x * 80 + tid] = (unsigned)stampv;
            if (tid == 0) {
                g_fa_stamps[blockIdx.x * 80 + 64] = (unsigned)t_end;
                g_fa_stamps[blockIdx.x * 80 + 65] = stamp_rt0;
                g_fa_stamps[blockIdx.x * 80 + 66] = rt_end;
                g_fa_stamps[blockIdx.x * 80 + 67] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
                g_fa_stamps[blockIdx.x * 80 + 68] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
            }
        }
#endif
    } else {
        // Split-KV, the reference's layout (one partial per key block in the workspace,
        // flash_attention_v2/CUDA/flash_attention_v2.h:243-341): a workgroup walks the key blocks
        // of its query tiles in order, chained like the final mode's items (block s's partial is
        // stored while block s+1's first step runs), and combines the tile's partials itself
        // once the last one is out -- its own stores, so no counter and no hand-off; the combine
        // runs with the registers free (between tiles), not inside the chain.
        const int ns = a.nsplit;
        for (int j = 0; j < nmine; ++j) {
            const Item t0 = j == 0 ? cur : item(j);
            if (j == 0) prologue_issue(t0);
            prologue_finish();
            Epi prev_ep = enone;
            for (int sp = 0;; ++sp) {
                const bool more = sp + 1 < ns;
                const Item it = split_of(t0, sp);
                const Item nx = split_of(t0, more ? sp + 1 : sp);
                step(C0{}, std::integral_constant<int, 1 | 4 | 32>{}, sa, sb, mx, tile_rsrc(it.k, 2), tile_rsrc(it.v, 1),
                     nx, prev_ep);
                step(C1{}, STEADY{}, sb, sa, mx, tile_rsrc(it.k, 3), tile_rsrc(it.v, 2), nx, enone);
                int t = 2;
                for (; t + 2 < ntiles; t += 2) {
                    step(C0{}, STEADY{}, sa, sb, mx, tile_rsrc(it.k, t + 2), tile_rsrc(it.v, t + 1), nx, enone);
                    step(C1{}, STEADY{}, sb, sa, mx, tile_rsrc(it.k, t + 3), tile_rsrc(it.v, t + 2), nx, enone);
                }
                // the next block's K(0), K(1), V(0) (the same Q^T: no reload); after the last
                // block empty ranges (zero tiles, an S(0) nobody reads)
                step(C0{}, STEADY{}, sa, sb, mx, more ? tile_rsrc(nx.k, 0) : none, tile_rsrc(it.v, t + 1), nx, enone);
                step(C1{}, STEADY{}, sb, sa, mx, more ? tile_rsrc(nx.k, 1) : none, more ? tile_rsrc(nx.v, 0) : none, nx,
                     enone);
                finish_partial();
                prev_ep = epi_of(it.blk);
                m[0] = mx[0];
                m[1] = mx[1];
                if (!more) break;
            }
            // the combine, the last block's partial from the registers (the others' stores out
            // first), with the next tile's first K / V tiles already on their way (the ring is
            // free: the last step's barrier retired its reads) and its Q^T loaded after it, so
            // that those registers stay free for the combine (the whole prologue before it
            // spilled).  A/B (profiles/r05/ab/r05t_*, ov2 = this, ov0 = all after the combine):
            // C4 at 4 partials +0.2 %, at 16 within noise.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const bool nx = j + 1 < nmine;
            const Item tn = item(nx ? j + 1 : j);
            if (nx) {
                dma_tile(tn.k, kring, 0);
                dma_tile(tn.v, vring, 0);
                dma_tile(tn.k, kring + TILEB, 1);
            }
            combine(t0.grp, t0.o_row0);
            if (nx) load_q(tn);
        }
    }
}

}  // namespace fa
