// fa_fwd_persist.hip -- persistent FA-v1 forward with per-XCD work queues (final mode,
// d = 32 / 64 / 128).
//
// Same maths, LDS tile image, LDS-DMA ring and step pipeline as fa_fwd_kernel (fa_fwd.hip;
// reference kernels flash_attention_v1/CUDA/flash_attention_v1.h:161,
// flash_attention_v1/CUDA/flash_attention_v1_opt1.h:264,
// flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230) -- outputs are bitwise equal --
// organised as resident workgroups that pull items (W*32-row query tile, b*h) from queues
// instead of one workgroup per item.  What the one-shot grid loses (phase stamps,
// scripts/stamps.py, C3 / C4):
//   * blocks go to XCDs round robin (b -> b % 8), so every XCD gets 1/8 of the work, but
//     under load the XCDs hold different clocks: at equal cycle counts per KV step the last
//     XCD finished 11 % after the first at C4.  Here each XCD drains its own queue (a
//     contiguous range of items, so the query tiles of one head share that XCD's L2) and
//     then helps the others;
//   * 16 % of a workgroup's life at C3 outside the KV loop.  Here the next item's K0, K1,
//     V0 (LDS-DMA into the ring slots the last step no longer reads) and Q (into the Q
//     registers, dead in the last step) are fetched during the item's last KV step, and the
//     next item's index is dequeued one item ahead.
// MEASURED (scripts/ab_run.sh, scripts/stamps_persist.py): slower than the one-shot
// grid at every shape, so it is off by default (FA_PERSIST=0).  Resident workgroups keep their
// age, and the older of the two on a CU keeps the VALU-issue priority: with static lists the
// workgroups' end times spread 1543-2072 us at C4 (C4 -5 %, C3 -10 %); with the queues that
// spread closes but a returning atomic under load costs ~6k cycles per item (C3 -25 %, C2 2x).
// FA_PQ_WAVES=8 (one 512-thread workgroup per CU, shared ring): the two barrier-synchronised
// waves of a SIMD run in lockstep, +24 % cycles per KV step (C3 -6 %, C2 -19 %).
// Queues: g_fa_queues holds 64 sets of {8 per-XCD heads, an exit counter}; a launch uses set
// (epoch % 64) and its last workgroup to exit zeroes the set for the next launch.  Two launches
// running at the same time must not share a set: at most 64 in flight (streams, graphs).
#include "fa_device.hpp"

#ifndef FA_PQ_STEAL
#define FA_PQ_STEAL 1  // 0: static per-XCD round robin (no queues), for A/B
#endif

// FA_STAMPS (diagnostic builds only): per workgroup, wave 0 accumulates s_memtime cycles of
// each phase over its items and writes them once at exit to g_fa_pq_stamps (never into an
// output): 0 entry, 1 exit, 2 sum of KV loops, 3 sum of item prologues (first QK^T), 4 sum
// of epilogues, 5 items, 6 hw_id, 7 xcc_id, 8 / 9 s_memrealtime at entry / exit.
#ifndef FA_STAMPS
#define FA_STAMPS 0
#endif
#if FA_STAMPS
__device__ unsigned long long g_fa_pq_stamps[4096 * 16];
extern "C" int fa_debug_pq_stamps(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fa_pq_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#define PQ_NOW() __builtin_amdgcn_s_memtime()
#else
#define PQ_NOW() 0ull
#endif

__device__ unsigned g_fa_queues[64 * 16];

namespace fa {

namespace {
// items of XCD x: [xbeg, xend) of n, split as evenly as xcd_remap splits blocks
__device__ __forceinline__ void xcd_range(int n, int x, int& beg, int& end) {
    const int q = n >> 3, r = n & 7;
    beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    end = beg + q + (x < r ? 1 : 0);
}
}  // namespace

template <typename T, int D, bool TAIL, int W>
__global__ __launch_bounds__(64 * W, 2) void fa_fwd_persist_kernel(FwdArgs a) {
    using M = Mma<T>;
    using v8 = typename M::v8;
    constexpr int ROWB = D * 2;               // bytes per LDS row
    constexpr int kBK = bk_for(D);            // keys per KV tile
    constexpr int TILEB = kBK * ROWB;         // bytes of one K (or V) tile
    constexpr int NKS = D / 16;               // MFMA k-steps of Q K^T
    constexpr int NDB = D / 32;               // 32-column blocks of O
    constexpr int NKB = kBK / 32;             // 32-key blocks per KV tile
    constexpr int BQ = 32 * W;                // query rows per item
    constexpr float kThr = 4.f;               // defer-max threshold (log2 units), as fa_fwd.hip

    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: K ring (2 slots), V ring (2 slots), then the dequeued item index
    char* const kring = smem;
    char* const vring = smem + 2 * TILEB;
    int* const next_slot = (int*)(smem + 4 * TILEB);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31;
    const int hf = lane >> 5;

    const int nitems = a.nqt * (int)a.BH;
    unsigned* const qset = g_fa_queues + 16 * (a.sched_epoch & 63);
    const int my_x = FA_PQ_STEAL ? (int)(__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 7) : (int)(blockIdx.x & 7);
    // next item (thread 0 only): own XCD's queue first, then the others'; -1 when all empty
    auto dequeue = [&]() -> int {
#if FA_PQ_STEAL
        for (int k = 0; k < 8; ++k) {
            const int y = (my_x + k) & 7;
            int beg, end;
            xcd_range(nitems, y, beg, end);
            if (beg >= end) continue;
            const unsigned i = __hip_atomic_fetch_add(qset + y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((int)i < end - beg) return beg + (int)i;
        }
        return -1;
#else
        return -1;  // static mode walks its own list (below)
#endif
    };
    int beg_s, end_s;  // static mode: blocks with equal b % 8 take one eighth, round robin
    xcd_range(nitems, (int)(blockIdx.x & 7), beg_s, end_s);
    [[maybe_unused]] const int J = (int)(gridDim.x >> 3), js = (int)(blockIdx.x >> 3);

    int item;
#if FA_PQ_STEAL
    if (tid == 0) *next_slot = dequeue();
    __syncthreads();
    item = __builtin_amdgcn_readfirstlane(*next_slot);
#else
    item = beg_s + js < end_s ? beg_s + js : -1;
#endif
    [[maybe_unused]] unsigned long long st_entry = PQ_NOW(), st_rt = FA_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0;
    [[maybe_unused]] unsigned long long st_loop = 0, st_pro = 0, st_epi = 0, st_n = 0, st_t0 = 0, st_t1 = 0;

    if (item >= 0) {
    const int nkv = (int)a.Lk;
    const int ntiles = (nkv + kBK - 1) / kBK;
    const float c = a.scale_log2;

    // ---- LDS-DMA geometry.  A tile is NDMA 1 KiB pieces; K pieces go to waves [0, NDMA),
    // V pieces to waves [W - NDMA, W) when a tile has fewer pieces than there are waves.
    constexpr int NDMA = TILEB / 1024;
    constexpr int DPW = NDMA >= W ? NDMA / W : 1;
    static_assert(NDMA % W == 0 || W % NDMA == 0, "tile pieces must split over waves");
    const int kpiece0 = NDMA >= W ? wid * DPW : wid;                // first K piece
    const int vpiece0 = NDMA >= W ? wid * DPW : wid - (W - NDMA);  // first V piece
    const bool kwave = NDMA >= W || wid < NDMA;
    const bool vwave = NDMA >= W || wid >= W - NDMA;
    auto src_of = [&](int piece) {  // source byte (in the tile) of this lane's 16 B of a piece
        const int b = piece * 1024 + lane * 16;
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        return row * ROWB + ch * 16;
    };
    int ksrc[DPW], vsrc[DPW];
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
        ksrc[i] = src_of(kpiece0 + i);
        vsrc[i] = src_of(vpiece0 + i);
    }
    auto tile_rsrc = [&](const unsigned short* base, int t) {
        const int rem = nkv - t * kBK;
        const int valid = TAIL ? __builtin_amdgcn_readfirstlane(rem < kBK ? (rem > 0 ? rem : 0) : kBK)
                               : (t < ntiles ? kBK : 0);
        return make_rsrc32((const char*)base + (int64_t)t * TILEB, valid * ROWB);
    };
    auto dma_k = [&](const unsigned short* base, char* slot, int t) {
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(base, t);
        if (kwave) {
#pragma unroll
            for (int i = 0; i < DPW; ++i) dma16(rs, slot + (kpiece0 + i) * 1024, ksrc[i], 0);
        }
    };
    auto dma_v = [&](const unsigned short* base, char* slot, int t) {
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(base, t);
        if (vwave) {
#pragma unroll
            for (int i = 0; i < DPW; ++i) dma16(rs, slot + (vpiece0 + i) * 1024, vsrc[i], 0);
        }
    };
    struct Item {
        const unsigned short *q, *k, *v;
        unsigned short* o;
        int64_t row0;  // first query row of this wave
    };
    auto item_at = [&](int it) {
        const int qt = it % a.nqt;
        const int64_t bh = it / a.nqt;
        Item r;
        r.row0 = (int64_t)qt * BQ + wid * 32;
        r.q = (const unsigned short*)a.q + bh * a.Lq * D;
        r.k = (const unsigned short*)a.k + bh * a.Lk * D;
        r.v = (const unsigned short*)a.v + bh * a.Lk * D;
        r.o = (unsigned short*)a.o + bh * a.Lq * D;
        return r;
    };
    v8 qf[NKS];
    // Q^T fragments (B operand) of an item: lane holds Q[row][16*ks + 8*hf + 0..7]; rows
    // past Lq read zeros (buffer range) and are never stored
    auto load_q = [&](const Item& it) {
        const __amdgpu_buffer_rsrc_t qrs = make_rsrc(it.q, a.Lq * ROWB);
        const int qoff = (int)((it.row0 + l32) * ROWB) + hf * 16;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[ks] = __builtin_bit_cast(v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, qoff + ks * 32, 0, 0));
    };

    // transposed-read geometry (constant per lane)
    const int grp = lane >> 4, gi = lane & 15;
    const int tr_row = 4 * (grp >> 1) + (gi >> 2);
    const int tr_col = 16 * (grp & 1) + 4 * (gi & 3);
    const unsigned vbase0 = (unsigned)(size_t)vring + lds_off<D>(tr_row, tr_col >> 3) + (tr_col & 7) * 2;
    const unsigned vbase1 =
        (unsigned)(size_t)vring + lds_off<D>(tr_row + 8, tr_col >> 3) + (tr_col & 7) * 2 - 8 * ROWB;
    auto read_v = [](auto slot_c, auto i_c, u32x2 (&vf)[2][2], unsigned vbase0, unsigned vbase1) {
        constexpr int SLOT = decltype(slot_c)::value, I = decltype(i_c)::value;
        constexpr int B2 = I / NDB, DB = I % NDB;
        constexpr int OFF = SLOT * TILEB + 4 * B2 * 8 * ROWB + 512 * DB;
        constexpr int SSO = 2 * 8 * ROWB;  // +16 key rows (k-step ss = 1)
        static_assert(OFF + SSO + 8 * ROWB < 65536, "ds offset field is 16 bits");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[0][0]) : "v"(vbase0), "i"(OFF) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[0][1]) : "v"(vbase1), "i"(OFF + 8 * ROWB) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[1][0]) : "v"(vbase0), "i"(OFF + SSO) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[1][1]) : "v"(vbase1), "i"(OFF + SSO + 8 * ROWB) : "memory");
    };
    auto vwait = [&](u32x2 (&vf)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vf[0][0]), "+v"(vf[0][1]), "+v"(vf[1][0]), "+v"(vf[1][1]));
    };

    f32x16 o[NDB];
    float m, l;

    // S^T[key][q] = K . Q^T for one tile; K fragments read in groups of two k-steps, one
    // group ahead (as fa_fwd.hip)
    auto qk = [&](const char* kb, f32x16 (&s)[NKB]) {
        constexpr int G2 = 2;
        v8 kf[2][NKB][G2];
        auto rd = [&](int g, v8 (&dst)[NKB][G2]) {
#pragma unroll
            for (int jj = 0; jj < G2; ++jj)
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2)
                    dst[b2][jj] = *(const v8*)(kb + lds_off<D>(b2 * 32 + l32, 2 * (g * G2 + jj) + hf));
        };
#pragma unroll
        for (int b2 = 0; b2 < NKB; ++b2) s[b2] = f32x16{};
        rd(0, kf[0]);
#pragma unroll
        for (int g = 0; g < NKS / G2; ++g) {
            if (g + 1 < NKS / G2) rd(g + 1, kf[(g + 1) & 1]);
#pragma unroll
            for (int jj = 0; jj < G2; ++jj)
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2) s[b2] = M::mma(kf[g & 1][b2][jj], qf[g * G2 + jj], s[b2]);
        }
    };
    auto exp_tile = [&](f32x16 (&s)[NKB]) {
        float sum4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s[b2][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[b2][i], c, -m));
                sum4[(b2 * 16 + i) & 3] += s[b2][i];
            }
        l += (sum4[0] + sum4[1]) + (sum4[2] + sum4[3]);
    };
    auto mask = [&](int t, f32x16 (&s)[NKB]) {
        const int valid = nkv - t * kBK;
        if (valid < kBK) {
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = b2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
                    if (key >= valid) s[b2][i] = -INFINITY;
                }
        }
    };
    auto rowmax = [&](const f32x16 (&s)[NKB], float& mx) {
        float mx4[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) mx4[jj] = s[0][jj];
#pragma unroll
        for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (b2 > 0 || i >= 4) mx4[i & 3] = fmaxf(mx4[i & 3], s[b2][i]);
        mx = pair_max(fmaxf(fmaxf(mx4[0], mx4[1]), fmaxf(mx4[2], mx4[3]))) * c;
    };

    Item cur = item_at(item);
    // One pipeline step for tile t (as fa_fwd.hip's step): DMA K(t+2), V(t+1); rescale
    // decision; QK^T(t+1) beside exp / sum of tile t; pack P; P.V(t); mask + row max of t+1;
    // barrier (drains the DMA).  LAST steps instead fetch the next item's K0 / K1 / V0 / Q.
    auto step = [&](auto par_c, auto flags_c, int t, f32x16 (&sc)[NKB], f32x16 (&sn)[NKB], float& mx,
                    bool has_next, const Item& nxt) {
        constexpr int P = decltype(par_c)::value;
        constexpr int F = decltype(flags_c)::value;
        constexpr bool MORE = F & 1, MASKNEXT = TAIL && (F & 2), DMAK = F & 4;
        if (__builtin_amdgcn_ballot_w64(mx > m + kThr)) {
            const float m_new = fmaxf(m, mx);
            const float alpha = __builtin_amdgcn_exp2f(m - m_new);
            m = m_new;
            l *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; ++db) o[db] *= alpha;
        }
        if constexpr (DMAK) dma_k(cur.k, kring + P * TILEB, t + 2);
        if constexpr (MORE) dma_v(cur.v, vring + (1 - P) * TILEB, t + 1);
        if constexpr (!MORE) {
            // last tile: no K is read any more, so both K slots take the next item's K0 / K1;
            // V0 goes to V slot 0 now if this tile's V sits in slot 1 (else after the P.V);
            // the Q registers are dead (no QK^T in this step): the next item's Q goes there
            if (has_next) {
                dma_k(nxt.k, kring, 0);
                if (ntiles > 1) dma_k(nxt.k, kring + TILEB, 1);
                if constexpr (P == 1) dma_v(nxt.v, vring, 0);
                load_q(nxt);
            }
        }
        if constexpr (MORE) qk(kring + (1 - P) * TILEB, sn);
        exp_tile(sc);
        v8 pb[NKB][2];
#pragma unroll
        for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                u32x4 u;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) u[jj] = pack2<T>(sc[b2][8 * ss + 2 * jj], sc[b2][8 * ss + 2 * jj + 1]);
                pb[b2][ss] = __builtin_bit_cast(v8, u);
            }
        u32x2 vcur[2][2], vnext[2][2];
        read_v(par_c, std::integral_constant<int, 0>{}, vcur, vbase0, vbase1);
        vwait(vcur);
        static_for<NKB * NDB>([&](auto i_c) {
            constexpr int I = decltype(i_c)::value;
            constexpr int B2 = I / NDB, DB = I % NDB;
            if constexpr (I + 1 < NKB * NDB)
                read_v(par_c, std::integral_constant<int, I + 1>{}, vnext, vbase0, vbase1);
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const u32x4 vv = {vcur[ss][0][0], vcur[ss][0][1], vcur[ss][1][0], vcur[ss][1][1]};
                o[DB] = M::mma(__builtin_bit_cast(v8, vv), pb[B2][ss], o[DB]);
            }
            if constexpr (I + 1 < NKB * NDB) {
                vwait(vnext);
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    vcur[ss][0] = vnext[ss][0];
                    vcur[ss][1] = vnext[ss][1];
                }
            }
        });
        if constexpr (MORE) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (MASKNEXT) mask(t + 1, sn);
            rowmax(sn, mx);
        }
        __syncthreads();  // drains the DMA (vmcnt(0)): K(t+2), V(t+1) (or the next item's) landed
        // last tile in V slot 0: the next item's V0 goes there once every wave is past its
        // P.V reads; it lands by the barrier after the next item's first QK^T
        if constexpr (!MORE && P == 0) {
            if (has_next) dma_v(nxt.v, vring, 0);
        }
    };

    // ---- first item: Q -> registers, K0, V0, K1 -> LDS
    load_q(cur);
    dma_k(cur.k, kring, 0);
    dma_v(cur.v, vring, 0);
    if (ntiles > 1) dma_k(cur.k, kring + TILEB, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f32x16 sa[NKB], sb[NKB];
    float mx;
    while (true) {
        st_t0 = PQ_NOW();
#if FA_PQ_STEAL
        // the next item, dequeued now (its latency hides under this item's first QK^T) and
        // passed to the other waves through LDS behind the barrier below
        int nq = 0;
        if (tid == 0) nq = dequeue();
#endif
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db] = f32x16{};
        m = -INFINITY;
        l = 0.f;
        qk(kring, sa);
        if constexpr (TAIL) mask(0, sa);
        rowmax(sa, mx);
#if FA_PQ_STEAL
        if (tid == 0) *next_slot = nq;
        __syncthreads();  // K slot 0 is rewritten by step 0's DMA of K(2); next_slot written
        const int nitem = __builtin_amdgcn_readfirstlane(*next_slot);
#else
        __syncthreads();  // K slot 0 is rewritten by step 0's DMA of K(2)
        const int nitem = item + J < end_s ? item + J : -1;
#endif
        const bool has_next = nitem >= 0;
        const Item nxt = item_at(has_next ? nitem : item);
        st_t1 = PQ_NOW();
        st_pro += st_t1 - st_t0;
        {
            using C0 = std::integral_constant<int, 0>;
            using C1 = std::integral_constant<int, 1>;
            using STEADY = std::integral_constant<int, 1 | 4>;
            using NEXTLAST = std::integral_constant<int, 1 | 2>;
            using NEXTLASTK = std::integral_constant<int, 1 | 2 | 4>;
            using LAST = std::integral_constant<int, 0>;
            int t = 0;
            for (; t + 2 < ntiles; t += 2) {
                step(C0{}, STEADY{}, t, sa, sb, mx, has_next, nxt);
                step(C1{}, NEXTLASTK{}, t + 1, sb, sa, mx, has_next, nxt);
            }
            if (ntiles - t == 2) {
                step(C0{}, NEXTLAST{}, t, sa, sb, mx, has_next, nxt);
                step(C1{}, LAST{}, t + 1, sb, sa, mx, has_next, nxt);
            } else {
                step(C0{}, LAST{}, t, sa, sb, mx, has_next, nxt);
            }
        }
        st_t0 = PQ_NOW();
        st_loop += st_t0 - st_t1;
        ++st_n;

        // ---- epilogue: O^T[dv][q] -> 16-bit rows, permlane32-widened dwordx4 stores (T21)
        const int64_t q_row = cur.row0 + l32;
        const float inv = 1.f / pair_sum(l);
        if (q_row < a.Lq) {
            unsigned short* Oh = cur.o + q_row * D;
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int gp = 0; gp < 4; gp += 2) {
                    unsigned x0 = pack2<T>(o[db][4 * gp + 0] * inv, o[db][4 * gp + 1] * inv);
                    unsigned x1 = pack2<T>(o[db][4 * gp + 2] * inv, o[db][4 * gp + 3] * inv);
                    unsigned y0 = pack2<T>(o[db][4 * gp + 4] * inv, o[db][4 * gp + 5] * inv);
                    unsigned y1 = pack2<T>(o[db][4 * gp + 6] * inv, o[db][4 * gp + 7] * inv);
                    const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                    const u32x4 u = {s0[0], s1[0], s0[1], s1[1]};
                    *(u32x4*)(Oh + db * 32 + 8 * gp + 8 * hf) = u;
                }
        }
        st_epi += PQ_NOW() - st_t0;
        if (!has_next) break;
        item = nitem;
        cur = nxt;
    }
    }  // item >= 0

#if FA_PQ_STEAL
    // the last workgroup out zeroes this launch's queue set (every other workgroup has made
    // its last dequeue before counting itself out)
    if (tid == 0) {
        const unsigned done = __hip_atomic_fetch_add(qset + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done + 1 == gridDim.x) {
#pragma unroll
            for (int k = 0; k < 9; ++k) __hip_atomic_store(qset + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#endif
#if FA_STAMPS
    if (tid == 0 && blockIdx.x < 4096) {
        unsigned long long* r = g_fa_pq_stamps + blockIdx.x * 16;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        r[0] = st_entry;
        r[1] = PQ_NOW();
        r[2] = st_loop;
        r[3] = st_pro;
        r[4] = st_epi;
        r[5] = st_n;
        r[6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        r[7] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
        r[8] = st_rt;
        r[9] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

#ifndef FA_PQ_WAVES
#define FA_PQ_WAVES 4
#endif

int persist_rows_per_item() { return 32 * FA_PQ_WAVES; }

template <typename T, int D>
static hipError_t launch_pq_d(const FwdArgs& a, hipStream_t s) {
    constexpr int W = FA_PQ_WAVES;
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const int64_t nitems = (int64_t)a.nqt * a.BH;
    // resident workgroups: 8 / W per CU (the register budget), a multiple of 8; a grid larger
    // than the items only adds workgroups that find the queues empty
    const int64_t slots = (int64_t)(ncu & ~7 ? ncu & ~7 : 8) * (8 / W);
    const int64_t grid = nitems < slots ? ((nitems + 7) & ~7) : slots;
    constexpr int TILEB = bk_for(D) * D * 2;
    const int lds = 4 * TILEB + 16;
    if (a.Lk % bk_for(D))
        hipLaunchKernelGGL((fa_fwd_persist_kernel<T, D, true, W>), dim3((unsigned)grid), dim3(64 * W), lds, s, a);
    else
        hipLaunchKernelGGL((fa_fwd_persist_kernel<T, D, false, W>), dim3((unsigned)grid), dim3(64 * W), lds, s, a);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_pq_t(int d, const FwdArgs& a, hipStream_t s) {
    switch (d) {
        case 32: return launch_pq_d<T, 32>(a, s);
        case 64: return launch_pq_d<T, 64>(a, s);
        case 128: return launch_pq_d<T, 128>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fwd_persist(Elem t, int d, const FwdArgs& a0, hipStream_t s) {
    static std::atomic<unsigned> epoch{0};
    FwdArgs a = a0;
    a.nqt = (int)((a.Lq + persist_rows_per_item() - 1) / persist_rows_per_item());
    a.sched_epoch = epoch.fetch_add(1, std::memory_order_relaxed);
    if (t == Elem::BF16) return launch_pq_t<__bf16>(d, a, s);
    if (t == Elem::F16) return launch_pq_t<_Float16>(d, a, s);
    return hipErrorInvalidValue;
}

}  // namespace fa
