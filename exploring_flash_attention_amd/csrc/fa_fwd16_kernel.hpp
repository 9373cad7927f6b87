// fa_fwd16_kernel.hpp -- the d = 128 final-mode forward (FA-v1 fused / d-tiled, contiguous
// [B, H, L, d], Lk a multiple of 64) on v_mfma_f32_16x16x32 instead of 32x32x16.
//   <- flash_attention_kernel    flash_attention_v1/CUDA/flash_attention_v1.h:161
//   <- flash_attention_kernel (tiled-d) flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230
//
// Why a second MFMA shape: the d = 128 loop is bound by the power the MFMA array draws on
// random operands, not by its cycles, and on this chip the
// 16x16x32 bf16 MFMA delivers more FLOP/s than the 32x32x16 at equal cycles per FLOP on random
// data (MI355X_MICROARCH.md, DVFS give-back item 7; cdna_hip_programming.md section 5.4 rule
// 28: build both at the same output tile per wave, keep the faster by wall).  Same workgroup
// (4 waves x 32 query rows), same 64-key tiles, same LDS-DMA ring and swizzled tile image, same
// Q^T-in-registers and S^T = K . Q^T orientation as fa_fwd_kernel.hpp; what changes is the
// fragment geometry:
//   * S^T tile [16 keys][16 queries] per MFMA: lane (g = lane >> 4, n = lane & 15) holds query
//     16*qb + n (two query blocks per wave) and keys 16*kb + R0(g) + i, i = 0..3, where the K
//     rows of a key block are read in the order rho(m) = 8*((m>>2)&1) + 4*(m>>3) + (m&3) so
//     that R0(g) = 8*(g&1) + 4*(g>>1): the transposed V reads of the four lane groups then hit
//     disjoint LDS banks (a plain order puts groups 0 and 1 on the same banks).
//   * P^T B operand of P.V: lane (g, n), k = 8*g + j <-> key 32*kk + R0(g) + 16*(j>>2) + (j&3):
//     the S^T registers of key blocks 2kk and 2kk+1, packed as they are (no lane movement);
//     the V^T A operand holds the same keys from two ds_read_b64_tr_b16 of 4 keys each.
//   * a query's 64 scores of a tile sit in 4 lanes (n, n+16, n+32, n+48): the row max takes a
//     v_permlane16_swap and a v_permlane32_swap; the row sums are one 16x16x32 MFMA per P^T
//     fragment with A = ones (every output row = the column sums).
//   * O^T tiles [16 dv][16 queries], 8 x 2 per wave (64 accumulator registers, as before);
//     the epilogue pairs dv blocks with v_permlane16_swap into 16-byte row stores.
// The steady step is pinned like fa_fwd_kernel.hpp's step_pinned: phase A = 16 slots of two
// QK^T(t+1) MFMAs (one K fragment, both query blocks) with the exponentials of tile t, the
// first key step's packing and the 8 DMA pieces; phase B = 16 slots of two P.V(t) MFMAs (one
// V^T operand, both query blocks) and 2 row-sum slots, with the rest of the exponentials and
// packing and the row max of tile t+1.
#pragma once
#include "fa_device.hpp"

namespace fa {

template <typename X> struct TypeTag { using type = X; };



// MODE: kFinal (O), kPartial (normalised partial O + lse in row layout, fa_combine.hip reads
// them) or kFused (partials in fragment order, combined by the last workgroup of each query
// tile), as fa_fwd_kernel.hpp; every split a multiple of 64 keys and non-empty.
// STR: q, k / v and o are [B, H, L, d] views addressed through their {batch, head, row}
// element strides (FwdArgs q_stride / k_stride / o_stride; d contiguous, rows 16-byte aligned),
// e.g. [B, L, H, d] tensors transposed, or the q row ranges of the multi-GPU partial path
// (fa_fwd_partial_ex).  Only the global addressing changes -- the DMA source offsets and tile
// descriptors take the row stride -- so a view gives the contiguous launch's bits.  (Partial
// mode writes its own row layout; o_stride is not used there.)
struct NoHook {
    __device__ void operator()() const {}
};

// One work item (query tile, split, b*h) of the kernel; `at_loop_end` runs once, right after
// the KV loop's last barrier (round 4's dynamic-claim experiment claimed its next item there;
// measured and removed).
template <typename T, typename PT, int D, int MODE, bool STR = false, typename Hook = NoHook>
__device__ __forceinline__ void fa_fwd16_item(const FwdArgs& a, const int w, const Hook& at_loop_end = Hook{}) {
    using M = Mma<T>;
    using v8 = typename M::v8;
    static_assert(D == 128, "16x16x32 kernel: d = 128");
    constexpr int ROWB = D * 2;        // bytes per LDS row
    constexpr int kBK = 64;            // keys per KV tile
    constexpr int TILEB = kBK * ROWB;  // bytes of one K (or V) tile image
    constexpr int NKS = D / 32;        // QK^T k-steps (32 dims each)
    constexpr int NKB = kBK / 16;      // 16-key blocks per tile
    constexpr int NQB = 2;             // 16-query blocks per wave
    constexpr int NDB = D / 16;        // 16-column blocks of O
    constexpr int NKK = kBK / 32;      // P.V k-steps (32 keys each)
    constexpr float kThr = 4.f;        // deferred rescale threshold (log2 units), as fa_fwd_kernel
    // Schedule constants, measured (A/B in one process): K fragments read
    // KA slots ahead and V^T operands VA MFMA pairs ahead (2 / 4 and 1 / 3: within 0.5 %), EXPA of
    // tile t's 32 exponentials in phase A (20 -> 28: +1 % at C3; 32: equal)
    constexpr int KA = 3, VA = 2;  // LDS reads in flight: K fragments, V^T operands
    constexpr int EXPA = 28;       // exponentials in phase A (the rest: phase B, 2 per slot)
    static_assert(EXPA >= 19 && EXPA <= 32, "key step 0 packs (phase A slots 6..13) follow their exponentials");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const kring = smem;              // K ring: 2 slots
    char* const vring = smem + 2 * TILEB;  // V ring: 2 slots

    int qt, split;
    int64_t bh;
    decode_item(a, w, qt, split, bh);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n16 = lane & 15, g = lane >> 4;
    // (FA_STAMPS diagnostic builds only, fa_fwd_kernel.hpp; slots as scripts/stamps.py reads them)
    FA_STAMP_V(8, __builtin_amdgcn_s_memrealtime());
    FA_STAMP(0);
    FA_STAMP_V(6, __builtin_amdgcn_s_getreg(4 | (31 << 11)));
    FA_STAMP_V(7, __builtin_amdgcn_s_getreg(20 | (31 << 11)));
    const int64_t kv_begin = (int64_t)split * a.kv_per_split;
    const int64_t kv_end = kv_begin + a.kv_per_split < a.Lk ? kv_begin + a.kv_per_split : a.Lk;
    const int ntiles = (int)((kv_end - kv_begin) / kBK);

    const int64_t q_tile0 = (int64_t)qt * kBQ;
    // row strides (bytes) and head bases (elements); contiguous launches fold them to constants
    const int qrb = STR ? (int)(a.q_stride[2] * 2) : ROWB;
    const int krb = STR ? (int)(a.k_stride[2] * 2) : ROWB;
    const int64_t hb = STR ? bh / a.H : 0, hh = STR ? bh - hb * a.H : 0;
    const int64_t q_head = STR ? hb * a.q_stride[0] + hh * a.q_stride[1] : bh * a.Lq * D;
    const int64_t k_head = STR ? hb * a.k_stride[0] + hh * a.k_stride[1] : bh * a.Lk * D;
    const int64_t o_head = STR ? hb * a.o_stride[0] + hh * a.o_stride[1] : bh * a.Lq * D;
    const int64_t orow = STR ? a.o_stride[2] : D;
    const unsigned short* Qh = (const unsigned short*)a.q + q_head + q_tile0 * (qrb / 2);
    const int64_t q_rows = a.Lq - q_tile0 < kBQ ? a.Lq - q_tile0 : kBQ;
    const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Qh, (q_rows - 1) * qrb + ROWB);
    const unsigned short* const kbase = (const unsigned short*)a.k + k_head + kv_begin * (krb / 2);
    const unsigned short* const vbase = (const unsigned short*)a.v + k_head + kv_begin * (krb / 2);
    // one K / V tile in global memory: its stride and the bytes its descriptor covers
    const int64_t tstride = STR ? (int64_t)kBK * krb : (int64_t)TILEB;
    const int tbytes = STR ? (kBK - 1) * krb + ROWB : TILEB;

    // The 32 dims of a QK^T k-step are split over the lane groups g as 8-dim chunk pg(g) =
    // (0, 3, 1, 2)[g] (A and B agree, so the sum is the same): ds_read_b128 serves a wave in the
    // lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH.md, LDS), and
    // with the plain chunk g two lanes of a group hit one bank (2-way, 8 instead of 4 cycles).
    const int pg = (0x2130 >> (4 * g)) & 3;
    // Q^T fragments (B operand of QK^T): lane (g, n) holds Q[32*wid + 16*qb + n][32*ks + 8*pg ..+7]
    v8 qf[NQB][NKS];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[qb][ks] = __builtin_bit_cast(
                v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, (wid * 32 + 16 * qb + n16) * qrb + ks * 64 + pg * 16, 0, 0));

    // LDS-DMA of a tile: 16 pieces of 1 KiB, 4 per wave, the swizzled image (lds_off) produced
    // by giving each lane the SOURCE chunk that lands at its destination (fa_fwd_kernel.hpp)
    constexpr int DPW = TILEB / 1024 / kWaves;
    int dma_src[DPW];
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
        const int b = (wid * DPW + i) * 1024 + lane * 16;
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        dma_src[i] = row * krb + ch * 16;
    }
    auto dma_tile = [&](const unsigned short* base, char* slot, int t) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc32((const char*)base + t * tstride, t < ntiles ? tbytes : 0);
#pragma unroll
        for (int i = 0; i < DPW; ++i) dma16(rs, slot + (wid * DPW + i) * 1024, dma_src[i], 0);
    };

    // K fragment (A operand of QK^T) of key block kb, k-step ks: lane (g, n) reads row
    // 16*kb + rho(n), 16-byte chunk 4*ks + pg; one base address + immediates
    const int rho = 8 * ((n16 >> 2) & 1) + 4 * (n16 >> 3) + (n16 & 3);
    const unsigned kaddr = (unsigned)(size_t)kring + (rho >> 3) * (8 * ROWB) + 64 * (rho & 7) + 16 * (pg ^ ((rho >> 2) & 3));
    // V^T operand (A of P.V) of key step kk, column block db: two transposed reads of the 4 keys
    // at rows 32*kk + R0(g) + (n >> 2) (+16), columns 16*db + 4*(n & 3); the swizzle makes odd
    // column blocks a second base address
    const int r0 = 8 * (g & 1) + 4 * (g >> 1) + (n16 >> 2);
    const int sw = (r0 >> 2) & 3, c0 = (n16 >> 1) & 1;
    const unsigned vrow = (unsigned)(size_t)vring + (r0 >> 3) * (8 * ROWB) + 64 * (r0 & 7) + 8 * (n16 & 1);
    const unsigned vb_e = vrow + 16 * (c0 ^ sw);
    const unsigned vb_o = vrow + 16 * ((2 + c0) ^ sw);

    f32x4 o[NDB][NQB];
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) o[db][qb] = f32x4{};
    f32x4 rs[NQB] = {f32x4{}, f32x4{}};  // row sums (every register the same value)
    float m[NQB];
    v8 ones;
    {
        constexpr unsigned kOne = std::is_same_v<T, __bf16> ? 0x3F80u : 0x3C00u;
        ones = __builtin_bit_cast(v8, u32x4{kOne | (kOne << 16), kOne | (kOne << 16), kOne | (kOne << 16),
                                            kOne | (kOne << 16)});
    }
    const float c = a.scale_log2;

    // (inline asm in nested generic lambdas must not capture: every operand is a parameter)
    auto kread_ = [](auto r_c, auto slot_c, u32x4 (&kf)[KA + 1], unsigned ka) {
        constexpr int R = decltype(r_c)::value, KS = R / NKB, KB = R % NKB, SL = decltype(slot_c)::value;
        constexpr int OFF = SL * TILEB + KB * 16 * ROWB + KS * 512;
        static_assert(OFF < 65536, "ds offset field is 16 bits");
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[R % (KA + 1)]) : "v"(ka), "i"(OFF) : "memory");
    };
    auto vread_ = [](auto p_c, auto slot_c, u32x2 (&vf)[VA + 1][2], unsigned ve, unsigned vo) {
        constexpr int PP = decltype(p_c)::value, KK = PP / NDB, DB = PP % NDB, SL = decltype(slot_c)::value;
        constexpr int OFF = SL * TILEB + KK * 32 * ROWB + 512 * (DB >> 1);
        static_assert(OFF + 16 * ROWB < 65536, "ds offset field is 16 bits");
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
    // closes an MFMA slot: hipcc keeps the slot's fillers with its MFMAs (the compiler-scheduled
    // step measured -1.5 ... -2.5 %)
    auto fence = [] { __builtin_amdgcn_sched_barrier(0); };

    // S^T(t) of one tile from K slot SL: 16 K fragments, each feeding both query blocks
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
    // row max (log2 units) of both query blocks of a tile: four v_maximum3 chains of 8 scores
    // (chain ch: query block ch / 2, key blocks 2 * (ch & 1) and 2 * (ch & 1) + 1)
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

    // One step for tile t (raw scores in sc, row max in mx): rescale decision; DMA K(t+2) and
    // V(t+1) into the slots freed by the previous step's barrier; QK^T(t+1) -> sn beside the
    // exponentials of sc; pack P; P.V(t) and the row sums; row max of sn; barrier.
    auto step = [&](auto par_c, auto flags_c, int t, f32x4 (&sc)[NKB][NQB], f32x4 (&sn)[NKB][NQB],
                    float (&mx)[NQB]) {
        constexpr int P = decltype(par_c)::value;
        constexpr int F = decltype(flags_c)::value;
        constexpr bool MORE = F & 1;  // tile t+1 exists
        constexpr bool DMAK = F & 4;  // K(t+2) is fetched now (zeros past the end)
        using SLN = std::integral_constant<int, 1 - P>;
        using SLC = std::integral_constant<int, P>;
        if (__builtin_amdgcn_ballot_w64(mx[0] > m[0] + kThr || mx[1] > m[1] + kThr)) {
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
        const __amdgpu_buffer_rsrc_t krs =
            make_rsrc32((const char*)kbase + (t + 2) * tstride, DMAK && t + 2 < ntiles ? tbytes : 0);
        const __amdgpu_buffer_rsrc_t vrs = make_rsrc32((const char*)vbase + (t + 1) * tstride, tbytes);
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

        // ---- phase A: QK^T(t+1) || exponentials of t
        // (the VALU-dense phase at priority 1, P.V at 0: C3 +0.4 %, L = 2048 +0.7 %, C4 0; the
        // reverse +0.3 / +0.6 / 0; half the workgroups at a static priority 1: 0)
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
            if constexpr (S % 2 == 1) dma(std::integral_constant<int, S / 2>{});
            if constexpr (MORE) fence();
        });

        // ---- phase B: P.V(t) || exponentials of t (rest), row max of t+1
        __builtin_amdgcn_s_setprio(0);
        // slot J: key step kk = J / 9; J % 9 < 8: P.V of column block J % 9, J % 9 == 8: row sums
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
                    o[JJ][qb] = M::mma16(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbu[KK][qb]), o[JJ][qb]);
            } else {
#pragma unroll
                for (int qb = 0; qb < NQB; ++qb) rs[qb] = M::mma16(ones, __builtin_bit_cast(v8, pbu[KK][qb]), rs[qb]);
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
        __syncthreads();  // hipcc drains the DMA (vmcnt(0)) here: K(t+2), V(t+1) landed
    };

    // prologue: K(0), V(0), K(1) -> LDS; S(0) = QK^T(0)
    dma_tile(kbase, kring, 0);
    dma_tile(vbase, vring, 0);
    if (ntiles > 1) dma_tile(kbase, kring + TILEB, 1);
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[qb][ks]));
    // the first QK^T needs Q (waited above) and K(0) only: V(0) and K(1) -- the DPW pieces each
    // issued after it; no K(1) for a single tile -- stay in flight; the barrier after the row max
    // drains them (A/B round 4, profiles/r04/ab_early_qk.txt: C3 +0.2 / +0.6 %, C4 +0.1 %,
    // L = 2048 +0.3 %, bitwise equal)
    static_assert(2 * DPW < 16, "vmcnt range");
    if (ntiles > 1)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * DPW) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(DPW) : "memory");
    FA_STAMP(1);
    f32x4 sa[NKB][NQB], sb[NKB][NQB];
    float mx[NQB];
    qk_all(std::integral_constant<int, 0>{}, sa);
    rowmax_all(sa, mx);
    m[0] = mx[0];  // the reference max starts at tile 0's row max (no step-0 rescale)
    m[1] = mx[1];
    __syncthreads();  // K slot 0 is rewritten by step 0's DMA of K(2)
    FA_STAMP(2);

    {
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using STEADY = std::integral_constant<int, 1 | 4>;  // MORE | DMAK
        using NEXTLAST = std::integral_constant<int, 1>;
        using LAST = std::integral_constant<int, 0>;
        int t = 0;
        for (; t + 2 < ntiles; t += 2) {
            step(C0{}, STEADY{}, t, sa, sb, mx);
            step(C1{}, STEADY{}, t + 1, sb, sa, mx);
        }
        if (ntiles - t == 2) {
            step(C0{}, NEXTLAST{}, t, sa, sb, mx);
            step(C1{}, LAST{}, t + 1, sb, sa, mx);
        } else {
            step(C0{}, LAST{}, t, sa, sb, mx);
        }
    }

    FA_STAMP(3);
    at_loop_end();
    // ---- epilogue: lane (g, n) holds O^T[16*db + 4*g + i][query 16*qb + n].  A 16-bit row is
    // stored 16 bytes per lane: dv blocks 2e and 2e+1 are paired by one v_permlane16_swap per
    // dword, lane group g then holds columns 32*e + 16*(g&1) + 8*(g>>1) .. +7.
    auto store_row16 = [&](auto ph_c, unsigned short* Oh, const f32x4 (&v)[NDB], float scale) {
        using PH = typename decltype(ph_c)::type;
#pragma unroll
        for (int e = 0; e < NDB / 2; ++e) {
            const unsigned x0 = pack2<PH>(v[2 * e][0] * scale, v[2 * e][1] * scale);
            const unsigned x1 = pack2<PH>(v[2 * e][2] * scale, v[2 * e][3] * scale);
            const unsigned y0 = pack2<PH>(v[2 * e + 1][0] * scale, v[2 * e + 1][1] * scale);
            const unsigned y1 = pack2<PH>(v[2 * e + 1][2] * scale, v[2 * e + 1][3] * scale);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
            const u32x4 u = {s0[0], s1[0], s0[1], s1[1]};
            *(u32x4*)(Oh + 32 * e + 16 * (g & 1) + 8 * (g >> 1)) = u;
        }
    };
    f32x4 ov[NQB][NDB];  // O by query block
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
        for (int db = 0; db < NDB; ++db) ov[qb][db] = o[db][qb];
    float lsum[NQB], inv[NQB];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
        lsum[qb] = rs[qb][0];
        inv[qb] = 1.f / lsum[qb];
    }
    constexpr bool SCALED = std::is_same_v<PT, f16s_t>;   // fp16 partials, per-row 2^-e
    using PH = std::conditional_t<SCALED, _Float16, T>;   // 16-bit partial element type
    float esc[NQB] = {0.f, 0.f};
    if constexpr (MODE != kFinal && SCALED) {
        // the row's largest |O / l| just below 1 after the exact scale 2^-e
        float mxa[NQB];
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            float mx = 0.f;
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmax_nc(mx, __builtin_fabsf(ov[qb][db][i]));
            mxa[qb] = mx;
        }
        quad_max2(mxa[0], mxa[1], mxa[0], mxa[1]);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            const int e = __builtin_amdgcn_frexp_expf(mxa[qb] * inv[qb]);
            esc[qb] = (float)e;
            inv[qb] = __builtin_amdgcn_ldexpf(inv[qb], -e);
        }
    }
    if constexpr (MODE == kFinal) {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            const int64_t q_row = q_tile0 + wid * 32 + 16 * qb + n16;
            if (q_row < a.Lq) store_row16(TypeTag<T>{}, (unsigned short*)a.o + o_head + q_row * orow, ov[qb], inv[qb]);
        }
#if FA_STAMPS
        FA_STAMP(4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        FA_STAMP(5);
        FA_STAMP_V(9, __builtin_amdgcn_s_memrealtime());
#endif
    } else if constexpr (MODE == kPartial) {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            const int64_t q_row = q_tile0 + wid * 32 + 16 * qb + n16;
            if (q_row >= a.Lq) continue;
            const int64_t chunk = q_row / a.chunk_rows, r_in = q_row % a.chunk_rows;
            const int64_t row_lin = chunk * a.BH * a.chunk_rows + bh * a.chunk_rows + r_in;
            PT* const Op = (PT*)a.o + split * a.split_stride + row_lin * D;
            if constexpr (sizeof(PT) == 4) {
#pragma unroll
                for (int db = 0; db < NDB; ++db) *(f32x4*)((float*)Op + 16 * db + 4 * g) = ov[qb][db] * inv[qb];
            } else {
                store_row16(TypeTag<PH>{}, (unsigned short*)Op, ov[qb], inv[qb]);
            }
            // lse in log2 units: m + log2(l)  (v_log_f32 is log2)
            const float lse = m[qb] + __builtin_amdgcn_logf(lsum[qb]);
            if (g == 0) {
                if constexpr (SCALED)
                    *(float2*)(a.lse + 2 * (split * a.BH * a.Lq + row_lin)) = make_float2(lse, esc[qb]);
                else
                    a.lse[split * a.BH * a.Lq + row_lin] = lse;
            }
        }
    } else {
        // Split-KV partials combined on chip (fa_fwd_kernel.hpp's workspace layout): every
        // workgroup but the last one at its query tile stores its normalised partial O (PT) and
        // lse in FRAGMENT order -- lane-linear pieces, coalesced for the stores and the
        // combine's loads -- with sc1 and drains them (vmcnt(0), a barrier); the last one sums
        // all partials, its own from the registers, rounded exactly as its store would round
        // them.  Who is last: one agent-scope atomic per workgroup on the tile's counter, in
        // one of two orders (FwdArgs::arrive_first, chosen by the launcher):
        //  * stores first, then the ARRIVAL count (low 16 bits): the last arriver has stored its
        //    partial too but never reads it back;
        //  * arrive_first: the ARRIVAL count first; all but the last then store and count their
        //    COMPLETION (high 16 bits), and the last waits for the others' completions -- they
        //    arrived, so they are running and only their stores are outstanding: the wait cannot
        //    deadlock -- and its partial never leaves the registers.  One more memory round trip
        //    on the tile's critical path when its workgroups finish together, so the launcher
        //    takes it only for long key blocks (fa_capi.cpp).
        constexpr int SC1 = 16;                // cache-policy bit: sc1
        constexpr int NF = NDB * NQB;          // fragments (4 values) per lane
        constexpr int BLK = kBQ * D;           // partial elements per (split, tile) block
        const int64_t grp = bh * a.nqt + qt;
        auto blk_of = [&](int sp) { return (int64_t)sp * a.BH * a.nqt + grp; };
        // (the own block's ranges are empty in the combine: its loads return 0 and move no bytes)
        auto o_rsrc = [&](int sp) {
            return make_rsrc((const PT*)a.o + blk_of(sp) * BLK, sp == split ? 0 : (int64_t)BLK * sizeof(PT));
        };
        auto l_rsrc = [&](int sp) { return make_rsrc(a.lse + blk_of(sp) * kBQ, sp == split ? 0 : (int64_t)kBQ * 4); };
        auto e_rsrc = [&](int sp) { return make_rsrc(a.esc + blk_of(sp) * kBQ, sp == split ? 0 : (int64_t)kBQ * 4); };
        auto frag_off = [&](int f) { return (((wid * NF + f) * 64 + lane) * 4) * (int)sizeof(PT); };
        auto lse_off = [&](int qb) { return (wid * 32 + 16 * qb + n16) * 4; };
        int* const last_flag = (int*)smem;  // LDS is free: the KV loop ended with a barrier
        const bool af = a.arrive_first != 0;
        auto arrive = [&]() {
            if (tid == 0) {
                const unsigned old = __hip_atomic_fetch_add(a.counters + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *last_flag = (old & 0xffffu) + 1 == (unsigned)a.nsplit;
            }
            __syncthreads();
            return __builtin_amdgcn_readfirstlane(*last_flag);
        };
        int last = af ? arrive() : 0;
#if FA_STAMPS
        // (diagnostic builds: 10 the hand-off verdict, 11 the combine's start, 12 = 1 for the
        // tile's last workgroup; 4 / 5 / 9 as in kFinal, for the last one after its O)
        if (af) FA_STAMP(10);
        FA_STAMP_V(12, last);
#endif
        // this block's partial as stored: 16-bit pairs (or fp32) per fragment, lse of the row
        using Frag = std::conditional_t<sizeof(PT) == 4, f32x4, u32x2>;
        Frag mine[NQB][NDB];
        float lse_mine[NQB];
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
#pragma unroll
            for (int db = 0; db < NDB; ++db) {
                const f32x4 x = ov[qb][db] * inv[qb];
                if constexpr (sizeof(PT) == 4)
                    mine[qb][db] = x;
                else
                    mine[qb][db] = u32x2{pack2<PH>(x[0], x[1]), pack2<PH>(x[2], x[3])};
            }
            // the row's lse as lane group 0 stores it
            const float lse = m[qb] + __builtin_amdgcn_logf(lsum[qb]);
            lse_mine[qb] = __int_as_float(__builtin_amdgcn_ds_bpermute(n16 * 4, __float_as_int(lse)));
        }
        if (!last) {
            const __amdgpu_buffer_rsrc_t ors = make_rsrc((const PT*)a.o + blk_of(split) * BLK, (int64_t)BLK * sizeof(PT));
            const __amdgpu_buffer_rsrc_t lrs = make_rsrc(a.lse + blk_of(split) * kBQ, (int64_t)kBQ * 4);
            const __amdgpu_buffer_rsrc_t ers = make_rsrc(a.esc + blk_of(split) * kBQ, (int64_t)kBQ * 4);
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) {
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    if constexpr (sizeof(PT) == 4)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, mine[qb][db]), ors,
                                                               frag_off(db * NQB + qb), 0, SC1);
                    else
                        __builtin_amdgcn_raw_buffer_store_b64(mine[qb][db], ors, frag_off(db * NQB + qb), 0, SC1);
                }
                if (g == 0) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lse_mine[qb]), lrs, lse_off(qb), 0, SC1);
                    if constexpr (SCALED)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(esc[qb]), ers, lse_off(qb), 0, SC1);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (af) {
                if (tid == 0) __hip_atomic_fetch_add(a.counters + grp, 0x10000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if FA_STAMPS
                FA_STAMP(4);
                FA_STAMP(5);
                FA_STAMP_V(9, __builtin_amdgcn_s_memrealtime());
#endif
                return;
            }
            last = arrive();
#if FA_STAMPS
            FA_STAMP(10);
            FA_STAMP_V(12, last);
            if (!last) {
                FA_STAMP(4);
                FA_STAMP(5);
                FA_STAMP_V(9, __builtin_amdgcn_s_memrealtime());
            }
#endif
            if (!last) return;
        }
        if (tid == 0) {
            if (af) {
                const unsigned want = (unsigned)(a.nsplit - 1) << 16;
                // (bounded: the others have arrived, so their completions come within
                // microseconds; a counter that was not zero at the launch -- a caller's broken
                // FA_V2_COUNTERS_ZERO promise -- ends in a wrong O after ~2^22 polls, not a hang)
                for (int it = 0; it < (1 << 22) &&
                                 (__hip_atomic_load(a.counters + grp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                                  0xffff0000u) != want;
                     ++it)
                    __builtin_amdgcn_s_sleep(1);
            }
            a.counters[grp] = 0;  // leave the counter zero for the next launch
        }
        __syncthreads();
        FA_STAMP(11);

        // Sum in split order 0, 1, ... whatever workgroup came last, so that O is bitwise
        // repeatable.
        const int ns = a.nsplit;
        auto widen = [&](const Frag& u) -> f32x4 {
            if constexpr (sizeof(PT) == 4) {
                return u;
            } else {
                // (16-bit halves by shifts: hipcc miscompiles a bit_cast of u[1] to a 2 x bf16 vector
                // into a second copy of u[0] and narrows the load to one dword)
                f32x4 r;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const unsigned wd = u[j >> 1];
                    r[j] = (float)__builtin_bit_cast(PH, (unsigned short)((j & 1) ? (wd >> 16) : (wd & 0xffff)));
                }
                return r;
            }
        };
        auto load_frag = [&](int sp, int f) -> Frag {
            if constexpr (sizeof(PT) == 4)
                return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(o_rsrc(sp), frag_off(f), 0, SC1));
            else
                return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(o_rsrc(sp), frag_off(f), 0, SC1));
        };
        // U key blocks' loads in flight at a time (one at a time, the combine is a chain of
        // memory latencies: the chained walk's C4 run went -10 % -> +9.5 % with this); an index
        // past the last block re-reads the last one, harmless to the maxima and given weight 0 in
        // the sums -- the same sums in the same order (acc never holds -0)
        constexpr int U = sizeof(PT) == 4 ? 2 : 4;
        auto clampsp = [&](int sp) { return sp < ns ? sp : ns - 1; };
        // (at most U blocks -- the library's splits at d = 128 -- everything is loaded in one
        // batch per query block.  Both query blocks in one batch (128 more VGPRs) spilled the
        // loaded partials and ran B1 H2 L4096 27.7 -> 31.4 us: profiles/r06/ab_*_combine_batch2)
        auto load_batch = [&](int qb, int sp0, float (&lv)[U], float (&ev)[U], Frag (&pv)[U][NDB]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sp = clampsp(sp0 + u);
                lv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(l_rsrc(sp), lse_off(qb), 0, SC1));
                if constexpr (SCALED)
                    ev[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(e_rsrc(sp), lse_off(qb), 0, SC1));
#pragma unroll
                for (int db = 0; db < NDB; ++db) pv[u][db] = load_frag(sp, db * NQB + qb);
                if (sp == split) {
                    lv[u] = lse_mine[qb];
                    ev[u] = esc[qb];
#pragma unroll
                    for (int db = 0; db < NDB; ++db) pv[u][db] = mine[qb][db];
                }
            }
        };
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            float Mx = -INFINITY, E = -1000.f;
            f32x4 acc[NDB];
#pragma unroll
            for (int db = 0; db < NDB; ++db) acc[db] = f32x4{};
            float wsum = 0.f;
            auto accumulate = [&](int sp0, const float (&lv)[U], const float (&ev)[U], const Frag (&pv)[U][NDB]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float wgt = sp0 + u < ns ? __builtin_amdgcn_exp2f(lv[u] - Mx) : 0.f;
                    float wv = wgt;
                    if constexpr (SCALED) wv = __builtin_amdgcn_ldexpf(wgt, (int)(ev[u] - E));
#pragma unroll
                    for (int db = 0; db < NDB; ++db) acc[db] += wv * widen(pv[u][db]);
                    wsum += wgt;
                }
            };
            if (ns <= U) {
                float lv[U], ev[U];
                Frag pv[U][NDB];
                load_batch(qb, 0, lv, ev, pv);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    Mx = fmaxf(Mx, lv[u]);
                    if constexpr (SCALED) E = fmaxf(E, ev[u]);
                }
                accumulate(0, lv, ev, pv);
            } else {
                for (int sp0 = 0; sp0 < ns; sp0 += U) {
                    float lv[U], ev[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int sp = clampsp(sp0 + u);
                        lv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(l_rsrc(sp), lse_off(qb), 0, SC1));
                        if constexpr (SCALED)
                            ev[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(e_rsrc(sp), lse_off(qb), 0, SC1));
                        if (sp == split) {
                            lv[u] = lse_mine[qb];
                            ev[u] = esc[qb];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        Mx = fmaxf(Mx, lv[u]);
                        if constexpr (SCALED) E = fmaxf(E, ev[u]);
                    }
                }
                for (int sp0 = 0; sp0 < ns; sp0 += U) {
                    float lv[U], ev[U];
                    Frag pv[U][NDB];
                    load_batch(qb, sp0, lv, ev, pv);
                    accumulate(sp0, lv, ev, pv);
                }
            }
            float inv_w = 1.f / wsum;
            if constexpr (SCALED) {
#pragma unroll
                for (int db = 0; db < NDB; ++db)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[db][i] = __builtin_amdgcn_ldexpf(acc[db][i] * inv_w, (int)E);
                inv_w = 1.f;
            }
            const int64_t q_row = q_tile0 + wid * 32 + 16 * qb + n16;
            if (q_row < a.Lq) store_row16(TypeTag<T>{}, (unsigned short*)a.o_final + o_head + q_row * orow, acc, inv_w);
        }
#if FA_STAMPS
        FA_STAMP(4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        FA_STAMP(5);
        FA_STAMP_V(9, __builtin_amdgcn_s_memrealtime());
#endif
    }
}

template <typename T, typename PT, int D, int MODE, bool STR = false>
__global__ __launch_bounds__(kThreads, 2) void fa_fwd16_kernel(FwdArgs a) {
    fa_fwd16_item<T, PT, D, MODE, STR>(a, xcd_remap(blockIdx.x, gridDim.x));
}

}  // namespace fa
