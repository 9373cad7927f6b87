// fa_fwd_kernel.hpp -- flash-attention forward kernel for MI355X (gfx950 / CDNA4), included by
// fa_fwd.hip (contiguous [B,H,L,d] launches) and fa_fwd_strided.hip (strided launches).
//
// One kernel template serves the three reference kernel families:
//   final mode   (MODE=kFinal): FA-v1 fused / d-tiled forward
//                 <- flash_attention_kernel    flash_attention_v1/CUDA/flash_attention_v1.h:161
//                 <- flash_attention_kernel_opt1 flash_attention_v1/CUDA/flash_attention_v1_opt1.h:264
//                 <- flash_attention_kernel (tiled-d) flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230
//   partial mode (MODE=kPartial): FA-v2 split-KV partial kernel (+ fa_combine.hip)
//                 <- partial_attention_kernel  flash_attention_v2/CUDA/flash_attention_v2.h:243
//   fused split  (MODE=kFused): the same partials, combined by the last workgroup of each
//                 query tile to finish (the reduction_kernel's maths,
//                 flash_attention_v2/CUDA/flash_attention_v2.h:356, without its HBM pass)
//
// Online-softmax recurrence per KV tile (flash_attention_v1/numpy_gpu_like_opt2.py:135-195):
//   S = Q K^T * scale; m_new = max(m, rowmax S); alpha = e^(m - m_new);
//   P = e^(S - m_new); l = l*alpha + rowsum P; O = O*alpha + P V;  finally O / l.
// Here the exponentials are base 2 with log2(e)/sqrt(d) folded into one FMA.
//
// Mapping to CDNA4 (see DESIGN.md for the derivation):
//   * workgroup = 4 waves x 32 query rows = 128 rows of one (b,h); KV tiles of 64 keys.
//   * S^T = K . Q^T on v_mfma_f32_32x32x16 (A = K rows from LDS via ds_read_b128,
//     B = Q^T fragments held in VGPRs for the whole KV loop): the accumulator puts one
//     query row per lane (lanes l and l+32 share a row), so row max / row sum are
//     in-lane plus one v_permlane32_swap.
//   * O^T = V^T . P^T: the S accumulator, exponentiated and packed to 16-bit, is already
//     the B operand (no LDS round trip); V^T fragments come from ds_read_b64_tr_b16
//     transposed LDS reads.  O_acc stays in VGPRs/AGPRs for the whole KV loop.
//   * K and V tiles go HBM -> LDS by LDS-DMA (buffer_load ... lds) into a double-buffered,
//     XOR-swizzled LDS image that is bank-conflict-free for both the row reads and the
//     transposed reads.
//   * blockIdx is remapped so that all query tiles of one (b,h) land on one XCD and
//     share that head's K/V in the XCD's L2.
#pragma once
#include <type_traits>

#include "fa_device.hpp"

// Per-head-dim tuning, fixed at the measured-best settings (A/B in one process, DESIGN.md
// section 5; the experiment builds that produced them are in git history, not in the product):
//  * row sums on v_mfma_f32_16x16x32 (A = a 0/1 pattern, B = each packed P^T fragment as it
//    is, so one MFMA per 16-key fragment sums both key halves of 16 query rows into 4
//    accumulator registers; lane l ends up with the sum of query row (l & 15) + 16 * (l >> 5))
//    at every d; at d = 32 only in the final no-tail contiguous kernel (the other d = 32
//    instantiations would spill inside the loop under their register bound).  C2 +3.5 %,
//    C3 +1.2 %, d = 64 +1.7 %, the C5 partial kernel +1.4 %; sums the same 16-bit-rounded P
//    the numerator uses;
//  * a scheduling fence between the P.V MFMAs and the next tile's row max at d = 256 (+1.7 %;
//    0 or negative elsewhere);
//  * the DMA's M0 destinations from an SGPR wave id at d = 32 (+3 %; d = 128 -1.7 %);
//  * the no-tail step specialisation at d = 32 / 128 / 256 (d = 64: -7 %);
//  * packed fp32 exponent arithmetic at d = 32 (C2 +2.4 %; d = 64 -4 %), its FMAs of a 32-key
//    block issued ahead of the block's exponentials (+2 %).
constexpr int kRowmaxFenceMask = 0x8;  // d = 256
constexpr int kUniformWidMask = 0x1;   // d = 32
constexpr int kNoTailMask = 0xD;       // d = 32, 128, 256
constexpr int kPackedMaxD = 32;
// (the row-sum MFMA table, rs16_on, and the launch bounds, kernel_wps, live in
// fa_internal.hpp: the host's split planner sizes its grids with the same occupancy)
static_assert(fa::kernel_wps(32, 0, false, false) == 4 && fa::kernel_wps(64, 2, true, false) == 3 &&
                  fa::kernel_wps(128, 0, false, false) == 2 && fa::kernel_wps(256, 0, false, false) == 1,
              "occupancy table");

// FA_STAMPS (diagnostic builds only): wave 0 of every workgroup writes s_memtime stamps at
// the phase boundaries into g_fa_stamps (never into an output), read back through
// fa_debug_stamps() by scripts/stamps.py.  Slots per workgroup: 0 entry, 1 Q/K0/V0/K1
// landed, 2 loop start, 3 loop end, 4 stores issued, 5 stores retired, 6 hw_id, 7 xcc_id,
// 8 / 9 s_memrealtime (100 MHz, one time base for all CUs) at entry / after the stores retired.
#ifndef FA_STAMPS
#define FA_STAMPS 0
#endif
#if FA_STAMPS && defined(FA_FWD_MAIN_TU)
// (only the contiguous launches of fa_fwd.hip are stamped: a device symbol shared between
// translation units would need relocatable device code)
#define FA_MAX_STAMP_WG 65536
__device__ unsigned long long g_fa_stamps[FA_MAX_STAMP_WG * 16];
extern "C" int fa_debug_stamps(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fa_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#define FA_STAMP_V(i, v)                                                                       \
    do {                                                                                       \
        if (tid == 0 && blockIdx.x < FA_MAX_STAMP_WG)                                          \
            __hip_atomic_store(&g_fa_stamps[blockIdx.x * 16 + (i)], (unsigned long long)(v),     \
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                     \
    } while (0)
#define FA_STAMP(i) FA_STAMP_V(i, __builtin_amdgcn_s_memtime())
#else
#define FA_STAMP_V(i, v) \
    do {                 \
    } while (0)
#define FA_STAMP(i) FA_STAMP_V(i, 0)
#endif

namespace fa {

// TAIL: Lk is not a multiple of the KV tile, so the last tile of a split is partial (key
// mask, clamped DMA descriptor).  Without it the steady-state step has no mask branch, which
// would otherwise split the step into basic blocks and push the row sums out of the MFMA block.
// STRIDED: Q, K, V and O addressed through per-tensor (batch, head, row) strides in elements
// (d contiguous, K and V sharing strides), e.g. [B, L, H, d] tensors viewed as [B, H, L, d];
// false (contiguous [B, H, L, d]) folds every stride to a constant.
template <typename T, typename PT, int D, int MODE, bool TAIL, bool STRIDED = false>
__global__ __launch_bounds__(kThreads, kernel_wps(D, MODE, TAIL, STRIDED)) void fa_fwd_kernel(FwdArgs a) {
    using M = Mma<T>;
    using v8 = typename M::v8;
    constexpr int RB = kRB;                   // 32-row query blocks per wave
    constexpr int ROWB = D * 2;               // bytes per LDS row
    constexpr int kBK = bk_for(D);            // keys per KV tile
    constexpr int TILEB = kBK * ROWB;         // bytes of one K (or V) tile
    constexpr int NKS = D / 16;               // MFMA k-steps of Q K^T
    constexpr int NDB = D / 32;               // 32-column blocks of O
    constexpr int NKB = kBK / 32;             // 32-key blocks per KV tile
    // Deferred rescale (defer-max): the reference max m of a row is only moved when some
    // row of the wave's block sees a tile max above m + kThr (log2 units); P is then
    // bounded by 2^kThr instead of 1.  kThr = 8 measurably loses accuracy on peaked rows
    // (the dominant p is no longer exactly 1.0 in bf16), 4 does not (tests).
    constexpr float kThr = 4.f;
    constexpr bool RS16 = rs16_on(D, MODE, TAIL, STRIDED);

    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: K ring (2 slots) then V ring (2 slots), one [kBK][D] tile image per slot.
    char* const kring = smem;
    char* const vring = smem + 2 * TILEB;

    const int w = xcd_remap(blockIdx.x, gridDim.x);
    int qt, split;
    int64_t bh;
    decode_item(a, w, qt, split, bh);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave-uniform and, where it pays, PROVABLY so (an SGPR): the LDS-DMA destinations (M0)
    // derived from it then need no v_readfirstlane per DMA
    // (the pinned d = 128 step, below, measured +0.5 % with it; the compiler-scheduled one -2.5 %)
    constexpr bool PIN = D == 128 && RB == 1 && !TAIL;
    const int wid = ((kUniformWidMask & d_bit(D)) || PIN) ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
    const int l32 = lane & 31;
    const int hf = lane >> 5;

    FA_STAMP_V(8, __builtin_amdgcn_s_memrealtime());
    FA_STAMP(0);
    FA_STAMP_V(6, __builtin_amdgcn_s_getreg(4 | (31 << 11)));   // HW_REG_HW_ID, 32 bits
    FA_STAMP_V(7, __builtin_amdgcn_s_getreg(20 | (31 << 11)));  // HW_REG_XCC_ID
    const int64_t kv_begin = (int64_t)split * a.kv_per_split;
    const int64_t kv_end = kv_begin + a.kv_per_split < a.Lk ? kv_begin + a.kv_per_split : a.Lk;
    const int nkv = (int)(kv_end - kv_begin);
    const int ntiles = (nkv + kBK - 1) / kBK;

    // row strides in bytes (compile-time ROWB for contiguous tensors) and head bases
    const int qrb = STRIDED ? (int)(a.q_stride[2] * 2) : ROWB;
    const int krb = STRIDED ? (int)(a.k_stride[2] * 2) : ROWB;
    const int64_t hb = STRIDED ? bh / a.H : 0, hh = STRIDED ? bh - hb * a.H : 0;
    const int64_t q_head = STRIDED ? hb * a.q_stride[0] + hh * a.q_stride[1] : bh * a.Lq * D;
    const int64_t k_head = STRIDED ? hb * a.k_stride[0] + hh * a.k_stride[1] : bh * a.Lk * D;
    // Q descriptor over this workgroup's query tile only, so that its 32-bit offsets stay
    // small however long the sequence (rows past Lq read zeros)
    const int64_t q_tile0 = (int64_t)qt * kBQ;
    const unsigned short* Qh = (const unsigned short*)a.q + q_head + q_tile0 * (qrb / 2);
    const int64_t q_rows = a.Lq - q_tile0 < kBQ ? a.Lq - q_tile0 : kBQ;
    const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Qh, STRIDED ? (q_rows - 1) * qrb + ROWB : q_rows * ROWB);
    // K/V of this split; a tile's descriptor (made per DMA, scalar arithmetic only) starts
    // at the tile and ends at the split's last key, so the hardware range check -- which
    // does not rely on soffset -- zero-fills the rows of a partial last tile.
    const unsigned short* const kbase = (const unsigned short*)a.k + k_head + kv_begin * (krb / 2);
    const unsigned short* const vbase = (const unsigned short*)a.v + k_head + kv_begin * (krb / 2);

    // Q^T fragments (B operand): lane holds Q[row][16*ks + 8*hf + 0..7] of each of its
    // RB row blocks.  Rows past Lq read zeros and are never stored.
    const int64_t q_row0 = q_tile0 + wid * kRowsPerWave + l32;
    v8 qf[RB][NKS];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int qoff = (wid * kRowsPerWave + l32 + 32 * r) * qrb + hf * 16;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[r][ks] = __builtin_bit_cast(v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, qoff + ks * 32, 0, 0));
    }

    // K/V tiles go HBM -> LDS by LDS-DMA (buffer_load ... lds): no staging VGPRs, no
    // ds_write pass.  One wave instruction writes 1 KiB of LDS lane-linearly (M0 base +
    // 16*lane), so the swizzled image is produced by giving each lane the SOURCE chunk
    // that lds_off() places at its destination byte.
    constexpr int NDMA = TILEB / 1024;                      // 1 KiB pieces per tile
    constexpr int DPW = NDMA >= kWaves ? NDMA / kWaves : 1;  // pieces per (active) wave
    static_assert(NDMA % kWaves == 0 || kWaves % NDMA == 0, "tile pieces must split over waves");
    const bool dma_wave = wid * DPW < NDMA;                  // waves past the last piece idle
    int dma_src[DPW];
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
        const int b = (wid * DPW + i) * 1024 + lane * 16;  // destination byte in the tile image
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        dma_src[i] = row * krb + ch * 16;
    }
    auto dma_tile = [&](const unsigned short* base, char* slot, int t) {
        // descriptor over exactly the tile's valid keys (32-bit scalar arithmetic)
        // (readfirstlane: hipcc evaluates the clamp with v_med3, and a descriptor word it
        // cannot prove uniform turns every buffer op into a waterfall loop -- T20)
        const int rem = nkv - t * kBK;
        const int valid = TAIL ? __builtin_amdgcn_readfirstlane(rem < kBK ? (rem > 0 ? rem : 0) : kBK)
                               : (t < ntiles ? kBK : 0);
        // (strided rows: the range ends at the last valid row's end)
        const int bytes = STRIDED ? (valid > 0 ? (valid - 1) * krb + ROWB : 0) : valid * ROWB;
        const __amdgpu_buffer_rsrc_t rs =
            make_rsrc32((const char*)base + (int64_t)t * (STRIDED ? (int64_t)kBK * krb : (int64_t)TILEB), bytes);
        if (NDMA >= kWaves || dma_wave) {
#pragma unroll
            for (int i = 0; i < DPW; ++i) dma16(rs, slot + (wid * DPW + i) * 1024, dma_src[i], 0);
        }
    };

    // transposed-read geometry (constant per lane)
    const int grp = lane >> 4, gi = lane & 15;
    const int tr_row = 4 * (grp >> 1) + (gi >> 2);
    const int tr_col = 16 * (grp & 1) + 4 * (gi & 3);

    f32x16 o[RB][NDB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[r][db] = f32x16{};
    float m[RB], l[RB];  // reference max (log2 units) and this lane's half of the row sum
    f32x4 ls16[RB];      // RS16: row sum of query (lane & 15) + 16 * (lane >> 5), in every register
#pragma unroll
    for (int r = 0; r < RB; ++r) ls16[r] = f32x4{};
    // A of the RS16 MFMA: output rows 0-7 sum lane groups 0 and 2 (query n, both key halves),
    // rows 8-15 groups 1 and 3 (query n + 16)
    v8 sel16;
    {
        constexpr unsigned kOne = std::is_same_v<T, __bf16> ? 0x3F80u : 0x3C00u;  // 1.0 in T
        const unsigned e = ((lane & 15) < 8) == (((lane >> 4) & 1) == 0) ? kOne | (kOne << 16) : 0u;
        sel16 = __builtin_bit_cast(v8, u32x4{e, e, e, e});
    }
    const int rs16_src = ((lane & 31) < 16 ? (lane & 31) : (lane & 31) + 16) * 4;  // holder of own row
    const int rs16_row = ((lane & 15) + 16 * (lane >> 5)) * 4;                      // row held here
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        m[r] = -INFINITY;
        l[r] = 0.f;
    }
    const float c = a.scale_log2;

    // S^T[key][q] = K . Q^T for one tile (two 32-key blocks), every K fragment feeding the
    // RB row blocks.  Fragments are read in groups of two k-steps, one group ahead.
    auto qk = [&](const char* kb, f32x16 (&s)[RB][NKB]) {
        constexpr int G = 2;  // k-steps per read group
        v8 kf[2][NKB][G];     // [buffer][b2][k-step in group]
        auto rd = [&](int g, v8 (&dst)[NKB][G]) {
#pragma unroll
            for (int j = 0; j < G; ++j)
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2)
                    dst[b2][j] = *(const v8*)(kb + lds_off<D>(b2 * 32 + l32, 2 * (g * G + j) + hf));
        };
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2) s[r][b2] = f32x16{};
        rd(0, kf[0]);
#pragma unroll
        for (int g = 0; g < NKS / G; ++g) {
            if (g + 1 < NKS / G) rd(g + 1, kf[(g + 1) & 1]);
#pragma unroll
            for (int j = 0; j < G; ++j)
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                    for (int r = 0; r < RB; ++r) s[r][b2] = M::mma(kf[g & 1][b2][j], qf[r][g * G + j], s[r][b2]);
        }
    };
    // P = 2^(S*c - m) in place, and (VALU-sum kernels) its row sum into l
    auto exp_tile = [&](f32x16 (&s)[RB][NKB]) {
        if constexpr (D <= kPackedMaxD && RS16) {
            // packed fp32 FMAs (the MFMA pipe is mostly idle at small d), all FMAs of a 32-key
            // block ahead of its exponentials: no exponential right behind the FMA that feeds
            // it (a hazard wait state each)
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const f32x2 c2 = {c, c}, nm2 = {-m[r], -m[r]};
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2) {
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {
                        f32x2 x = {s[r][b2][i], s[r][b2][i + 1]};
                        x = __builtin_elementwise_fma(x, c2, nm2);
                        s[r][b2][i] = x[0];
                        s[r][b2][i + 1] = x[1];
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) s[r][b2][i] = __builtin_amdgcn_exp2f(s[r][b2][i]);
                }
            }
            return;
        }
        if constexpr (D <= kPackedMaxD) {
            // packed fp32 (v_pk_fma_f32 / v_pk_add_f32): two scores per VALU instruction
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const f32x2 c2 = {c, c}, nm2 = {-m[r], -m[r]};
                f32x2 sum2[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
                for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {
                        f32x2 x = {s[r][b2][i], s[r][b2][i + 1]};
                        x = __builtin_elementwise_fma(x, c2, nm2);
                        x[0] = __builtin_amdgcn_exp2f(x[0]);
                        x[1] = __builtin_amdgcn_exp2f(x[1]);
                        s[r][b2][i] = x[0];
                        s[r][b2][i + 1] = x[1];
                        sum2[(i >> 1) & 1] += x;
                    }
                const f32x2 t = sum2[0] + sum2[1];
                l[r] += t[0] + t[1];
            }
            return;
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float sum4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    s[r][b2][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r][b2][i], c, -m[r]));
                    if (!RS16) sum4[(b2 * 16 + i) & 3] += s[r][b2][i];
                }
            if (!RS16) l[r] += (sum4[0] + sum4[1]) + (sum4[2] + sum4[3]);
        }
    };
    // keys past the end of the split (only in the last, partial tile) -> -inf
    auto mask = [&](int t, f32x16 (&s)[RB][NKB]) {
        const int valid = nkv - t * kBK;
        if (valid < kBK) {
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = b2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf;
                    if (key >= valid) {
#pragma unroll
                        for (int r = 0; r < RB; ++r) s[r][b2][i] = -INFINITY;
                    }
                }
        }
    };
    // row max of a (masked) tile, both lane halves, in log2 units (v_maximum3: no
    // canonicalising v_max x,x per MFMA result, unlike fmaxf)
    auto rowmax = [&](const f32x16 (&s)[RB][NKB], float (&mx)[RB]) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float mx4[4];  // 4 independent chains over the tile's 16*NKB values
#pragma unroll
            for (int j = 0; j < 4; ++j) mx4[j] = s[r][0][j];
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (b2 > 0 || i >= 4) mx4[i & 3] = fmax_nc(mx4[i & 3], s[r][b2][i]);
            mx[r] = pair_max(fmax_nc(fmax_nc(mx4[0], mx4[1]), fmax_nc(mx4[2], mx4[3]))) * c;
        }
    };
    // V^T fragments of (32-key block b2, 32-column block db): 4 transposed reads of 4
    // keys; element j of the A operand is key 16*ss + 8*(j>>2) + 4*hf + (j&3), the same
    // key as element j of the P^T B operand.  Inline asm: hipcc cannot prove the builtin
    // form disjoint from the in-flight LDS-DMA and would drain it (vmcnt(0)) before every
    // read; vwait() waits for them and names every destination.  Every read is one of two
    // per-lane base addresses (key rows +0 / +8, whose swizzles differ) plus an immediate:
    // lds_off(row + 32*b2 + 16*ss, ch + 4*db) = lds_off(row, ch) + (4*b2 + 2*ss)*8*ROWB + 512*db.
    // (the V ring's base is in the address registers, keeping every immediate < 64 KiB)
    const unsigned vbase0 =
        (unsigned)(size_t)vring + lds_off<D>(tr_row, tr_col >> 3) + (tr_col & 7) * 2;
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
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(vf[0][0]), "+v"(vf[0][1]), "+v"(vf[1][0]), "+v"(vf[1][1]));
    };

    // One pipeline step for tile t, whose raw (masked) scores are in sc and row max in mx:
    //   rescale decision; DMA K(t+2), V(t+1) into the ring slots freed by the previous step's
    //   barrier; QK^T(t+1) -> sn beside exp / sum of sc; pack P;
    //   P.V(t), then mask + row max of sn;  barrier (which also drains the DMA).
    // P = t & 1 is a compile-time constant (the loop runs steps in pairs).
    auto step = [&](auto par_c, auto flags_c, int t, f32x16 (&sc)[RB][NKB], f32x16 (&sn)[RB][NKB],
                    float (&mx)[RB]) {
        constexpr int P = decltype(par_c)::value;
        // Compile-time step flags, so that QK^T(t+1), the exponentials, the packing, P.V(t)
        // and the row max of tile t+1 form ONE basic block the scheduler can interleave
        // (runtime `if`s split it: hipcc hoisted the shared exp code into a join block,
        // away from the MFMAs).
        //   MORE      tile t+1 exists
        //   MASKNEXT  tile t+1 may be the partial last tile (needs the key mask)
        //   DMAK      tile t+2 exists (its K is prefetched now)
        constexpr int F = decltype(flags_c)::value;
        constexpr bool MORE = F & 1, MASKNEXT = TAIL && (F & 2), DMAK = F & 4;

#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (__builtin_amdgcn_ballot_w64(mx[r] > m[r] + kThr)) {
                const float m_new = fmaxf(m[r], mx[r]);
                const float alpha = __builtin_amdgcn_exp2f(m[r] - m_new);
                m[r] = m_new;
                l[r] *= alpha;
                if constexpr (RS16)
                    ls16[r] *= __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(rs16_row, __builtin_bit_cast(int, alpha)));
#pragma unroll
                for (int db = 0; db < NDB; ++db) o[r][db] *= alpha;
            }
        }

        // DMA issued in the MFMA block (the scheduler spreads the pieces among the MFMAs);
        // tile counts are checked against the compile-time MORE where possible
        if constexpr (DMAK) dma_tile(kbase, kring + P * TILEB, t + 2);
        if constexpr (MORE) dma_tile(vbase, vring + (1 - P) * TILEB, t + 1);
        if constexpr (MORE) qk(kring + (1 - P) * TILEB, sn);
        exp_tile(sc);
        v8 pb[RB][NKB][2];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int b2 = 0; b2 < NKB; ++b2)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    u32x4 u;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        u[j] = pack2<T>(sc[r][b2][8 * ss + 2 * j], sc[r][b2][8 * ss + 2 * j + 1]);
                    pb[r][b2][ss] = __builtin_bit_cast(v8, u);
                }

        // O^T[dv][q] += V^T[dv][key] . P^T[key][q]; reads of the next (b2, db) block
        // overlap this block's MFMAs.
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
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    o[r][DB] = M::mma(__builtin_bit_cast(v8, vv), pb[r][B2][ss], o[r][DB]);
                    if constexpr (RS16 && DB == 0) ls16[r] = M::mma16(sel16, pb[r][B2][ss], ls16[r]);
                }
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
            if constexpr ((kRowmaxFenceMask & d_bit(D)) != 0) __builtin_amdgcn_sched_barrier(0);
            if constexpr (MASKNEXT) mask(t + 1, sn);
            rowmax(sn, mx);
        }
        __syncthreads();  // hipcc drains the DMA (vmcnt(0)) here: K(t+2), V(t+1) landed
    };

    // ---- the d = 128 steady step with a pinned instruction schedule (no key tail, 32-row
    // waves).  The step is laid out as 36 MFMA slots, each closed by a scheduling barrier so
    // that hipcc keeps every slot's fillers with its MFMA (it still allocates registers and
    // inserts the hazard wait states):
    //   phase A, 16 slots: QK^T(t+1), two accumulation chains (32-key blocks) alternating;
    //     fillers: the FMA + exponential of 20 of tile t's 32 scores per lane, the packing of
    //     the first key block's P fragments, the K reads KA slots ahead, the 8 DMA pieces;
    //   phase B, 20 slots: P.V(t) by key block, (db, ss) inside, and the key block's two row-sum
    //     MFMAs after it; fillers: the remaining 12 exponentials and the second key block's
    //     packing (ahead of the MFMAs that read them), the V reads VA MFMAs ahead, the row max
    //     of tile t+1 (its QK^T finished >= 8 slots earlier).
    // Every LDS read is inline asm with an explicit counted lgkmcnt wait on the registers it
    // fills (so neither hipcc's waitcnt pass nor the in-flight LDS-DMA is involved).
    // Measured (round 3, A/B in one process): 2.74k -> 2.56k cycles per step at C3, C3 +3.1 %,
    // C4 +3.2 % wall (the chip holds a lower clock as the MFMAs pack closer: the loop is power-
    // bound); K / V reads one slot deeper, 24 exponentials in phase A: same;
    // the DMA pieces in phase B: C4 -3 %; VALU row sums instead of the row-sum MFMAs: C3 -1.5 %,
    // C4 -2.5 %; s_setprio by step parity (three patterns): C3 0, C4 -1.5 ... -2.3 %.
    constexpr int KA = 3, VA = 2;  // reads in flight: K fragments (slots), V operands (MFMAs)
    constexpr int EXPA = 20;       // exponentials in phase A (the rest: phase B, 2 per slot)
    const int swz = (l32 >> 2) & 3;
    const unsigned kaddr_e = (unsigned)(size_t)kring + (l32 >> 3) * 2048 + 64 * (l32 & 7) + 16 * (hf ^ swz);
    const unsigned kaddr_o = (unsigned)(size_t)kring + (l32 >> 3) * 2048 + 64 * (l32 & 7) + 16 * ((2 + hf) ^ swz);
    auto step_pinned = [&](auto par_c, auto flags_c, int t, f32x16 (&sc)[RB][NKB], f32x16 (&sn)[RB][NKB],
                           float (&mx)[RB]) {
        constexpr int P = decltype(par_c)::value;
        constexpr int F = decltype(flags_c)::value;
        constexpr bool DMAK = F & 4;
        static_assert(NKB == 2 && NKS == 8 && NDB == 4 && DPW == 4, "pinned schedule is for d = 128");
        if (__builtin_amdgcn_ballot_w64(mx[0] > m[0] + kThr)) {
            const float m_new = fmaxf(m[0], mx[0]);
            const float alpha = __builtin_amdgcn_exp2f(m[0] - m_new);
            m[0] = m_new;
            ls16[0] *= __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(rs16_row, __builtin_bit_cast(int, alpha)));
#pragma unroll
            for (int db = 0; db < NDB; ++db) o[0][db] *= alpha;
        }
        const float nm = -m[0];
        // DMA descriptors of K(t+2) (zeros past the end) and V(t+1), as dma_tile makes them
        constexpr int64_t TSTRIDE = STRIDED ? 0 : TILEB;  // (strided: kBK rows of krb bytes)
        const int64_t tstride = STRIDED ? (int64_t)kBK * krb : TSTRIDE;
        const int tbytes = STRIDED ? (kBK - 1) * krb + ROWB : TILEB;
        const __amdgpu_buffer_rsrc_t krs =
            make_rsrc32((const char*)kbase + (int64_t)(t + 2) * tstride, DMAK && t + 2 < ntiles ? tbytes : 0);
        const __amdgpu_buffer_rsrc_t vrs = make_rsrc32((const char*)vbase + (int64_t)(t + 1) * tstride, tbytes);
        char* const kdst = kring + P * TILEB + wid * DPW * 1024;
        char* const vdst = vring + (1 - P) * TILEB + wid * DPW * 1024;

        u32x4 kf[KA + 1];
        // (inline asm in a nested generic lambda must not capture: every operand is a parameter)
        auto kread_ = [](auto r_c, auto p_c, u32x4 (&kf)[KA + 1], unsigned ke, unsigned ko) {
            constexpr int R = decltype(r_c)::value, KS = R / 2, B2 = R % 2, PP = decltype(p_c)::value;
            constexpr int OFF = (1 - PP) * TILEB + B2 * 8192 + 512 * (KS >> 1);
            if constexpr (KS & 1)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[R % (KA + 1)]) : "v"(ko), "i"(OFF) : "memory");
            else
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[R % (KA + 1)]) : "v"(ke), "i"(OFF) : "memory");
        };
        auto kread = [&](auto r_c) { kread_(r_c, par_c, kf, kaddr_e, kaddr_o); };
        auto lwait = [](auto n_c, u32x4& reg) {
            asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(reg) : "i"(decltype(n_c)::value) : "memory");
        };
        auto lwait2 = [](auto n_c, u32x2 (&reg)[2]) {
            asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(reg[0]), "+v"(reg[1]) : "i"(decltype(n_c)::value) : "memory");
        };
        auto ex = [&](auto e_c) {  // FMA + exponential of score e of tile t
            constexpr int E = decltype(e_c)::value;
            sc[0][E / 16][E % 16] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[0][E / 16][E % 16], c, nm));
        };
        u32x4 pbu[2][2];  // packed P^T fragments [b2][ss]
        auto cvt = [&](auto k_c) {  // pair k of key block k / 8 -> fragment (k / 8, (k % 8) / 4), dword k % 4
            constexpr int K = decltype(k_c)::value, B2 = K / 8, SS = (K % 8) / 4, J = K % 4;
            pbu[B2][SS][J] = pack2<T>(sc[0][B2][8 * SS + 2 * J], sc[0][B2][8 * SS + 2 * J + 1]);
        };
        auto dma = [&](auto i_c) {
            constexpr int I = decltype(i_c)::value;
            if constexpr (I < 4) {
                if constexpr (DMAK) dma16(krs, kdst + I * 1024, dma_src[I], 0);
            } else {
                dma16(vrs, vdst + (I - 4) * 1024, dma_src[I - 4], 0);
            }
        };

        // ---- phase A: QK^T(t+1) || exp(t)
#pragma unroll
        for (int b2 = 0; b2 < NKB; ++b2) sn[0][b2] = f32x16{};
        static_for<KA>([&](auto r_c) { kread(r_c); });
        static_for<16>([&](auto s_c) {
            constexpr int S = decltype(s_c)::value;
            if constexpr (S + KA < 16) kread(std::integral_constant<int, S + KA>{});
            constexpr int AFTER = (S + KA < 16 ? S + KA : 15) - S;  // K reads issued after read S
            lwait(std::integral_constant<int, AFTER>{}, kf[S % (KA + 1)]);
            sn[0][S % 2] = M::mma(__builtin_bit_cast(v8, kf[S % (KA + 1)]), qf[0][S / 2], sn[0][S % 2]);
            constexpr int E0 = S * EXPA / 16, E1 = (S + 1) * EXPA / 16;  // exponentials 0..EXPA-1
            static_for<E1 - E0>([&](auto j_c) { ex(std::integral_constant<int, E0 + decltype(j_c)::value>{}); });
            if constexpr (S >= 6 && S < 14) cvt(std::integral_constant<int, S - 6>{});  // key block 0 packs
            if constexpr (S % 2 == 1) dma(std::integral_constant<int, S / 2>{});
            __builtin_amdgcn_sched_barrier(0);
        });

        // ---- phase B: P.V(t) || exp(t) rest, row max(t+1)
        // PV MFMA p (0..15): b2 = p / 8, db = (p % 8) / 2, ss = p % 2; its V^T operand is two
        // transposed reads, issued VA MFMAs ahead
        u32x2 vf[VA + 1][2];
        auto vread_ = [](auto p_c, auto par, u32x2 (&vf)[VA + 1][2], unsigned vb0, unsigned vb1) {
            constexpr int PP = decltype(p_c)::value, B2 = PP / 8, DB = (PP % 8) / 2, SS = PP % 2;
            constexpr int OFF = decltype(par)::value * TILEB + 4 * B2 * 8 * ROWB + 512 * DB + SS * 2 * 8 * ROWB;
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][0]) : "v"(vb0), "i"(OFF) : "memory");
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[PP % (VA + 1)][1]) : "v"(vb1), "i"(OFF + 8 * ROWB) : "memory");
        };
        auto vread = [&](auto p_c) { vread_(p_c, par_c, vf, vbase0, vbase1); };
        float m4[4];
        static_for<VA>([&](auto p_c) { vread(p_c); });
        static_for<20>([&](auto j_c) {
            constexpr int J = decltype(j_c)::value;
            // slot J: PV MFMA p, or a row-sum MFMA (J = 8, 9: key block 0; 18, 19: key block 1)
            constexpr bool RS = (J % 10) >= 8;
            constexpr int PP = J < 10 ? J : J - 2;
            if constexpr (!RS) {
                if constexpr (PP + VA < 16) vread(std::integral_constant<int, PP + VA>{});
                constexpr int AFTER = 2 * ((PP + VA < 16 ? PP + VA : 15) - PP);
                lwait2(std::integral_constant<int, AFTER>{}, vf[PP % (VA + 1)]);
                constexpr int B2 = PP / 8, DB = (PP % 8) / 2, SS = PP % 2;
                const u32x4 vv = {vf[PP % (VA + 1)][0][0], vf[PP % (VA + 1)][0][1], vf[PP % (VA + 1)][1][0],
                                  vf[PP % (VA + 1)][1][1]};
                o[0][DB] = M::mma(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbu[B2][SS]), o[0][DB]);
            } else {
                constexpr int B2 = J / 10, SS = J % 2;
                ls16[0] = M::mma16(sel16, __builtin_bit_cast(v8, pbu[B2][SS]), ls16[0]);
            }
            // exponentials EXPA..31 two per slot from slot 0, key block 1 packs in slots 2..9
            // (EXPA in [20, 24]: every pack comes after its exponentials in program order)
            static_assert(EXPA >= 20 && EXPA <= 24, "packs follow their exponentials in program order");
            if constexpr (EXPA + 2 * J < 32) ex(std::integral_constant<int, EXPA + 2 * J>{});
            if constexpr (EXPA + 2 * J + 1 < 32) ex(std::integral_constant<int, EXPA + 2 * J + 1>{});
            if constexpr (J >= 2 && J < 10) cvt(std::integral_constant<int, 8 + J - 2>{});
            // row max of tile t+1 in slots 8..19: four chains of v_maximum3 over 8 scores each
            if constexpr (J >= 8 && J < 16) {
                constexpr int CH = (J - 8) / 2, H = (J - 8) % 2;  // chain, half
                // chain CH holds scores i with i % 4 == CH of both key blocks
                if constexpr (H == 0)
                    m4[CH] = fmax_nc(fmax_nc(sn[0][0][CH], sn[0][0][CH + 4]), fmax_nc(sn[0][0][CH + 8], sn[0][0][CH + 12]));
                else
                    m4[CH] = fmax_nc(fmax_nc(m4[CH], fmax_nc(sn[0][1][CH], sn[0][1][CH + 4])),
                                     fmax_nc(sn[0][1][CH + 8], sn[0][1][CH + 12]));
            }
            if constexpr (J == 17) mx[0] = pair_max(fmax_nc(fmax_nc(m4[0], m4[1]), fmax_nc(m4[2], m4[3]))) * c;
            __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();  // hipcc drains the DMA (vmcnt(0)) here: K(t+2), V(t+1) landed
    };

    // prologue: K(0), V(0), K(1) -> LDS; S(0) = QK^T(0)
    dma_tile(kbase, kring, 0);
    dma_tile(vbase, vring, 0);
    if (ntiles > 1) dma_tile(kbase, kring + TILEB, 1);
    // Q's loads must retire here: otherwise hipcc's waitcnt pass carries them into the loop
    // header and, merging with the back edge, waits vmcnt(N) in front of every MFMA.
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[r][ks]));
    __syncthreads();
    FA_STAMP(1);
    f32x16 sa[RB][NKB], sb[RB][NKB];
    float mx[RB];
    qk(kring, sa);
    if constexpr (TAIL) mask(0, sa);
    rowmax(sa, mx);
    // the reference max starts at tile 0's row max (every tile holds a valid key): step 0
    // then never takes the rescale branch that a -inf start would force on every workgroup
#pragma unroll
    for (int r = 0; r < RB; ++r) m[r] = mx[r];
    __syncthreads();  // K slot 0 is rewritten by step 0's DMA of K(2)
    FA_STAMP(2);

    {
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        // flags: 1 = MORE, 2 = MASKNEXT, 4 = DMAK (see step)
        using STEADY = std::integral_constant<int, 1 | 4>;     // t+1, t+2 exist, t+1 not last
        using NEXTLAST = std::integral_constant<int, 1 | 2>;   // t+1 is the last tile
        using NEXTLASTK = std::integral_constant<int, 1 | 2 | 4>;
        using LAST = std::integral_constant<int, 0>;
        // (the pinned schedule for every step with a next tile; the last step has no QK^T)
        auto run = [&](auto par_c, auto flags_c, int t, f32x16 (&sc)[RB][NKB], f32x16 (&sn)[RB][NKB],
                       float (&mx)[RB]) {
            if constexpr (PIN && (decltype(flags_c)::value & 1)) step_pinned(par_c, flags_c, t, sc, sn, mx);
            else step(par_c, flags_c, t, sc, sn, mx);
        };
        int t = 0;
        for (; t + 2 < ntiles; t += 2) {
            // step t: tile t+1 is never the last one here.  Step t+1 may prefetch K(t+3)
            // past the end: the buffer range check turns it into zeros nobody reads, which
            // keeps the step branch-free.
            run(C0{}, STEADY{}, t, sa, sb, mx);
            run(C1{}, NEXTLASTK{}, t + 1, sb, sa, mx);
        }
        if (ntiles - t == 2) {  // t is even here
            run(C0{}, NEXTLAST{}, t, sa, sb, mx);
            run(C1{}, LAST{}, t + 1, sb, sa, mx);
        } else {
            run(C0{}, LAST{}, t, sa, sb, mx);
        }
    }

    FA_STAMP(3);
    // output row base (final O; the fused split mode's o_final)
    const int64_t o_head = STRIDED ? hb * a.o_stride[0] + hh * a.o_stride[1] : bh * a.Lq * D;
    const int64_t orow = STRIDED ? a.o_stride[2] : D;
    // ---- epilogue: lane holds O^T[dv][q_row] for dv = 32*db + (i&3) + 8*(i>>2) + 4*hf
    // store v * scale as one 16-bit output row (row base Oh).  Column groups g and g+1 of a
    // row sit in lanes l (cols 8g..+3, 8g+8..+11) and l+32 (8g+4..+7, 8g+12..+15); one
    // v_permlane32_swap per dword leaves 16 contiguous bytes in each lane -> one dwordx4
    // store per pair instead of two dwordx2 (cdna_hip_programming.md T21).
    auto store_row = [&](unsigned short* Oh, const f32x16 (&v)[NDB], float scale) {
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int gp = 0; gp < 4; gp += 2) {
                unsigned x0 = pack2<T>(v[db][4 * gp + 0] * scale, v[db][4 * gp + 1] * scale);
                unsigned x1 = pack2<T>(v[db][4 * gp + 2] * scale, v[db][4 * gp + 3] * scale);
                unsigned y0 = pack2<T>(v[db][4 * gp + 4] * scale, v[db][4 * gp + 5] * scale);
                unsigned y1 = pack2<T>(v[db][4 * gp + 6] * scale, v[db][4 * gp + 7] * scale);
                const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                const u32x4 u = {s0[0], s1[0], s0[1], s1[1]};
                *(u32x4*)(Oh + db * 32 + 8 * gp + 8 * hf) = u;
            }
    };
    auto row_sum = [&](int r) {
        return RS16 ? __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(rs16_src, __builtin_bit_cast(int, ls16[r][0])))
                    : pair_sum(l[r]);
    };
    if constexpr (MODE == kFused) {
        // Split-KV partials combined on chip.  Every workgroup stores its normalised partial
        // O (PT) and lse in FRAGMENT order -- lane-linear 16-byte pieces, so both the stores
        // and the combine's loads are fully coalesced -- then counts itself in its query
        // tile's counter; the workgroup that arrives last reads the other splits' partials
        // (just written: served by L2 / Infinity Cache) and writes O.  Hand-off protocol
        // (MI355X_MICROARCH.md, inter-workgroup visibility, first table row): all partial
        // stores and loads sc1; every wave waits vmcnt(0) after its stores; a barrier; ONE
        // lane's agent-scope atomic add; the adder that saw count nsplit-1 tells the other
        // waves through LDS behind a barrier.  No workgroup ever waits for another.
        constexpr int SC1 = 16;                    // cache-policy bit: sc1
        constexpr int NF = NDB * 4;                // fragments (4 values) per lane and row block
        constexpr int BLK = kBQ * D;               // partial elements per (split, tile) block
        const int64_t grp = bh * a.nqt + qt;
        auto blk_of = [&](int sp) { return (int64_t)sp * a.BH * a.nqt + grp; };
        auto o_rsrc = [&](int sp) {
            return make_rsrc((const PT*)a.o + blk_of(sp) * BLK, (int64_t)BLK * sizeof(PT));
        };
        auto l_rsrc = [&](int sp) { return make_rsrc(a.lse + blk_of(sp) * kBQ, (int64_t)kBQ * 4); };
        auto frag_off = [&](int r, int f) {  // byte offset of fragment f of row block r
            return ((((wid * RB + r) * NF + f) * 64 + lane) * 4) * (int)sizeof(PT);
        };
        const int lse_off = (wid * RB) * 32 * 4 + l32 * 4;  // + r*128

        constexpr bool SCALED = std::is_same_v<PT, f16s_t>;  // fp16 partials, per-row 2^-e
        using PH = std::conditional_t<SCALED, _Float16, T>;   // 16-bit partial element type
        auto e_rsrc = [&](int sp) { return make_rsrc(a.esc + blk_of(sp) * kBQ, (int64_t)kBQ * 4); };
        float inv[RB], lse_own[RB], esc_own[RB];
        {
            const __amdgpu_buffer_rsrc_t ors = o_rsrc(split), lrs = l_rsrc(split);
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const float l_tot = row_sum(r);
                inv[r] = 1.f / l_tot;
                lse_own[r] = m[r] + __builtin_amdgcn_logf(l_tot);
                esc_own[r] = 0.f;
                if constexpr (SCALED) {
                    // the row's largest |O / l| below 1 after the exact scale 2^-e
                    float mx = 0.f;
#pragma unroll
                    for (int db = 0; db < NDB; ++db)
#pragma unroll
                        for (int i = 0; i < 16; ++i) mx = fmax_nc(mx, __builtin_fabsf(o[r][db][i]));
                    const int e = __builtin_amdgcn_frexp_expf(pair_max(mx) * inv[r]);
                    esc_own[r] = (float)e;
                    inv[r] = __builtin_amdgcn_ldexpf(inv[r], -e);
                }
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int db = f >> 2, g4 = f & 3;
                    const f32x4 src = {o[r][db][4 * g4], o[r][db][4 * g4 + 1], o[r][db][4 * g4 + 2],
                                       o[r][db][4 * g4 + 3]};
                    if constexpr (sizeof(PT) == 4) {
                        const u32x4 u = {__float_as_uint(src[0] * inv[r]), __float_as_uint(src[1] * inv[r]),
                                         __float_as_uint(src[2] * inv[r]), __float_as_uint(src[3] * inv[r])};
                        __builtin_amdgcn_raw_buffer_store_b128(u, ors, frag_off(r, f), 0, SC1);
                    } else {
                        const u32x2 u = {pack2<PH>(src[0] * inv[r], src[1] * inv[r]),
                                         pack2<PH>(src[2] * inv[r], src[3] * inv[r])};
                        __builtin_amdgcn_raw_buffer_store_b64(u, ors, frag_off(r, f), 0, SC1);
                    }
                }
                if (hf == 0) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lse_own[r]), lrs, lse_off + r * 128, 0, SC1);
                    if constexpr (SCALED)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(esc_own[r]), e_rsrc(split),
                                                              lse_off + r * 128, 0, SC1);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* const last_flag = (int*)smem;  // LDS is free: the KV loop ended with a barrier
        if (tid == 0) {
            const unsigned old = __hip_atomic_fetch_add(a.counters + grp, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            const int last = old + 1 == (unsigned)a.nsplit;
            if (last) a.counters[grp] = 0;  // leave the counter zero for the next launch
            *last_flag = last;
        }
        __syncthreads();
        if (!*last_flag) return;

        // Sum in split order 0, 1, ... whatever workgroup came last (its own partial is read
        // back too), so that O is bitwise repeatable.
        const int ns = a.nsplit;
        auto load_lse = [&](int sp, int r) {
            return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(l_rsrc(sp), lse_off + r * 128, 0, SC1));
        };
        typedef unsigned frag_t __attribute__((ext_vector_type(sizeof(PT))));  // 4 x PT
        auto load_frags = [&](int sp, int r, frag_t (&dst)[NF]) {
            const __amdgpu_buffer_rsrc_t rs = o_rsrc(sp);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if constexpr (sizeof(PT) == 4)
                    dst[f] = __builtin_bit_cast(frag_t, __builtin_amdgcn_raw_buffer_load_b128(rs, frag_off(r, f), 0, SC1));
                else
                    dst[f] = __builtin_bit_cast(frag_t, __builtin_amdgcn_raw_buffer_load_b64(rs, frag_off(r, f), 0, SC1));
            }
        };
        auto unpack = [](const frag_t& u, int j) -> float {
            if constexpr (sizeof(PT) == 4) {
                return __uint_as_float(u[j]);
            } else {
                const unsigned w = u[j >> 1];
                const unsigned short h = (unsigned short)((j & 1) ? (w >> 16) : (w & 0xffff));
                return (float)__builtin_bit_cast(PH, h);
            }
        };
        // weight of split sp's stored values: 2^(lse - M), times 2^e for scaled partials
        auto load_esc = [&](int sp, int r) {
            if constexpr (SCALED)
                return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(e_rsrc(sp), lse_off + r * 128, 0, SC1));
            else
                return 0.f;
        };
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            float M = lse_own[r];
            // scaled partials: weights carry 2^(e - E), E the largest exponent of the row's
            // splits, and 2^E is applied after the division (2^e overflows near bf16's max)
            float E = -1000.f;
            for (int sp = 0; sp < ns; ++sp) {
                M = fmaxf(M, load_lse(sp, r));
                if constexpr (SCALED) E = fmaxf(E, load_esc(sp, r));
            }
            float wsum = 0.f;
            f32x16 acc[NDB];
#pragma unroll
            for (int db = 0; db < NDB; ++db) acc[db] = f32x16{};
            auto fma_split = [&](const frag_t (&fr)[NF], float w, float es) {
                const float wv = SCALED ? __builtin_amdgcn_ldexpf(w, (int)(es - E)) : w;
#pragma unroll
                for (int f = 0; f < NF; ++f)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[f >> 2][4 * (f & 3) + j] = __builtin_fmaf(wv, unpack(fr[f], j), acc[f >> 2][4 * (f & 3) + j]);
                wsum += w;
            };
            // two splits in flight: the loads of split sp+1 overlap the FMAs of split sp
            frag_t fa_[NF], fb_[NF];
            float wa, wb = 0.f, ea, eb = 0.f;
            load_frags(0, r, fa_);
            wa = __builtin_amdgcn_exp2f(load_lse(0, r) - M);
            ea = load_esc(0, r);
            for (int sp = 0; sp < ns; sp += 2) {
                if (sp + 1 < ns) {
                    load_frags(sp + 1, r, fb_);
                    wb = __builtin_amdgcn_exp2f(load_lse(sp + 1, r) - M);
                    eb = load_esc(sp + 1, r);
                }
                fma_split(fa_, wa, ea);
                if (sp + 1 < ns) {
                    if (sp + 2 < ns) {
                        load_frags(sp + 2, r, fa_);
                        wa = __builtin_amdgcn_exp2f(load_lse(sp + 2, r) - M);
                        ea = load_esc(sp + 2, r);
                    }
                    fma_split(fb_, wb, eb);
                }
            }
            const int64_t q_row = q_row0 + 32 * r;
            float inv_w = 1.f / wsum;
            if constexpr (SCALED) {
#pragma unroll
                for (int db = 0; db < NDB; ++db)
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc[db][i] = __builtin_amdgcn_ldexpf(acc[db][i] * inv_w, (int)E);
                inv_w = 1.f;
            }
            if (q_row < a.Lq)
                store_row((unsigned short*)a.o_final + o_head + q_row * orow, acc, inv_w);
        }
    } else {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int64_t q_row = q_row0 + 32 * r;
        const float l_tot = row_sum(r);
        float inv = 1.f / l_tot;
        if (q_row >= a.Lq) continue;
        if constexpr (MODE == kFinal) {
            store_row((unsigned short*)a.o + o_head + q_row * orow, o[r], inv);
        } else {
            const int64_t chunk = q_row / a.chunk_rows, r_in = q_row % a.chunk_rows;
            const int64_t row_lin = chunk * a.BH * a.chunk_rows + bh * a.chunk_rows + r_in;
            PT* Op = (PT*)a.o + split * a.split_stride + row_lin * D;
            // per-row scaled fp16 (as in the fused split): O/l * 2^-e with the row's largest
            // |O/l| just below 1; the lse buffer then holds {lse, e} per row
            constexpr bool SCALED = std::is_same_v<PT, f16s_t>;
            using PH = std::conditional_t<SCALED, _Float16, T>;
            float esc = 0.f;
            if constexpr (SCALED) {
                float mx = 0.f;
#pragma unroll
                for (int db = 0; db < NDB; ++db)
#pragma unroll
                    for (int i = 0; i < 16; ++i) mx = fmax_nc(mx, __builtin_fabsf(o[r][db][i]));
                const int e = __builtin_amdgcn_frexp_expf(pair_max(mx) * inv);
                esc = (float)e;
                inv = __builtin_amdgcn_ldexpf(inv, -e);
            }
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const int col = db * 32 + 8 * g4 + 4 * hf;
                    if constexpr (sizeof(PT) == 4) {
                        f32x4 f = {o[r][db][4 * g4 + 0] * inv, o[r][db][4 * g4 + 1] * inv,
                                   o[r][db][4 * g4 + 2] * inv, o[r][db][4 * g4 + 3] * inv};
                        *(f32x4*)(Op + col) = f;
                    } else {
                        u32x2 u;
                        u[0] = pack2<PH>(o[r][db][4 * g4 + 0] * inv, o[r][db][4 * g4 + 1] * inv);
                        u[1] = pack2<PH>(o[r][db][4 * g4 + 2] * inv, o[r][db][4 * g4 + 3] * inv);
                        *(u32x2*)((unsigned short*)Op + col) = u;
                    }
                }
            // lse in log2 units: m + log2(l)  (v_log_f32 is log2)
            const float lse = m[r] + __builtin_amdgcn_logf(l_tot);
            if (hf == 0) {
                if constexpr (SCALED)
                    *(float2*)(a.lse + 2 * (split * a.BH * a.Lq + row_lin)) = make_float2(lse, esc);
                else
                    a.lse[split * a.BH * a.Lq + row_lin] = lse;
            }
        }
    }
    }
#if FA_STAMPS
    FA_STAMP(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FA_STAMP(5);
    FA_STAMP_V(9, __builtin_amdgcn_s_memrealtime());
#endif
}

}  // namespace fa
