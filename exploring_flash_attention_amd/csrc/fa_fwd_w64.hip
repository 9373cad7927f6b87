// fa_fwd_w64.hip -- FA-v1 forward at d = 128 with 64 query rows per wave.
//
// Same algorithm, LDS image, LDS-DMA ring and step pipeline as fa_fwd_kernel (fa_fwd.hip),
// re-balanced for the issue-bound regime measured there: a wave owns TWO
// 32-row blocks, so every K fragment and every transposed V fragment read from LDS feeds
// two MFMAs, and the K/V DMA pieces per MFMA halve.  That needs 512 registers per lane
// (one wave per SIMD), which hipcc cannot allocate well by itself (its AGPR copies and
// spills made a plain-C++ 64-row build 1.6x slower), so the MFMA state lives in AGPRs
// owned by inline asm:
//   a[0:127]    O accumulators   block (rb, db) at a[16*(4*rb + db)]
//   a[128:191]  Q^T fragments    (rb, ks) at a[128 + 4*(8*rb + ks)]   (B operand of S^T)
//   a[192:255]  K fragments      (b2, ks) at a[192 + 4*(8*b2 + ks)]   (A operand of S^T)
// and only S, P, the V fragments and the softmax state are compiler-allocated VGPRs.
// Every MFMA is asm, so every MFMA hazard is handled here, not by the compiler:
//   * VALU write -> MFMA read (P packed by v_cvt_pk): s_nop 1 in front of the first MFMA
//     that reads a freshly packed P fragment;
//   * MFMA write -> VALU read (S^T for the row max / mask, O for a rescale or the epilogue):
//     s_nop padding tied to the data (asm operands), so it cannot be hoisted above it;
//   * accvgpr_write -> MFMA SrcC (rescale, zero-init): s_nop after the writes.
// The compiler must never place values of its own in these AGPRs: every asm that writes
// them lists them as clobbers, and the kernel keeps the compiler's VGPR demand under 256 so
// that it never spills into AGPRs (checked in the ISA).
#include "fa_device.hpp"

// FA_W64_PIN: a sched_barrier after every MFMA slot, so the compiler cannot move the
// slot's VALU fillers (it otherwise sinks the exponentials below the MFMA block)
#ifndef FA_W64_PIN
#define FA_W64_PIN 1
#endif
// FA_W64_PVNOP: s_nop 1 in front of every P.V MFMA (off: every P and V operand is written
// at least one MFMA slot before its use -- P by the pinned exponential slots, V by LDS loads)
#ifndef FA_W64_PVNOP
#define FA_W64_PVNOP 0
#endif
// FA_W64_QLDS: the next item's Q^T goes HBM -> LDS (a per-wave 16 KiB image, by the wave
// itself, early in the current item) and LDS -> AGPRs at the seam, instead of HBM -> AGPRs
// in the item's last step (whose latency the seam otherwise waits for)
#ifndef FA_W64_QLDS
#define FA_W64_QLDS 1
#endif
#ifndef FA_W64_KEARLY
#define FA_W64_KEARLY 1
#endif
#ifndef FA_W64_KREADS_AHEAD
#define FA_W64_KREADS_AHEAD 4  // K-step read groups (2 fragments each) kept in flight
#endif

namespace fa {

namespace {

// clobber lists of the asm-owned AGPRs
#define FA_CLOB_O \
    "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", \
    "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", \
    "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", \
    "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", \
    "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", \
    "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", \
    "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", \
    "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", \
    "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", \
    "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", \
    "a126", "a127"
#define FA_CLOB_Q \
    "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", \
    "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", \
    "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", \
    "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", \
    "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", \
    "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191"
#define FA_CLOB_K \
    "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", \
    "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", \
    "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", \
    "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", \
    "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", \
    "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"

template <typename T> struct MfmaOp;
template <> struct MfmaOp<__bf16> {
    // S^T block = K . Q^T:  dst (VGPRs) [+]= a[K..K+3] x a[Q..Q+3]
    template <int K, int Q>
    static __device__ __forceinline__ void qk_first(f32x16& s) {
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], 0"
                     : "=v"(s) : "i"(K), "i"(K + 3), "i"(Q), "i"(Q + 3));
    }
    template <int K, int Q>
    static __device__ __forceinline__ void qk(f32x16& s) {
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                     : "+v"(s) : "i"(K), "i"(K + 3), "i"(Q), "i"(Q + 3));
    }
    // O^T block (AGPRs) += V^T fragment x P^T fragment
    template <int O, bool FRESH_P>
    static __device__ __forceinline__ void pv(const u32x4& v, const u32x4& p) {
        if constexpr (FRESH_P)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                         :: "i"(O), "i"(O + 15), "v"(v), "v"(p) : FA_CLOB_O);
        else
            asm volatile("v_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                         :: "i"(O), "i"(O + 15), "v"(v), "v"(p) : FA_CLOB_O);
    }
};
template <> struct MfmaOp<_Float16> {
    template <int K, int Q>
    static __device__ __forceinline__ void qk_first(f32x16& s) {
        asm volatile("v_mfma_f32_32x32x16_f16 %0, a[%c1:%c2], a[%c3:%c4], 0"
                     : "=v"(s) : "i"(K), "i"(K + 3), "i"(Q), "i"(Q + 3));
    }
    template <int K, int Q>
    static __device__ __forceinline__ void qk(f32x16& s) {
        asm volatile("v_mfma_f32_32x32x16_f16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                     : "+v"(s) : "i"(K), "i"(K + 3), "i"(Q), "i"(Q + 3));
    }
    template <int O, bool FRESH_P>
    static __device__ __forceinline__ void pv(const u32x4& v, const u32x4& p) {
        if constexpr (FRESH_P)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                         :: "i"(O), "i"(O + 15), "v"(v), "v"(p) : FA_CLOB_O);
        else
            asm volatile("v_mfma_f32_32x32x16_f16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                         :: "i"(O), "i"(O + 15), "v"(v), "v"(p) : FA_CLOB_O);
    }
};


// small asm helpers (free functions: asm operands naming variables captured by a generic
// lambda do not compile)
template <int A>
__device__ __forceinline__ void agpr_write4(const u32x4& v) {
    asm volatile("v_accvgpr_write_b32 a%c1, %0" :: "v"(v[0]), "i"(A) : FA_CLOB_Q);
    asm volatile("v_accvgpr_write_b32 a%c1, %0" :: "v"(v[1]), "i"(A + 1) : FA_CLOB_Q);
    asm volatile("v_accvgpr_write_b32 a%c1, %0" :: "v"(v[2]), "i"(A + 2) : FA_CLOB_Q);
    asm volatile("v_accvgpr_write_b32 a%c1, %0" :: "v"(v[3]), "i"(A + 3) : FA_CLOB_Q);
}
template <int A>
__device__ __forceinline__ void agpr_scale(float alpha) {
    float tmp;
    asm volatile("v_accvgpr_read_b32 %0, a%c1\n\ts_nop 1\n\tv_mul_f32 %0, %2, %0\n\tv_accvgpr_write_b32 a%c1, %0"
                 : "=&v"(tmp) : "i"(A), "v"(alpha) : FA_CLOB_O);
}
template <int A>
__device__ __forceinline__ float agpr_read(void) {
    float x;
    asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(A));
    return x;
}
// 16 bytes per lane from a buffer straight into a[A..A+3] (Q^T fragments); the caller
// waits (vmcnt) before the first MFMA that reads them
template <int A>
__device__ __forceinline__ void buffer_load_agpr4(__amdgpu_buffer_rsrc_t rs, int voff) {
    asm volatile("buffer_load_dwordx4 a[%c1:%c2], %0, %3, 0 offen" :: "v"(voff), "i"(A), "i"(A + 3), "s"(rs)
                 : "memory", FA_CLOB_Q);
}
// 16 bytes per lane LDS -> a[A..A+3]
template <int A, int OFF>
__device__ __forceinline__ void ds_read_agpr4(unsigned addr) {
    asm volatile("ds_read_b128 a[%c1:%c2], %0 offset:%3" :: "v"(addr), "i"(A), "i"(A + 3), "i"(OFF)
                 : "memory", FA_CLOB_Q);
}
__device__ __forceinline__ void lds_wait(u32x2 (&vf)[2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vf[0][0]), "+v"(vf[0][1]), "+v"(vf[1][0]), "+v"(vf[1][1]));
}
__device__ __forceinline__ void mfma_fence(f32x16 (&s)[2][2]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(s[0][0]), "+v"(s[0][1]), "+v"(s[1][0]), "+v"(s[1][1]));
}

}  // namespace

template <typename T>
__global__ __launch_bounds__(256, 1) void fa_fwd_w64_kernel(FwdArgs a) {
    using MO = MfmaOp<T>;
    constexpr int D = 128, ROWB = 256, kBK = 64, TILEB = kBK * ROWB;  // 16 KiB tiles
    constexpr int BQ = 256;                                            // 4 waves x 64 rows
    constexpr float kThr = 4.f;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const kring = smem;
    char* const vring = smem + 2 * TILEB;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, hf = lane >> 5;
    const int nkv = (int)a.Lk;
    const int ntiles = (nkv + kBK - 1) / kBK;

    // Persistent: each workgroup walks work items (query tile, b*h) with a grid stride; the
    // next item's K(0), K(1), V(0) and Q^T are fetched during the current item's last KV
    // tile, so the epilogue / prologue seam overlaps the loads (one workgroup per CU leaves
    // no second workgroup to cover it).
    const int nitems = a.nqt * (int)a.BH;
    int item = blockIdx.x;
    struct Item {
        int64_t bh, q_row0;
        const unsigned short *q, *k, *v;
    };
    auto item_at = [&](int it) {
        const int w = xcd_remap(it, nitems);
        Item r;
        const int qt = w % a.nqt;
        r.bh = w / a.nqt;
        r.q_row0 = (int64_t)qt * BQ + wid * 64 + l32;
        r.q = (const unsigned short*)a.q + r.bh * a.Lq * D;
        r.k = (const unsigned short*)a.k + r.bh * a.Lk * D;
        r.v = (const unsigned short*)a.v + r.bh * a.Lk * D;
        return r;
    };
    Item cur = item_at(item), nxt = cur;
    // Q^T fragments of an item -> a[128:191]
    auto load_q = [&](const Item& it) {
        const __amdgpu_buffer_rsrc_t qrs = make_rsrc(it.q, a.Lq * ROWB);
        static_for<16>([&](auto i_c) {
            constexpr int I = decltype(i_c)::value, RB = I / 8, KS = I % 8;
            buffer_load_agpr4<128 + 4 * I>(qrs, (int)((it.q_row0 + 32 * RB) * ROWB) + hf * 16 + KS * 32);
        });
    };
    // per-wave Q image (64 rows, the K tile image layout) at LDS 64 KiB + 16 KiB * wid
    char* const qimg = smem + 4 * TILEB + wid * TILEB;
    auto dma_q = [&](const Item& it) {  // this wave's 64 rows, 16 pieces, by this wave
        const int64_t row_base = it.q_row0 - l32;
        const int64_t rows_left = a.Lq - row_base;
        const int nrows = __builtin_amdgcn_readfirstlane((int)(rows_left < 64 ? (rows_left > 0 ? rows_left : 0) : 64));
        const __amdgpu_buffer_rsrc_t rs = make_rsrc32((const char*)(it.q + row_base * D), nrows * ROWB);
        static_for<16>([&](auto i_c) {
            constexpr int I = decltype(i_c)::value;
            const int b = I * 1024 + lane * 16;
            const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
            const int row = 8 * rg + (rem % 512) / 64;
            const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
            dma16(rs, qimg + I * 1024, row * ROWB + ch * 16, 0);
        });
    };
    // this wave's Q image -> a[128:191]: fragment (rb, ks) = lds_off(32 rb + l32, 2 ks + hf)
    const unsigned qb0 = (unsigned)(size_t)qimg + (l32 >> 3) * 8 * ROWB + 64 * (l32 & 7) + 16 * (hf ^ ((l32 >> 2) & 3));
    const unsigned qb1 = qb0 ^ 32;  // chunk bit 1 flipped: ((hf ^ x) ^ 2) * 16
    auto read_q = [](unsigned qb0, unsigned qb1) {
        static_for<16>([&](auto i_c) {
            constexpr int I = decltype(i_c)::value, RB = I / 8, KS = I % 8;
            ds_read_agpr4<128 + 4 * I, RB * 8192 + 512 * (KS >> 1)>((KS & 1) ? qb1 : qb0);
        });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    auto zero_o = []() {
        static_for<128>([&](auto i_c) {
            asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(i_c)::value) : FA_CLOB_O);
        });
    };

    // ---- LDS-DMA of K / V tiles (as fa_fwd_kernel): 16 x 1 KiB pieces per tile, 4 per wave
    int dma_src[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int b = (wid * 4 + i) * 1024 + lane * 16;
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        dma_src[i] = row * ROWB + ch * 16;
    }
    auto dma_tile = [&](const unsigned short* base, char* slot, int t) {
        const int rem = nkv - t * kBK;
        const int valid = __builtin_amdgcn_readfirstlane(rem < kBK ? (rem > 0 ? rem : 0) : kBK);
        const __amdgpu_buffer_rsrc_t rs = make_rsrc32((const char*)base + (int64_t)t * TILEB, valid * ROWB);
#pragma unroll
        for (int i = 0; i < 4; ++i) dma16(rs, slot + (wid * 4 + i) * 1024, dma_src[i], 0);
    };

    // ---- K fragment reads (asm, into a[192:255]).  Lane address of fragment (b2, ks):
    // lds_off(32*b2 + l32, 2*ks + hf) = kb{ks&1} + 8192*b2 + 512*(ks>>1), two bases.
    const int xr = (l32 >> 2) & 3;
    const unsigned kb0 = (unsigned)(size_t)kring + (l32 >> 3) * 8 * ROWB + 64 * (l32 & 7) + 16 * (hf ^ xr);
    const unsigned kb1 = (unsigned)(size_t)kring + (l32 >> 3) * 8 * ROWB + 64 * (l32 & 7) + 16 * ((hf ^ xr) ^ 2);
    auto read_k_group = [](auto slot_c, auto ks_c, unsigned kb0, unsigned kb1) {
        constexpr int SLOT = decltype(slot_c)::value, KS = decltype(ks_c)::value;
        constexpr int OFF = SLOT * TILEB + 512 * (KS >> 1);
        constexpr int A0 = 192 + 4 * KS, A1 = 192 + 4 * (8 + KS);  // b2 = 0, 1
        const unsigned base = (KS & 1) ? kb1 : kb0;
        asm volatile("ds_read_b128 a[%c1:%c2], %0 offset:%3" :: "v"(base), "i"(A0), "i"(A0 + 3), "i"(OFF)
                     : "memory", FA_CLOB_K);
        asm volatile("ds_read_b128 a[%c1:%c2], %0 offset:%3" :: "v"(base), "i"(A1), "i"(A1 + 3), "i"(OFF + 8192)
                     : "memory", FA_CLOB_K);
    };

    // ---- V^T fragment reads (as fa_fwd_kernel, V ring base in the address registers)
    const int grp = lane >> 4, gi = lane & 15;
    const int tr_row = 4 * (grp >> 1) + (gi >> 2);
    const int tr_col = 16 * (grp & 1) + 4 * (gi & 3);
    const unsigned vb0 = (unsigned)(size_t)vring + lds_off<D>(tr_row, tr_col >> 3) + (tr_col & 7) * 2;
    const unsigned vb1 = (unsigned)(size_t)vring + lds_off<D>(tr_row + 8, tr_col >> 3) + (tr_col & 7) * 2 - 8 * ROWB;
    auto read_v = [](auto slot_c, auto i_c, u32x2 (&vf)[2][2], unsigned vb0, unsigned vb1) {
        constexpr int SLOT = decltype(slot_c)::value, I = decltype(i_c)::value;
        constexpr int B2 = I / 4, DB = I % 4;
        constexpr int OFF = SLOT * TILEB + 4 * B2 * 8 * ROWB + 512 * DB;
        constexpr int SSO = 2 * 8 * ROWB;
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[0][0]) : "v"(vb0), "i"(OFF) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[0][1]) : "v"(vb1), "i"(OFF + 8 * ROWB) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[1][0]) : "v"(vb0), "i"(OFF + SSO) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(vf[1][1]) : "v"(vb1), "i"(OFF + SSO + 8 * ROWB) : "memory");
    };

    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
    const float c = a.scale_log2;

    // S^T(tile in slot SLOT) for both row blocks into s[rb][b2]; K reads FA_W64_KREADS_AHEAD
    // k-steps ahead of the MFMAs, each wait counts only the reads still allowed in flight.
    auto qk_tile = [&](auto slot_c, f32x16 (&s)[2][2]) {
        constexpr int AH = FA_W64_KREADS_AHEAD;
        static_for<AH>([&](auto ks_c) { read_k_group(slot_c, ks_c, kb0, kb1); });
        static_for<8>([&](auto ks_c) {
            constexpr int KS = decltype(ks_c)::value;
            // reads issued so far: 2*min(8, AH + KS); those of k-step KS must have landed
            constexpr int ISSUED = 2 * (AH + KS < 8 ? AH + KS : 8);
            constexpr int ALLOWED = ISSUED - 2 * (KS + 1);
            asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(ALLOWED) : "memory");
            constexpr int K0 = 192 + 4 * KS, K1 = 192 + 4 * (8 + KS);
            constexpr int Q0 = 128 + 4 * KS, Q1 = 128 + 4 * (8 + KS);
            if constexpr (KS == 0) {
                MO::template qk_first<K0, Q0>(s[0][0]);
                MO::template qk_first<K0, Q1>(s[1][0]);
                MO::template qk_first<K1, Q0>(s[0][1]);
                MO::template qk_first<K1, Q1>(s[1][1]);
            } else {
                MO::template qk<K0, Q0>(s[0][0]);
                MO::template qk<K0, Q1>(s[1][0]);
                MO::template qk<K1, Q0>(s[0][1]);
                MO::template qk<K1, Q1>(s[1][1]);
            }
            if constexpr (KS + AH < 8) read_k_group(slot_c, std::integral_constant<int, KS + AH>{}, kb0, kb1);
        });
    };
    // MFMA results -> VALU: wait states tied to the accumulators
    auto s_fence = [](f32x16 (&s)[2][2]) { mfma_fence(s); };
    // branch-free (selects): a branch here would split the pinned MFMA slots into basic
    // blocks that hipcc then rearranges
    auto mask = [&](int t, f32x16 (&s)[2][2]) {
        const int valid = nkv - t * kBK;
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool out = b2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf >= valid;
                s[0][b2][i] = out ? -INFINITY : s[0][b2][i];
                s[1][b2][i] = out ? -INFINITY : s[1][b2][i];
            }
    };
    auto rowmax = [&](const f32x16 (&s)[2][2], float (&mx)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            float m4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) m4[j] = s[rb][0][j];
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (b2 > 0 || i >= 4) m4[i & 3] = fmax_nc(m4[i & 3], s[rb][b2][i]);
            mx[rb] = pair_max(fmax_nc(fmax_nc(m4[0], m4[1]), fmax_nc(m4[2], m4[3]))) * c;
        }
    };
    // O block rows of row block RB *= alpha (rare: defer-max)
    auto rescale_o = [](auto rb_c, float alpha) {
        constexpr int RB = decltype(rb_c)::value;
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        static_for<64>([&](auto i_c) { agpr_scale<64 * RB + decltype(i_c)::value>(alpha); });
        asm volatile("s_nop 3" ::: "memory");
    };

    // One pipeline step for tile t (raw scores of tile t in sc, their row max in mx):
    //   QK^T(t+1) (32 MFMAs) with the exponentials of key block 0 (+8 of block 1), the K
    //   fragment reads and the DMA pieces of K(t+2) / V(t+1) between them;
    //   P.V(t) (32 MFMAs) with the remaining exponentials (first half) and the mask + row
    //   max of tile t+1 (second half) between them; then the barrier.
    // hipcc keeps VALU code where the source puts it between the volatile asm MFMAs (it
    // does not interleave them by itself: left alone it ran all 32 QK^T MFMAs back to back
    // and the softmax after them), so the interleave below IS the schedule.
    auto step = [&](auto par_c, auto flags_c, int t, f32x16 (&sc)[2][2], f32x16 (&sn)[2][2], float (&mx)[2]) {
        constexpr int P = decltype(par_c)::value;
        constexpr int F = decltype(flags_c)::value;
        constexpr bool MORE = F & 1, MASKNEXT = F & 2, DMAK = F & 4;
        if (__builtin_amdgcn_ballot_w64(mx[0] > m[0] + kThr)) {
            const float m_new = fmaxf(m[0], mx[0]);
            const float alpha = __builtin_amdgcn_exp2f(m[0] - m_new);
            // (first tile: O is still zero in every lane -- skip the 192-instruction rescale)
            const bool started = __builtin_amdgcn_ballot_w64(m[0] != -INFINITY) != 0;
            m[0] = m_new;
            l[0] *= alpha;
            if (started) rescale_o(std::integral_constant<int, 0>{}, alpha);
        }
        if (__builtin_amdgcn_ballot_w64(mx[1] > m[1] + kThr)) {
            const float m_new = fmaxf(m[1], mx[1]);
            const float alpha = __builtin_amdgcn_exp2f(m[1] - m_new);
            // (first tile: O is still zero in every lane -- skip the 192-instruction rescale)
            const bool started = __builtin_amdgcn_ballot_w64(m[1] != -INFINITY) != 0;
            m[1] = m_new;
            l[1] *= alpha;
            if (started) rescale_o(std::integral_constant<int, 1>{}, alpha);
        }
        const float nm[2] = {-m[0], -m[1]};
        float sum[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        u32x4 pb[2][4];
        // exponential of element E: key block B2 = E/32, row block RB = (E/16)%2, entry I = E%16;
        // the odd entry of a pair also packs the pair into P^T (k16 = 2*B2 + I/8)
        auto exp_elem = [&](auto e_c) {
            constexpr int E = decltype(e_c)::value, B2 = E / 32, RB = (E / 16) % 2, I = E % 16;
            const float x = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[RB][B2][I], c, nm[RB]));
            sc[RB][B2][I] = x;
            sum[RB][I & 3] += x;
            if constexpr (I & 1) pb[RB][2 * B2 + I / 8][(I & 7) / 2] = pack2<T>(sc[RB][B2][I - 1], x);
        };
        // DMA descriptors of K(t+2) and V(t+1); one 1 KiB piece issued per call
        auto tile_rsrc = [&](const unsigned short* base, int tt) {
            const int rem = nkv - tt * kBK;
            const int valid = __builtin_amdgcn_readfirstlane(rem < kBK ? (rem > 0 ? rem : 0) : kBK);
            return make_rsrc32((const char*)base + (int64_t)tt * TILEB, valid * ROWB);
        };
        // (t + 2 past the end only when !DMAK; its descriptor is then never used)
        const __amdgpu_buffer_rsrc_t krs = tile_rsrc(cur.k, DMAK ? t + 2 : t);
        const __amdgpu_buffer_rsrc_t vrs = tile_rsrc(cur.v, MORE ? t + 1 : t);

        // the next item's K(0) one step early: with an even tile count, K slot 0 is free
        // from the second-to-last step on
        if constexpr (FA_W64_KEARLY && MORE && !DMAK && P == 0) {
            if (item + (int)gridDim.x < nitems) dma_tile(nxt.k, kring, 0);
        }
        if constexpr (MORE) {
            constexpr int AH = FA_W64_KREADS_AHEAD;
            static_for<AH>([&](auto ks_c) { read_k_group(std::integral_constant<int, 1 - P>{}, ks_c, kb0, kb1); });
            static_for<32>([&](auto q_c) {
                constexpr int Q = decltype(q_c)::value, KS = Q / 4, SUB = Q % 4;
                if constexpr (SUB == 0) {
                    constexpr int ISSUED = 2 * (AH + KS < 8 ? AH + KS : 8);
                    asm volatile("s_waitcnt lgkmcnt(%0)" :: "i"(ISSUED - 2 * (KS + 1)) : "memory");
                }
                constexpr int K0 = 192 + 4 * KS, K1 = 192 + 4 * (8 + KS);
                constexpr int Q0 = 128 + 4 * KS, Q1 = 128 + 4 * (8 + KS);
                constexpr int KA = SUB < 2 ? K0 : K1, QA = (SUB & 1) ? Q1 : Q0;
                if constexpr (KS == 0) MO::template qk_first<KA, QA>(sn[SUB & 1][SUB >> 1]);
                else MO::template qk<KA, QA>(sn[SUB & 1][SUB >> 1]);
                exp_elem(std::integral_constant<int, Q>{});
                if constexpr (SUB == 3) {
                    exp_elem(std::integral_constant<int, 32 + KS>{});
                    if constexpr (KS + AH < 8)
                        read_k_group(std::integral_constant<int, 1 - P>{}, std::integral_constant<int, KS + AH>{}, kb0, kb1);
                }
                if constexpr (SUB == 1 && KS < 4 && DMAK)
                    dma16(krs, kring + P * TILEB + (wid * 4 + KS) * 1024, dma_src[KS], 0);
                if constexpr (SUB == 1 && KS >= 4)
                    dma16(vrs, vring + (1 - P) * TILEB + (wid * 4 + KS - 4) * 1024, dma_src[KS - 4], 0);
                if constexpr (FA_W64_PIN) __builtin_amdgcn_sched_barrier(0);  // keep the slot's fillers in it
            });
        } else {
            // last tile of the item: no K is read any more, so both K slots are free for the
            // next item's K(0), K(1); V(0) goes to V slot 0 if this tile's V is in slot 1.
            // Q^T of the next item replaces this one's (no QK^T in this step).
            if (item + (int)gridDim.x < nitems) {
                if (!(FA_W64_KEARLY && (ntiles & 1) == 0 && ntiles > 1)) dma_tile(nxt.k, kring, 0);
                if (ntiles > 1) dma_tile(nxt.k, kring + TILEB, 1);
                if constexpr (P == 1) dma_tile(nxt.v, vring, 0);
                if (!FA_W64_QLDS) load_q(nxt);
            }
            static_for<40>([&](auto e_c) { exp_elem(e_c); });
        }
        // nothing of the softmax may sink into the P.V slots below (VALU -> MFMA hazards)
        __builtin_amdgcn_sched_barrier(0);

        // P.V(t): fragment f = (b2, db) = (f/4, f%4) read one fragment ahead; MFMA p uses
        // k16 = 2*b2 + ss and row block rb, p = 16*b2 + 4*db + 2*ss + rb
        // V fragments double-buffered by fragment parity (no register copies: a VALU copy
        // right in front of an MFMA would be a VALU -> MFMA hazard)
        u32x2 vbuf[2][2][2];
        read_v(par_c, std::integral_constant<int, 0>{}, vbuf[0], vb0, vb1);
        lds_wait(vbuf[0]);
        float m4[2][4];
        static_for<32>([&](auto p_c) {
            constexpr int PP = decltype(p_c)::value, FR = PP / 4, B2 = PP / 16, DB = (PP / 4) % 4;
            constexpr int SS = (PP / 2) % 2, RB = PP % 2;
            if constexpr (PP % 4 == 0 && FR + 1 < 8)
                read_v(par_c, std::integral_constant<int, FR + 1>{}, vbuf[(FR + 1) & 1], vb0, vb1);
            const u32x2 (&vc)[2][2] = vbuf[FR & 1];
            const u32x4 vv = {vc[SS][0][0], vc[SS][0][1], vc[SS][1][0], vc[SS][1][1]};
            // (the last tile's softmax is one block ahead of the P.V slots and hipcc sinks
            // parts of it below its if (has_next) branch: pad those steps' MFMAs)
            MO::template pv<16 * (4 * RB + DB), FA_W64_PVNOP || !MORE || MASKNEXT>(vv, pb[RB][2 * B2 + SS]);
            // remaining exponentials (needed from p = 16 on): entries 48-55, 40-47, 56-63
            if constexpr (PP < 16) {
                constexpr int LEFT[24] = {48, 49, 50, 51, 52, 53, 54, 55, 40, 41, 42, 43,
                                          44, 45, 46, 47, 56, 57, 58, 59, 60, 61, 62, 63};
                constexpr int J0 = PP / 2 * 3 + (PP % 2) * 2;  // 2, 1, 2, 1, ... per MFMA
                exp_elem(std::integral_constant<int, LEFT[J0]>{});
                if constexpr (PP % 2 == 0) exp_elem(std::integral_constant<int, LEFT[J0 + 1]>{});
            }
            // mask + row max of tile t+1, 4 scores per MFMA (QK^T(t+1) issued >= 16 MFMAs ago)
            if constexpr (MORE && PP >= 16) {
                if constexpr (PP == 16) {
                    asm volatile("" : "+v"(sn[0][0]), "+v"(sn[0][1]), "+v"(sn[1][0]), "+v"(sn[1][1]));
                    if constexpr (MASKNEXT) mask(t + 1, sn);
                }
                constexpr int R = (PP - 16) / 8, G = (PP - 16) % 8, MB = G / 4, I0 = 4 * (G % 4);
                static_for<4>([&](auto j_c) {
                    constexpr int J = decltype(j_c)::value;
                    if constexpr (MB == 0 && I0 == 0) m4[R][J] = sn[R][0][J];
                    else m4[R][J] = fmax_nc(m4[R][J], sn[R][MB][I0 + J]);
                });
            }
            if constexpr (PP % 4 == 3 && FR + 1 < 8) lds_wait(vbuf[(FR + 1) & 1]);
            if constexpr (FA_W64_PIN) __builtin_amdgcn_sched_barrier(0);
        });
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) l[rb] += (sum[rb][0] + sum[rb][1]) + (sum[rb][2] + sum[rb][3]);
        if constexpr (MORE) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
                mx[rb] = pair_max(fmax_nc(fmax_nc(m4[rb][0], m4[rb][1]), fmax_nc(m4[rb][2], m4[rb][3]))) * c;
        }
        __syncthreads();  // drains the DMA (vmcnt(0)): K(t+2), V(t+1) landed
    };

    // ---- first item's prologue: K(0), V(0), K(1) -> LDS, Q^T -> AGPRs, O = 0
    dma_tile(cur.k, kring, 0);
    dma_tile(cur.v, vring, 0);
    if (ntiles > 1) dma_tile(cur.k, kring + TILEB, 1);
    load_q(cur);
    zero_o();
    f32x16 sa[2][2], sb[2][2];
    float mx[2];
    while (true) {
        const bool has_next = item + (int)gridDim.x < nitems;
        if (has_next) nxt = item_at(item + (int)gridDim.x);
        m[0] = m[1] = -INFINITY;
        l[0] = l[1] = 0.f;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Q^T (asm loads) and the tiles
        __syncthreads();
        qk_tile(std::integral_constant<int, 0>{}, sa);
        s_fence(sa);
        mask(0, sa);
        rowmax(sa, mx);
        if (FA_W64_QLDS && has_next) dma_q(nxt);  // the image was read at this item's start
        __syncthreads();  // K slot 0 is rewritten by step 0's DMA of K(2)
        {
            using C0 = std::integral_constant<int, 0>;
            using C1 = std::integral_constant<int, 1>;
            using STEADY = std::integral_constant<int, 1 | 4>;
            using NEXTLAST = std::integral_constant<int, 1 | 2>;
            using NEXTLASTK = std::integral_constant<int, 1 | 2 | 4>;
            using LAST = std::integral_constant<int, 0>;
            int t = 0;
            for (; t + 2 < ntiles; t += 2) {
                step(C0{}, STEADY{}, t, sa, sb, mx);
                step(C1{}, NEXTLASTK{}, t + 1, sb, sa, mx);
            }
            if (ntiles - t == 2) {
                step(C0{}, NEXTLAST{}, t, sa, sb, mx);
                step(C1{}, LAST{}, t + 1, sb, sa, mx);
            } else {
                step(C0{}, LAST{}, t, sa, sb, mx);
            }
        }

        // ---- epilogue: O (AGPRs) -> VGPRs -> 16-bit rows (dwordx4 stores after permlane32 swaps)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        static_for<2>([&](auto rb_c) {
            constexpr int RB = decltype(rb_c)::value;
            const int64_t q_row = cur.q_row0 + 32 * RB;
            const float inv = 1.f / pair_sum(l[RB]);
            f32x16 ov[4];
            static_for<64>([&](auto i_c) {
                constexpr int I = decltype(i_c)::value;
                ov[I / 16][I % 16] = agpr_read<64 * RB + I>();
            });
            if (q_row < a.Lq) {
                unsigned short* Oh = (unsigned short*)a.o + cur.bh * a.Lq * D + q_row * D;
#pragma unroll
                for (int db = 0; db < 4; ++db)
#pragma unroll
                    for (int gp = 0; gp < 4; gp += 2) {
                        unsigned x0 = pack2<T>(ov[db][4 * gp + 0] * inv, ov[db][4 * gp + 1] * inv);
                        unsigned x1 = pack2<T>(ov[db][4 * gp + 2] * inv, ov[db][4 * gp + 3] * inv);
                        unsigned y0 = pack2<T>(ov[db][4 * gp + 4] * inv, ov[db][4 * gp + 5] * inv);
                        unsigned y1 = pack2<T>(ov[db][4 * gp + 6] * inv, ov[db][4 * gp + 7] * inv);
                        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                        const u32x4 u = {s0[0], s1[0], s0[1], s1[1]};
                        *(u32x4*)(Oh + db * 32 + 8 * gp + 8 * hf) = u;
                    }
            }
        });
        if (!has_next) break;
        if (FA_W64_QLDS) read_q(qb0, qb1);  // landed long ago (every step's barrier waits vmcnt(0))
        zero_o();
        asm volatile("s_nop 3" ::: "memory");  // accvgpr_write -> MFMA SrcC
        // V(0) of the next item, unless the last tile already fetched it (even tile count)
        if ((ntiles & 1) == 1) dma_tile(nxt.v, vring, 0);
        item += (int)gridDim.x;
        cur = nxt;
    }
}

int w64_rows_per_block() { return 256; }

hipError_t launch_fwd_w64(Elem t, const FwdArgs& a0, hipStream_t s) {
    FwdArgs a = a0;
    a.nqt = (int)((a.Lq + 255) / 256);
    const int64_t nitems = (int64_t)a.nqt * a.BH;
    static int ncu = 0;  // one workgroup per CU (512 registers per lane, 64 KiB LDS)
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    // a multiple of 8 keeps every workgroup's items on its XCD (xcd_remap)
    int64_t grid = nitems < ncu ? nitems : (ncu & ~7 ? ncu & ~7 : ncu);
    const int lds = (4 + 4 * FA_W64_QLDS) * 64 * 128 * 2;  // K/V rings 64 KiB (+ Q images 64 KiB)
    if (t == Elem::BF16) hipLaunchKernelGGL((fa_fwd_w64_kernel<__bf16>), dim3((unsigned)grid), dim3(256), lds, s, a);
    else if (t == Elem::F16) hipLaunchKernelGGL((fa_fwd_w64_kernel<_Float16>), dim3((unsigned)grid), dim3(256), lds, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace fa
