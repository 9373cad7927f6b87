// fa_fwd_dtiled.hip -- the d-tiled FA-v1 forward for head dims past one LDS tile (d = 384, 512),
// bf16 / fp16 storage, fp32 accumulate, on v_mfma_f32_16x16x32.
//   <- flash_attention_kernel (tiled-d)   flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230
//   <- flash_attention_kernel_opt         flash_attention_v1_tiled_d/CUDA/flash_attention_v1_opt.h:366
//   (semantics: flash_attention_v1_tiled_d/numpy_basic.py:13-151)
//
// The reference's tiled-d variant exists so that d can exceed what one tile holds: S = Q K^T is
// accumulated over d_tile_qk-wide column chunks of K (mat_mul_chunk_accumulate, :57), P V over
// d_tile_v-wide column chunks of V (accumulate_output_chunk, :105), and O_acc lives in registers
// for all d columns (:270-272).  Here the same: per 64-key tile, the K tile streams through LDS
// in [64 keys][d_tile_qk] chunks, the V tile in [64 keys][d_tile_v] chunks, and O^T stays in
// VGPRs (d/4 registers per lane: 16 query rows per wave, so that d = 512 fits).
//
// Tiles are honoured at the MFMA's granularity: a chunk is 32, 64 or 128 columns (the
// requested d_tile rounded down to one of them, at least 32 -- a QK^T k-step is 32 columns, a
// P.V output block 16; 32 | 384 and 512), set by the C ABI (fa_capi.cpp dtile_eff) in
// FwdArgs::d_tile_qk / d_tile_v.  The chunking changes the schedule, not the sums: QK^T
// accumulates the same 32-column k-steps in the same order whatever the chunk, so outputs are
// bitwise equal across tile choices (tests/test_gpu.py::test_tiled_d_wide).
//
// Geometry (differs from the d <= 256 kernels, whose O^T block per wave is 32 x d):
//   * workgroup = 4 waves x 16 query rows = 64 rows; the 16 queries of a wave are the B (N)
//     side of S^T = K . Q^T on v_mfma_f32_16x16x32 (16 keys x 16 queries per MFMA, 4 per tile);
//   * Q^T fragments in registers for the whole loop (d/32 x 4 VGPRs: 64 at d = 512);
//   * a query's 64 scores of a tile sit in 4 lanes (n, n+16, n+32, n+48): row max by two
//     permlane swaps, row sums by a 16x16x32 MFMA with A = ones (as fa_fwd16_kernel.hpp);
//   * LDS: a ring of 16 KiB chunk images (the swizzled 8-row x 32-column subtile image of
//     fa_device.hpp, row = 2 * chunk bytes; 3 slots at d = 384, 4 at d = 512), filled by LDS-DMA
//     NSLOT-1 chunks ahead of use: the chunk stream K(t,0..) V(t,0..) K(t+1,0..) ... runs one
//     raw barrier per chunk, the DMA of the next chunk issued right after the barrier that
//     retires the previous chunk's slot;
//   * registers: d = 384 and 512 both fit 256 (two workgroups per CU: 224 / 246-256 VGPRs);
//   * d = 512 pairs the waves (PAIR, below): P^T shared through LDS, each wave's P.V on half of
//     d for both query blocks of its pair -- half the V^T reads per MFMA.
#include "fa_device.hpp"
#include "fa_dtiled_stream.hpp"

namespace fa {

constexpr int kDtWaves = 4;
constexpr int kDtRows = 16 * kDtWaves;  // query rows per workgroup
constexpr int kDtBK = 64;               // keys per tile
constexpr int kDtMaxChunk = 128;        // columns per LDS chunk at most
constexpr int kDtSlotB = kDtBK * kDtMaxChunk * 2;
// ring slots: two workgroups per CU (one wave per SIMD each), 3 / 4 x 16 KiB each; one workgroup
// per CU would take 8 slots -- 7 chunks in flight -- and measured slower (d = 512: 903 vs 672 us
// at B32 H8 L1024, profiles/r04/ab_dtiled_g.log)
#ifndef FA_DT384_WPS
#define FA_DT384_WPS 2  // waves per SIMD at d = 384 (2: two workgroups per CU)
#endif
#ifndef FA_DT512_WPS
#define FA_DT512_WPS 2  // waves per SIMD at d = 512 (2: 252 VGPRs, no scratch; 1: 8 ring slots)
#endif
constexpr int dt_wps(int d) { return d <= 384 ? FA_DT384_WPS : FA_DT512_WPS; }
// ring slots at two workgroups per CU: 3 at d = 384, 4 at d = 512 (A/B, profiles/r04/
// ab_dtiled_ring.txt: d = 384 3 / 4 / 5 slots 505 / 519 / 521 us, d = 512 690 / 668 / 682 us)
#ifndef FA_DT_SLOTS2
#define FA_DT_SLOTS2 0  // 0: the measured choice above; n: n slots at both head dims (A/B builds)
#endif
constexpr int dt_slots(int d) {
    return dt_wps(d) == 2 ? (FA_DT_SLOTS2 > 0 ? FA_DT_SLOTS2 : d <= 384 ? 3 : 4) : 8;
}

int dtiled_rows_per_block() { return kDtRows; }
// d = 512 runs the kernel's PAIR form: its wave pairs exchange P^T, alpha and the row sums
// through an area behind the ring
constexpr int kDtXchB = kDtWaves * 2048 + kDtWaves * 64 + 64;
constexpr bool dt_pshare(int d) { return d == 512; }
int dtiled_lds_bytes(int d) { return dt_slots(d) * kDtSlotB + (dt_pshare(d) ? kDtXchB : 0); }

// s_waitcnt vmcnt(N), N a compile-time count of DMA pieces allowed to stay in flight
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One 1 KiB LDS-DMA piece (buffer_load_dwordx4 ... lds; M0 = the wave's LDS destination), as
// inline asm so that the compiler does not see it: for a compiler-visible LDS-DMA it places an
// s_waitcnt vmcnt(0) -- every piece in flight -- before each ds_read_b64_tr_b16 builtin (it
// cannot tell the transposed read from a read of the bytes being written), which would drain
// the ring at every V chunk.  The ring's own vmcnt waits and barriers order the DMAs and the
// reads.  M0 carries no other value in these kernels (no LDS-DMA builtin, no movrel).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16_asm(__amdgpu_buffer_rsrc_t rs, const char* lds, int voff) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds);
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rs)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// PAIR (d = 512, round 6): waves 2p and 2p+1 form a pair over 32
// query rows.  Each still computes S = K Q^T and the online softmax for its own 16 rows, writes
// its packed P^T (and, when it rescaled, its alpha) to an LDS area behind the ring before the
// tile's first V chunk barrier, and after it reads its partner's: each wave then runs P.V for
// both query blocks of the pair on its own half of the head dim (h = wave & 1), so every V^T
// operand it reads from LDS feeds two MFMAs -- half the V^T reads per MFMA.  A V chunk image
// then holds DV/2 columns of each half (its DMA source offsets interleave them), so every wave
// has work in every chunk.  O^T: d/2 columns x 32 rows per wave, the same register count; the
// partner's row sums come through LDS once at the end.  The same sums in the same order: bitwise
// the unpaired output.  A/B (profiles/r06/ab_d512_dtp*.txt): d = 512 B32 H8 L1024 651.6 ->
// 629.3 us, B4 H8 L4096 1145 -> 1084 us; d = 384 495.9 / 495.7 us (equal: unpaired there).
template <typename T, int D, int DQ, int DV>
__global__ __launch_bounds__(256, dt_wps(D)) void fa_fwd_dt_kernel(FwdArgs a) {
    using M = Mma<T>;
    using v8 = typename M::v8;
    static_assert(D % 128 == 0 && D > 256 && D <= 512, "d-tiled kernel: d = 384 or 512");
    constexpr bool PAIR = dt_pshare(D);
    static_assert(!PAIR || kDtWaves == 4, "wave pairs (0, 1), (2, 3)");
    constexpr int NKS = D / 32;  // QK^T k-steps
    constexpr int NDB = D / 16;  // O^T column blocks
    constexpr int NDH = NDB / 2;  // ... of one half (PAIR)
    constexpr int NKB = 4;       // 16-key blocks per tile
    constexpr int ROWD = 2 * D;  // bytes per global row
    constexpr int NSLOT = dt_slots(D);

    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = w % a.nqt;
    const int64_t bh = w / a.nqt;  // final mode: one split
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n16 = lane & 15, g = lane >> 4;
    const int nkv = (int)a.Lk;
    const int ntiles = (nkv + kDtBK - 1) / kDtBK;

    // chunk geometry (effective tiles: 32, 64 or 128 columns, dividing D; one instantiation
    // per pair, so every chunk boundary and every DMA count below is a compile-time constant)
#ifndef FA_DT_GROUP
#define FA_DT_GROUP 1  // 2: chunks made readable in pairs, one barrier per pair (4 slots)
#endif
    using S = DtStream<D, DQ, DV, NSLOT, PAIR ? 1 : FA_DT_GROUP>;
    constexpr int nqc = S::NQC, per_tile = S::PER_TILE;
    constexpr int kpc = DQ / 32;          // QK^T k-steps per K chunk
    constexpr int bpc = DV / 16;          // O^T column blocks per V chunk
    constexpr int bph = bpc / 2;          // ... of each half (PAIR)
    constexpr int rowq = 2 * DQ, rowv = 2 * DV;  // LDS image row bytes
    const int total = ntiles * per_tile;

    // Q^T fragments (B operand): lane (g, n) holds Q[16*wid + n][32*ks + 8*pg .. +7], the
    // 8-column chunk permuted over the lane groups as in fa_fwd16_kernel.hpp (A and B agree)
    const int pg = (0x2130 >> (4 * g)) & 3;
    const int64_t q_tile0 = (int64_t)qt * kDtRows;
    const unsigned short* Qh = (const unsigned short*)a.q + bh * a.Lq * D + q_tile0 * D;
    const int64_t q_rows = a.Lq - q_tile0 < kDtRows ? a.Lq - q_tile0 : kDtRows;
    const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Qh, q_rows * ROWD);
    v8 qf[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
        qf[ks] = __builtin_bit_cast(
            v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, (wid * 16 + n16) * ROWD + ks * 64 + pg * 16, 0, 0));

    const char* const kbase = (const char*)a.k + bh * a.Lk * ROWD;
    const char* const vbase = (const char*)a.v + bh * a.Lk * ROWD;

    // LDS-DMA source offsets of this lane's pieces of a chunk image: destination byte b of the
    // image (rows of `rowb` bytes, swizzled subtiles) <- source row / 16-byte chunk; PAIR: a V
    // image's columns past DV/2 come from the second half of d (D/2 - DV/2 further)
    auto src_off = [&](int piece, int rowb, bool isv) {
        const int b = piece * 1024 + lane * 16;
        const int rg = b / (8 * rowb), rem = b % (8 * rowb);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        return row * ROWD + ch * 16 + (PAIR && isv && 8 * ch >= DV / 2 ? D - DV : 0);
    };
    constexpr int kpw = S::KPW, vpw = S::VPW;  // pieces per wave of a K / V chunk (1, 2 or 4)
    int ksrc[kpw], vsrc[vpw];
#pragma unroll
    for (int p = 0; p < kpw; ++p) ksrc[p] = src_off(wid * kpw + p, rowq, false);
#pragma unroll
    for (int p = 0; p < vpw; ++p) vsrc[p] = src_off(wid * vpw + p, rowv, true);
    // The chunk stream K(t, 0..) V(t, 0..) K(t+1, 0..) ... through an NSLOT ring, NSLOT-1 chunks
    // ahead of use.  Chunk gi = t * per_tile + pos sits in slot gi % NSLOT (`cslot`, carried as
    // it advances); pos is static at every use, so is the chunk's kind and column offset.
    auto issue = [&](auto pos_c, int it, int islot) {
        constexpr int pos = decltype(pos_c)::value;
        constexpr bool isk = pos < nqc;
        constexpr int c = isk ? pos : pos - nqc, dt = isk ? DQ : DV;
        const int valid = nkv - it * kDtBK < kDtBK ? nkv - it * kDtBK : kDtBK;
        // rows past the last key read zeros (the range ends at the last valid row's chunk);
        // PAIR: V chunk c starts at column c * DV/2 and reaches D/2 + DV/2 columns further
        constexpr bool split = PAIR && !isk;
        const __amdgpu_buffer_rsrc_t rs = make_rsrc32(
            (isk ? kbase : vbase) + (int64_t)it * kDtBK * ROWD + (split ? c * dt : c * 2 * dt),
            (valid - 1) * ROWD + (split ? D + dt : 2 * dt));
        char* const slot = smem + islot * kDtSlotB;
        constexpr int pw = isk ? kpw : vpw;
#pragma unroll
        for (int p = 0; p < pw; ++p) dma16_asm(rs, slot + (wid * pw + p) * 1024, isk ? ksrc[p] : vsrc[p]);
    };
    // chunk gi = t * per_tile + pos (the next to consume) becomes readable: its pieces landed
    // (the protocol of fa_dtiled_stream.hpp: a counted wait, a barrier after which every wave is
    // done with the slots being refilled, the next chunk(s) issued into them)
    int cslot = 0;
    auto advance = [&](auto pos_c, int t) {
        constexpr int pos = decltype(pos_c)::value;
        if constexpr (S::syncs(pos)) {
            const int gi = t * per_tile + pos;
            if (S::steady(gi, total))
                wait_vm<S::after(pos)>();
            else
                wait_vm<0>();
            // the barrier as inline asm with a memory clobber: no memory operation (the next DMA
            // into a retired slot above all) may be moved across it, and no drain is implied
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            static_for<S::GRP>([&](auto j_c) {
                constexpr int j = decltype(j_c)::value, np = pos + S::LEAD + j;
                if (gi + S::LEAD + j < total)
                    issue(std::integral_constant<int, np % per_tile>{}, t + np / per_tile,
                          S::slot_after(cslot, S::LEAD + j));
            });
        }
        const char* const slot = smem + cslot * kDtSlotB;
        cslot = cslot == NSLOT - 1 ? 0 : cslot + 1;
        return slot;
    };

    // LDS read geometry (fa_fwd16_kernel.hpp): K rows read in the order rho(n), V^T by
    // transposed reads of the 4 keys at rows R0(g) + (n >> 2) (+16)
    const int rho = 8 * ((n16 >> 2) & 1) + 4 * (n16 >> 3) + (n16 & 3);
    const unsigned kl = (rho >> 3) * (8 * rowq) + 64 * (rho & 7) + 16 * (pg ^ ((rho >> 2) & 3));
    const int r0 = 8 * (g & 1) + 4 * (g >> 1) + (n16 >> 2);
    const int sw = (r0 >> 2) & 3, c0 = (n16 >> 1) & 1;
    const unsigned vrow = (r0 >> 3) * (8 * rowv) + 64 * (r0 & 7) + 8 * (n16 & 1);
    const unsigned vl_e = vrow + 16 * (c0 ^ sw), vl_o = vrow + 16 * ((2 + c0) ^ sw);
    const int R0 = 8 * (g & 1) + 4 * (g >> 1);  // this lane's first key of each 16-key block

    // O^T: unpaired, all D columns of the wave's rows; PAIR, the wave's half of the columns for
    // its own rows (o) and its partner's (op)
    f32x4 o[PAIR ? NDH : NDB], op[PAIR ? NDH : 1];
#pragma unroll
    for (int db = 0; db < (PAIR ? NDH : NDB); ++db) o[db] = f32x4{};
#pragma unroll
    for (int db = 0; db < (PAIR ? NDH : 1); ++db) op[db] = f32x4{};
    f32x4 rs = f32x4{};
    float m = -INFINITY;
    v8 ones;
    {
        constexpr unsigned kOne = std::is_same_v<T, __bf16> ? 0x3F80u : 0x3C00u;
        ones = __builtin_bit_cast(v8, u32x4{kOne | (kOne << 16), kOne | (kOne << 16), kOne | (kOne << 16),
                                            kOne | (kOne << 16)});
    }
    const float c = a.scale_log2;
    // PAIR's exchange area behind the ring: per wave P^T [2 key steps][64 lanes] x 16 B, alpha
    // (and at the end l) per query, a rescale flag
    const int hh = wid & 1, pw = wid ^ 1;  // (PAIR) column half / own query block; partner wave
    char* const xch = smem + NSLOT * kDtSlotB;
    auto xp = [&](int wv, int kk) { return (u32x4*)(xch + wv * 2048 + kk * 1024) + lane; };
    float* const xa = (float*)(xch + kDtWaves * 2048);                 // [wave][16 queries]
    int* const xf = (int*)(xch + kDtWaves * 2048 + kDtWaves * 64);  // [wave]

    // K fragments of one k-step (4 key blocks) / V^T operands of one column block (2 key
    // steps x 2 reads), as compiler-visible LDS loads: the compiler places the lgkmcnt waits and
    // may issue the reads of later k-steps of a chunk ahead of earlier MFMAs (it inserts no
    // vmcnt wait for the LDS-DMA -- the ring's own waits and barriers order those, and the
    // barrier's memory clobber keeps every read between its chunk's two barriers).  (Round 4's
    // first build used asm reads, each group waited right behind its issue: a read issued ahead
    // had let the compiler copy its not-yet-written register -- wrong results at d = 384; the
    // exposed latency then cost 15 k cycles per 64-key step at d = 512.)
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    auto kread = [](u32x4 (&kf)[NKB], const char* base, int rowq_) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) kf[kb] = *(const u32x4*)(base + kb * 16 * rowq_);
    };
    auto vread = [](u32x2 (&vf)[4], const char* vb, int rowv_) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            vf[2 * kk] = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                       (lds_s16x4*)(vb + kk * 32 * rowv_)));
            vf[2 * kk + 1] = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                           (lds_s16x4*)(vb + kk * 32 * rowv_ + 16 * rowv_)));
        }
    };

    // The first S::FILL chunks (positions and tiles static; total >= per_tile >= FILL): chunk 0,
    // then a fence that has the compiler wait for Q (vmcnt(0): it counts only the Q loads, and
    // chunk 0 went out before them), then the rest in flight.  Without the fence the compiler
    // places a wait for Q before each k-step's first MFMA, inside the loop, where its counts
    // would drain the ring.
    issue(std::integral_constant<int, 0>{}, 0, 0);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" : "+v"(qf[ks]));
    static_for<S::FILL - 1>([&](auto i_c) {
        constexpr int i = decltype(i_c)::value + 1;
        issue(std::integral_constant<int, i>{}, 0, i);
    });
    const char* slot = smem;
    for (int t = 0; t < ntiles; ++t) {
        // ---- S^T = K Q^T over the d_tile_qk chunks of K
        f32x4 s[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) s[kb] = f32x4{};
        static_for<NKS>([&](auto ks_c) {
            constexpr int ks = decltype(ks_c)::value;
            if constexpr (ks % kpc == 0) slot = advance(std::integral_constant<int, ks / kpc>{}, t);
            u32x4 kf[NKB];
            kread(kf, slot + kl + (ks % kpc) * 512, rowq);
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) s[kb] = M::mma16(__builtin_bit_cast(v8, kf[kb]), qf[ks], s[kb]);
        });
        // keys past the end (last tile only): score -inf
        if (nkv - t * kDtBK < kDtBK) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (t * kDtBK + 16 * kb + R0 + i >= nkv) s[kb][i] = -INFINITY;
        }
        // ---- online softmax (base 2): row max over the 4 lanes of a query, rescale, P
        float mx = fmax_nc(fmax_nc(s[0][0], s[0][1]), fmax_nc(s[0][2], s[0][3]));
#pragma unroll
        for (int kb = 1; kb < NKB; ++kb)
            mx = fmax_nc(mx, fmax_nc(fmax_nc(s[kb][0], s[kb][1]), fmax_nc(s[kb][2], s[kb][3])));
        {
            auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
            const float y = fmax_nc(__uint_as_float(r[0]), __uint_as_float(r[1]));
            auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
            mx = fmax_nc(__uint_as_float(q[0]), __uint_as_float(q[1]));
        }
        const float m_new = fmaxf(m, mx * c);
        if constexpr (PAIR) {
            const int resc = __builtin_amdgcn_ballot_w64(m_new > m) != 0;
            if (resc) {
                const float alpha = __builtin_amdgcn_exp2f(m - m_new);  // 0 on the first tile
                rs *= alpha;
#pragma unroll
                for (int db = 0; db < NDH; ++db) o[db] *= alpha;
                m = m_new;
                if (g == 0) xa[wid * 16 + n16] = alpha;
            }
            if (lane == 0) xf[wid] = resc;
        } else {
            if (__builtin_amdgcn_ballot_w64(m_new > m)) {
                const float alpha = __builtin_amdgcn_exp2f(m - m_new);  // 0 on the first tile
                rs *= alpha;
#pragma unroll
                for (int db = 0; db < NDB; ++db) o[db] *= alpha;
                m = m_new;
            }
        }
        u32x4 pbu[2];  // P^T fragments of the two 32-key k-steps (k-order as fa_fwd16_kernel)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kb = 2 * kk + (j >> 1), i = 2 * (j & 1);
                pbu[kk][j] = pack2<T>(__builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][i], c, -m)),
                                      __builtin_amdgcn_exp2f(__builtin_fmaf(s[kb][i + 1], c, -m)));
            }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            rs = M::mma16(ones, __builtin_bit_cast(v8, pbu[kk]), rs);
            if constexpr (PAIR) *xp(wid, kk) = pbu[kk];
        }

        // ---- O^T += V^T P^T over the d_tile_v chunks of V
        if constexpr (PAIR) {
            // both query blocks of the pair, this wave's half of the columns: local column block
            // b is image block hh * bph + b % bph of chunk b / bph
            u32x4 pbp[2];
            static_for<NDH>([&](auto b_c) {
                constexpr int b = decltype(b_c)::value;
                constexpr int cch = b / bph, j = b % bph;
                if constexpr (j == 0) slot = advance(std::integral_constant<int, nqc + cch>{}, t);
                if constexpr (b == 0) {
                    // the partner's P^T and (if it rescaled) its alpha, written before this barrier
                    pbp[0] = *xp(pw, 0);
                    pbp[1] = *xp(pw, 1);
                    if (__builtin_amdgcn_readfirstlane(xf[pw])) {
                        const float ap = xa[pw * 16 + n16];
#pragma unroll
                        for (int db = 0; db < NDH; ++db) op[db] *= ap;
                    }
                }
                const int jj = hh * bph + j;
                u32x2 vf[4];
                vread(vf, slot + ((jj & 1) ? vl_o : vl_e) + 512 * (jj >> 1), rowv);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    const u32x4 vv = {vf[2 * kk][0], vf[2 * kk][1], vf[2 * kk + 1][0], vf[2 * kk + 1][1]};
                    o[b] = M::mma16(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbu[kk]), o[b]);
                    op[b] = M::mma16(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbp[kk]), op[b]);
                }
            });
        } else {
            static_for<NDB>([&](auto db_c) {
                constexpr int db = decltype(db_c)::value;
                if constexpr (db % bpc == 0) slot = advance(std::integral_constant<int, nqc + db / bpc>{}, t);
                u32x2 vf[4];
                vread(vf, slot + ((db & 1) ? vl_o : vl_e) + 512 * ((db % bpc) >> 1), rowv);
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    const u32x4 vv = {vf[2 * kk][0], vf[2 * kk][1], vf[2 * kk + 1][0], vf[2 * kk + 1][1]};
                    o[db] = M::mma16(__builtin_bit_cast(v8, vv), __builtin_bit_cast(v8, pbu[kk]), o[db]);
                }
            });
        }
    }

    // ---- epilogue: lane (g, n) holds O^T[16*db + 4*g + i][query n]; dv blocks 2e and 2e+1 are
    // paired by v_permlane16_swap into one 16-byte store per lane (fa_fwd16_kernel.hpp)
    auto store_rows = [&](const auto& v, int rw, float inv, int col0) {
        constexpr int nb = std::extent_v<std::remove_reference_t<decltype(v)>>;
        const int64_t q_row = q_tile0 + rw * 16 + n16;
        if (q_row >= a.Lq) return;
        unsigned short* const Oh = (unsigned short*)a.o + (bh * a.Lq + q_row) * D + col0;
#pragma unroll
        for (int e = 0; e < nb / 2; ++e) {
            const unsigned x0 = pack2<T>(v[2 * e][0] * inv, v[2 * e][1] * inv);
            const unsigned x1 = pack2<T>(v[2 * e][2] * inv, v[2 * e][3] * inv);
            const unsigned y0 = pack2<T>(v[2 * e + 1][0] * inv, v[2 * e + 1][1] * inv);
            const unsigned y1 = pack2<T>(v[2 * e + 1][2] * inv, v[2 * e + 1][3] * inv);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
            const u32x4 u = {s0[0], s1[0], s0[1], s1[1]};
            *(u32x4*)(Oh + 32 * e + 16 * (g & 1) + 8 * (g >> 1)) = u;
        }
    };
    if constexpr (PAIR) {
        // the partner's row sums (every wave done with the last tile's alpha first)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g == 0) xa[wid * 16 + n16] = rs[0];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const float lp = xa[pw * 16 + n16];
        store_rows(o, wid, 1.f / rs[0], hh * (D / 2));
        store_rows(op, pw, 1.f / lp, hh * (D / 2));
    } else {
        store_rows(o, wid, 1.f / rs[0], 0);
    }
}

// the kernel geometry the C ABI reports for a wide head dim (fa_kernel_geometry)
void dtiled_geometry(Elem, int d, int* rows, int* threads, int* lds) {
    *rows = kDtRows;
    *threads = kDtWaves * 64;
    *lds = dtiled_lds_bytes(d);
}

template <typename T, int D>
static hipError_t launch_dt(const FwdArgs& a, const dim3& grid, int lds, hipStream_t s) {
    auto go = [&](auto kern) {
        note_kernel(dt_pshare(D) ? "fa_fwd_dt_kernel<paired>" : "fa_fwd_dt_kernel", grid.x);
        hipLaunchKernelGGL(kern, grid, dim3(kDtWaves * 64), lds, s, a);
        return hipGetLastError();
    };
    auto pick_v = [&](auto dq_c) -> hipError_t {
        constexpr int DQ = decltype(dq_c)::value;
        switch (a.d_tile_v) {
            case 32: return go(fa_fwd_dt_kernel<T, D, DQ, 32>);
            case 64: return go(fa_fwd_dt_kernel<T, D, DQ, 64>);
            case 128: return go(fa_fwd_dt_kernel<T, D, DQ, 128>);
        }
        return hipErrorInvalidValue;
    };
    switch (a.d_tile_qk) {
        case 32: return pick_v(std::integral_constant<int, 32>{});
        case 64: return pick_v(std::integral_constant<int, 64>{});
        case 128: return pick_v(std::integral_constant<int, 128>{});
    }
    return hipErrorInvalidValue;
}

hipError_t launch_fwd_dtiled(Elem t, int d, const FwdArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((int64_t)a.nqt * a.BH));
    const int lds = dtiled_lds_bytes(d);
    if (t == Elem::BF16) {
        if (d == 384) return launch_dt<__bf16, 384>(a, grid, lds, s);
        if (d == 512) return launch_dt<__bf16, 512>(a, grid, lds, s);
    } else if (t == Elem::F16) {
        if (d == 384) return launch_dt<_Float16, 384>(a, grid, lds, s);
        if (d == 512) return launch_dt<_Float16, 512>(a, grid, lds, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace fa
