// fa_fwd.hip -- flash-attention forward for MI355X (gfx950 / CDNA4).
//
// One kernel template serves the three reference kernel families:
//   final mode   (PARTIAL=false): FA-v1 fused / d-tiled forward
//                 <- flash_attention_kernel    flash_attention_v1/CUDA/flash_attention_v1.h:161
//                 <- flash_attention_kernel_opt1 flash_attention_v1/CUDA/flash_attention_v1_opt1.h:264
//                 <- flash_attention_kernel (tiled-d) flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230
//   partial mode (PARTIAL=true): FA-v2 split-KV partial kernel
//                 <- partial_attention_kernel  flash_attention_v2/CUDA/flash_attention_v2.h:243
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
//   * K and V tiles are register-staged (global_load_dwordx4 issued before the tile's
//     MFMAs, ds_write_b128 after them) into a double-buffered, XOR-swizzled LDS image
//     that is bank-conflict-free for both the row reads and the transposed reads.
//   * blockIdx is remapped so that all query tiles of one (b,h) land on one XCD and
//     share that head's K/V in the XCD's L2.
#include "fa_internal.hpp"

namespace fa {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct Mma;
template <> struct Mma<__bf16> {
    typedef __bf16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mma<_Float16> {
    typedef _Float16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

// LDS image of one [kBK][D] K or V tile: 8-row x 4-chunk (8 x 32 columns, 512 B)
// subtiles, subtile (row>>3, ch>>2) at (row>>3)*8*ROWB + 512*(ch>>2), and inside it row
// (row&7) at 64 B strides with the 16-byte chunk XOR-swizzled by (row>>2)&3.
// Bank analysis ("LDS image"): the ds_read_b128 row reads of the 32x32x16 A
// operand (16 distinct rows per lane group, one chunk) and the ds_read_b64_tr_b16
// transposed reads (4 consecutive rows x 4 chunks per 32-lane half) both touch 16
// distinct 16-byte bank slots -- conflict-free -- and both need only two base
// addresses per lane (every other read is base + an immediate).
template <int D>
__device__ __forceinline__ int lds_off(int row, int chunk) {
    return (row >> 3) * (8 * D * 2) + 512 * (chunk >> 2) + 64 * (row & 7) +
           16 * ((chunk & 3) ^ ((row >> 2) & 3));
}

// Bijective workgroup remap: blocks b and b+8 share an XCD (observed round-robin
// dispatch, speed only -- results never depend on it), so give each group of blocks
// with equal b % 8 a contiguous range of work items.
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ float pair_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <typename T> struct Pack;
template <> struct Pack<__bf16> { typedef __bf16 v2 __attribute__((ext_vector_type(2))); };
template <> struct Pack<_Float16> { typedef _Float16 v2 __attribute__((ext_vector_type(2))); };
typedef float f32x2 __attribute__((ext_vector_type(2)));

// two fp32 -> one dword of two 16-bit values (one v_cvt_pk_{bf16,f16}_f32, RNE)
template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a, b}, typename Pack<T>::v2));
}

// Buffer resource over [base, base + bytes): loads past the end return 0 (the hardware
// range check does the tail clamping, no per-lane address arithmetic in the KV loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                             (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff),
                                             0x00020000);
}

// One 16-byte-per-lane LDS-DMA piece: lane i's 16 bytes land at lds + 16*i.  Kept out of
// the kernel's lambdas: a builtin call inside a lambda made hipcc drop the kernel's host
// launch stub (undefined __device_stub__ at load time).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds, int voff, int soff) {
    typedef __attribute__((address_space(3))) void lds_void;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, voff, soff, 0, 0);
}

template <typename T, typename PT, int D, bool PARTIAL>
__global__ __launch_bounds__(kThreads, 2) void fa_fwd_kernel(FwdArgs a) {
    using M = Mma<T>;
    using v8 = typename M::v8;
    constexpr int ROWB = D * 2;               // bytes per LDS row
    constexpr int NCH = D / 8;                // 16-byte chunks per row
    constexpr int TILEB = kBK * ROWB;         // bytes of one K (or V) tile
    constexpr int NKS = D / 16;               // MFMA k-steps of Q K^T
    constexpr int NDB = D / 32;               // 32-column blocks of O
    // Deferred rescale (defer-max): the running max m is only moved when some row's tile
    // max exceeds it by more than kThr (log2 units), so most tiles skip the O *= alpha
    // pass; P is then bounded by 2^kThr instead of 1, well inside fp32/bf16 range.
    constexpr float kThr = 4.f;  // 8 costs accuracy on peaked rows (see tests)
    static_assert(kBK * NCH % kThreads == 0, "tile must split evenly over threads");

    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = w % a.nqt;
    const int rest = w / a.nqt;
    const int split = rest % a.nsplit;
    const int64_t bh = rest / a.nsplit;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int l32 = lane & 31;
    const int hf = lane >> 5;

    const int64_t kv_begin = (int64_t)split * a.kv_per_split;
    const int64_t kv_end = kv_begin + a.kv_per_split < a.Lk ? kv_begin + a.kv_per_split : a.Lk;
    const int ntiles = (int)((kv_end - kv_begin + kBK - 1) / kBK);

    // Buffer descriptors: K/V cover exactly this split's keys, so the staging loads of the
    // last (partial) tile read zeros past kv_end with no clamping code.
    const unsigned short* Qh = (const unsigned short*)a.q + bh * a.Lq * D;
    const __amdgpu_buffer_rsrc_t qrs = make_rsrc(Qh, a.Lq * ROWB);
    const __amdgpu_buffer_rsrc_t krs =
        make_rsrc((const unsigned short*)a.k + (bh * a.Lk + kv_begin) * D, (kv_end - kv_begin) * ROWB);
    const __amdgpu_buffer_rsrc_t vrs =
        make_rsrc((const unsigned short*)a.v + (bh * a.Lk + kv_begin) * D, (kv_end - kv_begin) * ROWB);

    // Q^T fragments (B operand): lane holds Q[row][16*ks + 8*hf + 0..7].  Rows past Lq
    // read zeros and are never stored.
    const int64_t q_row = (int64_t)qt * kBQ + wid * kRowsPerWave + l32;
    v8 qf[NKS];
    {
        const int qoff = (int)(q_row * ROWB) + hf * 16;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[ks] = __builtin_bit_cast(v8, __builtin_amdgcn_raw_buffer_load_b128(qrs, qoff + ks * 32, 0, 0));
    }

    // K/V tiles go HBM -> LDS by LDS-DMA (buffer_load ... lds): no staging VGPRs, no
    // ds_write pass.  One wave instruction writes 1 KiB of LDS lane-linearly (M0 base +
    // 16*lane), so the swizzled image is produced by giving each lane the SOURCE chunk
    // that lds_off() places at its destination byte.  Out-of-range lanes of the last,
    // partial tile read zeros (buffer range check).
    constexpr int NDMA = TILEB / 1024;              // 1 KiB pieces per tile and operand
    constexpr int DPW = NDMA / kWaves;              // pieces per wave
    static_assert(NDMA % kWaves == 0, "tile pieces must split evenly over waves");
    int dma_src[DPW];
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
        const int b = (wid * DPW + i) * 1024 + lane * 16;  // destination byte in the tile image
        const int rg = b / (8 * ROWB), rem = b % (8 * ROWB);
        const int row = 8 * rg + (rem % 512) / 64;
        const int ch = 4 * (rem / 512) + (((rem % 64) / 16) ^ ((row >> 2) & 3));
        dma_src[i] = row * ROWB + ch * 16;
    }
    auto stage = [&](int t, int buf) {
        char* kb = smem + buf * 2 * TILEB + wid * DPW * 1024;
        char* vb = kb + TILEB;
        const int soff = t * TILEB;
#pragma unroll
        for (int i = 0; i < DPW; ++i) {
            dma16(krs, kb + i * 1024, dma_src[i], soff);
            dma16(vrs, vb + i * 1024, dma_src[i], soff);
        }
    };

    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; ++db) o[db] = f32x16{};
    float m = -INFINITY;  // reference max of the row, in log2 units (scores * scale_log2)
    float l = 0.f;        // this lane's half of the running denominator
    const float c = a.scale_log2;

    // transposed-read geometry (constant per lane)
    const int grp = lane >> 4, gi = lane & 15;
    const int tr_row = 4 * (grp >> 1) + (gi >> 2);
    const int tr_col = 16 * (grp & 1) + 4 * (gi & 3);

    stage(0, 0);
    // Make the Q fragments' loads retire here: otherwise hipcc's waitcnt pass carries them
    // as pending into the loop header and, merging that state with the back edge, puts
    // vmcnt(7..0) waits in front of every QK^T MFMA -- draining the next tile's prefetch
    // on every iteration.
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]));
    __syncthreads();

    for (int t = 0; t < ntiles; ++t) {
        const bool has_next = t + 1 < ntiles;
        if (has_next) stage(t + 1, (t + 1) & 1);  // lands under this tile's MFMAs
        const char* kb = smem + (t & 1) * 2 * TILEB;
        const char* vb = kb + TILEB;

        // S^T[key][q] for 2 blocks of 32 keys
        // All K fragments of the tile are read up front (lgkmcnt-counted), so the MFMA
        // chain waits for each read only once instead of read -> wait -> MFMA serially.
        f32x16 s[2];
        v8 kf[2][NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
                kf[b2][ks] = *(const v8*)(kb + lds_off<D>(b2 * 32 + l32, 2 * ks + hf));
        s[0] = f32x16{};
        s[1] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2) s[b2] = M::mma(kf[b2][ks], qf[ks], s[b2]);
        // keep hipcc from sinking each read next to its MFMA: reads first, then the chain
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * NKS, 0);  // DS_READ
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NKS, 0);  // MFMA

        // V^T fragments of one 32-column O block: 8 transposed reads (4 keys each); the
        // A operand's element j must be the same key as pb's element j (see below).
        // Issued as inline asm: hipcc cannot prove the builtin form disjoint from the
        // in-flight LDS-DMA into the other buffer and would put vmcnt(0) -- a full drain of
        // the next tile's prefetch -- in front of every one.  Their lgkmcnt is waited for
        // by vwait() below, which names every destination.
        auto read_v = [&](int db, u32x2 (&vf)[2][2][2]) {
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int row = b2 * 32 + 16 * ss + tr_row;
                    const int col = db * 32 + tr_col;
                    const int sub = (col & 7) * 2;  // 0 or 8 bytes inside the chunk
                    const unsigned a0 = (unsigned)(size_t)(vb + lds_off<D>(row, col >> 3) + sub);
                    const unsigned a1 = (unsigned)(size_t)(vb + lds_off<D>(row + 8, col >> 3) + sub);
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vf[b2][ss][0]) : "v"(a0) : "memory");
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vf[b2][ss][1]) : "v"(a1) : "memory");
                }
        };
        auto vwait = [&](u32x2 (&vf)[2][2][2]) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(vf[0][0][0]), "+v"(vf[0][0][1]), "+v"(vf[0][1][0]), "+v"(vf[0][1][1]),
                           "+v"(vf[1][0][0]), "+v"(vf[1][0][1]), "+v"(vf[1][1][0]), "+v"(vf[1][1][1]));
        };
        // block 0's V reads go out now and land under the softmax VALU work
        u32x2 vcur[2][2][2];
        read_v(0, vcur);

        // mask keys past the end of this split (only the last, partial tile)
        const int valid = (int)(kv_end - kv_begin) - t * kBK;
        if (valid < kBK) {
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int key = b2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
                    if (key >= valid) s[b2][r] = -INFINITY;
                }
        }

        // row max: 4 independent chains, then the lane pair (l, l+32)
        float mx4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) mx4[j] = fmaxf(s[j >> 1][8 * (j & 1)], s[j >> 1][8 * (j & 1) + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 2; r < 8; ++r) mx4[j] = fmaxf(mx4[j], s[j >> 1][8 * (j & 1) + r]);
        const float mx = pair_max(fmaxf(fmaxf(mx4[0], mx4[1]), fmaxf(mx4[2], mx4[3]))) * c;

        // deferred rescale: wave-uniform decision, taken before any P of this tile exists
        if (__builtin_amdgcn_ballot_w64(mx > m + kThr)) {
            const float m_new = fmaxf(m, mx);
            const float alpha = __builtin_amdgcn_exp2f(m - m_new);
            m = m_new;
            l *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; ++db) o[db] *= alpha;
        }

        float sum4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[b2][r], c, -m));
                s[b2][r] = p;
                sum4[(b2 * 16 + r) & 3] += p;
            }
        l += (sum4[0] + sum4[1]) + (sum4[2] + sum4[3]);

        // P^T packed to 16-bit: registers 8*ss .. 8*ss+7 of block b2 form the B operand
        // of k-step ss; its element j is key 16*ss + 8*(j>>2) + 4*hf + (j&3) of the block.
        v8 pb[2][2];
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                u32x4 u;
#pragma unroll
                for (int j = 0; j < 4; ++j) u[j] = pack2<T>(s[b2][8 * ss + 2 * j], s[b2][8 * ss + 2 * j + 1]);
                pb[b2][ss] = __builtin_bit_cast(v8, u);
            }

        // O^T[dv][q] += V^T[dv][key] . P^T[key][q], block db's MFMAs overlapping the
        // reads of block db+1.
        vwait(vcur);
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
            u32x2 vnext[2][2][2];
            if (db + 1 < NDB) read_v(db + 1, vnext);
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const u32x4 vv = {vcur[b2][ss][0][0], vcur[b2][ss][0][1], vcur[b2][ss][1][0],
                                      vcur[b2][ss][1][1]};
                    o[db] = M::mma(__builtin_bit_cast(v8, vv), pb[b2][ss], o[db]);
                }
            if (db + 1 < NDB) {
                vwait(vnext);
#pragma unroll
                for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                        for (int h = 0; h < 2; ++h) vcur[b2][ss][h] = vnext[b2][ss][h];
            }
        }

        __syncthreads();  // hipcc puts vmcnt(0) here: tile t+1's DMA has landed
    }

    // ---- epilogue: lane holds O^T[dv][q_row] for dv = 32*db + (r&3) + 8*(r>>2) + 4*hf
    const float l_tot = pair_sum(l);
    const float inv = 1.f / l_tot;
    if (q_row >= a.Lq) return;
    if constexpr (!PARTIAL) {
        unsigned short* Oh = (unsigned short*)a.o + bh * a.Lq * D + q_row * D;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                u32x2 u;
                u[0] = pack2<T>(o[db][4 * g4 + 0] * inv, o[db][4 * g4 + 1] * inv);
                u[1] = pack2<T>(o[db][4 * g4 + 2] * inv, o[db][4 * g4 + 3] * inv);
                *(u32x2*)(Oh + db * 32 + 8 * g4 + 4 * hf) = u;
            }
    } else {
        const int64_t chunk = q_row / a.chunk_rows, r_in = q_row % a.chunk_rows;
        const int64_t row_lin = chunk * a.BH * a.chunk_rows + bh * a.chunk_rows + r_in;
        PT* Op = (PT*)a.o + split * a.split_stride + row_lin * D;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int col = db * 32 + 8 * g4 + 4 * hf;
                if constexpr (sizeof(PT) == 4) {
                    f32x4 f = {o[db][4 * g4 + 0] * inv, o[db][4 * g4 + 1] * inv,
                               o[db][4 * g4 + 2] * inv, o[db][4 * g4 + 3] * inv};
                    *(f32x4*)(Op + col) = f;
                } else {
                    u32x2 u;
                    u[0] = pack2<T>(o[db][4 * g4 + 0] * inv, o[db][4 * g4 + 1] * inv);
                    u[1] = pack2<T>(o[db][4 * g4 + 2] * inv, o[db][4 * g4 + 3] * inv);
                    *(u32x2*)((unsigned short*)Op + col) = u;
                }
            }
        // lse in log2 units: m + log2(l)  (v_log_f32 is log2)
        if (hf == 0) a.lse[split * a.BH * a.Lq + row_lin] = m + __builtin_amdgcn_logf(l_tot);
    }
}

int fwd_lds_bytes(int d) { return 2 * 2 * kBK * d * 2; }

template <typename T, typename PT, int D, bool PARTIAL>
static hipError_t launch_one(const FwdArgs& a, hipStream_t s) {
    const int64_t nblk = (int64_t)a.nqt * a.nsplit * a.BH;
    const int lds = fwd_lds_bytes(D);
    hipLaunchKernelGGL((fa_fwd_kernel<T, PT, D, PARTIAL>), dim3((unsigned)nblk), dim3(kThreads),
                       lds, s, a);
    return hipGetLastError();
}

template <typename T, typename PT, bool PARTIAL>
static hipError_t launch_d(int d, const FwdArgs& a, hipStream_t s) {
    switch (d) {
        case 32: return launch_one<T, PT, 32, PARTIAL>(a, s);
        case 64: return launch_one<T, PT, 64, PARTIAL>(a, s);
        case 128: return launch_one<T, PT, 128, PARTIAL>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fwd(Elem t, Elem pt, int d, bool partial, const FwdArgs& a, hipStream_t s) {
    if (!partial) {
        if (t == Elem::BF16) return launch_d<__bf16, __bf16, false>(d, a, s);
        if (t == Elem::F16) return launch_d<_Float16, _Float16, false>(d, a, s);
        return hipErrorInvalidValue;
    }
    if (t == Elem::BF16 && pt == Elem::BF16) return launch_d<__bf16, __bf16, true>(d, a, s);
    if (t == Elem::BF16 && pt == Elem::F32) return launch_d<__bf16, float, true>(d, a, s);
    if (t == Elem::F16 && pt == Elem::F16) return launch_d<_Float16, _Float16, true>(d, a, s);
    if (t == Elem::F16 && pt == Elem::F32) return launch_d<_Float16, float, true>(d, a, s);
    return hipErrorInvalidValue;
}

}  // namespace fa
