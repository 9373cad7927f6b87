// fa_fwd64.hip -- fp64 precision mode of the forward: the reference's
// USE_FP64 build (DATA_TYPE double, flash_attention_v1/CUDA/flash_attention_v1.h:29-41),
// here on the fp64 matrix cores (v_mfma_f64_16x16x4_f64) for both contractions.
//
// Not the performance path -- the bf16/fp16 kernels in fa_fwd.hip are -- but a bit-tight
// statement of the same tiled online softmax: every product, sum and exponential in fp64,
// so its outputs match the fp64 oracle and the reference's fp64 golden vectors to ~1e-15.
//
// Geometry: workgroup = 4 waves x 16 query rows; KV tiles of 16 keys staged in LDS
// (padded rows), single-buffered.  Per wave and tile:
//   S[16 x 16] = Q K^T   -- d/4 MFMAs, A = Q (registers), B = K^T (LDS)
//   online softmax on S  -- row max / sum over the 16 lanes that share a row (shuffles)
//   O[16 x d] += P V     -- P transposed through LDS into the A layout, B = V (LDS)
// v_mfma_f64_16x16x4_f64 lane layout (probed on gfx950, scripts/probe_mfma_f64.hip):
//   A[i][k]: lane i + 16k;  B[k][j]: lane j + 16k;  D[i][j]: lane 16*(i%4) + j, reg i/4.
#include "fa_internal.hpp"

namespace fa {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kBQ64 = 64;  // query rows per workgroup (4 waves x 16)
constexpr int kBK64 = 16;  // keys per tile

__device__ __forceinline__ double row16_max(double x) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) x = fmax(x, __shfl_xor(x, o, 16));
    return x;
}
__device__ __forceinline__ double row16_sum(double x) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) x += __shfl_xor(x, o, 16);
    return x;
}

template <int D, int MODE>
__global__ __launch_bounds__(256, 1) void fa_fwd64_kernel(FwdArgs a) {
    constexpr int LD = D + 1;        // padded LDS row (doubles): conflict-free column reads
    constexpr int NKS = D / 4;       // MFMA k-steps of Q K^T
    constexpr int NDB = D / 16;      // 16-column blocks of O
    __shared__ double ks[kBK64 * LD];
    __shared__ double vs[kBK64 * LD];
    __shared__ double ps[4][16 * 17];

    const int qt = blockIdx.x % a.nqt;
    const int rest = blockIdx.x / a.nqt;
    const int split = rest % a.nsplit;
    const int64_t bh = rest / a.nsplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, j16 = lane & 15;  // D layout: rows g + 4r, column j16

    const int64_t kv_begin = (int64_t)split * a.kv_per_split;
    const int64_t kv_end = kv_begin + a.kv_per_split < a.Lk ? kv_begin + a.kv_per_split : a.Lk;
    const int nkv = (int)(kv_end - kv_begin);
    const double* Q = (const double*)a.q + bh * a.Lq * D;
    const double* K = (const double*)a.k + (bh * a.Lk + kv_begin) * D;
    const double* V = (const double*)a.v + (bh * a.Lk + kv_begin) * D;
    const double c = a.scale_log2_64;  // log2(e) / sqrt(d)

    // Q as A operand: lane holds Q[row0 + (lane & 15)][4s + (lane >> 4)], s = 0..NKS-1
    const int64_t row0 = (int64_t)qt * kBQ64 + wid * 16;
    double qf[NKS];
    {
        const int64_t qr = row0 + j16;
#pragma unroll
        for (int s = 0; s < NKS; ++s) qf[s] = qr < a.Lq ? Q[qr * D + 4 * s + g] : 0.0;
    }
    f64x4 o[NDB];
#pragma unroll
    for (int nb = 0; nb < NDB; ++nb) o[nb] = f64x4{0, 0, 0, 0};
    double m[4], l[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = -INFINITY;
        l[r] = 0.0;
    }

    const int ntiles = (nkv + kBK64 - 1) / kBK64;
    for (int t = 0; t < ntiles; ++t) {
        __syncthreads();  // previous tile's LDS reads done
        for (int e = tid; e < kBK64 * D; e += 256) {
            const int row = e / D, col = e % D;
            const bool in = t * kBK64 + row < nkv;
            ks[row * LD + col] = in ? K[(int64_t)(t * kBK64 + row) * D + col] : 0.0;
            vs[row * LD + col] = in ? V[(int64_t)(t * kBK64 + row) * D + col] : 0.0;
        }
        __syncthreads();

        // S = Q K^T (B[k][j] = K[j][4s + k]: lane j16 + 16g reads ks[j16][4s + g])
        f64x4 sacc = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < NKS; ++s)
            sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(qf[s], ks[j16 * LD + 4 * s + g], sacc, 0, 0, 0);

        // online softmax, rows g + 4r, this lane's key j16
        const bool key_ok = t * kBK64 + j16 < nkv;
        double p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double s2 = key_ok ? sacc[r] * c : -INFINITY;
            const double m_new = fmax(m[r], row16_max(s2));
            const double alpha = exp2(m[r] - m_new);
            p[r] = exp2(s2 - m_new);
            l[r] = l[r] * alpha + row16_sum(p[r]);
            m[r] = m_new;
#pragma unroll
            for (int nb = 0; nb < NDB; ++nb) o[nb][r] *= alpha;
        }
        // P (D layout) -> LDS -> A layout: A[i][k] = P[i][4u + k] at lane i + 16k
        double* pw = ps[wid];
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[(g + 4 * r) * 17 + j16] = p[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double pa[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pa[u] = pw[j16 * 17 + 4 * u + g];
        // O += P V (B[k][n] = V[4u + k][16nb + n]: lane n + 16k reads vs[4u + g][16nb + j16])
#pragma unroll
        for (int nb = 0; nb < NDB; ++nb)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                o[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[u], vs[(4 * u + g) * LD + 16 * nb + j16], o[nb],
                                                             0, 0, 0);
        __builtin_amdgcn_wave_barrier();  // ps is rewritten next tile
    }

    // epilogue: rows g + 4r, columns 16nb + j16
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t q_row = row0 + g + 4 * r;
        if (q_row >= a.Lq) continue;
        const double inv = 1.0 / l[r];
        if constexpr (MODE == kFinal) {
            double* Oh = (double*)a.o + (bh * a.Lq + q_row) * D;
#pragma unroll
            for (int nb = 0; nb < NDB; ++nb) Oh[16 * nb + j16] = o[nb][r] * inv;
        } else {
            const int64_t chunk = q_row / a.chunk_rows, r_in = q_row % a.chunk_rows;
            const int64_t row_lin = chunk * a.BH * a.chunk_rows + bh * a.chunk_rows + r_in;
            double* Op = (double*)a.o + split * a.split_stride + row_lin * D;
#pragma unroll
            for (int nb = 0; nb < NDB; ++nb) Op[16 * nb + j16] = o[nb][r] * inv;
            if (j16 == 0) a.lse64[split * a.BH * a.Lq + row_lin] = m[r] + log2(l[r]);
        }
    }
}

// fp64 d-tiled forward for d = 384 / 512 (the head dims past one tile; the reference's tiled-d
// kernel, flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:230-309, in its USE_FP64 build):
// per 16-key tile, S = Q K^T accumulated over d_tile_qk-wide column chunks of Q and K staged in
// LDS -- Q's chunk re-read for every KV tile, as the reference does (:159-164) -- then the
// online softmax, then O += P V over d_tile_v-wide column chunks of V; O stays in registers
// (d/4 doubles per lane).  Chunks: the effective tiles of FwdArgs (32, 64 or 128 columns).
constexpr int kDt64Chunk = 128;  // columns per LDS chunk at most

template <int D>
__global__ __launch_bounds__(256, 1) void fa_fwd64_dt_kernel(FwdArgs a) {
    constexpr int LD = kDt64Chunk + 1;  // padded LDS row (doubles)
    constexpr int NDB = D / 16;
    __shared__ double qs[kBQ64 * LD];
    __shared__ double ks[kBK64 * LD];
    __shared__ double vs[kBK64 * LD];
    __shared__ double ps[4][16 * 17];

    const int qt = blockIdx.x % a.nqt;
    const int64_t bh = blockIdx.x / a.nqt;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, j16 = lane & 15;
    const int nkv = (int)a.Lk;
    const int dq = a.d_tile_qk, dv = a.d_tile_v, nqc = D / dq, bpc = dv / 16;
    const double* Q = (const double*)a.q + bh * a.Lq * D;
    const double* K = (const double*)a.k + bh * a.Lk * D;
    const double* V = (const double*)a.v + bh * a.Lk * D;
    const double c = a.scale_log2_64;
    const int64_t qrow0 = (int64_t)qt * kBQ64;
    const int64_t row0 = qrow0 + wid * 16;

    f64x4 o[NDB];
#pragma unroll
    for (int nb = 0; nb < NDB; ++nb) o[nb] = f64x4{0, 0, 0, 0};
    double m[4], l[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = -INFINITY;
        l[r] = 0.0;
    }
    const int ntiles = (nkv + kBK64 - 1) / kBK64;
    for (int t = 0; t < ntiles; ++t) {
        // S = sum over the K chunks of Q_c K_c^T
        f64x4 sacc = {0, 0, 0, 0};
        for (int cq = 0; cq < nqc; ++cq) {
            __syncthreads();  // previous chunk's reads done
            for (int e = tid; e < kBQ64 * dq; e += 256) {
                const int row = e / dq, col = e % dq;
                qs[row * LD + col] = qrow0 + row < a.Lq ? Q[(qrow0 + row) * D + cq * dq + col] : 0.0;
            }
            for (int e = tid; e < kBK64 * dq; e += 256) {
                const int row = e / dq, col = e % dq;
                ks[row * LD + col] = t * kBK64 + row < nkv ? K[(int64_t)(t * kBK64 + row) * D + cq * dq + col] : 0.0;
            }
            __syncthreads();
            for (int s4 = 0; s4 < dq / 4; ++s4)
                sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(qs[(wid * 16 + j16) * LD + 4 * s4 + g],
                                                            ks[j16 * LD + 4 * s4 + g], sacc, 0, 0, 0);
        }
        const bool key_ok = t * kBK64 + j16 < nkv;
        double p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double s2 = key_ok ? sacc[r] * c : -INFINITY;
            const double m_new = fmax(m[r], row16_max(s2));
            const double alpha = exp2(m[r] - m_new);
            p[r] = exp2(s2 - m_new);
            l[r] = l[r] * alpha + row16_sum(p[r]);
            m[r] = m_new;
#pragma unroll
            for (int nb = 0; nb < NDB; ++nb) o[nb][r] *= alpha;
        }
        double* pw = ps[wid];
#pragma unroll
        for (int r = 0; r < 4; ++r) pw[(g + 4 * r) * 17 + j16] = p[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double pa[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pa[u] = pw[j16 * 17 + 4 * u + g];
        // O += P V over the V chunks (column blocks in order; a new chunk every bpc blocks)
#pragma unroll
        for (int nb = 0; nb < NDB; ++nb) {
            if (nb % bpc == 0) {
                __syncthreads();
                const int cv = nb / bpc;
                for (int e = tid; e < kBK64 * dv; e += 256) {
                    const int row = e / dv, col = e % dv;
                    vs[row * LD + col] =
                        t * kBK64 + row < nkv ? V[(int64_t)(t * kBK64 + row) * D + cv * dv + col] : 0.0;
                }
                __syncthreads();
            }
            const int nl = nb % bpc;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                o[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[u], vs[(4 * u + g) * LD + 16 * nl + j16], o[nb], 0, 0,
                                                             0);
        }
        __builtin_amdgcn_wave_barrier();  // ps is rewritten next tile
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t q_row = row0 + g + 4 * r;
        if (q_row >= a.Lq) continue;
        const double inv = 1.0 / l[r];
        double* Oh = (double*)a.o + (bh * a.Lq + q_row) * D;
#pragma unroll
        for (int nb = 0; nb < NDB; ++nb) Oh[16 * nb + j16] = o[nb][r] * inv;
    }
}

hipError_t launch_fwd64_dtiled(int d, const FwdArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((int64_t)a.nqt * a.BH));
    note_kernel("fa_fwd64_dt_kernel", grid.x);
    if (d == 384) hipLaunchKernelGGL((fa_fwd64_dt_kernel<384>), grid, dim3(256), 0, s, a);
    else if (d == 512) hipLaunchKernelGGL((fa_fwd64_dt_kernel<512>), grid, dim3(256), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// O = sum_s 2^(lse_s - M) O_s / sum_s 2^(lse_s - M), one thread per output element.
template <int D>
__global__ __launch_bounds__(256) void fa_combine64_kernel(CombineArgs a) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= a.rows * D) return;
    const int64_t row = e / D;
    const double* lse = a.lse64;
    double M = -INFINITY;
    for (int s = 0; s < a.nsplit; ++s) M = fmax(M, lse[s * a.rows + row]);
    double num = 0.0, den = 0.0;
    for (int s = 0; s < a.nsplit; ++s) {
        const double w = exp2(lse[s * a.rows + row] - M);
        num += w * ((const double*)a.o_part)[(s * a.rows) * D + e];
        den += w;
    }
    ((double*)a.o)[e] = num / den;
}

int fwd64_rows_per_block() { return kBQ64; }
int fwd64_keys_per_tile() { return kBK64; }

hipError_t launch_fwd64(int d, Mode mode, const FwdArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((int64_t)a.nqt * a.nsplit * a.BH));
    auto go = [&](auto kern) {
        note_kernel(mode == kFinal ? "fa_fwd64_kernel<final>" : "fa_fwd64_kernel<partial>", grid.x);
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, a);
        return hipGetLastError();
    };
    if (mode == kFinal) {
        switch (d) {
            case 32: return go(fa_fwd64_kernel<32, kFinal>);
            case 64: return go(fa_fwd64_kernel<64, kFinal>);
            case 128: return go(fa_fwd64_kernel<128, kFinal>);
            case 256: return go(fa_fwd64_kernel<256, kFinal>);
        }
    } else if (mode == kPartial) {
        switch (d) {
            case 32: return go(fa_fwd64_kernel<32, kPartial>);
            case 64: return go(fa_fwd64_kernel<64, kPartial>);
            case 128: return go(fa_fwd64_kernel<128, kPartial>);
            case 256: return go(fa_fwd64_kernel<256, kPartial>);
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_combine64(int d, const CombineArgs& a, hipStream_t s) {
    const dim3 grid((unsigned)((a.rows * d + 255) / 256));
    note_kernel("fa_combine64_kernel", grid.x);
    switch (d) {
        case 32: hipLaunchKernelGGL((fa_combine64_kernel<32>), grid, dim3(256), 0, s, a); break;
        case 64: hipLaunchKernelGGL((fa_combine64_kernel<64>), grid, dim3(256), 0, s, a); break;
        case 128: hipLaunchKernelGGL((fa_combine64_kernel<128>), grid, dim3(256), 0, s, a); break;
        case 256: hipLaunchKernelGGL((fa_combine64_kernel<256>), grid, dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fa
