// fa_device.hpp -- device helpers shared by the gfx950 forward kernels (fa_fwd.hip,
// fa_fwd_w64.hip): vector types, MFMA wrappers, the swizzled LDS tile image, the XCD-aware
// workgroup remap, lane-pair reductions, 16-bit packing, buffer descriptors, LDS-DMA.
#pragma once
#include <utility>

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
    static __device__ __forceinline__ f32x4 mma16(v8 a, v8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mma<_Float16> {
    typedef _Float16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x4 mma16(v8 a, v8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
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

// max without fmaxf's IEEE quieting: llvm.maximum lowers to v_maximum3_f32 on gfx950 and
// needs no canonicalising v_max x,x in front of every MFMA result it reads (NaN propagates
// instead of being dropped -- scores are finite or -inf here)
__device__ __forceinline__ float fmax_nc(float a, float b) { return __builtin_elementwise_maximum(a, b); }

__device__ __forceinline__ float pair_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmax_nc(__uint_as_float(r[0]), __uint_as_float(r[1]));
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc32(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N), so that each
// body can feed i into an inline-asm "i" (immediate) operand.
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// One 16-byte-per-lane LDS-DMA piece: lane i's 16 bytes land at lds + 16*i.  Kept out of
// the kernel's lambdas: a builtin call inside a lambda made hipcc drop the kernel's host
// launch stub (undefined __device_stub__ at load time).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds, int voff, int soff) {
    typedef __attribute__((address_space(3))) void lds_void;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, voff, soff, 0, 0);
}

// Row max of both query blocks at once: x0 (query n) and x1 (query 16 + n) are per-lane partial
// maxima; the result is the max over the 4 lanes n, n+16, n+32, n+48 of each, in every lane.
// Three swaps for the pair (a quad reduction per value would take four and two copies):
// swap16(x0, x1) leaves rows 0 / 2 reducing x0 and rows 1 / 3 reducing x1 (one row = 16 lanes),
// swap32 finishes both, and a last swap16 hands each lane both totals.
__device__ __forceinline__ void quad_max2(float x0, float x1, float& m0, float& m1) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
    const float y = fmax_nc(__uint_as_float(r[0]), __uint_as_float(r[1]));
    auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
    const float z = fmax_nc(__uint_as_float(s[0]), __uint_as_float(s[1]));
    auto u = __builtin_amdgcn_permlane16_swap(__float_as_uint(z), __float_as_uint(z), false, false);
    m0 = __uint_as_float(u[0]);
    m1 = __uint_as_float(u[1]);
}

}  // namespace fa
