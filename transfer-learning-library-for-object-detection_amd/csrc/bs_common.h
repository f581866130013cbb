// Device helpers shared by the MFMA kernels (conv.hip, gemm.hip): vector types, the
// XCD-aware block remap, raw buffer loads with range-check zero fill, and the exact split
// of f32 operands into bf16 planes for the split-bf16 ("bf16xN") MFMA arithmetic.
#pragma once
#include <hip/hip_runtime.h>

namespace tlod {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// XCD-aware bijective remap: consecutive hardware ids round-robin over 8 XCDs; give
// each XCD a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pack_hi2(unsigned lo_elem, unsigned hi_elem) {
  return __builtin_amdgcn_perm(hi_elem, lo_elem, 0x07060302u);  // upper halves -> 2 x bf16
}

// split 8 floats into NPL bf16 planes (16 B each)
template <int NPL>
__device__ __forceinline__ void split8(const float (&v)[8], u32x4 (&out)[3]) {
  unsigned hb[8], mb[8], lb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const unsigned u = __float_as_uint(v[e]);
    hb[e] = u & 0xffff0000u;
    const float r = v[e] - __uint_as_float(hb[e]);
    mb[e] = __float_as_uint(r) & 0xffff0000u;
    if constexpr (NPL == 3) lb[e] = __float_as_uint(r - __uint_as_float(mb[e]));
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    out[0][q] = pack_hi2(hb[2 * q], hb[2 * q + 1]);
    out[1][q] = pack_hi2(mb[2 * q], mb[2 * q + 1]);
    if constexpr (NPL == 3) out[2][q] = pack_hi2(lb[2 * q], lb[2 * q + 1]);
  }
}

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ f32x4v raw_buffer_load_v4f32(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ float raw_buffer_load_f32(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.f32");

__device__ __forceinline__ i32x4 make_buffer_rsrc(const void* p, unsigned bytes) {
  struct __attribute__((packed)) R {
    const void* ptr;
    unsigned range;
    unsigned config;
  } r{p, bytes, 0x00020000u};
  return __builtin_bit_cast(i32x4, r);
}

constexpr int kBufOOB = (int)0x80000000;  // voffset past any range: the load returns 0

// bits [0, x) of a 4-bit mask, x clamped to [0, 4]
__device__ __forceinline__ unsigned lt_mask4(int x) { return (1u << min(max(x, 0), 4)) - 1u; }

// split 4 floats into NPL bf16 planes (8 B each)
template <int NPL>
__device__ __forceinline__ void split4(const float (&v)[4], unsigned (&out)[3][2]) {
  unsigned hb[4], mb[4], lb[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const unsigned u = __float_as_uint(v[e]);
    hb[e] = u & 0xffff0000u;
    const float r = v[e] - __uint_as_float(hb[e]);
    mb[e] = __float_as_uint(r) & 0xffff0000u;
    if constexpr (NPL == 3) lb[e] = __float_as_uint(r - __uint_as_float(mb[e]));
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    out[0][q] = pack_hi2(hb[2 * q], hb[2 * q + 1]);
    out[1][q] = pack_hi2(mb[2 * q], mb[2 * q + 1]);
    if constexpr (NPL == 3) out[2][q] = pack_hi2(lb[2 * q], lb[2 * q + 1]);
  }
}

}  // namespace tlod
