// Device helpers shared by the MFMA kernels (conv.hip, gemm.hip): vector types, the
// XCD-aware block remap, raw buffer loads with range-check zero fill, and the exact split
// of f32 operands into bf16 planes for the split-bf16 ("bf16xN") MFMA arithmetic.
#pragma once
#include <hip/hip_runtime.h>

namespace tlod {

// Packed 3x3 weight row (pack_bs_kernel in conv.hip, and the fused SGD in optim.hip that
// keeps the packs current): per 8-channel chunk 10 tap slots (9 + a zero pad) x 8 channels.
constexpr int kBsKP = 80;

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
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Exact split x = hi + mid + lo into bf16 terms: hi = the truncated top 8 significant bits
// (exact and finite for every finite x), mid and lo the round-to-nearest-even bf16 of the
// remainders (v_cvt_pk_bf16_f32, two elements per instruction; element 0 in the low half).
// The remainder x - hi is exact with <= 16 bits, mid keeps its top 8 (rounded) and lo the
// exact rest (<= 8 bits).  Round-to-nearest on mid and lo matters for accuracy, not
// exactness: the products the bf16x6 scheme drops (mid*lo, lo*mid, lo*lo) each carry a lo
// factor of random sign — with every term truncated (round 1) each remainder had the sign
// of its operand, every dropped term the sign of its product, and the sums shrank
// systematically (~3e-8 relative per product).  A round-to-nearest hi (round 2) needed a
// check for operands that round to bf16 infinity; the truncated hi needs none and costs the
// same one instruction per pair.  NaN / infinity operands give NaN products (their
// remainders are NaN), as the f32 MFMA path would propagate them.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ float bf_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

// f32 subtraction the compiler cannot SLP-pack into v_pk_add_f32: on gfx950 the packed f32
// ops are an anti-lever beside MFMAs (MI355X_MICROARCH.md, constants table: +22-26 cycles
// per packed op in an MFMA stream), and a producer wave sharing its SIMD with MFMA waves
// issued them at a fraction of the plain rate (wgrad_ws producers: ~48 cycles per
// instruction with the compiler's packed split).
__device__ __forceinline__ float sub_f32(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// one pair of floats -> its NPL packed bf16 planes
template <int NPL>
__device__ __forceinline__ void split2(float x0, float x1, unsigned& h, unsigned& m,
                                       unsigned& l) {
  const unsigned u0 = __float_as_uint(x0) & 0xffff0000u, u1 = __float_as_uint(x1) & 0xffff0000u;
  h = (u0 >> 16) | u1;  // v_perm_b32
  const float r0 = sub_f32(x0, __uint_as_float(u0)), r1 = sub_f32(x1, __uint_as_float(u1));
  m = cvt_pk_bf16(r0, r1);
  if constexpr (NPL == 3) l = cvt_pk_bf16(sub_f32(r0, bf_lo(m)), sub_f32(r1, bf_hi(m)));
}

// split 8 floats into NPL bf16 planes (16 B each)
template <int NPL>
__device__ __forceinline__ void split8(const float (&v)[8], u32x4 (&out)[3]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned h, m, l = 0;
    split2<NPL>(v[2 * q], v[2 * q + 1], h, m, l);
    out[0][q] = h;
    out[1][q] = m;
    if constexpr (NPL == 3) out[2][q] = l;
  }
}

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// One k-step of the split-bf16 product of a 32x32 tile (NP = 3 or 6 bf16 products),
// added to the running accumulator.  Accuracy (tools/probe/mfma_round.hip):
// the bf16 MFMA adds its products into the accumulator with the bits below the sum's
// precision truncated (8 products of 0.19 ulp each add nothing; one of 0.75 ulp rounds to
// nearest), so small products chained onto a large accumulator are floored — a coherent
// shrink (-1e-7 relative on length-4608 positive dot products, -3e-9 per conv layer on
// random data).  TLOD_BS_KSUM=1 sums each k-step's products from zero (small first) and
// adds that sum with one round-to-nearest f32 add: the shrink drops to -1.4e-9 and the rms
// error to 0.3x (below the f32 fmaf chain's).  Cost: a temporary per live tile and one
// VALU add per accumulator register per k-step.
// Off by default: the 32x32 kernels' 16-register temporaries spill (fwd_bs 0 -> 700 VGPRs,
// wgrad_bs 0 -> 64, gemm_bs 0 -> 21); in the warp-specialized 16x16x32 kernel
// (TLOD_BS_KSUM16) the temporary is 4 registers, but the adds beside the producers' split
// VALU cost the DAF step 4% (62.0 vs 64.6 img/s, one lease).
#ifndef TLOD_BS_KSUM
#define TLOD_BS_KSUM 0
#endif
#ifndef TLOD_BS_KSUM16
#define TLOD_BS_KSUM16 0
#endif
template <int NP>
__device__ __forceinline__ void bs_mac(f32x16& acc, u32x4 a0, u32x4 a1, u32x4 a2, u32x4 b0,
                                       u32x4 b1, u32x4 b2) {
  if (TLOD_BS_KSUM) {
    f32x16 t = mfma_bf16(a1, b0, f32x16{});
    t = mfma_bf16(a0, b1, t);
    if constexpr (NP == 6) {
      t = mfma_bf16(a2, b0, t);
      t = mfma_bf16(a1, b1, t);
      t = mfma_bf16(a0, b2, t);
    }
    acc += mfma_bf16(a0, b0, t);
  } else {
    acc = mfma_bf16(a0, b0, acc);
    acc = mfma_bf16(a1, b0, acc);
    acc = mfma_bf16(a0, b1, acc);
    if constexpr (NP == 6) {
      acc = mfma_bf16(a2, b0, acc);
      acc = mfma_bf16(a1, b1, acc);
      acc = mfma_bf16(a0, b2, acc);
    }
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ f32x4v raw_buffer_load_v4f32(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ float raw_buffer_load_f32(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.f32");
// (a store at an offset past the range — kBufOOB — is dropped by the hardware)
__device__ void raw_buffer_store_f32(float v, i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.f32");

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
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    unsigned h, m, l = 0;
    split2<NPL>(v[2 * q], v[2 * q + 1], h, m, l);
    out[0][q] = h;
    out[1][q] = m;
    if constexpr (NPL == 3) out[2][q] = l;
  }
}

}  // namespace tlod
