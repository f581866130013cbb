// Fused clip_gradient + SGD(momentum) over all trainable parameters.
//
// Replaces clip_gradient (lib/model/utils/net_utils.py:38-49: a Python loop of per-param
// .norm() and a .item() host sync, then a second loop of p.grad.mul_) followed by
// torch.optim.SGD (methods/DAF/DAF_train.py:406-408).  Three stream-ordered launches, no
// host sync, deterministic (fixed-order reductions):
//   0. (data parallel) g = grad_scale * G, G the all-reduced gradient sum (applied as read);
//   1. per-chunk sum of squares of the gradients;
//   2. one workgroup: total = sqrt(sum), scale = clip / max(total, clip);
//   3. per chunk: g' = scale*g; d = g' + wd*p; buf = m*buf + d; p -= lr*buf.
// HBM traffic: read g twice, read+write p and buf once: 6 x 4 B per parameter.
//
// tlod_sgd_clip_pack_f32: the 3x3 conv weights are updated by 32 x 32-channel tiles that also
// store the new weights' split-bf16 packs (the forward and input-gradient operand layouts of
// the conv kernels), so no pack launch runs between the step and the next forward: +6.7 B
// written per weight element and pack instead of a separate pass that re-reads the weight.
#include "common.h"
#include "bs_common.h"
#include "tlod.h"

#ifndef TLOD_SGD_NT
#define TLOD_SGD_NT 1
#endif

namespace tlod {

static_assert(sizeof(tlod_sgd_chunk) == 48, "descriptor layout (tlod/optim.py _DESC)");
static_assert(sizeof(tlod_sgd_pack_tile) == 96, "descriptor layout (tlod/optim.py _TILE)");

// 16-B vector path when the chunk's pointers are 16-B aligned and its count a multiple of
// 4 (the grads can be views into the DP reducer's flat buckets at any float offset).
__device__ __forceinline__ bool vec4_ok(const void* a, const void* b, const void* c,
                                        long long n) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
           reinterpret_cast<uintptr_t>(c)) & 15) == 0 && (n & 3) == 0;
}

__global__ void __launch_bounds__(256) sgd_sumsq_kernel(const tlod_sgd_chunk* __restrict__ chunks,
                                                        float gs, float* __restrict__ partials) {
  tlod_sgd_chunk c = chunks[blockIdx.x];
  c.count = c.count < 0 ? -c.count : c.count;  // (a norm-only row: see tlod_sgd_chunk)
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (vec4_ok(c.grad, c.grad, c.grad, c.count)) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4* g4 = reinterpret_cast<const v4*>(c.grad);
    const long long n4 = c.count / 4;
#pragma unroll 4
    for (long long i = threadIdx.x; i < n4; i += 256) {
      v4 g = g4[i];  // (a plain load: the update pass re-reads g, partly from the MALL)
      g *= gs;
      s0 += g.x * g.x; s1 += g.y * g.y; s2 += g.z * g.z; s3 += g.w * g.w;
    }
  } else {
    for (long long i = threadIdx.x; i < c.count; i += 256) {
      const float g = c.grad[i] * gs;
      s0 += g * g;
    }
  }
  float s = (s0 + s1) + (s2 + s3);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  __shared__ float ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (ws[0] + ws[1]) + (ws[2] + ws[3]);
}

__global__ void __launch_bounds__(256) sgd_norm_kernel(const float* __restrict__ partials, int n,
                                                       float clip, float* __restrict__ out) {
  __shared__ double ws[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += (double)partials[i];
  ws[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) ws[threadIdx.x] += ws[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(ws[0]);
    out[0] = total;
    out[1] = clip > 0.f ? clip / fmaxf(total, clip) : 1.f;  // net_utils.py:46
  }
}

__device__ __forceinline__ void sgd1(float g, float& p, float& b, float gs, float scale,
                                     float wd, float lr, float momentum) {
  const float d = (g * gs) * scale + wd * p;
  b = momentum * b + d;
  p = p - lr * b;
}

__global__ void __launch_bounds__(256) sgd_update_kernel(const tlod_sgd_chunk* __restrict__ chunks,
                                                         const float* __restrict__ norm_scale,
                                                         float gs, float momentum) {
  const tlod_sgd_chunk c = chunks[blockIdx.x];
  if (c.count < 0) return;  // norm-only row: a pack tile updates these elements
  if (c.active != nullptr && *c.active == 0.f) return;  // no rank produced this gradient
  const float scale = norm_scale[1];
  if (vec4_ok(c.grad, c.param, c.momentum_buf, c.count)) {
    const long long n4 = c.count / 4;
#if TLOD_SGD_NT
    // streaming: every element is touched once per step, ~15 ms and >10 GB of other traffic
    // apart, so the loads and stores bypass the caches' retention (nontemporal)
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4* gv = reinterpret_cast<const v4*>(c.grad);
    v4* pv = reinterpret_cast<v4*>(c.param);
    v4* bv = reinterpret_cast<v4*>(c.momentum_buf);
#pragma unroll 4
    for (long long i = threadIdx.x; i < n4; i += 256) {
      const v4 g = __builtin_nontemporal_load(gv + i);
      v4 p = __builtin_nontemporal_load(pv + i), b = __builtin_nontemporal_load(bv + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = p[e], be = b[e];
        sgd1(g[e], pe, be, gs, scale, c.weight_decay, c.lr, momentum);
        p[e] = pe;
        b[e] = be;
      }
      __builtin_nontemporal_store(b, bv + i);
      __builtin_nontemporal_store(p, pv + i);
    }
#else
    const float4* __restrict__ g4 = reinterpret_cast<const float4*>(c.grad);
    float4* __restrict__ p4 = reinterpret_cast<float4*>(c.param);
    float4* __restrict__ b4 = reinterpret_cast<float4*>(c.momentum_buf);
#pragma unroll 2
    for (long long i = threadIdx.x; i < n4; i += 256) {
      const float4 g = g4[i];
      float4 p = p4[i], b = b4[i];
      sgd1(g.x, p.x, b.x, gs, scale, c.weight_decay, c.lr, momentum);
      sgd1(g.y, p.y, b.y, gs, scale, c.weight_decay, c.lr, momentum);
      sgd1(g.z, p.z, b.z, gs, scale, c.weight_decay, c.lr, momentum);
      sgd1(g.w, p.w, b.w, gs, scale, c.weight_decay, c.lr, momentum);
      b4[i] = b;
      p4[i] = p;
    }
#endif
    return;
  }
  for (long long i = threadIdx.x; i < c.count; i += 256) {
    float p = c.param[i], b = c.momentum_buf[i];
    sgd1(c.grad[i], p, b, gs, scale, c.weight_decay, c.lr, momentum);
    c.momentum_buf[i] = b;
    c.param[i] = p;
  }
}


// One tile of a (cout, cin, 3, 3) weight: 32 output x 32 input channels x 9 taps.  The update
// is the one sgd_update_kernel applies; the updated tile is kept in LDS ([o][ci * 9 + tap],
// 289-float rows) and written out as the packed units of pack_bs_kernel (conv.hip): forward
// unit (o, chunk, tap) = 8 input channels, input-gradient unit (ci, chunk, 8 - tap) = 8
// output channels, 3 bf16 planes of 16 B each.  Zero padding of the packs (tap slot 9,
// channels past the last) is never rewritten; lanes past the last channel store zeros.
constexpr int kPT = 32;
constexpr int kPTRow = kPT * 9 + 1;

__device__ __forceinline__ void store_units(unsigned short* P, size_t plane, size_t off,
                                            const float (&v)[8]) {
  u32x4 sp[3];
  split8<3>(v, sp);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(P + pl * plane + off) = sp[pl];
}

__global__ void __launch_bounds__(256) sgd_pack_kernel(const tlod_sgd_pack_tile* __restrict__ tiles,
                                                       const float* __restrict__ norm_scale,
                                                       float gs, float momentum) {
  const tlod_sgd_pack_tile t = tiles[blockIdx.x];
  if (t.active != nullptr && *t.active == 0.f) return;
  __shared__ float w[kPT * kPTRow];
  const float scale = norm_scale[1];
  const int no = min(kPT, t.cout - t.o0), ni = min(kPT, t.cin - t.i0);
  const int seg = ni * 9;  // contiguous elements of one output channel inside the tile
#pragma unroll 4
  for (int idx = threadIdx.x; idx < kPT * kPT * 9; idx += 256) {
    const int ol = idx / (kPT * 9), j = idx - ol * (kPT * 9);
    float pv = 0.f;
    if (ol < no && j < seg) {
      const size_t e = ((size_t)(t.o0 + ol) * t.cin + t.i0) * 9 + j;
      const float g = __builtin_nontemporal_load(t.grad + e);
      float p = __builtin_nontemporal_load(t.param + e);
      float b = __builtin_nontemporal_load(t.momentum_buf + e);
      sgd1(g, p, b, gs, scale, t.weight_decay, t.lr, momentum);
      __builtin_nontemporal_store(b, t.momentum_buf + e);
      __builtin_nontemporal_store(p, t.param + e);
      pv = p;
    }
    w[ol * kPTRow + j] = pv;
  }
  __syncthreads();
  if (t.pack_fwd != nullptr) {
    const int rowlen = ((t.cin + 7) / 8) * kBsKP, ncl = ((ni + 7) / 8);
    const size_t plane = (size_t)t.cout * rowlen;
    for (int u = threadIdx.x; u < kPT * 4 * 9; u += 256) {
      const int s = u % 9, r = u / 9, cl = r & 3, ol = r >> 2;
      if (ol >= no || cl >= ncl) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = w[ol * kPTRow + (cl * 8 + e) * 9 + s];
      store_units(t.pack_fwd, plane,
                  (size_t)(t.o0 + ol) * rowlen + (size_t)(t.i0 / 8 + cl) * kBsKP + s * 8, v);
    }
  }
  if (t.pack_dgrad != nullptr || t.pack_dgrad_scaled != nullptr) {
    const int rowlen = ((t.cout + 7) / 8) * kBsKP, nocl = ((no + 7) / 8);
    const size_t plane = (size_t)t.cin * rowlen;
    for (int u = threadIdx.x; u < kPT * 4 * 9; u += 256) {
      const int s = u % 9, r = u / 9, ocl = r & 3, il = r >> 2;
      if (il >= ni || ocl >= nocl) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = w[(ocl * 8 + e) * kPTRow + il * 9 + (8 - s)];
      const size_t off = (size_t)(t.i0 + il) * rowlen + (size_t)(t.o0 / 8 + ocl) * kBsKP + s * 8;
      if (t.pack_dgrad != nullptr) store_units(t.pack_dgrad, plane, off, v);
      if (t.pack_dgrad_scaled != nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int o = t.o0 + ocl * 8 + e;
          if (o < t.cout) v[e] *= t.scale[o];
        }
        store_units(t.pack_dgrad_scaled, plane, off, v);
      }
    }
  }
}

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_sgd_clip_pack_f32(const tlod_sgd_chunk* chunks, int n_chunks, int n_update,
                                      const tlod_sgd_pack_tile* tiles, int n_tiles,
                                      float grad_scale, float momentum, float clip_norm,
                                      float* partials, float* norm_scale, tlod_stream_t stream) {
  TLOD_CHECK_ARG(n_chunks > 0 && chunks && partials && norm_scale, "bad arguments");
  TLOD_CHECK_ARG(n_update >= 0 && n_update <= n_chunks && n_tiles >= 0 && (n_tiles == 0 || tiles),
                 "bad update / tile counts");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sgd_sumsq_kernel, dim3(n_chunks), dim3(256), 0, s, chunks, grad_scale, partials);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(sgd_norm_kernel, dim3(1), dim3(256), 0, s, partials, n_chunks, clip_norm,
                     norm_scale);
  TLOD_LAUNCH_CHECK();
  if (n_update > 0) {
    hipLaunchKernelGGL(sgd_update_kernel, dim3(n_update), dim3(256), 0, s, chunks, norm_scale,
                       grad_scale, momentum);
    TLOD_LAUNCH_CHECK();
  }
  if (n_tiles > 0) {
    hipLaunchKernelGGL(sgd_pack_kernel, dim3(n_tiles), dim3(256), 0, s, tiles, norm_scale,
                       grad_scale, momentum);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}

extern "C" int tlod_sgd_clip_f32(const tlod_sgd_chunk* chunks, int n_chunks, float grad_scale,
                                 float momentum, float clip_norm, float* partials,
                                 float* norm_scale, tlod_stream_t stream) {
  return tlod_sgd_clip_pack_f32(chunks, n_chunks, n_chunks, nullptr, 0, grad_scale, momentum,
                                clip_norm, partials, norm_scale, stream);
}
