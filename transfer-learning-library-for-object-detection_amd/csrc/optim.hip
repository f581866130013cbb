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
#include "common.h"
#include "tlod.h"

#ifndef TLOD_SGD_NT
#define TLOD_SGD_NT 1
#endif

namespace tlod {

static_assert(sizeof(tlod_sgd_chunk) == 48, "descriptor layout (tlod/optim.py _DESC)");

// 16-B vector path when the chunk's pointers are 16-B aligned and its count a multiple of
// 4 (the grads can be views into the DP reducer's flat buckets at any float offset).
__device__ __forceinline__ bool vec4_ok(const void* a, const void* b, const void* c,
                                        long long n) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
           reinterpret_cast<uintptr_t>(c)) & 15) == 0 && (n & 3) == 0;
}

__global__ void __launch_bounds__(256) sgd_sumsq_kernel(const tlod_sgd_chunk* __restrict__ chunks,
                                                        float gs, float* __restrict__ partials) {
  const tlod_sgd_chunk c = chunks[blockIdx.x];
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

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_sgd_clip_f32(const tlod_sgd_chunk* chunks, int n_chunks, float grad_scale,
                                 float momentum, float clip_norm, float* partials,
                                 float* norm_scale, tlod_stream_t stream) {
  TLOD_CHECK_ARG(n_chunks > 0 && chunks && partials && norm_scale, "bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sgd_sumsq_kernel, dim3(n_chunks), dim3(256), 0, s, chunks, grad_scale, partials);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(sgd_norm_kernel, dim3(1), dim3(256), 0, s, partials, n_chunks, clip_norm,
                     norm_scale);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(sgd_update_kernel, dim3(n_chunks), dim3(256), 0, s, chunks, norm_scale,
                     grad_scale, momentum);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
