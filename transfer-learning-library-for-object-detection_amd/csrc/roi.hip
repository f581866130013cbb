// RoIAlign / RoIAlignAvg / RoIPool forward + backward for gfx950.
//
// Numerics follow the reference CUDA kernels literally (compiled here with
// -ffp-contract=off): lib/model/roi_align/src/roi_align_kernel.cu:15-143 — note the
// ``1.`` double literals, reproduced as double arithmetic — and
// lib/model/roi_pooling/src/roi_pooling_kernel.cu:24-93.
//
// Layout choices (MI355X-first, not a translation of the reference launch shape):
//   * RoIAlignAvg is fused: one workgroup per (roi, 64 channels) samples the
//     (ph+1)x(pw+1) grid into LDS and writes the 2x2/s1-averaged (ph,pw) output as one
//     contiguous, coalesced slab (the reference writes the 8x8 map to HBM, then a
//     second torch kernel re-reads it).  Backward fuses avg_pool2d's backward.
//   * RoIPool backward scatters through argmax (O(R*C*ph*pw) atomics) instead of the
//     reference's O(B*C*H*W*R) gather (roi_pooling_kernel.cu:128-203).
#include <algorithm>
#include <cfloat>

#include <hipcub/hipcub.hpp>

#include "common.h"
#include "tlod.h"

namespace tlod {

// roi_align_kernel.cu:30-53 for one sample (ph, pw) of roi r.
__device__ __forceinline__ void align_axis(float start, float end, int n_samples, int p,
                                           int limit, int* idx, float* ratio, bool* valid) {
  float len = fmaxf((float)((double)(end - start) + 1.), 0.f);
  float bin = (float)((double)len / ((double)n_samples - 1.));
  float v = (float)p * bin + start;
  int s = (int)fminf((float)floor((double)v), (float)(limit - 2));
  *idx = s;
  *ratio = v - (float)s;
  *valid = !(v < 0.f || v >= (float)limit);
}

__device__ __forceinline__ float align_sample(const float* __restrict__ plane, int W, int y,
                                              int x, float hr, float wr) {
  const float ul = plane[y * W + x], ur = plane[y * W + x + 1];
  const float dl = plane[(y + 1) * W + x], dr = plane[(y + 1) * W + x + 1];
  // bottom[ul]*(1.-h)*(1.-w) + bottom[ur]*(1.-h)*w + bottom[dl]*h*(1.-w) + bottom[dr]*h*w
  double t1 = ((double)ul * (1. - (double)hr)) * (1. - (double)wr);
  double t2 = ((double)ur * (1. - (double)hr)) * (double)wr;
  double t3 = (double)(dl * hr) * (1. - (double)wr);
  double t4 = (double)((dr * hr) * wr);
  return (float)(((t1 + t2) + t3) + t4);
}

// ------------------------------------------------------------ plain RoIAlign
__global__ void roi_align_fwd_kernel(int total, const float* __restrict__ feat, float scale,
                                     int C, int H, int W, int ah, int aw,
                                     const float* __restrict__ rois, float* __restrict__ out) {
  for (int index = blockIdx.x * blockDim.x + threadIdx.x; index < total;
       index += blockDim.x * gridDim.x) {
    const int pw = index % aw;
    const int ph = (index / aw) % ah;
    const int c = (index / aw / ah) % C;
    const int n = index / aw / ah / C;
    const float* r = rois + n * 5;
    const int b = (int)r[0];
    int y, x;
    float hr, wr;
    bool vy, vx;
    align_axis(r[2] * scale, r[4] * scale, ah, ph, H, &y, &hr, &vy);
    align_axis(r[1] * scale, r[3] * scale, aw, pw, W, &x, &wr, &vx);
    out[index] = (vy && vx)
                     ? align_sample(feat + ((size_t)b * C + c) * H * W, W, y, x, hr, wr)
                     : 0.f;
  }
}

__device__ __forceinline__ void align_scatter(float* __restrict__ plane, int W, int y, int x,
                                              float hr, float wr, float td) {
  // roi_align_kernel.cu:137-140 — atomicAdd arguments rounded to float as in the source.
  const float om = 1.f - wr;  // (1 - w_ratio) is float
  atomicAdd(plane + y * W + x, (float)(((double)td * (1. - (double)hr)) * (double)om));
  atomicAdd(plane + y * W + x + 1, (float)(((double)td * (1. - (double)hr)) * (double)wr));
  atomicAdd(plane + (y + 1) * W + x, (td * hr) * om);
  atomicAdd(plane + (y + 1) * W + x + 1, (td * hr) * wr);
}

__global__ void roi_align_bwd_kernel(int total, const float* __restrict__ top, float scale,
                                     int C, int H, int W, int ah, int aw,
                                     const float* __restrict__ rois, float* __restrict__ grad) {
  for (int index = blockIdx.x * blockDim.x + threadIdx.x; index < total;
       index += blockDim.x * gridDim.x) {
    const int pw = index % aw;
    const int ph = (index / aw) % ah;
    const int c = (index / aw / ah) % C;
    const int n = index / aw / ah / C;
    const float* r = rois + n * 5;
    const int b = (int)r[0];
    int y, x;
    float hr, wr;
    bool vy, vx;
    align_axis(r[2] * scale, r[4] * scale, ah, ph, H, &y, &hr, &vy);
    align_axis(r[1] * scale, r[3] * scale, aw, pw, W, &x, &wr, &vx);
    if (vy && vx) align_scatter(grad + ((size_t)b * C + c) * H * W, W, y, x, hr, wr, top[index]);
  }
}

// ------------------------------------------------------------ fused RoIAlignAvg
constexpr int kAvgCh = 64;     // channels per workgroup
constexpr int kAvgThreads = 256;

// grid (ceil(C/64), R).  S = (ph+1)*(pw+1) <= 64 samples per channel.
__global__ void __launch_bounds__(kAvgThreads) roi_align_avg_fwd_kernel(
    const float* __restrict__ feat, float scale, int C, int H, int W, int ph, int pw,
    const float* __restrict__ rois, float* __restrict__ out) {
  const int ah = ph + 1, aw = pw + 1, S = ah * aw;
  const int r = blockIdx.y, c0 = blockIdx.x * kAvgCh;
  const int nc = min(kAvgCh, C - c0);
  __shared__ int gy[8], gx[8];
  __shared__ float ghr[8], gwr[8];
  __shared__ bool gvy[8], gvx[8];
  __shared__ float samp[kAvgCh * 65];
  const float* ro = rois + r * 5;
  const int t = threadIdx.x;
  if (t < ah) align_axis(ro[2] * scale, ro[4] * scale, ah, t, H, &gy[t], &ghr[t], &gvy[t]);
  if (t >= 32 && t < 32 + aw) {
    const int p = t - 32;
    align_axis(ro[1] * scale, ro[3] * scale, aw, p, W, &gx[p], &gwr[p], &gvx[p]);
  }
  __syncthreads();
  const int b = (int)ro[0];
  const float* base = feat + ((size_t)b * C + c0) * H * W;
  for (int e = t; e < nc * S; e += kAvgThreads) {
    const int c = e / S, s = e % S;
    const int sy = s / aw, sx = s % aw;
    float v = 0.f;
    if (gvy[sy] && gvx[sx])
      v = align_sample(base + (size_t)c * H * W, W, gy[sy], gx[sx], ghr[sy], gwr[sx]);
    samp[c * 65 + s] = v;
  }
  __syncthreads();
  // avg_pool2d(2, s1): ((((0+a)+b)+c)+d)/4 in float, rows then columns.
  const int P = ph * pw;
  float* o = out + ((size_t)r * C + c0) * P;
  for (int e = t; e < nc * P; e += kAvgThreads) {
    const int c = e / P, q = e % P;
    const int oy = q / pw, ox = q % pw;
    const float* sp = samp + c * 65 + oy * aw + ox;
    float acc = 0.f;
    acc += sp[0];
    acc += sp[1];
    acc += sp[aw];
    acc += sp[aw + 1];
    o[e] = acc / 4.f;
  }
}

__global__ void __launch_bounds__(kAvgThreads) roi_align_avg_bwd_kernel(
    const float* __restrict__ top, float scale, int C, int H, int W, int ph, int pw,
    const float* __restrict__ rois, float* __restrict__ grad) {
  const int ah = ph + 1, aw = pw + 1, S = ah * aw, P = ph * pw;
  const int r = blockIdx.y, c0 = blockIdx.x * kAvgCh;
  const int nc = min(kAvgCh, C - c0);
  __shared__ int gy[8], gx[8];
  __shared__ float ghr[8], gwr[8];
  __shared__ bool gvy[8], gvx[8];
  __shared__ float g7[kAvgCh * 49 + 64];
  const float* ro = rois + r * 5;
  const int t = threadIdx.x;
  if (t < ah) align_axis(ro[2] * scale, ro[4] * scale, ah, t, H, &gy[t], &ghr[t], &gvy[t]);
  if (t >= 32 && t < 32 + aw) {
    const int p = t - 32;
    align_axis(ro[1] * scale, ro[3] * scale, aw, p, W, &gx[p], &gwr[p], &gvx[p]);
  }
  const float* tp = top + ((size_t)r * C + c0) * P;
  for (int e = t; e < nc * P; e += kAvgThreads) g7[e] = tp[e] / 4.f;  // coalesced slab
  __syncthreads();
  const int b = (int)ro[0];
  float* gbase = grad + ((size_t)b * C + c0) * H * W;
  for (int e = t; e < nc * S; e += kAvgThreads) {
    const int c = e / S, s = e % S;
    const int sy = s / aw, sx = s % aw;
    if (!(gvy[sy] && gvx[sx])) continue;
    // avg_pool2d backward: sum over covering windows, py outer, px inner (float).
    float g = 0.f;
    const float* gp = g7 + c * P;
    for (int py = max(0, sy - 1); py <= min(sy, ph - 1); ++py)
      for (int px = max(0, sx - 1); px <= min(sx, pw - 1); ++px) g += gp[py * pw + px];
    align_scatter(gbase + (size_t)c * H * W, W, gy[sy], gx[sx], ghr[sy], gwr[sx], g);
  }
}

// ------------------------------------------------------------ RoIAlignAvg backward, NHWC
// One thread per channel, one workgroup per (roi, 256 channels): every atomic
// wave-instruction adds 64 consecutive channels of one feature cell = 256 contiguous
// bytes of the (B,H,W,C) accumulator — the shape the memory-side atomic unit runs at
// full rate (one lane per row, the NCHW shape, runs ~17x slower).
constexpr int kNhwcThreads = 256;

__global__ void __launch_bounds__(kNhwcThreads) roi_align_avg_bwd_nhwc_kernel(
    const float* __restrict__ top, float scale, int C, int H, int W, int ph, int pw,
    const float* __restrict__ rois, float* __restrict__ acc_nhwc) {
  const int ah = ph + 1, aw = pw + 1, P = ph * pw;
  const int r = blockIdx.y, c0 = blockIdx.x * kNhwcThreads;
  const int nc = min(kNhwcThreads, C - c0);
  __shared__ int gy[8], gx[8];
  __shared__ float ghr[8], gwr[8];
  __shared__ bool gvy[8], gvx[8];
  __shared__ float g7[kNhwcThreads * 49];
  const float* ro = rois + r * 5;
  const int t = threadIdx.x;
  if (t < ah) align_axis(ro[2] * scale, ro[4] * scale, ah, t, H, &gy[t], &ghr[t], &gvy[t]);
  if (t >= 32 && t < 32 + aw) {
    const int p = t - 32;
    align_axis(ro[1] * scale, ro[3] * scale, aw, p, W, &gx[p], &gwr[p], &gvx[p]);
  }
  const float* tp = top + ((size_t)r * C + c0) * P;
  for (int e = t; e < nc * P; e += kNhwcThreads) g7[e] = tp[e] / 4.f;  // coalesced slab
  __syncthreads();
  if (t >= nc) return;
  const int b = (int)ro[0];
  float* base = acc_nhwc + (size_t)b * H * W * C + c0 + t;
  const float* gp = g7 + t * P;
  for (int sy = 0; sy < ah; ++sy) {
    if (!gvy[sy]) continue;
    const int y = gy[sy];
    const float hr = ghr[sy];
    for (int sx = 0; sx < aw; ++sx) {
      if (!gvx[sx]) continue;
      float g = 0.f;  // avg_pool2d backward: py outer, px inner
      for (int py = max(0, sy - 1); py <= min(sy, ph - 1); ++py)
        for (int px = max(0, sx - 1); px <= min(sx, pw - 1); ++px) g += gp[py * pw + px];
      const int x = gx[sx];
      const float wr = gwr[sx], om = 1.f - wr;
      float* p00 = base + ((size_t)y * W + x) * C;
      atomicAdd(p00, (float)(((double)g * (1. - (double)hr)) * (double)om));
      atomicAdd(p00 + C, (float)(((double)g * (1. - (double)hr)) * (double)wr));
      atomicAdd(p00 + (size_t)W * C, (g * hr) * om);
      atomicAdd(p00 + (size_t)W * C + C, (g * hr) * wr);
    }
  }
}

// ------------------------------------------------------------ RoIAlignAvg backward, gather
// No atomics at all: the scatter (roi, sample, tap) -> feature cell is inverted once per call
// and every (cell, channel) of bottom_grad is then a gather over its own contributions.
//   1. geometry: one thread per (roi, sample): the four taps' cell ids (sentinel for a sample
//      outside the map) and the sample's (hr, wr);
//   2. a stable radix sort of the taps by cell (hipCUB), then each cell's start by binary
//      search: the taps of a cell in ascending (roi, sample, tap) order — a fixed summation
//      order, so the result is deterministic (the atomic kernels' is not);
//   3. sample gradients sg[(roi, sample)][c] = avg_pool2d's backward of top_grad (the covering
//      windows' top / 4, py outer, px inner — the atomic kernels' per-sample value), one
//      coalesced (roi, sample) row of channels each;
//   4. gather, balanced by taps: a wave takes 64 consecutive sorted taps x 64 channels (lane =
//      channel; keys / tap ids broadcast by readlane, 16 sg rows in flight), applies
//      roi_align_kernel.cu:137-140's per-tap weight and rounding, and sums each run of equal
//      cells in order.  A run inside the segment is stored to a channels-last accumulator; a
//      run crossing segment boundaries leaves its pieces (the segment's head / tail run) in
//      carry rows, which a fixup pass adds in segment order (the run's first segment owns it);
//      then one tiled pass adds the accumulator into NCHW bottom_grad.  (Round 3's first
//      version gave each wave 4 cells: the cells under many RoIs serialized it, 114 us.)
// Traffic (DAF step: 556 RoIs x 64 samples x 512 channels, 2 x 37 x 75 map): top 56 MB read,
// sg 73 MB written and read once per tap (~290 MB, mostly L2 / Infinity-Cache hits),
// bottom_grad 11 MB read + written.

__global__ void __launch_bounds__(256) rbg_geom_kernel(const float* __restrict__ rois, int R,
                                                       float scale, int H, int W, int ph, int pw,
                                                       unsigned ncell,
                                                       unsigned* __restrict__ keys,
                                                       unsigned* __restrict__ vals,
                                                       float2* __restrict__ geo,
                                                       int* __restrict__ trow, int QH, int QW) {
  const int ah = ph + 1, aw = pw + 1, S = ah * aw;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * S) return;
  const int r = i / S, smp = i % S, sy = smp / aw, sx = smp % aw;
  const float* ro = rois + r * 5;
  int y, x;
  float hr, wr;
  bool vy, vx;
  align_axis(ro[2] * scale, ro[4] * scale, ah, sy, H, &y, &hr, &vy);
  align_axis(ro[1] * scale, ro[3] * scale, aw, sx, W, &x, &wr, &vx);
  const bool ok = vy && vx;
  const unsigned c00 = (unsigned)(((int)ro[0] * H + y) * W + x);
  geo[i] = make_float2(hr, wr);
  if (trow != nullptr) {  // S2: the output bin (2 hy, 2 hx) this sample feeds, or -1
    const int hy = sy >> 1, hx = sx >> 1;
    trow[i] = hy < QH && hx < QW ? (r * QH + hy) * QW + hx : -1;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    keys[4 * i + k] = ok ? c00 + (k >> 1) * W + (k & 1) : ncell;
    vals[4 * i + k] = 4u * i + k;
  }
}

// start[c] = first sorted tap of cell c (c = 0..ncell; start[ncell] = the valid tap count)
__global__ void rbg_start_kernel(const unsigned* __restrict__ keys, int n, unsigned ncell,
                                 int* __restrict__ start) {
  const unsigned c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > ncell) return;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < c) lo = mid + 1; else hi = mid;
  }
  start[c] = lo;
}

// grid (R, ceil(C / 64)), 256 threads: sg[(r*S + s)*C + c].  V = 4 (C % 4 == 0): thread
// (sample group t / 16, channel quad t % 16) writes 16-B stores, 16 lanes a 256-B row of one
// sample; V = 1: thread (part t / 64, channel t % 64), a 256-B row per wave and sample
template <int V>
__global__ void __launch_bounds__(256) rbg_sample_grad_kernel(const float* __restrict__ top,
                                                              int C, int ph, int pw,
                                                              float* __restrict__ sg) {
  const int ah = ph + 1, aw = pw + 1, S = ah * aw, P = ph * pw;
  const int r = blockIdx.x, c0 = blockIdx.y * 64, t = threadIdx.x;
  const int nc = min(64, C - c0);
  __shared__ float g7[64 * 49];
  const float* tp = top + ((size_t)r * C + c0) * P;
  for (int e = t; e < nc * P; e += 256) g7[e] = tp[e] / 4.f;  // coalesced slab
  __syncthreads();
  constexpr int LPS = 64 / V;       // lanes per sample row
  constexpr int SPI = 256 / LPS;    // samples per iteration
  const int ch = (t % LPS) * V;
  if (ch >= nc) return;
  float* o = sg + (size_t)r * S * C + c0 + ch;
  for (int smp = t / LPS; smp < S; smp += SPI) {
    const int sy = smp / aw, sx = smp % aw;
    float g[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float* gp = g7 + (ch + v) * P;
      float a = 0.f;  // avg_pool2d backward: py outer, px inner
      for (int py = max(0, sy - 1); py <= min(sy, ph - 1); ++py)
        for (int px = max(0, sx - 1); px <= min(sx, pw - 1); ++px) a += gp[py * pw + px];
      g[v] = a;
    }
    if constexpr (V == 4)
      *reinterpret_cast<float4*>(o + (size_t)smp * C) = make_float4(g[0], g[1], g[2], g[3]);
    else
      o[(size_t)smp * C] = g[0];
  }
}

// one tap's contribution, roi_align_kernel.cu:137-140 (as align_scatter)
__device__ __forceinline__ float tap_value(float g, float hr, float wr, int k) {
  const float om = 1.f - wr;
  switch (k) {
    case 0: return (float)(((double)g * (1. - (double)hr)) * (double)om);
    case 1: return (float)(((double)g * (1. - (double)hr)) * (double)wr);
    case 2: return (g * hr) * om;
    default: return (g * hr) * wr;
  }
}

// grid (ceil(nseg / 4), ceil(C / (64 V))), 4 waves: wave = segment of 64 sorted taps, lane =
// V consecutive channels (V = 4: one 16-B load per tap and lane, so a wave keeps 16 rows x
// 1 KB in flight instead of 16 x 256 B — the gather is bound by those dependent row loads;
// every channel's arithmetic and order unchanged).  flags[seg]: 1 = owns a run continuing into
// the next segments (its tail piece in carry_tail), 2 = one run covering the whole segment
// and continuing on both sides.
// S2 (the stride-2 head entry): no sample-gradient rows — sample (r, sy, sx) feeds exactly
// one output bin, so its gradient is that bin's top row / 4, read straight from the
// channels-last top gradient (R, QH, QW, C); trow (from rbg_geom_kernel) names the row.
template <int V>
struct VecF;
template <>
struct VecF<1> {
  typedef float T;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, T v) { *p = v; }
};
template <>
struct VecF<4> {
  typedef float4 T;
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void store(float* p, T v) { *reinterpret_cast<float4*>(p) = v; }
};
__device__ __forceinline__ float vscale(float v, float s) { return v * s; }
__device__ __forceinline__ float4 vscale(float4 v, float s) {
  return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
}
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ float4 vadd(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ void vtap(float& a, float g, float hr, float wr, int k) {
  a += tap_value(g, hr, wr, k);
}
__device__ __forceinline__ void vtap(float4& a, float4 g, float hr, float wr, int k) {
  a.x += tap_value(g.x, hr, wr, k);
  a.y += tap_value(g.y, hr, wr, k);
  a.z += tap_value(g.z, hr, wr, k);
  a.w += tap_value(g.w, hr, wr, k);
}

template <bool S2, int V>
__global__ void __launch_bounds__(256) rbg_seg_gather_kernel(
    const int* __restrict__ start, const unsigned* __restrict__ keys,
    const unsigned* __restrict__ vals, const float2* __restrict__ geo,
    const float* __restrict__ sg, int C, int ncell, float* __restrict__ acc,
    float* __restrict__ carry_head, float* __restrict__ carry_tail, int* __restrict__ flags,
    const int* __restrict__ trow) {
  using VF = VecF<V>;
  typedef typename VF::T vt;
  const int lane = threadIdx.x & 63;
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = start[ncell];  // valid taps (sorted to the front)
  const int j0 = seg * 64;
  if (j0 >= n) return;
  const int jn = min(64, n - j0);
  const int c = (blockIdx.y * 64 + lane) * V;
  const bool cok = c < C;  // (V = 4: C % 4 == 0)
  unsigned kl = 0xffffffffu, vl = 0;
  float2 gl = make_float2(0.f, 0.f);
  int tl = -1;
  if (lane < jn) {
    kl = keys[j0 + lane];
    vl = vals[j0 + lane];
    gl = geo[vl >> 2];
    if constexpr (S2) tl = trow[vl >> 2];
  }
  const unsigned kprev = j0 > 0 ? keys[j0 - 1] : 0xffffffffu;
  const unsigned knext = j0 + jn < n ? keys[j0 + jn] : 0xffffffffu;
  unsigned cur = __builtin_amdgcn_readfirstlane(kl);
  int runs = 0;
  vt a = VF::zero();
  auto flush = [&](bool last) {
    const bool cont_prev = runs == 0 && cur == kprev;
    const bool cont_next = last && cur == knext;
    if (cok) {
      if (cont_prev) VF::store(carry_head + (size_t)seg * C + c, a);
      else if (cont_next) VF::store(carry_tail + (size_t)seg * C + c, a);
      else VF::store(acc + (size_t)cur * C + c, a);
    }
    if (last && blockIdx.y == 0 && lane == 0)
      flags[seg] = (cont_next && !cont_prev ? 1 : 0) | (runs == 0 && cont_prev && cont_next ? 2 : 0);
    ++runs;
  };
  for (int j = 0; j < jn; j += 16) {
    vt sv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {  // 16 rows in flight
      if constexpr (S2) {
        // (a sample past the last selected bin — the last row / column of an even bin count —
        // keeps its taps with value 0, so the taps and their segments are those of the
        // zero-padded 7 x 7 backward: the same sums in the same association)
        const int tr = __builtin_amdgcn_readlane(tl, min(j + u, jn - 1));
        sv[u] = cok && tr >= 0 ? vscale(VF::load(sg + (size_t)tr * C + c), 0.25f) : VF::zero();  // = top / 4.f
      } else {
        const unsigned vu = __builtin_amdgcn_readlane(vl, min(j + u, jn - 1));
        sv[u] = cok ? VF::load(sg + (size_t)(vu >> 2) * C + c) : VF::zero();
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (j + u >= jn) break;
      const unsigned ku = __builtin_amdgcn_readlane(kl, j + u);
      if (ku != cur) {
        flush(false);
        cur = ku;
        a = VF::zero();
      }
      const unsigned vu = __builtin_amdgcn_readlane(vl, j + u);
      const float hr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl.x), j + u));
      const float wr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl.y), j + u));
      vtap(a, sv[u], hr, wr, (int)(vu & 3));
    }
  }
  flush(true);
}

// the runs crossing segments: the owning segment's tail piece, then the next segments' head
// pieces in order (deterministic); V channels per lane as in the gather
template <int V>
__global__ void __launch_bounds__(256) rbg_seg_fixup_kernel(
    const int* __restrict__ start, const unsigned* __restrict__ keys, int C, int ncell,
    const float* __restrict__ carry_head, const float* __restrict__ carry_tail,
    const int* __restrict__ flags, float* __restrict__ acc) {
  using VF = VecF<V>;
  typedef typename VF::T vt;
  const int lane = threadIdx.x & 63;
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = start[ncell];
  if (seg * 64 >= n || !(flags[seg] & 1)) return;
  const int c = (blockIdx.y * 64 + lane) * V;
  const unsigned cell = keys[min(seg * 64 + 64, n) - 1];
  // the run ends in the first later segment not flagged 2: found 64 flags at a time by the
  // lanes (a cell under hundreds of RoIs spans hundreds of segments), then its head pieces
  // summed in order with the loads batched
  int kend = seg + 1;
  for (int kb = seg + 1;; kb += 64) {
    const int k = kb + lane;
    const bool stop = k * 64 >= n || !(flags[k] & 2);
    const unsigned long long m = __ballot(stop);
    if (m) {
      kend = kb + __builtin_ctzll(m);
      break;
    }
  }
  if (kend * 64 >= n) --kend;
  if (c >= C) return;
  vt a = VF::load(carry_tail + (size_t)seg * C + c);
  int k = seg + 1;
  for (; k + 8 <= kend + 1; k += 8) {
    vt h[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) h[u] = VF::load(carry_head + (size_t)(k + u) * C + c);
#pragma unroll
    for (int u = 0; u < 8; ++u) a = vadd(a, h[u]);
  }
  for (; k <= kend; ++k) a = vadd(a, VF::load(carry_head + (size_t)k * C + c));
  VF::store(acc + (size_t)cell * C + c, a);
}

struct RbgWs {
  unsigned *keys, *vals, *keys_s, *vals_s;
  float2* geo;
  int *start, *flags, *trow;
  float *sg, *acc, *carry_head, *carry_tail;
  void* cub_tmp;
  size_t cub_bytes;
};

static size_t carve_rbg(Carve& cv, RbgWs& w, int B, int C, int H, int W, int R, int ph, int pw,
                        bool s2 = false) {
  const size_t S = (size_t)(ph + 1) * (pw + 1), n = (size_t)R * S * 4;
  w.keys = cv.take<unsigned>(n);
  w.vals = cv.take<unsigned>(n);
  w.keys_s = cv.take<unsigned>(n);
  w.vals_s = cv.take<unsigned>(n);
  w.geo = cv.take<float2>((size_t)R * S);
  w.trow = s2 ? cv.take<int>((size_t)R * S) : nullptr;
  w.start = cv.take<int>((size_t)B * H * W + 1);
  w.sg = s2 ? nullptr : cv.take<float>((size_t)R * S * C);
  const size_t nseg = (n + 63) / 64;
  w.acc = cv.take<float>((size_t)B * H * W * C);
  w.carry_head = cv.take<float>(nseg * C);
  w.carry_tail = cv.take<float>(nseg * C);
  w.flags = cv.take<int>(nseg);
  w.cub_bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, w.cub_bytes, (const unsigned*)nullptr,
                                           (unsigned*)nullptr, (const unsigned*)nullptr,
                                           (unsigned*)nullptr, (int)n);
  w.cub_tmp = cv.take<char>(w.cub_bytes);
  return align_up(cv.off, 256);
}

static int rbg_bits(unsigned v) {  // bits needed for keys 0..v
  int b = 1;
  while (b < 32 && (v >> b)) ++b;
  return b;
}

// bottom_grad (B,C,H,W) += acc (B,H,W,C): 64x64 tiles through LDS.
__global__ void __launch_bounds__(256) nhwc_add_to_nchw_kernel(const float* __restrict__ acc,
                                                               int C, int HW,
                                                               float* __restrict__ out) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* a = acc + (size_t)b * HW * C;
  float* o = out + (size_t)b * C * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int p = p0 + i, c = c0 + tx;
    tile[i][tx] = (p < HW && c < C) ? a[(size_t)p * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, p = p0 + tx;
    if (p < HW && c < C) o[(size_t)c * HW + p] += tile[tx][i];
  }
}

// ------------------------------------------------------------ ResNet RoI-head entry
// RCNN_top = layer4, whose first bottleneck subsamples by 2 (lib/DAF/resnet.py:64-102,
// :286-288): of RoIAlignAvg's ph x pw bins it reads only (2i, 2j), channels-last.  So the
// head entry computes exactly those bins, (R, QH, QW, C) with QH = ceil(ph / 2), from a
// channels-last copy of the feature map (every bilinear tap a coalesced row of channels;
// the NCHW kernel's lanes each read a different plane), and none of the 7 x 7 map, its
// permute to channels-last or the strided subsample copy is materialised.  Values are the
// fused NCHW kernel's bit for bit (same samples, same average order).  The bins (2i, 2j)
// cover disjoint 2 x 2 sample blocks, so the backward gives each sample its bin's top / 4
// with no sample-gradient pass (rbg_seg_gather_kernel<true>); the backward is therefore equal
// bit for bit to the 7 x 7 backward of a top gradient that is zero off the selected bins.

// out (B, HW, C) = in (B, C, HW): 64 x 64 tiles through LDS
__global__ void __launch_bounds__(256) nchw_to_nhwc_kernel(const float* __restrict__ in, int C,
                                                           int HW, float* __restrict__ out) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const float* a = in + (size_t)b * C * HW;
  float* o = out + (size_t)b * HW * C;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, p = p0 + tx;
    tile[i][tx] = (p < HW && c < C) ? a[(size_t)c * HW + p] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int p = p0 + i, c = c0 + tx;
    if (p < HW && c < C) o[(size_t)p * C + c] = tile[tx][i];
  }
}

// grid (R, ceil(C / (256 V))): thread = V consecutive channels (16-B loads for V = 4, each
// channel's arithmetic unchanged); out (R, QH, QW, C)
template <int V>
__global__ void __launch_bounds__(256) roi_align_avg_s2_fwd_kernel(
    const float* __restrict__ feat_nhwc, float scale, int C, int H, int W, int ph, int pw,
    const float* __restrict__ rois, float* __restrict__ out) {
  const int ah = ph + 1, aw = pw + 1, QH = (ph + 1) / 2, QW = (pw + 1) / 2;
  const int r = blockIdx.x, t = threadIdx.x, c = (blockIdx.y * 256 + t) * V;
  __shared__ int gy[8], gx[8];
  __shared__ float ghr[8], gwr[8];
  __shared__ bool gvy[8], gvx[8];
  const float* ro = rois + r * 5;
  if (t < ah) align_axis(ro[2] * scale, ro[4] * scale, ah, t, H, &gy[t], &ghr[t], &gvy[t]);
  if (t >= 32 && t < 32 + aw) {
    const int p = t - 32;
    align_axis(ro[1] * scale, ro[3] * scale, aw, p, W, &gx[p], &gwr[p], &gvx[p]);
  }
  __syncthreads();
  if (c >= C) return;
  const float* base = feat_nhwc + (size_t)(int)ro[0] * H * W * C + c;
  float* o = out + (size_t)r * QH * QW * C + c;
  for (int i = 0; i < QH; ++i)
    for (int j = 0; j < QW; ++j) {
      float sv[4][V];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sy = 2 * i + (k >> 1), sx = 2 * j + (k & 1);
        if (gvy[sy] && gvx[sx]) {
          const float* p = base + ((size_t)gy[sy] * W + gx[sx]) * C;
          float ul[V], ur[V], dl[V], dr[V];
          if constexpr (V == 4) {
            const float4 a = *reinterpret_cast<const float4*>(p);
            const float4 b = *reinterpret_cast<const float4*>(p + C);
            const float4 d = *reinterpret_cast<const float4*>(p + (size_t)W * C);
            const float4 e = *reinterpret_cast<const float4*>(p + (size_t)W * C + C);
            ul[0] = a.x; ul[1] = a.y; ul[2] = a.z; ul[3] = a.w;
            ur[0] = b.x; ur[1] = b.y; ur[2] = b.z; ur[3] = b.w;
            dl[0] = d.x; dl[1] = d.y; dl[2] = d.z; dl[3] = d.w;
            dr[0] = e.x; dr[1] = e.y; dr[2] = e.z; dr[3] = e.w;
          } else {
            ul[0] = p[0]; ur[0] = p[C]; dl[0] = p[(size_t)W * C]; dr[0] = p[(size_t)W * C + C];
          }
          const float hr = ghr[sy], wr = gwr[sx];
#pragma unroll
          for (int v = 0; v < V; ++v) {  // (align_sample's arithmetic on the channels-last map)
            const double t1 = ((double)ul[v] * (1. - (double)hr)) * (1. - (double)wr);
            const double t2 = ((double)ur[v] * (1. - (double)hr)) * (double)wr;
            const double t3 = (double)(dl[v] * hr) * (1. - (double)wr);
            const double t4 = (double)((dr[v] * hr) * wr);
            sv[k][v] = (float)(((t1 + t2) + t3) + t4);
          }
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) sv[k][v] = 0.f;
        }
      }
      // avg_pool2d(2, s1) as roi_align_avg_fwd_kernel: ((((0+a)+b)+c)+d)/4
      float res[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float acc = 0.f;
        acc += sv[0][v];
        acc += sv[1][v];
        acc += sv[2][v];
        acc += sv[3][v];
        res[v] = acc / 4.f;
      }
      float* q = o + (size_t)(i * QW + j) * C;
      if constexpr (V == 4) *reinterpret_cast<float4*>(q) = make_float4(res[0], res[1], res[2], res[3]);
      else q[0] = res[0];
    }
}

// ------------------------------------------------------------ RoIPool
__global__ void roi_pool_fwd_kernel(int total, const float* __restrict__ feat, float scale,
                                    int C, int H, int W, int PH, int PW,
                                    const float* __restrict__ rois, float* __restrict__ out,
                                    int32_t* __restrict__ argmax) {
  for (int index = blockIdx.x * blockDim.x + threadIdx.x; index < total;
       index += blockDim.x * gridDim.x) {
    const int pw = index % PW;
    const int ph = (index / PW) % PH;
    const int c = (index / PW / PH) % C;
    const int n = index / PW / PH / C;
    const float* r = rois + n * 5;
    const int b = (int)r[0];
    const int sw = (int)round(r[1] * scale), sh = (int)round(r[2] * scale);
    const int ew = (int)round(r[3] * scale), eh = (int)round(r[4] * scale);
    const int rw = max(ew - sw + 1, 1), rh = max(eh - sh + 1, 1);
    const float bh = (float)rh / (float)PH, bw = (float)rw / (float)PW;
    int hs = (int)floorf((float)ph * bh), ws = (int)floorf((float)pw * bw);
    int he = (int)ceilf((float)(ph + 1) * bh), we = (int)ceilf((float)(pw + 1) * bw);
    hs = min(max(hs + sh, 0), H);
    he = min(max(he + sh, 0), H);
    ws = min(max(ws + sw, 0), W);
    we = min(max(we + sw, 0), W);
    const bool empty = (he <= hs) || (we <= ws);
    float maxval = empty ? 0.f : -FLT_MAX;
    int maxidx = -1;
    const size_t off = ((size_t)b * C + c) * H * W;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        const float v = feat[off + h * W + w];
        if (v > maxval) { maxval = v; maxidx = (int)(off + h * W + w); }
      }
    out[index] = maxval;
    argmax[index] = maxidx;
  }
}

__global__ void roi_pool_bwd_kernel(int total, const float* __restrict__ top,
                                    const int32_t* __restrict__ argmax,
                                    float* __restrict__ grad) {
  for (int index = blockIdx.x * blockDim.x + threadIdx.x; index < total;
       index += blockDim.x * gridDim.x) {
    const int a = argmax[index];
    if (a >= 0) atomicAdd(grad + a, top[index]);
  }
}

static inline int grid_for(int total, int block) { return std::min(div_up(total, block), 256 * 32); }

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_roi_align_fwd_f32(const float* feat, int B, int C, int H, int W,
                                      const float* rois, int R, int ah, int aw, float scale,
                                      float* out, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0 && ah >= 2 && aw >= 2, "bad shape");
  const int total = R * C * ah * aw;
  if (total == 0) return kOk;
  hipLaunchKernelGGL(roi_align_fwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, total, feat, scale, C, H, W, ah, aw, rois, out);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_roi_align_bwd_f32(const float* top_grad, int B, int C, int H, int W,
                                      const float* rois, int R, int ah, int aw, float scale,
                                      float* bottom_grad, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0 && ah >= 2 && aw >= 2, "bad shape");
  const int total = R * C * ah * aw;
  if (total == 0) return kOk;
  hipLaunchKernelGGL(roi_align_bwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, total, top_grad, scale, C, H, W, ah, aw, rois,
                     bottom_grad);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_roi_align_avg_fwd_f32(const float* feat, int B, int C, int H, int W,
                                          const float* rois, int R, int ph, int pw, float scale,
                                          float* out, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0, "bad shape");
  TLOD_CHECK_ARG(ph >= 1 && pw >= 1 && ph <= 7 && pw <= 7, "fused RoIAlignAvg supports 1..7 bins");
  if (R == 0) return kOk;
  hipLaunchKernelGGL(roi_align_avg_fwd_kernel, dim3(div_up(C, kAvgCh), R), dim3(kAvgThreads), 0,
                     (hipStream_t)stream, feat, scale, C, H, W, ph, pw, rois, out);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" size_t tlod_roi_align_avg_bwd_workspace_bytes(int B, int C, int H, int W) {
  return (size_t)B * C * H * W * sizeof(float);
}

// The sorted-tap gather backward is the default; TLOD_ROI_BWD_GATHER=0 (read at every call,
// documented in tlod.h) selects the atomic kernels, and then the gather needs no workspace.
static bool roi_bwd_gather_on() {
  const char* v = getenv("TLOD_ROI_BWD_GATHER");
  return !(v && *v == '0');
}

extern "C" size_t tlod_roi_align_avg_bwd_gather_workspace_bytes(int B, int C, int H, int W, int R,
                                                               int ph, int pw) {
  if (!roi_bwd_gather_on()) return 0;
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || R <= 0 || ph <= 0 || pw <= 0) return 0;
  Carve cv(nullptr, 0);
  RbgWs w;
  return carve_rbg(cv, w, B, C, H, W, R, ph, pw);
}

extern "C" int tlod_roi_align_avg_bwd_f32(const float* top_grad, int B, int C, int H, int W,
                                          const float* rois, int R, int ph, int pw, float scale,
                                          float* bottom_grad, void* ws, size_t ws_bytes,
                                          tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0, "bad shape");
  TLOD_CHECK_ARG(ph >= 1 && pw >= 1 && ph <= 7 && pw <= 7, "fused RoIAlignAvg supports 1..7 bins");
  if (R == 0) return kOk;
  hipStream_t s = (hipStream_t)stream;
  // the sorted-tap gather by default (deterministic); TLOD_ROI_BWD_GATHER=0: the atomic kernels
  const bool gather_off = !roi_bwd_gather_on();
  const size_t ncell_sz = (size_t)B * H * W;
  if (!gather_off && ws != nullptr && ncell_sz < (1u << 31) &&
      ws_bytes >= tlod_roi_align_avg_bwd_gather_workspace_bytes(B, C, H, W, R, ph, pw)) {
    Carve cv(ws, ws_bytes);
    RbgWs w;
    carve_rbg(cv, w, B, C, H, W, R, ph, pw);
    const int S = (ph + 1) * (pw + 1), n = R * S * 4;
    const unsigned ncell = (unsigned)ncell_sz;
    hipLaunchKernelGGL(rbg_geom_kernel, dim3(div_up(R * S, 256)), dim3(256), 0, s, rois, R, scale,
                       H, W, ph, pw, ncell, w.keys, w.vals, w.geo, (int*)nullptr, 0, 0);
    TLOD_LAUNCH_CHECK();
    size_t cb = w.cub_bytes;
    TLOD_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, cb, w.keys, w.keys_s, w.vals, w.vals_s,
                                                n, 0, rbg_bits(ncell), s));
    hipLaunchKernelGGL(rbg_start_kernel, dim3(div_up((int)ncell + 1, 256)), dim3(256), 0, s,
                       w.keys_s, n, ncell, w.start);
    TLOD_LAUNCH_CHECK();
    if (C % 4 == 0)
      hipLaunchKernelGGL(rbg_sample_grad_kernel<4>, dim3(R, div_up(C, 64)), dim3(256), 0, s,
                         top_grad, C, ph, pw, w.sg);
    else
      hipLaunchKernelGGL(rbg_sample_grad_kernel<1>, dim3(R, div_up(C, 64)), dim3(256), 0, s,
                         top_grad, C, ph, pw, w.sg);
    TLOD_LAUNCH_CHECK();
    TLOD_HIP(hipMemsetAsync(w.acc, 0, ncell_sz * C * sizeof(float), s));
    const int nseg = div_up(n, 64);
    if (C % 4 == 0)
      hipLaunchKernelGGL((rbg_seg_gather_kernel<false, 4>), dim3(div_up(nseg, 4), div_up(C, 256)),
                         dim3(256), 0, s, w.start, w.keys_s, w.vals_s, w.geo, w.sg, C, (int)ncell,
                         w.acc, w.carry_head, w.carry_tail, w.flags, (const int*)nullptr);
    else
      hipLaunchKernelGGL((rbg_seg_gather_kernel<false, 1>), dim3(div_up(nseg, 4), div_up(C, 64)),
                         dim3(256), 0, s, w.start, w.keys_s, w.vals_s, w.geo, w.sg, C, (int)ncell,
                         w.acc, w.carry_head, w.carry_tail, w.flags, (const int*)nullptr);
    TLOD_LAUNCH_CHECK();
    if (C % 4 == 0)
      hipLaunchKernelGGL(rbg_seg_fixup_kernel<4>, dim3(div_up(nseg, 4), div_up(C, 256)), dim3(256),
                         0, s, w.start, w.keys_s, C, (int)ncell, w.carry_head, w.carry_tail,
                         w.flags, w.acc);
    else
      hipLaunchKernelGGL(rbg_seg_fixup_kernel<1>, dim3(div_up(nseg, 4), div_up(C, 64)), dim3(256),
                         0, s, w.start, w.keys_s, C, (int)ncell, w.carry_head, w.carry_tail,
                         w.flags, w.acc);
    TLOD_LAUNCH_CHECK();
    hipLaunchKernelGGL(nhwc_add_to_nchw_kernel, dim3(div_up(H * W, 64), div_up(C, 64), B), dim3(256),
                       0, s, w.acc, C, H * W, bottom_grad);
    TLOD_LAUNCH_CHECK();
    return kOk;
  }
  if (ws == nullptr) {  // no workspace: accumulate straight into NCHW (slow atomic shape)
    hipLaunchKernelGGL(roi_align_avg_bwd_kernel, dim3(div_up(C, kAvgCh), R), dim3(kAvgThreads), 0,
                       s, top_grad, scale, C, H, W, ph, pw, rois, bottom_grad);
    TLOD_LAUNCH_CHECK();
    return kOk;
  }
  if (ws_bytes < (size_t)B * C * H * W * sizeof(float)) {
    set_error("tlod_roi_align_avg_bwd_f32: workspace too small");
    return kWorkspace;
  }
  float* acc = static_cast<float*>(ws);
  TLOD_HIP(hipMemsetAsync(acc, 0, (size_t)B * C * H * W * sizeof(float), s));
  hipLaunchKernelGGL(roi_align_avg_bwd_nhwc_kernel, dim3(div_up(C, kNhwcThreads), R),
                     dim3(kNhwcThreads), 0, s, top_grad, scale, C, H, W, ph, pw, rois, acc);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(nhwc_add_to_nchw_kernel, dim3(div_up(H * W, 64), div_up(C, 64), B), dim3(256),
                     0, s, acc, C, H * W, bottom_grad);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

// ResNet RoI-head entry (see roi_align_avg_s2_fwd_kernel): the forward needs the
// channels-last map (B*H*W*C floats), the backward the gather workspace without its
// sample-gradient rows; one query covers both.
extern "C" size_t tlod_roi_align_avg_s2_workspace_bytes(int B, int C, int H, int W, int R, int ph,
                                                        int pw) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || R <= 0 || ph <= 0 || pw <= 0) return 0;
  Carve cv(nullptr, 0);
  RbgWs w;
  return std::max(carve_rbg(cv, w, B, C, H, W, R, ph, pw, true),
                  align_up((size_t)B * H * W * C * sizeof(float), 256));
}

extern "C" int tlod_roi_align_avg_s2_nhwc_fwd_f32(const float* feat, int B, int C, int H, int W,
                                                  const float* rois, int R, int ph, int pw,
                                                  float scale, float* out, void* ws,
                                                  size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0, "bad shape");
  TLOD_CHECK_ARG(ph >= 1 && pw >= 1 && ph <= 7 && pw <= 7, "fused RoIAlignAvg supports 1..7 bins");
  if (R == 0) return kOk;
  if (ws == nullptr || ws_bytes < (size_t)B * H * W * C * sizeof(float)) {
    set_error("tlod_roi_align_avg_s2_nhwc_fwd_f32: workspace too small");
    return kWorkspace;
  }
  hipStream_t s = (hipStream_t)stream;
  float* fn = static_cast<float*>(ws);
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(div_up(H * W, 64), div_up(C, 64), B), dim3(256), 0,
                     s, feat, C, H * W, fn);
  TLOD_LAUNCH_CHECK();
  if (C % 4 == 0)
    hipLaunchKernelGGL(roi_align_avg_s2_fwd_kernel<4>, dim3(R, div_up(C, 1024)), dim3(256), 0, s, fn,
                       scale, C, H, W, ph, pw, rois, out);
  else
    hipLaunchKernelGGL(roi_align_avg_s2_fwd_kernel<1>, dim3(R, div_up(C, 256)), dim3(256), 0, s, fn,
                       scale, C, H, W, ph, pw, rois, out);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_roi_align_avg_s2_nhwc_bwd_f32(const float* top_grad, int B, int C, int H,
                                                  int W, const float* rois, int R, int ph, int pw,
                                                  float scale, float* bottom_grad, void* ws,
                                                  size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H >= 2 && W >= 2 && R >= 0, "bad shape");
  TLOD_CHECK_ARG(ph >= 1 && pw >= 1 && ph <= 7 && pw <= 7, "fused RoIAlignAvg supports 1..7 bins");
  TLOD_CHECK_ARG((size_t)B * H * W < (1u << 31), "feature map too large");
  if (R == 0) return kOk;
  if (ws == nullptr || ws_bytes < tlod_roi_align_avg_s2_workspace_bytes(B, C, H, W, R, ph, pw)) {
    set_error("tlod_roi_align_avg_s2_nhwc_bwd_f32: workspace too small");
    return kWorkspace;
  }
  hipStream_t s = (hipStream_t)stream;
  Carve cv(ws, ws_bytes);
  RbgWs w;
  carve_rbg(cv, w, B, C, H, W, R, ph, pw, true);
  const int S = (ph + 1) * (pw + 1), n = R * S * 4;
  const int QH = (ph + 1) / 2, QW = (pw + 1) / 2;
  const unsigned ncell = (unsigned)((size_t)B * H * W);
  hipLaunchKernelGGL(rbg_geom_kernel, dim3(div_up(R * S, 256)), dim3(256), 0, s, rois, R, scale, H,
                     W, ph, pw, ncell, w.keys, w.vals, w.geo, w.trow, QH, QW);
  TLOD_LAUNCH_CHECK();
  size_t cb = w.cub_bytes;
  TLOD_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, cb, w.keys, w.keys_s, w.vals, w.vals_s, n,
                                              0, rbg_bits(ncell), s));
  hipLaunchKernelGGL(rbg_start_kernel, dim3(div_up((int)ncell + 1, 256)), dim3(256), 0, s, w.keys_s,
                     n, ncell, w.start);
  TLOD_LAUNCH_CHECK();
  TLOD_HIP(hipMemsetAsync(w.acc, 0, (size_t)ncell * C * sizeof(float), s));
  const int nseg = div_up(n, 64);
  if (C % 4 == 0)
    hipLaunchKernelGGL((rbg_seg_gather_kernel<true, 4>), dim3(div_up(nseg, 4), div_up(C, 256)),
                       dim3(256), 0, s, w.start, w.keys_s, w.vals_s, w.geo, top_grad, C, (int)ncell,
                       w.acc, w.carry_head, w.carry_tail, w.flags, w.trow);
  else
    hipLaunchKernelGGL((rbg_seg_gather_kernel<true, 1>), dim3(div_up(nseg, 4), div_up(C, 64)),
                       dim3(256), 0, s, w.start, w.keys_s, w.vals_s, w.geo, top_grad, C, (int)ncell,
                       w.acc, w.carry_head, w.carry_tail, w.flags, w.trow);
  TLOD_LAUNCH_CHECK();
  if (C % 4 == 0)
    hipLaunchKernelGGL(rbg_seg_fixup_kernel<4>, dim3(div_up(nseg, 4), div_up(C, 256)), dim3(256), 0,
                       s, w.start, w.keys_s, C, (int)ncell, w.carry_head, w.carry_tail, w.flags,
                       w.acc);
  else
    hipLaunchKernelGGL(rbg_seg_fixup_kernel<1>, dim3(div_up(nseg, 4), div_up(C, 64)), dim3(256), 0,
                       s, w.start, w.keys_s, C, (int)ncell, w.carry_head, w.carry_tail, w.flags,
                       w.acc);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(nhwc_add_to_nchw_kernel, dim3(div_up(H * W, 64), div_up(C, 64), B), dim3(256),
                     0, s, w.acc, C, H * W, bottom_grad);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_roi_pool_fwd_f32(const float* feat, int B, int C, int H, int W,
                                     const float* rois, int R, int ph, int pw, float scale,
                                     float* out, int32_t* argmax, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && H > 0 && W > 0 && R >= 0 && ph > 0 && pw > 0, "bad shape");
  TLOD_CHECK_ARG((size_t)B * C * H * W < (1ull << 31), "feature map too large for int32 argmax");
  const int total = R * C * ph * pw;
  if (total == 0) return kOk;
  hipLaunchKernelGGL(roi_pool_fwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, total, feat, scale, C, H, W, ph, pw, rois, out, argmax);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_roi_pool_bwd_f32(const float* top_grad, const int32_t* argmax, int R, int C,
                                     int ph, int pw, float* bottom_grad, tlod_stream_t stream) {
  TLOD_CHECK_ARG(R >= 0 && C > 0 && ph > 0 && pw > 0, "bad shape");
  const int total = R * C * ph * pw;
  if (total == 0) return kOk;
  hipLaunchKernelGGL(roi_pool_bwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, total, top_grad, argmax, bottom_grad);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
