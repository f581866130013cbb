// RPN anchor-target and R-CNN proposal-target assignment on device (gfx950).
//
// Replaces the pure torch/numpy host code of
//   _AnchorTargetLayer.forward   lib/model/rpn/anchor_target_layer.py:48-193
//   _ProposalTargetLayer.forward lib/model/rpn/proposal_target_layer_cascade.py:33-212
// which sync the host (nonzero, .item(), numpy RNG, Python loops) several times per
// step.  Here every stage is a kernel; the only optional host round trip is the
// explicit-permutation mode used to replay the reference's numpy draws in parity tests.
//
// IoU: bbox_overlaps_batch (lib/model/rpn/bbox_transform.py:168-257) including its
// masks (zero-area gt -> 0, zero-area anchor -> -1), one rounding per op
// (-ffp-contract=off) so overlaps and the `overlaps == gt_max` tie test are bit-exact.
#include <cmath>

#include "common.h"
#include "tlod.h"

namespace tlod {

constexpr int kBlk = 1024;   // single-workgroup phases
constexpr int kMaxG = 128;   // gt boxes per image

// bbox_overlaps_batch for one (box, gt) pair; box areas precomputed by the caller.
__device__ __forceinline__ float overlap(float ax1, float ay1, float ax2, float ay2, float aarea,
                                         bool azero, float gx1, float gy1, float gx2, float gy2,
                                         float garea, bool gzero) {
  if (azero) return -1.f;  // masked last (bbox_transform.py:210)
  if (gzero) return 0.f;
  float iw = fminf(ax2, gx2) - fmaxf(ax1, gx1) + 1.f;
  if (iw < 0.f) iw = 0.f;
  float ih = fminf(ay2, gy2) - fmaxf(ay1, gy1) + 1.f;
  if (ih < 0.f) ih = 0.f;
  const float ua = aarea + garea - iw * ih;
  return iw * ih / ua;
}

struct GtLds {
  float x1[kMaxG], y1[kMaxG], x2[kMaxG], y2[kMaxG], area[kMaxG];
  bool zero[kMaxG];
};

__device__ __forceinline__ void load_gts(GtLds& s, const float* __restrict__ gt, int G) {
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    const float* p = gt + g * 5;
    const float gx = p[2] - p[0] + 1.f, gy = p[3] - p[1] + 1.f;
    s.x1[g] = p[0]; s.y1[g] = p[1]; s.x2[g] = p[2]; s.y2[g] = p[3];
    s.area[g] = gx * gy;
    s.zero[g] = (gx == 1.f) && (gy == 1.f);
  }
}

// bbox_transform_batch (bbox_transform.py:36-75) for one pair.
__device__ __forceinline__ void box_delta(float ex1, float ey1, float ex2, float ey2, float gx1,
                                          float gy1, float gx2, float gy2, float* t) {
  const float ew = ex2 - ex1 + 1.0f, eh = ey2 - ey1 + 1.0f;
  const float ecx = ex1 + 0.5f * ew, ecy = ey1 + 0.5f * eh;
  const float gw = gx2 - gx1 + 1.0f, gh = gy2 - gy1 + 1.0f;
  const float gcx = gx1 + 0.5f * gw, gcy = gy1 + 0.5f * gh;
  t[0] = (gcx - ecx) / ew;
  t[1] = (gcy - ecy) / eh;
  t[2] = logf(gw / ew);
  t[3] = logf(gh / eh);
}

// ------------------------------------------------------------ block scan helpers
// Exclusive prefix sum over a 1024-thread block; returns the block total in *total.
__device__ int block_excl_scan(int v, int* total) {
  __shared__ int wsum[kBlk / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    int s = (lane < kBlk / 64) ? wsum[lane] : 0;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(s, o);
      if (lane >= o) s += y;
    }
    if (lane < kBlk / 64) wsum[lane] = s;  // inclusive per-wave prefix
  }
  __syncthreads();
  const int before = (wid > 0) ? wsum[wid - 1] : 0;
  *total = wsum[kBlk / 64 - 1];
  __syncthreads();
  return before + x - v;
}

__device__ int block_sum(int v) {
  int total;
  block_excl_scan(v, &total);
  return total;
}

// Stable compaction of the indices i in [0, n) with pred(i) into out[] (index order).
template <class Pred>
__device__ int block_compact(int n, Pred pred, int32_t* __restrict__ out) {
  const int per = (n + kBlk - 1) / kBlk;
  const int lo = min(n, (int)threadIdx.x * per), hi = min(n, lo + per);
  int c = 0;
  for (int i = lo; i < hi; ++i) c += pred(i) ? 1 : 0;
  int total;
  int pos = block_excl_scan(c, &total);
  for (int i = lo; i < hi; ++i)
    if (pred(i)) out[pos++] = i;
  __syncthreads();
  return total;
}

// Pick, uniformly at random, `m` of the `n` list entries (keys = rng(seed, stream,
// list[i])); calls act(list[i]) for each picked entry.  Radix select on 32-bit keys
// with index-order tie break — the device stand-in for list[perm[:m]] with
// perm = np.random.permutation(n).
template <class Act>
__device__ void block_random_subset(const int32_t* __restrict__ list, int n, int m,
                                    uint64_t seed, uint64_t stream, Act act) {
  if (m <= 0) return;
  if (m >= n) {
    for (int i = threadIdx.x; i < n; i += kBlk) act(list[i]);
    __syncthreads();
    return;
  }
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_need;
  if (threadIdx.x == 0) { s_prefix = 0; s_need = m; }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += kBlk) hist[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const uint32_t pmask = pass == 0 ? 0u : (0xffffffffu << (32 - 8 * pass));
    for (int i = threadIdx.x; i < n; i += kBlk) {
      const uint32_t k = (uint32_t)(rng_u64(seed, stream, (uint64_t)list[i]) >> 32);
      if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      // the first digit d whose cumulative count reaches `need`: one wave, lane l owning
      // digits 4l..4l+3 (a wave scan instead of a 256-step serial LDS walk on one lane —
      // that walk was most of this kernel's time)
      const int l = threadIdx.x, need = s_need;
      const int h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
      const int sl = h0 + h1 + h2 + h3;
      int incl = sl;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (l >= o) incl += y;
      }
      int acc = incl - sl;
      if (acc < need && need <= incl) {  // exactly one lane
        int d = 4 * l;
        if (acc + h0 < need) { acc += h0; ++d;
          if (acc + h1 < need) { acc += h1; ++d;
            if (acc + h2 < need) { acc += h2; ++d; } } }
        s_need = need - acc;
        s_prefix = prefix | ((uint32_t)d << shift);
      }
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix;
  const int need_eq = s_need;  // how many keys == T to pick (in list order)
  // keys < T are picked; keys == T: the first need_eq in list order.
  const int per = (n + kBlk - 1) / kBlk;
  const int lo = min(n, (int)threadIdx.x * per), hi = min(n, lo + per);
  int c = 0;
  for (int i = lo; i < hi; ++i)
    c += ((uint32_t)(rng_u64(seed, stream, (uint64_t)list[i]) >> 32) == T) ? 1 : 0;
  int total;
  int rank = block_excl_scan(c, &total);
  for (int i = lo; i < hi; ++i) {
    const uint32_t k = (uint32_t)(rng_u64(seed, stream, (uint64_t)list[i]) >> 32);
    if (k < T) act(list[i]);
    else if (k == T) { if (rank < need_eq) act(list[i]); ++rank; }
  }
  __syncthreads();
}

// ============================================================ anchor target
struct AtWs {
  float* maxov; int32_t* argmax; int8_t* label; uint32_t* gtmax; int32_t* list; int32_t* nex;
};

static void carve_at(Carve& c, AtWs& w, int B, int N, int G) {
  w.maxov = c.take<float>((size_t)B * N);
  w.argmax = c.take<int32_t>((size_t)B * N);
  w.label = c.take<int8_t>((size_t)B * N);
  w.gtmax = c.take<uint32_t>((size_t)B * G);
  w.list = c.take<int32_t>((size_t)B * N);
  w.nex = c.take<int32_t>(B);
}

struct AnchorGeo {
  const float* base; int A, H, W, stride;
  __device__ __forceinline__ void box(int idx, float* b) const {
    const int a = idx % A, hw = idx / A;
    const float sx = (float)((hw % W) * stride), sy = (float)((hw / W) * stride);
    b[0] = base[a * 4 + 0] + sx; b[1] = base[a * 4 + 1] + sy;
    b[2] = base[a * 4 + 2] + sx; b[3] = base[a * 4 + 3] + sy;
  }
};

__device__ __forceinline__ bool anchor_inside(const float* b, float imw, float imh, int border) {
  // anchor_target_layer.py:83-87: long(im_info[0][1]) truncates
  const float lw = (float)(long long)imw, lh = (float)(long long)imh;
  return b[0] >= (float)-border && b[1] >= (float)-border && b[2] < lw + (float)border &&
         b[3] < lh + (float)border;
}

__global__ void at_init_kernel(uint32_t* gtmax, int n, int32_t* counts, int nc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) gtmax[i] = f2ord(-INFINITY);
  if (i < nc) counts[i] = 0;
}

// grid (ceil(N/256), B): max/argmax over gts per inside anchor; per-gt max over anchors.
__global__ void __launch_bounds__(256) at_iou_kernel(AnchorGeo geo, const float* __restrict__ gt,
                                                     int G, const float* __restrict__ im_info,
                                                     int border, float* __restrict__ maxov,
                                                     int32_t* __restrict__ argmax,
                                                     uint32_t* __restrict__ gtmax) {
  __shared__ GtLds s;
  __shared__ uint32_t bmax[kMaxG];
  const int b = blockIdx.y, N = geo.H * geo.W * geo.A;
  load_gts(s, gt + (size_t)b * G * 5, G);
  for (int g = threadIdx.x; g < G; g += blockDim.x) bmax[g] = f2ord(-INFINITY);
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  bool ins = false;
  if (idx < N) {
    geo.box(idx, a);
    ins = anchor_inside(a, im_info[1], im_info[0], border);
  }
  // wave-uniform loop: each gt's max over the wave's inside anchors is reduced across the
  // 64 lanes first (max is order-free: same result as per-anchor atomics), then one LDS
  // atomic per wave instead of 64 contending on the same address
  const float ax = a[2] - a[0] + 1.f, ay = a[3] - a[1] + 1.f;
  const float area = ax * ay;
  const bool az = (ax == 1.f) && (ay == 1.f);
  const uint32_t kNone = f2ord(-INFINITY);
  float best = 0.f;
  int barg = 0;
  for (int g = 0; g < G; ++g) {
    const float o = overlap(a[0], a[1], a[2], a[3], area, az, s.x1[g], s.y1[g], s.x2[g],
                            s.y2[g], s.area[g], s.zero[g]);
    if (g == 0 || o > best) { best = o; barg = g; }
    uint32_t v = ins ? f2ord(o) : kNone;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    if ((threadIdx.x & 63) == 0 && v != kNone) atomicMax(&bmax[g], v);
  }
  if (ins) {
    maxov[(size_t)b * N + idx] = best;
    argmax[(size_t)b * N + idx] = barg;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += blockDim.x)
    if (bmax[g] != f2ord(-INFINITY)) atomicMax(&gtmax[(size_t)b * G + g], bmax[g]);
}

// grid (ceil(N/256), B): pre-sampling labels (anchor_target_layer.py:100-116).
__global__ void __launch_bounds__(256) at_label_kernel(AnchorGeo geo, const float* __restrict__ gt,
                                                       int G, const float* __restrict__ im_info,
                                                       tlod_rpn_cfg cfg,
                                                       const float* __restrict__ maxov,
                                                       const uint32_t* __restrict__ gtmax,
                                                       int8_t* __restrict__ label,
                                                       int32_t* __restrict__ counts) {
  __shared__ GtLds s;
  __shared__ float gm[kMaxG];
  __shared__ int cnt[2];
  const int b = blockIdx.y, N = geo.H * geo.W * geo.A;
  load_gts(s, gt + (size_t)b * G * 5, G);
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    float v = ord2f(gtmax[(size_t)b * G + g]);
    gm[g] = (v == 0.f) ? 1e-5f : v;  // gt_max_overlaps[gt_max_overlaps==0] = 1e-5
  }
  if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  int lab = -2;  // past the end: counts nowhere
  if (idx < N) {
    float a[4];
    geo.box(idx, a);
    int8_t l = -1;
    if (anchor_inside(a, im_info[1], im_info[0], cfg.allowed_border)) {
      const float mo = maxov[(size_t)b * N + idx];
      if (!cfg.clobber_positives && mo < cfg.neg_overlap) l = 0;
      const float ax = a[2] - a[0] + 1.f, ay = a[3] - a[1] + 1.f;
      const float area = ax * ay;
      const bool az = (ax == 1.f) && (ay == 1.f);
      bool tie = false;
      for (int g = 0; g < G && !tie; ++g)
        tie = overlap(a[0], a[1], a[2], a[3], area, az, s.x1[g], s.y1[g], s.x2[g], s.y2[g],
                      s.area[g], s.zero[g]) == gm[g];
      if (tie) l = 1;
      if (mo >= cfg.pos_overlap) l = 1;
      if (cfg.clobber_positives && mo < cfg.neg_overlap) l = 0;
    }
    label[(size_t)b * N + idx] = l;
    lab = l;
  }
  // per-wave ballot counts: one LDS atomic per wave and class
  const int n1 = __popcll(__ballot(lab == 1)), n0 = __popcll(__ballot(lab == 0));
  if ((threadIdx.x & 63) == 0) {
    if (n1) atomicAdd(&cnt[0], n1);
    if (n0) atomicAdd(&cnt[1], n0);
  }
  __syncthreads();
  if (threadIdx.x < 2 && cnt[threadIdx.x]) atomicAdd(&counts[b * 2 + threadIdx.x], cnt[threadIdx.x]);
}

// grid B, 1024 threads: fg/bg subsampling (anchor_target_layer.py:118-145).
__global__ void __launch_bounds__(kBlk) at_sample_kernel(int N, tlod_rpn_cfg cfg,
                                                         const int32_t* __restrict__ perm,
                                                         const int32_t* __restrict__ perm_off,
                                                         uint64_t seed, int8_t* __restrict__ label_all,
                                                         int32_t* __restrict__ list_all,
                                                         int32_t* __restrict__ nex) {
  const int b = blockIdx.x;
  int8_t* label = label_all + (size_t)b * N;
  int32_t* list = list_all + (size_t)b * N;
  const int num_fg = (int)(cfg.fg_fraction * (float)cfg.batch_size);
  // fg
  int nfg = block_compact(N, [&](int i) { return label[i] == 1; }, list);
  if (nfg > num_fg) {
    const int m = nfg - num_fg;
    if (perm) {
      const int32_t* p = perm + perm_off[2 * b];
      for (int q = threadIdx.x; q < m; q += kBlk) label[list[p[q]]] = -1;
      __syncthreads();
    } else {
      block_random_subset(list, nfg, m, seed, 2ull * b, [&](int i) { label[i] = -1; });
    }
  }
  const int fg_now = nfg > num_fg ? num_fg : nfg;
  const int num_bg = cfg.batch_size - fg_now;
  int nbg = block_compact(N, [&](int i) { return label[i] == 0; }, list);
  if (nbg > num_bg) {
    const int m = nbg - num_bg;
    if (perm) {
      const int32_t* p = perm + perm_off[2 * b + 1];
      for (int q = threadIdx.x; q < m; q += kBlk) label[list[p[q]]] = -1;
      __syncthreads();
    } else {
      block_random_subset(list, nbg, m, seed, 2ull * b + 1, [&](int i) { label[i] = -1; });
    }
  }
  __syncthreads();
  int c = 0;
  for (int i = threadIdx.x; i < N; i += kBlk) c += label[i] >= 0 ? 1 : 0;
  c = block_sum(c);
  if (threadIdx.x == 0) nex[b] = c;
}

// The same subsampling with the labels held as per-thread bitmasks and the candidates' keys
// in LDS (N <= kAtMax anchors, device RNG): thread t owns anchors t + kBlk j, so every label
// is read and written once, coalesced, and every key is hashed once — the list-based kernel
// above re-reads the list from memory and re-hashes every candidate in each of its six
// passes, a chain of dependent loads that made it ~85 us of the step's critical path.  Same
// result: the m picked candidates are the m smallest (key, anchor index) pairs — keys below
// the radix-selected threshold T, then the need_eq smallest anchor indices among keys == T
// (block_random_subset takes ties in list order, which is anchor order).
constexpr int kAtSlots = 38;                  // anchors per thread (keys: 152 KB of LDS)
constexpr int kAtMax = kBlk * kAtSlots;       // 38912 (12 x 38 x 75 = 34200 at 600 x 1200)

template <class Act>
__device__ void lds_random_subset(const uint32_t* __restrict__ skey, uint64_t cand, int n, int m,
                                  Act act) {
  if (m <= 0) return;
  const int t = threadIdx.x;
  if (m >= n) {
#pragma unroll
    for (int j = 0; j < kAtSlots; ++j)
      if ((cand >> j) & 1ull) act(j);
    return;
  }
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_need, s_min;
  if (t == 0) { s_prefix = 0; s_need = m; }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (t < 256) hist[t] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const uint32_t pmask = pass == 0 ? 0u : (0xffffffffu << (32 - 8 * pass));
#pragma unroll 8
    for (int j = 0; j < kAtSlots; ++j) {
      const uint32_t k = skey[j * kBlk + t];
      if (((cand >> j) & 1ull) && (k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
    }
    __syncthreads();
    if (t < 64) {  // the digit whose cumulative count reaches `need` (as block_random_subset)
      const int need = s_need;
      const int h0 = hist[4 * t], h1 = hist[4 * t + 1], h2 = hist[4 * t + 2], h3 = hist[4 * t + 3];
      const int sl = h0 + h1 + h2 + h3;
      int incl = sl;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (t >= o) incl += y;
      }
      int acc = incl - sl;
      if (acc < need && need <= incl) {
        int d = 4 * t;
        if (acc + h0 < need) { acc += h0; ++d;
          if (acc + h1 < need) { acc += h1; ++d;
            if (acc + h2 < need) { acc += h2; ++d; } } }
        s_need = need - acc;
        s_prefix = prefix | ((uint32_t)d << shift);
      }
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix;
  int need_eq = s_need;
  uint64_t tie = 0;
#pragma unroll
  for (int j = 0; j < kAtSlots; ++j) {
    if (!((cand >> j) & 1ull)) continue;
    const uint32_t k = skey[j * kBlk + t];
    if (k < T) act(j);
    else if (k == T) tie |= 1ull << j;
  }
  if (block_sum(__popcll(tie)) <= need_eq) {  // (the common case: every tie is picked)
#pragma unroll
    for (int j = 0; j < kAtSlots; ++j)
      if ((tie >> j) & 1ull) act(j);
    return;
  }
  for (; need_eq > 0; --need_eq) {  // the smallest anchor indices among the ties, one by one
    if (t == 0) s_min = 0x7fffffff;
    __syncthreads();
    if (tie) atomicMin(&s_min, t + kBlk * (__ffsll((unsigned long long)tie) - 1));
    __syncthreads();
    const int w = s_min;
    if (w % kBlk == t) {
#pragma unroll
      for (int j = 0; j < kAtSlots; ++j)  // (static slot indices: the caller's masks stay in registers)
        if (j == w / kBlk) act(j);
      tie &= ~(1ull << (w / kBlk));
    }
    __syncthreads();
  }
}

// dynamic LDS: kBlk * kAtSlots keys
__global__ void __launch_bounds__(kBlk) at_sample_lds_kernel(int N, tlod_rpn_cfg cfg, uint64_t seed,
                                                             int8_t* __restrict__ label_all,
                                                             int32_t* __restrict__ nex) {
  extern __shared__ uint32_t skey[];
  const int b = blockIdx.x, t = threadIdx.x;
  int8_t* label = label_all + (size_t)b * N;
  uint64_t fgm = 0, bgm = 0;  // slot j: label 1 / label 0 (else -1)
#pragma unroll
  for (int j = 0; j < kAtSlots; ++j) {
    const int i = t + kBlk * j;
    const int l = i < N ? label[i] : -1;
    fgm |= (uint64_t)(l == 1) << j;
    bgm |= (uint64_t)(l == 0) << j;
  }
  const int num_fg = (int)(cfg.fg_fraction * (float)cfg.batch_size);
  const int nfg = block_sum(__popcll(fgm));
  if (nfg > num_fg) {
#pragma unroll 4
    for (int j = 0; j < kAtSlots; ++j)
      if ((fgm >> j) & 1ull)
        skey[j * kBlk + t] = (uint32_t)(rng_u64(seed, 2ull * b, (uint64_t)(t + kBlk * j)) >> 32);
    lds_random_subset(skey, fgm, nfg, nfg - num_fg, [&](int j) { fgm &= ~(1ull << j); });
    __syncthreads();
  }
  const int num_bg = cfg.batch_size - (nfg > num_fg ? num_fg : nfg);
  const int nbg = block_sum(__popcll(bgm));
  if (nbg > num_bg) {
#pragma unroll 4
    for (int j = 0; j < kAtSlots; ++j)
      if ((bgm >> j) & 1ull)
        skey[j * kBlk + t] = (uint32_t)(rng_u64(seed, 2ull * b + 1, (uint64_t)(t + kBlk * j)) >> 32);
    lds_random_subset(skey, bgm, nbg, nbg - num_bg, [&](int j) { bgm &= ~(1ull << j); });
  }
#pragma unroll
  for (int j = 0; j < kAtSlots; ++j) {
    const int i = t + kBlk * j;
    if (i < N) label[i] = (int8_t)(((fgm >> j) & 1ull) ? 1 : (((bgm >> j) & 1ull) ? 0 : -1));
  }
  const int c = block_sum(__popcll(fgm) + __popcll(bgm));
  if (t == 0) nex[b] = c;
}

// grid (ceil(N/256), B): targets, weights, unmap, output layouts (:147-191).
__global__ void __launch_bounds__(256) at_output_kernel(
    AnchorGeo geo, const float* __restrict__ gt, int G, int B, float inside_weight,
    const int8_t* __restrict__ label, const int32_t* __restrict__ argmax,
    const int32_t* __restrict__ nex, float* __restrict__ labels_out, float* __restrict__ targets,
    float* __restrict__ inside_w, float* __restrict__ outside_w) {
  const int b = blockIdx.y, A = geo.A, H = geo.H, W = geo.W, N = H * W * A;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N) return;
  const int a = idx % A, hw = idx / A;
  const size_t HW = (size_t)H * W;
  const int8_t l = label[(size_t)b * N + idx];
  // num_examples of the LAST image (the loop variable i leaks, :154).
  const float wgt = (float)(1.0 / (double)nex[B - 1]);
  labels_out[(size_t)b * A * HW + a * HW + hw] = (float)l;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  float a4[4];
  geo.box(idx, a4);
  // targets exist for every inside anchor (bg ones too); outside -> 0 (the _unmap fill).
  // at_iou_kernel leaves argmax = -1 for outside anchors.
  const bool inside = argmax[(size_t)b * N + idx] >= 0;
  if (inside) {
    const float* g = gt + ((size_t)b * G + argmax[(size_t)b * N + idx]) * 5;
    box_delta(a4[0], a4[1], a4[2], a4[3], g[0], g[1], g[2], g[3], t);
  }
  const float iw = (l == 1) ? inside_weight : 0.f;
  const float ow = (l == 1 || l == 0) ? wgt : 0.f;
  const size_t base = (size_t)b * 4 * A * HW + (size_t)(4 * a) * HW + hw;
  for (int k = 0; k < 4; ++k) {
    targets[base + k * HW] = t[k];
    inside_w[base + k * HW] = iw;
    outside_w[base + k * HW] = ow;
  }
}

// ============================================================ proposal target
struct PtWs { float* maxov; int32_t* assign; int32_t* fg; int32_t* bg; int32_t* keep; };

static void carve_pt(Carve& c, PtWs& w, int B, int R, int G, int S) {
  const size_t n = (size_t)B * (R + G);
  w.maxov = c.take<float>(n);
  w.assign = c.take<int32_t>(n);
  w.fg = c.take<int32_t>(n);
  w.bg = c.take<int32_t>(n);
  w.keep = c.take<int32_t>((size_t)B * S);
}

__device__ __forceinline__ void pt_box(const float* rois, const float* gt, int R, int j, float* b) {
  if (j < R) {
    const float* p = rois + (size_t)j * 5 + 1;
    b[0] = p[0]; b[1] = p[1]; b[2] = p[2]; b[3] = p[3];
  } else {  // gt_boxes_append[:,:,1:5] = gt_boxes[:,:,:4]  (:39-43)
    const float* p = gt + (size_t)(j - R) * 5;
    b[0] = p[0]; b[1] = p[1]; b[2] = p[2]; b[3] = p[3];
  }
}

// grid B, 1024 threads: overlaps of all_rois vs gt (:122), candidate counts.
__global__ void __launch_bounds__(kBlk) pt_count_kernel(const float* __restrict__ rois_all, int R,
                                                        const float* __restrict__ gt_all, int G,
                                                        tlod_rcnn_cfg cfg, float* __restrict__ maxov_all,
                                                        int32_t* __restrict__ assign_all,
                                                        int32_t* __restrict__ counts) {
  __shared__ GtLds s;
  const int b = blockIdx.x, M = R + G;
  const float* rois = rois_all + (size_t)b * R * 5;
  const float* gt = gt_all + (size_t)b * G * 5;
  load_gts(s, gt, G);
  __syncthreads();
  int nf = 0, nb = 0;
  for (int j = threadIdx.x; j < M; j += kBlk) {
    float a[4];
    pt_box(rois, gt, R, j, a);
    const float ax = a[2] - a[0] + 1.f, ay = a[3] - a[1] + 1.f;
    const float area = ax * ay;
    const bool az = (ax == 1.f) && (ay == 1.f);
    float best = 0.f;
    int barg = 0;
    for (int g = 0; g < G; ++g) {
      const float o = overlap(a[0], a[1], a[2], a[3], area, az, s.x1[g], s.y1[g], s.x2[g],
                              s.y2[g], s.area[g], s.zero[g]);
      if (g == 0 || o > best) { best = o; barg = g; }
    }
    maxov_all[(size_t)b * M + j] = best;
    assign_all[(size_t)b * M + j] = barg;
    nf += best >= cfg.fg_thresh ? 1 : 0;
    nb += (best < cfg.bg_thresh_hi && best >= cfg.bg_thresh_lo) ? 1 : 0;
  }
  nf = block_sum(nf);
  nb = block_sum(nb);
  if (threadIdx.x == 0) { counts[b * 2] = nf; counts[b * 2 + 1] = nb; }
}

constexpr int kMaxSortPt = 4096;

// grid B, 1024 threads: sampling (:140-204), targets (:206-207) and outputs.
__global__ void __launch_bounds__(kBlk) pt_sample_kernel(
    const float* __restrict__ rois_all, int R, const float* __restrict__ gt_all, int G,
    tlod_rcnn_cfg cfg, int fg_per, const float* __restrict__ maxov_all,
    const int32_t* __restrict__ assign_all, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ perm_off, const double* __restrict__ rnd,
    const int32_t* __restrict__ rnd_off, uint64_t seed, int32_t* __restrict__ fg_all,
    int32_t* __restrict__ bg_all, int32_t* __restrict__ keep_all, float* __restrict__ rois_out,
    float* __restrict__ labels, float* __restrict__ targets, float* __restrict__ inside_w,
    float* __restrict__ outside_w) {
  __shared__ unsigned long long skeys[kMaxSortPt];
  __shared__ int s_fg_this;
  const int b = blockIdx.x, M = R + G, S = cfg.batch_size;
  const float* rois = rois_all + (size_t)b * R * 5;
  const float* gt = gt_all + (size_t)b * G * 5;
  const float* maxov = maxov_all + (size_t)b * M;
  const int32_t* assign = assign_all + (size_t)b * M;
  int32_t* fgl = fg_all + (size_t)b * M;
  int32_t* bgl = bg_all + (size_t)b * M;
  int32_t* keep = keep_all + (size_t)b * S;
  const int nfg = block_compact(M, [&](int j) { return maxov[j] >= cfg.fg_thresh; }, fgl);
  const int nbg = block_compact(
      M, [&](int j) { return maxov[j] < cfg.bg_thresh_hi && maxov[j] >= cfg.bg_thresh_lo; }, bgl);
  const uint64_t st_fg = 16ull + 2 * b, st_bg = 17ull + 2 * b;
  int fg_this;
  if (nfg > 0 && nbg > 0) {
    fg_this = min(fg_per, nfg);
    if (perm) {
      const int32_t* p = perm + perm_off[b];
      for (int q = threadIdx.x; q < fg_this; q += kBlk) keep[q] = fgl[p[q]];
    } else {
      // random order of a random subset: sort (key, position) and take the first fg_this
      int P = 1;
      while (P < nfg) P <<= 1;
      for (int i = threadIdx.x; i < P; i += kBlk)
        skeys[i] = (i < nfg) ? ((rng_u64(seed, st_fg, (uint64_t)i) & 0xffffffff00000000ull) |
                                (unsigned long long)i)
                             : ~0ull;
      __syncthreads();
      for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = threadIdx.x; i < P; i += kBlk) {
            const int l = i ^ j;
            if (l > i) {
              const unsigned long long x = skeys[i], y = skeys[l];
              const bool up = (i & k) == 0;
              if ((x > y) == up) { skeys[i] = y; skeys[l] = x; }
            }
          }
          __syncthreads();
        }
      for (int q = threadIdx.x; q < fg_this; q += kBlk) keep[q] = fgl[(int)(skeys[q] & 0xffffffffull)];
    }
    const int bg_this = S - fg_this;
    for (int q = threadIdx.x; q < bg_this; q += kBlk) {
      const double u = rnd ? rnd[rnd_off[b] + q] : rng_unit(seed, st_bg, (uint64_t)q);
      keep[fg_this + q] = bgl[(int)floor(u * (double)nbg)];
    }
  } else if (nfg > 0) {
    fg_this = S;
    for (int q = threadIdx.x; q < S; q += kBlk) {
      const double u = rnd ? rnd[rnd_off[b] + q] : rng_unit(seed, st_fg, (uint64_t)q);
      keep[q] = fgl[(int)floor(u * (double)nfg)];
    }
  } else if (nbg > 0) {
    fg_this = 0;
    for (int q = threadIdx.x; q < S; q += kBlk) {
      const double u = rnd ? rnd[rnd_off[b] + q] : rng_unit(seed, st_bg, (uint64_t)q);
      keep[q] = bgl[(int)floor(u * (double)nbg)];
    }
  } else {
    fg_this = -1;  // reference raises ValueError; emit an all-background, zero-roi sample
  }
  if (threadIdx.x == 0) s_fg_this = fg_this;
  __syncthreads();
  fg_this = s_fg_this;
  for (int q = threadIdx.x; q < S; q += kBlk) {
    float* ro = rois_out + ((size_t)b * S + q) * 5;
    float* tg = targets + ((size_t)b * S + q) * 4;
    float* iw = inside_w + ((size_t)b * S + q) * 4;
    float* ow = outside_w + ((size_t)b * S + q) * 4;
    if (fg_this < 0) {
      ro[0] = (float)b; ro[1] = ro[2] = ro[3] = ro[4] = 0.f;
      labels[(size_t)b * S + q] = 0.f;
      for (int k = 0; k < 4; ++k) { tg[k] = 0.f; iw[k] = 0.f; ow[k] = 0.f; }
      continue;
    }
    const int j = keep[q];
    float box[4];
    pt_box(rois, gt, R, j, box);
    ro[0] = (float)b; ro[1] = box[0]; ro[2] = box[1]; ro[3] = box[2]; ro[4] = box[3];
    const float* g = gt + (size_t)assign[j] * 5;
    const float lab = (q < fg_this) ? g[4] : 0.f;
    labels[(size_t)b * S + q] = lab;
    if (lab > 0.f) {
      float t[4];
      box_delta(box[0], box[1], box[2], box[3], g[0], g[1], g[2], g[3], t);
      for (int k = 0; k < 4; ++k) {
        tg[k] = (t[k] - cfg.means[k]) / cfg.stds[k];
        iw[k] = cfg.inside_weight[k];
        ow[k] = cfg.inside_weight[k] > 0.f ? 1.f : 0.f;
      }
    } else {
      for (int k = 0; k < 4; ++k) { tg[k] = 0.f; iw[k] = 0.f; ow[k] = 0.f; }
    }
  }
}

}  // namespace tlod

using namespace tlod;

// ------------------------------------------------------------ anchor target ABI
extern "C" size_t tlod_anchor_target_workspace_bytes(int B, int A, int H, int W, int G) {
  Carve c(nullptr, 0);
  AtWs w;
  carve_at(c, w, B, A * H * W, G);
  return align_up(c.off, 256);
}

static int at_check(int A, int H, int W, int B, int G, const tlod_rpn_cfg* cfg) {
  TLOD_CHECK_ARG(A > 0 && H > 0 && W > 0 && B > 0, "bad shape");
  TLOD_CHECK_ARG(G > 0 && G <= kMaxG, "G must be in 1..128");
  TLOD_CHECK_ARG(cfg != nullptr, "cfg is NULL");
  return kOk;
}

extern "C" int tlod_anchor_target_label_f32(const float* base_anchors, int A, int H, int W,
                                            int feat_stride, const float* gt_boxes, int B, int G,
                                            const float* im_info, const tlod_rpn_cfg* cfg,
                                            int32_t* counts, void* ws, size_t ws_bytes,
                                            tlod_stream_t stream) {
  int st = at_check(A, H, W, B, G, cfg);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  const int N = A * H * W;
  Carve c(ws, ws_bytes);
  AtWs w;
  carve_at(c, w, B, N, G);
  if (!c.ok()) { set_error("tlod_anchor_target: workspace too small"); return kWorkspace; }
  AnchorGeo geo{base_anchors, A, H, W, feat_stride};
  const int ninit = std::max(B * G, B * 2);
  hipLaunchKernelGGL(at_init_kernel, dim3(div_up(ninit, 256)), dim3(256), 0, s, w.gtmax, B * G,
                     counts, B * 2);
  TLOD_LAUNCH_CHECK();
  // argmax = -1 marks "outside" for the output kernel.
  TLOD_HIP(hipMemsetAsync(w.argmax, 0xff, sizeof(int32_t) * (size_t)B * N, s));
  hipLaunchKernelGGL(at_iou_kernel, dim3(div_up(N, 256), B), dim3(256), 0, s, geo, gt_boxes, G,
                     im_info, cfg->allowed_border, w.maxov, w.argmax, w.gtmax);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(at_label_kernel, dim3(div_up(N, 256), B), dim3(256), 0, s, geo, gt_boxes, G,
                     im_info, *cfg, w.maxov, w.gtmax, w.label, counts);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_anchor_target_sample_f32(const float* base_anchors, int A, int H, int W,
                                             int feat_stride, const float* gt_boxes, int B, int G,
                                             const tlod_rpn_cfg* cfg, const int32_t* perm,
                                             const int32_t* perm_off, uint64_t seed,
                                             float* labels, float* bbox_targets, float* inside_w,
                                             float* outside_w, void* ws, size_t ws_bytes,
                                             tlod_stream_t stream) {
  int st = at_check(A, H, W, B, G, cfg);
  if (st) return st;
  TLOD_CHECK_ARG(!perm || perm_off, "perm given without perm_off");
  hipStream_t s = (hipStream_t)stream;
  const int N = A * H * W;
  Carve c(ws, ws_bytes);
  AtWs w;
  carve_at(c, w, B, N, G);
  if (!c.ok()) { set_error("tlod_anchor_target: workspace too small"); return kWorkspace; }
  AnchorGeo geo{base_anchors, A, H, W, feat_stride};
  if (perm == nullptr && N <= kAtMax) {
    const int lds = kAtMax * (int)sizeof(uint32_t);
    TLOD_HIP(lds_attr((const void*)at_sample_lds_kernel, lds));
    hipLaunchKernelGGL(at_sample_lds_kernel, dim3(B), dim3(kBlk), lds, s, N, *cfg, seed, w.label,
                       w.nex);
  } else {
    hipLaunchKernelGGL(at_sample_kernel, dim3(B), dim3(kBlk), 0, s, N, *cfg, perm, perm_off, seed,
                       w.label, w.list, w.nex);
  }
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(at_output_kernel, dim3(div_up(N, 256), B), dim3(256), 0, s, geo, gt_boxes, G,
                     B, cfg->inside_weight, w.label, w.argmax, w.nex, labels, bbox_targets,
                     inside_w, outside_w);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_anchor_target_f32(const float* base_anchors, int A, int H, int W,
                                      int feat_stride, const float* gt_boxes, int B, int G,
                                      const float* im_info, const tlod_rpn_cfg* cfg, uint64_t seed,
                                      int32_t* counts, float* labels, float* bbox_targets,
                                      float* inside_w, float* outside_w, void* ws,
                                      size_t ws_bytes, tlod_stream_t stream) {
  int st = tlod_anchor_target_label_f32(base_anchors, A, H, W, feat_stride, gt_boxes, B, G,
                                        im_info, cfg, counts, ws, ws_bytes, stream);
  if (st) return st;
  return tlod_anchor_target_sample_f32(base_anchors, A, H, W, feat_stride, gt_boxes, B, G, cfg,
                                       nullptr, nullptr, seed, labels, bbox_targets, inside_w,
                                       outside_w, ws, ws_bytes, stream);
}

// ------------------------------------------------------------ proposal target ABI
extern "C" size_t tlod_proposal_target_workspace_bytes(int B, int R, int G) {
  Carve c(nullptr, 0);
  PtWs w;
  carve_pt(c, w, B, R, G, 4096);
  return align_up(c.off, 256);
}

static int pt_check(int B, int R, int G, const tlod_rcnn_cfg* cfg) {
  TLOD_CHECK_ARG(B > 0 && R >= 0 && G > 0 && G <= kMaxG, "bad shape");
  TLOD_CHECK_ARG(cfg && cfg->batch_size > 0 && cfg->batch_size <= 4096, "bad cfg");
  TLOD_CHECK_ARG(R + G <= kMaxSortPt, "R + G must be <= 4096");
  return kOk;
}

extern "C" int tlod_proposal_target_count_f32(const float* rois, int B, int R,
                                              const float* gt_boxes, int G,
                                              const tlod_rcnn_cfg* cfg, int32_t* counts, void* ws,
                                              size_t ws_bytes, tlod_stream_t stream) {
  int st = pt_check(B, R, G, cfg);
  if (st) return st;
  Carve c(ws, ws_bytes);
  PtWs w;
  carve_pt(c, w, B, R, G, 4096);
  if (!c.ok()) { set_error("tlod_proposal_target: workspace too small"); return kWorkspace; }
  hipLaunchKernelGGL(pt_count_kernel, dim3(B), dim3(kBlk), 0, (hipStream_t)stream, rois, R,
                     gt_boxes, G, *cfg, w.maxov, w.assign, counts);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_proposal_target_sample_f32(const float* rois, int B, int R,
                                               const float* gt_boxes, int G,
                                               const tlod_rcnn_cfg* cfg, const int32_t* fg_perm,
                                               const int32_t* perm_off, const double* rand,
                                               const int32_t* rand_off, uint64_t seed,
                                               float* rois_out, float* labels, float* targets,
                                               float* inside_w, float* outside_w, void* ws,
                                               size_t ws_bytes, tlod_stream_t stream) {
  int st = pt_check(B, R, G, cfg);
  if (st) return st;
  TLOD_CHECK_ARG((!fg_perm || perm_off) && (!rand || rand_off), "explicit draws need offsets");
  TLOD_CHECK_ARG((fg_perm == nullptr) == (rand == nullptr), "give both fg_perm and rand, or neither");
  Carve c(ws, ws_bytes);
  PtWs w;
  carve_pt(c, w, B, R, G, 4096);
  if (!c.ok()) { set_error("tlod_proposal_target: workspace too small"); return kWorkspace; }
  // fg_rois_per_image = int(np.round(FG_FRACTION * rois_per_image)), min 1 (:47-49)
  int fg_per = (int)std::nearbyint((double)cfg->fg_fraction * (double)cfg->batch_size);
  if (fg_per == 0) fg_per = 1;
  hipLaunchKernelGGL(pt_sample_kernel, dim3(B), dim3(kBlk), 0, (hipStream_t)stream, rois, R,
                     gt_boxes, G, *cfg, fg_per, w.maxov, w.assign, fg_perm, perm_off, rand,
                     rand_off, seed, w.fg, w.bg, w.keep, rois_out, labels, targets, inside_w,
                     outside_w);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_proposal_target_f32(const float* rois, int B, int R, const float* gt_boxes,
                                        int G, const tlod_rcnn_cfg* cfg, uint64_t seed,
                                        int32_t* counts, float* rois_out, float* labels,
                                        float* targets, float* inside_w, float* outside_w,
                                        void* ws, size_t ws_bytes, tlod_stream_t stream) {
  int st = tlod_proposal_target_count_f32(rois, B, R, gt_boxes, G, cfg, counts, ws, ws_bytes,
                                          stream);
  if (st) return st;
  return tlod_proposal_target_sample_f32(rois, B, R, gt_boxes, G, cfg, nullptr, nullptr, nullptr,
                                         nullptr, seed, rois_out, labels, targets, inside_w,
                                         outside_w, ws, ws_bytes, stream);
}
