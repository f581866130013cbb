// Warp-specialized split-bf16 weight gradient of a 3x3 / pad 1 / stride 1 convolution
// (the backbone's conv3_x .. conv5_x and RPN_Conv, lib/DAF/vgg16.py:49-53,
// lib/model/rpn/rpn.py:28; cuDNN's backward-filter in the reference):
//
//   dW[co][ci][t] = sum_n sum_p dY[n][co][p] * X[n][ci][p + off(t)]      (zero padding)
//
// as a GEMM with M = output channels, N = (tap, input channel), K = pixels.  Round 1-3's
// conv_wgrad_bs_kernel staged K as 16 flattened pixels of im2col rows: every (ci, tap)
// column of a tile staged and split its own 16 values, so each X element was split 9 times
// per tile and the kernel was VALU/issue-bound (53% issue stalls, MFMA pipes 59% busy).
// Here a K chunk is a 2D tile of 4 x 16 pixels:
//   * A = dY of BM = 128 output channels over the 64 pixels, staged [plane][co][k] (128-B
//     rows, 16-B slots XOR-swizzled by co & 7: conflict-free ds_read_b128 fragments);
//   * B = X of BC = 32 input channels over the tile's 6 x 18 halo patch, staged channels-last
//     per 8-channel octet [plane][octet][position][8 ch] — the 9 taps are 9 shifted views
//     of one patch (108 positions instead of 9 x 64 im2col values), read as the MFMA's B
//     operand with the gfx950 transposing ds_read_b64_tr_b16 (column = channel, rows =
//     the 4 pixels a lane group needs at tap t; conflict-free at the 1920-B octet pitch);
//   * 8 MFMA waves (each 32 rows x 16 channels x 9 taps: 18 tiles of v_mfma_f32_16x16x32_bf16)
//     and 4 producer waves that load two chunks ahead, split the f32 values exactly into
//     three bf16 planes (bs_common.h split2) and store them; one barrier per chunk (2 k-steps).
// K is split over workgroups (pixel-tile ranges); each workgroup writes its 128 x 288 partial
// tile in lane order to a slab, reduced in fixed split order (deterministic) into dW by
// wgws_reduce_kernel.  The bias gradient rides along: the producers of the ci-block-0
// workgroups sum the dY values they stage (db_slab, reduced by db_reduce_kernel).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "bs_common.h"

namespace tlod {

namespace wgws {
constexpr int BM = 128, BC = 32, TH = 4, TW = 16, KC = TH * TW;  // K chunk = 64 pixels
constexpr int PH = TH + 2, PW = TW + 2, PP = PH * PW;              // 6 x 18 = 108 positions
#ifndef TLOD_WGWS_NPW  // producer waves per workgroup (4: 3 waves per SIMD; 8: 4 per SIMD)
#define TLOD_WGWS_NPW 4
#endif
constexpr int NMW = 8, NPW = TLOD_WGWS_NPW;                        // MFMA / producer waves
constexpr int WAVES_PER_SIMD = (NMW + NPW) / 4;
constexpr int NT = (NMW + NPW) * 64;
constexpr int A_ROW = KC * 2;                 // 128 B per co row per plane
constexpr int A_PLANE = BM * A_ROW;           // 16384
constexpr int B_OCT = 120 * 16;               // 1920 (== 128 mod 256: conflict-free tr reads)
constexpr int B_PLANE = (BC / 8) * B_OCT;     // 7680
constexpr int A_BYTES = 3 * A_PLANE, B_BYTES = 3 * B_PLANE;
constexpr int BUF = A_BYTES + B_BYTES;        // 72192
constexpr int LDS_BYTES = 2 * BUF;            // 144384
constexpr int TILE_FLOATS = BM * BC * 9;      // partial tile per workgroup (36864)
constexpr int A_ITEMS = BM * TH * 2;          // (co, tile row, 8-pixel half)
constexpr int A_IT = A_ITEMS / (NPW * 64);    // 4 (NPW = 4)
constexpr int B_ITEMS = (BC / 8) * PP;        // (octet, position) = 432
constexpr int B_IT = (B_ITEMS + NPW * 64 - 1) / (NPW * 64);  // 2
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(A_ITEMS % (NPW * 64) == 0, "A staging");
}  // namespace wgws

// Diagnostic build only (TLOD_WGWS_STAMPS=1): per-wave s_memtime sums per segment for
// blocks < 256 (MFMA waves: 0 k-steps, 1 barrier waits, 2 epilogue, 3 first barrier;
// producers: 0 staging, 1 barrier waits), read back with tlod_debug_wgws_stamps.
// Timing-only ablations of the producers (wrong results): 1 = no global loads, 2 = no
// split (raw bits stored), 3 = no LDS stores.
#ifndef TLOD_WGWS_ABL
#define TLOD_WGWS_ABL 0
#endif
#ifndef TLOD_WGWS_BSPLIT  // 1: the MFMA waves stage B (the X patch), the producers only A
#define TLOD_WGWS_BSPLIT 1
#endif
#ifndef TLOD_WGRAD_WS  // A/B: 0 keeps every 3x3 bf16x6 wgrad on conv_wgrad_bs_kernel
#define TLOD_WGRAD_WS 1
#endif
#ifndef TLOD_WGWS_SPLIT_MAX  // A/B: cap of the split count (profiles/r04/split_caps_sweep.txt)
#define TLOD_WGWS_SPLIT_MAX 256
#endif
#ifndef TLOD_WGWS_KSUM  // per-k-step sums of the cross products (accuracy; see the k-step)
#define TLOD_WGWS_KSUM 0
#endif
#ifndef TLOD_WGWS_PRIO  // s_setprio of the producer waves (0: default)
#define TLOD_WGWS_PRIO 0
#endif
#ifndef TLOD_WGWS_MPRIO  // MFMA waves: 1 = waves 4-7 at priority 1; 2 = per k-step cluster
#define TLOD_WGWS_MPRIO 0
#endif
#ifndef TLOD_WGWS_STAMPS
#define TLOD_WGWS_STAMPS 0
#endif
#if TLOD_WGWS_STAMPS
__device__ unsigned long long g_wgws_stamps[256 * 12 * 4 + 512];
#define WG_STAMP_DECL                                                \
  unsigned long long wg_seg[4] = {0, 0, 0, 0};                       \
  const unsigned long long wg_r0 = __builtin_amdgcn_s_memrealtime(); \
  const unsigned long long wg_t0 = __builtin_amdgcn_s_memtime();     \
  unsigned long long wg_t = wg_t0
#define WG_STAMP(k)                                              \
  do {                                                           \
    const unsigned long long now = __builtin_amdgcn_s_memtime(); \
    wg_seg[k] += now - wg_t;                                     \
    wg_t = now;                                                  \
  } while (0)
#define WG_STAMP_SAVE                                                                  \
  do {                                                                                 \
    if (blockIdx.x < 256 && (threadIdx.x & 63) == 0)                                   \
      for (int k_ = 0; k_ < 4; ++k_)                                                   \
        g_wgws_stamps[(blockIdx.x * 12 + threadIdx.x / 64) * 4 + k_] = wg_seg[k_];     \
    if (blockIdx.x < 256 && threadIdx.x == 0) {                                        \
      g_wgws_stamps[256 * 48 + blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - wg_t0; \
      g_wgws_stamps[256 * 48 + blockIdx.x * 2 + 1] =                                   \
          __builtin_amdgcn_s_memrealtime() - wg_r0;                                    \
    }                                                                                  \
  } while (0)
#else
#define WG_STAMP_DECL do {} while (0)
#define WG_STAMP(k) do {} while (0)
#define WG_STAMP_SAVE do {} while (0)
#endif

__device__ __forceinline__ uint2 lds_read_tr16(const unsigned char* p) {
  typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 v4bf;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wold-style-cast"
  auto lp = (__attribute__((address_space(3))) v4bf*)(const_cast<unsigned char*>(p));
#pragma clang diagnostic pop
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(lp));
}

__device__ __forceinline__ f32x4 wgws_mfma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// The producer waves of wgrad_ws_kernel: chunk j of the workgroup's range is loaded into
// register slot j & 1 two chunks ahead, then split and stored into LDS buffer j & 1.
// A (dY): lane item (co row (ptid >> 3) + 32 i, slot s' = ptid & 7): quad sub = s' & 3 of
// tile rows rr = s' >> 2 and rr + 2 — the four lanes of a (co, row) read 64 contiguous bytes
// per instruction; the slot's 8 k values are (row rr, pixels 4 sub..+3), (row rr + 2, same)
// (the MFMA waves' B reads follow the same k order).  B (X): lane item (octet, position) of
// the 6 x 18 patch, 8 channel loads.  Rows past H / Cout and positions outside the map load
// out of range (zero); only a tile column past W (uniform per chunk) and a ragged last octet
// (Cin % 8, uniform) need element masks.
template <bool SUMS>
__device__ __forceinline__ void wgws_produce(const float* __restrict__ G, const float* __restrict__ X,
                                             unsigned char* smem, float* __restrict__ db_row,
                                             int N, int Cin, int H, int W, int Cout, int m0,
                                             int c0, int c_begin, int nch, int tcols,
                                             int per_img, int ptid) {
  using namespace wgws;
  if (TLOD_WGWS_PRIO) __builtin_amdgcn_s_setprio(TLOD_WGWS_PRIO);
  WG_STAMP_DECL;
  const int HW = H * W;
  const i32x4 g_rsrc = make_buffer_rsrc(G, (unsigned)((size_t)N * Cout * HW * 4));
  const i32x4 x_rsrc = make_buffer_rsrc(X, (unsigned)((size_t)N * Cin * HW * 4));
  const int a_s = ptid & 7, a_rr = a_s >> 2, a_px = 4 * (a_s & 3);
  int a_lds[A_IT], a_co[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    const int co_l = (ptid >> 3) + NPW * 8 * i;
    a_lds[i] = co_l * A_ROW + 16 * (a_s ^ (co_l & 7));
    a_co[i] = m0 + co_l < Cout ? m0 + co_l : -1;
  }
  int b_lds[B_IT], b_pr[B_IT], b_pc[B_IT], b_ci[B_IT];
#pragma unroll
  for (int i = 0; i < B_IT; ++i) {
    const int it = ptid + NPW * 64 * i;
    const int oct = it / PP, pos = it % PP;
    b_lds[i] = it < B_ITEMS ? oct * B_OCT + pos * 16 : -1;
    b_pr[i] = pos / PW - 1;
    b_pc[i] = pos % PW - 1;
    b_ci[i] = c0 + 8 * oct;
  }
  const bool cmask = (Cin & 7) != 0;
  float rs[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) rs[i] = 0.f;

  f32x4v ra[2][A_IT][2];
  float rb[2][B_IT][8];
  int anv[2];  // valid pixels of this lane's two 4-pixel A quads (edge chunks), else 4
  // load cursor: image ln, tile origin (lh0, lw0) of the next chunk to load; ld_left chunks
  // of the range remain (loads past it read out of range: zeros, never consumed)
  int ld_left = nch;
  int ln = c_begin / per_img;
  int lh0, lw0;
  {
    const int r = c_begin - ln * per_img;
    lh0 = (r / tcols) * TH;
    lw0 = (r % tcols) * TW;
  }
  auto load = [&](auto slc) {
    constexpr int S = decltype(slc)::value;
    anv[S] = min(max(W - (lw0 + a_px), 0), 4);
    const int w = lw0 + a_px;
    const bool live = ld_left-- > 0;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int h = lh0 + a_rr + 2 * hh;
        const int off = live && a_co[i] >= 0 && h < H && w < W ? (((ln * Cout + a_co[i]) * H + h) * W + w) * 4 : kBufOOB;
        ra[S][i][hh] = TLOD_WGWS_ABL == 1 ? f32x4v{(float)off, 1.f, 2.f, 3.f}
                                          : raw_buffer_load_v4f32(g_rsrc, off, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < (TLOD_WGWS_BSPLIT ? 0 : B_IT); ++i) {
      const int gh = lh0 + b_pr[i], gw = lw0 + b_pc[i];
      const bool ok = live && b_lds[i] >= 0 && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
      const int off = ok ? ((ln * Cin + b_ci[i]) * HW + gh * W + gw) * 4 : kBufOOB;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        rb[S][i][e] = TLOD_WGWS_ABL == 1 ? (float)(off + e) : raw_buffer_load_f32(x_rsrc, off, e * HW * 4, 0);
    }
    // advance the cursor (chunks are loaded in order)
    lw0 += TW;
    if (lw0 >= W) {
      lw0 = 0;
      lh0 += TH;
      if (lh0 >= H) {
        lh0 = 0;
        ++ln;
      }
    }
  };
  auto put = [&](unsigned char* dst, int plane_bytes, float (&v)[8]) {
    u32x4 sp[3];
    if (TLOD_WGWS_ABL == 2) {
      sp[0] = u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
      sp[1] = u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])};
      sp[2] = sp[0];
    } else {
      split8<3>(v, sp);
    }
    if (TLOD_WGWS_ABL == 3) {
      if (sp[0][0] == 0x7fc00001u && sp[1][1] == 0x7fc00001u && sp[2][2] == 0x7fc00001u) dst[0] = 1;
      return;
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(dst + pl * plane_bytes) = sp[pl];
  };
  auto store = [&](auto slc, unsigned char* buf) {
    constexpr int S = decltype(slc)::value;
#if TLOD_WGWS_STAMPS  // diagnostic: the wait for this slot's loads as a segment of its own
    WG_STAMP(0);
    if (TLOD_WGWS_BSPLIT) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    WG_STAMP(2);
#endif
    const int nv = anv[S];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ra[S][i][e >> 2][e & 3];
      if (nv < 4) {  // a tile column past W: pixels past the row end (uniform per chunk)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (e & 3) < nv ? v[e] : 0.f;
      }
      if constexpr (SUMS) {
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) t += v[e];
        rs[i] += t;
      }
      put(buf + a_lds[i], A_PLANE, v);
    }
#pragma unroll
    for (int i = 0; i < (TLOD_WGWS_BSPLIT ? 0 : B_IT); ++i) {
      if (b_lds[i] < 0) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rb[S][i][e];
      if (cmask) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = b_ci[i] + e < Cin ? v[e] : 0.f;
      }
      put(buf + A_BYTES + b_lds[i], B_PLANE, v);
    }
  };
  const std::integral_constant<int, 0> S0;
  const std::integral_constant<int, 1> S1;
  // Straight-line pairs of iterations (loads and stores unconditional: a store past the range
  // goes to the buffer nobody reads next, a load past it reads zeros), so the compiler's
  // vmcnt waits before a store leave the other slot's 8 loads in flight.  2 * ceil(nch / 2)
  // + 1 barriers, as the MFMA waves.
  load(S0);
  load(S1);
  store(S0, smem);
  load(S0);
  WG_STAMP(0);
  __syncthreads();
  WG_STAMP(1);
  for (int j = 0; j < nch; j += 2) {
    // iteration j: the MFMA waves read chunk j (buffer 0); stage chunk j + 1 (buffer 1)
    store(S1, smem + BUF);
    load(S1);
    WG_STAMP(0);
    __syncthreads();
    WG_STAMP(1);
    // iteration j + 1: stage chunk j + 2 (buffer 0)
    store(S0, smem);
    load(S0);
    WG_STAMP(0);
    __syncthreads();
    WG_STAMP(1);
  }
  if constexpr (SUMS) {  // the 8 lanes of a co row (ptid & 7), in a fixed order
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      float t = rs[i] + __shfl_xor(rs[i], 1);
      t = t + __shfl_xor(t, 2);
      t = t + __shfl_xor(t, 4);
      if (a_s == 0 && a_co[i] >= 0) db_row[a_co[i]] = t;
    }
  }
  WG_STAMP_SAVE;
}

// Grid: tiles_m x tiles_c x splits workgroups; workgroup (mt, ct, split) owns output
// channels [128 mt, +128), input channels [32 ct, +32) and pixel-tile chunks
// [split * cps, +cps) of the N x ceil(H/4) x ceil(W/16) chunk grid.
__global__ void __launch_bounds__(wgws::NT)
    __attribute__((amdgpu_waves_per_eu(wgws::WAVES_PER_SIMD, wgws::WAVES_PER_SIMD)))
wgrad_ws_kernel(const float* __restrict__ G, const float* __restrict__ X,
                float* __restrict__ slab, float* __restrict__ db_slab, int N, int Cin, int H,
                int W, int Cout, int tiles_m, int tiles_c, int splits, int cps) {
  using namespace wgws;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tiles = tiles_m * tiles_c;
  const int L = xcd_remap(blockIdx.x, tiles * splits);  // a split's tiles share an XCD
  const int split = L / tiles, tile = L % tiles;
  const int mt = tile % tiles_m, ct = tile / tiles_m;
  const int m0 = mt * BM, c0 = ct * BC;
  const int tcols = (W + TW - 1) / TW, trows = (H + TH - 1) / TH;
  const int per_img = tcols * trows;
  const int total = N * per_img;
  const int c_begin = min(total, split * cps), c_end = min(total, c_begin + cps);
  const int nch = c_end - c_begin;
  const int tid = threadIdx.x;

  if (tid >= NMW * 64) {
    // ================= producers (a uniform branch: only the ci-block-0 workgroups sum dY)
    if (db_slab != nullptr && ct == 0)
      wgws_produce<true>(G, X, smem, db_slab + (size_t)split * Cout, N, Cin, H, W, Cout, m0, c0,
                         c_begin, nch, tcols, per_img, tid - NMW * 64);
    else
      wgws_produce<false>(G, X, smem, nullptr, N, Cin, H, W, Cout, m0, c0, c_begin, nch, tcols,
                          per_img, tid - NMW * 64);
    return;
  }

  // ================= MFMA waves: wave w owns co rows 32 (w & 3) + [0, 32) (two 16-row
  // blocks) and input channels 16 (w >> 2) + [0, 16) at all 9 taps
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, p = l16 & 3;
  const int rp = w & 3, chh = w >> 2;
  // A fragment (rows 32 rp + 16 rbi + l16, k = 32 s + 8 g): slot (4 s + g) ^ (row & 7)
  const int a_row = (32 * rp + l16) * A_ROW;
  const int a_s0 = a_row + 16 * ((0 + g) ^ (l16 & 7));
  const int a_s1 = a_row + 16 * ((4 + g) ^ (l16 & 7));
  // B fragment (tr reads): lane 4q + p supplies position pos(k) + off(t) of k row
  // 32 s + 8 g + 4 h + q, channels 4p..4p+3 of the wave's 16 (octet 2 chh + (p >> 1))
  const int b_lane = A_BYTES + (2 * chh + (p >> 1)) * B_OCT + (4 * g + q) * 16 + (p & 1) * 8;
  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (TLOD_WGWS_MPRIO == 1 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256)
    __builtin_amdgcn_s_setprio(1);
  auto kstep = [&](const unsigned char* buf, int a_off, int b_off) {
    if (TLOD_WGWS_MPRIO == 2) __builtin_amdgcn_s_setprio(1);
    u32x4 a[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = *reinterpret_cast<const u32x4*>(buf + a_off + pl * A_PLANE + i * 16 * A_ROW);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int tap = ((t / 3) * PW + t % 3) * 16;
      u32x4 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const unsigned char* bp = buf + b_off + pl * B_PLANE + tap;
        const uint2 lo = lds_read_tr16(bp);
        const uint2 hi = lds_read_tr16(bp + 2 * PW * 16);  // tile row s + 2
        b[pl] = u32x4{lo.x, lo.y, hi.x, hi.y};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (TLOD_WGWS_KSUM) {
          // the k-step's five cross products summed from zero, then the f32 add of that
          // sum after hi*hi: the small products are not floored against the running
          // accumulator (bs_common.h bs_mac)
          f32x4 x = wgws_mfma(a[i][1], b[0], f32x4{0.f, 0.f, 0.f, 0.f});
          x = wgws_mfma(a[i][0], b[1], x);
          x = wgws_mfma(a[i][2], b[0], x);
          x = wgws_mfma(a[i][1], b[1], x);
          x = wgws_mfma(a[i][0], b[2], x);
          acc[i][t] = wgws_mfma(a[i][0], b[0], acc[i][t]) + x;
        } else {
          acc[i][t] = wgws_mfma(a[i][0], b[0], acc[i][t]);
          acc[i][t] = wgws_mfma(a[i][1], b[0], acc[i][t]);
          acc[i][t] = wgws_mfma(a[i][0], b[1], acc[i][t]);
          acc[i][t] = wgws_mfma(a[i][2], b[0], acc[i][t]);
          acc[i][t] = wgws_mfma(a[i][1], b[1], acc[i][t]);
          acc[i][t] = wgws_mfma(a[i][0], b[2], acc[i][t]);
        }
      }
    }
    if (TLOD_WGWS_MPRIO == 2) __builtin_amdgcn_s_setprio(0);
  };
  // B staging by the MFMA waves (TLOD_WGWS_BSPLIT): lane tid < 432 owns one (octet,
  // position) item of the patch; chunk j's 8 channel values are loaded two chunks ahead
  // into register slot j & 1 and split + stored between the two k-steps of chunk j - 1
  // (items spread evenly over the 8 waves, 54 lanes each, measured 1% slower)
  const bool b_item = TLOD_WGWS_BSPLIT && tid < B_ITEMS;
  const int b_oct = tid / PP, b_pos = tid % PP;
  const int b_lds = b_oct * B_OCT + b_pos * 16;
  const int b_pr = b_pos / PW - 1, b_pc = b_pos % PW - 1, b_ci = c0 + 8 * b_oct;
  const int HW = H * W;
  const i32x4 x_rsrc = make_buffer_rsrc(X, (unsigned)((size_t)N * Cin * HW * 4));
  const bool cmask = (Cin & 7) != 0;
  float rbv[2][8];
  int ld_left = nch;
  int ln = c_begin / per_img, lh0, lw0;
  {
    const int r = c_begin - ln * per_img;
    lh0 = (r / tcols) * TH;
    lw0 = (r % tcols) * TW;
  }
  auto loadB = [&](auto slc) {
    constexpr int S = decltype(slc)::value;
    const int gh = lh0 + b_pr, gw = lw0 + b_pc;
    const bool ok = ld_left-- > 0 && b_item && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
    const int off = ok ? ((ln * Cin + b_ci) * HW + gh * W + gw) * 4 : kBufOOB;
#pragma unroll
    for (int e = 0; e < 8; ++e) rbv[S][e] = raw_buffer_load_f32(x_rsrc, off, e * HW * 4, 0);
    lw0 += TW;
    if (lw0 >= W) {
      lw0 = 0;
      lh0 += TH;
      if (lh0 >= H) {
        lh0 = 0;
        ++ln;
      }
    }
  };
  auto storeB = [&](auto slc, unsigned char* buf) {
    constexpr int S = decltype(slc)::value;
    if (!b_item) return;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rbv[S][e];
    if (cmask) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = b_ci + e < Cin ? v[e] : 0.f;
    }
    u32x4 sp[3];
    split8<3>(v, sp);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      *reinterpret_cast<u32x4*>(buf + A_BYTES + pl * B_PLANE + b_lds) = sp[pl];
  };
  const std::integral_constant<int, 0> S0;
  const std::integral_constant<int, 1> S1;
  WG_STAMP_DECL;
  if (TLOD_WGWS_BSPLIT) {  // unconditional, as the producers' (see wgws_produce)
    loadB(S0);
    loadB(S1);
    storeB(S0, smem);
    loadB(S0);
  }
  __syncthreads();
  WG_STAMP(3);
  // iteration j reads buffer j & 1 and stages chunk j + 1's B into buffer (j + 1) & 1; the
  // odd count's last iteration computes nothing (its barrier pairs the producers')
  auto iter = [&](auto slc_next, int j) {
    unsigned char* buf = smem + (j & 1) * BUF;
    const bool live = j < nch;
    if (live) kstep(buf, a_s0, b_lane);
    if (TLOD_WGWS_BSPLIT) {
      storeB(slc_next, smem + ((j + 1) & 1) * BUF);
      loadB(slc_next);
    }
    if (live) kstep(buf, a_s1, b_lane + PW * 16);  // k rows 32..63: tile rows 1 and 3
    WG_STAMP(0);
    __syncthreads();
    WG_STAMP(1);
  };
  for (int j = 0; j < nch; j += 2) {
    iter(S1, j);
    iter(S0, j + 1);
  }
  // partial tile in lane order: [wave][i][t][lane][4]
  float* S = slab + ((size_t)split * tiles + tile) * TILE_FLOATS + (size_t)w * (2 * 9 * 256) + lane * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *reinterpret_cast<f32x4*>(S + (i * 9 + t) * 256) = acc[i][t];
  WG_STAMP(2);
  WG_STAMP_SAVE;
}

// dW (+)= sum over splits of the lane-ordered partial tiles, in split order.  One thread per
// (tile, wave, i, t, lane): 4 consecutive slab floats = rows co 4g..4g+3 of one (ci, tap).
__global__ void __launch_bounds__(256) wgws_reduce_kernel(const float* __restrict__ slab,
                                                          float* __restrict__ dw, int splits,
                                                          int tiles_m, int tiles_c, int Cin,
                                                          int Cout, int accumulate,
                                                          const float* __restrict__ row_scale) {
  using namespace wgws;
  const int tiles = tiles_m * tiles_c;
  const int idx = blockIdx.x * 256 + threadIdx.x;  // float4 index within one split's slab
  if (idx >= tiles * TILE_FLOATS / 4) return;
  const size_t stride4 = (size_t)tiles * TILE_FLOATS / 4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab) + idx;
  // split order kept (deterministic); four loads in flight per group (the loop issued one
  // load per dependent add: latency-bound)
  f32x4 sum = s4[0];
  int k = 1;
  for (; k + 4 <= splits; k += 4) {
    const f32x4 v0 = s4[k * stride4], v1 = s4[(k + 1) * stride4];
    const f32x4 v2 = s4[(k + 2) * stride4], v3 = s4[(k + 3) * stride4];
    sum += v0;
    sum += v1;
    sum += v2;
    sum += v3;
  }
  for (; k < splits; ++k) sum += s4[k * stride4];
  int r = idx;
  const int lane = r % 64; r /= 64;
  const int t = r % 9; r /= 9;
  const int i = r % 2; r /= 2;
  const int w = r % NMW; r /= NMW;
  const int tile = r;
  const int mt = tile % tiles_m, ct = tile / tiles_m;
  const int g = lane >> 4, l16 = lane & 15;
  const int ci = ct * BC + 16 * (w >> 2) + l16;
  if (ci >= Cin) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int co = mt * BM + 32 * (w & 3) + 16 * i + 4 * g + e;
    if (co >= Cout) continue;
    float* d = dw + ((size_t)co * Cin + ci) * 9 + t;
    const float v = row_scale != nullptr ? sum[e] * row_scale[co] : sum[e];
    *d = accumulate ? *d + v : v;
  }
}

// ---- host side

// Every 3x3 bf16x6 weight gradient (any channel counts and map sizes: ragged channel octets,
// pixel tiles past the map and rows past Cout are masked) whose tensors fit 32-bit buffer
// offsets (compile with -DTLOD_WGRAD_WS=0 to keep the im2col kernel, conv_wgrad_bs_kernel).
bool wgrad_ws_applies(int N, int Cin, int H, int W, int Cout, int KS, int nprod) {
  return TLOD_WGRAD_WS != 0 && KS == 3 && nprod == 6 &&
         (size_t)N * (std::max(Cin, Cout) + 8) * H * W * 4 < (1ull << 31);
}

struct WgwsPlan {
  int tiles_m, tiles_c, splits, cps;
};
static WgwsPlan wgws_plan(int N, int Cin, int H, int W, int Cout) {
  using namespace wgws;
  WgwsPlan p;
  p.tiles_m = div_up(Cout, BM);
  p.tiles_c = div_up(Cin, BC);
  const int tiles = p.tiles_m * p.tiles_c;
  const int chunks = N * div_up(H, TH) * div_up(W, TW);
  // cost: rounds x chunks per split x chunk time + the slab round trip (sp writes + sp
  // reads of the partial tiles); one resident workgroup per CU (139 KB LDS)
  const int slots = cached_slots((const void*)wgrad_ws_kernel, NT, LDS_BYTES);
  const double chunk_s = 1728.0 * 16.0 / 4.0 / 2.1e9 / 0.75;  // 1728 16x16x32 MFMAs per chunk
  const double tile_bytes = (double)TILE_FLOATS * 4.0;
  int best = 1;
  double best_t = 1e30;
  for (int sp = 1; sp <= std::min({256, TLOD_WGWS_SPLIT_MAX, chunks}); ++sp) {
    const int cps = div_up(chunks, sp);
    const int esp = div_up(chunks, cps);
    const long long rounds = ((long long)tiles * esp + slots - 1) / slots;
    const double t = (double)rounds * cps * chunk_s + 2.0 * esp * tiles * tile_bytes / 4e12 + 2e-6 * (esp > 1);
    if (t < best_t * 0.999) {
      best_t = t;
      best = esp;
    }
  }
  p.cps = div_up(chunks, best);
  p.splits = div_up(chunks, p.cps);
  return p;
}

size_t wgrad_ws_workspace(int N, int Cin, int H, int W, int Cout) {
  const WgwsPlan p = wgws_plan(N, Cin, H, W, Cout);
  return align_up((size_t)p.splits * p.tiles_m * p.tiles_c * wgws::TILE_FLOATS * sizeof(float), 16) +
         (size_t)p.splits * Cout * sizeof(float);
}

// db_reduce_kernel lives in conv.hip
int launch_db_reduce(const float* db_slab, int splits, int C, float* db, int accumulate,
                     hipStream_t s);

int wgrad_ws_launch(const float* dy, const float* x, float* dw, float* db, int accumulate,
                    const float* row_scale, int N, int Cin, int H, int W, int Cout, void* ws,
                    size_t ws_bytes, hipStream_t s) {
  using namespace wgws;
  const WgwsPlan p = wgws_plan(N, Cin, H, W, Cout);
  if (ws_bytes < wgrad_ws_workspace(N, Cin, H, W, Cout)) {
    set_error("tlod_conv_wgrad_bs_f32: workspace too small");
    return kWorkspace;
  }
  const int tiles = p.tiles_m * p.tiles_c;
  float* slab = static_cast<float*>(ws);
  float* db_slab = db ? reinterpret_cast<float*>(static_cast<char*>(ws) +
                                                 align_up((size_t)p.splits * tiles * TILE_FLOATS *
                                                              sizeof(float), 16))
                      : nullptr;
  TLOD_HIP(lds_attr((const void*)wgrad_ws_kernel, LDS_BYTES));
  hipLaunchKernelGGL(wgrad_ws_kernel, dim3((unsigned)(tiles * p.splits)), dim3(NT), LDS_BYTES, s,
                     dy, x, slab, db_slab, N, Cin, H, W, Cout, p.tiles_m, p.tiles_c, p.splits,
                     p.cps);
  TLOD_LAUNCH_CHECK();
  const int n4 = tiles * TILE_FLOATS / 4;
  hipLaunchKernelGGL(wgws_reduce_kernel, dim3((unsigned)div_up(n4, 256)), dim3(256), 0, s, slab, dw,
                     p.splits, p.tiles_m, p.tiles_c, Cin, Cout, accumulate, row_scale);
  TLOD_LAUNCH_CHECK();
  if (db) return launch_db_reduce(db_slab, p.splits, Cout, db, accumulate, s);
  return kOk;
}

}  // namespace tlod

#if TLOD_WGWS_STAMPS
extern "C" int tlod_debug_wgws_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(tlod::g_wgws_stamps), sizeof(tlod::g_wgws_stamps)) ==
                 hipSuccess ? 0 : 1;
}
#endif
