// Implicit-GEMM convolution (stride 1, "same" padding, KSxKS) on gfx950 MFMA, fp32.
//
// Replaces the cuDNN convolutions behind the VGG16 backbone and RPN conv
// (RCNN_base = torchvision vgg16().features[:-1], lib/DAF/vgg16.py:49; RPN_Conv
// lib/model/rpn/rpn.py:28).  The reference computes in fp32; so do we, on the f32-input
// MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, one rounding per accumulate), whose
// dense peak (157.3 TF) is the roofline these kernels are measured against.
//
//   fwd  : Y[n,co,p]  = sum_{ci,kh,kw} Wk[(ci,kh,kw)][co] * X[n,ci,p+(kh,kw)-pad]   (+bias, relu)
//   dgrad: the same kernel with X := dY and Wk := packed flipped/transposed weights
//   wgrad: dW[co][(ci,kh,kw)] = sum_{n,p} dY[n,co,p] * X[n,ci,p+(kh,kw)-pad]   (split-K slabs)
//
// Tiling (CDNA4-first): 256-thread workgroups of 4 wave64s; each wave owns MIx NJ
// 32x32 accumulator tiles (16 f32 regs each).  The input halo patch of CK channels is
// staged once in LDS and the KS*KS shifted views are read from it (9x less L2 traffic
// than an explicit im2col); operand tiles are double-buffered in LDS with the next
// chunk's global loads held in registers across the MFMA phase (issue early / write
// late).  Block ids are remapped so each XCD walks a contiguous run of tiles (its L2
// keeps the shared input patches).
#include "common.h"
#include "bs_common.h"
#include "tlod.h"

#include <algorithm>
#include <type_traits>
#include <cmath>

namespace tlod {


// These kernels run 1-2 workgroups of 8 waves per CU (LDS-bound), i.e. 2-4 waves per SIMD:
// telling the register allocator so lets the scheduler hoist LDS operand reads ahead of
// the MFMAs instead of minimising VGPRs for an occupancy the LDS never allows.
#ifndef TLOD_CONV_PF
#define TLOD_CONV_PF 2
#endif
#ifndef TLOD_CONV_SGB
#define TLOD_CONV_SGB 4
#endif
#ifndef TLOD_CONV_SGB_W
#define TLOD_CONV_SGB_W 0
#endif
// Split-bf16 forward: pair the 9 taps across consecutive input-channel chunks instead of
// padding each chunk to 10 tap slots (0 = pad, for A/B).
#ifndef TLOD_WG_SWZ
#define TLOD_WG_SWZ 1
#endif
#ifndef TLOD_TAP_PAIRING
#define TLOD_TAP_PAIRING 1
#endif
#ifndef TLOD_WS_PRIO
#define TLOD_WS_PRIO 0
#endif
#ifndef TLOD_CONV_OCC
#define TLOD_CONV_OCC __attribute__((amdgpu_waves_per_eu(2, 4)))
#endif
// Planner / kernel-selection A/B switches, compile time only (rebuild with -D to measure a
// variant; the shipped library holds no run-time variant paths).  Defaults are the measured
// choices: split caps (profiles/r04/split_caps_sweep.txt), the warp-specialized kernel and
// its flexible tiles, band tiles for padded narrow maps.
#ifndef TLOD_CONV_KSPLIT_MAX  // cap of the forward / dgrad K split
#define TLOD_CONV_KSPLIT_MAX 8
#endif
#ifndef TLOD_CONV_BAND  // 0: no band tiles
#define TLOD_CONV_BAND 1
#endif
#ifndef TLOD_CONV_WS  // 0: no warp-specialized forward / dgrad kernel
#define TLOD_CONV_WS 1
#endif
#ifndef TLOD_WS_MINCIN  // smallest Cin on the warp-specialized kernel (round 6: 64 — conv1_2 /
#define TLOD_WS_MINCIN 64  // conv2_1 0.5 / 1.7% faster than on the plain kernel, ws64 A/B)
#endif
#ifndef TLOD_WS_FLEX  // 0: warp-specialized tiles fixed at 16 x 32
#define TLOD_WS_FLEX 1
#endif
#ifndef TLOD_WG1X1_TILE  // 1x1 wgrad tile: 0 = cost model, 256 / 128 = forced
#define TLOD_WG1X1_TILE 0
#endif

// Out-of-range staging loads read this zero block instead of branching (a branch per
// load makes hipcc wait vmcnt(0) after each one; a select after the load pins the wait
// to the load instead of the LDS store that follows the MFMA phase).
__device__ __attribute__((aligned(16))) float g_zero[16];

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}


// Fused epilogue: y = act(acc * scale[co] + bias[co] + residual[n,co,p]); every pointer
// optional.  scale/bias carry a frozen BatchNorm folded per channel (ResNet: BN in eval
// mode with frozen affine, lib/DAF/resnet.py:261-284); residual is the bottleneck's
// identity/downsample branch (resnet.py:94-97).
struct Epi {
  const float* scale;
  const float* bias;
  const float* residual;
  int relu;
  float* pool;  // conv_fwd_bs_kernel (2D tiles, no split-K) only: write max_pool2d(2, 2) of
                // the result here (N, Cout, H/2, W/2) instead of the full map
  int s2d;      // conv_fwd_kernel only (MAF DRM, lib/MAF/drm.py:20-42): > 1 stores the result
                // cropped to (H/s*s, W/s*s) and space-to-depth rearranged, (N, Cout*s*s, H/s,
                // W/s) with channel co*s*s + (h%s)*s + w%s; no residual
  const float* mask;  // dgrad of a conv whose input is the previous conv's ReLU output: the
                      // result is zeroed where mask (that input, same layout as y) is not > 0
                      // — the previous layer's ReLU backward, applied in this epilogue
};

__device__ __forceinline__ float epi_mask(const Epi& e, size_t idx, float v) {
  return e.mask && !(e.mask[idx] > 0.f) ? 0.f : v;
}

// Element offset of output (n, co, h, w) under the epilogue's store layout; -1: cropped by
// the DRM space-to-depth.
__device__ __forceinline__ long long epi_out_index(const Epi& e, int n, int co, int h, int w,
                                                   int Cout, int H, int W) {
  if (e.s2d <= 1) return (((long long)n * Cout + co) * H + h) * W + w;
  const int s = e.s2d, Ho = H / s, Wo = W / s;
  if (h >= Ho * s || w >= Wo * s) return -1;
  const long long cc = ((long long)n * Cout + co) * s * s + (h % s) * s + w % s;
  return (cc * Ho + h / s) * Wo + w / s;
}

// ======================================================================= forward
// Block tile: BM = WM*MI*32 output channels x BN = TH*32 pixels (TH = WN*NJ rows of 32).
// K is consumed in chunks of CK input channels (KC = CK*KS*KS).  The 32x32x2 MFMA pairs
// GEMM rows k and k + KC/2 (lanes 0-31 / 32-63): since KC/2 = (CK/2)*KS*KS, row k+KC/2 is
// the same tap (kh,kw) CK/2 channels further, so every LDS operand read in the fully
// unrolled chunk is a lane-constant base plus a compile-time immediate.
template <int WM, int WN, int MI, int NJ, int CK, int KS>
struct FwdCfg {
  static_assert(CK % 2 == 0, "CK must be even (K pairing)");
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * MI * 32;
  static constexpr int TH = WN * NJ;
  static constexpr int TW = 32;
  static constexpr int PH = TH + KS - 1, PW = TW + KS - 1;
  static constexpr int KK = KS * KS;
  static constexpr int KC = CK * KK;              // GEMM K per chunk
  static constexpr int HALF = KC / 2;
  static constexpr int A_ELEMS = KC * BM;         // As[KC][BM]
  static constexpr int B_ELEMS = CK * PH * PW;    // Bs[CK][PH][PW]
  static constexpr int A_V4 = A_ELEMS / 4;
  static constexpr int A_PER = (A_V4 + NT - 1) / NT;
  static constexpr int B_PER = (B_ELEMS + NT - 1) / NT;
  static constexpr int LDS_FLOATS = 2 * (A_ELEMS + B_ELEMS) + 2 * BM;  // + scale/bias tiles
};

template <int WM, int WN, int MI, int NJ, int CK, int KS, bool VEC4>
__global__ void __launch_bounds__(WM* WN * 64) TLOD_CONV_OCC conv_fwd_kernel(
    const float* __restrict__ X, const float* __restrict__ Wk, Epi epi, float* __restrict__ Y,
    int N, int Cin, int H, int W, int Cout, int tiles_m, int tiles_w, int tiles_h, int dp_tiles,
    int ksplit, int cps, float* __restrict__ slab) {
  using C = FwdCfg<WM, WN, MI, NJ, CK, KS>;
  extern __shared__ __attribute__((aligned(16))) float lds[];

  // Schedule: workgroups [0, dp_tiles) each own a whole output tile (full K); the
  // remaining n_tail tiles are split ksplit ways over input-channel chunks, their raw
  // partial sums going to slab[(split, tail tile)] (reduced by fwd_tail_reduce_kernel).
  // Both ranges are XCD-remapped separately.
  const int n_tiles = tiles_m * tiles_w * tiles_h * N;
  const int n_tail = n_tiles - dp_tiles;
  const bool direct = (int)blockIdx.x < dp_tiles;
  int t, split = 0, ti = 0;
  if (direct) {
    t = xcd_remap(blockIdx.x, dp_tiles);
  } else {
    const int u = xcd_remap(blockIdx.x - dp_tiles, n_tail * ksplit);
    ti = u % n_tail;
    split = u / n_tail;
    t = dp_tiles + ti;
  }
  const int mt = t % tiles_m; t /= tiles_m;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h; t /= tiles_h;
  const int n = t;
  const int m0 = mt * C::BM, w0 = tw * C::TW, h0 = th * C::TH;
  const int pad = KS / 2;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, khalf = lane >> 5;

  const float* Xn = X + (size_t)n * Cin * H * W;
  const int nchunks = (Cin + CK - 1) / CK;
  const int Ktot = Cin * C::KK;

  // lane-constant operand bases (see header comment)
  const int a_base = khalf * C::HALF * C::BM + wm * MI * 32 + l32;
  const int b_base = khalf * (CK / 2) * C::PH * C::PW + wn * NJ * C::PW + l32;

  // ---- staging (strength-reduced): every thread keeps fixed 32-bit offsets; per chunk
  // only uniform bases change.  Loads are unconditional (invalid lanes read offset 0 of
  // the same buffer) and the validity bits zero the values at LDS-store time, after the
  // MFMA phase — a branch per load (or a select right after it) makes hipcc wait
  // vmcnt(0) at the load instead of at the store.
  constexpr int A_COLS = C::BM / 4;                 // float4 per A row
  constexpr int A_ROWS_IT = C::NT / A_COLS;          // A rows per iteration
  constexpr int A_IT = (C::KC + A_ROWS_IT - 1) / A_ROWS_IT;
  constexpr int PP = C::PH * C::PW;                  // patch positions per channel
  constexpr int B_PJ = (PP + C::NT - 1) / C::NT;     // positions per thread
  const int a_kk = tid / A_COLS, a_mm = (tid % A_COLS) * 4;
  const bool a_mok = m0 + a_mm < Cout;
  const int a_off = a_kk * Cout + m0 + a_mm;
  int b_r[B_PJ], b_c[B_PJ];
#pragma unroll
  for (int j = 0; j < B_PJ; ++j) {
    const int pos = tid + j * C::NT;
    b_r[j] = pos < PP ? pos / C::PW : 1 << 20;  // never in range when pos is past the patch
    b_c[j] = pos % C::PW;
  }
  const int HWi = H * W;
  float4 ra[A_IT];
  float rb[B_PJ][CK];
  unsigned amask = 0, bmask = 0;

  auto load_chunk = [&](int ch) {
    const int k0 = ch * C::KC;
    const float* Ab = Wk + (size_t)k0 * Cout;
    amask = 0;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int kk = a_kk + i * A_ROWS_IT;
      const bool ok = kk < C::KC && k0 + kk < Ktot && a_mok;
      amask |= (unsigned)ok << i;
      const int off = ok ? a_off + i * A_ROWS_IT * Cout : 0;
      if constexpr (VEC4) {
        ra[i] = *reinterpret_cast<const float4*>(Ab + off);
      } else {  // rows not 16-B aligned (e.g. dgrad of a 3-channel input): rare path
        const int m = m0 + a_mm;
        ra[i].x = Ab[off];
        ra[i].y = Ab[(ok && m + 1 < Cout) ? off + 1 : 0];
        ra[i].z = Ab[(ok && m + 2 < Cout) ? off + 2 : 0];
        ra[i].w = Ab[(ok && m + 3 < Cout) ? off + 3 : 0];
        if (!(m + 1 < Cout)) ra[i].y = 0.f;  // masked below only per float4
        if (!(m + 2 < Cout)) ra[i].z = 0.f;
        if (!(m + 3 < Cout)) ra[i].w = 0.f;
      }
    }
    const int ci0 = ch * CK;
    const int base = (ci0 * H + h0 - pad) * W + (w0 - pad);
    bmask = 0;
#pragma unroll
    for (int j = 0; j < B_PJ; ++j) {
      const int gh = h0 - pad + b_r[j], gw = w0 - pad + b_c[j];
      const bool pok = gh >= 0 && gh < H && gw >= 0 && gw < W;
      const int poff = base + b_r[j] * W + b_c[j];
#pragma unroll
      for (int i = 0; i < CK; ++i) {
        const bool ok = pok && ci0 + i < Cin;
        bmask |= (unsigned)ok << (j * CK + i);
        rb[j][i] = Xn[ok ? poff + i * HWi : 0];
      }
    }
  };
  auto store_chunk = [&](float* As, float* Bs) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int kk = a_kk + i * A_ROWS_IT;
      if (kk < C::KC) {
        const bool ok = (amask >> i) & 1;
        reinterpret_cast<float4*>(As)[kk * A_COLS + a_mm / 4] =
            ok ? ra[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < B_PJ; ++j) {
      const int pos = tid + j * C::NT;
      if (pos < PP) {
#pragma unroll
        for (int i = 0; i < CK; ++i)
          Bs[i * PP + pos] = ((bmask >> (j * CK + i)) & 1) ? rb[j][i] : 0.f;
      }
    }
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float* bias_s = lds + 2 * (C::A_ELEMS + C::B_ELEMS);
  float* scale_s = bias_s + C::BM;
  if (tid < C::BM) {
    const int co = min(m0 + tid, Cout - 1);
    bias_s[tid] = epi.bias ? epi.bias[co] : 0.f;
    scale_s[tid] = epi.scale ? epi.scale[co] : 1.f;
  }
  const int c_begin = direct ? 0 : split * cps;
  const int c_end = direct ? nchunks : min(nchunks, c_begin + cps);
  if (c_begin < c_end) {
    load_chunk(c_begin);
    store_chunk(lds, lds + C::A_ELEMS);
  }
  __syncthreads();

  for (int ch = c_begin; ch < c_end; ++ch) {
    const int it = ch - c_begin;
    const float* As = lds + (it & 1) * (C::A_ELEMS + C::B_ELEMS);
    const float* Bs = As + C::A_ELEMS;
    const float* Al = As + a_base;
    const float* Bl = Bs + b_base;
    const bool more = ch + 1 < c_end;
    if (more) load_chunk(ch + 1);
    // operands of step kk+PF are read while step kk's MFMAs run (PF-deep register ring;
    // every index is compile-time after unrolling)
    constexpr int PF = TLOD_CONV_PF;
    float a[PF + 1][MI], b[PF + 1][NJ];
    auto read_ops = [&](int kk, float (&ar)[MI], float (&br)[NJ]) {
      const int ci = kk / C::KK, s = kk % C::KK;
      const int boff = (ci * C::PH + s / KS) * C::PW + s % KS;
#pragma unroll
      for (int i = 0; i < MI; ++i) ar[i] = Al[kk * C::BM + i * 32];
#pragma unroll
      for (int j = 0; j < NJ; ++j) br[j] = Bl[boff + j * C::PW];
    };
#pragma unroll
    for (int kk = 0; kk < PF; ++kk) read_ops(kk, a[kk], b[kk]);
#pragma unroll
    for (int kk = 0; kk < C::HALF; ++kk) {
      if (kk + PF < C::HALF) read_ops(kk + PF, a[(kk + PF) % (PF + 1)], b[(kk + PF) % (PF + 1)]);
      const int q = kk % (PF + 1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma32(a[q][i], b[q][j], acc[i][j]);
#if TLOD_CONV_SGB
      // pin the interleave: this step's operand reads (for kk+PF) ahead of its MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, TLOD_CONV_SGB, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, MI * NJ, 0);
#endif
    }
    if (more) {
      float* Ad = lds + ((it + 1) & 1) * (C::A_ELEMS + C::B_ELEMS);
      store_chunk(Ad, Ad + C::A_ELEMS);
    }
    __syncthreads();
  }

  // epilogue: lane owns pixel column l32; rows (co) = (r&3) + 8*(r>>2) + 4*khalf.
  constexpr int TP = C::TH * C::TW;  // pixels per tile
  if (!direct) {  // raw partial sums, whole tile (the reduce bounds-checks)
    float* St = slab + ((size_t)split * n_tail + ti) * C::BM * TP;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
          St[ml * TP + (wn * NJ + j) * C::TW + l32] = acc[i][j][r];
        }
    return;
  }
  float* Yn = Y + (size_t)n * Cout * H * W;
  const float* Rn = epi.residual ? epi.residual + (size_t)n * Cout * H * W : nullptr;
  const bool has_scale = epi.scale != nullptr;
  const int w = w0 + l32;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int h = h0 + wn * NJ + j;
      if (h >= H || w >= W) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        const int co = m0 + ml;
        if (co < Cout) {
          const size_t idx = ((size_t)co * H + h) * W + w;
          float v = acc[i][j][r];
          if (has_scale) v *= scale_s[ml];
          v += bias_s[ml];
          if (Rn) v += Rn[idx];
          if (epi.relu) v = fmaxf(v, 0.f);
          v = epi_mask(epi, (size_t)n * Cout * H * W + idx, v);
          if (epi.s2d > 1) {
            const long long o = epi_out_index(epi, n, co, h, w, Cout, H, W);
            if (o >= 0) Y[o] = v;
          } else {
            Yn[idx] = v;
          }
        }
      }
    }
}

// ======================================================================= split-bf16 forward
// The same implicit GEMM on the bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16x the f32-input
// rate) with every f32 operand split exactly into three bf16 terms, x = hi + mid + lo
// (hi truncated, mid and lo round-to-nearest-even: hi keeps the top 8 mantissa bits, mid
// the next 8, lo the last 8; the remainders are exact in f32).  NP = 6 accumulates lo*hi, mid*mid, hi*lo, mid*hi, hi*mid,
// hi*hi (the dropped terms are < 2^-24 relative: f32-level error; measured normwise error
// vs fp64 ~1e-7, the same as the f32-input MFMA path); NP = 3 keeps the last three
// (~5e-6).  Products of bf16 pairs are exact in the f32 accumulator.
//
// KS = 3 only.  K order inside a chunk of 8 input channels is (tap, channel), and one
// 32x32x16 MFMA step covers two taps: lanes 0-31 take tap 2s, lanes 32-63 tap 2s+1 (step 4
// pairs tap 8 with a zero-weight pad tap), each reading its 8 channels as 16 contiguous
// bytes per plane.  Operands are split ONCE, when staged: the weights are pre-split in
// global memory (pack_bs_kernel, per weight version) and copied plane by plane; the input
// patch is split by the thread that stages it (one position x 8 channels) and stored as
// bf16 planes [pos][8 ch].  Weight rows use a 176-B pitch so the 16-lane ds_read_b128
// groups are conflict-free; patch positions are 16 B apart (conflict-free as is).

// kBsKP (bs_common.h): packed k per chunk, 10 taps (9 + zero pad) x 8 channels

// Band tiles (narrow maps, W <= ~100): a tile is 512 consecutive flattened pixels
// p = h*W + w (16 groups of 32, one per MFMA column block) instead of 16 rows x 32 columns,
// so a 37x75 map wastes 10% of the MFMA columns instead of 40%.  The staged input patch is
// then full-width rows h0-1 .. h1+1 of the band, at most kBandPos positions.
constexpr int kBandPos = 960;
__host__ __device__ constexpr bool band_fits(int W) { return (511 / W + 4) * (W + 2) <= kBandPos; }

template <int WM, int WN, int MI, int NJ, int NP, bool BAND = false>
struct BsCfg {
  static constexpr int NPL = NP == 6 ? 3 : 2;   // bf16 planes used
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * MI * 32;
  static constexpr int TH = WN * NJ, TW = 32;
  static constexpr int PH = TH + 2, PW = TW + 2, PP = PH * PW;
  static constexpr int CK = 8;
  static constexpr int STEPS = 5;               // tap pairs (0,1) (2,3) (4,5) (6,7) (8,pad)
  static constexpr int AROW = 176;              // bytes per weight row per plane (160 used)
  static constexpr int A_PLANE = BM * AROW;     // bytes
  static constexpr int BPOS = BAND ? kBandPos : PP;  // staged patch positions
  static constexpr int B_PLANE = BPOS * 16;     // bytes
  static constexpr int BUF = NPL * (A_PLANE + B_PLANE);
  static constexpr int LDS_BYTES = 2 * BUF + 2 * BM * 4;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int WM, int WN, int MI, int NJ, int NP, bool BAND>
__global__ void __launch_bounds__(WM* WN * 64) TLOD_CONV_OCC conv_fwd_bs_kernel(
    const float* __restrict__ X, const unsigned short* __restrict__ Wp, Epi epi,
    float* __restrict__ Y, int N, int Cin, int H, int W, int Cout, int tiles_m, int tiles_w,
    int tiles_h, int dp_tiles, int ksplit, int cps, float* __restrict__ slab) {
  using C = BsCfg<WM, WN, MI, NJ, NP, BAND>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int n_tiles = tiles_m * tiles_w * tiles_h * N;
  const int n_tail = n_tiles - dp_tiles;
  const bool direct = (int)blockIdx.x < dp_tiles;
  int t, split = 0, ti = 0;
  if (direct) {
    t = xcd_remap(blockIdx.x, dp_tiles);
  } else {
    const int u = xcd_remap(blockIdx.x - dp_tiles, n_tail * ksplit);
    ti = u % n_tail;
    split = u / n_tail;
    t = dp_tiles + ti;
  }
  const int mt = t % tiles_m; t /= tiles_m;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h; t /= tiles_h;
  const int n = t;
  const int HWi = H * W;
  // 2D tile: rows h0.., columns w0..; band tile: pixels p0 .. p0+511, patch rows from h0-1,
  // patch width PW = W + 2 (row pitch of the staged positions)
  const int m0 = mt * C::BM;
  const int p0 = tw * C::TH * C::TW;
  const int w0 = BAND ? 0 : tw * C::TW;
  const int h0 = BAND ? p0 / W : th * C::TH;
  const int PWr = BAND ? W + 2 : C::PW;
  const int PPr = BAND ? (min(p0 + C::TH * C::TW, HWi) - 1) / W - h0 + 3 : C::PH;  // patch rows
  const int npos = PPr * PWr;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, khalf = lane >> 5;

  const float* Xn = X + (size_t)n * Cin * H * W;
  const int nchunks = (Cin + C::CK - 1) / C::CK;
  const size_t wrow = (size_t)nchunks * kBsKP;       // packed row length (bf16)
  const size_t wplane = (size_t)Cout * wrow;         // packed plane length (bf16)

  // ---- operand byte offsets inside one LDS buffer
  const int a_base = (wm * MI * 32 + l32) * C::AROW + 16 * khalf;
  // B operand byte offset of tap t inside one buffer = b_lane (per lane) + tap_c(t) (uniform)
  const int b_lane = C::NPL * C::A_PLANE + (BAND ? 0 : (wn * NJ * C::PW + l32) * 16);
  auto tap_c = [&](int tap) {
    return (BAND ? (tap / 3 - 1) * PWr + tap % 3 - 1 : (tap / 3) * C::PW + tap % 3) * 16;
  };
  // offset of the pair (t0 for lanes 0-31, t1 for lanes 32-63)
  auto pair_off = [&](int t0, int t1) { return b_lane + (khalf ? tap_c(t1) : tap_c(t0)); };
  // band: this lane's pixel of column block j sits at patch position (h - h0 + 1, w + 1)
  int b_pix[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (BAND) {
      const int p = min(p0 + (wn * NJ + j) * 32 + l32, HWi - 1);
      const int h = p / W;
      b_pix[j] = ((h - h0 + 1) * PWr + p - h * W + 1) * 16;
    } else {
      b_pix[j] = j * C::PW * 16;
    }
  }

  // ---- staging.  A: NPL planes x BM rows x 10 16-B segments; B: PP positions x 8 ch.
  constexpr int A_SEG = kBsKP / 8;                   // 16-B segments per row per chunk
  constexpr int A_N = C::NPL * C::BM * A_SEG;
  constexpr int A_IT = (A_N + C::NT - 1) / C::NT;
  constexpr int B_IT = (C::BPOS + C::NT - 1) / C::NT;
  int a_lds[A_IT];
  unsigned a_gl[A_IT];  // element offsets of the chunk-0 segment (planes < 2^31 elements)
  unsigned a_valid = 0;
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    const int idx = tid + i * C::NT;
    const int pl = idx / (C::BM * A_SEG), rem = idx % (C::BM * A_SEG);
    const int row = rem / A_SEG, q = rem % A_SEG;
    const bool ok = idx < A_N && m0 + row < Cout;
    a_valid |= (unsigned)ok << i;
    a_lds[i] = idx < A_N ? pl * C::A_PLANE + row * C::AROW + 16 * q : -1;
    a_gl[i] = ok ? (unsigned)(pl * wplane + (size_t)(m0 + row) * wrow + 8 * q) : 0u;
  }
  int b_pos[B_IT], b_goff[B_IT];
  unsigned b_pvalid = 0;
#pragma unroll
  for (int i = 0; i < B_IT; ++i) {
    const int pos = tid + i * C::NT;
    const int r = pos / PWr, c = pos % PWr;
    const int gh = h0 - 1 + r, gw = w0 - 1 + c;
    const bool ok = pos < npos && gh >= 0 && gh < H && gw >= 0 && gw < W;
    b_pvalid |= (unsigned)ok << i;
    b_pos[i] = pos < npos ? C::NPL * C::A_PLANE + pos * 16 : -1;
    b_goff[i] = ok ? gh * W + gw : 0;
  }
  u32x4 ra[A_IT];
  float rb[B_IT][8];
  int nvalid = 0;  // input channels present in the staged chunk (uniform)

  // Loads are unconditional with 32-bit offsets from uniform per-chunk bases (invalid
  // positions read offset 0, channels past Cin re-read the last channel); validity is
  // applied when storing to LDS (see conv_fwd_kernel: a branch per load serialises them).
  auto load_chunk = [&](int ch) {
    const unsigned short* Wc = Wp + (size_t)ch * kBsKP;
#pragma unroll
    for (int i = 0; i < A_IT; ++i)
      ra[i] = *reinterpret_cast<const u32x4*>(Wc + a_gl[i]);
    const int ci0 = ch * C::CK;
    nvalid = min(C::CK, Cin - ci0);
    const float* Xc = Xn + (size_t)ci0 * HWi;
#pragma unroll
    for (int i = 0; i < B_IT; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) rb[i][e] = Xc[min(e, nvalid - 1) * HWi + b_goff[i]];
  };
  auto store_chunk = [&](unsigned char* buf) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i)
      if (a_lds[i] >= 0)
        *reinterpret_cast<u32x4*>(buf + a_lds[i]) = ((a_valid >> i) & 1) ? ra[i] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      if (b_pos[i] < 0) continue;
      float v[8];
      const bool pv = (b_pvalid >> i) & 1;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (pv && e < nvalid) ? rb[i][e] : 0.f;
      u32x4 sp[3];
      split8<C::NPL>(v, sp);
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        *reinterpret_cast<u32x4*>(buf + b_pos[i] + pl * C::B_PLANE) = sp[pl];
    }
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float* bias_s = reinterpret_cast<float*>(smem + 2 * C::BUF);
  float* scale_s = bias_s + C::BM;
  if (tid < C::BM) {
    const int co = min(m0 + tid, Cout - 1);
    bias_s[tid] = epi.bias ? epi.bias[co] : 0.f;
    scale_s[tid] = epi.scale ? epi.scale[co] : 1.f;
  }
  const int c_begin = direct ? 0 : split * cps;
  const int c_end = direct ? nchunks : min(nchunks, c_begin + cps);
  if (c_begin < c_end) {
    load_chunk(c_begin);
    store_chunk(smem);
  }
  if (c_begin + 1 < c_end) load_chunk(c_begin + 1);
  __syncthreads();

  // one k-step: A at per-lane byte offset aoff, B at boff (+ the lane's pixel offset)
  auto step = [&](const unsigned char* buf, int aoff, int boff) {
    u32x4 a[MI][3], b[NJ][3];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        a[i][pl] = *reinterpret_cast<const u32x4*>(buf + aoff + pl * C::A_PLANE + i * 32 * C::AROW);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        b[j][pl] = *reinterpret_cast<const u32x4*>(buf + boff + pl * C::B_PLANE + b_pix[j]);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bs_mac<NP>(acc[i][j], a[i][0], a[i][1], a[i][2], b[j][0], b[j][1], b[j][2]);
  };

  // Tap pairing over chunk pairs (no zero-pad MFMA work): the 18 (chunk, tap) units of the
  // pair (c, c+1) — chunk c in LDS buffer 0, chunk c+1 in buffer 1 — are consumed two per
  // k-step, unit u = 2s + khalf, so 9 k-steps cover 2 chunks instead of 10.  Chunk c+1 is
  // stored at step 2 and made visible before step 4 (the step that straddles the buffers);
  // chunk c+2 is stored into buffer 0 at step 6, after a barrier that retires step 4's
  // reads of it.  A lone last chunk runs (0,1) .. (6,7), (8, pad): the pad weights are 0.
  const int a_row = a_base - 16 * khalf;
  auto unit_a = [&](int u) { return (u >= 9 ? C::BUF : 0) + 16 * (u % 9); };
  auto unit_b = [&](int u) { return (u >= 9 ? C::BUF : 0) + tap_c(u % 9); };
  int c = c_begin;
  if (TLOD_TAP_PAIRING) {
    for (; c + 1 < c_end; c += 2) {
      const bool more2 = c + 2 < c_end;
#pragma unroll
      for (int st = 0; st < 9; ++st) {
        // (sched_barrier: the staging stays between the k-steps it was placed at — the
        // compiler otherwise sinks it below the remaining MFMAs, as in gemm.hip's K loop)
        if (st == 2) {
          __builtin_amdgcn_sched_barrier(0);
          store_chunk(smem + C::BUF);
          if (more2) load_chunk(c + 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (st == 4 || st == 5) __syncthreads();
        if (st == 6 && more2) {
          __builtin_amdgcn_sched_barrier(0);
          store_chunk(smem);
          if (c + 3 < c_end) load_chunk(c + 3);
          __builtin_amdgcn_sched_barrier(0);
        }
        step(smem, a_row + (khalf ? unit_a(2 * st + 1) : unit_a(2 * st)),
             b_lane + (khalf ? unit_b(2 * st + 1) : unit_b(2 * st)));
      }
      __syncthreads();
    }
  }
  for (; c < c_end; ++c) {  // lone last chunk (tap pairing) or every chunk (pad mode)
    const int it = c - c_begin;
    const bool more = c + 1 < c_end;
    const unsigned char* buf = smem + (it & 1) * C::BUF;
#pragma unroll
    for (int st = 0; st < C::STEPS; ++st) {
      if (more && st == 2) store_chunk(smem + ((it + 1) & 1) * C::BUF);
      step(buf, a_base + 32 * st, pair_off(min(2 * st, 8), min(2 * st + 1, 8)));
    }
    if (more && c + 2 < c_end) load_chunk(c + 2);
    __syncthreads();
  }

  // epilogue (identical to conv_fwd_kernel)
  constexpr int TP = C::TH * C::TW;
  if (!direct) {
    float* St = slab + ((size_t)split * n_tail + ti) * C::BM * TP;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
          St[ml * TP + (wn * NJ + j) * C::TW + l32] = acc[i][j][r];
        }
    return;
  }
  const bool has_scale = epi.scale != nullptr;
  if constexpr (!BAND && NJ == 2) {
    if (epi.pool) {
      // Fused max_pool2d(kernel 2, stride 2, floor): rows (j = 0, 1) are a window's two
      // rows, lanes (l32, l32 ^ 1) its two columns.  The window order and the update rule
      // (val > max || isnan(val)) are torch's max_pool2d forward, so the values are identical.
      const int Hp = H / 2, Wp = W / 2;
      float* Pn = epi.pool + (size_t)n * Cout * Hp * Wp;
      const int hp = (h0 + wn * NJ) / 2, wp = (w0 + l32) / 2;
      const bool writer = (l32 & 1) == 0 && hp < Hp && wp < Wp;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
          float v[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            v[j] = acc[i][j][r];
            if (has_scale) v[j] *= scale_s[ml];
            v[j] += bias_s[ml];
            if (epi.relu) v[j] = fmaxf(v[j], 0.f);
          }
          const float c0 = __shfl_xor(v[0], 1), c1 = __shfl_xor(v[1], 1);
          float m = v[0];
          if (c0 > m || __builtin_isnan(c0)) m = c0;
          if (v[1] > m || __builtin_isnan(v[1])) m = v[1];
          if (c1 > m || __builtin_isnan(c1)) m = c1;
          if (writer && m0 + ml < Cout) Pn[((size_t)(m0 + ml) * Hp + hp) * Wp + wp] = m;
        }
      return;
    }
  }
  float* Yn = Y + (size_t)n * Cout * H * W;
  const float* Rn = epi.residual ? epi.residual + (size_t)n * Cout * H * W : nullptr;
  const int w = w0 + l32;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int h = h0 + wn * NJ + j;
      const int pband = p0 + (wn * NJ + j) * 32 + l32;
      if (BAND ? pband >= HWi : (h >= H || w >= W)) continue;
      const int pix = BAND ? pband : h * W + w;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        const int co = m0 + ml;
        if (co < Cout) {
          const size_t idx = (size_t)co * HWi + pix;
          float v = acc[i][j][r];
          if (has_scale) v *= scale_s[ml];
          v += bias_s[ml];
          if (Rn) v += Rn[idx];
          if (epi.relu) v = fmaxf(v, 0.f);
          Yn[idx] = epi_mask(epi, (size_t)n * Cout * HWi + idx, v);
        }
      }
    }
}

// ------------------------------------------------------------ warp-specialized variant
// conv_fwd_bs_kernel's tile (64 output channels x TH x TW <= 512 pixels) and K order, with
//  * the staging on kProdWaves extra producer waves (one per SIMD): the 8 MFMA waves only
//    read LDS fragments and issue MFMAs, so the global-load waits, the split VALU and the
//    LDS stores of the next chunk overlap the other waves' MFMAs instead of stalling both
//    waves of a SIMD at once;
//  * 16x16x32 MFMAs (v_mfma_f32_16x16x32_bf16): the chip holds a higher clock on this shape
//    than on 32x32x16 for the same work (measured 2.10 vs 1.95 GHz on conv3_3).
// One work item per workgroup: a whole tile, or one split-K piece of a tail tile (an
// exiting workgroup's output stores drain while the next one stages; a persistent variant
// measured slower, round 3).  K is walked in frames of four chunks (chunks c, c+2 in LDS
// buffer 0, c+1, c+3 in buffer 1; 36 (tap, 8-channel) units = nine 16x16x32 k-steps), then
// chunk pairs (18 units = four 16x16x32 steps + one 16x16x16 step), then a lone chunk.
// Producers and MFMA waves run separate loops with the same barrier sequence, so neither
// carries the other's registers (the kernel fits 3 waves per SIMD).
constexpr int kProdWaves = 4;

// LDS image of one buffer: NPL weight planes [64 rows][160 B] (a row = 9 taps + a zero pad
// slot of 8 channels), then NPL input planes [(TH + 2) patch rows][PS positions][8
// channels].  Bank rules (MI355X_MICROARCH.md §LDS; modelled lane by lane with
// tools/lds/ws_model.py before the first run):
//  * A fragments (ds_read_b128, lane = (row l16, unit group g)): rows at the 160-B pitch put
//    each 16-lane group's two 8-row halves on the even slots of the bank row, offset by
//    their units' slots; units 4s+g and 4s+g+1 are an odd number of 16-B slots apart (one
//    tap, or the odd buffer size BUF / 16 +- 8) — conflict-free.
//  * B fragments are read as two ds_read_b64 (32-lane groups g = 0, 1 and g = 2, 3): in the
//    first read the even-g lanes take bytes 0-7 of their unit and the odd-g lanes bytes
//    8-15, in the second the other halves, so the two unit groups of a 32-lane group use
//    disjoint bank halves whatever their taps.  The odd-g lanes' fragment is then (channels
//    4-7, 0-3), so the producers store the weight units odd-g lanes read (units 4s+g odd,
//    i.e. tap + buffer odd) with their 8-B halves swapped.  A block of 16 pixels must then
//    cover 16 distinct bank slots: the patch row pitch PS is TW + 16 when a block can wrap a
//    tile row (PS = TW mod 16), TW + 2 when it cannot (TW a multiple of 16).
//    (Round 4's single ds_read_b128 per unit conflicted 2-way in most groups: the two unit
//    groups of a 16-lane group read taps 1 .. PW apart — 20% of the kernel's LDS cycles.)
//  * the producers' stores are contiguous 16-B slots (ds_write_b128).
constexpr int kWsPos = 768;     // real patch positions (TH + 2) (TW + 2): 3 per producer lane
constexpr int kWsAlloc = 1056;  // staged positions (TH + 2) * PS, row padding included
__host__ __device__ constexpr int ws_pitch(int tw) { return tw % 16 == 0 ? tw + 2 : tw + 16; }
template <int WM, int WN, int MI, int NJ, int NP>
struct WsCfg : BsCfg<WM, WN, MI, NJ, NP, false> {
  using B = BsCfg<WM, WN, MI, NJ, NP, false>;
  // plane strides 16 B past a multiple of 512 B: the compiler would otherwise fuse two
  // planes' ds_read_b64 into one ds_read2st64_b64 (mod-32 banks in 16-lane groups: 2x the
  // conflicts, measured)
  static constexpr int AROW = 160;
  static constexpr int A_PLANE = B::BM * AROW + 16;
  static constexpr int TPIX = B::TH * B::TW;  // MFMA pixels per tile (512)
  static constexpr int B_PLANE = kWsAlloc * 16 + 16;
  static constexpr int BUF0 = B::NPL * (A_PLANE + B_PLANE);
  static constexpr int BUF = (BUF0 / 16) % 2 == 0 ? BUF0 + 16 : BUF0;  // odd # of 16-B slots
  static constexpr int AUX = 2 * BUF;  // (bias, scale) of the item
  static constexpr int LDS_BYTES = AUX + 2 * B::BM * 4;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

typedef short bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16_bf16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16k16_bf16(u32x2 a, u32x2 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(bf16x4, a),
                                                   __builtin_bit_cast(bf16x4, b), c, 0, 0, 0);
}
// bs_mac on a 16x16 tile: the k-step's products summed from zero (small ones first), then
// added to the running accumulator with one f32 add (TLOD_BS_KSUM16, see bs_mac)
template <int NP, typename V, typename F>
__device__ __forceinline__ void bs_mac16(f32x4& acc, const V (&a)[3], const V (&b)[3], F mf) {
  if (TLOD_BS_KSUM16) {
    f32x4 t = mf(a[1], b[0], f32x4{0.f, 0.f, 0.f, 0.f});
    t = mf(a[0], b[1], t);
    if constexpr (NP == 6) {
      t = mf(a[2], b[0], t);
      t = mf(a[1], b[1], t);
      t = mf(a[0], b[2], t);
    }
    acc += mf(a[0], b[0], t);
    return;
  }
  acc = mf(a[0], b[0], acc);
  acc = mf(a[1], b[0], acc);
  acc = mf(a[0], b[1], acc);
  if constexpr (NP == 6) {
    acc = mf(a[2], b[0], acc);
    acc = mf(a[1], b[1], acc);
    acc = mf(a[0], b[2], acc);
  }
}

// The work item of workgroup v: a whole tile (direct) or one split-K piece of a tail tile,
// decoded exactly as conv_fwd_bs_kernel decodes its block id.
struct WsItem {
  int direct, split, ti, n, m0, h0, w0, c_begin, c_end;
};
__device__ __forceinline__ WsItem ws_item(int v, int tiles_m, int tiles_w, int tiles_h,
                                          int dp_tiles, int n_tail, int ksplit, int cps,
                                          int nchunks, int BM, int TH, int TW) {
  WsItem it;
  int t;
  it.direct = v < dp_tiles;
  if (it.direct) {
    t = xcd_remap(v, dp_tiles);
    it.split = it.ti = 0;
  } else {
    const int u = xcd_remap(v - dp_tiles, n_tail * ksplit);
    it.ti = u % n_tail;
    it.split = u / n_tail;
    t = dp_tiles + it.ti;
  }
  const int mt = t % tiles_m; t /= tiles_m;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h; t /= tiles_h;
  it.n = t;
  it.m0 = mt * BM;
  it.w0 = tw * TW;
  it.h0 = th * TH;
  it.c_begin = it.direct ? 0 : it.split * cps;
  it.c_end = it.direct ? nchunks : min(nchunks, it.c_begin + cps);
  return it;
}

template <int WM, int WN, int MI, int NJ, int NP>
__global__ void __launch_bounds__(WM* WN * 64 + kProdWaves * 64)
    __attribute__((amdgpu_waves_per_eu(3, 3))) conv_fwd_bs_ws_kernel(
        const float* __restrict__ X, const unsigned short* __restrict__ Wp, Epi epi,
        float* __restrict__ Y, int N, int Cin, int H, int W, int Cout, int tiles_m, int tiles_w,
        int tiles_h, int dp_tiles, int ksplit, int cps, float* __restrict__ slab, int TH, int TW) {
  using C = WsCfg<WM, WN, MI, NJ, NP>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int n_tail = tiles_m * tiles_w * tiles_h * N - dp_tiles;
  const int HWi = H * W;
  const int nchunks = (Cin + C::CK - 1) / C::CK;
  const int tid = threadIdx.x;
  const int PW = TW + 2, PP = (TH + 2) * PW;  // real patch: row length, positions
  const int PS = ws_pitch(TW);                 // staged row pitch (positions)
  const WsItem it = ws_item(blockIdx.x, tiles_m, tiles_w, tiles_h, dp_tiles, n_tail, ksplit,
                            cps, nchunks, C::BM, TH, TW);
  const int c_begin = it.c_begin, c_end = it.c_end;

  if (tid >= C::NT) {
    // ================= producers: stage chunks into the two LDS buffers
    // Chunk p of the item sits in register slot p & 1 (= its LDS buffer) from its load until
    // its store, which then loads chunk p + 2 into the slot: a chunk's loads have two
    // chunk-steps to land.  Raw buffer loads, no element masks: rows past Cout and
    // positions outside the map take offset kBufOOB, channels past Cin fall past the
    // image's range — all read 0 (no 64-bit address math, no selects).
    constexpr int PT = kProdWaves * 64;
    const int ptid = tid - C::NT;
    const unsigned wrow = (unsigned)nchunks * kBsKP;  // packed row length (bf16)
    const unsigned wplane = (unsigned)Cout * wrow;    // packed plane length (bf16)
    const i32x4 w_rsrc = make_buffer_rsrc(Wp, wplane * C::NPL * 2u);
    const i32x4 x_rsrc = make_buffer_rsrc(X + (size_t)it.n * Cin * HWi, (unsigned)Cin * HWi * 4u);
    constexpr int A_SEG = kBsKP / 8;  // 16-B segments (tap slots) per weight row
    constexpr int A_N = C::NPL * C::BM * A_SEG;
    constexpr int A_IT = (A_N + PT - 1) / PT;
    constexpr int B_IT = (kWsPos + PT - 1) / PT;
    // a lane's segments all have the parity of ptid (PT and the row / plane lengths are
    // even): the segment of tap q in buffer S is stored half-swapped iff q + S is odd
    const bool a_odd = ptid & 1;
    int a_lds[A_IT], a_vo[A_IT];
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int idx = ptid + i * PT;
      const int pl = idx / (C::BM * A_SEG), rem = idx % (C::BM * A_SEG);
      const int row = rem / A_SEG, q = rem % A_SEG;
      a_lds[i] = idx < A_N ? pl * C::A_PLANE + row * C::AROW + 16 * q : -1;
      a_vo[i] = idx < A_N && it.m0 + row < Cout
                    ? (int)(((unsigned)pl * wplane + 8u * q + (unsigned)(it.m0 + row) * wrow) * 2u)
                    : kBufOOB;
    }
    int b_lds[B_IT], b_vo[B_IT];
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int pos = ptid + i * PT;
      const int r = pos / PW, c = pos % PW;
      const int gh = it.h0 - 1 + r, gw = it.w0 - 1 + c;
      b_lds[i] = pos < PP ? C::NPL * C::A_PLANE + (r * PS + c) * 16 : -1;
      b_vo[i] = pos < PP && gh >= 0 && gh < H && gw >= 0 && gw < W ? (gh * W + gw) * 4 : kBufOOB;
    }
    u32x4 ra2[2][A_IT];
    float rb2[2][B_IT][8];
    auto load2 = [&](auto slc, int ch) {  // chunk ch -> slot S (unconditional)
      constexpr int S = decltype(slc)::value;
      const int cbytes = ch * C::CK * HWi * 4;
#pragma unroll
      for (int i = 0; i < A_IT; ++i)
        ra2[S][i] = __builtin_bit_cast(u32x4, raw_buffer_load_v4f32(w_rsrc, a_vo[i], ch * (kBsKP * 2), 0));
#pragma unroll
      for (int i = 0; i < B_IT; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          rb2[S][i][e] = raw_buffer_load_f32(x_rsrc, b_vo[i], cbytes + e * HWi * 4, 0);
    };
    auto store2 = [&](auto slc, int ch_next) {  // slot S -> LDS buffer S; load ch_next into S
      constexpr int S = decltype(slc)::value;
      unsigned char* buf = smem + S * C::BUF;
      const bool swap = a_odd != (S == 1);
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        const u32x4 v = ra2[S][i];
        const u32x4 vs = swap ? u32x4{v[2], v[3], v[0], v[1]} : v;
        if (a_lds[i] >= 0) *reinterpret_cast<u32x4*>(buf + a_lds[i]) = vs;
      }
#pragma unroll
      for (int i = 0; i < B_IT; ++i) {
        if (b_lds[i] < 0) continue;
        u32x4 sp[3];
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v8[e] = rb2[S][i][e];
        split8<C::NPL>(v8, sp);
#pragma unroll
        for (int pl = 0; pl < C::NPL; ++pl)
          *reinterpret_cast<u32x4*>(buf + b_lds[i] + pl * C::B_PLANE) = sp[pl];
      }
      // unconditional (a chunk past the item reads zeros / stale pack rows, never stored),
      // so the compiler's vmcnt waits keep the other slot's loads in flight
      load2(slc, ch_next);
    };
    const std::integral_constant<int, 0> S0;
    const std::integral_constant<int, 1> S1;
    load2(S0, c_begin);
    if (c_begin + 1 < c_end) load2(S1, c_begin + 1);
    store2(S0, c_begin + 2);                            // chunk c_begin
    if (c_end - c_begin >= 2) store2(S1, c_begin + 3);  // chunk c_begin + 1
    __syncthreads();
    int c = c_begin;
    for (; c + 3 < c_end; c += 4) {  // barriers F1..F7 as in the MFMA waves' frame
      if (c != c_begin) store2(S1, c + 3);  // chunk c+1 (buffer 1 retired at F7)
      __syncthreads();                      // F1: c+1 visible
      __syncthreads();                      // F2: buffer 0 (chunk c) retired
      store2(S0, c + 4);                    // chunk c+2
      __syncthreads();                      // F3: c+2 visible
      __syncthreads();                      // F4: buffer 1 (chunk c+1) retired
      store2(S1, c + 5);                    // chunk c+3
      __syncthreads();                      // F5: c+3 visible
      __syncthreads();                      // F6: buffer 0 (chunk c+2) retired
      if (c + 4 < c_end) store2(S0, c + 6);  // chunk c+4
      __syncthreads();                      // F7: buffer 1 retired, c+4 visible
    }
    for (; c + 1 < c_end; c += 2) {
      if (c != c_begin) store2(S1, c + 3);  // chunk c+1
      __syncthreads();
      __syncthreads();
      if (c + 2 < c_end) store2(S0, c + 4);  // chunk c+2
      __syncthreads();
    }
    if ((c_end - c_begin) & 1) __syncthreads();  // the lone last chunk retires buffer 0
    return;
  }

  // ================= MFMA waves
  // The wave's 64 x 64 output block is 4 x 4 tiles of 16 x 16 (row block rb = 16 output
  // channels; column block cb = 16 pixels).  One k-step takes four (tap, 8-channel) units,
  // lane group g = lane / 16 reading unit 4s + g; the 16x16x16 step takes units 16, 17
  // (lanes 0-31 / 32-63, 8-B halves by (lane / 16) & 1).
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int l16 = lane & 15, g = lane >> 4;
  constexpr int RB = MI * 2, CB = NJ * 2;
  const int a_lane = (wm * MI * 32 + l16) * C::AROW;
  auto tap_c = [&](int tap) { return ((tap / 3) * PS + tap % 3) * 16; };
  // column block cb: this lane's pixel q = 64 wn + 16 cb + l16 of the tile in row-major (r,
  // c) = (q / TW, q % TW) order (a block may wrap a tile row), at staged position r PS + c
  // for tap (0, 0), plus the lane's first-read half (8 B for odd g); pixels past the tile
  // read a pixel of the tile (their results are never stored)
  const int hb = 8 * (g & 1);
  int bpix[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const int q = (wn * 64 + cb * 16 + l16) % (TH * TW);
    bpix[cb] = C::NPL * C::A_PLANE + ((q / TW) * PS + q % TW) * 16 + hb;
  }
  // (the asm keeps the compiler from hoisting all 20 (unit, block) sums out of the loop
  // into registers)
  auto baddr = [&](int cb, int bo) {
    int bp = bpix[cb];
    asm volatile("" : "+v"(bp));
    return bo + bp;
  };
  auto ua = [&](int u) { return (u >= 9 ? C::BUF : 0) + 16 * (u % 9); };
  auto ub = [&](int u) { return (u >= 9 ? C::BUF : 0) + tap_c(u % 9); };
  // k-step s of a four-chunk frame: lane group g reads unit u = 4s + g of the frame's 36,
  // i.e. chunk u / 9 (buffer (u / 9) & 1), tap u % 9; steps 0-3 are also the pair steps
  // (computed per step from an opaque copy of g: nine hoisted offset pairs spill)
  auto aoff_s = [&](int s) {
    int gg = g;
    asm volatile("" : "+v"(gg));
    return a_lane + ua((4 * s + gg) % 18);
  };
  auto boff_s = [&](int s) {
    int gg = g;
    asm volatile("" : "+v"(gg));
    return ub((4 * s + gg) % 18);
  };
  // 16x16x16 step of a pair: lanes 0-31 unit 16 (unswapped), 32-63 unit 17 (stored
  // half-swapped: the A half is the other one)
  const int aoff4 = a_lane + ua(16 + (lane >> 5)) + ((lane >> 5) ? 8 - hb : hb);
  const int boff4 = ub(16 + (lane >> 5));
  // lone last chunk: (8, pad) — slot 9 of a weight row is zero; tap 8 of buffer 0 unswapped
  const int aoffL = a_lane + 16 * (8 + (lane >> 5)) + hb, boffL = tap_c(8);

  f32x4 acc[RB][CB];
  auto step16 = [&](int ao, int bo) {
    u32x4 a[RB][3];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        a[rb][pl] = *reinterpret_cast<const u32x4*>(smem + ao + pl * C::A_PLANE + rb * 16 * C::AROW);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int b0 = baddr(cb, bo), b1 = b0 ^ 8;  // this lane's two 8-B halves, in order
      u32x4 b[3];
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + b0 + pl * C::B_PLANE);
        const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + b1 + pl * C::B_PLANE);
        b[pl] = u32x4{lo[0], lo[1], hi[0], hi[1]};
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) bs_mac16<NP>(acc[rb][cb], a[rb], b, mfma16_bf16);
    }
  };
  auto step8 = [&](int ao, int bo) {
    u32x2 a[RB][3];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        a[rb][pl] = *reinterpret_cast<const u32x2*>(smem + ao + pl * C::A_PLANE + rb * 16 * C::AROW);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      u32x2 b[3];
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        b[pl] = *reinterpret_cast<const u32x2*>(smem + baddr(cb, bo) + pl * C::B_PLANE);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) bs_mac16<NP>(acc[rb][cb], a[rb], b, mfma16k16_bf16);
    }
  };

  constexpr int TP = C::TPIX;
  const bool has_scale = epi.scale != nullptr;
  float* bias_s = reinterpret_cast<float*>(smem + C::AUX);
  float* scale_s = bias_s + C::BM;
  if (tid < C::BM) {
    const int co = min(it.m0 + tid, Cout - 1);
    bias_s[tid] = epi.bias ? epi.bias[co] : 0.f;
    scale_s[tid] = epi.scale ? epi.scale[co] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  int c = c_begin;
  // Four chunks (36 (tap, 8-channel) units) are nine 16x16x32 k-steps; a chunk pair's 18
  // units leave a 16x16x16 step, which issues at the 16x16x32's 16 cycles for half the
  // work (tools/probe/mfma_rate.hip), so whole frames run first.  Steps 2, 4 and 6 read
  // two chunks (both buffers); a buffer is refilled once its chunk's last step is done.
  for (; c + 3 < c_end; c += 4) {
    step16(aoff_s(0), boff_s(0));
    step16(aoff_s(1), boff_s(1));
    __syncthreads();  // F1
    step16(aoff_s(2), boff_s(2));
    __syncthreads();  // F2
    step16(aoff_s(3), boff_s(3));
    __syncthreads();  // F3
    step16(aoff_s(4), boff_s(4));
    __syncthreads();  // F4
    step16(aoff_s(5), boff_s(5));
    __syncthreads();  // F5
    step16(aoff_s(6), boff_s(6));
    __syncthreads();  // F6
    step16(aoff_s(7), boff_s(7));
    step16(aoff_s(8), boff_s(8));
    __syncthreads();  // F7
  }
  for (; c + 1 < c_end; c += 2) {
    step16(aoff_s(0), boff_s(0));
    step16(aoff_s(1), boff_s(1));
    __syncthreads();  // chunk c+1 visible
    step16(aoff_s(2), boff_s(2));
    __syncthreads();  // buffer 0 retired
    step16(aoff_s(3), boff_s(3));
    step8(aoff4, boff4);
    __syncthreads();
  }
  if (c < c_end) {
    step16(aoff_s(0), boff_s(0));
    step16(aoff_s(1), boff_s(1));
    step8(aoffL, boffL);
    __syncthreads();
  }

  // epilogue: the lane holds rows 4g..4g+3 of column l16 of each 16 x 16 tile
  if (!it.direct) {
    float* St = slab + ((size_t)it.split * n_tail + it.ti) * C::BM * TP;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wm * MI * 32 + rb * 16 + 4 * g + r;
          St[ml * TP + wn * 64 + cb * 16 + l16] = acc[rb][cb][r];
        }
    return;
  }
  if constexpr (NJ == 2) {
    if (epi.pool) {
      // max_pool2d(2, 2) window (16 x 32 tiles only, see ws_tile): pixel rows j = 0, 1
      // (column blocks hh and 2 + hh), columns (l16, l16 ^ 1); torch's window order and
      // update rule, as conv_fwd_bs_kernel
      const int Hp = H / 2, Wp2 = W / 2;
      float* Pn = epi.pool + (size_t)it.n * Cout * Hp * Wp2;
      const int hp = (it.h0 + wn * NJ) / 2;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int wp = (it.w0 + hh * 16 + l16) / 2;
        const bool writer = (l16 & 1) == 0 && hp < Hp && wp < Wp2;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ml = wm * MI * 32 + rb * 16 + 4 * g + r;
            float v2[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              v2[j] = acc[rb][j * 2 + hh][r];
              if (has_scale) v2[j] *= scale_s[ml];
              v2[j] += bias_s[ml];
              if (epi.relu) v2[j] = fmaxf(v2[j], 0.f);
            }
            const float c0 = __shfl_xor(v2[0], 1), c1 = __shfl_xor(v2[1], 1);
            float m = v2[0];
            if (c0 > m || __builtin_isnan(c0)) m = c0;
            if (v2[1] > m || __builtin_isnan(v2[1])) m = v2[1];
            if (c1 > m || __builtin_isnan(c1)) m = c1;
            if (writer && it.m0 + ml < Cout) Pn[((size_t)(it.m0 + ml) * Hp + hp) * Wp2 + wp] = m;
          }
      }
      return;
    }
  }
  // Branch-free: 32-bit offsets into the image's planes through buffer resources; an
  // element outside the tile / map / Cout gets offset kBufOOB, which the hardware drops
  // (store) or reads as 0 (residual / mask load).  The per-element bounds checks and 64-bit
  // addresses of a plain store epilogue compiled to ~10 branchy instructions per element:
  // 29k of a tile's 317k cycles with the stores themselves removed (round 4).
  const size_t img_off = (size_t)it.n * Cout * HWi;
  const unsigned plane_bytes = (unsigned)Cout * HWi * 4u;
  const i32x4 y_rsrc = make_buffer_rsrc(Y + img_off, plane_bytes);
  const float* Rn = epi.residual ? epi.residual + img_off : nullptr;
  const float* Mn = epi.mask ? epi.mask + img_off : nullptr;
  const i32x4 r_rsrc = make_buffer_rsrc(Rn ? Rn : Y, Rn ? plane_bytes : 0u);
  const i32x4 m_rsrc = make_buffer_rsrc(Mn ? Mn : Y, Mn ? plane_bytes : 0u);
  int pixo[CB];  // byte offset of the lane's pixel in a channel plane (-1: none)
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const int q = wn * 64 + cb * 16 + l16;
    const int h = it.h0 + q / TW, w = it.w0 + q % TW;
    pixo[cb] = q < TH * TW && h < H && w < W ? (h * W + w) * 4 : -1;
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    int off[CB][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = it.m0 + wm * MI * 32 + rb * 16 + 4 * g + r;
      const int rowo = co < Cout ? co * HWi * 4 : -1;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) off[cb][r] = (rowo | pixo[cb]) >= 0 ? rowo + pixo[cb] : kBufOOB;
    }
    // residual / mask operands of the row block loaded together, ahead of its stores
    float ext[CB][4], msk[CB][4];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ext[cb][r] = Rn ? raw_buffer_load_f32(r_rsrc, off[cb][r], 0, 0) : 0.f;
        msk[cb][r] = Mn ? raw_buffer_load_f32(m_rsrc, off[cb][r], 0, 0) : 1.f;
      }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = wm * MI * 32 + rb * 16 + 4 * g + r;
        float val = acc[rb][cb][r];
        if (has_scale) val *= scale_s[ml];
        val += bias_s[ml];
        if (Rn) val += ext[cb][r];
        if (epi.relu) val = fmaxf(val, 0.f);
        if (Mn && !(msk[cb][r] > 0.f)) val = 0.f;
        raw_buffer_store_f32(val, y_rsrc, off[cb][r], 0, 0);
      }
  }
}

// Packed, pre-split weights for conv_fwd_bs_kernel: three bf16 planes (hi, mid, lo of the
// exact split: truncated hi, round-to-nearest-even mid and lo; bs_common.h split2), each P[pl][o][c*80 + s*8 + e] = weight of output row o, input
// channel c*8+e, tap s (0 for s = 9 — the pad tap — and past the last channel).  dgrad = 1
// packs the transposed, flipped operand (rows = input channels, inputs = output channels,
// tap 8-s).
__global__ void pack_bs_kernel(const float* __restrict__ Wt, unsigned short* __restrict__ P,
                               int rows, int ins, int nchunks, int dgrad,
                               const float* __restrict__ oscale) {
  // oscale (optional): weight[co] * oscale[co] per output channel co before the split (a
  // frozen BatchNorm's scale after the conv, tlod_conv_pack_bs_ex)
  // one thread per (row o, chunk c, tap slot s): 8 input channels -> one 16-B store per plane
  const size_t rowlen = (size_t)nchunks * kBsKP;
  const size_t plane = (size_t)rows * rowlen;
  const size_t units = (size_t)rows * nchunks * 10;
  for (size_t u = blockIdx.x * (size_t)blockDim.x + threadIdx.x; u < units;
       u += (size_t)gridDim.x * blockDim.x) {
    const int s = (int)(u % 10);
    const size_t oc = u / 10;
    const int c = (int)(oc % nchunks), o = (int)(oc / nchunks);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int in = c * 8 + e;
      v[e] = 0.f;
      if (in < ins && s < 9) {
        v[e] = dgrad ? Wt[((size_t)in * rows + o) * 9 + (8 - s)] : Wt[((size_t)o * ins + in) * 9 + s];
        if (oscale != nullptr) v[e] *= oscale[dgrad ? in : o];
      }
    }
    u32x4 sp[3];
    split8<3>(v, sp);
    const size_t i0 = (size_t)o * rowlen + (size_t)c * kBsKP + s * 8;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(P + pl * plane + i0) = sp[pl];
  }
}

// ======================================================================= wgrad
// Block tile: BM = WM*MI*32 output channels x BN = WN*NJ*32 GEMM columns n=(ci,kh,kw);
// K = pixels, chunked as TH=2 rows x 32 columns.  The MFMA pairs pixel (0, c) with
// (1, c) (lanes 0-31 / 32-63): +1 row, a lane-constant offset.  grid.y = split-K slices.
template <int WM, int WN, int MI, int NJ, int KS, int TH_>
struct WgCfg {
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * MI * 32;
  static constexpr int BN = WN * NJ * 32;
  static constexpr int KK = KS * KS;
  static constexpr int TH = TH_, TW = 32, P = TH * TW;  // pixels per chunk
  static constexpr int KSTEPS = P / 2;
  static constexpr int PH = TH + KS - 1, PW = TW + KS - 1;
  // LDS patch pitch: row pitch PWP = KS (mod 32) and channel stride CSTR = KK (mod 32), so
  // the 32 consecutive GEMM columns (ci, kh, kw) a half-wave reads hit 32 distinct banks.
  // (KS == 1: one tap per channel, so an odd channel stride suffices.)
  static constexpr int PWP = KS == 1 ? PW : PW + (((KS - PW) % 32) + 32) % 32;
  static constexpr int CSTR =
      KS == 1 ? (PH * PW) | 1 : PH * PWP + (((KK - PH * PWP) % 32) + 32) % 32;
  // MFMA k pairing: lanes 32-63 take pixel p + P/2 (next row if TH == 2, +16 cols if 1)
  static constexpr int PAIR_X = (TH == 2) ? PWP : 16;
  static constexpr int NCI = BN / KK + 2;           // channels a column tile can span
  static constexpr int GP = BM + 1;                  // padded pitch of Gs[p][m]
  static constexpr int G_ELEMS = P * GP;
  static constexpr int X_ELEMS = NCI * CSTR + 48;    // + a zero row for dead columns
  static constexpr int LDS_FLOATS = 2 * (G_ELEMS + X_ELEMS);
  static_assert(TH == 1 || TH == 2, "TH");
  static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};

template <int WM, int WN, int MI, int NJ, int KS, int TH>
__global__ void __launch_bounds__(WM* WN * 64) TLOD_CONV_OCC conv_wgrad_kernel(
    const float* __restrict__ G, const float* __restrict__ X, float* __restrict__ slab, int N,
    int Cin, int H, int W, int Cout, int tiles_m, int tiles_n, int splits, int chunks_per_split) {
  using C = WgCfg<WM, WN, MI, NJ, KS, TH>;
  extern __shared__ __attribute__((aligned(16))) float lds[];

  const int nwg = tiles_m * tiles_n * splits;
  int t = xcd_remap(blockIdx.x, nwg);
  const int mt = t % tiles_m; t /= tiles_m;
  const int nt = t % tiles_n;
  const int split = t / tiles_n;
  const int m0 = mt * C::BM, n0 = nt * C::BN;
  const int Ktot = Cin * C::KK;
  const int cb = n0 / C::KK;
  const int pad = KS / 2;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, khalf = lane >> 5;

  const int cw = (W + C::TW - 1) / C::TW, chh = (H + C::TH - 1) / C::TH;
  const int total_chunks = N * chh * cw;
  const int c_begin = split * chunks_per_split;
  const int c_end = min(total_chunks, c_begin + chunks_per_split);

  // per-lane B column offsets into Xs (+1 patch row for the khalf=1 pixel row); dead
  // columns read the zero row at the end of the patch
  const int zero_row = C::NCI * C::CSTR;
  int boff[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + wn * NJ * 32 + j * 32 + l32;
    if (col < Ktot) {
      const int ci = col / C::KK - cb, s = col % C::KK;
      boff[j] = ci * C::CSTR + (s / KS) * C::PWP + s % KS + khalf * C::PAIR_X;
    } else {
      boff[j] = zero_row;
    }
  }
  const int a_base = khalf * (C::P / 2) * C::GP + wm * MI * 32 + l32;

  // ---- staging (strength-reduced, see conv_fwd_kernel)
  constexpr int G_ROWS_IT = C::NT / C::P;            // G rows (channels) per iteration
  constexpr int G_IT = C::BM / G_ROWS_IT;
  constexpr int PP = C::PH * C::PW;
  constexpr int X_CS = C::NT / PP > 0 ? C::NT / PP : 1;  // channel sub-groups
  constexpr int X_IT = (C::NCI + X_CS - 1) / X_CS;
  static_assert(C::NT % C::P == 0 && C::BM % G_ROWS_IT == 0, "G staging shape");
  static_assert(PP <= C::NT, "X patch row must fit the workgroup");
  const int g_p = tid % C::P, g_m = tid / C::P;
  const int g_dh = g_p / C::TW, g_dw = g_p % C::TW;
  const int x_pos = tid % PP, x_cs = tid / PP;
  const bool x_act = x_cs < X_CS;
  const int x_r = x_pos / C::PW, x_c = x_pos % C::PW;
  const int HWi = H * W;
  float rg[G_IT];
  float rx[X_IT];
  unsigned gmask = 0, xmask = 0;

  auto load_chunk = [&](int c) {
    const int cwi = c % cw, r = c / cw;
    const int chi = r % chh, n = r / chh;
    const int h0 = chi * C::TH, w0 = cwi * C::TW;
    const float* Gn = G + (size_t)n * Cout * HWi;
    const float* Xn = X + (size_t)n * Cin * HWi;
    const bool pok = (h0 + g_dh < H) && (w0 + g_dw < W);
    const int goff = (m0 + g_m) * HWi + (h0 + g_dh) * W + w0 + g_dw;
    gmask = 0;
#pragma unroll
    for (int i = 0; i < G_IT; ++i) {
      const bool ok = pok && (m0 + g_m + i * G_ROWS_IT < Cout);
      gmask |= (unsigned)ok << i;
      rg[i] = Gn[ok ? goff + i * G_ROWS_IT * HWi : 0];
    }
    const int gh = h0 - pad + x_r, gw = w0 - pad + x_c;
    const bool xpok = x_act && gh >= 0 && gh < H && gw >= 0 && gw < W;
    const int xoff = (cb + x_cs) * HWi + gh * W + gw;
    xmask = 0;
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
      const int ci = x_cs + i * X_CS;
      const bool ok = xpok && ci < C::NCI && cb + ci < Cin;
      xmask |= (unsigned)ok << i;
      rx[i] = Xn[ok ? xoff + i * X_CS * HWi : 0];
    }
  };
  auto store_chunk = [&](float* Gs, float* Xs) {
#pragma unroll
    for (int i = 0; i < G_IT; ++i)
      Gs[g_p * C::GP + g_m + i * G_ROWS_IT] = ((gmask >> i) & 1) ? rg[i] : 0.f;
    if (x_act) {
#pragma unroll
      for (int i = 0; i < X_IT; ++i) {
        const int ci = x_cs + i * X_CS;
        if (ci < C::NCI) Xs[ci * C::CSTR + x_r * C::PWP + x_c] = ((xmask >> i) & 1) ? rx[i] : 0.f;
      }
    }
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int BUF = C::G_ELEMS + C::X_ELEMS;
  for (int i = tid; i < C::X_ELEMS - zero_row; i += C::NT) {
    lds[C::G_ELEMS + zero_row + i] = 0.f;
    lds[BUF + C::G_ELEMS + zero_row + i] = 0.f;
  }
  if (c_begin < c_end) {
    load_chunk(c_begin);
    store_chunk(lds, lds + C::G_ELEMS);
  }
  __syncthreads();
  for (int c = c_begin; c < c_end; ++c) {
    const int it = c - c_begin;
    const float* Gs = lds + (it & 1) * BUF;
    const float* Xs = Gs + C::G_ELEMS;
    const float* Gl = Gs + a_base;
    const bool more = c + 1 < c_end;
    if (more) load_chunk(c + 1);
#pragma unroll
    for (int ks = 0; ks < C::KSTEPS; ++ks) {
      float a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = Gl[ks * C::GP + i * 32];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = Xs[boff[j] + ks];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
#if TLOD_CONV_SGB_W
      __builtin_amdgcn_sched_group_barrier(0x100, TLOD_CONV_SGB_W, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, MI * NJ, 0);
#endif
    }
    if (more) {
      float* Gd = lds + ((it + 1) & 1) * BUF;
      store_chunk(Gd, Gd + C::G_ELEMS);
    }
    __syncthreads();
  }

  // slab[split][co][col]
  float* S = slab + (size_t)split * Cout * Ktot;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + wn * NJ * 32 + j * 32 + l32;
      if (col >= Ktot) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = m0 + wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (co < Cout) S[(size_t)co * Ktot + col] = acc[i][j][r];
      }
    }
}

// ------------------------------------------------------------ split-bf16 wgrad
// The same GEMM on the bf16 MFMA (v_mfma_f32_32x32x16_bf16) with both operands split
// exactly into NPL bf16 planes at staging time (as conv_fwd_bs_kernel), NP products per
// f32 product.  K = pixels, flattened per image (p = h*W + w), so narrow maps waste no
// MFMA lanes on row padding; a chunk is TK = 16 consecutive pixels = one MFMA k-step.
// Both operands are staged K-contiguous ([row][16 px] bf16 per plane): A = dY rows (co),
// B = the im2col rows (ci,kh,kw), element p of B-row (ci,kh,kw) = X[ci][p + (kh-pad)*W +
// (kw-pad)] when that tap lies inside the map (else 0).
//
// Staging is VALU-lean because VALU, not MFMA, bounds a split-operand kernel: each lane
// owns one 4-pixel segment of two A rows and two B rows and fetches each with ONE raw
// buffer_load_dwordx4 (unaligned is fine; the per-dword range check zero-fills the tail of
// the tensor and rows past Cout / columns past Cin*KS*KS, which read at offset 2^31).  The
// in-map mask of a B segment is a few bit-range ops from (h, w) of its first pixel (one
// float-reciprocal division per chunk, shared by all four segments).  A B segment starting
// before the tensor (image 0, channel 0, first row: the dwordx4 would read all zeros) only
// occurs in the first chunks of image 0, which take a per-dword load path (uniform branch).
// Row pitch 48 B puts the 16 rows a ds_read_b128 lane group reads on 16 distinct 16-B
// slots of the 256-B bank row (3r mod 16).  256x256 tiles (8 waves, 4x2 accumulators of
// 32x32 each) give each staged element 256 uses.

template <int WM, int WN, int MI, int NJ, int NP>
struct WgBsCfg {
  static constexpr int NPL = NP == 6 ? 3 : 2;
  static constexpr int NT = WM * WN * 64;
  static constexpr int BM = WM * MI * 32;
  static constexpr int BN = WN * NJ * 32;
  static constexpr int TK = 16;                    // pixels per chunk (one k-step)
  // bytes per row per plane: 32 (dense) with the two 16-B halves swapped on rows with bit 3
  // set — conflict-free for both the staging ds_write_b64 (16-lane groups = 4 rows) and the
  // fragment ds_read_b128; TLOD_WG_SWZ=0: the padded 48-B pitch (2-way write conflicts)
  static constexpr int PITCH = TLOD_WG_SWZ ? 32 : 48;
  static constexpr int A_PLANE = BM * PITCH;
  static constexpr int B_PLANE = BN * PITCH;
  static constexpr int BUF = NPL * (A_PLANE + B_PLANE);
  static constexpr int LDS_BYTES = 2 * BUF;
  static constexpr int ROWS_PER_IT = NT / 4;       // 4 segments of 4 px per row
  static constexpr int A_IT = BM / ROWS_PER_IT, B_IT = BN / ROWS_PER_IT;
  static_assert(BM % ROWS_PER_IT == 0 && BN % ROWS_PER_IT == 0, "staging");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// byte offset of pixel px (a multiple of 4) of a staged row inside the row (see WgBsCfg)
__device__ __forceinline__ int wg_slot(int row, int px) {
  return TLOD_WG_SWZ ? (((px >> 3) ^ ((row >> 3) & 1)) << 4) + ((px & 4) << 1) : 2 * px;
}

// db_slab != nullptr: the bias gradient rides along — the workgroups of column tile 0 also
// sum their staged (masked) dY rows per split, db_slab[split][co] (reduced in split order by
// db_reduce_kernel): the conv's db = sum_p dY[co][p] without a pass of its own over dY.
template <int WM, int WN, int MI, int NJ, int KS, int NP>
__global__ void __launch_bounds__(WM* WN * 64) TLOD_CONV_OCC conv_wgrad_bs_kernel(
    const float* __restrict__ G, const float* __restrict__ X, float* __restrict__ slab, int N,
    int Cin, int H, int W, int Cout, int tiles_m, int tiles_n, int splits, int chunks_per_split,
    float inv_w, float* __restrict__ db_slab) {
  using C = WgBsCfg<WM, WN, MI, NJ, NP>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int KK = KS * KS;

  const int nwg = tiles_m * tiles_n * splits;
  int t = xcd_remap(blockIdx.x, nwg);
  const int mt = t % tiles_m; t /= tiles_m;
  const int nt = t % tiles_n;
  const int split = t / tiles_n;
  const int m0 = mt * C::BM, n0 = nt * C::BN;
  const int Ktot = Cin * KK;
  const int P = H * W;
  const int cpi = (P + C::TK - 1) / C::TK;
  const int total_chunks = N * cpi;
  const int c_begin = split * chunks_per_split;
  const int c_end = min(total_chunks, c_begin + chunks_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, khalf = lane >> 5;

  const i32x4 g_rsrc = make_buffer_rsrc(G, (unsigned)N * Cout * P * 4u);
  const i32x4 x_rsrc = make_buffer_rsrc(X, (unsigned)N * Cin * P * 4u);

  // ---- per-lane staging constants: segment s4..s4+3 of A rows / B rows tid/4 + i*NT/4
  const int s4 = (tid & 3) * 4;
  int a_off[C::A_IT], a_lds[C::A_IT];
#pragma unroll
  for (int i = 0; i < C::A_IT; ++i) {
    const int row = (tid >> 2) + i * C::ROWS_PER_IT;
    a_off[i] = m0 + row < Cout ? (m0 + row) * P + s4 : -1;  // -1: row past Cout
    a_lds[i] = row * C::PITCH + wg_slot(row, s4);
  }
  int b_off[C::B_IT], b_lds[C::B_IT], b_dh[C::B_IT], b_dw[C::B_IT];
#pragma unroll
  for (int i = 0; i < C::B_IT; ++i) {
    const int cl = (tid >> 2) + i * C::ROWS_PER_IT;
    const int col = n0 + cl;
    const bool ok = col < Ktot;
    const int ci = ok ? col / KK : 0, s = ok ? col % KK : 0;
    b_dh[i] = ok ? s / KS - KS / 2 : -(1 << 20);  // dead column: never in the map
    b_dw[i] = s % KS - KS / 2;
    b_off[i] = ok ? ci * P + b_dh[i] * W + b_dw[i] + s4 : s4;
    b_lds[i] = C::NPL * C::A_PLANE + cl * C::PITCH + wg_slot(cl, s4);
  }
  f32x4v ra[C::A_IT], rb[C::B_IT];
  unsigned a_mask = 0, b_mask[C::B_IT];

  auto load_chunk = [&](int c) {
    const int n = c / cpi;
    const int pc = (c - n * cpi) * C::TK;   // first pixel of the chunk
    const int pb = pc + s4;                 // first pixel of this lane's segments
    const int gbase = n * Cout * P + pc, xbase = n * Cin * P + pc;
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i)
      ra[i] = raw_buffer_load_v4f32(g_rsrc, a_off[i] >= 0 ? (gbase + a_off[i]) * 4 : kBufOOB, 0, 0);
    if (n == 0 && pc <= W) {
      // segments that may start before the tensor: per-dword loads, elements before the
      // tensor (outside the map anyway) sent out of range.  The select also keeps the
      // backend from merging the four loads back into one dwordx4 at the negative start.
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int o = xbase + b_off[i] + e;
          rb[i][e] = raw_buffer_load_f32(x_rsrc, o >= 0 ? o * 4 : kBufOOB, 0, 0);
        }
    } else {
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i)
        rb[i] = raw_buffer_load_v4f32(x_rsrc, (xbase + b_off[i]) * 4, 0, 0);
    }
    // masks: pixels past the image (tail chunk), then the taps' in-map test
    const unsigned tmask = lt_mask4(P - pb);
    a_mask = tmask;
    const int h0 = (int)fmaf((float)pb, inv_w, 0.5f * inv_w);  // floor((pb + 0.5) / W)
    const int w0 = pb - h0 * W;
    if (W >= 4) {
      // the 4 pixels are (h0, w0 + e) for e < ew, then (h0 + 1, e - ew): one wrap at most
      const int ew = W - w0;
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i) {
        const int dw = b_dw[i], dwp = max(dw, 0), dwn = max(-dw, 0);
        const bool r0 = (unsigned)(h0 + b_dh[i]) < (unsigned)H;
        const bool r1 = (unsigned)(h0 + 1 + b_dh[i]) < (unsigned)H;
        const unsigned m0v = lt_mask4(ew - dwp) & ~lt_mask4(-w0 - dw);
        const unsigned m1v = 0xfu & ~lt_mask4(ew + dwn);
        b_mask[i] = ((r0 ? m0v : 0u) | (r1 ? m1v : 0u)) & tmask;
      }
    } else {
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i) {
        unsigned m = 0;
        int h = h0, w = w0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = (unsigned)(h + b_dh[i]) < (unsigned)H && (unsigned)(w + b_dw[i]) < (unsigned)W;
          m |= (unsigned)ok << e;
          if (++w == W) { w = 0; ++h; }
        }
        b_mask[i] = m & tmask;
      }
    }
  };
  auto store_seg = [&](unsigned char* dst, int plane_bytes, f32x4v r, unsigned m) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ((m >> e) & 1) ? r[e] : 0.f;
    unsigned sp[3][2];
    split4<C::NPL>(v, sp);
#pragma unroll
    for (int pl = 0; pl < C::NPL; ++pl)
      *reinterpret_cast<uint2*>(dst + pl * plane_bytes) = make_uint2(sp[pl][0], sp[pl][1]);
  };
  const bool row_sums = db_slab != nullptr && nt == 0;
  float rs[C::A_IT];  // this lane's 4-pixel segment sums of its dY rows (row_sums)
#pragma unroll
  for (int i = 0; i < C::A_IT; ++i) rs[i] = 0.f;
  auto store_chunk = [&](unsigned char* buf) {
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      store_seg(buf + a_lds[i], C::A_PLANE, ra[i], a_mask);
      if (row_sums) {
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) t += ((a_mask >> e) & 1) ? ra[i][e] : 0.f;
        rs[i] += t;
      }
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) store_seg(buf + b_lds[i], C::B_PLANE, rb[i], b_mask[i]);
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int a_rd = (wm * MI * 32 + l32) * C::PITCH + wg_slot(l32, 8 * khalf);
  const int b_rd = C::NPL * C::A_PLANE + (wn * NJ * 32 + l32) * C::PITCH + wg_slot(l32, 8 * khalf);
  // chunk c + 1 is split + stored half way through chunk c's MFMAs, and the registers are
  // reloaded with chunk c + 2 right after: every chunk's loads have a whole chunk of MFMAs to
  // land.  sched_barrier keeps the staging there — the compiler otherwise sinks it (and its
  // vmcnt wait) below the MFMAs, where the SIMD's two waves split while the matrix pipe idles
  // (the same fix as gemm.hip's K loop).
  if (c_begin < c_end) {
    load_chunk(c_begin);
    store_chunk(smem);
    if (c_begin + 1 < c_end) load_chunk(c_begin + 1);
  }
  __syncthreads();
  for (int c = c_begin; c < c_end; ++c) {
    const int it = c - c_begin;
    const unsigned char* buf = smem + (it & 1) * C::BUF;
    const bool more = c + 1 < c_end;
    u32x4 b[NJ][3];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        b[j][pl] = *reinterpret_cast<const u32x4*>(buf + b_rd + pl * C::B_PLANE + j * 32 * C::PITCH);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      u32x4 a[3];
#pragma unroll
      for (int pl = 0; pl < C::NPL; ++pl)
        a[pl] = *reinterpret_cast<const u32x4*>(buf + a_rd + pl * C::A_PLANE + i * 32 * C::PITCH);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (more && i * NJ + j == MI * NJ / 2) {
          __builtin_amdgcn_sched_barrier(0);
          store_chunk(smem + ((it + 1) & 1) * C::BUF);
          if (c + 2 < c_end) load_chunk(c + 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        bs_mac<NP>(acc[i][j], a[0], a[1], a[2], b[j][0], b[j][1], b[j][2]);
      }
    }
    __syncthreads();
  }

  if (row_sums) {  // the 4 lanes of a row (tid & 3 = segment), in a fixed order
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      float t = rs[i] + __shfl_xor(rs[i], 1);
      t = t + __shfl_xor(t, 2);
      const int row = (tid >> 2) + i * C::ROWS_PER_IT;
      if ((tid & 3) == 0 && m0 + row < Cout) db_slab[(size_t)split * Cout + m0 + row] = t;
    }
  }
  float* S = slab + (size_t)split * Cout * Ktot;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + wn * NJ * 32 + j * 32 + l32;
      if (col >= Ktot) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = m0 + wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (co < Cout) S[(size_t)co * Ktot + col] = acc[i][j][r];
      }
    }
}

// dW = (accumulate ? dW : 0) + sum_s slab[s], summed in split order (deterministic).
// row_scale (optional, per output channel, row_len = Cin*KS*KS): dW = (accumulate ? dW : 0)
// + row_scale[co] * sum_s slab[s] — a frozen BatchNorm's scale folded into the weight gradient
// of the conv before it (tlod_conv_wgrad_bs_ex_f32).
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int splits, size_t count,
                                   float* __restrict__ out, int accumulate,
                                   const float* __restrict__ row_scale, int row_len) {
  const size_t n4 = count / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    // (the unscaled form keeps the round-3 order: the existing dW first, then the splits)
    float4 s = accumulate && row_scale == nullptr ? reinterpret_cast<const float4*>(out)[i]
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
    // unrolled: eight split loads in flight, the adds still in split order
#pragma unroll 8
    for (int k = 0; k < splits; ++k) {
      const float4 v = reinterpret_cast<const float4*>(slab + (size_t)k * count)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (row_scale != nullptr) {  // per component: a float4 may straddle two rows
      const size_t e = 4 * i, rl = (size_t)row_len;
      s.x *= row_scale[e / rl];
      s.y *= row_scale[(e + 1) / rl];
      s.z *= row_scale[(e + 2) / rl];
      s.w *= row_scale[(e + 3) / rl];
      if (accumulate) {
        const float4 o = reinterpret_cast<const float4*>(out)[i];
        s.x = o.x + s.x; s.y = o.y + s.y; s.z = o.z + s.z; s.w = o.w + s.w;
      }
    }
    reinterpret_cast<float4*>(out)[i] = s;
  }
}

// db = (accumulate ? db : 0) + sum_s db_slab[s], in split order (deterministic).
__global__ void db_reduce_kernel(const float* __restrict__ db_slab, int splits, int C,
                                 float* __restrict__ db, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = accumulate ? db[c] : 0.f;
  for (int k = 0; k < splits; ++k) s += db_slab[(size_t)k * C + c];
  db[c] = s;
}

// y = act(sum_s slab[s] + bias), summed in split order (deterministic).
// Sum the split-K partial tiles of the tail tiles in fixed split order (deterministic),
// apply the epilogue and scatter to Y.  One workgroup per (tail tile, 1024 elements).
// A tile is th_rows x tw_cols pixels (band: tp consecutive flattened pixels), its slab
// rows tp apart.
__global__ void __launch_bounds__(256) fwd_tail_reduce_kernel(
    const float* __restrict__ slab, int ksplit, int n_tail, int dp_tiles, int bm, int tp,
    int th_rows, int tw_cols, int tiles_m, int tiles_w, int tiles_h, Epi epi, int Cout, int H,
    int W, float* __restrict__ Y, int band) {
  // a thread takes 4 consecutive slab elements (one channel: tp is a multiple of 4) with one
  // 16-B load per split piece; the channel's scale / bias once
  const int tile_elems = bm * tp;
  const int per_tile = (tile_elems + 1023) / 1024;
  const int ti = blockIdx.x / per_tile;
  int t = dp_tiles + ti;
  const int mt = t % tiles_m; t /= tiles_m;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h; t /= tiles_h;
  const int n = t;
  const size_t stride = (size_t)n_tail * tile_elems;
  const float* S = slab + (size_t)ti * tile_elems;
  const int e0 = (blockIdx.x % per_tile) * 1024 + 4 * threadIdx.x;
  if (e0 >= tile_elems) return;
  const int ml = e0 / tp, pix0 = e0 % tp;
  const int co = mt * bm + ml;
  if (co >= Cout) return;
  float4 v = *reinterpret_cast<const float4*>(S + e0);
  // unrolled: four split loads in flight, the adds in split order
#pragma unroll 4
  for (int k = 1; k < ksplit; ++k) {
    const float4 u = *reinterpret_cast<const float4*>(S + k * stride + e0);
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  const float sc = epi.scale ? epi.scale[co] : 1.f, bi = epi.bias ? epi.bias[co] : 0.f;
  const float vv[4] = {v.x, v.y, v.z, v.w};
  const size_t cbase = ((size_t)n * Cout + co) * (size_t)(H * W);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int pix = pix0 + e;
    int p;  // flattened pixel
    if (band) {
      p = tw * tp + pix;
      if (p >= H * W) continue;
    } else {
      const int h = th * th_rows + pix / tw_cols, w = tw * tw_cols + pix % tw_cols;
      if (pix >= th_rows * tw_cols || h >= H || w >= W) continue;
      p = h * W + w;
    }
    const size_t idx = cbase + p;
    float x = vv[e];
    if (epi.scale) x *= sc;
    x += bi;
    if (epi.residual) x += epi.residual[idx];
    if (epi.relu) x = fmaxf(x, 0.f);
    if (epi.s2d > 1) {
      const long long o = epi_out_index(epi, n, co, p / W, p % W, Cout, H, W);
      if (o >= 0) Y[o] = x;
    } else {
      Y[idx] = epi_mask(epi, idx, x);
    }
  }
}

// ======================================================================= helpers
// Wk[(ci*KK + s)][co] = W[co][ci][s]   (forward operand, K-major)
__global__ void pack_fwd_kernel(const float* __restrict__ Wt, float* __restrict__ Wk, int Cout,
                                int Ktot) {
  const size_t total = (size_t)Cout * Ktot;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % Cout);
    const size_t k = i / Cout;
    Wk[i] = Wt[(size_t)co * Ktot + k];
  }
}

// Wd[(co*KK + s')][ci] = W[co][ci][KK-1-s']   (dgrad operand: transposed + flipped)
__global__ void pack_dgrad_kernel(const float* __restrict__ Wt, float* __restrict__ Wd, int Cout,
                                  int Cin, int KK) {
  const size_t total = (size_t)Cout * Cin * KK;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Cin);
    const size_t r = i / Cin;
    const int s = (int)(r % KK);
    const int co = (int)(r / KK);
    Wd[i] = Wt[((size_t)co * Cin + ci) * KK + (KK - 1 - s)];
  }
}

// G0 = dY * (Y > 0) (when Y given); db[co] (+)= sum over n,p of G0; G = G0 * scale[co]
// (scale: a folded frozen BatchNorm, optional); G0 also stored to Graw when given (the
// residual branch of a bottleneck takes the unscaled gradient).  grid (Cout, N).
// One workgroup per channel, looping over the N images: db[co] is written (not accumulated),
// so the caller needs no zero fill, and the sum order is fixed (deterministic).
// One workgroup of 1024 threads per channel (the per-channel bias sum stays in one block:
// deterministic, no second pass); each thread keeps 4 float4 loads of dY and Y in flight,
// so the kernel streams near the HBM rate even with one workgroup per CU.
constexpr int kReluThreads = 1024;
__global__ void __launch_bounds__(kReluThreads) relu_bwd_bias_kernel(
    const float* __restrict__ dY, const float* __restrict__ Y, const float* __restrict__ scale,
    float* __restrict__ G, float* __restrict__ Graw, float* __restrict__ db, int N, int Cout,
    int HW) {
  const int co = blockIdx.x;
  const float sc = scale ? scale[co] : 1.f;
  const bool write_g = G != dY || Y != nullptr || scale != nullptr;
  float s = 0.f;
  auto apply = [&](float4 d, float4 y, bool has_y) {
    if (has_y) {
      d.x = y.x > 0.f ? d.x : 0.f; d.y = y.y > 0.f ? d.y : 0.f;
      d.z = y.z > 0.f ? d.z : 0.f; d.w = y.w > 0.f ? d.w : 0.f;
    }
    return d;
  };
  const bool vec = (HW % 4) == 0;
  for (int n = 0; n < N; ++n) {
    const size_t base = ((size_t)n * Cout + co) * HW;
    if (vec) {
      const float4* d4 = reinterpret_cast<const float4*>(dY + base);
      const float4* y4 = Y ? reinterpret_cast<const float4*>(Y + base) : nullptr;
      float4* g4 = reinterpret_cast<float4*>(G + base);
      float4* r4 = Graw ? reinterpret_cast<float4*>(Graw + base) : nullptr;
      const int n4 = HW / 4;
      constexpr int U = 4;
      int i = threadIdx.x;
      for (; i + (U - 1) * kReluThreads < n4; i += U * kReluThreads) {
        float4 d[U], y[U] = {};
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = d4[i + u * kReluThreads];
        if (y4) {
#pragma unroll
          for (int u = 0; u < U; ++u) y[u] = y4[i + u * kReluThreads];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float4 v = apply(d[u], y[u], y4 != nullptr);
          if (r4) r4[i + u * kReluThreads] = v;
          s += (v.x + v.y) + (v.z + v.w);
          if (write_g)
            g4[i + u * kReluThreads] = scale ? make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc) : v;
        }
      }
      for (; i < n4; i += kReluThreads) {
        const float4 v = apply(d4[i], y4 ? y4[i] : make_float4(0.f, 0.f, 0.f, 0.f), y4 != nullptr);
        if (r4) r4[i] = v;
        s += (v.x + v.y) + (v.z + v.w);
        if (write_g) g4[i] = scale ? make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc) : v;
      }
    } else {
      for (int i = threadIdx.x; i < HW; i += kReluThreads) {
        float d = dY[base + i];
        if (Y) d = Y[base + i] > 0.f ? d : 0.f;
        if (Graw) Graw[base + i] = d;
        s += d;
        G[base + i] = scale ? d * sc : d;
      }
    }
  }
  if (!db) return;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  __shared__ float ws[kReluThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < kReluThreads / 64; ++w) t += ws[w];
    db[co] = t;
  }
}

// ======================================================================= launchers

struct FwdPlan {
  int tiles_m, tiles_w, tiles_h;
  int dp_tiles;  // tiles computed whole (full K)
  int ksplit;    // split count of the remaining tail tiles (1: no tail)
  int cps;       // input-channel chunks per split piece
  int n_tail() const { return tiles_m * tiles_w * tiles_h * n - dp_tiles; }
  int n;
  int th = 0, tw = 0;  // warp-specialized kernel: tile rows x columns (ws_tile)
  size_t slab_bytes(int bm, int th) const {
    return ksplit > 1 ? (size_t)ksplit * n_tail() * bm * th * 32 * sizeof(float) : 0;
  }
};

// Resident workgroup slots of a kernel on this device (occupancy x CUs), cached per
// (kernel, device) in runtime.hip.  Without a device (CPU build checks) assume 256.
template <typename K>
static int resident_slots(K kern, int threads, size_t lds) {
  return cached_slots((const void*)kern, threads, lds);
}

// Wave quantization: a grid of T whole tiles on S resident slots runs ceil(T/S) rounds,
// so e.g. conv3_3 (1216 tiles on 512 slots) idles 21% of the chip in its last round.
// The last partial round (or, for small maps, every tile) is instead split over input
// channels into ksplit pieces that fill the slots, at the cost of a slab round trip
// through HBM.  Cost model in seconds: tiles at ~65% of the f32 MFMA peak per slot,
// slab traffic (k writes + k reads + 1 write per tail tile) at 4 TB/s, 6 us per reduce.
static FwdPlan plan_schedule(int tiles_m, int tiles_w, int tiles_h, int N, int nchunks,
                             double tile_flops, int tile_elems, int slots, bool allow_split = true,
                             int cps_align = 1) {
  FwdPlan p{tiles_m, tiles_w, tiles_h, 0, 1, nchunks, N};
  const long long T = (long long)tiles_m * tiles_w * tiles_h * N;
  p.dp_tiles = (int)T;
  if (!allow_split) return p;
  const double tile_s = tile_flops / (157.3e12 * 0.65 / slots);
  double best = (double)((T + slots - 1) / slots) * tile_s;
  const int kmax = std::min({8, TLOD_CONV_KSPLIT_MAX, nchunks / 2});
  const long long q = T / slots;
  for (int k = 2; k <= kmax; ++k) {
    const int cps = div_up(div_up(nchunks, k), cps_align) * cps_align;
    const int kk = div_up(nchunks, cps);
    if (kk < 2) continue;
    for (long long dp : {q * slots, 0ll}) {
      const long long tail = T - dp;
      if (tail <= 0) continue;
      const double piece_s = tile_s * cps / nchunks;
      const double t = (double)dp / slots * tile_s +
                       (double)((tail * kk + slots - 1) / slots) * piece_s +
                       (2.0 * kk + 1.0) * tail * tile_elems * 4.0 / 4e12 + 6e-6;
      if (t < best * 0.97) {
        best = t;
        p.dp_tiles = (int)dp;
        p.ksplit = kk;
        p.cps = cps;
      }
    }
  }
  return p;
}

template <int WM, int WN, int MI, int NJ, int CK, int KS>
static FwdPlan plan_fwd(int N, int Cin, int H, int W, int Cout) {
  using C = FwdCfg<WM, WN, MI, NJ, CK, KS>;
  const int slots = resident_slots(conv_fwd_kernel<WM, WN, MI, NJ, CK, KS, true>, C::NT,
                                          C::LDS_FLOATS * sizeof(float));
  const int nchunks = div_up(Cin, CK);
  return plan_schedule(div_up(Cout, C::BM), div_up(W, C::TW), div_up(H, C::TH), N, nchunks,
                       2.0 * C::BM * C::TH * C::TW * (double)nchunks * C::KC,
                       C::BM * C::TH * C::TW, slots);
}

template <int WM, int WN, int MI, int NJ, int CK, int KS, bool VEC4>
static int launch_fwd(const float* X, const float* Wk, Epi epi, float* Y, int N, int Cin, int H,
                      int W, int Cout, float* slab, size_t slab_bytes, hipStream_t s) {
  using C = FwdCfg<WM, WN, MI, NJ, CK, KS>;
  const FwdPlan p = plan_fwd<WM, WN, MI, NJ, CK, KS>(N, Cin, H, W, Cout);
  const long long nwg = (long long)p.dp_tiles + (long long)p.n_tail() * (p.ksplit > 1 ? p.ksplit : 0);
  TLOD_CHECK_ARG(nwg < (1ll << 31), "grid too large");
  if (p.ksplit > 1 && slab_bytes < p.slab_bytes(C::BM, C::TH)) {
    set_error("tlod_conv: workspace too small for split-K");
    return kWorkspace;
  }
  const size_t lds = C::LDS_FLOATS * sizeof(float);
  auto kern = conv_fwd_kernel<WM, WN, MI, NJ, CK, KS, VEC4>;
  TLOD_HIP(lds_attr((const void*)kern, (int)lds));
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), lds, s, X, Wk, epi, Y, N, Cin, H, W,
                     Cout, p.tiles_m, p.tiles_w, p.tiles_h, p.dp_tiles, p.ksplit, p.cps, slab);
  TLOD_LAUNCH_CHECK();
  if (p.ksplit > 1) {
    const int per_tile = div_up(C::BM * C::TH * C::TW, 1024);
    hipLaunchKernelGGL(fwd_tail_reduce_kernel, dim3(p.n_tail() * per_tile), dim3(256), 0, s, slab,
                       p.ksplit, p.n_tail(), p.dp_tiles, C::BM, C::TH * C::TW, C::TH, C::TW,
                       p.tiles_m, p.tiles_w, p.tiles_h, epi, Cout, H, W, Y, 0);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}

template <int WM, int WN, int MI, int NJ, int CK, int KS>
static int launch_fwd_v(const float* X, const float* Wk, Epi epi, float* Y, int N, int Cin,
                        int H, int W, int Cout, float* slab, size_t sb, hipStream_t s) {
  if ((Cout & 3) == 0)
    return launch_fwd<WM, WN, MI, NJ, CK, KS, true>(X, Wk, epi, Y, N, Cin, H, W, Cout, slab, sb, s);
  return launch_fwd<WM, WN, MI, NJ, CK, KS, false>(X, Wk, epi, Y, N, Cin, H, W, Cout, slab, sb, s);
}

// Dispatch on (KS, Cout): the tile configs used by the backbone.  ws_query != nullptr:
// only report the split-K slab bytes the call would need.
static int conv_fwd_dispatch(const float* X, const float* Wk, Epi epi, float* Y, int N,
                             int Cin, int H, int W, int Cout, int KS, float* slab, size_t sb,
                             hipStream_t s, size_t* ws_query = nullptr) {
#define TLOD_FWD_CFG(WM_, WN_, MI_, NJ_, CK_, KS_)                                              \
  do {                                                                                          \
    if (ws_query) {                                                                             \
      using C_ = FwdCfg<WM_, WN_, MI_, NJ_, CK_, KS_>;                                          \
      *ws_query = plan_fwd<WM_, WN_, MI_, NJ_, CK_, KS_>(N, Cin, H, W, Cout)                    \
                      .slab_bytes(C_::BM, C_::TH);                                              \
      return kOk;                                                                               \
    }                                                                                           \
    return launch_fwd_v<WM_, WN_, MI_, NJ_, CK_, KS_>(X, Wk, epi, Y, N, Cin, H, W, Cout, slab,  \
                                                       sb, s);                                  \
  } while (0)
  if (KS == 3) {
    if (Cout <= 64) TLOD_FWD_CFG(1, 8, 2, 2, 8, 3);
    TLOD_FWD_CFG(2, 4, 2, 2, 8, 3);
  }
  if (KS == 1) {
    if (Cout <= 64) TLOD_FWD_CFG(1, 8, 2, 2, 32, 1);
    TLOD_FWD_CFG(2, 4, 2, 2, 32, 1);
  }
#undef TLOD_FWD_CFG
  set_error("conv: only 1x1 and 3x3 kernels (stride 1) are implemented");
  return kUnsupported;
}

// ---- split-bf16 forward launch (KS = 3)
// Band tiles pay off where 32-wide column tiles pad the map badly (conv5 / RPN at 37x75:
// 40% padding; 75x150: 6%), and fit the staged patch only for narrow maps.
static bool use_band(int H, int W) {
  if (!band_fits(W) || TLOD_CONV_BAND == 0) return false;
  const double util2d = (double)H * W / ((double)div_up(H, 16) * 16 * div_up(W, 32) * 32);
  const double utilb = (double)H * W / ((double)div_up(H * W, 512) * 512);
  return utilb > util2d * 1.05;
}

// Warp-specialized forward kernel (conv_fwd_bs_ws_kernel) instead of conv_fwd_bs_kernel.
// Warp-specialized forward for 2D tiles with >= 16 input-channel chunks (Cin >= 128):
// measured 5-8% faster on conv3/conv4 fwd and dgrad, ~2% slower at Cin = 64 (4 chunk pairs
// per tile: the per-tile prologue dominates).
// One predicate for the plan (resident slots) and the launch.
static bool use_ws(int Cin, int Cout, int H, int W) {
  // raw buffer loads / stores: 32-bit byte offsets into one image (+ 8 channels of headroom)
  return TLOD_CONV_WS != 0 && Cin >= TLOD_WS_MINCIN && (size_t)(std::max(Cin, Cout) + 8) * H * W * 4 < (1ull << 31);
}

// Tile of the warp-specialized kernel for an H x W map: the fewest tiles of TH x TW <= 512
// pixels whose patch fits the staging (real (TH + 2) x (TW + 2) <= kWsPos positions, staged
// (TH + 2) x ws_pitch(TW) <= kWsAlloc); ties go to the smaller halo (patch / pixels, to
// 0.05), then the wider tile (coalesced staging rows).  Pooling epilogues keep 16 x 32.
struct WsTile {
  int th, tw;
};
static WsTile ws_tile(int H, int W, bool pool) {
  if (pool || TLOD_WS_FLEX == 0) return {16, 32};
  WsTile best{16, 32};
  long long best_t = (long long)div_up(H, 16) * div_up(W, 32);
  int best_h = 24;  // halo of 16 x 32 (612 / 512 = 1.195) in units of 0.05
  for (int th = 1; th <= std::min(H, 64); ++th)
    for (int tw = 8; tw <= std::min(512 / th, W); ++tw) {
      if ((th + 2) * (tw + 2) > kWsPos || (th + 2) * ws_pitch(tw) > kWsAlloc) continue;
      const long long t = (long long)div_up(H, th) * div_up(W, tw);
      const int halo = (int)std::lround(20.0 * (th + 2) * (tw + 2) / (th * tw));
      if (t < best_t || (t == best_t && (halo < best_h || (halo == best_h && tw > best.tw)))) {
        best = {th, tw};
        best_t = t;
        best_h = halo;
      }
    }
  return best;
}

template <int WM, int WN, int MI, int NJ, int NP>
static int ws_slots() {
  const int slots = resident_slots(conv_fwd_bs_ws_kernel<WM, WN, MI, NJ, NP>,
                                          WM * WN * 64 + kProdWaves * 64,
                                          WsCfg<WM, WN, MI, NJ, NP>::LDS_BYTES);
  return slots;
}

template <int WM, int WN, int MI, int NJ, int NP, bool BAND>
static FwdPlan plan_fwd_bs(int N, int Cin, int H, int W, int Cout, bool allow_split = true) {
  using C = BsCfg<WM, WN, MI, NJ, NP, BAND>;
  const int slots_plain = resident_slots(conv_fwd_bs_kernel<WM, WN, MI, NJ, NP, BAND>,
                                                C::NT, C::LDS_BYTES);
  int slots = slots_plain;
  WsTile wt{C::TH, C::TW};
  bool ws = false;
  if constexpr (!BAND)
    if (use_ws(Cin, Cout, H, W)) {
      ws = true;
      slots = ws_slots<WM, WN, MI, NJ, NP>();
      wt = ws_tile(H, W, !allow_split);  // allow_split == false: the pooling epilogue
    }
  const int nchunks = div_up(Cin, C::CK);
  // cost model in f32-MFMA-equivalent time: the split products run ~16/NP x faster
  const int tw = BAND ? div_up(H * W, C::TH * C::TW) : div_up(W, wt.tw);
  const int th = BAND ? 1 : div_up(H, wt.th);
  // (warp-specialized pieces in whole four-chunk frames where the K allows)
  FwdPlan p = plan_schedule(div_up(Cout, C::BM), tw, th, N, nchunks,
                            2.0 * C::BM * C::TH * C::TW * (double)nchunks * 72 * NP / 16.0,
                            C::BM * C::TH * C::TW, slots, allow_split,
                            ws && nchunks >= 16 ? 4 : 1);
  if (ws) {
    p.th = wt.th;
    p.tw = wt.tw;
  }
  return p;
}

template <int WM, int WN, int MI, int NJ, int NP, bool BAND>
static int launch_fwd_bs(const float* X, const unsigned short* Wp, Epi epi, float* Y, int N,
                         int Cin, int H, int W, int Cout, float* slab, size_t slab_bytes,
                         hipStream_t s) {
  using C = BsCfg<WM, WN, MI, NJ, NP, BAND>;
  const FwdPlan p = plan_fwd_bs<WM, WN, MI, NJ, NP, BAND>(N, Cin, H, W, Cout, epi.pool == nullptr);
  const long long nwg = (long long)p.dp_tiles + (long long)p.n_tail() * (p.ksplit > 1 ? p.ksplit : 0);
  TLOD_CHECK_ARG(nwg < (1ll << 31), "grid too large");
  if (p.ksplit > 1 && slab_bytes < p.slab_bytes(C::BM, C::TH)) {
    set_error("tlod_conv_bs: workspace too small for split-K");
    return kWorkspace;
  }
  bool launched = false;
  if constexpr (!BAND) {
    // warp-specialized kernel: one work item per workgroup
    if (use_ws(Cin, Cout, H, W)) {
      using WC = WsCfg<WM, WN, MI, NJ, NP>;
      auto kern = conv_fwd_bs_ws_kernel<WM, WN, MI, NJ, NP>;
      TLOD_HIP(lds_attr((const void*)kern, (int)WC::LDS_BYTES));
      hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT + kProdWaves * 64), WC::LDS_BYTES,
                         s, X, Wp, epi, Y, N, Cin, H, W, Cout, p.tiles_m, p.tiles_w, p.tiles_h,
                         p.dp_tiles, p.ksplit, p.cps, slab, p.th, p.tw);
      launched = true;
    }
  }
  if (!launched) {
    const size_t lds = C::LDS_BYTES;
    auto kern = conv_fwd_bs_kernel<WM, WN, MI, NJ, NP, BAND>;
    TLOD_HIP(lds_attr((const void*)kern, (int)lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), lds, s, X, Wp, epi, Y, N, Cin, H, W,
                       Cout, p.tiles_m, p.tiles_w, p.tiles_h, p.dp_tiles, p.ksplit, p.cps, slab);
  }
  TLOD_LAUNCH_CHECK();
  if (p.ksplit > 1) {
    const int per_tile = div_up(C::BM * C::TH * C::TW, 1024);
    const int th = p.th ? p.th : C::TH, tw = p.th ? p.tw : C::TW;
    hipLaunchKernelGGL(fwd_tail_reduce_kernel, dim3(p.n_tail() * per_tile), dim3(256), 0, s, slab,
                       p.ksplit, p.n_tail(), p.dp_tiles, C::BM, C::TH * C::TW, th, tw, p.tiles_m,
                       p.tiles_w, p.tiles_h, epi, Cout, H, W, Y, BAND ? 1 : 0);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}

static int conv_fwd_bs_dispatch(const float* X, const unsigned short* Wp, Epi epi, float* Y,
                                int N, int Cin, int H, int W, int Cout, int KS, int nprod,
                                float* slab, size_t sb, hipStream_t s, size_t* ws_query = nullptr) {
  if (KS != 3) {
    set_error("conv_bs: only 3x3 kernels");
    return kUnsupported;
  }
  if (nprod != 3 && nprod != 6) {
    set_error("conv_bs: nprod must be 3 or 6");
    return kInvalidArg;
  }
#define TLOD_BS_CFG(WM_, WN_, MI_, NJ_, NP_, BAND_)                                             \
  do {                                                                                          \
    if (ws_query) {                                                                             \
      using C_ = BsCfg<WM_, WN_, MI_, NJ_, NP_, BAND_>;                                         \
      *ws_query = plan_fwd_bs<WM_, WN_, MI_, NJ_, NP_, BAND_>(N, Cin, H, W, Cout)               \
                      .slab_bytes(C_::BM, C_::TH);                                              \
      return kOk;                                                                               \
    }                                                                                           \
    return launch_fwd_bs<WM_, WN_, MI_, NJ_, NP_, BAND_>(X, Wp, epi, Y, N, Cin, H, W, Cout,     \
                                                         slab, sb, s);                          \
  } while (0)
  // pooling: 2D tiles; the warp-specialized kernel's flexible tiles replace band tiles
  const bool band = use_band(H, W) && epi.pool == nullptr &&
                    !(use_ws(Cin, Cout, H, W) && TLOD_WS_FLEX != 0);
  if (nprod == 6 && band) TLOD_BS_CFG(1, 8, 2, 2, 6, true);
  if (nprod == 6) TLOD_BS_CFG(1, 8, 2, 2, 6, false);
  if (band) TLOD_BS_CFG(1, 8, 2, 2, 3, true);
  TLOD_BS_CFG(1, 8, 2, 2, 3, false);
#undef TLOD_BS_CFG
}

// Split count over pixel chunks: the weight-gradient tiles alone (Cout/128 x 9Cin/256 =
// 18 for conv3_3) cannot fill the chip, so the reduction over pixels is split into slabs.
// Pick the count whose grid best fills whole rounds of resident workgroups (a grid of
// 1.04 rounds runs as long as 2), keeping >= 8 pixel chunks per workgroup.
static int pick_splits(int tiles, int chunks, int slots) {
  const int smax = std::max(1, std::min(64, chunks / 8));
  int best = 1;
  double best_eff = -1.0;
  for (int sp = 1; sp <= smax; ++sp) {
    const long long nwg = (long long)tiles * sp;
    const long long rounds = (nwg + slots - 1) / slots;
    const double eff = (double)nwg / (double)(rounds * slots);
    if (eff > best_eff + 1e-9) { best_eff = eff; best = sp; }
  }
  return best;
}

template <int WM, int WN, int MI, int NJ, int KS, int TH>
struct Wgrad {
  using C = WgCfg<WM, WN, MI, NJ, KS, TH>;
  static constexpr size_t kLds = C::LDS_FLOATS * sizeof(float);
  static int splits(int N, int Cin, int H, int W, int Cout) {
    const int tiles = div_up(Cout, C::BM) * div_up(Cin * C::KK, C::BN);
    const int chunks = N * div_up(H, C::TH) * div_up(W, C::TW);
    const int slots =
        resident_slots(conv_wgrad_kernel<WM, WN, MI, NJ, KS, TH>, C::NT, kLds);
    return pick_splits(tiles, chunks, slots);
  }
  static int launch(const float* G, const float* X, float* slab, int splits, int N, int Cin,
                    int H, int W, int Cout, hipStream_t s) {
    const int Ktot = Cin * C::KK;
    const int tiles_m = div_up(Cout, C::BM), tiles_n = div_up(Ktot, C::BN);
    const int total_chunks = N * div_up(H, C::TH) * div_up(W, C::TW);
    const int cps = div_up(total_chunks, splits);
    const int nwg = tiles_m * tiles_n * splits;
    auto kern = conv_wgrad_kernel<WM, WN, MI, NJ, KS, TH>;
    TLOD_HIP(lds_attr((const void*)kern, (int)kLds));
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(C::NT), kLds, s, G, X, slab, N, Cin, H, W, Cout,
                       tiles_m, tiles_n, splits, cps);
    TLOD_LAUNCH_CHECK();
    return kOk;
  }
};

// The wgrad tile config per kernel size.
template <typename F>
static int with_wgrad_cfg(int KS, F&& f) {
  if (KS == 3) return f(Wgrad<2, 4, 2, 2, 3, 1>{});
  if (KS == 1) return f(Wgrad<2, 2, 2, 2, 1, 2>{});
  return -1;
}

static int wgrad_splits(int N, int Cin, int H, int W, int Cout, int KS) {
  return with_wgrad_cfg(KS, [&](auto cfg) { return cfg.splits(N, Cin, H, W, Cout); });
}

// Split count by cost: rounds x chunks per split x chunk time + the slab round trip
// (sp writes + sp reads + 1 write of Cout*Ktot floats).  Small maps (conv5 / RPN at
// 37x75) cannot afford the 16-64 splits that fill the chip on conv3.
static int pick_splits_cost(long long tiles, int chunks, int slots, double chunk_s,
                            double dw_bytes, double* t_out = nullptr) {
  int best = 1;
  double best_t = 1e30;
  const int smax = std::max(1, std::min(128, chunks / 4));
  for (int sp = 1; sp <= smax; ++sp) {
    const int cps = div_up(chunks, sp);
    const int esp = div_up(chunks, cps);
    const long long rounds = (tiles * esp + slots - 1) / slots;
    const double t = (double)rounds * cps * chunk_s + (2.0 * esp + 1.0) * dw_bytes / 4e12;
    if (t < best_t * 0.999) {
      best_t = t;
      best = esp;
    }
  }
  if (t_out) *t_out = best_t;
  return best;
}

template <int WM, int WN, int MI, int NJ, int KS, int NP>
struct WgradBs {
  using C = WgBsCfg<WM, WN, MI, NJ, NP>;
  static int splits(int N, int Cin, int H, int W, int Cout, double* t_out = nullptr) {
    const int slots =
        resident_slots(conv_wgrad_bs_kernel<WM, WN, MI, NJ, KS, NP>, C::NT, C::LDS_BYTES);
    const long long tiles = (long long)div_up(Cout, C::BM) * div_up(Cin * KS * KS, C::BN);
    const int chunks = N * div_up(H * W, C::TK);
    // bf16 MFMA time of one chunk per resident slot at ~50% of the dense peak (a 128 x 128
    // tile reads twice the LDS bytes per MFMA of a 256 x 256 one: ~40%)
    const double eff = C::BM * C::BN >= 256 * 256 ? 0.5 : 0.4;
    const double chunk_s = 2.0 * C::BM * C::BN * C::TK * NP / (2516.6e12 * eff / slots);
    return pick_splits_cost(tiles, chunks, slots, chunk_s, 4.0 * Cout * Cin * KS * KS, t_out);
  }
  static int launch(const float* G, const float* X, float* slab, float* db_slab, int splits,
                    int N, int Cin, int H, int W, int Cout, hipStream_t s) {
    const int tiles_m = div_up(Cout, C::BM), tiles_n = div_up(Cin * KS * KS, C::BN);
    const int total_chunks = N * div_up(H * W, C::TK);
    const int cps = div_up(total_chunks, splits);
    const long long nwg = (long long)tiles_m * tiles_n * splits;
    TLOD_CHECK_ARG(nwg < (1ll << 31), "grid too large");
    auto kern = conv_wgrad_bs_kernel<WM, WN, MI, NJ, KS, NP>;
    TLOD_HIP(lds_attr((const void*)kern, C::LDS_BYTES));
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), C::LDS_BYTES, s, G, X, slab, N, Cin,
                       H, W, Cout, tiles_m, tiles_n, splits, cps, 1.0f / (float)W, db_slab);
    TLOD_LAUNCH_CHECK();
    return kOk;
  }
};

// 1x1 weight gradients have small outputs (Cout x Cin) over long K (all pixels), so the
// 256 x 256 tiles leave a handful of tiles that must be split many ways over the pixels, each
// split writing a full dW slab: 256 -> 1024 at 38x75 ran 4 tiles x 64 splits (64 MB of
// slabs).  128 x 128 tiles give 4x the tiles for 1/4 of the slab traffic at a lower MFMA
// efficiency; the cost model picks.
static bool wgrad1x1_small_tile(int N, int Cin, int H, int W, int Cout, int nprod) {
  if (TLOD_WG1X1_TILE == 256) return false;
  if (TLOD_WG1X1_TILE == 128) return true;
  double t_big = 0, t_small = 0;
  if (nprod == 6) {
    WgradBs<2, 4, 4, 2, 1, 6>::splits(N, Cin, H, W, Cout, &t_big);
    WgradBs<2, 4, 2, 1, 1, 6>::splits(N, Cin, H, W, Cout, &t_small);
  } else {
    WgradBs<2, 4, 4, 2, 1, 3>::splits(N, Cin, H, W, Cout, &t_big);
    WgradBs<2, 4, 2, 1, 1, 3>::splits(N, Cin, H, W, Cout, &t_small);
  }
  return t_small < t_big;
}

template <typename F>
static int with_wgrad_bs_cfg(int N, int Cin, int H, int W, int Cout, int KS, int nprod, F&& f) {
  if (KS == 3 && nprod == 6) return f(WgradBs<2, 4, 4, 2, 3, 6>{});
  if (KS == 3 && nprod == 3) return f(WgradBs<2, 4, 4, 2, 3, 3>{});
  if (KS == 1) {
    const bool small = wgrad1x1_small_tile(N, Cin, H, W, Cout, nprod);
    if (nprod == 6) return small ? f(WgradBs<2, 4, 2, 1, 1, 6>{}) : f(WgradBs<2, 4, 4, 2, 1, 6>{});
    if (nprod == 3) return small ? f(WgradBs<2, 4, 2, 1, 1, 3>{}) : f(WgradBs<2, 4, 4, 2, 1, 3>{});
  }
  return -1;
}

}  // namespace tlod

using namespace tlod;


extern "C" int tlod_conv_pack_fwd_f32(const float* weight, int Cout, int Cin, int KS, float* wk,
                                      tlod_stream_t stream) {
  TLOD_CHECK_ARG(Cout > 0 && Cin > 0 && KS > 0, "bad shape");
  const size_t total = (size_t)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(pack_fwd_kernel, dim3((unsigned)std::min<size_t>(div_up((int)std::min<size_t>(total, 1u << 30), 256), 4096)),
                     dim3(256), 0, (hipStream_t)stream, weight, wk, Cout, Cin * KS * KS);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_conv_pack_dgrad_f32(const float* weight, int Cout, int Cin, int KS, float* wd,
                                        tlod_stream_t stream) {
  TLOD_CHECK_ARG(Cout > 0 && Cin > 0 && KS > 0, "bad shape");
  const size_t total = (size_t)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(pack_dgrad_kernel, dim3((unsigned)std::min<size_t>(div_up((int)std::min<size_t>(total, 1u << 30), 256), 4096)),
                     dim3(256), 0, (hipStream_t)stream, weight, wd, Cout, Cin, KS * KS);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" size_t tlod_conv_fwd_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS) {
  size_t b = 0;
  conv_fwd_dispatch(nullptr, nullptr, Epi{}, nullptr, N, Cin, H, W, Cout, KS, nullptr, 0, nullptr,
                    &b);
  return b;
}

extern "C" size_t tlod_conv_dgrad_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS) {
  return tlod_conv_fwd_workspace_bytes(N, Cout, H, W, Cin, KS);
}

extern "C" int tlod_conv_fwd_f32(const float* x, const float* wk, const float* bias, float* y,
                                 int N, int Cin, int H, int W, int Cout, int KS, int relu,
                                 void* ws, size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  return conv_fwd_dispatch(x, wk, Epi{nullptr, bias, nullptr, relu}, y, N, Cin, H, W, Cout, KS,
                           (float*)ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int tlod_conv_fwd_ex_f32(const float* x, const float* wk, const float* scale,
                                    const float* bias, const float* residual, float* y, int N,
                                    int Cin, int H, int W, int Cout, int KS, int relu, void* ws,
                                    size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  TLOD_CHECK_ARG(residual != y || residual == nullptr, "residual must not alias y");
  return conv_fwd_dispatch(x, wk, Epi{scale, bias, residual, relu}, y, N, Cin, H, W, Cout, KS,
                           (float*)ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int tlod_drm_fwd_f32(const float* x, const float* wk, float* y, int N, int Cin,
                                int H, int W, int Cout, int scale, void* ws, size_t ws_bytes,
                                tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && Cout > 0 && scale > 1 && H >= scale && W >= scale,
                 "bad shape (need scale > 1, H, W >= scale)");
  Epi e{nullptr, nullptr, nullptr, 1};
  e.s2d = scale;
  return conv_fwd_dispatch(x, wk, e, y, N, Cin, H, W, Cout, 1, (float*)ws, ws_bytes,
                           (hipStream_t)stream);
}

extern "C" int tlod_conv_dgrad_f32(const float* dy, const float* wd, float* dx, int N, int Cin,
                                   int H, int W, int Cout, int KS, void* ws, size_t ws_bytes,
                                   tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  // dx[n, ci] = sum_{co, s'} Wd[(co, s')][ci] * dy[n, co, p + s' - pad]: forward form
  return conv_fwd_dispatch(dy, wd, Epi{}, dx, N, Cout, H, W, Cin, KS, (float*)ws, ws_bytes,
                           (hipStream_t)stream);
}

extern "C" size_t tlod_conv_wgrad_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS) {
  const int sp = wgrad_splits(N, Cin, H, W, Cout, KS);
  return sp > 0 ? (size_t)sp * Cout * Cin * KS * KS * sizeof(float) : 0;
}

extern "C" int tlod_conv_wgrad_f32(const float* dy, const float* x, float* dw, int accumulate,
                                   int N, int Cin, int H, int W, int Cout, int KS, void* ws,
                                   size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  TLOD_CHECK_ARG((Cout * Cin * KS * KS) % 4 == 0, "Cout*Cin*KS*KS must be a multiple of 4");
  hipStream_t s = (hipStream_t)stream;
  TLOD_CHECK_ARG(KS == 1 || KS == 3, "conv wgrad: only 1x1 and 3x3 kernels");
  const int splits = wgrad_splits(N, Cin, H, W, Cout, KS);
  if (ws_bytes < (size_t)splits * Cout * Cin * KS * KS * sizeof(float)) {
    set_error("tlod_conv_wgrad_f32: workspace too small");
    return kWorkspace;
  }
  float* slab = static_cast<float*>(ws);
  const int st = with_wgrad_cfg(KS, [&](auto cfg) {
    return cfg.launch(dy, x, slab, splits, N, Cin, H, W, Cout, s);
  });
  if (st) return st;
  const size_t count = (size_t)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)std::min<size_t>((count / 4 + 255) / 256, 2048)),
                     dim3(256), 0, s, slab, splits, count, dw, accumulate, nullptr, 1);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

// workspace: the split slabs of dW, then (16-B aligned) the split slabs of db
static size_t wgrad_bs_ws(int sp, int Cin, int Cout, int KS) {
  return align_up((size_t)sp * Cout * Cin * KS * KS * sizeof(float), 16) +
         (size_t)sp * Cout * sizeof(float);
}

namespace tlod {
// csrc/wgrad_ws.hip: the warp-specialized 3x3 weight gradient (2D pixel-tile chunks)
bool wgrad_ws_applies(int N, int Cin, int H, int W, int Cout, int KS, int nprod);
size_t wgrad_ws_workspace(int N, int Cin, int H, int W, int Cout);
int wgrad_ws_launch(const float* dy, const float* x, float* dw, float* db, int accumulate,
                    const float* row_scale, int N, int Cin, int H, int W, int Cout, void* ws,
                    size_t ws_bytes, hipStream_t s);
int launch_db_reduce(const float* db_slab, int splits, int C, float* db, int accumulate,
                     hipStream_t s) {
  hipLaunchKernelGGL(db_reduce_kernel, dim3(div_up(C, 256)), dim3(256), 0, s, db_slab, splits, C,
                     db, accumulate);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
}  // namespace tlod

extern "C" size_t tlod_conv_wgrad_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS,
                                                     int nprod) {
  if (wgrad_ws_applies(N, Cin, H, W, Cout, KS, nprod)) return wgrad_ws_workspace(N, Cin, H, W, Cout);
  const int sp = with_wgrad_bs_cfg(N, Cin, H, W, Cout, KS, nprod, [&](auto cfg) { return cfg.splits(N, Cin, H, W, Cout); });
  return sp > 0 ? wgrad_bs_ws(sp, Cin, Cout, KS) : 0;
}

extern "C" int tlod_conv_wgrad_bs_f32(const float* dy, const float* x, float* dw, float* db,
                                      int accumulate, int N, int Cin, int H, int W, int Cout,
                                      int KS, int nprod, void* ws, size_t ws_bytes,
                                      tlod_stream_t stream) {
  return tlod_conv_wgrad_bs_ex_f32(dy, x, dw, db, accumulate, nullptr, N, Cin, H, W, Cout, KS,
                                   nprod, ws, ws_bytes, stream);
}

extern "C" int tlod_conv_wgrad_bs_ex_f32(const float* dy, const float* x, float* dw, float* db,
                                         int accumulate, const float* row_scale, int N, int Cin,
                                         int H, int W, int Cout, int KS, int nprod, void* ws,
                                         size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  TLOD_CHECK_ARG((Cout * Cin * KS * KS) % 4 == 0, "Cout*Cin*KS*KS must be a multiple of 4");
  TLOD_CHECK_ARG(KS == 1 || KS == 3, "conv wgrad: only 1x1 and 3x3 kernels");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "conv wgrad bs: nprod must be 3 or 6");
  // 32-bit buffer byte offsets; exact float-reciprocal pixel -> (h, w) below 2^21 pixels
  TLOD_CHECK_ARG((size_t)N * std::max(Cin, Cout) * H * W * 4 < (1ull << 31), "tensor too large");
  TLOD_CHECK_ARG((size_t)H * W < (1u << 21), "map too large");
  hipStream_t s = (hipStream_t)stream;
  if (wgrad_ws_applies(N, Cin, H, W, Cout, KS, nprod))
    return wgrad_ws_launch(dy, x, dw, db, accumulate, row_scale, N, Cin, H, W, Cout, ws, ws_bytes, s);
  const int splits =
      with_wgrad_bs_cfg(N, Cin, H, W, Cout, KS, nprod, [&](auto cfg) { return cfg.splits(N, Cin, H, W, Cout); });
  if (ws_bytes < wgrad_bs_ws(splits, Cin, Cout, KS)) {
    set_error("tlod_conv_wgrad_bs_f32: workspace too small");
    return kWorkspace;
  }
  float* slab = static_cast<float*>(ws);
  float* db_slab = db ? reinterpret_cast<float*>(static_cast<char*>(ws) +
                                                 align_up((size_t)splits * Cout * Cin * KS * KS *
                                                              sizeof(float), 16))
                      : nullptr;
  const int st = with_wgrad_bs_cfg(N, Cin, H, W, Cout, KS, nprod, [&](auto cfg) {
    return cfg.launch(dy, x, slab, db_slab, splits, N, Cin, H, W, Cout, s);
  });
  if (st) return st;
  const size_t count = (size_t)Cout * Cin * KS * KS;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)std::min<size_t>((count / 4 + 255) / 256, 2048)),
                     dim3(256), 0, s, slab, splits, count, dw, accumulate, row_scale,
                     Cin * KS * KS);
  TLOD_LAUNCH_CHECK();
  if (db) {
    hipLaunchKernelGGL(db_reduce_kernel, dim3(div_up(Cout, 256)), dim3(256), 0, s, db_slab, splits,
                       Cout, db, accumulate);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}

// dx = dgrad(dy) * (mask > 0): tlod_conv_fwd_bs_f32's dgrad form with the previous layer's
// ReLU backward in the epilogue (mask = that layer's ReLU output = this conv's input).
extern "C" int tlod_conv_dgrad_bs_mask_f32(const float* dy, const void* wp, const float* mask,
                                           float* dx, int N, int Cin, int H, int W, int Cout,
                                           int nprod, void* ws, size_t ws_bytes,
                                           tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && dy && wp && dx, "bad shape");
  TLOD_CHECK_ARG(mask != dx, "mask must not alias dx");
  Epi e{nullptr, nullptr, nullptr, 0};
  e.mask = mask;
  return conv_fwd_bs_dispatch(dy, (const unsigned short*)wp, e, dx, N, Cin, H, W, Cout, 3, nprod,
                              (float*)ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int tlod_relu_bwd_bias_f32(const float* dy, const float* y, float* g, float* db,
                                      int N, int C, int HW, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && HW > 0, "bad shape");
  hipLaunchKernelGGL(relu_bwd_bias_kernel, dim3(C), dim3(kReluThreads), 0, (hipStream_t)stream,
                     dy, y, nullptr, g, nullptr, db, N, C, HW);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_relu_bwd_ex_f32(const float* dy, const float* y, const float* scale, float* g,
                                    float* g_raw, float* db, int N, int C, int HW,
                                    tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && HW > 0 && dy && g, "bad arguments");
  TLOD_CHECK_ARG(g_raw != g || g_raw == nullptr, "g_raw must not alias g");
  hipLaunchKernelGGL(relu_bwd_bias_kernel, dim3(C), dim3(kReluThreads), 0, (hipStream_t)stream,
                     dy, y, scale, g, g_raw, db, N, C, HW);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" size_t tlod_conv_pack_bs_bytes(int Cout, int Cin, int KS, int dgrad) {
  if (KS != 3) return 0;
  const int rows = dgrad ? Cin : Cout, ins = dgrad ? Cout : Cin;
  return 3 * (size_t)rows * div_up(ins, 8) * kBsKP * sizeof(unsigned short);
}

extern "C" int tlod_conv_pack_bs(const float* weight, int Cout, int Cin, int KS, int dgrad,
                                 void* packed, tlod_stream_t stream) {
  return tlod_conv_pack_bs_ex(weight, nullptr, Cout, Cin, KS, dgrad, packed, stream);
}

extern "C" int tlod_conv_pack_bs_ex(const float* weight, const float* scale, int Cout, int Cin,
                                    int KS, int dgrad, void* packed, tlod_stream_t stream) {
  TLOD_CHECK_ARG(Cout > 0 && Cin > 0 && weight && packed, "bad arguments");
  TLOD_CHECK_ARG(KS == 3, "split-bf16 conv: 3x3 only");
  const int rows = dgrad ? Cin : Cout, ins = dgrad ? Cout : Cin;
  const size_t plane = (size_t)rows * div_up(ins, 8) * 10;  // threads: (row, chunk, tap slot)
  hipLaunchKernelGGL(pack_bs_kernel, dim3((unsigned)std::min<size_t>((plane + 255) / 256, 4096)),
                     dim3(256), 0, (hipStream_t)stream, weight, (unsigned short*)packed, rows, ins,
                     div_up(ins, 8), dgrad, scale);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" size_t tlod_conv_fwd_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS,
                                                   int nprod) {
  size_t b = 0;
  if (conv_fwd_bs_dispatch(nullptr, nullptr, Epi{}, nullptr, N, Cin, H, W, Cout, KS, nprod,
                           nullptr, 0, nullptr, &b) != kOk)
    return 0;
  return b;
}

extern "C" int tlod_conv_fwd_bs_f32(const float* x, const void* wp, const float* scale,
                                    const float* bias, const float* residual, float* y, int N,
                                    int Cin, int H, int W, int Cout, int KS, int relu, int nprod,
                                    void* ws, size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0, "bad shape");
  TLOD_CHECK_ARG(residual != y || residual == nullptr, "residual must not alias y");
  return conv_fwd_bs_dispatch(x, (const unsigned short*)wp, Epi{scale, bias, residual, relu}, y,
                              N, Cin, H, W, Cout, KS, nprod, (float*)ws, ws_bytes,
                              (hipStream_t)stream);
}

extern "C" int tlod_conv_fwd_bs_pool_f32(const float* x, const void* wp, const float* scale,
                                         const float* bias, float* y_pooled, int N, int Cin,
                                         int H, int W, int Cout, int KS, int relu, int nprod,
                                         tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H >= 2 && W >= 2 && Cout > 0 && y_pooled, "bad shape");
  Epi e{scale, bias, nullptr, relu};
  e.pool = y_pooled;
  return conv_fwd_bs_dispatch(x, (const unsigned short*)wp, e, nullptr, N, Cin, H, W, Cout, KS,
                              nprod, nullptr, 0, (hipStream_t)stream);
}
