// Warp-specialized split-bf16 GEMM (round 4): the detection head's fully connected layers
// (fc6 / fc7, lib/DAF/vgg16.py:67-71; the DA instance head, lib/DAF/DA.py:53-73) and the
// ResNet101 RoI head's convolutions run as GEMMs (lib/DAF/resnet.py _head_to_tail over
// layer4) — forward, input gradient and weight gradient of nn.Linear, cuBLAS SGEMM in the
// reference:
//
//   C[m][n] = sum_k A(m,k) * B(n,k)  (+ bias[n])
//   A(m,k) = A[m*K + k] (AK = 1, "K-contiguous") or A[k*M + m] (AK = 0); B likewise (BK)
//
// gemm.hip's gemm_bs_kernel (8 waves that all stage and all compute, 256 x 256 x 16 tiles on
// v_mfma_f32_32x32x16_bf16) kept its matrix pipes ~45% busy.  Here, as in the convolutions'
// warp-specialized kernels:
//   * 4 producer waves load the next chunks (raw buffer dwordx4 loads, two chunks ahead in
//     two register slots, unconditional straight-line staging), split every f32 exactly into
//     three bf16 planes (bs_common.h split2) and store them to the LDS buffer the MFMA waves
//     are not reading;
//   * 8 MFMA waves, each a (16 MT) x 64 block of the BM x 128 tile (BM = 64 MT: 256, or 192
//     when that pads M less — the 556 RoI rows of the VGG16 head), read fragments and issue
//     v_mfma_f32_16x16x32_bf16 (the 16x16 shape holds a higher clock than 32x32,
//     MI355X_MICROARCH.md DVFS item 7): one 32-deep k-step per chunk, six products per tile;
//   * one barrier per chunk for both roles, two LDS buffers of 3 planes x (BM + 128) x 32.
// Fragment k order: lane group g (lanes 16g..16g+15) holds k quads g and g + 4 (k = 4g..4g+3,
// 16+4g..16+4g+3) of its row — any permutation of K shared by A and B gives the same sums,
// and this one makes both LDS images conflict-free:
//   * K-contiguous operands are staged [row][32 k] (64 B per row per plane), 16-B slot
//     g ^ ((row >> 1) & 3) holding quads g, g + 4: one ds_read_b128 per fragment;
//   * M/N-contiguous operands are staged [k][R] with a row pitch of 8 mod 64 dwords and read
//     with ds_read_b64_tr_b16 (lane 4q + p of group g supplies k row 4g + q (then 16 + 4g + q),
//     columns 4p..4p+3; lane i receives column i's 4 k), so every global load is a coalesced
//     dwordx4 whatever the layout.
// K past the end reads zeros (out-of-range offsets) or is masked (a K-contiguous vector that
// straddles K).  Whole rounds of tiles run the full K; the tail round is split over K into
// fixed pieces written in lane order and reduced in split order (deterministic), with the bias.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "bs_common.h"

namespace tlod {

namespace gws {
constexpr int BN = 128, KC = 32;  // N tile, K chunk (one 16x16x32 k-step)
constexpr int NMW = 8, NPW = 4, NT = (NMW + NPW) * 64;
constexpr int ROWK = KC * 2;  // K-contiguous image: 64 B per row per plane
// [k][R] image row pitch in bytes: 8 mod 64 dwords, so the 8 k rows a 32-lane half of a tr
// read touches cover all 64 banks
constexpr int pitch_mn(int R) { return R <= 128 ? 288 : 544; }
template <int KCONT, int R>
struct Img {
  static constexpr int PLANE = KCONT ? R * ROWK : KC * pitch_mn(R);
};
template <int AK, int BK, int MT>
struct Cfg {
  static constexpr int BM = 64 * MT;
  static constexpr int A_PL = Img<AK, BM>::PLANE, B_PL = Img<BK, BN>::PLANE;
  static constexpr int BUF = 3 * (A_PL + B_PL);
  static constexpr int LDS_BYTES = 2 * BUF;
  static constexpr int TILE_FLOATS = BM * BN;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};
}  // namespace gws

__device__ __forceinline__ uint2 gws_read_tr16(const unsigned char* p) {
  typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 v4bf;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wold-style-cast"
  auto lp = (__attribute__((address_space(3))) v4bf*)(const_cast<unsigned char*>(p));
#pragma clang diagnostic pop
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(lp));
}

__device__ __forceinline__ f32x4 gws_mfma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// One operand's staging by the producer waves: R rows of the operand (its M or N extent is
// Rtot) x 32 k per chunk = 8 R / 4 float4 vectors, IT per producer lane.
template <int KCONT, int R>
struct GwsStager {
  static constexpr int IT = 8 * R / (gws::NPW * 64);
  static_assert(8 * R % (gws::NPW * 64) == 0, "staging");
  // vector idx = ptid + 256 i: K-contiguous row idx >> 3, k quad idx & 7; M/N-contiguous k
  // row idx / (R / 4), columns 4 (idx % (R / 4)).  Offsets are recomputed per use from ptid
  // (a handful of integer ops) instead of being held in registers across the loop.
  i32x4 rsrc;
  int ptid, r0, Rtot, K;
  f32x4v v[2][IT];

  __device__ void init(const float* P, int Rtot_, int K_, int r0_, int ptid_) {
    rsrc = make_buffer_rsrc(P, (unsigned)Rtot_ * (unsigned)K_ * 4u);
    ptid = ptid_;
    r0 = r0_;
    Rtot = Rtot_;
    K = K_;
  }
  __device__ static int row_of(int idx) { return KCONT ? idx >> 3 : idx / (R / 4); }
  __device__ static int col_of(int idx) { return KCONT ? 4 * (idx & 7) : 4 * (idx % (R / 4)); }
  // chunk at k0; loads past K read zeros (MN: past the buffer) or are masked at the store
  template <int S>
  __device__ void load(int k0) {
    int pt = ptid;
    asm volatile("" : "+v"(pt));  // opaque: keeps the per-vector offsets out of the loop
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = pt + i * gws::NPW * 64;
      const int a = row_of(idx), b = col_of(idx);
      int o;
      if (KCONT) o = r0 + a < Rtot ? ((r0 + a) * K + k0 + b) * 4 : kBufOOB;
      else o = ((k0 + a) * Rtot + r0 + b) * 4;
      v[S][i] = raw_buffer_load_v4f32(rsrc, o, 0, 0);
    }
  }
  template <int S>
  __device__ void store(unsigned char* img, int kleft) const {
    int pt = ptid;
    asm volatile("" : "+v"(pt));
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = pt + i * gws::NPW * 64;
      const int a = row_of(idx), b = col_of(idx);
      const unsigned m = KCONT ? lt_mask4(kleft - b) : lt_mask4(Rtot - (r0 + b));
      const int lds = KCONT ? a * gws::ROWK + 16 * (((b >> 2) & 3) ^ ((a >> 1) & 3)) + ((b & 16) >> 1)
                            : a * gws::pitch_mn(R) + 2 * b;
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = ((m >> e) & 1) ? v[S][i][e] : 0.f;
      unsigned sp[3][2];
      split4<3>(x, sp);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        *reinterpret_cast<uint2*>(img + pl * gws::Img<KCONT, R>::PLANE + lds) = make_uint2(sp[pl][0], sp[pl][1]);
    }
  }
};

// Fragment of rows base + l16 (16 of them) at the lane group's k quads from one plane image.
template <int KCONT, int R>
__device__ __forceinline__ u32x4 gws_frag(const unsigned char* img, int lane_off, int base) {
  if (KCONT) return *reinterpret_cast<const u32x4*>(img + lane_off + base * gws::ROWK);
  const unsigned char* p = img + lane_off + 2 * base;
  const uint2 lo = gws_read_tr16(p);
  const uint2 hi = gws_read_tr16(p + 16 * gws::pitch_mn(R));
  return u32x4{lo.x, lo.y, hi.x, hi.y};
}
template <int KCONT, int R>
__device__ __forceinline__ int gws_lane_off(int lane) {
  const int g = lane >> 4, l16 = lane & 15;
  if (KCONT) return l16 * gws::ROWK + 16 * (g ^ ((l16 >> 1) & 3));
  return (4 * g + (l16 >> 2)) * gws::pitch_mn(R) + 8 * (l16 & 3);
}

// Grid: dp_tiles direct workgroups, then n_tail x ksplit split pieces (see gemm_ws_plan).
template <int AK, int BK, int MT>
__global__ void __launch_bounds__(gws::NT) __attribute__((amdgpu_waves_per_eu(3, 3)))
gemm_ws_kernel(const float* __restrict__ A, const float* __restrict__ B,
               const float* __restrict__ bias, const float* __restrict__ residual, int relu,
               float* __restrict__ C, float* __restrict__ slab, int M, int N, int K, int tiles_m,
               int dp_tiles, int n_tail, int ksplit, int cps) {
  using namespace gws;
  using G = Cfg<AK, BK, MT>;
  constexpr int BM = G::BM;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

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
  const int mt = t % tiles_m, nt = t / tiles_m;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nchunks = (K + KC - 1) / KC;
  const int c_begin = direct ? 0 : min(nchunks, split * cps);
  const int c_end = direct ? nchunks : min(nchunks, c_begin + cps);
  const int nch = c_end - c_begin;
  const int tid = threadIdx.x;

  if (tid >= NMW * 64) {
    // ================= producers: chunk j of the range sits in register slot j & 1 from its
    // load (two chunks ahead) to its split + store into LDS buffer j & 1.  Straight-line and
    // unconditional: a load past the range reads zeros or masked values into the buffer that
    // is not read next, so the vmcnt wait before a store leaves the other slot's loads in
    // flight.  1 + 2 ceil(nch / 2) barriers, as the MFMA waves.
#ifdef TLOD_GWS_NOPROD
    for (int j = 0; j < 1 + 2 * ((nch + 1) / 2); ++j) __syncthreads();
    return;
#endif
    const int ptid = tid - NMW * 64;
    GwsStager<AK, BM> sa;
    GwsStager<BK, BN> sb;
    sa.init(A, M, K, m0, ptid);
    sb.init(B, N, K, n0, ptid);
    int kl = c_begin * KC;  // k0 of the next chunk to load
    int ks[2];              // K - k0 of the chunk in each slot (K-contiguous masks)
    auto load = [&](auto slc) {
      constexpr int S = decltype(slc)::value;
      sa.template load<S>(kl);
      sb.template load<S>(kl);
      ks[S] = K - kl;
      kl += KC;
    };
    auto store = [&](auto slc, unsigned char* buf) {
      constexpr int S = decltype(slc)::value;
      sa.template store<S>(buf, ks[S]);
      sb.template store<S>(buf + 3 * G::A_PL, ks[S]);
    };
    const std::integral_constant<int, 0> S0;
    const std::integral_constant<int, 1> S1;
    load(S0);
    load(S1);
    store(S0, smem);
    load(S0);
    __syncthreads();
    for (int j = 0; j < nch; j += 2) {
      store(S1, smem + G::BUF);  // chunk j + 1
      load(S1);                  // chunk j + 3
      __syncthreads();
      store(S0, smem);           // chunk j + 2
      load(S0);                  // chunk j + 4
      __syncthreads();
    }
    return;
  }

#ifdef TLOD_GWS_NOMFMA
  for (int j = 0; j < 1 + 2 * ((nch + 1) / 2); ++j) __syncthreads();
  if (tid < 100000) return;
#endif
  // ================= MFMA waves: wave w owns rows 16 MT (w & 3) + [0, 16 MT) and columns
  // 64 (w >> 2) + [0, 64) of the tile: MT x 4 tiles of 16 x 16
  const int lane = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;
  const int a_lane = gws_lane_off<AK, BM>(lane);
  const int b_lane = 3 * G::A_PL + gws_lane_off<BK, BN>(lane);
  f32x4 acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();
  auto iter = [&](int j) {
    if (j < nch) {
      const unsigned char* buf = smem + (j & 1) * G::BUF;
      u32x4 b[4][3];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          b[jj][pl] = gws_frag<BK, BN>(buf + pl * G::B_PL, b_lane, 64 * wn + 16 * jj);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        u32x4 a[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[pl] = gws_frag<AK, BM>(buf + pl * G::A_PL, a_lane, 16 * MT * wm + 16 * i);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc[i][jj] = gws_mfma(a[0], b[jj][0], acc[i][jj]);
          acc[i][jj] = gws_mfma(a[1], b[jj][0], acc[i][jj]);
          acc[i][jj] = gws_mfma(a[0], b[jj][1], acc[i][jj]);
          acc[i][jj] = gws_mfma(a[2], b[jj][0], acc[i][jj]);
          acc[i][jj] = gws_mfma(a[1], b[jj][1], acc[i][jj]);
          acc[i][jj] = gws_mfma(a[0], b[jj][2], acc[i][jj]);
        }
      }
    }
    __syncthreads();
  };
  for (int j = 0; j < nch; j += 2) {
    iter(j);
    iter(j + 1);  // the odd count's last iteration computes nothing (pairs the producers')
  }

  if (!direct) {  // partial tile in lane order: [wave][i][j][lane][4]
    float* S = slab + ((size_t)split * n_tail + ti) * G::TILE_FLOATS + (size_t)w * (MT * 4 * 256) + lane * 4;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) *reinterpret_cast<f32x4*>(S + (i * 4 + jj) * 256) = acc[i][jj];
    return;
  }
  // direct: C = act(acc (+ bias) (+ residual)), branch-free (out-of-range offsets: the
  // residual loads read 0, the stores are dropped); a column's residuals are loaded ahead of
  // its stores
  const int g = lane >> 4, l16 = lane & 15;
  const unsigned mn4 = (unsigned)M * (unsigned)N * 4u;
  const i32x4 c_rsrc = make_buffer_rsrc(C, mn4);
  const i32x4 r_rsrc = make_buffer_rsrc(residual != nullptr ? residual : C, residual != nullptr ? mn4 : 0u);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int n = n0 + 64 * wn + 16 * jj + l16;
    const float bv = bias != nullptr ? bias[min(n, N - 1)] : 0.f;
    float res[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 16 * MT * wm + 16 * i + 4 * g + e;
        res[i][e] = residual != nullptr
                        ? raw_buffer_load_f32(r_rsrc, m < M && n < N ? (m * N + n) * 4 : kBufOOB, 0, 0)
                        : 0.f;
      }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 16 * MT * wm + 16 * i + 4 * g + e;
        float v = acc[i][jj][e] + bv;
        if (residual != nullptr) v += res[i][e];
        if (relu) v = fmaxf(v, 0.f);
        raw_buffer_store_f32(v, c_rsrc, m < M && n < N ? (m * N + n) * 4 : kBufOOB, 0, 0);
      }
  }
}

// Tail tiles: C = act(sum over splits of the lane-ordered pieces (split order) + bias
// (+ residual)).  One thread
// per float4 of a piece: rows 4g..4g+3 of one column.
template <int MT>
__global__ void __launch_bounds__(256) gemm_ws_reduce_kernel(const float* __restrict__ slab,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ residual,
                                                             int relu, float* __restrict__ C, int M, int N,
                                                             int tiles_m, int dp_tiles,
                                                             int n_tail, int ksplit) {
  using namespace gws;
  constexpr int TF4 = 64 * MT * BN / 4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= n_tail * TF4) return;
  const size_t stride4 = (size_t)n_tail * TF4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab) + idx;
  f32x4 sum = s4[0];
  int k = 1;
  for (; k + 4 <= ksplit; k += 4) {  // four loads in flight, adds in split order
    const f32x4 v0 = s4[k * stride4], v1 = s4[(k + 1) * stride4];
    const f32x4 v2 = s4[(k + 2) * stride4], v3 = s4[(k + 3) * stride4];
    sum += v0;
    sum += v1;
    sum += v2;
    sum += v3;
  }
  for (; k < ksplit; ++k) sum += s4[k * stride4];
  int r = idx;
  const int ti = r / TF4;
  r -= ti * TF4;
  const int lane = r % 64; r /= 64;
  const int jj = r % 4; r /= 4;
  const int i = r % MT;
  const int w = r / MT;
  const int t = dp_tiles + ti;
  const int mt = t % tiles_m, nt = t / tiles_m;
  const int n = nt * BN + 64 * (w >> 2) + 16 * jj + (lane & 15);
  if (n >= N) return;
  const float bv = bias != nullptr ? bias[n] : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = mt * 64 * MT + 16 * MT * (w & 3) + 16 * i + 4 * (lane >> 4) + e;
    if (m >= M) continue;
    float v = sum[e] + bv;
    if (residual != nullptr) v += residual[(size_t)m * N + n];
    if (relu) v = fmaxf(v, 0.f);
    C[(size_t)m * N + n] = v;
  }
}

// ---- host side

namespace {

struct GwsPlan {
  int mt, tiles_m, tiles_n, dp_tiles, ksplit, cps;
};

// M tile 192 when it pads M less (the 556 RoI rows of the VGG16 head: 576 vs 768).  Whole
// rounds of tiles over the full K, the last partial round split over K when that beats a
// mostly idle round (tile time at ~80% of the MFMA rate at 2.1 GHz, the slab round trip at
// 4 TB/s, 6 us per reduce launch); one resident workgroup per CU.
GwsPlan gemm_ws_plan(int M, int N, int K) {
  GwsPlan p;
  p.mt = div_up(M, 192) * 192 < div_up(M, 256) * 256 ? 3 : 4;
  const int bm = 64 * p.mt;
  p.tiles_m = div_up(M, bm);
  p.tiles_n = div_up(N, gws::BN);
  const int T = p.tiles_m * p.tiles_n;
  const int nchunks = div_up(K, gws::KC);
  const int slots = 256;
  // per chunk and SIMD: 2 MFMA waves x MT x 4 tiles x 6 MFMAs x 16 cycles
  const double chunk_s = 2.0 * p.mt * 4 * 6 * 16 / (2.1e9 * 0.8);
  const double tile_s = chunk_s * nchunks + 2e-6;
  const double tile_bytes = 4.0 * bm * gws::BN;
  p.dp_tiles = T;
  p.ksplit = 1;
  p.cps = nchunks;
  double best = (double)((T + slots - 1) / slots) * tile_s;
  const int q = T / slots;
  for (int k = 2; k <= std::min(32, nchunks / 2); ++k) {
    const int cps = div_up(nchunks, k);
    const int kk = div_up(nchunks, cps);
    for (int dp : {q * slots, 0}) {
      const int tail = T - dp;
      if (tail <= 0) continue;
      const double t = (double)dp / slots * tile_s +
                       (double)(((long long)tail * kk + slots - 1) / slots) * (chunk_s * cps + 2e-6) +
                       (2.0 * kk + 1.0) * tail * tile_bytes / 4e12 + 6e-6;
      if (t < best * 0.97) {
        best = t;
        p.dp_tiles = dp;
        p.ksplit = kk;
        p.cps = cps;
      }
    }
  }
  return p;
}

template <int AK, int BK, int MT>
int gemm_ws_run(const float* a, const float* b, const float* bias, const float* res, int relu,
                float* c, int M, int N, int K, const GwsPlan& p, float* ws, hipStream_t s) {
  using G = gws::Cfg<AK, BK, MT>;
  auto kern = gemm_ws_kernel<AK, BK, MT>;
  static bool attr = false;
  if (!attr) {
    TLOD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES));
    attr = true;
  }
  const int n_tail = p.tiles_m * p.tiles_n - p.dp_tiles;
  const int nwg = p.dp_tiles + (p.ksplit > 1 ? n_tail * p.ksplit : 0);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(gws::NT), G::LDS_BYTES, s, a, b, bias, res, relu, c, ws, M, N, K,
                     p.tiles_m, p.dp_tiles, n_tail, p.ksplit, p.cps);
  TLOD_LAUNCH_CHECK();
  if (p.ksplit > 1) {
    const int n4 = n_tail * G::TILE_FLOATS / 4;
    hipLaunchKernelGGL(gemm_ws_reduce_kernel<MT>, dim3(div_up(n4, 256)), dim3(256), 0, s, ws, bias,
                       res, relu, c, M, N, p.tiles_m, p.dp_tiles, n_tail, p.ksplit);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}

}  // namespace

// bf16x6 GEMMs whose output fits 32-bit buffer offsets, opt-in (TLOD_GEMM_WS=1): measured
// slower than gemm_bs_kernel on the VGG16 head (fc7 0.111 -> 0.128 ms, fc6 wgrad 0.617 ->
// 0.697; DAF step 71.0 -> 70.0 img/s, one lease) — the 64 x 64 wave tiles of 16x16 MFMAs read
// 33% more LDS bytes per flop than gemm_bs_kernel's 128 x 64 tiles of 32x32 MFMAs, and the
// 96 tiles of the 556-row head leave CUs idle at any even K split.
bool gemm_ws_applies(int M, int N, int K, int nprod) {
  static const bool on = [] {
    const char* v = getenv("TLOD_GEMM_WS");
    return v && *v && atoi(v) != 0;
  }();
  (void)K;
  return on && nprod == 6 && (size_t)M * N * 4 < (1ull << 31);
}

size_t gemm_ws_workspace(int M, int N, int K) {
  const GwsPlan p = gemm_ws_plan(M, N, K);
  if (p.ksplit <= 1) return 0;
  return (size_t)p.ksplit * (p.tiles_m * p.tiles_n - p.dp_tiles) * 64 * p.mt * gws::BN * sizeof(float);
}

int gemm_ws_launch(const float* a, const float* b, const float* bias, const float* res, int relu,
                   float* c, int M, int N, int K, int a_kcontig, int b_kcontig, void* ws,
                   size_t ws_bytes, hipStream_t s) {
  const GwsPlan p = gemm_ws_plan(M, N, K);
  if (ws_bytes < gemm_ws_workspace(M, N, K)) {
    set_error("tlod_gemm_bs_f32: workspace too small");
    return kWorkspace;
  }
  float* w = static_cast<float*>(ws);
  const int ak = a_kcontig ? 1 : 0, bk = b_kcontig ? 1 : 0;
#define TLOD_GWS_CASE(A_, B_)                                                           \
  if (ak == A_ && bk == B_)                                                            \
    return p.mt == 3 ? gemm_ws_run<A_, B_, 3>(a, b, bias, res, relu, c, M, N, K, p, w, s)         \
                     : gemm_ws_run<A_, B_, 4>(a, b, bias, res, relu, c, M, N, K, p, w, s);
  TLOD_GWS_CASE(1, 1)
  TLOD_GWS_CASE(1, 0)
  TLOD_GWS_CASE(0, 0)
  TLOD_GWS_CASE(0, 1)
#undef TLOD_GWS_CASE
  return kInvalidArg;
}

}  // namespace tlod
