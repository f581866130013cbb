// Split-bf16 GEMM for the detection head's fully connected layers (gfx950).
//
// Replaces the cuBLAS/hipBLASLt fp32 GEMMs behind nn.Linear in RCNN_top (fc6 25088->4096,
// fc7 4096->4096; lib/DAF/vgg16.py:67-71 via torchvision classifier[:-1]) and the DA
// instance head (lib/DAF/DA.py:53-73): forward, input gradient and weight gradient.
//
//   C[m][n] = sum_k A(m,k) * B(n,k)  (+ bias[n])
//   A(m,k) = A[m*K + k] ("K-contiguous", AK = 1) or A[k*M + m] (AK = 0)
//   B(n,k) = B[n*K + k] (BK = 1)                  or B[k*N + n] (BK = 0)
// fc forward y = x W^T:    A = x [R][I] (AK=1), B = W [O][I] (BK=1)
// fc dgrad  dx = dy W:     A = dy [R][O] (AK=1), B = W as [K=O][N=I] (BK=0)
// fc wgrad  dW = dy^T x:   A = dy as [K=R][M=O] (AK=0), B = x as [K=R][N=I] (BK=0)
//
// Arithmetic: f32 operands split exactly into three bf16 planes (hi, mid, lo) when staged,
// nprod = 6 (or 3) bf16 products per f32 product on v_mfma_f32_32x32x16_bf16, f32
// accumulation — the same f32-level error as the conv kernels (tests/test_linear_gpu.py).
// Tiles 256 x 256 x 16 (8 waves, 4x2 accumulators of 32x32 each), LDS double-buffered.
// K-contiguous operands are staged [row][16 k] (pitch 48 B, ds_read_b128 conflict-free);
// M/N-contiguous ones [16 k][256] (pitch 576 B) and read with the gfx950 transposing
// ds_read_b64_tr_b16, so every global load is a coalesced buffer_load_dwordx4 whatever the
// layout.  Rows/columns past M/N read out of the buffer range (zero).  Split-K over
// workgroups writes fixed-order slabs (deterministic), reduced with the bias.
#include "common.h"
#include "bs_common.h"
#include "tlod.h"

#include <algorithm>

namespace tlod {

namespace {

#ifndef TLOD_MID_STORE
#define TLOD_MID_STORE 1  // stage the next chunk mid-MFMA-phase (see conv.hip)
#endif

constexpr int kBN = 256, kTK = 16, kNT = 512;
constexpr int kWM = 2, kWN = 4, kNJ = 2;  // M tile 64*MI (MI = 4 or 3), N tile 256
constexpr int kPitchK = 48;    // [row][16 k] images
constexpr int kPitchMN = 576;  // [16 k][256] images: rows 16 banks apart for the tr reads

template <int KC>
struct Img {  // one operand's LDS image per plane
  static constexpr int PLANE = KC ? 256 * kPitchK : kTK * kPitchMN;
};

__device__ __forceinline__ uint2 ds_read_tr16(const unsigned char* p) {
  typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 v4bf;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wold-style-cast"
  auto lp = (__attribute__((address_space(3))) v4bf*)(const_cast<unsigned char*>(p));
#pragma clang diagnostic pop
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(lp));
}

// Staging of one operand tile of RT rows (the operand's M or N extent is R).
template <int KC, int NPL, int RT>
struct Stager {
  static constexpr int VECS = RT * kTK / 4;          // 4-element vectors per chunk
  static constexpr int IT = (VECS + kNT - 1) / kNT;
  static constexpr int LPR = RT / 4;                 // MN: lanes per k row
  i32x4 rsrc;
  int off[IT];     // element offset of this lane's 4-vector at chunk 0 (or -1: dead)
  int lds[IT];     // byte offset inside one plane image (-1: no slot)
  int lim[IT];     // for the tail mask: K - k (KC) or R - r (MN)
  f32x4v r[IT];
  unsigned mask[IT];

  __device__ void init(const float* P, int R, int K, int r0, int tid) {
    rsrc = make_buffer_rsrc(P, (unsigned)R * (unsigned)K * 4u);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = tid + i * kNT;
      const bool slot = idx < VECS;
      if (KC) {  // vector idx: row idx/4, k segment 4 (idx & 3)
        const int row = idx >> 2, k4 = (idx & 3) * 4;
        off[i] = slot && r0 + row < R ? (r0 + row) * K + k4 : -1;
        lds[i] = slot ? row * kPitchK + 2 * k4 : -1;
        lim[i] = K - k4;
      } else {   // vector idx: k row idx / LPR, columns 4 (idx % LPR)
        const int kr = idx / LPR, c4 = (idx % LPR) * 4;
        off[i] = kr * R + r0 + c4;
        lds[i] = slot ? kr * kPitchMN + 2 * c4 : -1;
        lim[i] = R - (r0 + c4);
      }
    }
  }
  __device__ void load(int kc, int R) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (KC) {
        r[i] = raw_buffer_load_v4f32(rsrc, off[i] >= 0 ? (off[i] + kc) * 4 : kBufOOB, 0, 0);
        mask[i] = lt_mask4(lim[i] - kc);
      } else {  // k rows past K fall past the buffer end (zero)
        r[i] = raw_buffer_load_v4f32(rsrc, lds[i] >= 0 ? (off[i] + kc * R) * 4 : kBufOOB, 0, 0);
        mask[i] = lt_mask4(lim[i]);
      }
    }
  }
  __device__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (lds[i] < 0) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ((mask[i] >> e) & 1) ? r[i][e] : 0.f;
      unsigned sp[3][2];
      split4<NPL>(v, sp);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        *reinterpret_cast<uint2*>(img + pl * Img<KC>::PLANE + lds[i]) = make_uint2(sp[pl][0], sp[pl][1]);
    }
  }
};

// MFMA operand (8 k values of row/column `base + l32`) from one plane image.
template <int KC>
__device__ __forceinline__ u32x4 read_operand(const unsigned char* img, int base, int lane) {
  const int l32 = lane & 31, khalf = lane >> 5;
  if (KC) return *reinterpret_cast<const u32x4*>(img + (base + l32) * kPitchK + 16 * khalf);
  // tr reads: lane 4q+p of 16-lane group g supplies row k0+q, columns 4p..4p+3 of the
  // group's 16 columns; it receives its own column's 4 consecutive k
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int k0 = 8 * (g >> 1) + q;
  const uint2 lo = ds_read_tr16(img + k0 * kPitchMN + 2 * col);
  const uint2 hi = ds_read_tr16(img + (k0 + 4) * kPitchMN + 2 * col);
  return u32x4{lo.x, lo.y, hi.x, hi.y};
}

template <int AK, int BK, int NP, int MI>
__global__ void __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm_bs_kernel(const float* __restrict__ A, const float* __restrict__ B,
               const float* __restrict__ bias, float* __restrict__ C, int M, int N, int K,
               int tiles_m, int tiles_n, int splits, int chunks_per_split) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  constexpr int A_PL = Img<AK>::PLANE, B_PL = Img<BK>::PLANE;
  constexpr int BUF = NPL * (A_PL + B_PL);
  constexpr int BM = kWM * MI * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = tiles_m * tiles_n * splits;
  int t = xcd_remap(blockIdx.x, nwg);
  const int mt = t % tiles_m; t /= tiles_m;
  const int nt = t % tiles_n;
  const int split = t / tiles_n;
  const int m0 = mt * BM, n0 = nt * kBN;
  const int nchunks = (K + kTK - 1) / kTK;
  const int c_begin = split * chunks_per_split;
  const int c_end = min(nchunks, c_begin + chunks_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / kWN, wn = wid % kWN;

  Stager<AK, NPL, BM> sa;
  Stager<BK, NPL, kBN> sb;
  sa.init(A, M, K, m0, tid);
  sb.init(B, N, K, n0, tid);

  f32x16 acc[MI][kNJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < kNJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto store = [&](unsigned char* buf) {
    sa.store(buf);
    sb.store(buf + NPL * A_PL);
  };
  if (c_begin < c_end) {
    sa.load(c_begin * kTK, M);
    sb.load(c_begin * kTK, N);
    store(smem);
  }
  __syncthreads();
  for (int c = c_begin; c < c_end; ++c) {
    const int it = c - c_begin;
    const unsigned char* buf = smem + (it & 1) * BUF;
    const bool more = c + 1 < c_end;
    if (more) {
      sa.load((c + 1) * kTK, M);
      sb.load((c + 1) * kTK, N);
    }
    u32x4 b[kNJ][3];
#pragma unroll
    for (int j = 0; j < kNJ; ++j)
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        b[j][pl] = read_operand<BK>(buf + NPL * A_PL + pl * B_PL, wn * kNJ * 32 + j * 32, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if (TLOD_MID_STORE && more && i == MI / 2) store(smem + ((it + 1) & 1) * BUF);
      u32x4 a[3];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        a[pl] = read_operand<AK>(buf + pl * A_PL, wm * MI * 32 + i * 32, lane);
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        if constexpr (NP == 6) {
          acc[i][j] = mfma_bf16(a[2], b[j][0], acc[i][j]);
          acc[i][j] = mfma_bf16(a[1], b[j][1], acc[i][j]);
          acc[i][j] = mfma_bf16(a[0], b[j][2], acc[i][j]);
        }
        acc[i][j] = mfma_bf16(a[1], b[j][0], acc[i][j]);
        acc[i][j] = mfma_bf16(a[0], b[j][1], acc[i][j]);
        acc[i][j] = mfma_bf16(a[0], b[j][0], acc[i][j]);
      }
    }
    if (!TLOD_MID_STORE && more) store(smem + ((it + 1) & 1) * BUF);
    __syncthreads();
  }

  // splits == 1: C (+ bias); else slab[split][M][N] (bias added by the reduce)
  float* out = splits == 1 ? C : C + (size_t)split * M * N;
  const bool add_bias = splits == 1 && bias != nullptr;
  const int l32 = lane & 31, khalf = lane >> 5;
#pragma unroll
  for (int j = 0; j < kNJ; ++j) {
    const int n = n0 + wn * kNJ * 32 + j * 32 + l32;
    if (n >= N) continue;
    const float bv = add_bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (m < M) out[(size_t)m * N + n] = acc[i][j][r] + bv;
      }
  }
}

// C[m][n] = sum_s slab[s][m][n] (+ bias[n]), fixed split order.
__global__ void gemm_slab_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                        const float* __restrict__ bias, float* __restrict__ C) {
  const size_t count = (size_t)M * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
       i += (size_t)gridDim.x * blockDim.x) {
    float s = slab[i];
    for (int k = 1; k < splits; ++k) s += slab[(size_t)k * count + i];
    if (bias) s += bias[i % N];
    C[i] = s;
  }
}

template <typename K>
int slots_of(K kern, size_t lds) {
  static int cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kNT, lds) != hipSuccess ||
      per_cu < 1 || cus < 1) {
    (void)hipGetLastError();
    return 256;
  }
  return cached = per_cu * cus;
}

// Split count: fill whole rounds of the resident slots, >= 8 chunks per piece, and do not
// let the slab round trip (2 sp + 1 passes over M*N floats) outweigh the compute saved.
int pick_gemm_splits(int tiles, int nchunks, int slots, double chunk_s, double mn_bytes) {
  int best = 1;
  double best_t = 1e30;
  for (int sp = 1; sp <= std::max(1, std::min(64, nchunks / 8)); ++sp) {
    const int cps = div_up(nchunks, sp);
    const int esp = div_up(nchunks, cps);
    const long long rounds = ((long long)tiles * esp + slots - 1) / slots;
    const double t = (double)rounds * cps * chunk_s + (esp > 1 ? (2.0 * esp + 1.0) * mn_bytes / 4e12 : 0.0);
    if (t < best_t * 0.999) {
      best_t = t;
      best = esp;
    }
  }
  return best;
}

template <int AK, int BK, int NP, int MI>
struct Gemm {
  static constexpr int NPL = NP == 6 ? 3 : 2;
  static constexpr int kBM = kWM * MI * 32;
  static constexpr size_t kLds = 2 * NPL * (Img<AK>::PLANE + Img<BK>::PLANE);
  static int splits(int M, int N, int K) {
    const int slots = slots_of(gemm_bs_kernel<AK, BK, NP, MI>, kLds);
    const int tiles = div_up(M, kBM) * div_up(N, kBN);
    const double chunk_s = 2.0 * kBM * kBN * kTK * NP / (2516.6e12 * 0.5 / slots);
    return pick_gemm_splits(tiles, div_up(K, kTK), slots, chunk_s, 4.0 * M * N);
  }
  static int run(const float* A, const float* B, const float* bias, float* C, int M, int N, int K,
                 float* ws, size_t ws_bytes, hipStream_t s) {
    const int sp = splits(M, N, K);
    if (sp > 1 && ws_bytes < (size_t)sp * M * N * sizeof(float)) {
      set_error("tlod_gemm_bs_f32: workspace too small");
      return kWorkspace;
    }
    const int tiles_m = div_up(M, kBM), tiles_n = div_up(N, kBN);
    const int cps = div_up(div_up(K, kTK), sp);
    auto kern = gemm_bs_kernel<AK, BK, NP, MI>;
    static bool attr = false;
    if (!attr) {
      TLOD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds));
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(tiles_m * tiles_n * sp), dim3(kNT), kLds, s, A, B, bias,
                       sp > 1 ? ws : C, M, N, K, tiles_m, tiles_n, sp, cps);
    TLOD_LAUNCH_CHECK();
    if (sp > 1) {
      const size_t count = (size_t)M * N;
      hipLaunchKernelGGL(gemm_slab_reduce_kernel, dim3((unsigned)std::min<size_t>((count + 255) / 256, 4096)),
                         dim3(256), 0, s, ws, sp, M, N, bias, C);
      TLOD_LAUNCH_CHECK();
    }
    return kOk;
  }
};

template <typename F>
int with_gemm(int M, int ak, int bk, int nprod, F&& f) {
  // M tile 192 when it pads M less (the 556 RoI rows of the head: 576 vs 768)
  const bool m192 = div_up(M, 192) * 192 < div_up(M, 256) * 256;
#define TLOD_GEMM_CASE(A_, B_)                                                 \
  if (ak == A_ && bk == B_) {                                                  \
    if (m192) return nprod == 6 ? f(Gemm<A_, B_, 6, 3>{}) : f(Gemm<A_, B_, 3, 3>{}); \
    return nprod == 6 ? f(Gemm<A_, B_, 6, 4>{}) : f(Gemm<A_, B_, 3, 4>{});     \
  }
  TLOD_GEMM_CASE(1, 1)
  TLOD_GEMM_CASE(1, 0)
  TLOD_GEMM_CASE(0, 0)
  TLOD_GEMM_CASE(0, 1)
#undef TLOD_GEMM_CASE
  return kUnsupported;
}

}  // namespace

}  // namespace tlod

using namespace tlod;

extern "C" size_t tlod_gemm_bs_workspace_bytes(int M, int N, int K, int a_kcontig, int b_kcontig,
                                               int nprod) {
  if (M <= 0 || N <= 0 || K <= 0 || (nprod != 3 && nprod != 6)) return 0;
  const int sp = with_gemm(M, a_kcontig ? 1 : 0, b_kcontig ? 1 : 0, nprod,
                           [&](auto g) { return g.splits(M, N, K); });
  return sp > 1 ? (size_t)sp * M * N * sizeof(float) : 0;
}

extern "C" int tlod_gemm_bs_f32(const float* a, const float* b, const float* bias, float* c, int M,
                                int N, int K, int a_kcontig, int b_kcontig, int nprod, void* ws,
                                size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(M > 0 && N > 0 && K > 0 && a && b && c, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  // 32-bit buffer byte offsets
  TLOD_CHECK_ARG((size_t)std::max(M, N) * K * 4 < (1ull << 31), "operand too large");
  return with_gemm(M, a_kcontig ? 1 : 0, b_kcontig ? 1 : 0, nprod, [&](auto g) {
    return g.run(a, b, bias, c, M, N, K, static_cast<float*>(ws), ws_bytes, (hipStream_t)stream);
  });
}
