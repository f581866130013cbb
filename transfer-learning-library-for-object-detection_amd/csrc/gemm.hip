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
// K-contiguous operands are staged [row][16 k] (32-B rows, the 16-B halves swapped on rows
// with bit 3 set: conflict-free for the staging ds_write_b64 and the fragment reads);
// M/N-contiguous ones [16 k][256] (pitch 576 B) and read with the gfx950 transposing
// ds_read_b64_tr_b16, so every global load is a coalesced buffer_load_dwordx4 whatever the
// layout.  Rows/columns past M/N read out of the buffer range (zero).  Split-K over
// workgroups writes fixed-order slabs (deterministic), reduced with the bias.
#include "common.h"
#include "bs_common.h"
#include "tlod.h"

#include <algorithm>
#include <type_traits>

namespace tlod {

namespace {

// 1: priority 1 around each chunk's MFMA cluster (cdna_hip_programming.md T5): fc6 fwd /
// wgrad -1.2% / -2.4%, fc7 wgrad -2.5% (two interleaved pairs, one lease).  The same around
// the ws conv's and wgrad_ws's k-steps (TLOD_WS_PRIO=2, TLOD_WGWS_MPRIO=2) made them slower
// (conv3_3 dgrad 0.399 -> 0.411 ms); the static form (waves 4-7 at priority 1, =1) measured
// within noise.
#ifndef TLOD_GEMM_PRIO
#define TLOD_GEMM_PRIO 1
#endif
#ifndef TLOD_CONV1X1_OCC2  // (see conv_gemm_bs_kernel)
#define TLOD_CONV1X1_OCC2 1
#endif
#ifndef TLOD_GEMM_DEPTH2  // two chunks of loads in flight (mainloop, MI <= 2 tiles)
#define TLOD_GEMM_DEPTH2 1
#endif

constexpr int kBN = 256, kTK = 16, kNT = 512;
constexpr int kWM = 2, kWN = 4, kNJ = 2;  // M tile 64*MI (MI = 4 or 3), N tile 256
// [row][16 k] images: 32-B rows, k half h of row r at byte 16 (h ^ bit 3 of r).  The
// staging ds_write_b64 (16-lane groups = 4 rows x 4 k segments: 128 contiguous bytes) and
// the fragment reads (ds_read_b128 of one half of 32 rows; ds_read_b64 of 16 rows) then
// touch every bank once per lane group (tools/lds/banks.py).  Round 4's 48-B pitch had 2-way
// conflicts on the staging stores: 29% of the <1,1> GEMM's LDS cycles (profiles/r04/pmc_gemm.txt).
constexpr int kPitchK = 32;
__device__ __forceinline__ int kimg_off(int row, int half) {
  return row * kPitchK + 16 * (half ^ ((row >> 3) & 1));
}
// [16 k][256] images: rows 16 banks apart (the tr reads of one 32-lane group take 4 k rows
// x 2 column halves)
constexpr int kPitchMN = 576;

template <int KC, int R = 256>
struct Img {  // one operand's LDS image per plane (K-contiguous: R rows; M/N-contiguous: 256)
  static constexpr int PLANE = KC ? R * kPitchK : kTK * kPitchMN;
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
  f32x4v r[IT], r2[IT];  // data slots 0 / 1 (mainloop's prefetch depth)
  unsigned mask[IT], mask2[IT];
  // M/N-contiguous operands only: element (r, k) *= kscale[k] when staged (a frozen BN's
  // scale on the conv weight's output channels, the 1x1 dgrad's K); nullptr: none
  const float* kscale = nullptr;
  int ktot = 0, kb[3] = {0, 0, 0};

  int tid0 = 0;
  __device__ int tid_of(int i) const { return tid0 + i * kNT; }  // vector index of slot i

  __device__ void init(const float* P, int R, int K, int r0, int tid) {
    rsrc = make_buffer_rsrc(P, (unsigned)R * (unsigned)K * 4u);
    ktot = K;
    tid0 = tid;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = tid + i * kNT;
      const bool slot = idx < VECS;
      if (KC) {  // vector idx: row idx/4, k segment 4 (idx & 3)
        const int row = idx >> 2, k4 = (idx & 3) * 4;
        off[i] = slot && r0 + row < R ? (r0 + row) * K + k4 : -1;
        lds[i] = slot ? kimg_off(row, k4 >> 3) + 2 * (k4 & 7) : -1;
        lim[i] = K - k4;
      } else {   // vector idx: k row idx / LPR, columns 4 (idx % LPR)
        const int kr = idx / LPR, c4 = (idx % LPR) * 4;
        off[i] = kr * R + r0 + c4;
        lds[i] = slot ? kr * kPitchMN + 2 * c4 : -1;
        lim[i] = R - (r0 + c4);
      }
    }
  }
  template <int S = 0>
  __device__ void load(int kc, int R) {
    f32x4v* rr = S ? r2 : r;
    unsigned* mm = S ? mask2 : mask;
    kb[S] = kc;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (KC) {
        rr[i] = raw_buffer_load_v4f32(rsrc, off[i] >= 0 ? (off[i] + kc) * 4 : kBufOOB, 0, 0);
        mm[i] = lt_mask4(lim[i] - kc);
      } else {  // k rows past K fall past the buffer end (zero)
        rr[i] = raw_buffer_load_v4f32(rsrc, lds[i] >= 0 ? (off[i] + kc * R) * 4 : kBufOOB, 0, 0);
        mm[i] = lt_mask4(lim[i]);
      }
    }
  }
  template <int S = 0>
  __device__ void store(unsigned char* img) const {
    const f32x4v* rr = S ? r2 : r;
    const unsigned* mm = S ? mask2 : mask;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      // (a slot check only where a lane can lack a slot: the store stays branch-free, so the
      // staging can be interleaved with the MFMAs of its basic block)
      if constexpr (VECS % kNT != 0) {
        if (lds[i] < 0) continue;
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ((mm[i] >> e) & 1) ? rr[i][e] : 0.f;
      if (!KC && kscale != nullptr) {  // uniform branch; k rows past K are zero already
        const float sc = kscale[min(kb[S] + (tid_of(i) / LPR), ktot - 1)];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= sc;
      }
      unsigned sp[3][2];
      split4<NPL>(v, sp);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        *reinterpret_cast<uint2*>(img + pl * Img<KC, RT>::PLANE + lds[i]) = make_uint2(sp[pl][0], sp[pl][1]);
    }
  }
};

// Implicit im2col of channels-last 3x3 / pad-1 maps (the ResNet RoI head's conv2, round 6):
// rows m = (r, h, w) of R maps of H x W with Cimg channels; column (tap, c), tap = 3 kh + kw,
// reads X[m + (kh - 1) W + (kw - 1)][c], 0 outside the map (its RoI's 4 x 4 bins).  The
// (R H W) x 9 Cimg matrix the head materialised (im2col3x3_nhwc, then col2im3x3_nhwc for
// its gradient) is never written.
//  * NhwcStagerK: the K-contiguous operand A(m, k = tap Cimg + c) (Cimg % 16 == 0: a 16-deep
//    chunk lies in one tap);
//  * NhwcStagerN: the N-contiguous operand B(n = tap Cimg + c, k = m) of the weight gradient
//    (Cimg % 256 == 0: a 256-wide column tile lies in one tap).
struct NhwcGeom {
  int H, W, C, rows;  // map rows x columns, channels, R H W
};
template <int NPL, int RT>
struct NhwcStagerK : Stager<1, NPL, RT> {
  using Base = Stager<1, NPL, RT>;
  int rm[Base::IT], rh[Base::IT], rw[Base::IT];  // the lane's tile rows m (-1: none), h, w
  NhwcGeom g;
  __device__ void init(const float* P, NhwcGeom g_, int r0, int tid) {
    g = g_;
    this->rsrc = make_buffer_rsrc(P, (unsigned)g.rows * (unsigned)g.C * 4u);
    this->ktot = 9 * g.C;
    this->tid0 = tid;
#pragma unroll
    for (int i = 0; i < Base::IT; ++i) {
      const int idx = tid + i * kNT;
      const bool slot = idx < Base::VECS;
      const int row = idx >> 2, k4 = (idx & 3) * 4;
      const int m = r0 + row;
      rm[i] = slot && m < g.rows ? m : -1;
      rh[i] = (m % (g.H * g.W)) / g.W;
      rw[i] = m % g.W;
      this->off[i] = k4;
      this->lds[i] = slot ? kimg_off(row, k4 >> 3) + 2 * (k4 & 7) : -1;
      this->lim[i] = 1 << 30;
    }
  }
  template <int S = 0>
  __device__ void load(int kc, int) {
    f32x4v* rr = S ? this->r2 : this->r;
    unsigned* mm = S ? this->mask2 : this->mask;
    this->kb[S] = kc;
    const int tap = kc / g.C, cc = kc - tap * g.C;
    const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < Base::IT; ++i) {
      const bool ok = rm[i] >= 0 && (unsigned)(rh[i] + dh) < (unsigned)g.H &&
                      (unsigned)(rw[i] + dw) < (unsigned)g.W && kc < 9 * g.C;
      rr[i] = raw_buffer_load_v4f32(
          this->rsrc, ok ? ((rm[i] + dh * g.W + dw) * g.C + cc + this->off[i]) * 4 : kBufOOB, 0, 0);
      mm[i] = 0xfu;
    }
  }
};
template <int NPL, int RT>
struct NhwcStagerN : Stager<0, NPL, RT> {
  using Base = Stager<0, NPL, RT>;
  int kr[Base::IT], cb[Base::IT];  // the lane's k row in the chunk (-1: none), channel
  int dh, dw;                      // the column tile's tap
  NhwcGeom g;
  __device__ void init(const float* P, NhwcGeom g_, int n0, int tid) {
    g = g_;
    this->rsrc = make_buffer_rsrc(P, (unsigned)g.rows * (unsigned)g.C * 4u);
    this->tid0 = tid;
    const int tap = n0 / g.C;
    dh = tap / 3 - 1;
    dw = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < Base::IT; ++i) {
      const int idx = tid + i * kNT;
      const bool slot = idx < Base::VECS;
      const int k = idx / Base::LPR, c4 = (idx % Base::LPR) * 4;
      kr[i] = slot ? k : -1;
      cb[i] = n0 - tap * g.C + c4;
      this->lds[i] = slot ? k * kPitchMN + 2 * c4 : -1;
      this->off[i] = 0;
      this->lim[i] = 4;
    }
  }
  template <int S = 0>
  __device__ void load(int kc, int) {
    f32x4v* rr = S ? this->r2 : this->r;
    unsigned* mm = S ? this->mask2 : this->mask;
    this->kb[S] = kc;
#pragma unroll
    for (int i = 0; i < Base::IT; ++i) {
      const int m = kc + kr[i];
      const int h = (m % (g.H * g.W)) / g.W, w = m % g.W;
      const bool ok = kr[i] >= 0 && m < g.rows && (unsigned)(h + dh) < (unsigned)g.H &&
                      (unsigned)(w + dw) < (unsigned)g.W;
      rr[i] = raw_buffer_load_v4f32(
          this->rsrc, ok ? ((m + dh * g.W + dw) * g.C + cb[i]) * 4 : kBufOOB, 0, 0);
      mm[i] = 0xfu;
    }
  }
};

// MFMA operand (8 k values of row/column `base + l32`) from one plane image.
template <int KC>
__device__ __forceinline__ u32x4 read_operand(const unsigned char* img, int base, int lane) {
  const int l32 = lane & 31, khalf = lane >> 5;
  if (KC) return *reinterpret_cast<const u32x4*>(img + kimg_off(base + l32, khalf));
  // tr reads: lane 4q+p of 16-lane group g supplies row k0+q, columns 4p..4p+3 of the
  // group's 16 columns; it receives its own column's 4 consecutive k
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int col = base + 16 * (g & 1) + 4 * p;
  const int k0 = 8 * (g >> 1) + q;
  const uint2 lo = ds_read_tr16(img + k0 * kPitchMN + 2 * col);
  const uint2 hi = ds_read_tr16(img + (k0 + 4) * kPitchMN + 2 * col);
  return u32x4{lo.x, lo.y, hi.x, hi.y};
}

// Accumulators of one wave's (MI*32) x (kNJ*32) output block: MI x kNJ tiles of 32x32.
template <int MI>
struct Acc {
  f32x16 t[MI][kNJ];
};
// element (e) of tile (a, b) of the lane: its row / column inside the wave's block
__device__ __forceinline__ int acc_row(int a, int e, int lane) {
  return a * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int b, int lane) { return b * 32 + (lane & 31); }
constexpr int kAccRegs = 16;  // registers per tile
template <int MI>
constexpr int acc_rows() { return MI; }
constexpr int kAccCols = kNJ;

// The K loop shared by the GEMM and the implicit-GEMM convolution: double-buffered LDS
// images of the two operands, the next chunk loaded to registers during the MFMAs and
// split + stored to the other buffer half way through them.
template <int AK, int BK, int NP, int MI, class SA, class SB>
__device__ __forceinline__ void mainloop(SA& sa, SB& sb, Acc<MI>& acc_, int c_begin,
                                         int c_end, unsigned char* smem, int Ra, int Rb) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  constexpr int A_PL = Img<AK, kWM * MI * 32>::PLANE, B_PL = Img<BK, kBN>::PLANE;
  constexpr int BUF = NPL * (A_PL + B_PL);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / kWN, wn = wid % kWN;
  auto& acc = acc_.t;
#pragma unroll
  for (int i = 0; i < acc_rows<MI>(); ++i)
#pragma unroll
    for (int j = 0; j < kAccCols; ++j)
#pragma unroll
      for (int r = 0; r < kAccRegs; ++r) acc[i][j][r] = 0.f;

  if constexpr (TLOD_GEMM_DEPTH2 && MI <= 2) {
    // Two chunks in flight: chunk j of the range sits in data slot j & 1 of the stagers from
    // its load until its split + store, half way through chunk j - 1's MFMAs; the store then
    // loads chunk j + 2 into the slot.  Loads and stores are unconditional (a chunk past the
    // range reads zeros / masked values into the buffer that is not read next), so the loop
    // body is straight-line and the compiler's vmcnt wait before a store leaves the other
    // slot's loads in flight (one slot loaded at the top of the iteration gave its loads
    // half an iteration).  (MI >= 3, the fc GEMMs: spills, no register room.)
    const int n = c_end - c_begin;
    sa.template load<0>(c_begin * kTK, Ra);
    sb.template load<0>(c_begin * kTK, Rb);
    sa.template load<1>((c_begin + 1) * kTK, Ra);
    sb.template load<1>((c_begin + 1) * kTK, Rb);
    sa.template store<0>(smem);
    sb.template store<0>(smem + NPL * A_PL);
    sa.template load<0>((c_begin + 2) * kTK, Ra);
    sb.template load<0>((c_begin + 2) * kTK, Rb);
    __syncthreads();
    auto iter = [&](auto slc, int j) {
      constexpr int S = decltype(slc)::value;  // slot of chunk j + 1
      const unsigned char* buf = smem + (j & 1) * BUF;
      unsigned char* nbuf = smem + ((j + 1) & 1) * BUF;
      auto mid = [&]() {
        sa.template store<S>(nbuf);
        sb.template store<S>(nbuf + NPL * A_PL);
        sa.template load<S>((c_begin + j + 3) * kTK, Ra);
        sb.template load<S>((c_begin + j + 3) * kTK, Rb);
      };
      if (TLOD_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
      u32x4 b[kNJ][3];
#pragma unroll
      for (int jj = 0; jj < kNJ; ++jj)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
          b[jj][pl] = read_operand<BK>(buf + NPL * A_PL + pl * B_PL, wn * kNJ * 32 + jj * 32, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        u32x4 a[3];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
          a[pl] = read_operand<AK>(buf + pl * A_PL, wm * MI * 32 + i * 32, lane);
#pragma unroll
        for (int jj = 0; jj < kNJ; ++jj) {
          if (i * kNJ + jj == MI * kNJ / 2) {  // half way (as in the one-slot loop below)
            __builtin_amdgcn_sched_barrier(0);
            mid();
            __builtin_amdgcn_sched_barrier(0);
          }
          bs_mac<NP>(acc[i][jj], a[0], a[1], a[2], b[jj][0], b[jj][1], b[jj][2]);
        }
      }
      if (TLOD_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
      __syncthreads();
    };
    const std::integral_constant<int, 0> S0;
    const std::integral_constant<int, 1> S1;
    for (int j = 0; j < n; j += 2) {
      iter(S1, j);  // chunk j from buffer 0; chunk j + 1 (slot 1) -> buffer 1
      if (j + 1 >= n) break;
      iter(S0, j + 1);  // chunk j + 1 from buffer 1; chunk j + 2 (slot 0) -> buffer 0
    }
    return;
  }
  // One data slot (MI >= 3: no register room for a second): chunk c + 1 is split + stored
  // half way through chunk c's MFMAs and the slot is reloaded with chunk c + 2 right after,
  // so every chunk's loads have a whole chunk of MFMAs to land (loaded at the top of the
  // chunk they had half of one: the stores waited on them, fc6 forward +19%).
  auto store = [&](unsigned char* buf) {
    sa.store(buf);
    sb.store(buf + NPL * A_PL);
  };
  if (c_begin < c_end) {
    sa.load(c_begin * kTK, Ra);
    sb.load(c_begin * kTK, Rb);
    store(smem);
    if (c_begin + 1 < c_end) {
      sa.load((c_begin + 1) * kTK, Ra);
      sb.load((c_begin + 1) * kTK, Rb);
    }
  }
  __syncthreads();
  for (int c = c_begin; c < c_end; ++c) {
    const int it = c - c_begin;
    const unsigned char* buf = smem + (it & 1) * BUF;
    // (unconditional: past the range the loads read zeros — raw buffer range checks and the
    // K masks — into the buffer nobody reads next, and the loop body stays one basic block)
    auto mid = [&]() {
      store(smem + ((it + 1) & 1) * BUF);
      sa.load((c + 2) * kTK, Ra);
      sb.load((c + 2) * kTK, Rb);
    };
    if (TLOD_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
    u32x4 b[kNJ][3];
#pragma unroll
    for (int j = 0; j < kNJ; ++j)
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        b[j][pl] = read_operand<BK>(buf + NPL * A_PL + pl * B_PL, wn * kNJ * 32 + j * 32, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      u32x4 a[3];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        a[pl] = read_operand<AK>(buf + pl * A_PL, wm * MI * 32 + i * 32, lane);
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        if (i * kNJ + j == MI * kNJ / 2) {
          // kept half way through the MFMAs: the compiler otherwise sinks the split + stores
          // (and their vmcnt wait) below every MFMA, where the two waves of a SIMD split
          // together while the matrix pipe idles
          __builtin_amdgcn_sched_barrier(0);
          mid();
          __builtin_amdgcn_sched_barrier(0);
        }
        bs_mac<NP>(acc[i][j], a[0], a[1], a[2], b[j][0], b[j][1], b[j][2]);
      }
    }
    if (TLOD_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  }
}

// IM: 0 = plain operands; 1 = A is the implicit channels-last 3x3 im2col of geo's maps
// (NhwcStagerK); 2 = B is (NhwcStagerN)
template <int AK, int BK, int NP, int MI, int IM = 0>
__global__ void __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm_bs_kernel(const float* __restrict__ A, const float* __restrict__ B,
               const float* __restrict__ bias, const float* __restrict__ res, int relu,
               const float* __restrict__ mask, float* __restrict__ C, float* __restrict__ slab, int M, int N, int K, int tiles_m,
               int tiles_n, int dp_tiles, int ksplit, int chunks_per_split, NhwcGeom geo) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  constexpr int BM = kWM * MI * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // whole tiles first, then the tail tiles split over K (plan_tail)
  const int n_tail = tiles_m * tiles_n - dp_tiles;
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
  const int mt = t % tiles_m;
  const int nt = t / tiles_m;
  const int m0 = mt * BM, n0 = nt * kBN;
  const int nchunks = (K + kTK - 1) / kTK;
  const int c_begin = direct ? 0 : split * chunks_per_split;
  const int c_end = direct ? nchunks : min(nchunks, c_begin + chunks_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / kWN, wn = wid % kWN;

  Acc<MI> acc_;
  if constexpr (IM == 1) {
    NhwcStagerK<NPL, BM> sa;
    Stager<BK, NPL, kBN> sb;
    sa.init(A, geo, m0, tid);
    sb.init(B, N, K, n0, tid);
    mainloop<AK, BK, NP, MI>(sa, sb, acc_, c_begin, c_end, smem, M, N);
  } else if constexpr (IM == 2) {
    Stager<AK, NPL, BM> sa;
    NhwcStagerN<NPL, kBN> sb;
    sa.init(A, M, K, m0, tid);
    sb.init(B, geo, n0, tid);
    mainloop<AK, BK, NP, MI>(sa, sb, acc_, c_begin, c_end, smem, M, N);
  } else {
    Stager<AK, NPL, BM> sa;
    Stager<BK, NPL, kBN> sb;
    sa.init(A, M, K, m0, tid);
    sb.init(B, N, K, n0, tid);
    mainloop<AK, BK, NP, MI>(sa, sb, acc_, c_begin, c_end, smem, M, N);
  }
  auto& acc = acc_.t;

  // direct tiles: C = act(acc + bias + res); tail pieces: tile-local slab (the epilogue is
  // the reduce's)
  if (!direct) {
    float* St = slab + ((size_t)split * n_tail + ti) * BM * kBN;
#pragma unroll
    for (int j = 0; j < kAccCols; ++j) {
      const int nl = wn * kNJ * 32 + acc_col(j, lane);
#pragma unroll
      for (int i = 0; i < acc_rows<MI>(); ++i)
#pragma unroll
        for (int r = 0; r < kAccRegs; ++r)
          St[(wm * MI * 32 + acc_row(i, r, lane)) * kBN + nl] = acc[i][j][r];
    }
    return;
  }
  if ((size_t)(M + BM) * N * 4 < (1ull << 31)) {
    // Branch-free (the conv epilogues' form, round 6): 32-bit byte offsets into C through a
    // buffer resource; a row past M lies past the range (dropped store, zero load) and a
    // column past N takes kBufOOB, so no element needs a bounds branch or a 64-bit address.
    // Residual / mask operands of a 32-row block are loaded together ahead of its stores.
    const unsigned bytes = (unsigned)M * (unsigned)N * 4u;
    const i32x4 c_rsrc = make_buffer_rsrc(C, bytes);
    const i32x4 r_rsrc = make_buffer_rsrc(res ? res : C, res ? bytes : 0u);
    const i32x4 k_rsrc = make_buffer_rsrc(mask ? mask : C, mask ? bytes : 0u);
#pragma unroll
    for (int j = 0; j < kAccCols; ++j) {
      const int n = n0 + wn * kNJ * 32 + acc_col(j, lane);
      const float bv = bias != nullptr && n < N ? bias[n] : 0.f;
      const int noff = n < N ? n * 4 : kBufOOB;
#pragma unroll
      for (int i = 0; i < acc_rows<MI>(); ++i) {
        int off[kAccRegs];
#pragma unroll
        for (int r = 0; r < kAccRegs; ++r) {
          const int m = m0 + wm * MI * 32 + acc_row(i, r, lane);
          off[r] = noff == kBufOOB ? kBufOOB : m * N * 4 + noff;
        }
        float ext[kAccRegs], mk[kAccRegs];
        if (res != nullptr || mask != nullptr) {
#pragma unroll
          for (int r = 0; r < kAccRegs; ++r) {
            ext[r] = res != nullptr ? raw_buffer_load_f32(r_rsrc, off[r], 0, 0) : 0.f;
            mk[r] = mask != nullptr ? raw_buffer_load_f32(k_rsrc, off[r], 0, 0) : 1.f;
          }
        }
#pragma unroll
        for (int r = 0; r < kAccRegs; ++r) {
          float v = acc[i][j][r] + bv;
          if (res != nullptr) v += ext[r];
          if (relu) v = fmaxf(v, 0.f);
          if (mask != nullptr) v = mk[r] > 0.f ? v : 0.f;
          raw_buffer_store_f32(v, c_rsrc, off[r], 0, 0);
        }
      }
    }
    return;
  }
  if (res == nullptr && !relu && mask == nullptr) {  // (plain: a short-K tile's cost is in it)
#pragma unroll
    for (int j = 0; j < kAccCols; ++j) {
      const int n = n0 + wn * kNJ * 32 + acc_col(j, lane);
      const float bv = bias != nullptr && n < N ? bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < acc_rows<MI>(); ++i)
#pragma unroll
        for (int r = 0; r < kAccRegs; ++r) {
          const int m = m0 + wm * MI * 32 + acc_row(i, r, lane);
          if (m < M && n < N) C[(size_t)m * N + n] = acc[i][j][r] + bv;
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < kAccCols; ++j) {
    const int n = n0 + wn * kNJ * 32 + acc_col(j, lane);
    const float bv = bias != nullptr && n < N ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < acc_rows<MI>(); ++i) {
      // a block's residuals and mask values loaded together, ahead of its stores (one
      // latency, not one per element)
      float ext[kAccRegs], mk[kAccRegs];
#pragma unroll
      for (int r = 0; r < kAccRegs; ++r) {
        const int m = m0 + wm * MI * 32 + acc_row(i, r, lane);
        const bool in = m < M && n < N;
        ext[r] = res != nullptr && in ? res[(size_t)m * N + n] : 0.f;
        mk[r] = mask != nullptr && in ? mask[(size_t)m * N + n] : 1.f;
      }
#pragma unroll
      for (int r = 0; r < kAccRegs; ++r) {
        const int m = m0 + wm * MI * 32 + acc_row(i, r, lane);
        float v = acc[i][j][r] + bv;
        if (res != nullptr) v += ext[r];
        if (relu) v = fmaxf(v, 0.f);
        if (mask != nullptr) v = mk[r] > 0.f ? v : 0.f;
        if (m < M && n < N) C[(size_t)m * N + n] = v;
      }
    }
  }
}

// Tail tiles: C[m][n] = sum_s slab[s][tile][m][n] (+ bias[n]), fixed split order.  One
// workgroup per (tail tile, 1024 elements).
__global__ void __launch_bounds__(256) gemm_tail_reduce_kernel(
    const float* __restrict__ slab, int ksplit, int n_tail, int dp_tiles, int bm, int tiles_m,
    int M, int N, const float* __restrict__ bias, const float* __restrict__ res, int relu,
    const float* __restrict__ mask, float* __restrict__ C) {
  // a thread takes 4 consecutive slab elements of one row (16-B loads per split piece; one
  // 16-B store when the row is 16-B aligned in C)
  const int tile_elems = bm * kBN;
  const int per_tile = tile_elems / 1024;
  const int ti = blockIdx.x / per_tile;
  const int t = dp_tiles + ti;
  const int mt = t % tiles_m, nt = t / tiles_m;
  const size_t stride = (size_t)n_tail * tile_elems;
  const float* S = slab + (size_t)ti * tile_elems;
  const int e = (blockIdx.x % per_tile) * 1024 + 4 * threadIdx.x;
  const int m = mt * bm + e / kBN, n = nt * kBN + e % kBN;
  if (m >= M || n >= N) return;
  float4 v = *reinterpret_cast<const float4*>(S + e);
#pragma unroll 4  // four split loads in flight, the adds in split order
  for (int k = 1; k < ksplit; ++k) {
    const float4 u = *reinterpret_cast<const float4*>(S + k * stride + e);
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  float* c = C + (size_t)m * N + n;
  if (bias) {
    v.x += bias[n];
    if (n + 1 < N) v.y += bias[n + 1];
    if (n + 2 < N) v.z += bias[n + 2];
    if (n + 3 < N) v.w += bias[n + 3];
  }
  if (res) {
    const float* rr = res + (size_t)m * N + n;
    v.x += rr[0];
    if (n + 1 < N) v.y += rr[1];
    if (n + 2 < N) v.z += rr[2];
    if (n + 3 < N) v.w += rr[3];
  }
  if (relu) {
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
  }
  if (mask) {
    const float* mm = mask + (size_t)m * N + n;
    if (!(mm[0] > 0.f)) v.x = 0.f;
    if (n + 1 < N && !(mm[1] > 0.f)) v.y = 0.f;
    if (n + 2 < N && !(mm[2] > 0.f)) v.z = 0.f;
    if (n + 3 < N && !(mm[3] > 0.f)) v.w = 0.f;
  }
  if (n + 3 < N && ((reinterpret_cast<uintptr_t>(c) & 15) == 0)) {
    *reinterpret_cast<float4*>(c) = v;
  } else {
    c[0] = v.x;
    if (n + 1 < N) c[1] = v.y;
    if (n + 2 < N) c[2] = v.z;
    if (n + 3 < N) c[3] = v.w;
  }
}

// resident workgroups of a kernel chip-wide, cached per kernel (the instantiations share one
// function-pointer type, so a per-type static would mix kernels of different occupancy)
template <typename K>
int slots_of(K kern, size_t lds) {
  return cached_slots((const void*)kern, kNT, lds);
}

struct TailPlan {
  int dp_tiles, ksplit, cps;
};

// Whole rounds of tiles over the full K, the last partial round split over K when that
// beats running it as a mostly idle round (cost model: tile time at the slot rate, the
// slab round trip at 4 TB/s, 6 us per reduce launch).
#ifndef TLOD_SPLIT_BW  // slab bytes per second the split-K cost model assumes (A/B knob)
#define TLOD_SPLIT_BW 4e12
#endif
TailPlan plan_tail(int T, int nchunks, int slots, double tile_s, double tile_bytes) {
  TailPlan p{T, 1, nchunks};
  double best = (double)((T + slots - 1) / slots) * tile_s;
  const int q = T / slots;
  for (int k = 2; k <= std::min(16, nchunks / 2); ++k) {
    const int cps = div_up(nchunks, k);
    const int kk = div_up(nchunks, cps);
    for (int dp : {q * slots, 0}) {
      const int tail = T - dp;
      if (tail <= 0) continue;
      const double t = (double)dp / slots * tile_s +
                       (double)(((long long)tail * kk + slots - 1) / slots) * tile_s * cps / nchunks +
                       (2.0 * kk + 1.0) * tail * tile_bytes / TLOD_SPLIT_BW + 6e-6;
      if (t < best * 0.97) {
        best = t;
        p = TailPlan{dp, kk, cps};
      }
    }
  }
  return p;
}

template <int AK, int BK, int NP, int MI, int IM = 0>
struct Gemm {
  static constexpr int NPL = NP == 6 ? 3 : 2;
  static constexpr int kBM = kWM * MI * 32;
  static constexpr size_t kLds = 2 * NPL * (Img<AK, kBM>::PLANE + Img<BK>::PLANE);
  static TailPlan plan(int M, int N, int K) {
    const int slots = slots_of(gemm_bs_kernel<AK, BK, NP, MI, IM>, kLds);
    const int tiles = div_up(M, kBM) * div_up(N, kBN);
    const int nchunks = div_up(K, kTK);
    // bf16 MFMA time of one whole tile per resident slot at ~50% of the dense peak
    const double tile_s = 2.0 * kBM * kBN * kTK * NP * nchunks / (2516.6e12 * 0.5 / slots);
    return plan_tail(tiles, nchunks, slots, tile_s, 4.0 * kBM * kBN);
  }
  static size_t ws_bytes(int M, int N, int K) {
    const TailPlan p = plan(M, N, K);
    const int tiles = div_up(M, kBM) * div_up(N, kBN);
    return p.ksplit > 1 ? (size_t)p.ksplit * (tiles - p.dp_tiles) * kBM * kBN * sizeof(float) : 0;
  }
  static int run(const float* A, const float* B, const float* bias, float* C, int M, int N, int K,
                 float* ws, size_t ws_bytes_, hipStream_t s, const float* res = nullptr,
                 int relu = 0, const float* mask = nullptr, NhwcGeom geo = NhwcGeom{0, 0, 0, 0}) {
    const TailPlan p = plan(M, N, K);
    if (ws_bytes_ < ws_bytes(M, N, K)) {
      set_error("tlod_gemm_bs_f32: workspace too small");
      return kWorkspace;
    }
    const int tiles_m = div_up(M, kBM), tiles_n = div_up(N, kBN);
    const int n_tail = tiles_m * tiles_n - p.dp_tiles;
    auto kern = gemm_bs_kernel<AK, BK, NP, MI, IM>;
    TLOD_HIP(lds_attr((const void*)kern, (int)kLds));
    const int nwg = p.dp_tiles + (p.ksplit > 1 ? n_tail * p.ksplit : 0);
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(kNT), kLds, s, A, B, bias, res, relu, mask, C, ws, M,
                       N, K, tiles_m, tiles_n, p.dp_tiles, p.ksplit, p.cps, geo);
    TLOD_LAUNCH_CHECK();
    if (p.ksplit > 1) {
      hipLaunchKernelGGL(gemm_tail_reduce_kernel, dim3(n_tail * (kBM * kBN / 1024)), dim3(256), 0,
                         s, ws, p.ksplit, n_tail, p.dp_tiles, kBM, tiles_m, M, N, bias, res, relu,
                         mask, C);
      TLOD_LAUNCH_CHECK();
    }
    return kOk;
  }
};

#ifndef TLOD_GEMM_SMALL_MI  // A/B knob: 64- / 128-row tiles (1 / 2) for GEMMs of < 64 tiles
#define TLOD_GEMM_SMALL_MI 0
#endif
template <typename F>
auto with_gemm(int M, int ak, int bk, int nprod, F&& f, int N = 0) {
  // M tile 192 when it pads M less (the 556 RoI rows of the head: 576 vs 768)
  const bool m192 = div_up(M, 192) * 192 < div_up(M, 256) * 256;
  const bool small = TLOD_GEMM_SMALL_MI && N > 0 && nprod == 6 &&
                     div_up(M, m192 ? 192 : 256) * div_up(N, kBN) < 64;
#define TLOD_GEMM_CASE(A_, B_)                                                 \
  if (ak == A_ && bk == B_) {                                                  \
    if (small) return f(Gemm<A_, B_, 6, TLOD_GEMM_SMALL_MI ? TLOD_GEMM_SMALL_MI : 3>{}); \
    if (m192) return nprod == 6 ? f(Gemm<A_, B_, 6, 3>{}) : f(Gemm<A_, B_, 3, 3>{}); \
    return nprod == 6 ? f(Gemm<A_, B_, 6, 4>{}) : f(Gemm<A_, B_, 3, 4>{});     \
  }
  TLOD_GEMM_CASE(1, 1)
  TLOD_GEMM_CASE(1, 0)
  TLOD_GEMM_CASE(0, 0)
#undef TLOD_GEMM_CASE
  // (0, 1): the callers pass 0/1 flags, so the four cases are exhaustive
  if (small) return f(Gemm<0, 1, 6, TLOD_GEMM_SMALL_MI ? TLOD_GEMM_SMALL_MI : 3>{});
  if (m192) return nprod == 6 ? f(Gemm<0, 1, 6, 3>{}) : f(Gemm<0, 1, 3, 3>{});
  return nprod == 6 ? f(Gemm<0, 1, 6, 4>{}) : f(Gemm<0, 1, 3, 4>{});
}

// The channels-last 3x3 GEMM of a mode (tlod_gemm_nhwc3_bs_f32): 0 forward (A implicit,
// B the (O, 9C) weight rows), 1 input gradient (A implicit over dY's O channels, B the
// (9 O, C) tap-flipped weight), 2 weight gradient (A = dY^T, B implicit); the M tile as
// with_gemm.
template <typename F>
auto with_nhwc3(int mode, int M, int nprod, F&& f) {
  const bool m192 = div_up(M, 192) * 192 < div_up(M, 256) * 256;
#define TLOD_NHWC3_CASE(A_, B_, IM_)                                                      \
  if (m192) return nprod == 6 ? f(Gemm<A_, B_, 6, 3, IM_>{}) : f(Gemm<A_, B_, 3, 3, IM_>{}); \
  return nprod == 6 ? f(Gemm<A_, B_, 6, 4, IM_>{}) : f(Gemm<A_, B_, 3, 4, IM_>{});
  if (mode == 0) { TLOD_NHWC3_CASE(1, 1, 1) }
  if (mode == 1) { TLOD_NHWC3_CASE(1, 0, 1) }
  TLOD_NHWC3_CASE(0, 0, 2)
#undef TLOD_NHWC3_CASE
}

struct Nhwc3Shape {
  int M, N, K;
  NhwcGeom geo;
};
// GEMM extents and the implicit operand's geometry of a mode (see tlod.h)
static Nhwc3Shape nhwc3_shape(int mode, int R, int H, int W, int C, int O) {
  const int rows = R * H * W;
  if (mode == 0) return {rows, O, 9 * C, NhwcGeom{H, W, C, rows}};
  if (mode == 1) return {rows, C, 9 * O, NhwcGeom{H, W, O, rows}};
  return {O, 9 * C, rows, NhwcGeom{H, W, C, rows}};
}

// ---------------------------------------------------------------- 3x3 conv as GEMM
// Implicit GEMM for the stride-1 "same" 3x3 convolution with >= 256 output channels:
//   Y[img][m][p] = act(scale[m] * sum_k A(m,k) B(p,k) + bias[m] + residual[img][m][p])
// K = C*9 over (c, tap), B(p, (c,tap)) = X[img][c][p + (tap/3-1)*W + tap%3-1] when the tap
// lies inside the map, else 0 (the im2col row, gathered straight from NCHW with one
// buffer_load_dwordx4 per 4 pixels and a bit-range in-map mask; staged [16 k][256 px] and
// read transposed like the GEMM's N-contiguous operand).  A = the weights as
// [Cout][C*9] (forward: nn.Conv2d's own layout, AK = 1) or tlod_conv_pack_dgrad_f32's
// [(co, tap)][ci] (dgrad: the transposed, flipped kernel, AK = 0).
struct ConvEpi {
  const float* scale;
  const float* bias;
  const float* residual;
  int relu;
  const float* mask = nullptr;  // y *= (mask > 0) last: a dgrad's previous-layer ReLU backward
  const float* wscale = nullptr;  // 1x1 dgrad (w_layout 1): W[co][ci] * wscale[co] as staged
};

template <int NPL>
struct Im2colStager {
  static constexpr int IT = 2;  // 16 k rows x 256 pixels / 512 lanes / 4
  i32x4 rsrc;
  int xoff, kr, p, c4, h0, w0, C, H, W, P, K;
  bool neg_risk;
  unsigned tmask;
  f32x4v r[IT], r2[IT];  // data slots 0 / 1
  unsigned mask[IT], mask2[IT];

  __device__ void init(const float* X, int N, int C_, int H_, int W_, int img, int p0, int tid) {
    C = C_; H = H_; W = W_; P = H * W; K = C * 9;
    rsrc = make_buffer_rsrc(X, (unsigned)N * (unsigned)C * (unsigned)P * 4u);
    xoff = img * C * P;
    kr = tid >> 6;
    c4 = (tid & 63) * 4;
    p = p0 + c4;
    const int pc = min(p, P - 1);
    h0 = pc / W;
    w0 = pc - h0 * W;
    tmask = lt_mask4(P - p);
    // a tap vector can start before the tensor only in image 0's first row band
    neg_risk = img == 0 && p0 <= W;
  }
  template <int S = 0>
  __device__ void load(int kc, int) {
    f32x4v* r = S ? this->r2 : this->r;
    unsigned* mask = S ? this->mask2 : this->mask;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int k = kc + kr + 8 * i;
      const int c = k / 9, t = k - 9 * c;
      const int dh = t / 3 - 1, dw = t - 3 * (t / 3) - 1;
      const int o = xoff + c * P + dh * W + dw + p;
      unsigned m;
      if (W >= 4) {  // (h0, w0 + e) for e < ew, then (h0 + 1, e - ew): one wrap at most
        const int ew = W - w0;
        const bool r0 = (unsigned)(h0 + dh) < (unsigned)H;
        const bool r1 = (unsigned)(h0 + 1 + dh) < (unsigned)H;
        const unsigned m0v = lt_mask4(ew - max(dw, 0)) & ~lt_mask4(-w0 - dw);
        const unsigned m1v = 0xfu & ~lt_mask4(ew + max(-dw, 0));
        m = (r0 ? m0v : 0u) | (r1 ? m1v : 0u);
      } else {
        m = 0;
        int h = h0, w = w0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          m |= (unsigned)((unsigned)(h + dh) < (unsigned)H && (unsigned)(w + dw) < (unsigned)W) << e;
          if (++w == W) { w = 0; ++h; }
        }
      }
      mask[i] = k < K ? m & tmask : 0u;
      if (neg_risk && kc < 9) {
        // per-dword: negative element offsets read out of range (0); the select keeps the
        // backend from merging the four loads into one dwordx4 at the negative start
#pragma unroll
        for (int e = 0; e < 4; ++e)
          r[i][e] = raw_buffer_load_f32(rsrc, o + e >= 0 ? (o + e) * 4 : kBufOOB, 0, 0);
      } else {
        r[i] = raw_buffer_load_v4f32(rsrc, k < K ? o * 4 : kBufOOB, 0, 0);
      }
    }
  }
  template <int S = 0>
  __device__ void store(unsigned char* img) const {
    const f32x4v* r = S ? this->r2 : this->r;
    const unsigned* mask = S ? this->mask2 : this->mask;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ((mask[i] >> e) & 1) ? r[i][e] : 0.f;
      unsigned sp[3][2];
      split4<NPL>(v, sp);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        *reinterpret_cast<uint2*>(img + pl * Img<0>::PLANE + (kr + 8 * i) * kPitchMN + 2 * c4) =
            make_uint2(sp[pl][0], sp[pl][1]);
    }
  }
};

// Schedule: the first dp_tiles tiles (whole rounds of the resident slots) run over the full
// K; the remaining tail tiles, which would leave most of the chip idle in a last partial
// round, are split over K into ksplit pieces written to fixed slabs and reduced in order.
// MI = 1 (64-row tiles, 74 KB of LDS since the K-contiguous image is sized by the tile rows):
// two workgroups per CU when the registers fit 128 (TLOD_CONV1X1_OCC2=1)
#ifndef TLOD_CONV1X1_OCC2
#define TLOD_CONV1X1_OCC2 1
#endif
template <int AK, int NP, int MI, int KS>
__global__ void __launch_bounds__(kNT)
    __attribute__((amdgpu_waves_per_eu(TLOD_CONV1X1_OCC2 && MI == 1 && AK == 1 ? 4 : 2,
                                       TLOD_CONV1X1_OCC2 && MI == 1 && AK == 1 ? 4 : 2)))
conv_gemm_bs_kernel(const float* __restrict__ X, const float* __restrict__ Wt, ConvEpi epi,
                    float* __restrict__ Y, float* __restrict__ slab, int N, int C, int H, int W,
                    int Cout, int tiles_m, int tiles_n, int dp_tiles, int ksplit,
                    int chunks_per_split) {
  constexpr int NPL = NP == 6 ? 3 : 2;
  constexpr int BM = kWM * MI * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int P = H * W, K = C * KS * KS;
  const int n_tiles = tiles_m * tiles_n * N;
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
  const int nt = t % tiles_n; t /= tiles_n;
  const int img = t;
  const int m0 = mt * BM, p0 = nt * kBN;
  const int nchunks = (K + kTK - 1) / kTK;
  const int c_begin = direct ? 0 : split * chunks_per_split;
  const int c_end = direct ? nchunks : min(nchunks, c_begin + chunks_per_split);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / kWN, wn = wid % kWN;

  Stager<AK, NPL, BM> sa;
  sa.init(Wt, Cout, K, m0, tid);
  Acc<MI> acc_;
  if constexpr (KS == 3) {
    Im2colStager<NPL> sb;
    sb.init(X, N, C, H, W, img, p0, tid);
    mainloop<AK, 0, NP, MI>(sa, sb, acc_, c_begin, c_end, smem, Cout, 0);
  } else {  // 1x1: B(p, c) = X[img][c][p], the image's map as an N-contiguous operand
    if constexpr (AK == 0) sa.kscale = epi.wscale;
    Stager<0, NPL, kBN> sb;
    sb.init(X + (size_t)img * C * P, P, C, p0, tid);
    mainloop<AK, 0, NP, MI>(sa, sb, acc_, c_begin, c_end, smem, Cout, P);
  }
  auto& acc = acc_.t;

  const size_t ybase = (size_t)img * Cout * P;
  const int nl0 = wn * kNJ * 32;
  if (!direct) {  // tile-local slab, reduced by conv_tail_reduce_kernel
    float* St = slab + ((size_t)split * n_tail + ti) * BM * kBN;
#pragma unroll
    for (int i = 0; i < acc_rows<MI>(); ++i)
#pragma unroll
      for (int r = 0; r < kAccRegs; ++r)
#pragma unroll
        for (int j = 0; j < kAccCols; ++j)
          St[(wm * MI * 32 + acc_row(i, r, lane)) * kBN + nl0 + acc_col(j, lane)] = acc[i][j][r];
    return;
  }
  // Direct epilogue, branch-free: elements outside the map / Cout get an out-of-range buffer
  // offset (their residual loads read 0, their stores are dropped).  The residual operands
  // of one accumulator row block are loaded together ahead of its stores — loaded one by one
  // between the stores, every load paid a full memory latency (256 -> 1024 at 38x75 with a
  // residual: 67 us per launch).
  const i32x4 y_rsrc = make_buffer_rsrc(Y + ybase, (unsigned)Cout * (unsigned)P * 4u);
  const i32x4 r_rsrc = make_buffer_rsrc(epi.residual ? epi.residual + ybase : Y + ybase,
                                        epi.residual ? (unsigned)Cout * (unsigned)P * 4u : 0u);
  const i32x4 k_rsrc = make_buffer_rsrc(epi.mask ? epi.mask + ybase : Y + ybase,
                                        epi.mask ? (unsigned)Cout * (unsigned)P * 4u : 0u);
  int pix4[kAccCols];
#pragma unroll
  for (int j = 0; j < kAccCols; ++j) {
    const int pix = p0 + nl0 + acc_col(j, lane);
    pix4[j] = pix < P ? pix * 4 : kBufOOB;
  }
#pragma unroll
  for (int i = 0; i < acc_rows<MI>(); ++i) {
    float res[kAccRegs][kAccCols], msk[kAccRegs][kAccCols];
    if (epi.residual || epi.mask) {
#pragma unroll
      for (int r = 0; r < kAccRegs; ++r) {
        const int co = m0 + wm * MI * 32 + acc_row(i, r, lane);
#pragma unroll
        for (int j = 0; j < kAccCols; ++j) {
          const int o = co < Cout && pix4[j] != kBufOOB ? co * P * 4 + pix4[j] : kBufOOB;
          res[r][j] = epi.residual ? raw_buffer_load_f32(r_rsrc, o, 0, 0) : 0.f;
          msk[r][j] = epi.mask ? raw_buffer_load_f32(k_rsrc, o, 0, 0) : 1.f;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kAccRegs; ++r) {
      const int co = m0 + wm * MI * 32 + acc_row(i, r, lane);
      const int cc = min(co, Cout - 1);
      const float sc = epi.scale ? epi.scale[cc] : 1.f, bi = epi.bias ? epi.bias[cc] : 0.f;
#pragma unroll
      for (int j = 0; j < kAccCols; ++j) {
        float v = acc[i][j][r];
        if (epi.scale) v *= sc;
        v += bi;
        if (epi.residual) v += res[r][j];
        if (epi.relu) v = fmaxf(v, 0.f);
        if (epi.mask) v = msk[r][j] > 0.f ? v : 0.f;
        raw_buffer_store_f32(v, y_rsrc, co < Cout && pix4[j] != kBufOOB ? co * P * 4 + pix4[j] : kBufOOB, 0, 0);
      }
    }
  }
}

// Tail tiles: Y = act(sum_s slab[s][tile] * scale + bias + residual), fixed split order.
// One workgroup per (tail tile, 1024 elements); a thread takes 4 consecutive pixels of one
// channel (16-B loads per split piece, four pieces in flight).
__global__ void __launch_bounds__(256) conv_tail_reduce_kernel(
    const float* __restrict__ slab, int ksplit, int n_tail, int dp_tiles, int bm, int tiles_m,
    int tiles_n, int Cout, int P, ConvEpi epi, float* __restrict__ Y) {
  const int tile_elems = bm * kBN;
  const int per_tile = tile_elems / 1024;
  const int ti = blockIdx.x / per_tile;
  int t = dp_tiles + ti;
  const int mt = t % tiles_m; t /= tiles_m;
  const int nt = t % tiles_n;
  const int img = t / tiles_n;
  const size_t stride = (size_t)n_tail * tile_elems;
  const float* S = slab + (size_t)ti * tile_elems;
  const int e = (blockIdx.x % per_tile) * 1024 + 4 * threadIdx.x;
  const int co = mt * bm + e / kBN, p0 = nt * kBN + e % kBN;
  if (co >= Cout || p0 >= P) return;
  float4 v = *reinterpret_cast<const float4*>(S + e);
#pragma unroll 4
  for (int k = 1; k < ksplit; ++k) {
    const float4 u = *reinterpret_cast<const float4*>(S + k * stride + e);
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  const float vv[4] = {v.x, v.y, v.z, v.w};
  const float sc = epi.scale ? epi.scale[co] : 1.f, bi = epi.bias ? epi.bias[co] : 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = p0 + q;
    if (p >= P) break;
    const size_t idx = ((size_t)img * Cout + co) * P + p;
    float x = vv[q];
    if (epi.scale) x *= sc;
    if (epi.bias) x += bi;
    if (epi.residual) x += epi.residual[idx];
    if (epi.relu) x = fmaxf(x, 0.f);
    if (epi.mask) x = epi.mask[idx] > 0.f ? x : 0.f;
    Y[idx] = x;
  }
}


template <int AK, int NP, int MI, int KS = 3>
struct ConvGemm {
  static constexpr int NPL = NP == 6 ? 3 : 2;
  static constexpr int kBM = kWM * MI * 32;
  static constexpr size_t kLds = 2 * NPL * (Img<AK, kBM>::PLANE + Img<0>::PLANE);
  static TailPlan plan(int N, int C, int H, int W, int Cout) {
    const int slots = slots_of(conv_gemm_bs_kernel<AK, NP, MI, KS>, kLds);
    const int tiles = div_up(Cout, kBM) * div_up(H * W, kBN) * N;
    const int nchunks = div_up(C * KS * KS, kTK);
    // bf16 MFMA time of one whole tile per resident slot at ~50% of the dense peak
    const double tile_s = 2.0 * kBM * kBN * kTK * NP * nchunks / (2516.6e12 * 0.5 / slots);
    return plan_tail(tiles, nchunks, slots, tile_s, 4.0 * kBM * kBN);
  }
  static size_t ws_bytes(int N, int C, int H, int W, int Cout) {
    const TailPlan p = plan(N, C, H, W, Cout);
    const int tiles = div_up(Cout, kBM) * div_up(H * W, kBN) * N;
    return p.ksplit > 1 ? (size_t)p.ksplit * (tiles - p.dp_tiles) * kBM * kBN * sizeof(float) : 0;
  }
  static int run(const float* X, const float* Wt, ConvEpi epi, float* Y, int N, int C, int H,
                 int W, int Cout, float* ws, size_t ws_bytes_, hipStream_t s) {
    const TailPlan p = plan(N, C, H, W, Cout);
    if (ws_bytes_ < ws_bytes(N, C, H, W, Cout)) {
      set_error("tlod_conv3x3_gemm_bs_f32: workspace too small");
      return kWorkspace;
    }
    const int tiles_m = div_up(Cout, kBM), tiles_n = div_up(H * W, kBN);
    const int n_tail = tiles_m * tiles_n * N - p.dp_tiles;
    auto kern = conv_gemm_bs_kernel<AK, NP, MI, KS>;
    TLOD_HIP(lds_attr((const void*)kern, (int)kLds));
    const int nwg = p.dp_tiles + (p.ksplit > 1 ? n_tail * p.ksplit : 0);
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(kNT), kLds, s, X, Wt, epi, Y, ws, N, C, H, W, Cout,
                       tiles_m, tiles_n, p.dp_tiles, p.ksplit, p.cps);
    TLOD_LAUNCH_CHECK();
    if (p.ksplit > 1) {
      hipLaunchKernelGGL(conv_tail_reduce_kernel, dim3(n_tail * (kBM * kBN / 1024)), dim3(256), 0, s,
                         ws, p.ksplit, n_tail, p.dp_tiles, kBM, tiles_m, tiles_n, Cout, H * W, epi, Y);
      TLOD_LAUNCH_CHECK();
    }
    return kOk;
  }
};

template <typename F>
auto with_conv_gemm(int w_layout, int nprod, F&& f) {
  if (w_layout == 0) return nprod == 6 ? f(ConvGemm<1, 6, 4>{}) : f(ConvGemm<1, 3, 4>{});
  return nprod == 6 ? f(ConvGemm<0, 6, 4>{}) : f(ConvGemm<0, 3, 4>{});
}

// 1x1: the M tile (output channels) is 64, 128 or 256 rows (MI = 1, 2, 4), whichever runs
// the grid in the least time by a rounds x tile-rows / efficiency model (256 resident
// slots; a 256-row tile reuses each staged pixel 4x as often as a 64-row one: relative
// efficiency 1 / 0.8 / 0.55) — the bottleneck's 1x1 convs have 64..2048 output channels on
// maps of 38x75..150x300, so e.g. 256 -> 1024 at 38x75 takes 128-row tiles (192 tiles, not
// 96).
#ifndef TLOD_1X1_MI  // 0: the model below; 1 / 2 / 4 forced (A/B knob)
#define TLOD_1X1_MI 0
#endif
static int conv1x1_mi(int N, int H, int W, int Cout) {
  if (TLOD_1X1_MI) return TLOD_1X1_MI;
  const long long pt = (long long)div_up(H * W, kBN) * N;
  int best = 4;
  double best_c = 1e30;
  for (int mi : {4, 2, 1}) {
    const int bm = kWM * mi * 32;
    const long long tiles = div_up(Cout, bm) * pt;
    const double eff = mi == 4 ? 1.0 : mi == 2 ? 0.8 : 0.55;
    const double c = (double)((tiles + 255) / 256) * bm / eff;
    if (c < best_c * 0.999) {
      best_c = c;
      best = mi;
    }
  }
  return best;
}
template <int AK, int NP, typename F>
auto with_conv1x1_tile(int mi, F&& f) {
  if (mi == 1) return f(ConvGemm<AK, NP, 1, 1>{});
  if (mi == 2) return f(ConvGemm<AK, NP, 2, 1>{});
  return f(ConvGemm<AK, NP, 4, 1>{});
}
template <typename F>
auto with_conv1x1_gemm(int w_layout, int nprod, int N, int H, int W, int Cout, F&& f) {
  const int mi = conv1x1_mi(N, H, W, Cout);
  if (w_layout == 0)
    return nprod == 6 ? with_conv1x1_tile<1, 6>(mi, f) : with_conv1x1_tile<1, 3>(mi, f);
  return nprod == 6 ? with_conv1x1_tile<0, 6>(mi, f) : with_conv1x1_tile<0, 3>(mi, f);
}

}  // namespace

}  // namespace tlod

using namespace tlod;

extern "C" size_t tlod_gemm_bs_workspace_bytes(int M, int N, int K, int a_kcontig, int b_kcontig,
                                               int nprod) {
  if (M <= 0 || N <= 0 || K <= 0 || (nprod != 3 && nprod != 6)) return 0;
  return with_gemm(M, a_kcontig ? 1 : 0, b_kcontig ? 1 : 0, nprod,
                   [&](auto g) { return g.ws_bytes(M, N, K); }, N);
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
  }, N);
}

extern "C" int tlod_gemm_bs_ex_f32(const float* a, const float* b, const float* bias,
                                   const float* residual, int relu, float* c, int M, int N, int K,
                                   int a_kcontig, int b_kcontig, int nprod, void* ws,
                                   size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(M > 0 && N > 0 && K > 0 && a && b && c, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(residual != c || residual == nullptr, "residual must not alias c");
  TLOD_CHECK_ARG((size_t)std::max(M, N) * K * 4 < (1ull << 31), "operand too large");
  return with_gemm(M, a_kcontig ? 1 : 0, b_kcontig ? 1 : 0, nprod, [&](auto g) {
    return g.run(a, b, bias, c, M, N, K, static_cast<float*>(ws), ws_bytes, (hipStream_t)stream,
                 residual, relu);
  }, N);
}

extern "C" int tlod_gemm_bs_mask_f32(const float* a, const float* b, const float* residual,
                                     const float* mask, float* c, int M, int N, int K,
                                     int a_kcontig, int b_kcontig, int nprod, void* ws,
                                     size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(M > 0 && N > 0 && K > 0 && a && b && c && mask, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(residual != c && mask != c, "residual / mask must not alias c");
  TLOD_CHECK_ARG((size_t)std::max(M, N) * K * 4 < (1ull << 31), "operand too large");
  return with_gemm(M, a_kcontig ? 1 : 0, b_kcontig ? 1 : 0, nprod, [&](auto g) {
    return g.run(a, b, nullptr, c, M, N, K, static_cast<float*>(ws), ws_bytes,
                 (hipStream_t)stream, residual, 0, mask);
  }, N);
}

extern "C" size_t tlod_conv3x3_gemm_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout,
                                                       int w_layout, int nprod) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Cout <= 0 || (nprod != 3 && nprod != 6)) return 0;
  return with_conv_gemm(w_layout, nprod, [&](auto g) { return g.ws_bytes(N, Cin, H, W, Cout); });
}

extern "C" int tlod_conv3x3_gemm_bs_f32(const float* x, const float* w, int w_layout,
                                        const float* scale, const float* bias,
                                        const float* residual, float* y, int N, int Cin, int H,
                                        int W, int Cout, int relu, int nprod, void* ws,
                                        size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && x && w && y, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(w_layout == 0 || w_layout == 1, "w_layout must be 0 or 1");
  TLOD_CHECK_ARG(residual != y || residual == nullptr, "residual must not alias y");
  // 32-bit buffer byte offsets
  TLOD_CHECK_ARG((size_t)N * Cin * H * W * 4 < (1ull << 31) && (size_t)Cout * Cin * 9 * 4 < (1ull << 31) &&
                     (size_t)Cout * H * W * 4 < (1ull << 31),
                 "operand too large");
  return with_conv_gemm(w_layout, nprod, [&](auto g) {
    return g.run(x, w, ConvEpi{scale, bias, residual, relu}, y, N, Cin, H, W, Cout,
                 static_cast<float*>(ws), ws_bytes, (hipStream_t)stream);
  });
}

extern "C" size_t tlod_conv1x1_gemm_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout,
                                                       int w_layout, int nprod) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Cout <= 0 || (nprod != 3 && nprod != 6)) return 0;
  return with_conv1x1_gemm(w_layout, nprod, N, H, W, Cout,
                           [&](auto g) { return g.ws_bytes(N, Cin, H, W, Cout); });
}

extern "C" int tlod_conv1x1_gemm_bs_ex_f32(const float* x, const float* w, int w_layout,
                                           const float* scale, const float* bias,
                                           const float* residual, const float* mask,
                                           const float* w_scale, float* y, int N, int Cin, int H,
                                           int W, int Cout, int relu, int nprod, void* ws,
                                           size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(mask != y || mask == nullptr, "mask must not alias y");
  TLOD_CHECK_ARG(w_scale == nullptr || w_layout == 1, "w_scale: the dgrad layout only");
  ConvEpi e{scale, bias, residual, relu};
  e.mask = mask;
  e.wscale = w_scale;
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && x && w && y, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(w_layout == 0 || w_layout == 1, "w_layout must be 0 or 1");
  TLOD_CHECK_ARG(residual != y || residual == nullptr, "residual must not alias y");
  TLOD_CHECK_ARG((size_t)Cin * H * W * 4 < (1ull << 31) && (size_t)Cout * Cin * 4 < (1ull << 31) &&
                     (size_t)Cout * H * W * 4 < (1ull << 31),
                 "operand too large");
  return with_conv1x1_gemm(w_layout, nprod, N, H, W, Cout, [&](auto g) {
    return g.run(x, w, e, y, N, Cin, H, W, Cout, static_cast<float*>(ws), ws_bytes,
                 (hipStream_t)stream);
  });
}

extern "C" int tlod_conv1x1_gemm_bs_f32(const float* x, const float* w, int w_layout,
                                        const float* scale, const float* bias,
                                        const float* residual, float* y, int N, int Cin, int H,
                                        int W, int Cout, int relu, int nprod, void* ws,
                                        size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && x && w && y, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(w_layout == 0 || w_layout == 1, "w_layout must be 0 or 1");
  TLOD_CHECK_ARG(residual != y || residual == nullptr, "residual must not alias y");
  // 32-bit buffer byte offsets (per image for x and y)
  TLOD_CHECK_ARG((size_t)Cin * H * W * 4 < (1ull << 31) && (size_t)Cout * Cin * 4 < (1ull << 31) &&
                     (size_t)Cout * H * W * 4 < (1ull << 31),
                 "operand too large");
  return with_conv1x1_gemm(w_layout, nprod, N, H, W, Cout, [&](auto g) {
    return g.run(x, w, ConvEpi{scale, bias, residual, relu}, y, N, Cin, H, W, Cout,
                 static_cast<float*>(ws), ws_bytes, (hipStream_t)stream);
  });
}

extern "C" size_t tlod_gemm_nhwc3_bs_workspace_bytes(int mode, int R, int H, int W, int C, int O,
                                                    int nprod) {
  if (mode < 0 || mode > 2 || R <= 0 || H <= 0 || W <= 0 || C <= 0 || O <= 0 ||
      (nprod != 3 && nprod != 6))
    return 0;
  const Nhwc3Shape sh = nhwc3_shape(mode, R, H, W, C, O);
  return with_nhwc3(mode, sh.M, nprod, [&](auto g) { return g.ws_bytes(sh.M, sh.N, sh.K); });
}

extern "C" int tlod_gemm_nhwc3_bs_f32(int mode, const float* a, const float* b, const float* bias,
                                      const float* residual, const float* mask, int relu,
                                      float* c, int R, int H, int W, int C, int O, int nprod,
                                      void* ws, size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(mode >= 0 && mode <= 2, "mode must be 0 (forward), 1 (input gradient) or 2");
  TLOD_CHECK_ARG(R > 0 && H > 0 && W > 0 && C > 0 && O > 0 && a && b && c, "bad arguments");
  TLOD_CHECK_ARG(nprod == 3 || nprod == 6, "nprod must be 3 or 6");
  TLOD_CHECK_ARG(mode == 0 ? C % 16 == 0 : mode == 1 ? O % 16 == 0 : C % 256 == 0,
                 "channel count: the implicit operand's chunks / tiles must not straddle taps");
  TLOD_CHECK_ARG(mode != 2 || (bias == nullptr && residual == nullptr && mask == nullptr && !relu),
                 "the weight gradient takes no epilogue");
  TLOD_CHECK_ARG(residual != c && mask != c, "residual / mask must not alias c");
  const Nhwc3Shape sh = nhwc3_shape(mode, R, H, W, C, O);
  // 32-bit buffer byte offsets (the implicit operand: rows x channels; the weights: 9 C O)
  TLOD_CHECK_ARG((size_t)sh.geo.rows * std::max(C, O) * 4 < (1ull << 31) &&
                     (size_t)9 * C * O * 4 < (1ull << 31) &&
                     (size_t)std::max(sh.M, sh.N) * sh.K * 4 < (1ull << 31),
                 "operand too large");
  return with_nhwc3(mode, sh.M, nprod, [&](auto g) {
    return g.run(a, b, bias, c, sh.M, sh.N, sh.K, static_cast<float*>(ws), ws_bytes,
                 (hipStream_t)stream, residual, relu, mask, sh.geo);
  });
}
