// Greedy NMS, entirely on device (gfx950).
//
// Semantics: lib/model/nms/src/nms_cuda_kernel.cu:31-39 (devIoU, "+1" areas, strict >)
// and :131-144 (greedy scan over the suppression bitmask).  Differences by design:
//   * the 64x64 tile kernel skips the lower-triangle tiles the scan never reads;
//   * the scan runs on the device (one workgroup, removal bitmask in LDS) instead of an
//     18 MB D2H copy + host loop + H2D of keep (nms_cuda_kernel.cu:117-154);
//   * optional early exit after max_keep survivors (identical first max_keep indices).
// wave64 == the reference's 64-box tile (threadsPerBlock = 64), one wave per tile.
// Compiled with -ffp-contract=off: IoU is bit-identical to the float32 oracle.
#include "common.h"
#include "tlod.h"
#include "nms_impl.h"

namespace tlod {

__device__ __forceinline__ float dev_iou(float a0, float a1, float a2, float a3,
                                         float b0, float b1, float b2, float b3) {
  float left = fmaxf(a0, b0), right = fminf(a2, b2);
  float top = fmaxf(a1, b1), bottom = fminf(a3, b3);
  float width = fmaxf(right - left + 1.f, 0.f), height = fmaxf(bottom - top + 1.f, 0.f);
  float inter = width * height;
  float sa = (a2 - a0 + 1.f) * (a3 - a1 + 1.f);
  float sb = (b2 - b0 + 1.f) * (b3 - b1 + 1.f);
  return inter / (sa + sb - inter);
}

// grid (col_blocks, row_blocks), block 64.  mask[i * ld + cb] bit j set iff
// box i suppresses box cb*64+j (j > i); ld = col_blocks rounded up to even (16-B
// aligned column pairs for the scan).  Diagonal tiles also write the transposed
// words: diag_t[b * 64 + j] bit i set iff box b*64+i suppresses box b*64+j (i < j).
__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int n,
                                                      int dim, float thresh,
                                                      unsigned long long* __restrict__ mask,
                                                      unsigned long long* __restrict__ diag_t,
                                                      int col_blocks, int ld) {
  const int rb = blockIdx.y, cb = blockIdx.x;
  if (cb < rb) return;  // never read by the scan
  const int t = threadIdx.x;
  const int row_size = min(n - rb * 64, 64);
  const int col_size = min(n - cb * 64, 64);
  __shared__ float4 cols[64];
  if (t < col_size) {
    const float* p = boxes + (size_t)(cb * 64 + t) * dim;
    cols[t] = make_float4(p[0], p[1], p[2], p[3]);
  }
  __syncthreads();
  if (t < row_size) {
    const int i = rb * 64 + t;
    const float* p = boxes + (size_t)i * dim;
    const float a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
    unsigned long long bits = 0;
    const int start = (rb == cb) ? t + 1 : 0;
    for (int j = start; j < col_size; ++j) {
      const float4 b = cols[j];
      if (dev_iou(a0, a1, a2, a3, b.x, b.y, b.z, b.w) > thresh) bits |= 1ull << j;
    }
    mask[(size_t)i * ld + cb] = bits;
  }
  if (rb == cb && t < col_size) {  // same IoU(a = row box, b = column box) as above
    const float4 b = cols[t];
    unsigned long long bits = 0;
    for (int i = 0; i < t; ++i) {
      const float4 a = cols[i];
      if (dev_iou(a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w) > thresh) bits |= 1ull << i;
    }
    diag_t[cb * 64 + t] = bits;
  }
}

constexpr int kScanThreads = 1024;
constexpr int kMaxColBlocks = 2048;  // n <= 131072
constexpr int kFastColBlocks = 256;  // n <= 16384: the pipelined scan below

// Pipelined greedy scan for n <= 16384 (the proposal layer: 12000 / 6000 boxes).
// Thread (g = t/128, c2 = t%128) owns mask columns 2*c2, 2*c2+1 (one 16-B load per row) for
// rows g*8..g*8+7 of each 64-row block.  Within a block, wave 0 solves the greedy recurrence
//   kept_j = cand_j AND NOT OR_{i<j} (kept_i AND sup(i, j))
// as a fixed-point iteration over the 64 lanes (lane j holds its suppressor column
// diag_t): the recurrence has a unique solution, iterate k fixes lanes < k, so it
// converges in <= 64 ballots and usually in 2-3 (identical to the sequential scan).
// The scan is bound by its one CU's vector-memory instruction rate (per-wave stamps: the
// four row groups of the 16 x 8-B layout finished ~1400 cycles apart every block), so the
// far-column rows are fetched as 16-B column pairs: half the load instructions.
__global__ void __launch_bounds__(kScanThreads) nms_scan_fast_kernel(
    const unsigned long long* __restrict__ mask, const unsigned long long* __restrict__ diag_t,
    int n, int col_blocks, int ld, int max_keep, int32_t* __restrict__ keep,
    int32_t* __restrict__ num_keep) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  __shared__ unsigned long long remv[kFastColBlocks];
  __shared__ unsigned long long s_kept[4];
  // s_done is double-buffered by block parity: thread 0 may set block b+1's flag before a
  // slower wave has read block b's after the barrier (a single flag would be a data race)
  __shared__ int s_total, s_done[2];
  const int t = threadIdx.x;
  const int c2 = t & 127, g = t >> 7;
  if (t < kFastColBlocks) remv[t] = 0ull;
  if (t < 4) s_kept[t] = 0ull;
  if (t == 0) { s_total = 0; s_done[0] = s_done[1] = 0; }

  // Iteration b: wave 0 resolves block b, then ORs its survivors' words of columns b+1, b+2
  // into remv itself (from 2 words per lane it prefetched: the near columns); meanwhile
  // every thread fetches the rows of block b-1's SURVIVORS only and ORs block b-2's
  // survivors, fetched in the previous iteration, into the columns beyond b.  One barrier
  // per block, and the mask rows of suppressed boxes are never read.  A wave's rows are one
  // g, so the survivor test per row is wave-uniform.
  u64x2 r0[8], r1[8];  // survivor rows (column pairs), by block % 2
  unsigned long long d0 = 0ull, d1 = 0ull;  // wave 0: block's diagonal words
  unsigned long long n0[2] = {0ull, 0ull}, n1[2] = {0ull, 0ull};  // wave 0: near columns
  // 32-bit byte offsets from the uniform base (n * ld * 8 <= 32 MiB): one VGPR per address
  const char* mbase = reinterpret_cast<const char*>(mask);
  auto word = [&](unsigned row, unsigned col) {
    return *reinterpret_cast<const unsigned long long*>(mbase + (row * (unsigned)ld + col) * 8u);
  };
  auto pair = [&](unsigned row, unsigned cp) {
    return *reinterpret_cast<const u64x2*>(mbase + (row * (unsigned)ld + 2u * cp) * 8u);
  };
  // Register discipline for the loads: every row register is READ unconditionally when its
  // block is consumed (a select drops the non-survivors), so no load is still pending when
  // the register is next written.  hipcc then issues a survivor's row load behind a
  // wave-uniform branch without first waiting for every load in flight (it inserted
  // vmcnt(0) there while a conditional consumer could leave an older load pending), and
  // suppressed rows cost no load instruction at all.  Lanes past the live columns read
  // word (0, 0) inside the same instruction.
  // wave 0's words of block bb: diagonal, and columns bb+1, bb+2 of its 64 rows
  auto load_w0 = [&](int bb, unsigned long long& d, unsigned long long (&nw)[2]) {
    const bool w0 = t < 64;
    const int b1 = min(bb, col_blocks - 1);
    d = diag_t[w0 ? b1 * 64 + t : 0];
    const unsigned row = w0 ? (unsigned)min(b1 * 64 + t, n - 1) : 0u;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      nw[q] = word(row, w0 ? (unsigned)min(b1 + 1 + q, col_blocks - 1) : 0u);
  };
  // rows of block p's survivors (kept mask kp), for the columns > p + 2 they are used for
  auto load_rows = [&](int p, unsigned long long kp, u64x2 (&r)[8]) {
    const unsigned kg = (unsigned)(kp >> (g * 8)) & 0xffu;
    const bool cols = 2 * c2 + 1 > p + 2 && 2 * c2 < col_blocks;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((kg >> j) & 1u)
        r[j] = pair(cols ? (unsigned)(p * 64 + g * 8 + j) : 0u, cols ? (unsigned)c2 : 0u);
  };
  load_w0(0, d0, n0);
  __syncthreads();

  // Unrolled x2 below so the register sets never move (a copy of a register with a load
  // in flight would wait for that load): iteration b loads rows of block b-1 into set
  // (b-1) % 2 and uses set b % 2 (block b-2's rows).
  auto step = [&](int b, unsigned long long dcur, const unsigned long long (&ncur)[2],
                  unsigned long long& dnext, unsigned long long (&nnext)[2],
                  u64x2 (&rload)[8], const u64x2 (&ruse)[8]) -> bool {
    load_rows(b - 1, s_kept[(b - 1) & 3], rload);  // b = 0: s_kept[3] == 0, no rows
    load_w0(b + 1, dnext, nnext);
    if (t < 64) {  // wave 0: resolve block b
      const int valid = min(n - b * 64, 64);
      const unsigned long long vmask = valid == 64 ? ~0ull : ((1ull << valid) - 1ull);
      const int total = s_total;
      const int room = (max_keep > 0) ? (max_keep - total) : 0x7fffffff;
      const unsigned long long cand = ~remv[b] & vmask;
      unsigned long long kept = cand;
      for (int it = 0; it < 64; ++it) {
        const unsigned long long nx = cand & __ballot((dcur & kept) == 0ull);
        if (nx == kept) break;
        kept = nx;
      }
      int kc = __popcll(kept);
      if (kc > room) {  // the sequential scan stops at the room-th survivor
        unsigned long long k2 = 0ull;
        for (int r = 0; r < room; ++r) {
          const unsigned long long low = kept & ~k2;
          k2 |= low & (~low + 1ull);
        }
        kept = k2;
        kc = room;
      }
      if ((kept >> t) & 1ull) {
        keep[total + __popcll(kept & ((1ull << t) - 1ull))] = b * 64 + t;
#pragma unroll
        for (int q = 0; q < 2; ++q)  // near columns b+1, b+2
          if (b + 1 + q < col_blocks && ncur[q]) atomicOr(&remv[b + 1 + q], ncur[q]);
      }
      if (t == 0) {
        s_kept[b & 3] = kept;
        s_total = total + kc;
        if (max_keep > 0 && total + kc >= max_keep) s_done[b & 1] = 1;
      }
    }
    {  // block b-2's survivors into the columns beyond b (b < 2: s_kept[2 or 3] == 0)
      const unsigned kg = (unsigned)(s_kept[(b - 2) & 3] >> (g * 8)) & 0xffu;
      u64x2 v = {0ull, 0ull};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u64x2 x = ruse[j];  // unconditional read (see above)
        v |= ((kg >> j) & 1u) ? x : u64x2{0ull, 0ull};
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int col = 2 * c2 + q;
        if (col > b && col < col_blocks && v[q]) atomicOr(&remv[col], v[q]);
      }
    }
    __syncthreads();
    return s_done[b & 1] != 0;
  };
  for (int b = 0; b < col_blocks; b += 2) {
    if (step(b, d0, n0, d1, n1, r1, r0) || b + 1 >= col_blocks) break;
    if (step(b + 1, d1, n1, d0, n0, r0, r1)) break;
  }
  if (t == 0) *num_keep = s_total;
}

// General scan (n <= 131072).  One workgroup.  remv[] (removal bits per 64-box block) lives in LDS.  Block b's
// survivors are resolved by wave 0 with the in-block (diagonal) mask words, then all
// 16 waves OR the survivors' rows into remv for the later blocks.
__global__ void __launch_bounds__(kScanThreads) nms_scan_kernel(
    const unsigned long long* __restrict__ mask, int n, int col_blocks, int ld, int max_keep,
    int32_t* __restrict__ keep, int32_t* __restrict__ num_keep) {
  __shared__ unsigned long long remv[kMaxColBlocks];
  __shared__ int kept_rows[64];
  __shared__ int s_kcount, s_total, s_done;
  const int t = threadIdx.x;
  for (int c = t; c < col_blocks; c += kScanThreads) remv[c] = 0ull;
  if (t == 0) { s_total = 0; s_done = 0; }
  __syncthreads();
  for (int b = 0; b < col_blocks; ++b) {
    if (t < 64) {  // wave 0: resolve block b sequentially
      const int i = b * 64 + t;
      const unsigned long long diag = (i < n) ? mask[(size_t)i * ld + b] : 0ull;
      unsigned long long w = remv[b];
      const int valid = min(n - b * 64, 64);
      int total = s_total;
      int kc = 0;
      const int room = (max_keep > 0) ? (max_keep - total) : 0x7fffffff;
      for (int j = 0; j < valid; ++j) {
        const unsigned long long dj =
            ((unsigned long long)__shfl((int)(diag >> 32), j) << 32) |
            (unsigned long long)(unsigned)__shfl((int)(diag & 0xffffffffull), j);
        if (!((w >> j) & 1ull)) {
          if (kc < room) {
            if (t == 0) { keep[total + kc] = i - t + j; kept_rows[kc] = i - t + j; }
            ++kc;
            w |= dj;
          } else {
            break;
          }
        }
      }
      if (t == 0) {
        s_kcount = kc;
        s_total = total + kc;
        if (max_keep > 0 && total + kc >= max_keep) s_done = 1;
      }
    }
    __syncthreads();
    if (s_done) break;
    const int kc = s_kcount;
    const int ncols = col_blocks - b - 1;
    if (kc > 0 && ncols > 0) {
      const int lane_col = t & 255, grp = t >> 8;  // 4 groups over kept rows
      for (int co = lane_col; co < ncols; co += 256) {
        const int c = b + 1 + co;
        unsigned long long v = 0ull;
        for (int k = grp; k < kc; k += 4) v |= mask[(size_t)kept_rows[k] * ld + c];
        if (v) atomicOr(&remv[c], v);
      }
    }
    __syncthreads();
  }
  if (t == 0) *num_keep = s_total;
}

static int mask_ld(int cb) { return cb + (cb & 1); }

size_t nms_ws_bytes(int n) {
  const int cb = div_up(n > 0 ? n : 1, 64);
  return (align_up((size_t)n * mask_ld(cb), 32) + (size_t)cb * 64) * sizeof(unsigned long long);
}

int nms_launch(const float* boxes, int n, int dim, float thresh, int max_keep, int32_t* keep,
               int32_t* num_keep, void* ws, size_t ws_bytes, hipStream_t s) {
  TLOD_CHECK_ARG(n >= 0 && dim >= 4, "bad n/dim");
  if (n == 0) {
    TLOD_HIP(hipMemsetAsync(num_keep, 0, sizeof(int32_t), s));
    return kOk;
  }
  const int cb = div_up(n, 64);
  TLOD_CHECK_ARG(cb <= kMaxColBlocks, "n too large (max 131072)");
  if (ws_bytes < nms_ws_bytes(n)) {
    set_error("tlod_nms: workspace too small");
    return kWorkspace;
  }
  auto* mask = static_cast<unsigned long long*>(ws);
  const int ld = mask_ld(cb);
  auto* diag_t = mask + align_up((size_t)n * ld, 32);
  hipLaunchKernelGGL(nms_mask_kernel, dim3(cb, cb), dim3(64), 0, s, boxes, n, dim, thresh,
                     mask, diag_t, cb, ld);
  TLOD_LAUNCH_CHECK();
  if (cb <= kFastColBlocks)
    hipLaunchKernelGGL(nms_scan_fast_kernel, dim3(1), dim3(kScanThreads), 0, s, mask, diag_t, n,
                       cb, ld, max_keep, keep, num_keep);
  else
    hipLaunchKernelGGL(nms_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, mask, n, cb, ld,
                       max_keep, keep, num_keep);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

}  // namespace tlod

extern "C" size_t tlod_nms_workspace_bytes(int n) { return tlod::nms_ws_bytes(n); }

extern "C" int tlod_nms_f32(const float* dets, int n, int dim, float thresh, int max_keep,
                            int32_t* keep, int32_t* num_keep, void* ws, size_t ws_bytes,
                            tlod_stream_t stream) {
  return tlod::nms_launch(dets, n, dim, thresh, max_keep, keep, num_keep, ws, ws_bytes,
                          (hipStream_t)stream);
}
