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

// grid (col_blocks, row_blocks), block 64.  mask[i * col_blocks + cb] bit j set iff
// box i suppresses box cb*64+j (j > i).
__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int n,
                                                      int dim, float thresh,
                                                      unsigned long long* __restrict__ mask,
                                                      int col_blocks) {
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
    mask[(size_t)i * col_blocks + cb] = bits;
  }
}

constexpr int kScanThreads = 1024;
constexpr int kMaxColBlocks = 2048;  // n <= 131072

// One workgroup.  remv[] (removal bits per 64-box block) lives in LDS.  Block b's
// survivors are resolved by wave 0 with the in-block (diagonal) mask words, then all
// 16 waves OR the survivors' rows into remv for the later blocks.
__global__ void __launch_bounds__(kScanThreads) nms_scan_kernel(
    const unsigned long long* __restrict__ mask, int n, int col_blocks, int max_keep,
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
      const unsigned long long diag = (i < n) ? mask[(size_t)i * col_blocks + b] : 0ull;
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
        for (int k = grp; k < kc; k += 4) v |= mask[(size_t)kept_rows[k] * col_blocks + c];
        if (v) atomicOr(&remv[c], v);
      }
    }
    __syncthreads();
  }
  if (t == 0) *num_keep = s_total;
}

size_t nms_ws_bytes(int n) {
  const int cb = div_up(n > 0 ? n : 1, 64);
  return align_up((size_t)n * cb * sizeof(unsigned long long), 256);
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
  hipLaunchKernelGGL(nms_mask_kernel, dim3(cb, cb), dim3(64), 0, s, boxes, n, dim, thresh,
                     mask, cb);
  TLOD_LAUNCH_CHECK();
  hipLaunchKernelGGL(nms_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, mask, n, cb,
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
