// Test-time detection post-processing for one image, every class in one launch.
//
// Replaces the per-class host loop of the test drivers (methods/DAF/DAF_test.py:282-321,
// same in the other methods' *_test.py): bbox deltas de-normalised by
// BBOX_NORMALIZE_STDS / MEANS (:284-292), bbox_transform_inv + clip_boxes
// (lib/model/rpn/bbox_transform.py:77-103, :125-133), division by the image scale (:298;
// a true division, as torch 0.4's THC div by a scalar — README.md:49 pins torch 0.4.0),
// then per class j >= 1: scores > thresh (nonzero, a host sync), torch.sort descending,
// cat with the boxes, nms(cls_dets, TEST.NMS) (a device -> host -> device round trip per
// class, lib/model/nms/nms_gpu.py) and the kept rows.
//
// One workgroup (1024 threads = 16 waves) per class, everything in LDS:
//   decode + clip + rescale of the class's R boxes, stable descending bitonic sort of the
//   candidates (score, then index — the reference's torch.sort is not stable; with distinct
//   scores both orders agree), then the greedy NMS scan: for each surviving box in order,
//   every thread tests its boxes behind it (devIoU semantics: "+1" areas, suppress if
//   IoU > thresh, nms_cuda_kernel.cu:31-39) — one barrier per kept box.
// Float semantics: one rounding per op (-ffp-contract=off), expf from ocml (the decode
// agrees with the reference's torch.exp to ~1 ulp; the tests compare the NMS on the
// device-decoded boxes, as for the proposal layer).
#include "common.h"
#include "tlod.h"

namespace tlod {
namespace {

constexpr int kMaxR = 2048;
constexpr int kThreads = 1024;

__device__ __forceinline__ float iou_plus1(const float4 a, const float4 b) {
  const float left = fmaxf(a.x, b.x), right = fminf(a.z, b.z);
  const float top = fmaxf(a.y, b.y), bottom = fminf(a.w, b.w);
  const float width = fmaxf(right - left + 1.f, 0.f), height = fmaxf(bottom - top + 1.f, 0.f);
  const float inter = width * height;
  const float sa = (a.z - a.x + 1.f) * (a.w - a.y + 1.f);
  const float sb = (b.z - b.x + 1.f) * (b.w - b.y + 1.f);
  return inter / (sa + sb - inter);
}

// key order: larger score first, then smaller index
__device__ __forceinline__ bool before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}

__global__ void __launch_bounds__(kThreads) detect_kernel(
    const float* __restrict__ rois, const float* __restrict__ cls_prob,
    const float* __restrict__ bbox_pred, int R, int C, int agnostic, float im_h, float im_w,
    float im_scale, float4 stds, float4 means, float score_thresh, float nms_thresh,
    float* __restrict__ dets, int32_t* __restrict__ counts, float* __restrict__ boxes_out) {
  __shared__ float4 box[kMaxR];
  __shared__ float key[kMaxR];
  __shared__ int idx[kMaxR];
  __shared__ unsigned char removed[kMaxR];
  __shared__ int n_cand;
  const int j = blockIdx.x + 1;  // class (0 = background is skipped)
  const int t = threadIdx.x;
  if (t == 0) n_cand = 0;
  // 1. decode / clip / rescale every RoI for class j; candidates score > thresh
  for (int r = t; r < R; r += kThreads) {
    const float* ro = rois + (size_t)r * 5;
    const float x1 = ro[1], y1 = ro[2], x2 = ro[3], y2 = ro[4];
    const float* d = bbox_pred + (size_t)r * (agnostic ? 4 : 4 * C) + (agnostic ? 0 : 4 * j);
    const float dx = d[0] * stds.x + means.x, dy = d[1] * stds.y + means.y;
    const float dw = d[2] * stds.z + means.z, dh = d[3] * stds.w + means.w;
    const float widths = x2 - x1 + 1.0f, heights = y2 - y1 + 1.0f;
    const float cx = x1 + 0.5f * widths, cy = y1 + 0.5f * heights;
    const float pcx = dx * widths + cx, pcy = dy * heights + cy;
    const float pw = expf(dw) * widths, ph = expf(dh) * heights;
    float4 b;
    b.x = fminf(fmaxf(pcx - 0.5f * pw, 0.f), im_w - 1.f) / im_scale;
    b.y = fminf(fmaxf(pcy - 0.5f * ph, 0.f), im_h - 1.f) / im_scale;
    b.z = fminf(fmaxf(pcx + 0.5f * pw, 0.f), im_w - 1.f) / im_scale;
    b.w = fminf(fmaxf(pcy + 0.5f * ph, 0.f), im_h - 1.f) / im_scale;
    if (boxes_out) reinterpret_cast<float4*>(boxes_out)[(size_t)r * C + j] = b;
    box[r] = b;
  }
  __syncthreads();
  // compact the candidates (any order: the sort below fixes it)
  for (int r = t; r < R; r += kThreads) {
    const float s = cls_prob[(size_t)r * C + j];
    if (s > score_thresh) {
      const int k = atomicAdd(&n_cand, 1);
      key[k] = s;
      idx[k] = r;
    }
  }
  __syncthreads();
  const int n = n_cand;
  int p2 = 1;
  while (p2 < n) p2 <<= 1;
  for (int k = n + t; k < p2; k += kThreads) {
    key[k] = -INFINITY;
    idx[k] = 0x7fffffff;
  }
  __syncthreads();
  // 2. bitonic sort of (key, idx) into descending order
  for (int size = 2; size <= p2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int k = t; k < p2; k += kThreads) {
        const int l = k ^ stride;
        if (l > k) {
          const bool asc_block = (k & size) != 0;  // this block sorts the other way
          const float sk = key[k], sl = key[l];
          const int ik = idx[k], il = idx[l];
          const bool swap = asc_block ? before(sk, ik, sl, il) : before(sl, il, sk, ik);
          if (swap) {
            key[k] = sl; key[l] = sk;
            idx[k] = il; idx[l] = ik;
          }
        }
      }
      __syncthreads();
    }
  }
  // 3. greedy NMS over the sorted candidates
  for (int k = t; k < n; k += kThreads) removed[k] = 0;
  __syncthreads();
  int kept = 0;
  float* out = dets + ((size_t)j * R) * 5;
  for (int i = 0; i < n; ++i) {
    if (removed[i]) continue;  // uniform: written before the last barrier
    const float4 bi = box[idx[i]];
    if (t == 0) {
      float* o = out + (size_t)kept * 5;
      o[0] = bi.x; o[1] = bi.y; o[2] = bi.z; o[3] = bi.w; o[4] = key[i];
    }
    ++kept;
    for (int k = i + 1 + t; k < n; k += kThreads)
      if (!removed[k] && iou_plus1(bi, box[idx[k]]) > nms_thresh) removed[k] = 1;
    __syncthreads();
  }
  if (t == 0) counts[j] = kept;
}

}  // namespace
}  // namespace tlod

using namespace tlod;

extern "C" int tlod_detect_f32(const float* rois, const float* cls_prob, const float* bbox_pred,
                               int R, int C, int class_agnostic, const float* stds,
                               const float* means, float im_h, float im_w, float im_scale,
                               float score_thresh, float nms_thresh, float* dets,
                               int32_t* counts, float* boxes_out, tlod_stream_t stream) {
  TLOD_CHECK_ARG(rois && cls_prob && bbox_pred && stds && means && dets && counts,
                 "null pointer");
  TLOD_CHECK_ARG(R > 0 && R <= kMaxR && C >= 2 && im_scale > 0.f, "bad sizes");
  hipStream_t s = (hipStream_t)stream;
  TLOD_HIP(hipMemsetAsync(counts, 0, sizeof(int32_t), s));  // class 0 (background)
  hipLaunchKernelGGL(detect_kernel, dim3(C - 1), dim3(kThreads), 0, s, rois, cls_prob, bbox_pred,
                     R, C, class_agnostic, im_h, im_w, im_scale,
                     make_float4(stds[0], stds[1], stds[2], stds[3]),
                     make_float4(means[0], means[1], means[2], means[3]), score_thresh,
                     nms_thresh, dets, counts, boxes_out);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
