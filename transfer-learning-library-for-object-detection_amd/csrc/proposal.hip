// RPN proposal layer on device: decode + clip -> stable descending sort -> top pre_nms
// -> NMS -> top post_nms -> zero-padded rois.  Replaces _ProposalLayer.forward
// (lib/model/rpn/proposal_layer.py:49-161), which builds anchors with numpy on the host,
// sorts with torch, loops over images in Python and round-trips NMS through the host.
//
// Float semantics: bbox_transform_inv (lib/model/rpn/bbox_transform.py:77-103) and
// clip_boxes (:125-133), one rounding per op (-ffp-contract=off), expf from ocml.
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "nms_impl.h"
#include "tlod.h"

namespace tlod {

// One thread per anchor of image `img`: idx = (h*W + w)*A + a (proposal_layer.py:90-103).
__global__ void proposal_decode_kernel(const float* __restrict__ cls_prob,
                                       const float* __restrict__ deltas,
                                       const float* __restrict__ im_info,
                                       const float* __restrict__ base_anchors, int img, int A,
                                       int H, int W, int stride, float* __restrict__ scores,
                                       int32_t* __restrict__ ids, float4* __restrict__ props,
                                       float* __restrict__ props_out) {
  const int N = H * W * A;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N) return;
  const int a = idx % A;
  const int hw = idx / A;
  const int w = hw % W, h = hw / W;
  const size_t HW = (size_t)H * W;
  const float sx = (float)(w * stride), sy = (float)(h * stride);
  const float x1 = base_anchors[a * 4 + 0] + sx, y1 = base_anchors[a * 4 + 1] + sy;
  const float x2 = base_anchors[a * 4 + 2] + sx, y2 = base_anchors[a * 4 + 3] + sy;
  const float* d = deltas + ((size_t)img * 4 * A + 4 * a) * HW + hw;
  const float dx = d[0], dy = d[HW], dw = d[2 * HW], dh = d[3 * HW];
  const float widths = x2 - x1 + 1.0f, heights = y2 - y1 + 1.0f;
  const float cx = x1 + 0.5f * widths, cy = y1 + 0.5f * heights;
  const float pcx = dx * widths + cx, pcy = dy * heights + cy;
  const float pw = expf(dw) * widths, ph = expf(dh) * heights;
  const float imh = im_info[img * 3 + 0], imw = im_info[img * 3 + 1];
  const float xm = imw - 1.f, ym = imh - 1.f;
  float4 p;
  p.x = fminf(fmaxf(pcx - 0.5f * pw, 0.f), xm);
  p.y = fminf(fmaxf(pcy - 0.5f * ph, 0.f), ym);
  p.z = fminf(fmaxf(pcx + 0.5f * pw, 0.f), xm);
  p.w = fminf(fmaxf(pcy + 0.5f * ph, 0.f), ym);
  props[idx] = p;
  if (props_out) reinterpret_cast<float4*>(props_out)[(size_t)img * N + idx] = p;
  scores[idx] = cls_prob[((size_t)img * 2 * A + A + a) * HW + hw];
  ids[idx] = idx;
}

__global__ void gather_sorted_kernel(const float4* __restrict__ props,
                                     const int32_t* __restrict__ order, int n,
                                     float4* __restrict__ dets) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dets[i] = props[order[i]];
}

// rois_out[img] = (img, box) for kept, zero padding after (proposal_layer.py:154-159).
__global__ void write_rois_kernel(const float4* __restrict__ dets, const int32_t* __restrict__ keep,
                                  const int32_t* __restrict__ num_keep, int img, int post,
                                  float* __restrict__ rois) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= post) return;
  float* o = rois + ((size_t)img * post + j) * 5;
  o[0] = (float)img;
  if (j < *num_keep) {
    const float4 b = dets[keep[j]];
    o[1] = b.x; o[2] = b.y; o[3] = b.z; o[4] = b.w;
  } else {
    o[1] = 0.f; o[2] = 0.f; o[3] = 0.f; o[4] = 0.f;
  }
}

struct ProposalWs {
  float* scores; float* scores_sorted; int32_t* ids; int32_t* ids_sorted;
  float4* props; float4* dets; int32_t* keep; int32_t* num_keep;
  void* cub_tmp; size_t cub_bytes; void* nms_ws; size_t nms_bytes;
};

static size_t cub_sort_bytes(int N) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const float*)nullptr,
                                               (float*)nullptr, (const int32_t*)nullptr,
                                               (int32_t*)nullptr, N);
  return bytes;
}

static size_t carve_proposal(Carve& c, ProposalWs& w, int A, int H, int W, int pre_nms) {
  const int N = H * W * A;
  const int n_top = (pre_nms > 0 && pre_nms < N) ? pre_nms : N;
  w.scores = c.take<float>(N);
  w.scores_sorted = c.take<float>(N);
  w.ids = c.take<int32_t>(N);
  w.ids_sorted = c.take<int32_t>(N);
  w.props = c.take<float4>(N);
  w.dets = c.take<float4>(n_top);
  w.keep = c.take<int32_t>(n_top);
  w.num_keep = c.take<int32_t>(1);
  w.cub_bytes = cub_sort_bytes(N);
  w.cub_tmp = c.take<char>(w.cub_bytes);
  w.nms_bytes = nms_ws_bytes(n_top);
  w.nms_ws = c.take<char>(w.nms_bytes);
  return align_up(c.off, 256);
}

}  // namespace tlod

using namespace tlod;

extern "C" size_t tlod_proposal_workspace_bytes(int B, int A, int H, int W, int pre_nms) {
  (void)B;
  Carve c(nullptr, 0);
  ProposalWs w;
  return carve_proposal(c, w, A, H, W, pre_nms);
}

extern "C" int tlod_proposal_f32(const float* cls_prob, const float* bbox_deltas,
                                 const float* im_info, const float* base_anchors, int B, int A,
                                 int H, int W, int feat_stride, int pre_nms, int post_nms,
                                 float nms_thresh, float* rois_out, float* props_out, void* ws,
                                 size_t ws_bytes, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && A > 0 && H > 0 && W > 0 && post_nms > 0, "bad shape");
  hipStream_t s = (hipStream_t)stream;
  Carve c(ws, ws_bytes);
  ProposalWs w;
  carve_proposal(c, w, A, H, W, pre_nms);
  if (!c.ok()) {
    set_error("tlod_proposal_f32: workspace too small");
    return kWorkspace;
  }
  const int N = H * W * A;
  // proposal_layer.py:134: pre_nms_topN compared against numel over the whole batch.
  const int n_top = (pre_nms > 0 && pre_nms < B * N) ? std::min(pre_nms, N) : N;
  for (int img = 0; img < B; ++img) {
    hipLaunchKernelGGL(proposal_decode_kernel, dim3(div_up(N, 256)), dim3(256), 0, s, cls_prob,
                       bbox_deltas, im_info, base_anchors, img, A, H, W, feat_stride, w.scores,
                       w.ids, w.props, props_out);
    TLOD_LAUNCH_CHECK();
    size_t cb = w.cub_bytes;
    TLOD_HIP(hipcub::DeviceRadixSort::SortPairsDescending(w.cub_tmp, cb, w.scores,
                                                          w.scores_sorted, w.ids, w.ids_sorted,
                                                          N, 0, 32, s));
    hipLaunchKernelGGL(gather_sorted_kernel, dim3(div_up(n_top, 256)), dim3(256), 0, s, w.props,
                       w.ids_sorted, n_top, w.dets);
    TLOD_LAUNCH_CHECK();
    int st = nms_launch(reinterpret_cast<const float*>(w.dets), n_top, 4, nms_thresh, post_nms,
                        w.keep, w.num_keep, w.nms_ws, w.nms_bytes, s);
    if (st != kOk) return st;
    hipLaunchKernelGGL(write_rois_kernel, dim3(div_up(post_nms, 256)), dim3(256), 0, s, w.dets,
                       w.keep, w.num_keep, img, post_nms, rois_out);
    TLOD_LAUNCH_CHECK();
  }
  return kOk;
}
