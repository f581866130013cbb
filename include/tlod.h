/*
 * tlod.h — C ABI of the MI355X-native (gfx950) hot path for the domain-adaptive
 * Faster R-CNN training step of Transfer-Learning-Library-for-Object-Detection.
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes; no framework types cross this boundary;
 *   - every call is stream-ordered and asynchronous on `stream` (a hipStream_t; NULL =
 *     the legacy default stream).  No entry point allocates, frees or synchronises, so a
 *     caller may capture any of them into a hipGraph;
 *   - scratch is caller-provided (`ws`, `ws_bytes`); query sizes with *_workspace_bytes;
 *   - return 0 on success, a negative tlod_status on failure with a message available
 *     from tlod_last_error() (thread-local).  Nothing ever calls exit() (the reference's
 *     launchers do: roi_align_kernel.cu:84-88);
 *   - tensors are contiguous NCHW float32 (the reference's layout and dtype).
 *
 * Environment switches (they choose between kernels that compute the same result — none is
 * needed for correctness):
 *   TLOD_ROI_BWD_GATHER=0  RoIAlignAvg backward on the atomic kernels instead of the
 *                          deterministic sorted-tap gather (the gather workspace query then
 *                          returns 0; read at every call, so set it before the query);
 *   TLOD_CU_RESERVE=n      initial value of tlod_set_cu_reserve (CUs the planners leave out);
 * the workspace queries follow the same switches, so query after setting them.  The conv
 * planners' tiling / split A/B switches (TLOD_CONV_WS, TLOD_WS_FLEX, TLOD_CONV_KSPLIT_MAX,
 * TLOD_WGRAD_WS, ...) are compile-time defines in the csrc .hip sources, not run-time switches.
 *
 * Each entry point names the reference interface it replaces (paths relative to the
 * reference checkout).
 */
#ifndef TLOD_H_
#define TLOD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* tlod_stream_t; /* hipStream_t */

enum tlod_status {
  TLOD_OK = 0,
  TLOD_EINVAL = -1,
  TLOD_EHIP = -2,
  TLOD_EWORKSPACE = -3,
  TLOD_EUNSUPPORTED = -4
};

int tlod_abi_version(void);
const char* tlod_last_error(void);
/* CUs the split-K / round planners leave out (default 0, or env TLOD_CU_RESERVE): set by the
 * data-parallel reducer (tlod/dist.py) while its all-reduces run beside the backward, whose
 * kernels then hold a few CUs; process-wide, read at every launch.  0 <= cus <= 1024. */
int tlod_set_cu_reserve(int cus);

/* ------------------------------------------------------------------ NMS
 * Replaces: nms_cuda(THCudaIntTensor* keep_out, THCudaTensor* boxes, THCudaIntTensor*
 *   num_out, float thresh)            lib/model/nms/src/nms_cuda.c:8-19
 *   -> nms_cuda_compute(...)          lib/model/nms/src/nms_cuda_kernel.cu:87-161
 * dets: n x dim (dim >= 4: x1,y1,x2,y2[,score]) already sorted by score, descending.
 * keep: int32[n] indices into dets (only the first *num_keep are written);
 * num_keep: one int32 on device.  max_keep > 0 stops after that many survivors (the
 * caller's keep[:post_nms_topN], proposal_layer.py:151-152); <= 0 keeps all.
 * IoU semantics of devIoU (nms_cuda_kernel.cu:31-39): "+1" areas, suppress if IoU > thresh.
 * Everything (mask and the greedy scan) runs on the device: no host round trip. */
size_t tlod_nms_workspace_bytes(int n);
int tlod_nms_f32(const float* dets, int n, int dim, float thresh, int max_keep,
                 int32_t* keep, int32_t* num_keep, void* ws, size_t ws_bytes,
                 tlod_stream_t stream);

/* ------------------------------------------------------------------ RoIAlign
 * Replaces: roi_align_forward_cuda / roi_align_backward_cuda
 *   lib/model/roi_align/src/roi_align_cuda.c:7-76 (kernels roi_align_kernel.cu:15-143).
 * feat (B,C,H,W), rois (R,5) = (batch, x1, y1, x2, y2) in image coords.
 * fwd writes out (R,C,ah,aw) (no pre-zeroing needed).  bwd ACCUMULATES into
 * bottom_grad (B,C,H,W): zero it first (the reference's caller does, roi_align.py:42).
 * The *_avg variants fuse RoIAlignAvg (modules/roi_align.py:18-29): align at
 * (ph+1)x(pw+1) then avg_pool2d(2, stride 1) -> (R,C,ph,pw), forward and backward. */
int tlod_roi_align_fwd_f32(const float* feat, int B, int C, int H, int W,
                           const float* rois, int R, int ah, int aw, float scale,
                           float* out, tlod_stream_t stream);
int tlod_roi_align_bwd_f32(const float* top_grad, int B, int C, int H, int W,
                           const float* rois, int R, int ah, int aw, float scale,
                           float* bottom_grad, tlod_stream_t stream);
int tlod_roi_align_avg_fwd_f32(const float* feat, int B, int C, int H, int W,
                               const float* rois, int R, int ph, int pw, float scale,
                               float* out, tlod_stream_t stream);
/* avg backward, ADDED into bottom_grad (roi_align_kernel.cu:94-143 + avg_pool2d's backward).
 * With ws_bytes >= tlod_roi_align_avg_bwd_gather_workspace_bytes: no atomics — the taps are
 * sorted by feature cell and every (cell, channel) gathers its contributions in a fixed
 * order (deterministic; ~R*64*(C+16)*4 B of workspace).  Otherwise, with ws_bytes >=
 * tlod_roi_align_avg_bwd_workspace_bytes: float atomics into a (B,H,W,C) accumulator then
 * added into bottom_grad; ws == NULL: atomics straight into NCHW. */
size_t tlod_roi_align_avg_bwd_gather_workspace_bytes(int B, int C, int H, int W, int R, int ph,
                                                     int pw);
size_t tlod_roi_align_avg_bwd_workspace_bytes(int B, int C, int H, int W);
int tlod_roi_align_avg_bwd_f32(const float* top_grad, int B, int C, int H, int W,
                               const float* rois, int R, int ph, int pw, float scale,
                               float* bottom_grad, void* ws, size_t ws_bytes,
                               tlod_stream_t stream);
/* ResNet RoI-head entry: RoIAlignAvg's bins (2i, 2j) only, channels-last — what
 * RCNN_top = layer4 reads of pool5 (its first bottleneck subsamples by 2:
 * lib/DAF/resnet.py:64-102, :286-288 via _head_to_tail).  out (R, QH, QW, C) with
 * QH = ceil(ph / 2), QW = ceil(pw / 2), equal bit for bit to
 * tlod_roi_align_avg_fwd_f32's out[r][c][2i][2j]; the backward ADDS the gradient of that
 * selection into bottom_grad (B,C,H,W), deterministic (the sorted-tap gather), equal to
 * tlod_roi_align_avg_bwd_f32 of a top gradient that is zero off the selected bins.  One
 * workspace query covers both directions. */
size_t tlod_roi_align_avg_s2_workspace_bytes(int B, int C, int H, int W, int R, int ph, int pw);
int tlod_roi_align_avg_s2_nhwc_fwd_f32(const float* feat, int B, int C, int H, int W,
                                       const float* rois, int R, int ph, int pw, float scale,
                                       float* out, void* ws, size_t ws_bytes,
                                       tlod_stream_t stream);
int tlod_roi_align_avg_s2_nhwc_bwd_f32(const float* top_grad, int B, int C, int H, int W,
                                       const float* rois, int R, int ph, int pw, float scale,
                                       float* bottom_grad, void* ws, size_t ws_bytes,
                                       tlod_stream_t stream);

/* ------------------------------------------------------------------ RoIPool
 * Replaces: roi_pooling_forward_cuda / roi_pooling_backward_cuda
 *   lib/model/roi_pooling/src/roi_pooling_cuda.c (kernels roi_pooling_kernel.cu:24-203).
 * argmax: int32 (R,C,ph,pw), flat index into feat or -1 for an empty bin.
 * bwd ACCUMULATES into bottom_grad (zero it first); it scatters through argmax
 * (equal sums to the reference's O(B*C*H*W*R) gather). */
int tlod_roi_pool_fwd_f32(const float* feat, int B, int C, int H, int W,
                          const float* rois, int R, int ph, int pw, float scale,
                          float* out, int32_t* argmax, tlod_stream_t stream);
int tlod_roi_pool_bwd_f32(const float* top_grad, const int32_t* argmax, int R, int C,
                          int ph, int pw, float* bottom_grad, tlod_stream_t stream);

/* ------------------------------------------------------------------ Proposal layer
 * Replaces: _ProposalLayer.forward   lib/model/rpn/proposal_layer.py:49-161
 * cls_prob (B,2A,H,W) (fg = channels A..2A-1), bbox_deltas (B,4A,H,W), im_info (B,3),
 * base_anchors (A,4) [generate_anchors order].  rois_out (B,post_nms,5), zero padded,
 * column 0 = batch index.  Decode+clip, stable descending sort, top pre_nms, NMS,
 * top post_nms — all on device.  `props_out` (optional, may be NULL) receives the
 * decoded+clipped boxes (B, H*W*A, 4) in anchor order. */
size_t tlod_proposal_workspace_bytes(int B, int A, int H, int W, int pre_nms);
int tlod_proposal_f32(const float* cls_prob, const float* bbox_deltas, const float* im_info,
                      const float* base_anchors, int B, int A, int H, int W,
                      int feat_stride, int pre_nms, int post_nms, float nms_thresh,
                      float* rois_out, float* props_out, void* ws, size_t ws_bytes,
                      tlod_stream_t stream);

/* ------------------------------------------------------------------ Anchor target
 * Replaces: _AnchorTargetLayer.forward   lib/model/rpn/anchor_target_layer.py:48-193
 * Two phases so the reference's host-RNG draws can be replayed exactly:
 *   1. tlod_anchor_target_label_f32: inside filter (image 0's size, :83-87), IoU with
 *      the reference's masks, max/argmax, gt-max ties, thresholds -> pre-sampling
 *      labels; writes counts[B*2] = (#fg, #bg) per image (device int32).
 *   2. tlod_anchor_target_sample_f32: fg/bg subsampling, targets, weights, unmap and
 *      the output layouts labels (B,1,A*H,W), targets/inside_w/outside_w (B,4A,H,W).
 *      Permutations: if `perm` is non-NULL it holds the np.random.permutation draws in
 *      the reference's call order (:131 then :143, image by image), concatenated;
 *      perm_off[2*B+1] (device int32 prefix offsets) delimits them: image b's fg draw is
 *      perm[perm_off[2b] .. perm_off[2b+1]), its bg draw perm[perm_off[2b+1] ..
 *      perm_off[2b+2]) (empty when that image did not subsample).  If `perm` is NULL a
 *      counter-based device RNG keyed by `seed` draws the same distribution.
 * tlod_anchor_target_f32 = both phases with the device RNG (no host sync).
 * gt_boxes (B,G,5), im_info (B,3). */
typedef struct tlod_rpn_cfg {
  float pos_overlap;   /* 0.7 RPN_POSITIVE_OVERLAP */
  float neg_overlap;   /* 0.3 RPN_NEGATIVE_OVERLAP */
  float fg_fraction;   /* 0.5 RPN_FG_FRACTION */
  int batch_size;      /* 256 RPN_BATCHSIZE */
  int clobber_positives; /* 0 */
  float inside_weight; /* 1.0 RPN_BBOX_INSIDE_WEIGHTS[0] */
  int allowed_border;  /* 0 */
} tlod_rpn_cfg;

size_t tlod_anchor_target_workspace_bytes(int B, int A, int H, int W, int G);
int tlod_anchor_target_label_f32(const float* base_anchors, int A, int H, int W, int feat_stride,
                                 const float* gt_boxes, int B, int G, const float* im_info,
                                 const tlod_rpn_cfg* cfg, int32_t* counts, void* ws,
                                 size_t ws_bytes, tlod_stream_t stream);
int tlod_anchor_target_sample_f32(const float* base_anchors, int A, int H, int W, int feat_stride,
                                  const float* gt_boxes, int B, int G, const tlod_rpn_cfg* cfg,
                                  const int32_t* perm, const int32_t* perm_off, uint64_t seed,
                                  float* labels, float* bbox_targets, float* inside_w,
                                  float* outside_w, void* ws, size_t ws_bytes,
                                  tlod_stream_t stream);
int tlod_anchor_target_f32(const float* base_anchors, int A, int H, int W, int feat_stride,
                           const float* gt_boxes, int B, int G, const float* im_info,
                           const tlod_rpn_cfg* cfg, uint64_t seed, int32_t* counts,
                           float* labels, float* bbox_targets, float* inside_w,
                           float* outside_w, void* ws, size_t ws_bytes, tlod_stream_t stream);

/* ------------------------------------------------------------------ Proposal target
 * Replaces: _ProposalTargetLayer.forward  lib/model/rpn/proposal_target_layer_cascade.py:33-212
 * rois (B,R,5) + gt (B,G,5) appended (:39-43) -> S sampled RoIs per image.
 * Phase 1 writes counts[B*2] = (#fg, #bg candidates).  Phase 2 samples: explicit mode
 * takes, per image, the np.random.permutation(#fg) draw (fg_perm, concatenated, offsets
 * perm_off[B+1]) and the np.random.rand(k) draw as float64 (rand, concatenated,
 * offsets rand_off[B+1]); NULL -> device RNG keyed by `seed`.
 * Outputs rois_out (B,S,5), labels (B,S), targets (B,S,4) normalised by means/stds,
 * inside_w, outside_w (B,S,4). */
typedef struct tlod_rcnn_cfg {
  int batch_size;      /* 256 TRAIN.BATCH_SIZE (cfgs/vgg16.yml) */
  float fg_fraction;   /* 0.25 */
  float fg_thresh;     /* 0.5 */
  float bg_thresh_hi;  /* 0.5 */
  float bg_thresh_lo;  /* 0.0 (cfgs/vgg16.yml) */
  float means[4];      /* 0,0,0,0 */
  float stds[4];       /* .1,.1,.2,.2 */
  float inside_weight[4]; /* 1,1,1,1 */
} tlod_rcnn_cfg;

size_t tlod_proposal_target_workspace_bytes(int B, int R, int G);
int tlod_proposal_target_count_f32(const float* rois, int B, int R, const float* gt_boxes,
                                   int G, const tlod_rcnn_cfg* cfg, int32_t* counts,
                                   void* ws, size_t ws_bytes, tlod_stream_t stream);
int tlod_proposal_target_sample_f32(const float* rois, int B, int R, const float* gt_boxes,
                                    int G, const tlod_rcnn_cfg* cfg, const int32_t* fg_perm,
                                    const int32_t* perm_off, const double* rand,
                                    const int32_t* rand_off, uint64_t seed,
                                    float* rois_out, float* labels, float* targets,
                                    float* inside_w, float* outside_w, void* ws,
                                    size_t ws_bytes, tlod_stream_t stream);
int tlod_proposal_target_f32(const float* rois, int B, int R, const float* gt_boxes, int G,
                             const tlod_rcnn_cfg* cfg, uint64_t seed, int32_t* counts,
                             float* rois_out, float* labels, float* targets,
                             float* inside_w, float* outside_w, void* ws, size_t ws_bytes,
                             tlod_stream_t stream);


/* ------------------------------------------------------------------ Convolution
 * Replaces: the cuDNN fp32 convolutions behind the VGG16 backbone and RPN conv
 *   (RCNN_base = torchvision vgg16().features[:-1], lib/DAF/vgg16.py:49; RPN_Conv
 *   lib/model/rpn/rpn.py:28; the DA heads' 1x1 convs lib/DAF/DA.py:40-41).
 * Stride 1, zero padding KS/2, KS in {1, 3}; NCHW fp32, f32-input MFMA (exact f32 FMAs).
 * Weight operands are packed once per weight version:
 *   tlod_conv_pack_fwd_f32  : wk[(ci*KS*KS + s)][co]          = weight[co][ci][s]
 *   tlod_conv_pack_dgrad_f32: wd[(co*KS*KS + s)][ci]          = weight[co][ci][KS*KS-1-s]
 * fwd  : y = conv(x, weight) (+ bias) (then ReLU if relu != 0)      y (N,Cout,H,W)
 * dgrad: dx = conv_transpose(dy, weight)                            dx (N,Cin,H,W)
 * wgrad: dw (+)= sum_n,p dy (x) x-patches, deterministic split-K    dw (Cout,Cin,KS,KS)
 *        (accumulate != 0 adds into dw, like autograd grad accumulation)
 * fwd/dgrad split the input channels over workgroups (deterministic slab reduction) when
 * the output tiles cannot fill the chip; *_workspace_bytes reports the slab size (0 when no
 * split is used).
 * relu_bwd_bias: g = dy * (y > 0) (y may be NULL: g = dy), db = sum over n,h,w of g
 *        (written, not accumulated: no zero fill needed; db may be NULL).  g may alias dy.
 * fwd_ex: y = act(conv * scale[co] + bias[co] + residual) — the ResNet bottleneck epilogue
 *        (frozen BatchNorm folded to scale/bias, lib/DAF/resnet.py:261-284; identity or
 *        downsample branch added before the ReLU, resnet.py:94-97).  Any of scale, bias,
 *        residual may be NULL; residual (N,Cout,H,W) must not alias y.
 * relu_bwd_ex: g0 = dy * (y > 0); g = g0 * scale[c] (scale may be NULL); g_raw = g0 when
 *        g_raw != NULL (the residual branch's gradient); db = sum g0 when db != NULL. */
int tlod_conv_pack_fwd_f32(const float* weight, int Cout, int Cin, int KS, float* wk,
                           tlod_stream_t stream);
int tlod_conv_pack_dgrad_f32(const float* weight, int Cout, int Cin, int KS, float* wd,
                             tlod_stream_t stream);
size_t tlod_conv_fwd_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS);
size_t tlod_conv_dgrad_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS);
int tlod_conv_fwd_f32(const float* x, const float* wk, const float* bias, float* y, int N,
                      int Cin, int H, int W, int Cout, int KS, int relu, void* ws,
                      size_t ws_bytes, tlod_stream_t stream);
int tlod_conv_dgrad_f32(const float* dy, const float* wd, float* dx, int N, int Cin, int H,
                        int W, int Cout, int KS, void* ws, size_t ws_bytes, tlod_stream_t stream);
size_t tlod_conv_wgrad_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS);
int tlod_conv_wgrad_f32(const float* dy, const float* x, float* dw, int accumulate, int N,
                        int Cin, int H, int W, int Cout, int KS, void* ws, size_t ws_bytes,
                        tlod_stream_t stream);
int tlod_relu_bwd_bias_f32(const float* dy, const float* y, float* g, float* db, int N, int C,
                           int HW, tlod_stream_t stream);
int tlod_conv_fwd_ex_f32(const float* x, const float* wk, const float* scale, const float* bias,
                         const float* residual, float* y, int N, int Cin, int H, int W, int Cout,
                         int KS, int relu, void* ws, size_t ws_bytes, tlod_stream_t stream);
int tlod_relu_bwd_ex_f32(const float* dy, const float* y, const float* scale, float* g,
                         float* g_raw, float* db, int N, int C, int HW, tlod_stream_t stream);

/* ------------------------------------------------------------------ Split-bf16 3x3 conv
 * The forward / dgrad of tlod_conv_fwd_f32 on the bf16 MFMA: each f32 operand is split
 * exactly into three bf16 terms (x = hi + mid + lo: hi the truncated top 8 significant bits,
 * mid and lo the round-to-nearest-even bf16 of the remainders) and nprod = 6 products
 * (hi*hi, hi*mid, mid*hi, hi*lo, mid*mid, lo*hi) are accumulated in f32 — error at the
 * level of f32 rounding (normwise ~1e-7 vs fp64, like the f32-input MFMA path) at up to
 * 2.7x its MFMA rate; nprod = 3 (hi*hi, hi*mid, mid*hi) trades that for ~5e-6.
 * Weights are packed (and pre-split) per weight version into three bf16 planes
 * (hi, mid, lo): pack_bs(dgrad=0): P[pl][co][c*80 + s*8 + e] = split(weight[co][8c+e][s])[pl];
 * pack_bs(dgrad=1): P[pl][ci][c*80 + s*8 + e] = split(weight[8c+e][ci][8-s])[pl] (zero for
 * the pad tap s = 9 and past the last channel).  dgrad = tlod_conv_fwd_bs_f32(dy, P_dgrad, ..., Cin := Cout,
 * Cout := Cin).  KS = 3 only. */
size_t tlod_conv_pack_bs_bytes(int Cout, int Cin, int KS, int dgrad);
int tlod_conv_pack_bs(const float* weight, int Cout, int Cin, int KS, int dgrad, void* packed,
                      tlod_stream_t stream);
/* tlod_conv_pack_bs of weight[co] * scale[co] (scale: Cout floats, a frozen BatchNorm's scale
 * after the conv; NULL: 1), the product rounded to f32 before the split. */
int tlod_conv_pack_bs_ex(const float* weight, const float* scale, int Cout, int Cin, int KS,
                         int dgrad, void* packed, tlod_stream_t stream);
size_t tlod_conv_fwd_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS,
                                        int nprod);
int tlod_conv_fwd_bs_f32(const float* x, const void* wp, const float* scale, const float* bias,
                         const float* residual, float* y, int N, int Cin, int H, int W, int Cout,
                         int KS, int relu, int nprod, void* ws, size_t ws_bytes,
                         tlod_stream_t stream);
/* Split-bf16 wgrad: tlod_conv_wgrad_f32's result (same argument meaning, deterministic
 * split-K slab reduction in fixed split order) with dy and x split into bf16 planes on the
 * fly and nprod (6 or 3) products on the bf16 MFMA.  No weight pack.  KS = 1 or 3 (3x3 with
 * nprod = 6: the warp-specialized kernel over 4 x 16 pixel tiles, csrc/wgrad_ws.hip).  db
 * (optional, Cout floats): the bias gradient sum_{n,h,w} dy, from the staged dy rows in the
 * same launch (replaces the bias-gradient half of the ReLU backward pass). */
size_t tlod_conv_wgrad_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout, int KS,
                                          int nprod);
int tlod_conv_wgrad_bs_f32(const float* dy, const float* x, float* dw, float* db, int accumulate,
                           int N, int Cin, int H, int W, int Cout, int KS, int nprod, void* ws,
                           size_t ws_bytes, tlod_stream_t stream);
/* tlod_conv_wgrad_bs_f32 with dW[co] = (accumulate ? dW[co] : 0) + row_scale[co] * (the
 * gradient) (row_scale: Cout floats, may be NULL): a frozen BatchNorm's scale after the conv
 * (ResNet bottlenecks, lib/DAF/resnet.py:80-99) folded into the weight gradient's reduce
 * instead of a pass over dW. */
int tlod_conv_wgrad_bs_ex_f32(const float* dy, const float* x, float* dw, float* db,
                              int accumulate, const float* row_scale, int N, int Cin, int H,
                              int W, int Cout, int KS, int nprod, void* ws, size_t ws_bytes,
                              tlod_stream_t stream);
/* Direct 3x3 conv (stride 1, pad 1) for Cin <= 4 — VGG16 conv1_1 on the image
 * (lib/DAF/vgg16.py:49 features[0]): y = act(conv(x, weight) + bias), weight the nn.Conv2d
 * (Cout, Cin, 3, 3) tensor as is, exact f32 FMA chains (27 per output for Cin = 3). */
int tlod_conv3x3_direct_f32(const float* x, const float* weight, const float* bias, float* y,
                            int N, int Cin, int H, int W, int Cout, int relu,
                            tlod_stream_t stream);
/* Split-bf16 3x3 dgrad with the previous layer's ReLU backward in the epilogue:
 * dx = tlod_conv_fwd_bs_f32(dy, P_dgrad, ...) * (mask > 0), mask (N, Cin, H, W) = the
 * previous conv's ReLU output (this conv's input, lib/DAF/vgg16.py:49 features).  Cin / Cout
 * as in tlod_conv_fwd_bs_f32's dgrad form (Cin := the layer's Cout, Cout := the layer's Cin);
 * workspace: tlod_conv_fwd_bs_workspace_bytes of that form. */
int tlod_conv_dgrad_bs_mask_f32(const float* dy, const void* wp, const float* mask, float* dx,
                                int N, int Cin, int H, int W, int Cout, int nprod, void* ws,
                                size_t ws_bytes, tlod_stream_t stream);

/* ------------------------------------------------------------------ Split-bf16 GEMM
 * Replaces: the cuBLAS fp32 GEMMs of nn.Linear in RCNN_top (fc6/fc7, lib/DAF/vgg16.py:67-71
 *   = torchvision vgg16().classifier[:-1]) and the DA instance head (lib/DAF/DA.py:53-73):
 *   forward x W^T, input gradient dy W and weight gradient dy^T x.
 * c[m][n] = sum_k A(m,k) B(n,k) (+ bias[n], may be NULL), c row-major M x N, contiguous.
 * A(m,k) = a[m*K + k] if a_kcontig else a[k*M + m];  B(n,k) = b[n*K + k] if b_kcontig else
 * b[k*N + n].  Operands split exactly into bf16 planes, nprod (6 or 3) products per f32
 * product on the bf16 MFMA, f32 accumulation; split-K through a caller workspace of
 * tlod_gemm_bs_workspace_bytes (fixed-order reduction: deterministic). */
size_t tlod_gemm_bs_workspace_bytes(int M, int N, int K, int a_kcontig, int b_kcontig, int nprod);
int tlod_gemm_bs_f32(const float* a, const float* b, const float* bias, float* c, int M, int N,
                     int K, int a_kcontig, int b_kcontig, int nprod, void* ws, size_t ws_bytes,
                     tlod_stream_t stream);
/* c = act(A B^T + bias + residual): tlod_gemm_bs_f32 with the ResNet101 RoI head's
 * bottleneck epilogue (lib/DAF/resnet.py Bottleneck.forward: out += residual; relu) fused —
 * residual (M x N, may be NULL, must not alias c), relu 0/1.  Same workspace. */
int tlod_gemm_bs_ex_f32(const float* a, const float* b, const float* bias, const float* residual,
                        int relu, float* c, int M, int N, int K, int a_kcontig, int b_kcontig,
                        int nprod, void* ws, size_t ws_bytes, tlod_stream_t stream);
/* The input gradient of a GEMM whose input is a ReLU output (the ResNet RoI head's bottleneck
 * convs as GEMMs, lib/DAF/resnet.py Bottleneck.backward through relu(bn1(conv1(x))) ...):
 * c = (a.b + residual) * (mask > 0) — residual (M x N, may be NULL): the identity shortcut's
 * gradient added first; mask (M x N): the ReLU output the GEMM's input is.  One GEMM instead
 * of the GEMM, autograd's sum of the two gradients and a ReLU-backward pass.  Same
 * workspace as tlod_gemm_bs_f32; residual and mask must not alias c. */
int tlod_gemm_bs_mask_f32(const float* a, const float* b, const float* residual,
                          const float* mask, float* c, int M, int N, int K, int a_kcontig,
                          int b_kcontig, int nprod, void* ws, size_t ws_bytes,
                          tlod_stream_t stream);

/* The ResNet RoI head's 3x3 conv (layer4's bottleneck conv2 on the RoIs' 4 x 4 maps,
 * lib/DAF/resnet.py:66-102 via RCNN_top :286-288; the reference runs nn.Conv2d / cuDNN) as
 * an implicit split-bf16 GEMM over channels-last maps: the (R H W) x 9 C im2col matrix, taps
 * in (kh, kw, c) order with zero padding 1, is never materialised (it replaces
 * tlod_im2col3x3_nhwc_f32 + tlod_gemm_bs_* and, for the input gradient,
 * tlod_col2im3x3_nhwc_mask_f32).  Maps: R maps of H x W, channels-last rows (R H W, .).
 *   mode 0 (forward):        c (R H W, O) = act(im2col(a) . b^T + bias (+ residual));
 *                            a = x (R H W, C), b = the weight rows (O, 9 C) in (kh, kw, c)
 *                            order; C % 16 == 0
 *   mode 1 (input gradient): c (R H W, C) = (im2col(a) . b (+ residual)) * (mask > 0 if mask);
 *                            a = dy (R H W, O), b = (9 O, C): row (t, o) = weight row o at tap
 *                            8 - t (the flipped kernel); O % 16 == 0
 *   mode 2 (weight grad):    c (O, 9 C) = a^T . im2col(b); a = dy (R H W, O), b = x; C % 256
 *                            == 0; no epilogue (bias, residual, mask NULL, relu 0)
 * Split-K pieces reduced in a fixed order (deterministic); workspace:
 * tlod_gemm_nhwc3_bs_workspace_bytes(mode, ...). */
size_t tlod_gemm_nhwc3_bs_workspace_bytes(int mode, int R, int H, int W, int C, int O, int nprod);
int tlod_gemm_nhwc3_bs_f32(int mode, const float* a, const float* b, const float* bias,
                           const float* residual, const float* mask, int relu, float* c, int R,
                           int H, int W, int C, int O, int nprod, void* ws, size_t ws_bytes,
                           tlod_stream_t stream);

/* Split-bf16 3x3 convolution as an implicit GEMM over (c, tap) x flattened pixels, for
 * wide outputs (Cout >= 256): the forward of tlod_conv_fwd_ex_f32 (w_layout = 0: w is the
 * nn.Conv2d weight [Cout][Cin][3][3] as is) or the dgrad (w_layout = 1: w is
 * tlod_conv_pack_dgrad_f32's [(co*9 + s)][ci] pack, x = dy, Cin := the layer's Cout,
 * Cout := the layer's Cin).  y = act(conv * scale + bias + residual), every epilogue
 * pointer optional.  Workspace: tlod_conv3x3_gemm_bs_workspace_bytes (split-K slabs). */
size_t tlod_conv3x3_gemm_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout,
                                            int w_layout, int nprod);
int tlod_conv3x3_gemm_bs_f32(const float* x, const float* w, int w_layout, const float* scale,
                             const float* bias, const float* residual, float* y, int N, int Cin,
                             int H, int W, int Cout, int relu, int nprod, void* ws,
                             size_t ws_bytes, tlod_stream_t stream);
/* The same for 1x1 convolutions (replaces the cuDNN 1x1 convs of the ResNet101 bottlenecks,
 * lib/DAF/resnet.py:64-102 — conv1 / conv3 / downsample, with the frozen BatchNorm folded into
 * scale / bias and the residual add + ReLU of conv3 in the epilogue — and the DA heads'
 * 1x1 convs, lib/DAF/DA.py:19-33): per image y = W (Cout x Cin) . x (Cin x H*W).  w_layout =
 * 0: w is the nn.Conv2d weight (Cout, Cin, 1, 1) (forward); 1: the input gradient, x = dy,
 * w the same (layer Cout, layer Cin) weight read transposed, Cin := the layer's Cout,
 * Cout := the layer's Cin.  Output-channel tiles of 64 / 128 / 256 rows, whichever fills the
 * chip best (conv1x1_mi). */
size_t tlod_conv1x1_gemm_bs_workspace_bytes(int N, int Cin, int H, int W, int Cout,
                                            int w_layout, int nprod);
int tlod_conv1x1_gemm_bs_f32(const float* x, const float* w, int w_layout, const float* scale,
                             const float* bias, const float* residual, float* y, int N, int Cin,
                             int H, int W, int Cout, int relu, int nprod, void* ws,
                             size_t ws_bytes, tlod_stream_t stream);
/* tlod_conv1x1_gemm_bs_f32 with a final y *= (mask > 0) (mask (N, Cout, H, W), may be NULL,
 * must not alias y): the dgrad form (w_layout = 1) of a ResNet bottleneck conv1 / conv3 with
 * the previous layer's ReLU backward in the epilogue, after the residual (the identity
 * shortcut's gradient) is added.  w_scale (w_layout = 1 only, may be NULL): the weight taken as
 * W[co][ci] * w_scale[co] (a frozen BatchNorm's scale after the conv), applied as it is
 * staged.  Same workspace. */
int tlod_conv1x1_gemm_bs_ex_f32(const float* x, const float* w, int w_layout, const float* scale,
                                const float* bias, const float* residual, const float* mask,
                                const float* w_scale, float* y, int N, int Cin, int H, int W,
                                int Cout, int relu, int nprod, void* ws, size_t ws_bytes,
                                tlod_stream_t stream);

/* 1x1 convolutions with 1 <= Cout <= 4, NCHW f32 (stride 1): the image-level domain
 * classifier's last layer, _ImageDA.Conv2 = nn.Conv2d(512, 2, 1, bias=False)
 * (lib/DAF/DA.py:36-50; ATF: three of them, on layer1 / layer2 / layer3 maps,
 * lib/ATF/faster_rcnn.py).  Streaming kernels, deterministic (fixed summation orders).
 * fwd: y (N, Cout, H, W) = weight (Cout, Cin) . x (+ bias[Cout], may be NULL).
 * dgrad: dx (N, Cin, H, W) = weight^T . dy (written, not accumulated).
 * wgrad: dweight (Cout, Cin) and dbias (Cout, may be NULL) written (not accumulated);
 * workspace from tlod_conv1x1_small_wgrad_workspace_bytes. */
int tlod_conv1x1_small_fwd_f32(const float* x, int N, int Cin, int H, int W, const float* weight,
                               const float* bias, int Cout, float* y, tlod_stream_t stream);
int tlod_conv1x1_small_dgrad_f32(const float* dy, int N, int Cout, int H, int W,
                                 const float* weight, int Cin, float* dx, tlod_stream_t stream);
size_t tlod_conv1x1_small_wgrad_workspace_bytes(int N, int Cin, int H, int W, int Cout);
int tlod_conv1x1_small_wgrad_f32(const float* dy, const float* x, int N, int Cin, int H, int W,
                                 int Cout, float* dweight, float* dbias, void* ws,
                                 size_t ws_bytes, tlod_stream_t stream);

/* ------------------------------------------------------------------ Max pooling
 * Replaces: nn.MaxPool2d(kernel_size=2, stride=2) (floor mode) in RCNN_base (torchvision
 *   vgg16().features, lib/DAF/vgg16.py:49) and, backward, its routing fused with the
 *   preceding conv's ReLU backward.
 * maxpool2x2: y (N,C,H/2,W/2) = window max, torch's tie rule (first max, NaN wins).
 * maxpool2x2_relu_bwd: y = the pool input (the conv's ReLU output, (N,C,H,W)), dp the
 *   pooled gradient; g (N,C,H,W) = dp routed to each window's argmax (recomputed from y with
 *   max_pool2d's rule) where y > 0, else 0; db[c] = sum of g (written; db may be NULL).
 * conv_fwd_bs_pool: tlod_conv_fwd_bs_f32 followed by maxpool2x2 in the kernel epilogue
 *   (the full-resolution map is never written): y_pooled (N,Cout,H/2,W/2).  For frozen
 *   layers whose output only feeds the pool (VGG16 conv1_2 / conv2_2). */
int tlod_maxpool2x2_f32(const float* x, int N, int C, int H, int W, float* y,
                        tlod_stream_t stream);
int tlod_maxpool2x2_relu_bwd_f32(const float* dp, const float* y, int N, int C, int H, int W,
                                 float* g, float* db, tlod_stream_t stream);
int tlod_conv_fwd_bs_pool_f32(const float* x, const void* wp, const float* scale,
                              const float* bias, float* y_pooled, int N, int Cin, int H, int W,
                              int Cout, int KS, int relu, int nprod, tlod_stream_t stream);

/* ------------------------------------------------------------------ ResNet101 extras
 * Replaces: cuDNN for the ResNet101 stem conv1 7x7/2 + bn1 + relu (lib/DAF/resnet.py:107-110,
 *   frozen, forward only) and the stride-2 1x1 convolutions of the caffe-style bottleneck
 *   (resnet.py:71 conv1 stride, :133-135 downsample).
 * stem: x (N,3,H,W) -> y (N,64,Ho,Wo), Ho = (H-1)/2+1; weight (64,3,7,7); y = act(conv *
 *   scale + bias) (scale/bias: folded bn1, may be NULL).
 * subsample2: y = x[:, :, ::2, ::2]  (N,C,(H+1)/2,(W+1)/2) — a stride-2 1x1 conv is the
 *   stride-1 conv of this; upsample2_zero is its adjoint (dx (N,C,H,W), zeros off-grid). */
int tlod_stem_conv7x7s2_f32(const float* x, const float* weight, const float* scale,
                            const float* bias, float* y, int N, int H, int W, int relu,
                            tlod_stream_t stream);
int tlod_subsample2_f32(const float* x, int N, int C, int H, int W, float* y,
                        tlod_stream_t stream);
int tlod_upsample2_zero_f32(const float* dy, int N, int C, int H, int W, float* dx,
                            tlod_stream_t stream);
/* RoI head (layer4 on R RoI maps, lib/DAF/resnet.py:64-102 applied by RCNN_top, :277-288)
 * channels-last 3x3 convs as GEMMs: col[(r,h,w)][(kh,kw,c)] = x[r][h+kh-1][w+kw-1][c]
 * (zero padding 1), x (R,H,W,C), col (R*H*W, 9*C); col2im is its adjoint (dx = sum over the
 * 9 taps, in (kh,kw) order).  C % 4 == 0, 16-B aligned. */
int tlod_im2col3x3_nhwc_f32(const float* x, int R, int H, int W, int C, float* col,
                            tlod_stream_t stream);
int tlod_col2im3x3_nhwc_f32(const float* col, int R, int H, int W, int C, float* dx,
                            tlod_stream_t stream);
/* col2im with the previous layer's ReLU backward: dx = col2im(col) * (mask > 0), mask the
 * (R, H, W, C) ReLU output that was im2col's input (may be NULL). */
int tlod_col2im3x3_nhwc_mask_f32(const float* col, int R, int H, int W, int C, const float* mask,
                                 float* dx, tlod_stream_t stream);


/* ------------------------------------------------------------------ Optimiser step
 * Replaces: clip_gradient(model, 10.) lib/model/utils/net_utils.py:38-49 (per-param norm
 *   loop + .item() host sync) + torch.optim.SGD(momentum) methods/DAF/DAF_train.py:323,408.
 * chunks: device array of n_chunks descriptors (each <= 65536 elements of one tensor);
 * per element: g = grad_scale * grad (data parallel: 1/world of the all-reduced sum, the
 * DataParallel loss.mean() semantics; 1 otherwise); g' = g * clip/max(||g||, clip);
 * d = g' + wd*p; buf = m*buf + d; p -= lr*buf
 * (torch SGD semantics, dampening 0; buf starts at 0, so step 1 gives buf = d).
 * clip_norm <= 0 disables clipping.  partials: float[n_chunks] scratch.  norm_scale: 2
 * device floats receiving (total grad norm, applied scale).  Deterministic.
 * active: NULL, or a device float; a chunk whose *active == 0 is left untouched (data
 * parallel: the number of ranks that produced the gradient, all-reduced with it — a
 * parameter no rank used is skipped like a None .grad in torch.optim.SGD; its gradient
 * slot is zero, so it adds nothing to the norm).
 * count < 0: the chunk's -count elements only enter the gradient norm (their parameter is
 * updated by tlod_sgd_clip_pack_f32's tiles), so a table lists every parameter in one order
 * whether or not packs are kept. */
typedef struct tlod_sgd_chunk {
  float* param;
  const float* grad;
  float* momentum_buf;
  long long count;
  float lr;
  float weight_decay;
  const float* active;
} tlod_sgd_chunk;

int tlod_sgd_clip_f32(const tlod_sgd_chunk* chunks, int n_chunks, float grad_scale,
                      float momentum, float clip_norm, float* partials, float* norm_scale,
                      tlod_stream_t stream);

/* The same step with the split-bf16 weight packs of 3x3 conv weights written by the update
 * itself (no per-weight tlod_conv_pack_bs launches before the next forward / backward).
 * chunks[0, n_update) are updated as above (except norm-only rows, count < 0);
 * chunks[n_update, n_chunks) only enter the gradient norm: their parameters are the 3x3
 * weights the tiles update.  A tile is 32 output
 * x 32 input channels x 9 taps of one (cout, cin, 3, 3) weight (o0, i0: its first output /
 * input channel, multiples of 32); it applies the SGD update to its elements and stores the
 * new weights into each non-NULL pack — pack_fwd: the tlod_conv_pack_bs(dgrad = 0) layout,
 * pack_dgrad: dgrad = 1, pack_dgrad_scaled: tlod_conv_pack_bs_ex(scale, dgrad = 1) — bit
 * for bit what those functions would produce from the updated weight.  The packs must have
 * been made once by those functions (the tiles do not write their zero padding).  active as
 * for chunks (the tile, weight and packs are left untouched). */
typedef struct tlod_sgd_pack_tile {
  float* param;
  const float* grad;
  float* momentum_buf;
  const float* active;
  unsigned short* pack_fwd;
  unsigned short* pack_dgrad;
  unsigned short* pack_dgrad_scaled;
  const float* scale;
  float lr;
  float weight_decay;
  int cout, cin;
  int o0, i0;
  int reserved[2];
} tlod_sgd_pack_tile;

int tlod_sgd_clip_pack_f32(const tlod_sgd_chunk* chunks, int n_chunks, int n_update,
                           const tlod_sgd_pack_tile* tiles, int n_tiles, float grad_scale,
                           float momentum, float clip_norm, float* partials, float* norm_scale,
                           tlod_stream_t stream);

/* ------------------------------------------------------------------ Input blob
 * Replaces: the data layer's per-image host chain — scipy imread (RGB) -> BGR -> flip
 *   (lib/roi_data_layer/minibatch.py:62-82) -> astype(float32) -= PIXEL_MEANS ->
 *   cv2.resize(fx = fy = im_scale, INTER_LINEAR) (lib/model/utils/blob.py:35-52) -> crop /
 *   zero-pad to the aspect group's shape, HWC -> CHW (lib/roi_data_layer/roibatchLoader.py:
 *   94-207).  src: decoded RGB image, H x W x 3 uint8 on the device.  lut: 3 x 256 float,
 *   lut[c*256 + v] = float32(v - PIXEL_MEANS[c]) for BGR channel c (rounded once from
 *   double, as numpy's in-place float32 -= float64).  xtab (Wr entries) / ytab (Hr
 *   entries): device arrays of {int i0, int i1, float w0, float w1} — the cv::resize
 *   INTER_LINEAR source index pair and weights of each resized column / row, flip already
 *   applied to the column indices; every index must lie in [0, W) / [0, H) (the host
 *   builds them, tlod/data/blob.py).  The kept region is Hd x Wd at (y0, x0) of the Hr x Wr
 *   resized image (y0 + Hd <= Hr, x0 + Wd <= Wr).  out: 3 x Ho x Wo float32,
 *   out[c][y][x] = resized[y + y0][x + x0][c] for y < Hd, x < Wd, else 0 (zero padding). */
int tlod_image_blob_u8(const uint8_t* src, int H, int W, const float* lut, const void* xtab,
                       const void* ytab, int Hr, int Wr, int y0, int x0, int Hd, int Wd, int Ho,
                       int Wo, float* out, tlod_stream_t stream);

/* ------------------------------------------------------------------ Test-time detections
 * Replaces: the per-class loop of the test drivers (methods/DAF/DAF_test.py:282-321): box
 *   deltas * BBOX_NORMALIZE_STDS + MEANS, bbox_transform_inv + clip_boxes
 *   (lib/model/rpn/bbox_transform.py:77-103, :125-133), / im_scale, then per class j >= 1
 *   scores > score_thresh, descending sort, nms(TEST.NMS) (nms_cuda_kernel.cu semantics).
 * rois (R, 5) of one image, cls_prob (R, C), bbox_pred (R, 4C) (or (R, 4) when
 * class_agnostic); stds / means: 4 floats each in HOST memory; im_h, im_w: im_info[0:2].
 * R <= 2048.  dets (C, R, 5) receives, for class j, counts[j] rows (x1, y1, x2, y2, score)
 * in descending score order (ties: lower RoI index first); counts[0] = 0.  boxes_out
 * (R, C, 4), optional (NULL to skip): every decoded, clipped, rescaled box. */
int tlod_detect_f32(const float* rois, const float* cls_prob, const float* bbox_pred, int R,
                    int C, int class_agnostic, const float* stds, const float* means, float im_h,
                    float im_w, float im_scale, float score_thresh, float nms_thresh, float* dets,
                    int32_t* counts, float* boxes_out, tlod_stream_t stream);

/* ------------------------------------------------------------------ MAF DRM
 * Replaces: the chunk / reshape / cat loops of DRM.forward, lib/MAF/drm.py:23-40 (a
 *   Python double loop over (H/s)*(W/s) chunks).  x: (B, C, H, W); the map is cropped
 *   to Ho = floor(H/s), Wo = floor(W/s) blocks (drm.py:23-26) and
 *   y[b, c*s*s + i*s + j, h, w] = x[b, c, h*s + i, w*s + j]   (y: B x C*s*s x Ho x Wo),
 *   i.e. pixel_unshuffle of the cropped map.  depth_to_space is its adjoint: dx gets dy
 *   scattered back and zeros on the cropped-away border. */
int tlod_space_to_depth_f32(const float* x, int B, int C, int H, int W, int scale, float* y,
                            tlod_stream_t stream);
int tlod_depth_to_space_f32(const float* dy, int B, int C, int H, int W, int scale, float* dx,
                            tlod_stream_t stream);
/* The whole DRM forward, lib/MAF/drm.py:10-42 (conv_low_dim 1x1 without bias -> ReLU ->
 * crop -> space-to-depth) as one conv launch whose epilogue stores each ReLU output at its
 * space-to-depth position: x (N, Cin, H, W), wk = tlod_conv_pack_fwd_f32 of the (Cout, Cin,
 * 1, 1) weight, y (N, Cout*s*s, H/s, W/s); the full-resolution map is never written.  ws:
 * tlod_conv_fwd_workspace_bytes(N, Cin, H, W, Cout, 1).  tlod_drm_relu_bwd_f32 is its
 * backward up to the conv, in one pass: g (N, Cout, H, W) = depth_to_space(dy * (y > 0))
 * (0 on the cropped border) — the gradient that conv_low_dim's dgrad / wgrad consume. */
int tlod_drm_fwd_f32(const float* x, const float* wk, float* y, int N, int Cin, int H, int W,
                     int Cout, int scale, void* ws, size_t ws_bytes, tlod_stream_t stream);
int tlod_drm_relu_bwd_f32(const float* dy, const float* y, int B, int C, int H, int W, int scale,
                          float* g, tlod_stream_t stream);

/* ------------------------------------------------------------------ FC head activation
 * Replaces: nn.ReLU(inplace) + nn.Dropout(p) after the head's Linear layers
 *   (lib/DAF/vgg16.py:67-71, lib/DAF/DA.py:53-73).  out = y > 0 and kept ? y / (1 - p) : 0,
 *   kept <=> a counter-based uniform(seed, i) >= p (p = 0: plain ReLU).  Backward:
 *   g = out > 0 ? dout / (1 - p) : 0 (the mask is recovered from out, never stored). */
int tlod_relu_dropout_f32(const float* y, float* out, long long n, float p,
                          unsigned long long seed, tlod_stream_t stream);
/* Backward precondition: dout, out and g are 16-byte aligned (float4 path); else the
 * call returns an argument error.  NaN inputs pass through both ways (torch semantics). */
int tlod_relu_dropout_bwd_f32(const float* dout, const float* out, float* g, long long n,
                              float p, tlod_stream_t stream);

/* ------------------------------------------------------------------ Fused losses
 * One forward launch (single workgroup, fixed-order double accumulation: deterministic)
 * and one backward launch (writes every gradient element) per loss family.  grad_loss
 * points to the upstream gradients of the scalar losses on the device (no host sync).
 *
 * RPN (lib/model/rpn/rpn.py:89-108): score = RPN_cls_score (B, 2A, H, W) — the
 *   reference's score_reshape (B, 2, A*H, W) permuted to 2-column rows; labels
 *   (B, 1, A*H, W) in {-1, 0, 1}; bbox / targets / inside / outside (B, 4A, H, W).
 *   loss[0] = cross entropy averaged over rows with label != -1 (the reference
 *   index_selects them with nonzero(), a host sync; count[0] = max(kept, 1) is saved for
 *   the backward); loss[1] = _smooth_l1_loss(sigma, dim=[1,2,3]) (net_utils.py:72-86).
 *   Backward: score / bbox may hold B_total >= B images of which the first B are the
 *   loss's; dscore (B_total, 2A, H, W) and dbbox (B_total, 4A, H, W) are written in full
 *   (zero past image B). */
/* Precondition (both RPN calls): bbox, targets, inside and outside are contiguous
 * (B, 4A, H, W) tensors at 16-byte aligned addresses (the box terms are read as float4);
 * a misaligned pointer returns an argument error. */
int tlod_rpn_loss_f32(const float* score, const float* labels, const float* bbox,
                      const float* targets, const float* inside, const float* outside, int B,
                      int A, int H, int W, float sigma, float* loss, float* count,
                      tlod_stream_t stream);
int tlod_rpn_loss_bwd_f32(const float* score, const float* labels, const float* bbox,
                          const float* targets, const float* inside, const float* outside,
                          int B, int B_total, int A, int H, int W, float sigma,
                          const float* grad_loss, const float* count, float* dscore,
                          float* dbbox, tlod_stream_t stream);
/* RCNN head (lib/DAF/faster_rcnn.py:158-177): cls_score (R, C), bbox_pred (R, 4C) or
 *   (R, 4) when agnostic, labels int64 (R) in [0, C).  cls_prob = softmax(cls_score);
 *   bbox_sel (R, 4) = bbox_pred gathered at the label's 4 columns (may be NULL);
 *   loss[0] = F.cross_entropy, loss[1] = _smooth_l1_loss(sigma, dim=[1]).  Backward:
 *   cls_score / bbox_pred may hold R_total >= R rows of which the first R are the loss's;
 *   dcls (R_total, C) and dbbox (R_total, 4C | 4) are written in full (zeros off the
 *   label's columns and past row R). */
int tlod_rcnn_loss_f32(const float* cls_score, const float* bbox_pred, const long long* labels,
                       const float* targets, const float* inside, const float* outside, int R,
                       int C, int agnostic, float sigma, float* cls_prob, float* bbox_sel,
                       float* loss, tlod_stream_t stream);
int tlod_rcnn_loss_bwd_f32(const float* cls_prob, const float* bbox_pred,
                           const long long* labels, const float* targets, const float* inside,
                           const float* outside, int R, int R_total, int C, int agnostic,
                           float sigma, const float* grad_loss, float* dcls, float* dbbox,
                           tlod_stream_t stream);
/* DAF domain losses (lib/DAF/faster_rcnn.py:181-220) for the source (s) and target (t)
 *   domains: image-level logits score (B, 2, H, W), need_backprop (B) float (the image
 *   label, ImageLabelResizeLayer), instance sigmoid outputs ins (n) with the
 *   InstanceLabelResizeLayer labels (1, rows [256 i, 256 (i+1)) := need[i]).
 *   loss[0..2] = source (nll(log_softmax), binary_cross_entropy, MSE-sum consistency
 *   against softmax(score_s)[:,1].mean()), loss[3..5] = target (same, channel 0);
 *   cons[2] = the two detached softmax means (saved for the backward). */
int tlod_da_loss_f32(const float* score_s, const float* score_t, const float* need_s,
                     const float* need_t, const float* ins_s, const float* ins_t, int Bs,
                     int Bt, int Hs, int Ws, int Ht, int Wt, int n_s, int n_t, float* loss,
                     float* cons, tlod_stream_t stream);
int tlod_da_loss_bwd_f32(const float* score_s, const float* score_t, const float* need_s,
                         const float* need_t, const float* ins_s, const float* ins_t, int Bs,
                         int Bt, int Hs, int Ws, int Ht, int Wt, int n_s, int n_t,
                         const float* grad_loss, const float* cons, float* dscore_s,
                         float* dscore_t, float* dins_s, float* dins_t, tlod_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TLOD_H_ */
