// Fused detector / domain-adaptation losses, forward and backward.
//
// The reference builds each loss from a chain of small torch ops (softmax, index_select,
// cross_entropy, pow, abs, comparisons, sums, means, ...; lib/model/rpn/rpn.py:89-108,
// lib/model/utils/net_utils.py:72-86, lib/DAF/faster_rcnn.py:158-220), which in a training
// step is ~200 launches, each a few microseconds of GPU time and ~10 us of host time.  Here
// each family is one forward launch (one workgroup per reduction, fixed-order double
// accumulation: deterministic) and one backward launch that writes every gradient element
// (no zero fill).  Upstream gradients of the scalar losses are read from device memory, so
// nothing synchronises with the host.
#include <algorithm>

#include "common.h"
#include "tlod.h"

namespace tlod {
namespace {

constexpr int kRedThreads = 1024;

// Block-wide sum of NV doubles (every thread gets the totals).
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_down(v[k], o);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) sh[wave * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int w = 0; w < nw; ++w) s += sh[w * NV + k];
    v[k] = s;
  }
  __syncthreads();
}

// Smooth-L1 term of _smooth_l1_loss (net_utils.py:72-86) for one element and its
// derivative with respect to the prediction.
__device__ __forceinline__ float smooth_l1(float pred, float tgt, float in_w, float out_w,
                                           float s2, float* dpred) {
  const float d = in_w * (pred - tgt);
  const float ad = fabsf(d);
  const bool quad = ad < 1.f / s2;
  const float l = quad ? d * d * (s2 * 0.5f) : ad - 0.5f / s2;
  if (dpred) *dpred = out_w * (quad ? s2 * d : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f))) * in_w;
  return out_w * l;
}

// 2-way log_softmax in torch's form: ls_c = (x_c - m) - log(exp(x0-m) + exp(x1-m)) (the
// shift is subtracted before the log term is, so a near-certain class keeps its tiny loss).
struct LogSoftmax2 {
  float l0, l1;
  __device__ __forceinline__ LogSoftmax2(float a, float b) {
    const float m = fmaxf(a, b);
    const float lz = logf(expf(a - m) + expf(b - m));
    l0 = (a - m) - lz;
    l1 = (b - m) - lz;
  }
};

// ------------------------------------------------------------------ RPN
// score (B, 2A, H, W) raw RPN_cls_score: the reference's score_reshape (B, 2, A*H, W)
// permuted to rows ((b, a*H + h, w), class), so for row r of image b at in-image offset q,
// class c is score[b*2*AHW + c*AHW + q]; labels (B, 1, A*H, W) in the same row order.
__global__ void __launch_bounds__(kRedThreads)
rpn_loss_fwd_kernel(const float* __restrict__ score, const float* __restrict__ labels,
                    const float* __restrict__ bbox, const float* __restrict__ tgt,
                    const float* __restrict__ inw, const float* __restrict__ outw, int B,
                    int AHW, float s2, float* __restrict__ loss, float* __restrict__ count) {
  __shared__ double sh[16 * 3];
  double v[3] = {0.0, 0.0, 0.0};  // ce sum, kept rows, smooth-l1 sum
  const long long rows = (long long)B * AHW;
  // one workgroup (fixed-order reduction); 4 rows in flight per thread so the label loads
  // of a mostly-ignored (-1) anchor set do not serialise on memory latency
  for (long long r0 = threadIdx.x; r0 < rows; r0 += 4LL * blockDim.x) {
    float lab[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long r = r0 + (long long)u * blockDim.x;
      lab[u] = r < rows ? labels[r] : -1.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (lab[u] == -1.f) continue;
      const long long r = r0 + (long long)u * blockDim.x;
      const long long b = r / AHW, q = r - b * AHW;
      const float s0 = score[b * 2 * AHW + q], s1 = score[b * 2 * AHW + AHW + q];
      const LogSoftmax2 ls(s0, s1);
      v[0] -= (double)((long long)lab[u] == 1 ? ls.l1 : ls.l0);
      v[1] += 1.0;
    }
  }
  // box terms: rows x 4 contiguous floats per operand, read as float4 (torch allocations
  // are 16-B aligned)
  const float4* b4 = reinterpret_cast<const float4*>(bbox);
  const float4* t4 = reinterpret_cast<const float4*>(tgt);
  const float4* i4 = reinterpret_cast<const float4*>(inw);
  const float4* o4 = reinterpret_cast<const float4*>(outw);
  for (long long i = threadIdx.x; i < rows; i += blockDim.x) {
    const float4 p = b4[i], t = t4[i], iw = i4[i], ow = o4[i];
    v[2] += (double)smooth_l1(p.x, t.x, iw.x, ow.x, s2, nullptr);
    v[2] += (double)smooth_l1(p.y, t.y, iw.y, ow.y, s2, nullptr);
    v[2] += (double)smooth_l1(p.z, t.z, iw.z, ow.z, s2, nullptr);
    v[2] += (double)smooth_l1(p.w, t.w, iw.w, ow.w, s2, nullptr);
  }
  block_sum<3>(v, sh);
  if (threadIdx.x == 0) {
    const double kept = v[1] > 1.0 ? v[1] : 1.0;
    loss[0] = (float)(v[0] / kept);
    loss[1] = (float)(v[2] / B);
    count[0] = (float)kept;
  }
}

__global__ void __launch_bounds__(256)
rpn_loss_bwd_kernel(const float* __restrict__ score, const float* __restrict__ labels,
                    const float* __restrict__ bbox, const float* __restrict__ tgt,
                    const float* __restrict__ inw, const float* __restrict__ outw, int B,
                    int B_total, int AHW, float s2, const float* __restrict__ gloss,
                    const float* __restrict__ count, float* __restrict__ dscore,
                    float* __restrict__ dbbox) {
  // images B .. B_total-1 of score / bbox take no part in the loss: zero gradient
  const long long rows = (long long)B_total * AHW, lrows = (long long)B * AHW;
  const long long ne = rows * 4, lne = lrows * 4;
  const float gc = gloss[0] / count[0], gb = gloss[1] / B;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < rows + ne;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < rows) {
      const long long b = i / AHW, q = i - b * AHW;
      const long long i0 = b * 2 * AHW + q, i1 = i0 + AHW;
      const float lab = i < lrows ? labels[i] : -1.f;
      float d0 = 0.f, d1 = 0.f;
      if (lab != -1.f) {
        const float s0 = score[i0], s1 = score[i1];
        const LogSoftmax2 ls(s0, s1);
        const float p0 = expf(ls.l0), p1 = expf(ls.l1);
        const bool one = (long long)lab == 1;
        d0 = gc * (p0 - (one ? 0.f : 1.f));
        d1 = gc * (p1 - (one ? 1.f : 0.f));
      }
      dscore[i0] = d0;
      dscore[i1] = d1;
    } else {
      const long long e = i - rows;
      float dp = 0.f;
      if (e < lne) smooth_l1(bbox[e], tgt[e], inw[e], outw[e], s2, &dp);
      dbbox[e] = gb * dp;
    }
  }
}

// ------------------------------------------------------------------ RCNN
// cls (R, C), box (R, 4C) (class-specific) or (R, 4) (agnostic), labels int64 (R).
__global__ void __launch_bounds__(kRedThreads)
rcnn_loss_fwd_kernel(const float* __restrict__ cls, const float* __restrict__ box,
                     const long long* __restrict__ labels, const float* __restrict__ tgt,
                     const float* __restrict__ inw, const float* __restrict__ outw, int R,
                     int C, int agnostic, float s2, float* __restrict__ prob,
                     float* __restrict__ box_sel, float* __restrict__ loss) {
  __shared__ double sh[16 * 2];
  double v[2] = {0.0, 0.0};
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const float* s = cls + (size_t)r * C;
    float m = s[0];
    for (int c = 1; c < C; ++c) m = fmaxf(m, s[c]);
    float z = 0.f;
    for (int c = 0; c < C; ++c) z += expf(s[c] - m);
    const float lz = logf(z);
    for (int c = 0; c < C; ++c) prob[(size_t)r * C + c] = expf(s[c] - m) / z;
    long long lab = labels[r];
    lab = lab < 0 || lab >= C ? 0 : lab;  // labels come from the proposal target: [0, C)
    v[0] -= (double)((s[lab] - m) - lz);
    const float* bp = box + (agnostic ? (size_t)r * 4 : (size_t)r * 4 * C + 4 * lab);
    for (int k = 0; k < 4; ++k) {
      const float p = bp[k];
      if (box_sel) box_sel[(size_t)r * 4 + k] = p;
      v[1] += (double)smooth_l1(p, tgt[r * 4 + k], inw[r * 4 + k], outw[r * 4 + k], s2, nullptr);
    }
  }
  block_sum<2>(v, sh);
  if (threadIdx.x == 0) {
    loss[0] = (float)(v[0] / R);
    loss[1] = (float)(v[1] / R);
  }
}

__global__ void __launch_bounds__(256)
rcnn_loss_bwd_kernel(const float* __restrict__ prob, const float* __restrict__ box,
                     const long long* __restrict__ labels, const float* __restrict__ tgt,
                     const float* __restrict__ inw, const float* __restrict__ outw, int R,
                     int R_total, int C, int agnostic, float s2,
                     const float* __restrict__ gloss, float* __restrict__ dcls,
                     float* __restrict__ dbox) {
  // rows R .. R_total-1 of cls_score / bbox_pred take no part in the loss: zero gradient
  const float gc = gloss[0] / R, gb = gloss[1] / R;
  const int BW = agnostic ? 4 : 4 * C;
  const long long nc = (long long)R_total * C, nb = (long long)R_total * BW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nc + nb;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < nc) {
      const int r = (int)(i / C), c = (int)(i - (long long)r * C);
      if (r >= R) {
        dcls[i] = 0.f;
        continue;
      }
      const long long l = labels[r];
      dcls[i] = gc * (prob[i] - ((l < 0 || l >= C ? 0 : l) == c ? 1.f : 0.f));
    } else {
      const long long e = i - nc;
      const int r = (int)(e / BW), j = (int)(e - (long long)r * BW);
      if (r >= R) {
        dbox[e] = 0.f;
        continue;
      }
      const long long l = labels[r];
      const int lab = agnostic || l < 0 || l >= C ? 0 : (int)l;
      float d = 0.f;
      if (j / 4 == lab) {
        const int k = j & 3;
        smooth_l1(box[e], tgt[r * 4 + k], inw[r * 4 + k], outw[r * 4 + k], s2, &d);
        d *= gb;
      }
      dbox[e] = d;
    }
  }
}

// ------------------------------------------------------------------ DA (DAF)
struct DaDomain {
  const float* score;  // (B, 2, H, W) image-level domain logits
  const float* need;   // (B) need_backprop: the image label, .long()
  const float* ins;    // (n) instance sigmoid outputs
  float* dscore;
  float* dins;
  int B, HW, n;
  int cons_ch;         // softmax channel averaged for the consistency target
};

struct DaArgs {
  DaDomain d[2];
  int minibatch;       // InstanceLabelResizeLayer's 256-row blocks
};

// Instance label (LabelResizeLayer.py:41-57): 1, except rows [i*mb, (i+1)*mb) := need[i].
__device__ __forceinline__ float ins_label(const DaDomain& d, int r, int mb) {
  const int i = r / mb;
  return i < d.B ? d.need[i] : 1.f;
}

// One workgroup per domain; loss[3*dom + {0,1,2}] = image nll, instance BCE, consistency
// MSE (sum); cons[dom] = the detached softmax mean (saved for the backward).
__global__ void __launch_bounds__(kRedThreads)
da_loss_fwd_kernel(DaArgs a, float* __restrict__ loss, float* __restrict__ cons) {
  __shared__ double sh[16 * 2];
  const DaDomain d = a.d[blockIdx.x];
  double v[2] = {0.0, 0.0};  // nll sum, softmax[cons_ch] sum
  const long long npix = (long long)d.B * d.HW;
  for (long long p = threadIdx.x; p < npix; p += blockDim.x) {
    const long long b = p / d.HW, q = p - b * d.HW;
    const float s0 = d.score[b * 2 * d.HW + q], s1 = d.score[b * 2 * d.HW + d.HW + q];
    const LogSoftmax2 ls(s0, s1);
    const long long lab = (long long)d.need[b];
    v[0] -= (double)(lab == 1 ? ls.l1 : ls.l0);
    v[1] += (double)expf(d.cons_ch ? ls.l1 : ls.l0);
  }
  block_sum<2>(v, sh);
  const float c = (float)(v[1] / (double)npix);
  double w[2] = {0.0, 0.0};  // BCE sum, squared-error sum
  for (int r = threadIdx.x; r < d.n; r += blockDim.x) {
    const float x = d.ins[r], y = ins_label(d, r, a.minibatch);
    const float lx = fmaxf(logf(x), -100.f), l1x = fmaxf(logf(1.f - x), -100.f);
    w[0] += (double)((y - 1.f) * l1x - y * lx);  // torch binary_cross_entropy
    const float e = x - c;
    w[1] += (double)(e * e);
  }
  block_sum<2>(w, sh);
  if (threadIdx.x == 0) {
    loss[3 * blockIdx.x + 0] = (float)(v[0] / (double)npix);
    loss[3 * blockIdx.x + 1] = (float)(w[0] / (d.n > 0 ? d.n : 1));
    loss[3 * blockIdx.x + 2] = (float)w[1];
    cons[blockIdx.x] = c;
  }
}

// grid.y = domain.  gloss as in the forward's loss layout.
__global__ void __launch_bounds__(256)
da_loss_bwd_kernel(DaArgs a, const float* __restrict__ gloss, const float* __restrict__ cons) {
  const int dom = blockIdx.y;
  const DaDomain d = a.d[dom];
  const long long npix = (long long)d.B * d.HW;
  const float gi = gloss[3 * dom + 0] / (float)npix;
  const float gb = gloss[3 * dom + 1] / (float)(d.n > 0 ? d.n : 1);
  const float gm = gloss[3 * dom + 2];
  const float c = cons[dom];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix + d.n;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < npix) {
      const long long b = i / d.HW, q = i - b * d.HW;
      const long long i0 = b * 2 * d.HW + q, i1 = i0 + d.HW;
      const float s0 = d.score[i0], s1 = d.score[i1];
      const LogSoftmax2 ls(s0, s1);
      const bool one = (long long)d.need[b] == 1;
      d.dscore[i0] = gi * (expf(ls.l0) - (one ? 0.f : 1.f));
      d.dscore[i1] = gi * (expf(ls.l1) - (one ? 1.f : 0.f));
    } else {
      const int r = (int)(i - npix);
      const float x = d.ins[r], y = ins_label(d, r, a.minibatch);
      const float bce = (x - y) / fmaxf((1.f - x) * x, 1e-12f);
      d.dins[r] = gb * bce + gm * 2.f * (x - c);
    }
  }
}

int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

}  // namespace
}  // namespace tlod

using namespace tlod;

extern "C" {

int tlod_rpn_loss_f32(const float* score, const float* labels, const float* bbox,
                      const float* targets, const float* inside, const float* outside, int B,
                      int A, int H, int W, float sigma, float* loss, float* count,
                      tlod_stream_t stream) {
  TLOD_CHECK_ARG(score && labels && bbox && targets && inside && outside && loss && count,
                 "null pointer");
  TLOD_CHECK_ARG(B > 0 && A > 0 && H > 0 && W > 0 && sigma > 0.f, "bad shape / sigma");
  TLOD_CHECK_ARG(((uintptr_t)bbox | (uintptr_t)targets | (uintptr_t)inside | (uintptr_t)outside) %
                         16 == 0,
                 "box operands must be 16-byte aligned");
  rpn_loss_fwd_kernel<<<1, kRedThreads, 0, (hipStream_t)stream>>>(
      score, labels, bbox, targets, inside, outside, B, A * H * W, sigma * sigma, loss, count);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

int tlod_rpn_loss_bwd_f32(const float* score, const float* labels, const float* bbox,
                          const float* targets, const float* inside, const float* outside,
                          int B, int B_total, int A, int H, int W, float sigma,
                          const float* grad_loss, const float* count, float* dscore,
                          float* dbbox, tlod_stream_t stream) {
  TLOD_CHECK_ARG(score && labels && bbox && targets && inside && outside && grad_loss &&
                 count && dscore && dbbox, "null pointer");
  TLOD_CHECK_ARG(B > 0 && B_total >= B && A > 0 && H > 0 && W > 0 && sigma > 0.f,
                 "bad shape / sigma");
  const long long rows = (long long)B_total * A * H * W;
  rpn_loss_bwd_kernel<<<grid_for(rows * 5), 256, 0, (hipStream_t)stream>>>(
      score, labels, bbox, targets, inside, outside, B, B_total, A * H * W, sigma * sigma,
      grad_loss, count, dscore, dbbox);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

int tlod_rcnn_loss_f32(const float* cls_score, const float* bbox_pred, const long long* labels,
                       const float* targets, const float* inside, const float* outside, int R,
                       int C, int agnostic, float sigma, float* cls_prob, float* bbox_sel,
                       float* loss, tlod_stream_t stream) {
  TLOD_CHECK_ARG(cls_score && bbox_pred && labels && targets && inside && outside && cls_prob &&
                 loss, "null pointer");
  TLOD_CHECK_ARG(R > 0 && C > 0 && sigma > 0.f, "bad shape / sigma");
  rcnn_loss_fwd_kernel<<<1, kRedThreads, 0, (hipStream_t)stream>>>(
      cls_score, bbox_pred, labels, targets, inside, outside, R, C, agnostic, sigma * sigma,
      cls_prob, bbox_sel, loss);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

int tlod_rcnn_loss_bwd_f32(const float* cls_prob, const float* bbox_pred,
                           const long long* labels, const float* targets, const float* inside,
                           const float* outside, int R, int R_total, int C, int agnostic,
                           float sigma, const float* grad_loss, float* dcls, float* dbbox,
                           tlod_stream_t stream) {
  TLOD_CHECK_ARG(cls_prob && bbox_pred && labels && targets && inside && outside &&
                 grad_loss && dcls && dbbox, "null pointer");
  TLOD_CHECK_ARG(R > 0 && R_total >= R && C > 0 && sigma > 0.f, "bad shape / sigma");
  const long long n = (long long)R_total * C + (long long)R_total * (agnostic ? 4 : 4 * C);
  rcnn_loss_bwd_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(
      cls_prob, bbox_pred, labels, targets, inside, outside, R, R_total, C, agnostic,
      sigma * sigma, grad_loss, dcls, dbbox);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

static int da_args(const float* score_s, const float* score_t, const float* need_s,
                   const float* need_t, const float* ins_s, const float* ins_t, int Bs, int Bt,
                   int Hs, int Ws, int Ht, int Wt, int n_s, int n_t, float* dscore_s,
                   float* dscore_t, float* dins_s, float* dins_t, DaArgs* a) {
  TLOD_CHECK_ARG(score_s && score_t && need_s && need_t && (ins_s || n_s == 0) &&
                 (ins_t || n_t == 0), "null pointer");
  TLOD_CHECK_ARG(Bs > 0 && Bt > 0 && Hs > 0 && Ws > 0 && Ht > 0 && Wt > 0 && n_s >= 0 &&
                 n_t >= 0, "bad shape");
  a->d[0] = DaDomain{score_s, need_s, ins_s, dscore_s, dins_s, Bs, Hs * Ws, n_s, 1};
  a->d[1] = DaDomain{score_t, need_t, ins_t, dscore_t, dins_t, Bt, Ht * Wt, n_t, 0};
  a->minibatch = 256;
  return kOk;
}

int tlod_da_loss_f32(const float* score_s, const float* score_t, const float* need_s,
                     const float* need_t, const float* ins_s, const float* ins_t, int Bs,
                     int Bt, int Hs, int Ws, int Ht, int Wt, int n_s, int n_t, float* loss,
                     float* cons, tlod_stream_t stream) {
  TLOD_CHECK_ARG(loss && cons, "null pointer");
  DaArgs a;
  const int st = da_args(score_s, score_t, need_s, need_t, ins_s, ins_t, Bs, Bt, Hs, Ws, Ht,
                         Wt, n_s, n_t, nullptr, nullptr, nullptr, nullptr, &a);
  if (st != kOk) return st;
  da_loss_fwd_kernel<<<2, kRedThreads, 0, (hipStream_t)stream>>>(a, loss, cons);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

int tlod_da_loss_bwd_f32(const float* score_s, const float* score_t, const float* need_s,
                         const float* need_t, const float* ins_s, const float* ins_t, int Bs,
                         int Bt, int Hs, int Ws, int Ht, int Wt, int n_s, int n_t,
                         const float* grad_loss, const float* cons, float* dscore_s,
                         float* dscore_t, float* dins_s, float* dins_t, tlod_stream_t stream) {
  TLOD_CHECK_ARG(grad_loss && cons && dscore_s && dscore_t && (dins_s || n_s == 0) &&
                 (dins_t || n_t == 0), "null pointer");
  DaArgs a;
  const int st = da_args(score_s, score_t, need_s, need_t, ins_s, ins_t, Bs, Bt, Hs, Ws, Ht,
                         Wt, n_s, n_t, dscore_s, dscore_t, dins_s, dins_t, &a);
  if (st != kOk) return st;
  const long long n = std::max((long long)Bs * Hs * Ws + n_s, (long long)Bt * Ht * Wt + n_t);
  dim3 grid(grid_for(n), 2);
  da_loss_bwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a, grad_loss, cons);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

}  // extern "C"
