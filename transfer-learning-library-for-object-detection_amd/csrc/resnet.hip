// ResNet101 pieces the implicit-GEMM conv does not cover (lib/DAF/resnet.py):
//
//   * the stem: conv1 7x7 / stride 2 / pad 3, 3 -> 64 channels, frozen (resnet.py:107-108,
//     249), with bn1 folded into a per-channel scale/bias and the ReLU fused.  Forward only
//     (conv1, bn1 and layer1 are frozen, so no gradient flows below layer2).  A direct
//     kernel: 147 MACs per output channel do not fill an MFMA K-tile usefully, and the
//     layer is ~1% of the backbone FLOPs;
//   * stride-2 1x1 convolutions (the caffe-style bottleneck puts the stride on conv1,
//     resnet.py:71, and on the downsample, :133-135): a 1x1 conv with stride 2 and no
//     padding equals the stride-1 1x1 conv of x[:, :, ::2, ::2], so these two permutation
//     kernels (subsample, and its adjoint: scatter into a zeroed map) put them on the
//     MFMA conv path.
#include "common.h"
#include "tlod.h"

namespace tlod {

__global__ void __launch_bounds__(256) subsample2_kernel(const float* __restrict__ x, int H, int W,
                                                         int Ho, int Wo, size_t total,
                                                         float* __restrict__ y) {
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int w = (int)(o % Wo);
    const size_t r = o / Wo;
    const int h = (int)(r % Ho);
    const size_t nc = r / Ho;
    y[o] = x[(nc * H + 2 * h) * W + 2 * w];
  }
}

__global__ void __launch_bounds__(256) upsample2_zero_kernel(const float* __restrict__ dy, int H,
                                                             int W, int Ho, int Wo, size_t total,
                                                             float* __restrict__ dx) {
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int w = (int)(o % W);
    const size_t r = o / W;
    const int h = (int)(r % H);
    const size_t nc = r / H;
    dx[o] = ((h | w) & 1) ? 0.f : dy[(nc * Ho + (h >> 1)) * Wo + (w >> 1)];
  }
}

// Stem: tile of 8 output rows x 32 columns per 256-thread workgroup, one output pixel x 64
// channels per thread.  Weights live in LDS as [ci][kh][kw][co] so the 64 channels of a tap
// are 16 broadcast float4 reads; the input patch (3 x 21 x 69) is staged once per tile.
constexpr int kStemCo = 64, kStemK = 7, kStemTH = 8, kStemTW = 32;
constexpr int kStemPH = kStemTH * 2 + kStemK - 2, kStemPW = kStemTW * 2 + kStemK - 2;  // 21 x 69
constexpr int kStemTaps = 3 * kStemK * kStemK;                                             // 147

__global__ void __launch_bounds__(256) stem_conv_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ y, int H, int W,
                                                        int Ho, int Wo, int tiles_w, int tiles_h,
                                                        int relu) {
  __shared__ __attribute__((aligned(16))) float ws[kStemTaps * kStemCo];
  __shared__ float xs[3 * kStemPH * kStemPW];
  const int tid = threadIdx.x;
  int t = blockIdx.x;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h;
  const int n = t / tiles_h;
  const int oh0 = th * kStemTH, ow0 = tw * kStemTW;
  const int ih0 = oh0 * 2 - 3, iw0 = ow0 * 2 - 3;
  for (int i = tid; i < kStemTaps * kStemCo; i += 256) {  // w[co][tap] -> ws[tap][co]
    const int co = i / kStemTaps, tap = i % kStemTaps;
    ws[tap * kStemCo + co] = w[i];
  }
  const float* xn = x + (size_t)n * 3 * H * W;
  for (int i = tid; i < 3 * kStemPH * kStemPW; i += 256) {
    const int ci = i / (kStemPH * kStemPW), r = (i / kStemPW) % kStemPH, c = i % kStemPW;
    const int ih = ih0 + r, iw = iw0 + c;
    xs[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xn[((size_t)ci * H + ih) * W + iw] : 0.f;
  }
  __syncthreads();
  const int lr = tid / kStemTW, lc = tid % kStemTW;
  float acc[kStemCo];
#pragma unroll
  for (int co = 0; co < kStemCo; ++co) acc[co] = 0.f;
  for (int ci = 0; ci < 3; ++ci)
    for (int kh = 0; kh < kStemK; ++kh) {
      const float* xrow = xs + (ci * kStemPH + 2 * lr + kh) * kStemPW + 2 * lc;
      const float* wrow = ws + ((ci * kStemK + kh) * kStemK) * kStemCo;
#pragma unroll
      for (int kw = 0; kw < kStemK; ++kw) {
        const float xv = xrow[kw];
        const float4* w4 = reinterpret_cast<const float4*>(wrow + kw * kStemCo);
#pragma unroll
        for (int q = 0; q < kStemCo / 4; ++q) {
          const float4 wv = w4[q];
          acc[4 * q + 0] = fmaf(xv, wv.x, acc[4 * q + 0]);
          acc[4 * q + 1] = fmaf(xv, wv.y, acc[4 * q + 1]);
          acc[4 * q + 2] = fmaf(xv, wv.z, acc[4 * q + 2]);
          acc[4 * q + 3] = fmaf(xv, wv.w, acc[4 * q + 3]);
        }
      }
    }
  const int oh = oh0 + lr, ow = ow0 + lc;
  if (oh >= Ho || ow >= Wo) return;
  float* yn = y + (size_t)n * kStemCo * Ho * Wo + (size_t)oh * Wo + ow;
#pragma unroll
  for (int co = 0; co < kStemCo; ++co) {
    float v = acc[co];
    if (scale) v *= scale[co];
    if (bias) v += bias[co];
    if (relu) v = fmaxf(v, 0.f);
    yn[(size_t)co * Ho * Wo] = v;
  }
}

static unsigned grid_for(size_t total) {
  return (unsigned)std::min<size_t>((total + 255) / 256, 16384);
}

// RoI head 3x3 convs (layer4 on R x 4 x 4 maps, channels-last) as GEMMs over a 9-tap
// gather: col[(r,h,w)][(kh,kw,c)] = x[r][h+kh-1][w+kw-1][c] (zero outside the map), one
// thread per (row, 4 channels), 9 16-B loads and stores; the adjoint sums the 9 taps of each
// input element in (kh, kw) order (a gather: no atomics, deterministic).  Replaces F.pad +
// 9 slices + torch.cat (and their backward: 9 zero-filled slice gradients summed by autograd).
__global__ void im2col3x3_nhwc_kernel(const float4* __restrict__ x, int H, int W, int C4,
                                      size_t total, float4* __restrict__ col) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    const size_t row = i / C4;
    const int w = (int)(row % W), h = (int)((row / W) % H);
    const size_t r = row / ((size_t)H * W);
    float4* o = col + row * 9 * C4 + c;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hh = h + t / 3 - 1, ww = w + t % 3 - 1;
      const float4 v = (hh >= 0 && hh < H && ww >= 0 && ww < W)
                           ? x[((r * H + hh) * W + ww) * C4 + c]
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      // streaming store: the 9x tap matrix (GBs on ATF's thousands of RoIs) does not fit
      // the caches, so it bypasses them (nontemporal)
      typedef float v4 __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(v4{v.x, v.y, v.z, v.w},
                                  reinterpret_cast<v4*>(o + (size_t)t * C4));
    }
  }
}

__global__ void col2im3x3_nhwc_kernel(const float4* __restrict__ col, int H, int W, int C4,
                                      size_t total, const float4* __restrict__ mask,
                                      float4* __restrict__ dx) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    const size_t row = i / C4;
    const int w = (int)(row % W), h = (int)((row / W) % H);
    const size_t r = row / ((size_t)H * W);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < 9; ++t) {  // output pixel (h - kh + 1, w - kw + 1) took x(h, w) as tap t
      const int oh = h - t / 3 + 1, ow = w - t % 3 + 1;
      if (oh >= 0 && oh < H && ow >= 0 && ow < W) {
        typedef float v4 __attribute__((ext_vector_type(4)));
        const v4 vv = __builtin_nontemporal_load(
            reinterpret_cast<const v4*>(col + (((r * H + oh) * W + ow) * 9 + t) * C4 + c));
        const float4 v = make_float4(vv.x, vv.y, vv.z, vv.w);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
    }
    if (mask != nullptr) {  // the previous layer's ReLU backward (its output is x)
      const float4 m = mask[i];
      a.x = m.x > 0.f ? a.x : 0.f;
      a.y = m.y > 0.f ? a.y : 0.f;
      a.z = m.z > 0.f ? a.z : 0.f;
      a.w = m.w > 0.f ? a.w : 0.f;
    }
    dx[i] = a;
  }
}

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_subsample2_f32(const float* x, int N, int C, int H, int W, float* y,
                                   tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && H > 0 && W > 0 && x && y, "bad arguments");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const size_t total = (size_t)N * C * Ho * Wo;
  hipLaunchKernelGGL(subsample2_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     x, H, W, Ho, Wo, total, y);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_upsample2_zero_f32(const float* dy, int N, int C, int H, int W, float* dx,
                                       tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && H > 0 && W > 0 && dy && dx, "bad arguments");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const size_t total = (size_t)N * C * H * W;
  hipLaunchKernelGGL(upsample2_zero_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, dy, H, W, Ho, Wo, total, dx);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_im2col3x3_nhwc_f32(const float* x, int R, int H, int W, int C, float* col,
                                      tlod_stream_t stream) {
  TLOD_CHECK_ARG(R > 0 && H > 0 && W > 0 && C > 0 && (C & 3) == 0 && x && col, "bad arguments");
  TLOD_CHECK_ARG(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(col)) & 15) == 0,
                 "16-B aligned tensors");
  const size_t total = (size_t)R * H * W * (C / 4);
  hipLaunchKernelGGL(im2col3x3_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const float4*>(x), H, W, C / 4, total,
                     reinterpret_cast<float4*>(col));
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_col2im3x3_nhwc_mask_f32(const float* col, int R, int H, int W, int C,
                                           const float* mask, float* dx, tlod_stream_t stream) {
  TLOD_CHECK_ARG(R > 0 && H > 0 && W > 0 && C > 0 && (C & 3) == 0 && col && dx, "bad arguments");
  TLOD_CHECK_ARG(((reinterpret_cast<uintptr_t>(col) | reinterpret_cast<uintptr_t>(dx) |
                   reinterpret_cast<uintptr_t>(mask)) & 15) == 0,
                 "16-B aligned tensors");
  const size_t total = (size_t)R * H * W * (C / 4);
  hipLaunchKernelGGL(col2im3x3_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const float4*>(col), H, W, C / 4, total,
                     reinterpret_cast<const float4*>(mask), reinterpret_cast<float4*>(dx));
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_col2im3x3_nhwc_f32(const float* col, int R, int H, int W, int C, float* dx,
                                      tlod_stream_t stream) {
  return tlod_col2im3x3_nhwc_mask_f32(col, R, H, W, C, nullptr, dx, stream);
}

extern "C" int tlod_stem_conv7x7s2_f32(const float* x, const float* weight, const float* scale,
                                       const float* bias, float* y, int N, int H, int W, int relu,
                                       tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && H > 0 && W > 0 && x && weight && y, "bad arguments");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int tiles_w = div_up(Wo, kStemTW), tiles_h = div_up(Ho, kStemTH);
  const long long nwg = (long long)tiles_w * tiles_h * N;
  TLOD_CHECK_ARG(nwg < (1ll << 31), "grid too large");
  hipLaunchKernelGGL(stem_conv_kernel, dim3((unsigned)nwg), dim3(256), 0, (hipStream_t)stream, x,
                     weight, scale, bias, y, H, W, Ho, Wo, tiles_w, tiles_h, relu);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
