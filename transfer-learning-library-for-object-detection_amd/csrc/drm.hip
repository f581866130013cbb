// MAF DRM space-to-depth (lib/MAF/drm.py:20-42) and its adjoint.
//
// The reference builds the (B, C*s*s, H/s, W/s) map with torch.chunk over rows, then
// over columns, a reshape of every (B, C, s, s) chunk to (B, C*s*s, 1, 1) and two cats
// (drm.py:30-40) — (H/s)*(W/s) tiny kernels.  Here it is one permutation pass each way:
// HBM-bound, one thread per output element (coalesced writes, s-strided reads).
#include "common.h"
#include "tlod.h"

namespace tlod {

__global__ void __launch_bounds__(256) s2d_kernel(const float* __restrict__ x, int C, int H,
                                                  int W, int s, int Ho, int Wo, size_t total,
                                                  float* __restrict__ y) {
  const int ss = s * s;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int w = (int)(o % Wo);
    size_t r = o / Wo;
    const int h = (int)(r % Ho);
    r /= Ho;
    const int cc = (int)(r % ((size_t)C * ss));
    const size_t b = r / ((size_t)C * ss);
    const int c = cc / ss, ij = cc % ss;
    const int i = ij / s, j = ij % s;
    y[o] = x[((b * C + c) * H + (size_t)(h * s + i)) * W + (size_t)(w * s + j)];
  }
}

// dx = depth_to_space(dy) (cropped positions 0); with y (the forward's ReLU output in the
// space-to-depth layout) also the ReLU backward: dx = depth_to_space(dy * (y > 0)).
__global__ void __launch_bounds__(256) d2s_kernel(const float* __restrict__ dy,
                                                  const float* __restrict__ y, int C, int H,
                                                  int W, int s, int Ho, int Wo, size_t total,
                                                  float* __restrict__ dx) {
  const int ss = s * s;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int xw = (int)(o % W);
    size_t r = o / W;
    const int xh = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    const size_t b = r / C;
    const int h = xh / s, w = xw / s;
    float v = 0.f;
    if (h < Ho && w < Wo) {
      const int cc = c * ss + (xh % s) * s + (xw % s);
      const size_t i = ((b * C * ss + cc) * Ho + h) * Wo + w;
      v = dy[i];
      if (y && !(y[i] > 0.f)) v = 0.f;
    }
    dx[o] = v;
  }
}

static unsigned grid_for(size_t total) {
  return (unsigned)std::min<size_t>((total + 255) / 256, 8192);
}

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_space_to_depth_f32(const float* x, int B, int C, int H, int W, int scale,
                                       float* y, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && scale > 0 && H >= scale && W >= scale && x && y,
                 "bad shape (need H, W >= scale)");
  const int Ho = H / scale, Wo = W / scale;
  const size_t total = (size_t)B * C * scale * scale * Ho * Wo;
  hipLaunchKernelGGL(s2d_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, C,
                     H, W, scale, Ho, Wo, total, y);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_depth_to_space_f32(const float* dy, int B, int C, int H, int W, int scale,
                                       float* dx, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && scale > 0 && H >= scale && W >= scale && dy && dx,
                 "bad shape (need H, W >= scale)");
  const int Ho = H / scale, Wo = W / scale;
  const size_t total = (size_t)B * C * H * W;
  hipLaunchKernelGGL(d2s_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, dy,
                     nullptr, C, H, W, scale, Ho, Wo, total, dx);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

// Backward of the fused DRM forward (tlod_drm_fwd_f32: 1x1 conv + ReLU + crop +
// space-to-depth, lib/MAF/drm.py:10-42) up to the conv: g = depth_to_space(dy * (y > 0)),
// one pass (the reference runs the cat/reshape/chunk backward and the ReLU backward apart).
extern "C" int tlod_drm_relu_bwd_f32(const float* dy, const float* y, int B, int C, int H, int W,
                                     int scale, float* g, tlod_stream_t stream) {
  TLOD_CHECK_ARG(B > 0 && C > 0 && scale > 1 && H >= scale && W >= scale && dy && y && g,
                 "bad shape (need scale > 1, H, W >= scale)");
  const int Ho = H / scale, Wo = W / scale;
  const size_t total = (size_t)B * C * H * W;
  hipLaunchKernelGGL(d2s_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, dy, y,
                     C, H, W, scale, Ho, Wo, total, g);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
