// ReLU + dropout of the fully connected head (RCNN_top = classifier[:-1]:
// Linear ReLU(inplace) Dropout(0.5) Linear ReLU Dropout, lib/DAF/vgg16.py:67-71, and the DA
// instance head's dc_relu / dc_drop pairs, lib/DAF/DA.py:53-73) as one elementwise pass
// forward and one backward, instead of torch's clamp + fused_dropout / masked_scale +
// threshold_backward.  The keep mask comes from the counter-based RNG of common.h (seeded
// per call by the host) and is never stored: the backward reads it back from the output,
// out > 0  <=>  y > 0 and the element was kept (scale >= 1 never underflows y > 0).
// NaN passes through both ways as in torch.relu / nn.Dropout (a diverging head must reach
// the loss as NaN): the tests are written !(v <= 0), which is true for NaN.
#include "common.h"
#include "tlod.h"

namespace tlod {
namespace {

__global__ void __launch_bounds__(256) relu_dropout_kernel(const float* __restrict__ y,
                                                           float* __restrict__ out, long long n,
                                                           float p, float scale,
                                                           unsigned long long seed) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float v = y[i];
    const bool keep = p <= 0.f || rng_unit(seed, 0x5eed, (unsigned long long)i) >= (double)p;
    out[i] = (keep && !(v <= 0.f)) ? v * scale : 0.f;
  }
}

__global__ void __launch_bounds__(256) relu_dropout_bwd_kernel(const float* __restrict__ dout,
                                                               const float* __restrict__ out,
                                                               float* __restrict__ g, long long n,
                                                               float scale) {
  const long long n4 = n / 4;
  const float4* d4 = reinterpret_cast<const float4*>(dout);
  const float4* o4 = reinterpret_cast<const float4*>(out);
  float4* g4 = reinterpret_cast<float4*>(g);
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 d = d4[i], o = o4[i];
    g4[i] = make_float4(!(o.x <= 0.f) ? d.x * scale : 0.f, !(o.y <= 0.f) ? d.y * scale : 0.f,
                        !(o.z <= 0.f) ? d.z * scale : 0.f, !(o.w <= 0.f) ? d.w * scale : 0.f);
  }
  for (long long i = n4 * 4 + blockIdx.x * 256ll + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    g[i] = !(out[i] <= 0.f) ? dout[i] * scale : 0.f;
}

unsigned grid256(long long n) {
  const long long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace
}  // namespace tlod

using namespace tlod;

extern "C" int tlod_relu_dropout_f32(const float* y, float* out, long long n, float p,
                                     unsigned long long seed, tlod_stream_t stream) {
  TLOD_CHECK_ARG(y && out && n > 0 && p >= 0.f && p < 1.f, "bad arguments");
  relu_dropout_kernel<<<grid256(n), 256, 0, (hipStream_t)stream>>>(y, out, n, p,
                                                                   1.f / (1.f - p), seed);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_relu_dropout_bwd_f32(const float* dout, const float* out, float* g,
                                         long long n, float p, tlod_stream_t stream) {
  TLOD_CHECK_ARG(dout && out && g && n > 0 && p >= 0.f && p < 1.f, "bad arguments");
  TLOD_CHECK_ARG(((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(out) |
                   reinterpret_cast<uintptr_t>(g)) & 15) == 0, "16-B aligned tensors expected");
  relu_dropout_bwd_kernel<<<grid256(n / 4 + 1), 256, 0, (hipStream_t)stream>>>(
      dout, out, g, n, 1.f / (1.f - p));
  TLOD_LAUNCH_CHECK();
  return kOk;
}
