// Direct 3x3 convolution for tiny input-channel counts: VGG16's conv1_1 (3 -> 64 channels on
// the 600x1200 image, frozen, forward only; lib/DAF/vgg16.py:49 features[0..1]).
//
// Its implicit GEMM has K = 27: the split-bf16 MFMA kernels pad one 8-channel chunk with 5
// zero channels (62% of the MFMA work is padding) and ran at 30 TF f32-equivalent (0.165 ms
// per DAF step).  The layer's floor is the HBM write of its output (2 x 64 x 600 x 1200 f32
// = 368 MB, ~60 us), and its arithmetic is small (5 GFLOP): one thread per output pixel
// keeps the 27 inputs of its 3x3x3 window in registers and runs 27 exact f32 FMAs per output
// channel with the channel's weights as wave-uniform scalar operands (s_load, the scalar
// cache), then bias + ReLU, one coalesced row store per channel.  f32 FMA chains — the same
// arithmetic class as the reference's fp32 cuDNN conv.
#include "common.h"
#include "tlod.h"

namespace tlod {

constexpr int kDirectMaxK = 36;  // Cin * 9 <= 36 (Cin <= 4)

template <int CIN>
__global__ void __launch_bounds__(256) conv3x3_direct_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             float* __restrict__ y, int H, int W,
                                                             int Cout, int relu) {
  const int n = blockIdx.z, h = blockIdx.y, wq = blockIdx.x * 256 + threadIdx.x;
  const size_t HW = (size_t)H * W;
  const float* xn = x + (size_t)n * CIN * HW;
  float in[CIN * 9];
#pragma unroll
  for (int c = 0; c < CIN; ++c)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int hh = h + kh - 1, ww = wq + kw - 1;
        in[(c * 3 + kh) * 3 + kw] =
            (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xn[c * HW + (size_t)hh * W + ww] : 0.f;
      }
  if (wq >= W) return;
  float* yp = y + (size_t)n * Cout * HW + (size_t)h * W + wq;
  // two output channels per step as packed FMAs (v_pk_fma_f32: two f32 FMAs per lane and
  // instruction), each lane's input broadcast to both halves; co is wave-uniform, so the
  // weights load as scalars
  typedef float f2 __attribute__((ext_vector_type(2)));
  int co = 0;
  for (; co + 1 < Cout; co += 2) {
    const float* w0 = w + co * CIN * 9;
    f2 acc = {bias ? bias[co] : 0.f, bias ? bias[co + 1] : 0.f};
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) {
      const f2 wk = {w0[k], w0[CIN * 9 + k]};
      const f2 xk = {in[k], in[k]};
      acc = __builtin_elementwise_fma(xk, wk, acc);
    }
    // streaming stores: the 64-channel output (368 MB for two 600x1200 images) is read back
    // only by conv1_2, long after it has left the caches
    __builtin_nontemporal_store(relu ? fmaxf(acc.x, 0.f) : acc.x, yp + (size_t)co * HW);
    __builtin_nontemporal_store(relu ? fmaxf(acc.y, 0.f) : acc.y, yp + (size_t)(co + 1) * HW);
  }
  if (co < Cout) {
    const float* wc = w + co * CIN * 9;
    float acc = bias ? bias[co] : 0.f;
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) acc = fmaf(in[k], wc[k], acc);
    yp[(size_t)co * HW] = relu ? fmaxf(acc, 0.f) : acc;
  }
}

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_conv3x3_direct_f32(const float* x, const float* weight, const float* bias,
                                       float* y, int N, int Cin, int H, int W, int Cout, int relu,
                                       tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && x && weight && y, "bad shape");
  TLOD_CHECK_ARG(Cin * 9 <= kDirectMaxK, "direct conv: Cin <= 4 only");
  TLOD_CHECK_ARG(N <= 65535 && H <= 65535, "grid too large");
  const dim3 grid(div_up(W, 256), H, N);
  hipStream_t s = (hipStream_t)stream;
  switch (Cin) {
    case 1: hipLaunchKernelGGL(conv3x3_direct_kernel<1>, grid, dim3(256), 0, s, x, weight, bias, y, H, W, Cout, relu); break;
    case 2: hipLaunchKernelGGL(conv3x3_direct_kernel<2>, grid, dim3(256), 0, s, x, weight, bias, y, H, W, Cout, relu); break;
    case 3: hipLaunchKernelGGL(conv3x3_direct_kernel<3>, grid, dim3(256), 0, s, x, weight, bias, y, H, W, Cout, relu); break;
    default: hipLaunchKernelGGL(conv3x3_direct_kernel<4>, grid, dim3(256), 0, s, x, weight, bias, y, H, W, Cout, relu); break;
  }
  TLOD_LAUNCH_CHECK();
  return kOk;
}
