// 2x2 / stride-2 max pooling of the VGG16 backbone (nn.MaxPool2d(kernel_size=2, stride=2),
// floor mode: torchvision vgg16().features, lib/DAF/vgg16.py:49) and its backward fused with
// the preceding conv's ReLU backward (the pool's input is the conv's ReLU output y):
//   fwd: p[n][c][i][j] = max of y[n][c][2i..2i+1][2j..2j+1]
//   bwd: g[n][c][h][w] = dp[n][c][h/2][w/2] if (h, w) is its window's argmax and y > 0,
//        else 0;  db[c] = sum g  (the conv bias gradient)
// The argmax is recomputed from y with torch's rule (window order (0,0) (0,1) (1,0) (1,1),
// update if val > max or val is NaN: the first maximum wins), so no index tensor is stored
// and the routing is identical to max_pool2d's.  Rows/columns past 2*(H/2), 2*(W/2) (odd
// sizes, floor mode) get zero gradient.
#include "common.h"
#include "tlod.h"

namespace tlod {

__device__ __forceinline__ int window_argmax(float a, float b, float c, float d, float& m) {
  int k = 0;
  m = a;
  if (b > m || __builtin_isnan(b)) { m = b; k = 1; }
  if (c > m || __builtin_isnan(c)) { m = c; k = 2; }
  if (d > m || __builtin_isnan(d)) { m = d; k = 3; }
  return k;
}

// one thread per output element; grid-stride
__global__ void maxpool2x2_kernel(const float* __restrict__ x, int NC, int H, int W,
                                  float* __restrict__ y) {
  const int Hp = H / 2, Wp = W / 2;
  const size_t total = (size_t)NC * Hp * Wp;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < total;
       o += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(o % Wp);
    const size_t t = o / Wp;
    const int i = (int)(t % Hp);
    const size_t nc = t / Hp;
    const float* r0 = x + (nc * H + 2 * i) * (size_t)W + 2 * j;
    const float* r1 = r0 + W;
    float m;
    window_argmax(r0[0], r0[1], r1[0], r1[1], m);
    y[o] = m;
  }
}

// One workgroup of 1024 threads per channel c looping over the N images (db written,
// deterministic order); each thread handles two windows per iteration, reading the window
// rows as float2 pairs when W is even (8-byte aligned rows), so two loads of y, one of dp
// and two stores of g per window are in flight together.
constexpr int kPoolThreads = 1024;
__global__ void __launch_bounds__(kPoolThreads) maxpool2x2_relu_bwd_kernel(
    const float* __restrict__ dp, const float* __restrict__ y, int N, int C, int H, int W,
    float* __restrict__ g, float* __restrict__ db) {
  const int c = blockIdx.x;
  const int Hp = H / 2, Wp = W / 2;
  const int nw = Hp * Wp;
  float s = 0.f;
  auto window = [&](const float a, const float b, const float cc, const float d, float gv,
                    float (&out)[4]) {
    float m;
    const int k = window_argmax(a, b, cc, d, m);
    const float v[4] = {a, b, cc, d};
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = (e == k && v[e] > 0.f) ? gv : 0.f;
    s += (out[0] + out[1]) + (out[2] + out[3]);
  };
  for (int n = 0; n < N; ++n) {
    const size_t base = ((size_t)n * C + c) * H * W;
    const size_t pbase = ((size_t)n * C + c) * Hp * Wp;
    if ((W & 1) == 0) {
      for (int o0 = threadIdx.x; o0 < nw; o0 += 2 * kPoolThreads) {
        float2 r0[2], r1[2];
        float gv[2];
        int idx[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int o = min(o0 + u * kPoolThreads, nw - 1);
          const int i = o / Wp, jj = o - i * Wp;
          idx[u] = (2 * i) * W + 2 * jj;
          r0[u] = *reinterpret_cast<const float2*>(y + base + idx[u]);
          r1[u] = *reinterpret_cast<const float2*>(y + base + idx[u] + W);
          gv[u] = dp[pbase + o];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (o0 + u * kPoolThreads >= nw) continue;
          float out[4];
          window(r0[u].x, r0[u].y, r1[u].x, r1[u].y, gv[u], out);
          *reinterpret_cast<float2*>(g + base + idx[u]) = make_float2(out[0], out[1]);
          *reinterpret_cast<float2*>(g + base + idx[u] + W) = make_float2(out[2], out[3]);
        }
      }
    } else {
      for (int o = threadIdx.x; o < nw; o += kPoolThreads) {
        const int i = o / Wp, j = o - i * Wp;
        const size_t i00 = base + (size_t)(2 * i) * W + 2 * j;
        float out[4];
        window(y[i00], y[i00 + 1], y[i00 + W], y[i00 + W + 1], dp[pbase + o], out);
        g[i00] = out[0];
        g[i00 + 1] = out[1];
        g[i00 + W] = out[2];
        g[i00 + W + 1] = out[3];
      }
    }
    // floor mode: the odd last column / row get no gradient
    if (W & 1)
      for (int h = threadIdx.x; h < H; h += kPoolThreads) g[base + (size_t)h * W + W - 1] = 0.f;
    if (H & 1)
      for (int w = threadIdx.x; w < W; w += kPoolThreads) g[base + (size_t)(H - 1) * W + w] = 0.f;
  }
  if (!db) return;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  __shared__ float ws[kPoolThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < kPoolThreads / 64; ++w) t += ws[w];
    db[c] = t;
  }
}

}  // namespace tlod

using namespace tlod;

extern "C" int tlod_maxpool2x2_f32(const float* x, int N, int C, int H, int W, float* y,
                                   tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && H >= 2 && W >= 2 && x && y, "bad arguments");
  const size_t total = (size_t)N * C * (H / 2) * (W / 2);
  hipLaunchKernelGGL(maxpool2x2_kernel, dim3((unsigned)std::min<size_t>((total + 255) / 256, 16384)),
                     dim3(256), 0, (hipStream_t)stream, x, N * C, H, W, y);
  TLOD_LAUNCH_CHECK();
  return kOk;
}

extern "C" int tlod_maxpool2x2_relu_bwd_f32(const float* dp, const float* y, int N, int C, int H,
                                            int W, float* g, float* db, tlod_stream_t stream) {
  TLOD_CHECK_ARG(N > 0 && C > 0 && H >= 2 && W >= 2 && dp && y && g, "bad arguments");
  hipLaunchKernelGGL(maxpool2x2_relu_bwd_kernel, dim3(C), dim3(kPoolThreads), 0,
                     (hipStream_t)stream, dp, y, N, C, H, W, g, db);
  TLOD_LAUNCH_CHECK();
  return kOk;
}
