// Probe: issue rate of v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 on gfx950
// (shader cycles per instruction, one and two waves per SIMD, 8 independent accumulators,
// random operands in registers).  Diagnostic program (not part of libtlod).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/mfma_rate tools/probe/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr int kIters = 2048;

template <int K32>
__global__ void __launch_bounds__(512) rate_kernel(const unsigned* seed, float* out,
                                                   unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  unsigned s = seed[0] + lane * 2654435761u + threadIdx.x;
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int i = 0; i < 8; ++i) {
    s = s * 1664525u + 1013904223u;
    a8[i] = (short)(0x3f00 | (s >> 25));
    s = s * 1664525u + 1013904223u;
    b8[i] = (short)(0x3f00 | (s >> 25));
  }
  for (int i = 0; i < 4; ++i) {
    a4[i] = a8[i];
    b4[i] = b8[i + 4];
  }
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const unsigned long long t0 = clock64();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (K32)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[j], 0, 0, 0);
      else
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[j], 0, 0, 0);
    }
  }
  const unsigned long long t1 = clock64();
  float r = 0.f;
  for (int j = 0; j < 8; ++j) r += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (lane == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int K32>
static void run(int waves_per_simd) {
  const int threads = 256 * waves_per_simd, blocks = 256;
  unsigned* seed;
  float* out;
  unsigned long long* cyc;
  CK(hipMalloc(&seed, 4));
  CK(hipMemset(seed, 7, 4));
  CK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CK(hipMalloc(&cyc, (size_t)blocks * 16 * 8));
  CK(hipMemset(cyc, 0, (size_t)blocks * 16 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(rate_kernel<K32>, dim3(blocks), dim3(threads), 0, 0, seed, out, cyc);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(rate_kernel<K32>, dim3(blocks), dim3(threads), 0, 0, seed, out, cyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[16];
  CK(hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost));
  const int nw = threads / 64;
  double c = 0;
  for (int i = 0; i < nw; ++i) c += h[i];
  c /= nw;
  const double n_mfma = (double)kIters * 8;
  const double flops = 2.0 * 16 * 16 * (K32 ? 32 : 16) * n_mfma * (threads / 64) * blocks * reps;
  printf("16x16x%d  waves/SIMD %d: %.2f cycles per MFMA per wave (%.2f per SIMD), %.1f TFLOP/s wall\n",
         K32 ? 32 : 16, waves_per_simd, c / n_mfma, c / n_mfma / waves_per_simd,
         flops / (ms * 1e-3) / 1e12);
  CK(hipFree(seed));
  CK(hipFree(out));
  CK(hipFree(cyc));
}

int main() {
  for (int wps = 1; wps <= 2; ++wps) {
    run<1>(wps);
    run<0>(wps);
  }
  return 0;
}
