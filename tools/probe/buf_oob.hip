// Probe: raw buffer dwordx4 loads that straddle the buffer range (per-dword or whole-vector
// zeroing?) and 32-bit offset wrap-around for negative offsets.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ f32x4 raw_load4(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__global__ void k(const float* p, float* out) {
  struct __attribute__((packed)) R { const void* ptr; unsigned range; unsigned cfg; } r{p + 4, 32, 0x00020000};
  i32x4 rs = __builtin_bit_cast(i32x4, r);
  const int offs[6] = {0, 24, -8, -16, 4, 28};
  for (int i = 0; i < 6; ++i) {
    f32x4 v = raw_load4(rs, offs[i], 0, 0);
    if (threadIdx.x == 0) for (int e = 0; e < 4; ++e) out[i * 4 + e] = v[e];
  }
}
int main() {
  float h[16]; for (int i = 0; i < 16; ++i) h[i] = i + 1;
  float *d, *o; (void)hipMalloc(&d, 64); (void)hipMalloc(&o, 96);
  (void)hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o);
  float r[24]; (void)hipMemcpy(r, o, 96, hipMemcpyDeviceToHost);
  const char* names[6] = {"off 0", "off 24 (2 in, 2 out)", "off -8 (2 out, 2 in)", "off -16", "off 4 (unaligned)", "off 28 (1 in, 3 out)"};
  for (int i = 0; i < 6; ++i) printf("%-22s %g %g %g %g\n", names[i], r[4*i], r[4*i+1], r[4*i+2], r[4*i+3]);
  return 0;
}
