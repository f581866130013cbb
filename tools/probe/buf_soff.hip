// Probe: is the scalar offset (soffset) of a raw buffer load included in the range check?
// Descriptor over 8 floats (32 B) of a 64-float buffer holding 1..64.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ float raw_load1(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
__global__ void k(const float* p, float* out, int s0, int s1, int s2) {
  struct __attribute__((packed)) R { const void* ptr; unsigned range; unsigned cfg; } r{p, 32, 0x00020000};
  i32x4 rs = __builtin_bit_cast(i32x4, r);
  if (threadIdx.x == 0) {
    out[0] = raw_load1(rs, 0, s0, 0);    // voff 0, soff 64: past the range only via soffset
    out[1] = raw_load1(rs, 28, s1, 0);   // voff 28 (in), soff 8 -> 36
    out[2] = raw_load1(rs, 4, s2, 0);    // voff 4, soff 16 -> 20 (in)
    out[3] = raw_load1(rs, 40, 0, 0);    // voff 40: past the range via voffset
  }
}
int main() {
  float h[64]; for (int i = 0; i < 64; ++i) h[i] = i + 1;
  float *d, *o; (void)hipMalloc(&d, 256); (void)hipMalloc(&o, 64);
  (void)hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o, 64, 8, 16);
  float res[4]; (void)hipMemcpy(res, o, 16, hipMemcpyDeviceToHost);
  printf("voff 0 soff 64: %g (17 = soffset not range-checked, 0 = checked)\n", res[0]);
  printf("voff 28 soff 8: %g (10 = not checked, 0 = checked)\n", res[1]);
  printf("voff 4 soff 16: %g (6 expected)\n", res[2]);
  printf("voff 40: %g (0 expected)\n", res[3]);
  return 0;
}
