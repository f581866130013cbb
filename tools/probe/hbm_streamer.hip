// Diagnostic (tools/overlap_probe.py --contend, never in libtlod): an RCCL stand-in for the
// 8-GPU pre-read — a few workgroups (RCCL's ring kernels run on a few dozen CUs) streaming a
// buffer through HBM, so the DAF-VGG16 backward can be timed while another kernel holds CUs
// and HBM bandwidth the way a ring all-reduce of the fc6 bucket would.
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/hbm_streamer.hip -o tools/probe/libstreamer.so
#include <hip/hip_runtime.h>

// one wave per workgroup; each copies its contiguous slice with 16-B loads / stores, `passes`
// times over (re-reading the slice: the bytes moved = passes x slice)
__global__ void __launch_bounds__(64) hbm_stream_kernel(const float4* __restrict__ src,
                                                        float4* __restrict__ dst, size_t n4,
                                                        int passes) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  for (int p = 0; p < passes; ++p)
    for (size_t i = b + threadIdx.x; i < e; i += 64) {
      float4 v = src[i];
      v.x += 1.f;
      dst[i] = v;
    }
}

extern "C" int streamer_launch(const void* src, void* dst, size_t bytes, int wgs, int passes,
                               void* stream) {
  hipLaunchKernelGGL(hbm_stream_kernel, dim3(wgs), dim3(64), 0, (hipStream_t)stream,
                     (const float4*)src, (float4*)dst, bytes / 16, passes);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
