// Shared helpers for the tlod HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

namespace tlod {

// Per-thread last error, surfaced through tlod_last_error().  Entry points never exit().
void set_error(const std::string& msg);
const char* last_error();

enum Status : int {
  kOk = 0,
  kInvalidArg = -1,
  kHipError = -2,
  kWorkspace = -3,
  kUnsupported = -4,
};

#define TLOD_CHECK_ARG(cond, msg)                      \
  do {                                                 \
    if (!(cond)) {                                     \
      ::tlod::set_error(std::string(__func__) + ": " + (msg)); \
      return ::tlod::kInvalidArg;                      \
    }                                                  \
  } while (0)

#define TLOD_HIP(call)                                                          \
  do {                                                                          \
    hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess) {                                                     \
      ::tlod::set_error(std::string(__func__) + ": " + #call + ": " +           \
                        hipGetErrorString(e_));                                 \
      return ::tlod::kHipError;                                                 \
    }                                                                           \
  } while (0)

#define TLOD_LAUNCH_CHECK() TLOD_HIP(hipGetLastError())

// Per-(kernel, device), thread-safe launch facts (runtime.hip): the kernel's dynamic-LDS
// limit raised to `bytes` once; resident workgroups of the kernel chip-wide.
hipError_t lds_attr(const void* kern, int bytes);
int cached_slots(const void* kern, int threads, size_t lds);

inline int div_up(int a, int b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace (256-B aligned carves).
struct Carve {
  char* base;
  size_t cap, off = 0;
  Carve(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <class T>
  T* take(size_t n) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += n * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

// Monotone float <-> uint32 map so atomicMax on uint orders floats (incl. negatives).
__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Counter-based RNG (splitmix64 finaliser over seed ^ stream ^ index): used by the
// production sampling path in place of the reference's host numpy RNG.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rng_u64(uint64_t seed, uint64_t stream, uint64_t idx) {
  return mix64(mix64(seed ^ (stream * 0xd1b54a32d192ed03ull)) + idx);
}
__device__ __forceinline__ double rng_unit(uint64_t seed, uint64_t stream, uint64_t idx) {
  return (double)(rng_u64(seed, stream, idx) >> 11) * (1.0 / 9007199254740992.0);  // [0,1)
}

}  // namespace tlod
