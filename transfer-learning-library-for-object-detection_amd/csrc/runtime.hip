// Error plumbing and ABI version for libtlod (C ABI in include/tlod.h).
#include "common.h"
#include "tlod.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

namespace tlod {

// Launch facts cached per (kernel, device) under one lock: several host threads may launch
// concurrently, and a process may drive several devices (round-4 advisor: these were
// unsynchronised process-wide statics keyed by kernel only).
namespace {
std::mutex g_launch_mu;
std::map<std::pair<const void*, int>, int> g_lds_set, g_slots;
int current_device() {
  int dev = 0;
  return hipGetDevice(&dev) == hipSuccess ? dev : 0;
}
}  // namespace

hipError_t lds_attr(const void* kern, int bytes) {
  const auto key = std::make_pair(kern, current_device());
  std::lock_guard<std::mutex> lk(g_launch_mu);
  auto it = g_lds_set.find(key);
  if (it != g_lds_set.end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) g_lds_set[key] = bytes;
  return e;
}

// CUs the planners leave out of their rounds (tlod_set_cu_reserve): while a data-parallel
// all-reduce runs beside the backward, its kernels occupy a few CUs that a 1-workgroup-per-CU
// kernel then cannot use, and a grid planned for exactly one round of all CUs would run a
// second round for the few workgroups left over.
std::atomic<int> g_cu_reserve{[] {
  const char* v = getenv("TLOD_CU_RESERVE");
  return v && *v ? atoi(v) : 0;
}()};

int cached_slots(const void* kern, int threads, size_t lds) {
  const int dev = current_device();
  const auto key = std::make_pair(kern, dev);
  int packed = -1;  // per_cu * 65536 + cus
  {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    auto it = g_slots.find(key);
    if (it != g_slots.end()) packed = it->second;
  }
  if (packed < 0) {
    int cus = 0, per_cu = 0;
    if (lds_attr(kern, (int)lds) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) == hipSuccess &&
        per_cu >= 1 && cus >= 1) {
      packed = per_cu * 65536 + cus;
    } else {
      (void)hipGetLastError();
      packed = 65536 + 256;  // no device (CPU build checks): one workgroup on each of 256 CUs
    }
    std::lock_guard<std::mutex> lk(g_launch_mu);
    g_slots[key] = packed;
  }
  const int per_cu = packed / 65536, cus = packed % 65536;
  return per_cu * std::max(1, cus - g_cu_reserve.load(std::memory_order_relaxed));
}
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }
}  // namespace tlod

extern "C" int tlod_abi_version(void) { return 1; }
extern "C" int tlod_set_cu_reserve(int cus) {
  if (cus < 0 || cus > 1024) {
    tlod::set_error("tlod_set_cu_reserve: 0 <= cus <= 1024");
    return tlod::kInvalidArg;
  }
  tlod::g_cu_reserve.store(cus, std::memory_order_relaxed);
  return tlod::kOk;
}
extern "C" const char* tlod_last_error(void) { return tlod::last_error(); }
