// Error plumbing and ABI version for libtlod (C ABI in include/tlod.h).
#include "common.h"
#include "tlod.h"

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

int cached_slots(const void* kern, int threads, size_t lds) {
  const int dev = current_device();
  const auto key = std::make_pair(kern, dev);
  {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    auto it = g_slots.find(key);
    if (it != g_slots.end()) return it->second;
  }
  int cus = 0, per_cu = 0, slots = 256;
  if (lds_attr(kern, (int)lds) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) == hipSuccess &&
      per_cu >= 1 && cus >= 1)
    slots = per_cu * cus;
  else
    (void)hipGetLastError();
  std::lock_guard<std::mutex> lk(g_launch_mu);
  g_slots[key] = slots;
  return slots;
}
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }
}  // namespace tlod

extern "C" int tlod_abi_version(void) { return 1; }
extern "C" const char* tlod_last_error(void) { return tlod::last_error(); }
