// Error plumbing and ABI version for libtlod (C ABI in include/tlod.h).
#include "common.h"
#include "tlod.h"

namespace tlod {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }
}  // namespace tlod

extern "C" int tlod_abi_version(void) { return 1; }
extern "C" const char* tlod_last_error(void) { return tlod::last_error(); }
