// Error reporting for the C ABI (thread-local, no global mutable state).
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace sldm {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

void clear_error() { g_last_error[0] = '\0'; }

}  // namespace sldm

extern "C" int sldm_abi_version(void) { return SLDM_ABI_VERSION; }
extern "C" const char* sldm_last_error(void) { return sldm::g_last_error; }
