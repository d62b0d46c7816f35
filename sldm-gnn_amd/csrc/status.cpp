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

namespace {
__global__ __launch_bounds__(256) void zero_words_kernel(uint32_t* p, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0u;
}
}  // namespace

int zero_words(void* ptr, size_t words, void* stream) {
  if (words == 0) return SLDM_OK;
  const size_t grid = (words + 255) / 256;
  SLDM_REQUIRE(ptr && grid < ((size_t)1 << 31), "zero_words: bad arguments");
  zero_words_kernel<<<(unsigned)grid, 256, 0, as_stream(stream)>>>(reinterpret_cast<uint32_t*>(ptr),
                                                                   words);
  SLDM_LAUNCH_CHECK("zero_words_kernel");
  return SLDM_OK;
}

static thread_local const uint64_t* g_seed_source = nullptr;
const uint64_t* seed_source() { return g_seed_source; }

}  // namespace sldm

extern "C" int sldm_abi_version(void) { return SLDM_ABI_VERSION; }
extern "C" const char* sldm_last_error(void) { return sldm::g_last_error; }
extern "C" void sldm_set_dropout_seed_source(const uint64_t* device_word) {
  sldm::g_seed_source = device_word;
}
