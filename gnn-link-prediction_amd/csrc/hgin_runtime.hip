// Error reporting for the C ABI (include/hgin.h).
#include <cstdarg>

#include "hgin_common.h"

namespace hgin {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

bool xcd_remap_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_XCD");
    return !(v && v[0] == '0');
  }();
  return on;
}

bool gemm_split_enabled() {
  static const bool on = [] {
    const char* v = getenv("HGIN_F32_GEMM");
    return !(v && std::string(v) == "mfma32");
  }();
  return on;
}

}  // namespace hgin

extern "C" int hgin_abi_version(void) { return HGIN_ABI_VERSION; }

extern "C" const char* hgin_last_error(void) { return hgin::g_last_error.c_str(); }
