// Error reporting for the C ABI (include/hgin.h).
#include <atomic>
#include <cstdarg>
#include <cstring>
#include <mutex>

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

static std::atomic<bool> g_trace{false};
static std::mutex g_trace_mu;
static std::string g_trace_buf;

bool trace_on() { return g_trace.load(std::memory_order_relaxed); }

void trace_launch(const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lk(g_trace_mu);
  g_trace_buf += buf;
  g_trace_buf += '\n';
}

bool xcd_remap_enabled() { return true; }

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

extern "C" int hgin_host_alloc(size_t bytes, void** ptr) {
  HGIN_ARG_CHECK(ptr && bytes > 0, "hgin_host_alloc: bad args");
  *ptr = nullptr;
  const hipError_t e = hipHostMalloc(ptr, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) {
    hgin::set_error("hgin_host_alloc: hipHostMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    return (int)e;
  }
  return HGIN_OK;
}

extern "C" int hgin_host_free(void* ptr) {
  if (!ptr) return HGIN_OK;
  const hipError_t e = hipHostFree(ptr);
  if (e != hipSuccess) {
    hgin::set_error("hgin_host_free: %s", hipGetErrorString(e));
    return (int)e;
  }
  return HGIN_OK;
}

extern "C" int hgin_trace_enable(int on) {
  std::lock_guard<std::mutex> lk(hgin::g_trace_mu);
  hgin::g_trace_buf.clear();
  hgin::g_trace.store(on != 0, std::memory_order_relaxed);
  return HGIN_OK;
}

extern "C" size_t hgin_trace_read(char* buf, size_t cap) {
  std::lock_guard<std::mutex> lk(hgin::g_trace_mu);
  const size_t n = hgin::g_trace_buf.size();
  if (buf && cap > 0) {
    const size_t c = n < cap - 1 ? n : cap - 1;
    std::memcpy(buf, hgin::g_trace_buf.data(), c);
    buf[c] = '\0';
    if (c == n) hgin::g_trace_buf.clear();
  }
  return n;
}
