// Library runtime: error reporting for the C ABI (thread-local last error).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "nsm_common.h"

namespace nsm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

}  // namespace nsm

extern "C" int nsm_version(void) { return 1; }

extern "C" int nsm_get_last_error(char* buf, size_t n) {
  if (!buf || n == 0) return NSM_E_ARG;
  size_t k = nsm::g_last_error.size();
  if (k >= n) k = n - 1;
  memcpy(buf, nsm::g_last_error.data(), k);
  buf[k] = 0;
  return 0;
}
