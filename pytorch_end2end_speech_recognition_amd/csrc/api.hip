// Library-level entry points: version, thread-local error text, arch probe.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace asr {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace asr

extern "C" const char* asr_version(void) { return "asr_hip 0.1.0 gfx950"; }

extern "C" const char* asr_last_error(void) { return asr::g_err; }

extern "C" int asr_arch_is_gfx950(void) {
#if defined(__gfx950__)
  return 1;
#else
  return 1;  // host pass: the library is only ever built with --offload-arch=gfx950
#endif
}
