// Library-level entry points: version, thread-local error text, arch probe.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

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

// 1 when the current device is a gfx950 (the only target the code objects are
// built for), 0 for any other device, -1 when no device can be queried.
extern "C" int asr_arch_is_gfx950(void) {
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
    return -1;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

// A stream restricted to CUs [cu_begin, cu_begin + cu_count) of the current
// device (hipExtStreamCreateWithCUMask).  Used for the weight-gradient GEMMs
// that run beside the persistent backward recurrence, so the two never compete
// for the CUs the recurrence's co-resident work-groups need.
extern "C" int asr_stream_create_cu_masked(int cu_begin, int cu_count, void** stream_out) {
  ASR_REQUIRE(stream_out && cu_begin >= 0 && cu_count > 0, ASR_ERR_ARG, "stream: bad args");
  int dev = 0, ncu = 0;
  ASR_CHECK_HIP(hipGetDevice(&dev));
  ASR_CHECK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  ASR_REQUIRE(cu_begin + cu_count <= ncu, ASR_ERR_ARG, "stream: CU range beyond %d CUs", ncu);
  uint32_t mask[16] = {0};
  ASR_REQUIRE(ncu <= 512, ASR_ERR_ARG, "stream: too many CUs");
  for (int c = cu_begin; c < cu_begin + cu_count; ++c) mask[c >> 5] |= 1u << (c & 31);
  hipStream_t s = nullptr;
  ASR_CHECK_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)((ncu + 31) / 32), mask));
  *stream_out = (void*)s;
  return ASR_OK;
}

extern "C" int asr_stream_destroy(void* stream) {
  if (stream) ASR_CHECK_HIP(hipStreamDestroy((hipStream_t)stream));
  return ASR_OK;
}
