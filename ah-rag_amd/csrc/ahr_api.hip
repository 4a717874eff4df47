// Error channel and process-level queries of the C ABI (include/ahr.h).
#include "ahr_common.h"
#include "ahr.h"

#include <string>

namespace ahr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return AHR_EHIP;
}

}  // namespace ahr

extern "C" {

int ahr_abi_version(void) { return AHR_ABI_VERSION; }

const char* ahr_last_error(void) { return ahr::g_last_error.c_str(); }

int ahr_device_count(int* n) {
  if (!n) return ahr::fail(AHR_EINVAL, "null out pointer");
  AHR_HIP(hipGetDeviceCount(n));
  return AHR_OK;
}

}  // extern "C"
