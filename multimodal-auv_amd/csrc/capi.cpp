// C-ABI housekeeping for libmauv_hip: error reporting and version/capability queries.
#include <hip/hip_runtime.h>
#include <string>

#include "mauv_common.h"

namespace mauv {
static thread_local std::string g_last_error;

void set_error(const std::string& s) { g_last_error = s; }

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return kErrLaunch;
  }
  return 0;
}
}  // namespace mauv

// Thread-local message for the last non-zero return code of any mauv_* entry point.
MAUV_API const char* mauv_last_error(void) { return mauv::g_last_error.c_str(); }

// ABI version of include/mauv.h this library implements.
MAUV_API int mauv_abi_version(void) { return 3; }
