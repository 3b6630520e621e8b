// C-ABI housekeeping for libmauv_hip: error reporting and version/capability queries.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
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
// The measured-fastest routes; f32_math
// starts from MAUV_F32_MATH=split|split1|split3|exact when set.
static MauvRoute default_route() {
  MauvRoute r;
  memset(&r, 0, sizeof r);
  r.f32_math = 6;
  r.halo3 = 1;
  r.big16 = 1;
  r.big16_min_k = 512;
  r.haloc16 = 1;
  r.expand16 = 1;
  r.reparam_kernels = 3;
  if (const char* e = getenv("MAUV_F32_MATH"))
    r.f32_math = !strcmp(e, "exact") ? 0 : !strcmp(e, "split3") ? 3 : !strcmp(e, "split1") ? 5 : 6;
  return r;
}
MauvRoute g_route = default_route();
}  // namespace mauv

// Thread-local message for the last non-zero return code of any mauv_* entry point.
MAUV_API const char* mauv_last_error(void) { return mauv::g_last_error.c_str(); }

// ABI version of include/mauv.h this library implements.
MAUV_API int mauv_abi_version(void) { return 4; }

// The process-wide routing of include/mauv.h (MauvRoute).
MAUV_API int mauv_get_route(MauvRoute* out) {
  if (!out) { mauv::set_error("get_route: out is NULL"); return mauv::kErrArg; }
  *out = mauv::g_route;
  return 0;
}

MAUV_API int mauv_set_route(const MauvRoute* in) {
  if (!in) { mauv::set_error("set_route: in is NULL"); return mauv::kErrArg; }
  const MauvRoute& r = *in;
  const char* bad = nullptr;
  if (r.f32_math != 0 && r.f32_math != 3 && r.f32_math != 5 && r.f32_math != 6)
    bad = "f32_math must be 0 (exact), 3 (split3), 5 (split1) or 6 (split)";
  else if (r.halo3 != 0 && r.halo3 != 1) bad = "halo3 must be 0 or 1";
  else if (r.big16 < 0 || r.big16 > 2) bad = "big16 must be 0, 1 or 2";
  else if (r.big16_min_k < 512) bad = "big16_min_k must be >= 512 (the K range conv_big16 is tested on)";
  else if (r.haloc16 < 0 || r.haloc16 > 3) bad = "haloc16 must be 0..3";
  else if (r.expand16 < 0 || r.expand16 > 3) bad = "expand16 must be 0..3";
  else if (r.reparam_kernels < 0 || r.reparam_kernels > 3) bad = "reparam_kernels must be 0..3";
  if (bad) { mauv::set_error(std::string("set_route: ") + bad); return mauv::kErrArg; }
  mauv::g_route = r;
  return 0;
}
