// tpe_util.hip -- error reporting shared by every C-ABI entry point.
#include <stdarg.h>
#include <stdio.h>

#include "tpe_common.hpp"

namespace tpe {
namespace {
thread_local char g_err[512] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return TPE_E_LAUNCH;
  }
  return TPE_OK;
}
}  // namespace tpe

extern "C" const char* tpe_last_error(void) { return tpe::g_err; }
extern "C" int tpe_abi_version(void) { return TPE_ABI_VERSION; }

// sizes of the ABI structs, so bindings can check their mirrors
extern "C" int tpe_struct_sizes(int32_t* out, int n) {
  const int32_t s[9] = {(int32_t)sizeof(tpe_seg),     (int32_t)sizeof(tpe_cat_seg),
                        (int32_t)sizeof(tpe_job),     (int32_t)sizeof(tpe_best),
                        (int32_t)sizeof(tpe_table),   (int32_t)sizeof(tpe_gather),
                        (int32_t)sizeof(tpe_history), (int32_t)sizeof(tpe_prior),
                        (int32_t)sizeof(tpe_op)};
  for (int i = 0; i < n && i < 9; ++i) out[i] = s[i];
  return 9;
}
