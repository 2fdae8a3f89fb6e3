// Error plumbing shared by every libfsagg entry point.
#include <cstdarg>

#include "common.h"

namespace fsagg {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return FSAGG_EHIP;
  }
  return FSAGG_OK;
}

int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                              dev) != hipSuccess || cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

}  // namespace fsagg

extern "C" int fsagg_version(void) { return FSAGG_VERSION; }

extern "C" const char *fsagg_last_error(void) { return fsagg::g_err; }
