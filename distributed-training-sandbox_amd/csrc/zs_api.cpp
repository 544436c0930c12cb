// ABI version and thread-local error reporting for the zero_amd C ABI.
#include <cstdarg>
#include <cstdio>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "zs_common.h"

namespace {
thread_local char g_last_error[1024] = "";
}

namespace zs {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
  va_end(ap);
}
}  // namespace zs

extern "C" {
int zs_abi_version(void) { return ZS_ABI_VERSION; }
const char* zs_last_error(void) { return g_last_error; }

// roctx ranges around the step's phases, named like the reference's record_function ranges
// (zero1.py:80-91): visible to `rocprofv3 --marker-trace` beside the kernels they enclose.
int zs_range_push(const char* name) {
  ZS_REQUIRE(name != nullptr, "zs_range_push: name is NULL");
  roctxRangePushA(name);
  return ZS_OK;
}

int zs_range_pop(void) {
  roctxRangePop();
  return ZS_OK;
}
}
