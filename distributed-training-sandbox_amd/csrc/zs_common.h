// Shared helpers for the zero_amd C ABI: thread-local error text and status mapping.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/zero_amd.h"

namespace zs {

void set_error(const char* fmt, ...);

// zs_tune("sync_host_flags"): 1 (default) = new flag syncs take pinned host words, 0 = device words
// (the fallback when pinned memory is refused; zs_comm.cpp)
int& sync_host_flags();

// zs_tune("sync_write_kernel"): 1 (default) = a flag record is flag_write_kernel (zs_kernels.hip),
// 0 = hipStreamWriteValue64; flag_write enqueues the former (declared where hip types are known)
int& sync_write_kernel();
// zs_tune("sync_write_fence"): 1 (default) = the record kernel's store is a system-scope release,
// 0 = relaxed; zs_tune("sync_wait_kernel"): 1 (default) = a flag wait is flag_wait_kernel (a
// polling wave with s_sleep), 0 = hipStreamWaitValue64
int& sync_write_fence();
int& sync_wait_kernel();

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

}  // namespace zs

#define ZS_REQUIRE(cond, ...)                           \
  do {                                                  \
    if (!(cond)) return zs::fail(ZS_ERR_INVALID, __VA_ARGS__); \
  } while (0)

#define ZS_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return zs::fail(ZS_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                      __FILE__, __LINE__);                                             \
  } while (0)
