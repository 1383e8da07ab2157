// xrs_runtime.cpp — library identification and the thread-local error channel
// behind xrs_last_error() (include/xrs.h).
#include <atomic>
#include <cstdarg>
#include <cstdio>

#include <hip/hip_runtime.h>

#include "../../include/xrs.h"

namespace {
thread_local char g_last_error[1024] = "";
std::atomic<int64_t> g_testing[XRS_TESTING_NUM_KNOBS];   // zero-initialised: product paths
}

void xrs_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int64_t xrs_testing_value(int knob) {
  return knob > 0 && knob < XRS_TESTING_NUM_KNOBS ? g_testing[knob].load() : 0;
}

extern "C" int64_t xrs_testing_set(int knob, int64_t value) {
  if (knob <= 0 || knob >= XRS_TESTING_NUM_KNOBS) {
    xrs_set_error("xrs_testing_set: unknown knob %d", knob);
    return XRS_ERR_ARG;
  }
  return g_testing[knob].exchange(value);
}

extern "C" const char* xrs_version(void) { return "xrs 0.1.0 (gfx950)"; }

extern "C" const char* xrs_last_error(void) { return g_last_error; }

extern "C" int xrs_host_register(void* ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) {
    xrs_set_error("xrs_host_register: invalid argument");
    return XRS_ERR_ARG;
  }
  const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault);
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    (void)hipGetLastError();
    return 1;
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    xrs_set_error("hipHostRegister: %s", hipGetErrorString(e));
    return XRS_ERR_HIP;
  }
  return XRS_OK;
}

extern "C" int xrs_host_unregister(void* ptr) {
  if (!ptr) {
    xrs_set_error("xrs_host_unregister: invalid argument");
    return XRS_ERR_ARG;
  }
  const hipError_t e = hipHostUnregister(ptr);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    xrs_set_error("hipHostUnregister: %s", hipGetErrorString(e));
    return XRS_ERR_HIP;
  }
  return XRS_OK;
}

extern "C" int xrs_copy_async(void* dst, const void* src, int64_t bytes, void* stream) {
  if (!dst || !src || bytes < 0) {
    xrs_set_error("xrs_copy_async: invalid argument");
    return XRS_ERR_ARG;
  }
  if (bytes == 0) return XRS_OK;
  const hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault,
                                      static_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    xrs_set_error("hipMemcpyAsync: %s", hipGetErrorString(e));
    return XRS_ERR_HIP;
  }
  return XRS_OK;
}
