// xrs_runtime.cpp — library identification and the thread-local error channel
// behind xrs_last_error() (include/xrs.h).
#include <atomic>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include <unistd.h>

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

// Page-locking is page-granular: the runtime pins (and later unpins) every
// page the range touches.  A range that does not start and end on page
// boundaries shares its first / last page with whatever the allocator put
// beside it (a numpy array from malloc starts 16 bytes into an mmap page, or
// inside the brk heap below glibc's dynamic mmap threshold of up to 32 MiB),
// so two registrations can cover one page and unregistering one changes the
// pinning of memory the other — or a later allocation reusing the freed
// range — still relies on.  Only whole pages the caller owns are accepted
// (DESIGN.md §2).
extern "C" int xrs_host_register(void* ptr, int64_t bytes) {
  const int64_t page = (int64_t)sysconf(_SC_PAGESIZE);
  if (!ptr || bytes <= 0) {
    xrs_set_error("xrs_host_register: invalid argument");
    return XRS_ERR_ARG;
  }
  if (reinterpret_cast<uintptr_t>(ptr) % (uintptr_t)page != 0 || bytes % page != 0) {
    xrs_set_error("xrs_host_register: the range must start on a page boundary and span whole "
                  "pages (%lld-byte pages; got offset %lld, %lld bytes)", (long long)page,
                  (long long)(reinterpret_cast<uintptr_t>(ptr) % (uintptr_t)page),
                  (long long)bytes);
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

// The caller names the streams that used the range (include/xrs.h): each is
// synchronised before the pages are unpinned, so no copy queued on them
// outlives the pinning, and nothing else waits — in a multi-device process
// other threads' streams keep running (a device-wide drain stalled them).
extern "C" int xrs_host_unregister(void* ptr, void* const* streams, int64_t nstreams) {
  if (!ptr || nstreams < 1 || nstreams > 64 || !streams) {
    xrs_set_error("xrs_host_unregister: invalid argument (ptr and 1..64 streams required, "
                  "got %lld)", (long long)nstreams);
    return XRS_ERR_ARG;
  }
  for (int64_t k = 0; k < nstreams; ++k) {
    const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(streams[k]));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      xrs_set_error("xrs_host_unregister: synchronising stream %lld: %s", (long long)k,
                    hipGetErrorString(e));
      return XRS_ERR_HIP;
    }
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
