// xrs_runtime.cpp — library identification and the thread-local error channel
// behind xrs_last_error() (include/xrs.h).
#include <cstdarg>
#include <cstdio>

#include "../../include/xrs.h"

namespace {
thread_local char g_last_error[1024] = "";
}

void xrs_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

extern "C" const char* xrs_version(void) { return "xrs 0.1.0 (gfx950)"; }

extern "C" const char* xrs_last_error(void) { return g_last_error; }
