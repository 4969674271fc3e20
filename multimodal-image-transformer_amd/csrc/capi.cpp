// C-ABI bookkeeping for libmit_hip.so: thread-local error strings and the ABI version.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mit_hip.h"

static thread_local char g_err[512] = "";

int mit_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return 0;
}

extern "C" const char* mit_last_error(void) { return g_err; }
extern "C" int mit_abi_version(void) { return 1; }
