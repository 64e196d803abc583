// hfa_common.cpp — thread-local error string + library identity for the libhfa C-ABI.
#include "hfa_common.h"

#include <stdarg.h>

namespace {
thread_local char g_last_error[512] = "";
}

namespace hfa {
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}
}  // namespace hfa

extern "C" {
const char* hfa_last_error(void) { return g_last_error; }
int hfa_abi_version(void) { return 1; }
const char* hfa_build_arch(void) { return "gfx950"; }
}
