// hfa_common.cpp — thread-local error string + library identity for the libhfa C-ABI.
#include "hfa_common.h"
#include "hfa.h"

#include <atomic>
#include <stdarg.h>

namespace {
thread_local char g_last_error[512] = "";
thread_local int g_grid_cap = 0;
}

namespace hfa {
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

int grid_cap() { return g_grid_cap; }

int device_cus() {
    static std::atomic<int> cache[64];            // 0 = not asked yet
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}
}  // namespace hfa

extern "C" {
const char* hfa_last_error(void) { return g_last_error; }
int hfa_abi_version(void) { return HFA_ABI_VERSION; }
const char* hfa_build_arch(void) { return "gfx950"; }

int hfa_set_grid_cap(int wgs) {
    if (wgs < 0) {
        hfa::set_error("hfa_set_grid_cap: wgs must be >= 0");
        return HFA_EINVAL;
    }
    g_grid_cap = wgs;
    return HFA_OK;
}
}
