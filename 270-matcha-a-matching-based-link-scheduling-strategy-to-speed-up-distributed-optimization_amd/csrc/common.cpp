// common.cpp -- library identity and error plumbing for the C ABI.
#include <stdarg.h>

#include "mx_common.h"

namespace mx {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int g_mean_wgpc = 3;

int lds_per_cu() {
    static int v = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 160 * 1024;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || n <= 0)
            return 160 * 1024;
        return n;
    }();
    return v;
}

size_t lds_cap_pad(int static_bytes, int wg_per_cu) {
    if (wg_per_cu <= 0 || static_bytes <= 0) return 0;
    const int cap = lds_per_cu();
    const int want = (cap / (wg_per_cu + 1) + cap / wg_per_cu) / 2 / 256 * 256;
    return want > static_bytes ? (size_t)(want - static_bytes) : 0;
}
}  // namespace mx

extern "C" const char* mx_version(void) { return "matcha-gossip gfx950 0.1"; }
extern "C" const char* mx_last_error(void) { return mx::g_err; }
