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
}  // namespace mx

extern "C" const char* mx_version(void) { return "matcha-gossip gfx950 0.1"; }
extern "C" const char* mx_last_error(void) { return mx::g_err; }
