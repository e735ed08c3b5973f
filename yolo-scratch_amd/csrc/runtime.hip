// Library-level runtime: error reporting and version.
#include <stdarg.h>
#include <string.h>

#include "common.h"

namespace ym {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace ym

extern "C" const char* ym_last_error(void) { return ym::g_err; }
extern "C" int ym_version(void) { return 1; }
extern "C" unsigned ym_policy_generation(void) { return ym::g_policy_gen.load(std::memory_order_relaxed); }
