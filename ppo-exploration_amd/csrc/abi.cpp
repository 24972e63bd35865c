// Library identification and the thread-local error channel of the C ABI.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "common.h"

namespace ppox {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

}  // namespace ppox

extern "C" const char* ppox_version(void) { return "ppox 0.1.0 gfx950"; }

extern "C" const char* ppox_last_error(void) { return ppox::g_last_error.c_str(); }
