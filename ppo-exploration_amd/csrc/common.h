// Internal helpers shared by the libppox translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/ppox.h"

namespace ppox {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned ceil_div(long long a, long long b) { return static_cast<unsigned>((a + b - 1) / b); }

// An A/B switch's environment variable (kernel forms, gates): read only under PPOX_AB=1, else null (the
// compiled-in default) — a stray PPOX_* variable never changes the product path (native.py ab_env)
inline const char* ab_env(const char* name) {
    const char* ab = std::getenv("PPOX_AB");
    return ab && ab[0] == '1' && ab[1] == 0 ? std::getenv(name) : nullptr;
}

// bench.py's per-kernel timing (ppox_ktime_arm): the armed event is recorded on the stream where an entry point's
// trailing reduce is about to launch, so the timed window ends with the main kernel — rocprofv3's per-kernel view,
// not the entry point's (whose reduce may queue behind the other stream's persistent kernels)
struct KTime {
    void* ev = nullptr;
    int used = 0;
};
inline KTime& ktime() {
    static thread_local KTime t;
    return t;
}
inline void ktime_mark(hipStream_t s) {
    KTime& t = ktime();
    if (t.ev && !t.used) {
        (void)hipEventRecord(reinterpret_cast<hipEvent_t>(t.ev), s);
        t.used = 1;
    }
}

}  // namespace ppox

#define PPOX_REQUIRE(cond, ...)                    \
    do {                                           \
        if (!(cond)) {                             \
            ::ppox::set_error(__VA_ARGS__);        \
            return PPOX_EINVAL;                    \
        }                                          \
    } while (0)

#define PPOX_LAUNCHED(name)                                                         \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) {                                                     \
            ::ppox::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
            return -static_cast<int>(e_);                                           \
        }                                                                           \
        return PPOX_OK;                                                             \
    } while (0)

// launch check that falls through on success (for entry points launching several kernels)
#define PPOX_LAUNCHED_NORET(name)                                                   \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) {                                                     \
            ::ppox::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
            return -static_cast<int>(e_);                                           \
        }                                                                           \
    } while (0)

#define PPOX_HIP(call, name)                                                         \
    do {                                                                             \
        hipError_t e_ = (call);                                                      \
        if (e_ != hipSuccess) {                                                      \
            ::ppox::set_error("%s: %s failed: %s", name, #call, hipGetErrorString(e_)); \
            return -static_cast<int>(e_);                                            \
        }                                                                            \
    } while (0)
