// gs_common.h -- error plumbing shared by the translation units of libgibbs_hip.so
#pragma once
#include <hip/hip_runtime.h>
#include <string>

namespace gs_detail {

// one thread-local message for the whole library (gs_last_error)
inline thread_local std::string g_last_error;

inline int set_error(const std::string& msg) {
    g_last_error = msg;
    return -1;
}

// library options (include/gibbs_capi.h gs_option_set): the value of a
// registered option, or nullptr when it is unset.  Read when a plan, SHT or
// masked context is created; the library reads no environment variables.
const char* option(const char* name);

}  // namespace gs_detail

#define GS_CHECK(expr)                                                                        \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return gs_detail::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

#define GS_LAUNCH_CHECK(name)                                                                 \
    do {                                                                                      \
        hipError_t _e = hipGetLastError();                                                    \
        if (_e != hipSuccess)                                                                 \
            return gs_detail::set_error(std::string("launch ") + (name) + ": " + hipGetErrorString(_e)); \
    } while (0)

// device bounds assertions of the debug build (-DGS_DEBUG, build.py variant
// "debug"): a failed check prints where and traps the kernel; compiled out
// otherwise
#if defined(GS_DEBUG)
#include <cstdio>
#define GS_ASSERT(cond)                                                                       \
    do {                                                                                      \
        if (!(cond)) {                                                                        \
            printf("GS_ASSERT %s:%d: %s\n", __FILE__, __LINE__, #cond);                      \
            __builtin_trap();                                                                 \
        }                                                                                     \
    } while (0)
#else
#define GS_ASSERT(cond) do { } while (0)
#endif
