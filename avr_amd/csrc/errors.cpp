// Thread-local error reporting for the C-ABI (include/avr_hip.h).
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"

namespace avr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(e);
        return (int)e;
    }
    return 0;
}

}  // namespace avr

extern "C" const char* avr_last_error(void) { return avr::g_last_error.c_str(); }

extern "C" int avr_abi_version(void) { return AVR_ABI_VERSION; }
