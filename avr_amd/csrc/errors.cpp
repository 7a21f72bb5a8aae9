// Thread-local error reporting for the C-ABI (include/avr_hip.h).
#include <hip/hip_runtime.h>

#include <mutex>
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

int device_cus() {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static int cus[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
    std::call_once(once[dev], [dev] {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
        cus[dev] = n;
    });
    return cus[dev];
}

}  // namespace avr

extern "C" const char* avr_last_error(void) { return avr::g_last_error.c_str(); }

extern "C" int avr_abi_version(void) { return AVR_ABI_VERSION; }

extern "C" int avr_pinned_alloc(int64_t bytes, void** host_ptr, void** dev_ptr) {
    AVR_REQUIRE(bytes > 0 && host_ptr && dev_ptr, "avr_pinned_alloc: bad args");
    *host_ptr = nullptr;
    *dev_ptr = nullptr;
    hipError_t e = hipHostMalloc(host_ptr, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return avr::fail((int)e, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    e = hipHostGetDevicePointer(dev_ptr, *host_ptr, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(*host_ptr);
        *host_ptr = nullptr;
        return avr::fail((int)e, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
    return 0;
}

extern "C" int avr_pinned_free(void* host_ptr) {
    if (!host_ptr) return 0;
    const hipError_t e = hipHostFree(host_ptr);
    if (e != hipSuccess) return avr::fail((int)e, std::string("hipHostFree: ") + hipGetErrorString(e));
    return 0;
}

// Launch of an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec)
// without torch's replay prologue, which refreshes the device RNG's
// seed/offset tensors: the render graphs draw nothing on the device.
extern "C" int avr_graph_launch(void* graph_exec, void* stream) {
    AVR_REQUIRE(graph_exec != nullptr, "avr_graph_launch: null graph");
    const hipError_t e = hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream);
    if (e != hipSuccess) return avr::fail((int)e, std::string("hipGraphLaunch: ") + hipGetErrorString(e));
    return 0;
}
