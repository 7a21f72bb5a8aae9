// optim.hip — gradient post-processing of the training loop
// (avr_runner.py:190-196) in one launch:
//
//   torch.nn.utils.clip_grad_norm_(params, max_norm=1)     # scale by coef
//   for p in params: p.grad[p.grad != p.grad] = 0           # NaN -> 0
//                    p.grad[torch.isinf(p.grad)] = 0        # +-Inf -> 0
//
// The caller computes the clamped clip coefficient on the device (torch's
// own foreach norm), so there is no host sync; this kernel applies
// g = finite(g * coef) ? g * coef : 0 to every gradient tensor.  It replaces
// clip_grad_norm_'s foreach multiply and the reference's 4-6 launches per
// parameter tensor.
#include "common.h"

using namespace avr;

namespace {

constexpr int kMaxTensors = 32;  // per launch (kernel-argument table)

struct TensorTable {
    float* ptr[kMaxTensors];
    int64_t n[kMaxTensors];
};

__global__ __launch_bounds__(256) void scale_sanitize_kernel(TensorTable tab,
                                                             const float* __restrict__ coef) {
    const int t = blockIdx.y;
    float* __restrict__ p = tab.ptr[t];
    const int64_t n = tab.n[t];
    const float c = coef ? *coef : 1.0f;
    const int64_t n4 = ((reinterpret_cast<uintptr_t>(p) & 15) == 0) ? n / 4 : 0;
    f32x4* p4 = reinterpret_cast<f32x4*>(p);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        f32x4 v = p4[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float s = v[k] * c;
            v[k] = isfinite(s) ? s : 0.0f;
        }
        p4[i] = v;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float s = p[i] * c;
        p[i] = isfinite(s) ? s : 0.0f;
    }
}

}  // namespace

extern "C" int avr_scale_sanitize(int32_t n_tensors, float* const* ptrs, const int64_t* sizes,
                                  const float* coef, void* stream) {
    AVR_REQUIRE(n_tensors >= 0 && (n_tensors == 0 || (ptrs && sizes)),
                "avr_scale_sanitize: bad args");
    for (int base = 0; base < n_tensors; base += kMaxTensors) {
        TensorTable tab{};
        const int cnt = n_tensors - base < kMaxTensors ? n_tensors - base : kMaxTensors;
        int64_t biggest = 1;
        for (int i = 0; i < cnt; ++i) {
            AVR_REQUIRE(ptrs[base + i] || sizes[base + i] == 0, "avr_scale_sanitize: null tensor");
            tab.ptr[i] = ptrs[base + i];
            tab.n[i] = sizes[base + i];
            if (sizes[base + i] > biggest) biggest = sizes[base + i];
        }
        int64_t blocks = (biggest / 4 + 255) / 256;
        if (blocks > 1024) blocks = 1024;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(scale_sanitize_kernel, dim3((unsigned)blocks, cnt), dim3(256), 0,
                           as_stream(stream), tab, coef);
        if (int e = check_launch("avr_scale_sanitize")) return e;
    }
    return 0;
}
