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

// ----------------------------------------------------------------------------
// Fused gradient post-processing + Adam (avr_runner.py:190-200: clip,
// NaN/Inf zeroing, optimizer.step() of torch.optim.Adam(betas, eps,
// weight_decay), amsgrad off): per element, in one pass over p, g, m, v,
//
//   g = finite(g * coef) ? g * coef : 0        (scale_sanitize_kernel above)
//   g = g + wd * p                             (L2 weight decay, if wd != 0)
//   m = m + (1 - b1) * (g - m)
//   v = v * b2 + (1 - b2) * g * g
//   p = p - step_size * (m / (sqrt(v) / bc2_sqrt + eps))
//
// with step_size = lr / (1 - b1^step) and bc2_sqrt = sqrt(1 - b2^step) per
// tensor: the fp32 arithmetic of the reference's default (foreach)
// torch.optim.Adam step, operation for operation.  28 bytes per element
// (4 reads, 3 writes; the sanitised gradient is not written back: the loop
// drops it at the next zero_grad) instead of 16 + 36 through
// scale_sanitize + torch's fused Adam.
namespace {

struct AdamTable {
    float* p[kMaxTensors];
    const float* g[kMaxTensors];
    float* m[kMaxTensors];
    float* v[kMaxTensors];
    int64_t n[kMaxTensors];
    float step_size[kMaxTensors];
    float bc2_sqrt[kMaxTensors];
};

struct AdamHyper {
    float b2, omb1, omb2, eps, wd;  // omb = 1 - beta, rounded once from double on the host
};

// the arithmetic of torch.optim.Adam's default (foreach) step, in its order:
// lerp for m (weight 1-b1 < 0.5: m + w (g - m)), mul + addcmul for v,
// sqrt / bc2_sqrt + eps, addcdiv
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float c, float ss, float bc2s,
                                          const AdamHyper& hp) {
    float s = g * c;
    s = isfinite(s) ? s : 0.0f;
    if (hp.wd != 0.0f) s = s + hp.wd * p;
    m = m + hp.omb1 * (s - m);
    v = v * hp.b2;
    v = v + hp.omb2 * s * s;
    const float denom = sqrtf(v) / bc2s + hp.eps;
    p = p - ss * (m / denom);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamTable tab, AdamHyper hp, const float* __restrict__ coef) {
    const int t = blockIdx.y;
    float* __restrict__ p = tab.p[t];
    const float* __restrict__ g = tab.g[t];
    float* __restrict__ m = tab.m[t];
    float* __restrict__ v = tab.v[t];
    const int64_t n = tab.n[t];
    const float c = coef ? *coef : 1.0f;
    const float ss = tab.step_size[t], bc2s = tab.bc2_sqrt[t];
    const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                       reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
    const int64_t n4 = vec ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        f32x4 pv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
        const f32x4 gv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i);
        f32x4 mv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m) + i);
        f32x4 vv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v) + i);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float pk = pv[k], mk = mv[k], vk = vv[k];
            adam_elem(pk, gv[k], mk, vk, c, ss, bc2s, hp);
            pv[k] = pk;
            mv[k] = mk;
            vv[k] = vk;
        }
        __builtin_nontemporal_store(pv, reinterpret_cast<f32x4*>(p) + i);
        __builtin_nontemporal_store(mv, reinterpret_cast<f32x4*>(m) + i);
        __builtin_nontemporal_store(vv, reinterpret_cast<f32x4*>(v) + i);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        adam_elem(p[i], g[i], m[i], v[i], c, ss, bc2s, hp);
}

}  // namespace

extern "C" int avr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads,
                             float* const* exp_avg, float* const* exp_avg_sq, const int64_t* sizes,
                             const float* step_size, const float* bc2_sqrt, double beta1, double beta2,
                             float eps, float weight_decay, const float* coef, void* stream) {
    AVR_REQUIRE(n_tensors >= 0 && (n_tensors == 0 || (params && grads && exp_avg && exp_avg_sq && sizes &&
                                                       step_size && bc2_sqrt)),
                "avr_adam_step: bad args");
    const AdamHyper hp{(float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), eps, weight_decay};
    for (int base = 0; base < n_tensors; base += kMaxTensors) {
        AdamTable tab{};
        const int cnt = n_tensors - base < kMaxTensors ? n_tensors - base : kMaxTensors;
        int64_t biggest = 1;
        for (int i = 0; i < cnt; ++i) {
            const int j = base + i;
            AVR_REQUIRE(sizes[j] >= 0, "avr_adam_step: negative size");
            AVR_REQUIRE(sizes[j] == 0 || (params[j] && grads[j] && exp_avg[j] && exp_avg_sq[j]),
                        "avr_adam_step: null tensor");
            AVR_REQUIRE(bc2_sqrt[j] > 0.0f, "avr_adam_step: bias correction must be > 0 (step >= 1)");
            tab.p[i] = params[j];
            tab.g[i] = grads[j];
            tab.m[i] = exp_avg[j];
            tab.v[i] = exp_avg_sq[j];
            tab.n[i] = sizes[j];
            tab.step_size[i] = step_size[j];
            tab.bc2_sqrt[i] = bc2_sqrt[j];
            if (sizes[j] > biggest) biggest = sizes[j];
        }
        // enough workgroups per tensor to fill the chip on the big hash tables
        int64_t blocks = (biggest / 4 + 255) / 256;
        if (blocks > 2048) blocks = 2048;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks, cnt), dim3(256), 0, as_stream(stream), tab, hp,
                           coef);
        if (int e = check_launch("avr_adam_step")) return e;
    }
    return 0;
}
