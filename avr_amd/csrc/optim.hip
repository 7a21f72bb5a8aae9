// optim.hip — gradient post-processing of the training loop
// (avr_runner.py:190-196) in one launch:
//
//   torch.nn.utils.clip_grad_norm_(params, max_norm=1)     # scale by coef
//   for p in params: p.grad[p.grad != p.grad] = 0           # NaN -> 0
//                    p.grad[torch.isinf(p.grad)] = 0        # +-Inf -> 0
//
// The clamped clip coefficient stays on the device (no host sync): torch's
// own foreach norm (clip_and_sanitize_), or avr_grad_clip_coef below (the
// fused Adam path); scale_sanitize_kernel applies
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

// ----------------------------------------------------------------------------
// clip_grad_norm_'s total norm and coefficient in two launches (one read of
// every gradient): blocks of the first write one partial sum of squares each
// to a fixed slot, the second sums the slots in a fixed order, so the result
// is the same on every run.  fp32 throughout, as torch's foreach norm; a NaN
// or Inf gradient element makes the total NaN / Inf exactly as there.
constexpr int kNormBlocks = 256;  // partial sums per tensor at most
constexpr int kNormThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.0f;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    return t;
}

struct NormTable {
    const float* ptr[kMaxTensors];
    int64_t n[kMaxTensors];
    int64_t slot[kMaxTensors];  // first partial-sum slot of the tensor
};

__global__ __launch_bounds__(kNormThreads) void grad_sumsq_kernel(NormTable tab, float* __restrict__ part) {
    __shared__ float red[kNormThreads / 64];
    const int t = blockIdx.y;
    const int64_t n = tab.n[t];
    const float* __restrict__ g = tab.ptr[t];
    const int64_t nb = (n + 4 * kNormThreads - 1) / (4 * kNormThreads) < kNormBlocks
                           ? (n + 4 * kNormThreads - 1) / (4 * kNormThreads) : kNormBlocks;
    if (blockIdx.x >= nb) return;  // (the grid is sized for the largest tensor)
    const int64_t n4 = ((reinterpret_cast<uintptr_t>(g) & 15) == 0) ? n / 4 : 0;
    const int64_t stride = nb * kNormThreads;
    float acc = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * kNormThreads + threadIdx.x; i < n4; i += stride) {
        // (plain loads: the gradients stay in the caches for the Adam pass next)
        const f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
        acc += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * kNormThreads + threadIdx.x; i < n; i += stride)
        acc += g[i] * g[i];
    const float s = block_sum(acc, red);
    if (threadIdx.x == 0) part[tab.slot[t] + blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void clip_coef_kernel(const float* __restrict__ part, int64_t n_part, float max_norm,
                                                         float* __restrict__ total, float* __restrict__ coef) {
    __shared__ float red[16];
    float acc = 0.0f;
    for (int64_t i = threadIdx.x; i < n_part; i += blockDim.x) acc += part[i];
    const float s = block_sum(acc, red);
    if (threadIdx.x == 0) {
        const float tn = sqrtf(s);
        const float c = max_norm / (tn + 1e-6f);  // torch: max_norm / (total + 1e-6), clamped at 1
        *total = tn;
        *coef = c > 1.0f ? 1.0f : c;  // a NaN stays NaN (torch.clamp), so every gradient is zeroed
    }
}

int64_t norm_blocks(int64_t n) {
    const int64_t b = (n + 4 * kNormThreads - 1) / (4 * kNormThreads);
    return b < kNormBlocks ? b : kNormBlocks;
}

}  // namespace

extern "C" int avr_grad_clip_workspace(int32_t n_tensors, const int64_t* sizes, int64_t* bytes) {
    AVR_REQUIRE(n_tensors >= 0 && bytes && (n_tensors == 0 || sizes), "avr_grad_clip_workspace: bad args");
    int64_t slots = 1;
    for (int i = 0; i < n_tensors; ++i) {
        AVR_REQUIRE(sizes[i] >= 0, "avr_grad_clip_workspace: negative size");
        slots += norm_blocks(sizes[i]);
    }
    *bytes = slots * (int64_t)sizeof(float);  // one partial sum of squares per block
    return 0;
}

extern "C" int avr_grad_clip_coef(int32_t n_tensors, const float* const* ptrs, const int64_t* sizes, float max_norm,
                                  void* workspace, int64_t workspace_bytes, float* total, float* coef,
                                  void* stream) {
    AVR_REQUIRE(n_tensors >= 0 && total && coef && workspace && (n_tensors == 0 || (ptrs && sizes)),
                "avr_grad_clip_coef: bad args");
    int64_t need = 0;
    if (int e = avr_grad_clip_workspace(n_tensors, sizes, &need)) return e;
    AVR_REQUIRE(workspace_bytes >= need, "avr_grad_clip_coef: workspace too small (avr_grad_clip_workspace)");
    hipStream_t st = as_stream(stream);
    float* part = static_cast<float*>(workspace);
    int64_t n_part = 0;
    for (int base = 0; base < n_tensors; base += kMaxTensors) {
        NormTable tab{};
        const int cnt = n_tensors - base < kMaxTensors ? n_tensors - base : kMaxTensors;
        int64_t blocks = 1;
        for (int i = 0; i < cnt; ++i) {
            AVR_REQUIRE(ptrs[base + i] || sizes[base + i] == 0, "avr_grad_clip_coef: null tensor");
            tab.ptr[i] = ptrs[base + i];
            tab.n[i] = sizes[base + i];
            tab.slot[i] = n_part;
            n_part += norm_blocks(sizes[base + i]);
            if (norm_blocks(sizes[base + i]) > blocks) blocks = norm_blocks(sizes[base + i]);
        }
        hipLaunchKernelGGL(grad_sumsq_kernel, dim3((unsigned)blocks, cnt), dim3(kNormThreads), 0, st, tab, part);
        if (int e = check_launch("avr_grad_clip_coef")) return e;
    }
    hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1024), 0, st, part, n_part, max_norm, total, coef);
    return check_launch("avr_grad_clip_coef");
}

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
