// Calibration probe (not part of the library): cycles per
// v_mfma_f32_32x32x16_f16 for the exact head's inner loop shape -- B operand
// in registers (32 fragments), A operand read from LDS kDepth k-steps
// ahead, 8 waves per workgroup, one workgroup per CU -- with and without a
// workgroup barrier after every chain of 32 (BAR) and with the exact head's
// epilogue VALU (EPI).  Prints microseconds and cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int frag8 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BAR, int EPI, int DEPTH>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void probe(const frag8* __restrict__ w,
                                                                                  float* out, int iters) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    frag8 wf[32];
    for (int i = 0; i < 32; ++i) wf[i] = w[(threadIdx.x + 512 * i) & 4095];
    for (int i = threadIdx.x; i < 64 * 1040 / 16; i += 512) ((frag8*)lds)[i] = w[i & 4095];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const char* a = lds + (lane & 31) * 1040 + 16 * (lane >> 5);
    float zl = 0.f;
    for (int it = 0; it < iters; ++it) {
        frag8 fr[DEPTH];
#pragma unroll
        for (int i = 0; i < DEPTH; ++i) fr[i] = *(const frag8*)(a + 32 * i);
        f32x16 acc = {};
#pragma unroll
        for (int ks = 0; ks < 32; ++ks) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, fr[ks % DEPTH]),
                                                         __builtin_bit_cast(f16x8, wf[ks]), acc, 0, 0, 0);
            if (ks + DEPTH < 32) fr[ks % DEPTH] = *(const frag8*)(a + 32 * (ks + DEPTH));
        }
        __builtin_amdgcn_sched_group_barrier(0x100, DEPTH, 0);
#pragma unroll
        for (int ks = 0; ks < 32; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (ks + DEPTH < 32) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if (EPI) {
#pragma unroll
            for (int r = 0; r < 16; ++r) zl = fmaf(0.5f, __half2float(__float2half(acc[r])), zl);
        } else {
            zl += acc[0];
        }
        if (BAR) __syncthreads();
    }
    out[blockIdx.x * 512 + threadIdx.x] = zl;
}

template <int BAR, int EPI, int DEPTH>
void run(const char* name, frag8* w, float* out, int iters) {
    const size_t lds = 140 * 1024;
    hipFuncSetAttribute((const void*)probe<BAR, EPI, DEPTH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((probe<BAR, EPI, DEPTH>), dim3(256), dim3(512), lds, 0, w, out, iters);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((probe<BAR, EPI, DEPTH>), dim3(256), dim3(512), lds, 0, w, out, iters);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    // per SIMD: 2 waves x iters x 32 MFMAs
    const double mfma_per_simd = 2.0 * iters * 32;
    printf("%-28s %8.1f us  %6.1f ns/MFMA/SIMD  (%.1f cycles at 2.1 GHz)\n", name, ms * 1e3,
           ms * 1e6 / mfma_per_simd, ms * 1e6 / mfma_per_simd * 2.1);
}

int main() {
    frag8* w;
    float* out;
    hipMalloc(&w, 4096 * sizeof(frag8));
    hipMemset(w, 0x11, 4096 * sizeof(frag8));
    hipMalloc(&out, 256 * 512 * sizeof(float));
    const int iters = 2000;
    run<0, 0, 8>("chain, no barrier", w, out, iters);
    run<1, 0, 8>("chain + barrier", w, out, iters);
    run<1, 1, 8>("chain + epilogue + barrier", w, out, iters);
    run<0, 1, 8>("chain + epilogue", w, out, iters);
    run<1, 1, 4>("depth 4, epi + barrier", w, out, iters);
    return 0;
}
