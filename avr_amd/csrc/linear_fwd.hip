// Hidden layers of the signal network on the matrix cores: y = relu(x W^T)
// for the width-512 layers (model.py:176-180, tcnn FullyFusedMLP /
// CutlassMLP with ReLU, no bias), 16-bit operands, fp32 accumulation, one
// rounding to the 16-bit type (as the GEMM epilogue rounds).
//
// Shape: x [M, 512], W [N, 512] (nn.Linear layout, both contiguous in k),
// y [M, N] with N a multiple of 32 and M ~ 262,144 rows at config 2.  The
// layer moves x once and y once (537 MB: ~85 us at HBM speed) for 137 GFLOP
// (~55 us at the 2.5 PF fp16 peak).  hipBLASLt's solution (MT256x256x32)
// reads x once per 256-column slice and runs at 0.80-0.85 PFLOP/s.
//
// x stationary (round 4).  A work item is 256 rows of x.  Each wave loads
// its rows' MFMA fragments ONCE, from HBM straight into registers (32 rows =
// 128 VGPRs at K = 512), then the item sweeps N in 32-column tiles: W
// (512 KB at N = 512, resident in every XCD's L2) streams through a 4-tile
// LDS ring by LDS-DMA in fragment order (avr_linear_pack_w), one 1 KiB
// fragment per k-step.  So x crosses HBM once for all N columns and only
// W's 32 KB per tile moves through LDS-DMA.
//
// Each MFMA computes the TRANSPOSED tile, C^T = W_tile x_rows^T (A = the W
// fragment, B = the x fragment: the same registers as x^T's), so a lane holds
// 16 columns of one row; the two lane halves swap 8-byte groups
// (v_permlane32_swap) so that every lane owns 8 consecutive columns and the
// epilogue (ReLU, one rounding) leaves as 16-byte stores, 32 rows x 32 B per
// wave-instruction.  No LDS round trip for the output.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));

constexpr int kLK = 512;             // K
constexpr int kLKS = kLK / 16;       // k-steps
constexpr int kLRows = 256;          // rows of x per work item
constexpr int kLRing = 4;            // W tiles in the LDS ring (3 in flight)
constexpr int kLTile = kLKS * 1024;  // one 32-column W tile in fragment order
constexpr size_t kLLds = (size_t)kLRing * kLTile;

template <typename E>
__device__ __forceinline__ f32x16 lmfma(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

__device__ __forceinline__ void ldma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

#define AVR_LVMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))

template <typename E, int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4, WAVES / 4))) void
linear_xs_kernel(int64_t M, int N, const E* __restrict__ x, const frag8* __restrict__ Wf, E* __restrict__ y,
                 int relu) {
    constexpr int NB = kLRing, RPW = kLRows / WAVES, NQ = RPW / 32, DPW = kLKS / WAVES;
    static_assert(DPW * (NB - 2) <= 63, "ring");
    extern __shared__ __attribute__((aligned(16))) char lds_l[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int64_t m0 = (int64_t)blockIdx.x * kLRows + RPW * wave;  // the wave's first row
    const int nt = N / 32;

    const uint32_t ring_lds = (uint32_t)(uintptr_t)lds_l;
    auto issue = [&](int tau, int slot) {  // this wave's DPW pieces of W tile tau
        const char* src = reinterpret_cast<const char*>(Wf) + (int64_t)tau * kLTile + wave * DPW * 1024 + 16 * lane;
        const uint32_t dst = ring_lds + slot * kLTile + wave * DPW * 1024;
#pragma unroll
        for (int d = 0; d < DPW; ++d) ldma16(src + d * 1024, dst + d * 1024);
    };
    for (int i = 0; i < NB - 1; ++i)
        if (i < nt) issue(i, i);
    // the wave's rows (rows past M repeat the last one; their stores are dropped)
    frag8 a[NQ][kLKS];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const E* xr = x + min(m0 + 32 * q + j, M - 1) * kLK + 8 * half;
#pragma unroll
        for (int ks = 0; ks < kLKS; ++ks) a[q][ks] = *reinterpret_cast<const frag8*>(xr + 16 * ks);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int ks = 0; ks < kLKS; ++ks) asm volatile("" ::"v"(a[q][ks]));
    AVR_LVMCNT(0);
    __syncthreads();

    for (int tau = 0; tau < nt; ++tau) {
        if (tau + NB - 1 < nt) issue(tau + NB - 1, (tau + NB - 1) % NB);  // the slot tile tau-1 left
        const char* bsrc = lds_l + (tau % NB) * kLTile + 16 * lane;
        constexpr int D = 8;
        frag8 bw[D];
#pragma unroll
        for (int u = 0; u < D; ++u) bw[u] = *reinterpret_cast<const frag8*>(bsrc + u * 1024);
        f32x16 acc[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < kLKS; ++ks) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[q] = lmfma<E>(bw[ks % D], a[q][ks], acc[q]);
            if (ks + D < kLKS) bw[ks % D] = *reinterpret_cast<const frag8*>(bsrc + (ks + D) * 1024);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
#pragma unroll
        for (int ks = 0; ks < kLKS; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x008, NQ, 0);
            if (ks + D < kLKS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        // epilogue: register r of acc[q] is column 32 tau + (r & 3) + 8 (r >> 2)
        // + 4 half of row m0 + 32 q + j.  Group pair (2p, 2p + 1) = columns
        // 16p + 4 half + 0..3 and 16p + 8 + 4 half + 0..3: after the half swap
        // a lane owns columns 16p + 8 half + 0..7
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int64_t row = m0 + 32 * q + j;
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = acc[q][8 * pp + e];
                    if (relu) v[e] = fmaxf(v[e], 0.0f);
                }
                const uint32_t x0 = pack16<E>(v[0], v[1]), x1 = pack16<E>(v[2], v[3]);
                const uint32_t y0 = pack16<E>(v[4], v[5]), y1 = pack16<E>(v[6], v[7]);
                const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                const u32x4 o = u32x4{(uint32_t)s0[0], (uint32_t)s1[0], (uint32_t)s0[1], (uint32_t)s1[1]};
                if (row < M)
                    *reinterpret_cast<u32x4*>(y + row * N + 32 * tau + 16 * pp + 8 * half) = o;
            }
        }
        if (tau + 1 < nt) {  // this wave's pieces of tile tau+1 have landed (younger tiles may fly)
            switch (min(NB - 2, nt - 2 - tau)) {
                case 0: AVR_LVMCNT(0); break;
                case 1: AVR_LVMCNT(DPW); break;
                default: AVR_LVMCNT(2 * DPW); break;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // every LDS read of tile tau done
        __builtin_amdgcn_s_barrier();
    }
}

// W [N][K] -> Wf: for column tile tau and k-step ks, the 64 lanes' 16-byte
// MFMA fragments (lane (j, half): W[32 tau + j][16 ks + 8 half + 0..7])
// contiguous
__global__ __launch_bounds__(256) void linear_pack_w_kernel(const uint16_t* __restrict__ W, frag8* __restrict__ Wf,
                                                            int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int lane = (int)(i & 63);
        const int64_t r = i >> 6;
        const int ks = (int)(r % kLKS);
        const int tau = (int)(r / kLKS);
        const int nn = 32 * tau + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
        Wf[i] = *reinterpret_cast<const frag8*>(W + (int64_t)nn * kLK + k0);
    }
}

int lin_waves() {
    const char* e = getenv("AVR_LINEAR_WAVES_PROBE");
    return (e && atoi(e) == 4) ? 4 : 8;
}

}  // namespace

extern "C" int avr_linear_pack_w(int32_t N, int32_t K, const void* W, int32_t dtype, void* Wf, void* stream) {
    AVR_REQUIRE(W && Wf && K == kLK && N >= 32 && N % 32 == 0, "avr_linear_pack_w: K must be 512, N a multiple of 32");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_linear_pack_w: fp16 or bf16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(W) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_linear_pack_w: W and Wf must be 16-byte aligned");
    const int64_t n = (int64_t)(N / 32) * kLKS * 64;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(linear_pack_w_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), (const uint16_t*)W,
                       (frag8*)Wf, n);
    return check_launch("avr_linear_pack_w");
}

extern "C" int avr_linear_relu_fwd(int64_t M, int32_t N, int32_t K, const void* x, const void* Wf, int32_t dtype,
                                   int32_t relu, void* y, void* stream) {
    AVR_REQUIRE(M >= 1 && x && Wf && y, "avr_linear_relu_fwd: bad args");
    AVR_REQUIRE(K == kLK, "avr_linear_relu_fwd: K must be 512");
    AVR_REQUIRE(N >= 32 && N % 32 == 0, "avr_linear_relu_fwd: N must be a multiple of 32");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_linear_relu_fwd: fp16 or bf16 operands");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(y) % 16 == 0,
                "avr_linear_relu_fwd: x, Wf and y must be 16-byte aligned");
    const int64_t items = (M + kLRows - 1) / kLRows;
    AVR_REQUIRE(items < (1ll << 31), "avr_linear_relu_fwd: too many rows");
    hipStream_t st = as_stream(stream);
    auto go = [&](auto kern, auto e, int waves) {
        using E = decltype(e);
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLLds);
        hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(64 * waves), kLLds, st, M, (int)N, (const E*)x,
                           (const frag8*)Wf, (E*)y, (int)relu);
    };
    const bool w4 = lin_waves() == 4;
    if (dtype == AVR_DTYPE_F16) {
        if (w4) go(linear_xs_kernel<__half, 4>, __half{}, 4);
        else go(linear_xs_kernel<__half, 8>, __half{}, 8);
    } else {
        if (w4) go(linear_xs_kernel<__hip_bfloat16, 4>, __hip_bfloat16{}, 4);
        else go(linear_xs_kernel<__hip_bfloat16, 8>, __hip_bfloat16{}, 8);
    }
    return check_launch("avr_linear_relu_fwd");
}
