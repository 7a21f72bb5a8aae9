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
#include "probe.h"
#include "stationary.h"

#include <algorithm>

using namespace avr;

AVR_PROBE_TU(avr_probe_set_linear)

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));

constexpr int kLK = 512;             // K
constexpr int kLKS = kLK / 16;       // k-steps
constexpr int kLTile = kLKS * 1024;  // one 32-column W tile in fragment order

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

// s_waitcnt vmcnt(n) for a run-time n (the immediate is a constant: one
// case per value; n > 63 is clamped to 63, a shorter wait)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define AVR_VMC(K) case K: AVR_LVMCNT(K); break;
        AVR_VMC(0) AVR_VMC(1) AVR_VMC(2) AVR_VMC(3) AVR_VMC(4) AVR_VMC(5) AVR_VMC(6) AVR_VMC(7)
        AVR_VMC(8) AVR_VMC(9) AVR_VMC(10) AVR_VMC(11) AVR_VMC(12) AVR_VMC(13) AVR_VMC(14) AVR_VMC(15)
        AVR_VMC(16) AVR_VMC(17) AVR_VMC(18) AVR_VMC(19) AVR_VMC(20) AVR_VMC(21) AVR_VMC(22) AVR_VMC(23)
        AVR_VMC(24) AVR_VMC(25) AVR_VMC(26) AVR_VMC(27) AVR_VMC(28) AVR_VMC(29) AVR_VMC(30) AVR_VMC(31)
#undef AVR_VMC
        default: AVR_LVMCNT(31); break;
    }
}

// CT = 32 or 64 columns per W tile (64: half the barriers and DMA waits per
// item, two accumulators per wave; the ring then holds 2 tiles of 64 KiB).
template <typename E, int CT, int WAVES, int NB>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_xs_kernel(
    int64_t M, int N, const E* __restrict__ x, const frag8* __restrict__ Wf, E* __restrict__ y, int relu) {
    constexpr int ROWS = 32 * WAVES;  // rows of x per work item
    constexpr int NC = CT / 32, TILEB = NC * kLTile;
    constexpr int DPW = NC * kLKS / WAVES;  // 1 KiB DMAs per wave and tile
    constexpr int ST = 2 * NC;              // 16-byte stores per wave and tile
    static_assert(NB >= 2 && DPW * NB <= 63, "ring");
    AVR_PROBE_DECL;
    extern __shared__ __attribute__((aligned(16))) char lds_l[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int64_t r0 = (int64_t)blockIdx.x * ROWS;  // the item's first row
    const int nt = N / CT;

    const uint32_t ring_lds = (uint32_t)(uintptr_t)lds_l;
    auto issue = [&](int tau, int slot) {  // this wave's DPW pieces of W tile tau
        const char* src = reinterpret_cast<const char*>(Wf) + (int64_t)tau * TILEB + wave * DPW * 1024 + 16 * lane;
        const uint32_t dst = ring_lds + slot * TILEB + wave * DPW * 1024;
#pragma unroll
        for (int d = 0; d < DPW; ++d) ldma16(src + d * 1024, dst + d * 1024);
    };
    // the wave's 32 rows (rows past M repeat the last one; their stores are
    // dropped), whole rows by LDS-DMA through the (still idle) ring
    frag8 a[kLKS];
    {
        const E* xr = x + min(r0 + 32 * wave + j, M - 1) * kLK;
        stat_load_rows512(reinterpret_cast<frag8_t(&)[32]>(a), reinterpret_cast<const uint16_t*>(xr),
                          lds_l + wave * 16384);
    }
    __syncthreads();  // every wave is done with the staging area: the ring may fill
    for (int i = 0; i < NB - 1; ++i)
        if (i < nt) issue(i, i);
    AVR_LVMCNT(0);
    __syncthreads();
    AVR_PROBE_MARK(2);
    // the item's rows of y as a buffer resource: stores to rows past M fall
    // outside it and are dropped without a branch, so every wave issues the
    // same number of stores (the vmcnt accounting below relies on it)
    const int64_t nrows = min<int64_t>(ROWS, M - r0);
    const __amdgpu_buffer_rsrc_t yres =
        __builtin_amdgcn_make_buffer_rsrc((void*)(y + r0 * N), (short)0, (int)(nrows * N * 2), 0x00020000);
    const int rl = 32 * wave + j;  // the lane's row within the item

    for (int tau = 0; tau < nt; ++tau) {
        AVR_PROBE_BEGIN(comp);
        // W tile tau + NB - 1 into the slot tile tau - 1 left, its DMA pieces
        // issued inside the MFMA chain (one every DSTEP k-steps): issued back
        // to back each stalls the wave behind the previous one, between MFMAs
        // the stall overlaps the matrix pipe (csrc/head_exact.hip, round 4)
        const bool dnext = tau + NB - 1 < nt;
        const char* dsrc =
            reinterpret_cast<const char*>(Wf) + (int64_t)(tau + NB - 1) * TILEB + wave * DPW * 1024 + 16 * lane;
        const uint32_t ddst = ring_lds + ((tau + NB - 1) % NB) * TILEB + wave * DPW * 1024;
        constexpr int DSTEP = kLKS / DPW;
        const char* bsrc = lds_l + (tau % NB) * TILEB + 16 * lane;
        constexpr int D = 8 / NC;  // k-steps of B fragments read ahead
        frag8 bw[D][NC];
#pragma unroll
        for (int u = 0; u < D; ++u)
#pragma unroll
            for (int c = 0; c < NC; ++c) bw[u][c] = *reinterpret_cast<const frag8*>(bsrc + c * kLTile + u * 1024);
        f32x16 acc[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < kLKS; ++ks) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                acc[c] = lmfma<E>(bw[ks % D][c], a[ks], acc[c]);
                if (ks + D < kLKS) bw[ks % D][c] = *reinterpret_cast<const frag8*>(bsrc + c * kLTile + (ks + D) * 1024);
            }
            if (ks % DSTEP == 0 && dnext) ldma16(dsrc + (ks / DSTEP) * 1024, ddst + (ks / DSTEP) * 1024);
        }
        // epilogue: register r of acc[c] is column CT tau + 32 c + (r & 3) +
        // 8 (r >> 2) + 4 half of row rl.  Group pair (2p, 2p + 1) = columns
        // 16p + 4 half + 0..3 and 16p + 8 + 4 half + 0..3: after the half swap
        // a lane owns columns 16p + 8 half + 0..7
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = acc[c][8 * pp + e];
                    if (relu) v[e] = fmaxf(v[e], 0.0f);
                }
                const uint32_t x0 = pack16<E>(v[0], v[1]), x1 = pack16<E>(v[2], v[3]);
                const uint32_t y0 = pack16<E>(v[4], v[5]), y1 = pack16<E>(v[6], v[7]);
                const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                const u32x4 o = u32x4{(uint32_t)s0[0], (uint32_t)s1[0], (uint32_t)s0[1], (uint32_t)s1[1]};
                __builtin_amdgcn_raw_buffer_store_b128(o, yres, (rl * N + CT * tau + 32 * c + 16 * pp + 8 * half) * 2,
                                                       0, 0);
            }
        AVR_PROBE_END(comp, 6);
        AVR_PROBE_BEGIN(dma);
        if (tau + 1 < nt) {
            // this wave's pieces of tile tau+1 have landed.  vmcnt counts the
            // output stores too, in issue order: younger than tile tau+1's
            // DMAs are the ring's later tiles (at most NB-2) and the stores of
            // the iterations since tile tau+1 was issued (NB-1 of them, or
            // 0 .. tau while it came from the prologue), so the wait covers
            // the DMA only, never a store in flight
            const int iters = (tau + 2 - NB >= 0) ? NB - 1 : tau + 1;
            wait_vm(min(NB - 2, nt - 2 - tau) * DPW + iters * ST);
        }
        AVR_PROBE_END(dma, 4);
        AVR_PROBE_BEGIN(bar);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // every LDS read of tile tau done
        __builtin_amdgcn_s_barrier();
        AVR_PROBE_END(bar, 5);
    }
    AVR_PROBE_FLUSH(blockIdx.x * WAVES + wave);
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

// Item shape (probe: AVR_LINEAR_SHAPE_PROBE): 0 = 128 rows, 32-column tiles,
// two workgroups per CU (one's prologue under the other's MFMAs); 1 = 256
// rows, 64-column tiles, one workgroup per CU; 2 = 256 rows, 32-column tiles
int lin_shape(int N) {
    const char* e = AVR_PROBE_ENV("AVR_LINEAR_SHAPE_PROBE");
    const int v = e ? atoi(e) : 0;
    if (v == 1 && N % 64 == 0) return 1;
    return v == 2 ? 2 : 0;
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
    const int shape = lin_shape(N);
    const int rows = shape == 0 ? 128 : 256;
    const int64_t items = (M + rows - 1) / rows;
    AVR_REQUIRE(items < (1ll << 31), "avr_linear_relu_fwd: too many rows");
    hipStream_t st = as_stream(stream);
    auto run = [&](auto e_tag) {
        using E = decltype(e_tag);
        auto go = [&](auto kern, int waves, size_t lds) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(64 * waves), lds, st, M, (int)N, (const E*)x,
                               (const frag8*)Wf, (E*)y, (int)relu);
        };
        if (shape == 0) go(linear_xs_kernel<E, 32, 4, 2>, 4, 2 * (size_t)kLTile);
        else if (shape == 1) go(linear_xs_kernel<E, 64, 8, 2>, 8, 4 * (size_t)kLTile);
        else go(linear_xs_kernel<E, 32, 8, 4>, 8, 4 * (size_t)kLTile);
    };
    if (dtype == AVR_DTYPE_F16)
        run(__half{});
    else
        run(__hip_bfloat16{});
    return check_launch("avr_linear_relu_fwd");
}
