// Hidden layers of the signal network on the matrix cores: y = relu(x W^T)
// for the width-512 layers (model.py:176-180, tcnn FullyFusedMLP /
// CutlassMLP with ReLU, no bias), 16-bit operands, fp32 accumulation, one
// rounding to the 16-bit type (as the GEMM epilogue rounds).
//
// Shape: x [M, 512], W [N, 512] (nn.Linear layout, so both operands are
// contiguous in k), y [M, N] with N a multiple of 256 and M ~ 262,144 rows
// at config 2.  hipBLASLt's solution for it (MT256x256x32, 16x16 MFMAs) runs
// at 0.80-0.85 PFLOP/s; its bytes need ~85 us at HBM speed.
//
// Status: bit-identical to hipBLASLt and as fast (162-169 us
// against 161-162 us warmed up, interleaved in one process), so it is opt-in
// (AVR_LINEAR=1).  Its streaming skeleton alone (no MFMA, no stores) takes
// ~110 us: both N-slices of a tile DMA it (536 MB through LDS-DMA per layer).
//
// Work: persistent workgroups of 8 waves, one per CU.  A workgroup owns a
// 256-wide slice of N: wave w's 32 rows of W are its MFMA B operand, held
// in 128 VGPRs for the whole launch (loaded once, like head_exact.hip's W).
// x streams through LDS in 32-row tiles by LDS-DMA (one 1 KiB row per
// instruction, row stride 1040 B: a 32-row fragment read is conflict-free),
// three tiles in flight behind the one being computed.  The two N-slices of a
// tile run on one XCD at the same time (blockIdx 8 apart), so x is read from
// HBM once and from that L2 the second time.  Per tile a wave runs a chain
// of 32 v_mfma_f32_32x32x16 (32 rows x 32 columns), its A fragments read 6
// k-steps ahead; the epilogue applies the ReLU, rounds, pairs adjacent
// columns and stores dwords.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));

constexpr int kLK = 512;                // K
constexpr int kLKS = kLK / 16;          // k-steps
constexpr int kLTR = 32;                // rows per x tile
constexpr int kLBuf = 4;                // tiles in the LDS ring (3 in flight)
constexpr int kLRowB = kLK * 2 + 16;    // LDS row stride (bytes)
constexpr int kLWaves = 8;
constexpr int kLSlice = 32 * kLWaves;   // N per workgroup
constexpr size_t kLLds = kLBuf * (size_t)kLTR * kLRowB;

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
__device__ __forceinline__ void ldma16_nt(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

template <typename E>
__device__ __forceinline__ unsigned short to16(float v) {
    if constexpr (std::is_same<E, __half>::value)
        return __half_as_ushort(__float2half(v));
    else {
        const __hip_bfloat16 b = __float2bfloat16(v);
        return *reinterpret_cast<const unsigned short*>(&b);
    }
}

// grid: 8 * pairs_per_xcd * nslices workgroups; workgroup g sits on XCD g % 8,
// slice (g / 8) % nslices, pair (g / 8) / nslices of that XCD.  XCD x owns
// the tiles x, x + 8, ... and its pairs split them round-robin.
template <typename E>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_relu_kernel(
    int64_t M, int N, const E* __restrict__ x, const E* __restrict__ W, E* __restrict__ y, int relu, int nslices,
    int pairs, int dbg) {
    constexpr int KS = kLKS, TR = kLTR, ROWB = kLRowB, RPW = TR / kLWaves;
    extern __shared__ __attribute__((aligned(16))) char lds_l[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int xcd = blockIdx.x & 7, r = blockIdx.x >> 3;
    const int slice = r % nslices, pair = r / nslices;
    const int64_t ntiles = (M + TR - 1) / TR;
    // tiles of this workgroup: xcd + 8 * (pair + pairs * i)
    const int64_t first = xcd + 8 * (int64_t)pair, step = 8 * (int64_t)pairs;
    const int64_t mine = first < ntiles ? (ntiles - 1 - first) / step + 1 : 0;
    const int n0 = slice * kLSlice + wave * 32;  // this wave's 32 columns

    frag8 wf[KS];
    {
        const E* wrow = W + (int64_t)(n0 + j) * kLK + 8 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const frag8*>(wrow + 16 * ks);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(wf[ks]));  // landed before the DMAs start
    }
#define AVR_LVMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
    auto issue = [&](int64_t i) {  // this wave's RPW rows of the workgroup's i-th tile
        const int64_t m0 = (first + step * i) * TR;
        char* a = lds_l + (i % kLBuf) * TR * ROWB + wave * RPW * ROWB;
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
            const int64_t row = min(m0 + wave * RPW + rr, M - 1);
            if (dbg & 4)  // experiment: non-temporal policy on the x stream
                ldma16_nt(x + row * kLK + 8 * lane, (uint32_t)(uintptr_t)(a + rr * ROWB));
            else
                ldma16(x + row * kLK + 8 * lane, (uint32_t)(uintptr_t)(a + rr * ROWB));
        }
    };
    // vector-memory bookkeeping (uniform): operations issued by this wave
    // (DMAs and the epilogue's buffer stores, a fixed count each), and the
    // count right after each pending tile's DMAs (FIFO, oldest first)
    constexpr int PD = kLBuf - 1, kStores = 8;
    int issued = 0, npend = 0;
    int fifo[PD];
#pragma unroll
    for (int k = 0; k < PD; ++k) fifo[k] = 0;
    auto push = [&](int64_t i) {
        issue(i);
        issued += RPW;
#pragma unroll
        for (int k = 0; k < PD; ++k)
            if (k == npend) fifo[k] = issued;
        ++npend;
    };
    auto pop_wait = [&]() {  // the oldest pending tile has landed (this wave's rows)
        const int n = issued - fifo[0];
#pragma unroll
        for (int k = 0; k + 1 < PD; ++k) fifo[k] = fifo[k + 1];
        --npend;
        // at most n operations younger than that tile's DMAs may stay
        // outstanding (rounded down to an encodable step: waiting longer is safe)
        if (n >= 40) AVR_LVMCNT(40);
        else if (n >= 32) AVR_LVMCNT(32);
        else if (n >= 24) AVR_LVMCNT(24);
        else if (n >= 20) AVR_LVMCNT(20);
        else if (n >= 16) AVR_LVMCNT(16);
        else if (n >= 12) AVR_LVMCNT(12);
        else if (n >= 8) AVR_LVMCNT(8);
        else if (n >= 4) AVR_LVMCNT(4);
        else AVR_LVMCNT(0);
    };
    constexpr int kDepth = 6;
    for (int64_t i = 0; i < PD && i < mine; ++i) push(i);
    if (mine > 0) {
        pop_wait();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    for (int64_t i = 0; i < mine; ++i) {
        // into the slot tile i - 1 used: every wave left it at the last barrier
        if (i + PD < mine) push(i + PD);
        const char* a = lds_l + (i % kLBuf) * TR * ROWB + j * ROWB + 16 * half;
        f32x16 acc = {};
        frag8 fr[kDepth];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) fr[d] = *reinterpret_cast<const frag8*>(a + 32 * d);
        if (dbg & 2) {  // timing experiment: LDS fragment reads without the MFMAs
#pragma unroll
            for (int n = 0; n < KS; ++n) {
                acc[n & 15] += __uint_as_float(fr[n % kDepth][0]);
                if (n + kDepth < KS) fr[n % kDepth] = *reinterpret_cast<const frag8*>(a + 32 * (n + kDepth));
            }
        } else {
#pragma unroll
            for (int n = 0; n < KS; ++n) {
                acc = lmfma<E>(fr[n % kDepth], wf[n], acc);
                if (n + kDepth < KS) fr[n % kDepth] = *reinterpret_cast<const frag8*>(a + 32 * (n + kDepth));
            }
        }
        __builtin_amdgcn_sched_group_barrier(0x100, kDepth, 0);
#pragma unroll
        for (int n = 0; n < KS; ++n) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (n + kDepth < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if (i + 1 < mine) pop_wait();  // tile i + 1's rows from this wave have landed
        // epilogue: acc[4g + e] is row 8g + 4 half + e of the tile, column
        // n0 + j.  Rows 2p, 2p + 1 of a quad pair up: an even lane stores its
        // value and its odd neighbour's (row 2p, columns j, j + 1), an odd
        // lane the pair of row 2p + 1 (columns j - 1, j): 8 dword stores per
        // lane through a buffer resource over the tile's rows, so rows past M
        // are dropped without control flow (the store count stays fixed)
        const int64_t m0 = (first + step * i) * TR;
        const int rows = (int)min<int64_t>(TR, M - m0);
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(reinterpret_cast<unsigned short*>(y) + m0 * N), (short)0, rows * N * 2, 0x00020000);
        const bool odd = j & 1;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int pq = 0; pq < 2; ++pq) {
                float v0 = acc[4 * g + 2 * pq], v1 = acc[4 * g + 2 * pq + 1];
                if (relu) {
                    v0 = fmaxf(v0, 0.0f);
                    v1 = fmaxf(v1, 0.0f);
                }
                const uint32_t u0 = to16<E>(v0), u1 = to16<E>(v1);
                const uint32_t send = odd ? u0 : u1;
                const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
                const uint32_t word = odd ? (recv | (u1 << 16)) : (u0 | (recv << 16));
                const int row = 8 * g + 4 * half + 2 * pq + (odd ? 1 : 0);
                const int col = n0 + (j & ~1);
                // dbg & 1 (timing experiment): every store offset out of range (dropped)
                // non-temporal (aux 2): 162-169 us against 164-176 plain
                __builtin_amdgcn_raw_buffer_store_b32(word, rsrc, (dbg & 1) ? 0x7ffffff0 : (row * N + col) * 2, 0, 2);
            }
        issued += kStores;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LDS reads of tile i are done
        __builtin_amdgcn_s_barrier();        // every wave's: tile i + 1 is in LDS, tile i's slot is free
        asm volatile("" ::: "memory");
    }
#undef AVR_LVMCNT
    __builtin_amdgcn_s_waitcnt(0);
}

}  // namespace

extern "C" int avr_linear_relu_fwd(int64_t M, int32_t N, int32_t K, const void* x, const void* W, int32_t dtype,
                                   int32_t relu, void* y, void* stream) {
    AVR_REQUIRE(M >= 1 && x && W && y, "avr_linear_relu_fwd: bad args");
    AVR_REQUIRE(K == kLK, "avr_linear_relu_fwd: K must be 512");
    AVR_REQUIRE(N >= kLSlice && N % kLSlice == 0, "avr_linear_relu_fwd: N must be a multiple of 256");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_linear_relu_fwd: fp16 or bf16 operands");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0,
                "avr_linear_relu_fwd: x and W must be 16-byte aligned");
    const int nslices = N / kLSlice;
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // one workgroup per CU: per XCD, pairs * nslices workgroups
    const int64_t ntiles = (M + kLTR - 1) / kLTR;
    int pairs = std::max(1, (cus / 8) / nslices);
    pairs = (int)std::min<int64_t>(pairs, std::max<int64_t>(1, (ntiles + 7) / 8));
    const dim3 grid((unsigned)(8 * pairs * nslices));
    hipStream_t st = as_stream(stream);
    const char* dbg_env = getenv("AVR_LINEAR_DBG");  // timing experiments only (results wrong)
    const int dbg = dbg_env ? atoi(dbg_env) : 0;
    auto go = [&](auto kern, auto e) {
        using E = decltype(e);
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLLds);
        hipLaunchKernelGGL(kern, grid, dim3(512), kLLds, st, M, (int)N, (const E*)x, (const E*)W, (E*)y, (int)relu,
                           nslices, pairs, dbg);
    };
    if (dtype == AVR_DTYPE_F16)
        go(linear_relu_kernel<__half>, __half{});
    else
        go(linear_relu_kernel<__hip_bfloat16>, __hip_bfloat16{});
    return check_launch("avr_linear_relu_fwd");
}
