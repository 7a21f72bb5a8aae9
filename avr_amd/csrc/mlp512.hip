// The signal network's width-512 hidden layers, two at a time, in one launch
// (model.py:176-180: tcnn CutlassMLP, ReLU, no bias; AVRModel's layers 1 and
// 2 of `_model_signal` at inference, the input h1 coming from the fused
// sigma kernel):
//
//   y = relu( relu(x W1^T) W2^T ),   x, y [M][512], W1, W2 [512][512], 16-bit
//
// Each layer accumulates in fp32 on the matrix cores over K = 512 in k order
// (one v_mfma_f32_32x32x16 chain per 32x32 output tile, k-steps ascending)
// and rounds its output once to the 16-bit type, as the unfused layers do.
// The intermediate activation never leaves the chip: HBM traffic is x read
// once and y written once (537 MB at M = 262,144), half that of two layers.
//
// Rows stationary.  A workgroup is one wave per SIMD (4 waves); a work item
// is 128 rows, 32 per wave.  A wave holds its rows' layer-1 operand (32 rows
// x 512 k: 128 VGPRs) and layer 2's accumulators for all 512 output columns
// (16 tiles x 16 = 256 accumulator registers).  Layer 1 runs 32 columns at a
// time; each such tile, rectified and rounded, is two k-steps of layer 2's
// operand, which the transposed product C^T = W_tile x_rows^T leaves in
// registers in fragment order after one v_permlane32_swap per pair of 8-byte
// groups (the linear_fwd.hip epilogue), and layer 2 takes those two k-steps
// into all 16 of its accumulators at once.  So layer 2 never needs the whole
// intermediate activation, and nothing but the 32 x 512 accumulators is kept.
//
// W streams from L2 (both layers, 1 MiB) through a two-slot LDS ring of
// 64 KiB pairs P(c) = {layer-1 tile c (32 rows of W1, all k),
// layer-2 slice c - 1 (all 512 rows of W2, k-steps 2c - 2, 2c - 1)}: the two
// halves of a pair are independent (the slice uses the previous tile's
// output), so their 64 MFMAs interleave with the epilogue of the tile.  The
// ring is register-staged: each wave loads its quarter of pair q + 2 while
// pair q computes and writes the quarter of pair q + 1 it loaded one pair
// earlier into the free slot; every load and LDS access is an ordinary
// compiler-counted instruction.  One barrier per pair.  The pairs repeat with
// period 16 over the items, so layer 2's last slice of an item runs in the
// next item's first pair, followed by that item's output epilogue.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

// Compile-time variants (tools/xbench_mlp.py; the defaults are the product):
// AVR_MLP_DMA 1: the W ring filled by LDS-DMA (global_load_lds_dwordx4) a
// whole pair ahead instead of register staging; AVR_MLP_DBG (timing probes,
// wrong results): bit 0 no W staging, bit 1 no barrier, bit 2 no y stores
// (skipped at run time), bit 3 no layer-1 epilogue (raw accumulator bits).
#ifndef AVR_MLP_DMA
#define AVR_MLP_DMA 0
#endif
#ifndef AVR_MLP_DBG
#define AVR_MLP_DBG 0
#endif
// AVR_MLP_TSTORE 1: y leaves through a per-wave LDS transpose as whole
// 128-byte lines (else each store instruction writes 32 B into 32 rows)
// AVR_MLP_SCHED 1: the pair's MFMA / ring-read order pinned by sched_group_barrier
#ifndef AVR_MLP_SCHED
#define AVR_MLP_SCHED 0
#endif
#ifndef AVR_MLP_TSTORE
#define AVR_MLP_TSTORE 0
#endif

// s_waitcnt vmcnt(n) (gfx9 encoding; expcnt / lgkmcnt not waited on)
#define AVR_MLP_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))

// lane i's 16 bytes at sbase + voff land at LDS byte lds + 16 i (scalar base,
// 32-bit lane offset: one VGPR for every piece)
__device__ __forceinline__ void mlp_dma16(const void* sbase, uint32_t voff, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(voff), "s"(sbase)
                 : "memory", "m0");
}

// workgroup barrier that waits for the LDS traffic only: the W staging
// loads and y stores in flight are not waited for (the compiler waits for a
// load where its registers are used); "memory" keeps LDS accesses on their side
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));

constexpr int kMK = 512;                  // width (K and N of both layers)
constexpr int kMKS = kMK / 16;            // k-steps (32)
constexpr int kMN = kMK / 32;             // 32-column output tiles per layer (16)
constexpr int kMPair = 2 * kMKS * 1024;   // bytes of one pair: 32 + 32 pieces of 1 KiB
constexpr int kMRows = 128;               // rows per work item (4 waves x 32)
constexpr int kMShare = 2 * kMKS / 4;     // 1 KiB pieces of a pair per wave (16)

template <typename E>
__device__ __forceinline__ f32x16 mma(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

// acc = C^T of a 32x32 tile (lane (j, half), register r: row j, column
// (r & 3) + 8 (r >> 2) + 4 half), rectified and rounded to E: the fragments
// f[p] (p = 0, 1) a lane then holds are columns 16 p + 8 half + 0..7 of row j
template <typename E>
__device__ __forceinline__ void epilogue(const f32x16& acc, frag8 (&f)[2]) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(acc[8 * pp + e], 0.0f);
        const uint32_t x0 = pack16<E>(v[0], v[1]), x1 = pack16<E>(v[2], v[3]);
        const uint32_t y0 = pack16<E>(v[4], v[5]), y1 = pack16<E>(v[6], v[7]);
        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        f[pp] = frag8{(uint32_t)s0[0], (uint32_t)s1[0], (uint32_t)s0[1], (uint32_t)s1[1]};
    }
}

template <typename E>
__global__ __launch_bounds__(256, 1) void mlp512x2_kernel(int64_t M, const E* __restrict__ x,
                                                          const frag8* __restrict__ Wf, E* __restrict__ y,
                                                          int nitems) {
    extern __shared__ __attribute__((aligned(16))) char lds_m[];  // [2][kMPair]
    const int lane = threadIdx.x & 63, half = lane >> 5, j = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = gridDim.x;
    if ((int)blockIdx.x >= nitems) return;  // (the host launches at most nitems workgroups)

    frag8 ax[kMKS];      // layer-1 operand: the item's rows
    f32x16 acc2[kMN];    // layer-2 accumulators, 512 columns
    frag8 bx[2];         // layer-2 operand: two k-steps (the last layer-1 tile's output)
    frag8 stg[kMShare / 2];  // half of this wave's quarter of a pair, in flight

    // pair p (0..15) of the stream: this wave's pieces 16 wave + 8 h + i
    auto load_half = [&](int p, int h) {
        const frag8* src = Wf + (int64_t)p * (kMPair / 16) + (kMShare * wave + 8 * h) * 64 + lane;
#pragma unroll
        for (int i = 0; i < kMShare / 2; ++i) stg[i] = src[i * 64];
    };
    // LDS-DMA form: this wave's 16 pieces of pair p into ring slot `slot`
    auto dma_pair = [&](int p, int slot) {
        const char* src = reinterpret_cast<const char*>(Wf) + (int64_t)p * kMPair + kMShare * wave * 1024;
        const uint32_t dst = (uint32_t)(uintptr_t)(lds_m + slot * kMPair) + kMShare * wave * 1024;
#pragma unroll
        for (int i = 0; i < kMShare; ++i) mlp_dma16(src + i * 1024, 16 * lane, dst + i * 1024);
    };
    auto write_half = [&](int slot, int h) {
        frag8* dst = reinterpret_cast<frag8*>(lds_m + slot * kMPair) + (kMShare * wave + 8 * h) * 64 + lane;
#pragma unroll
        for (int i = 0; i < kMShare / 2; ++i) dst[i * 64] = stg[i];
    };
    // the wave's 32 rows of item `it` (rows past M repeat the last one; their
    // outputs are dropped), fragment ks = 16-byte group 2 ks + half
    auto load_rows = [&](int it) {
        const int64_t r = std::min<int64_t>((int64_t)it * kMRows + 32 * wave + j, M - 1);
        const frag8* xr = reinterpret_cast<const frag8*>(x + r * kMK) + half;
#pragma unroll
        for (int ks = 0; ks < kMKS; ++ks) ax[ks] = xr[2 * ks];
    };
    // layer 2's output of item `it`: rectified, rounded, 16-byte stores
    auto store_out = [&](int it) {
        const int64_t r0 = (int64_t)it * kMRows;
        const int64_t nrows = std::min<int64_t>(kMRows, M - r0);
        const __amdgpu_buffer_rsrc_t yres =
            __builtin_amdgcn_make_buffer_rsrc((void*)(y + r0 * kMK), (short)0, (int)(nrows * kMK * 2), 0x00020000);
        const bool st_on = !(AVR_MLP_DBG & 4) || M < 0;  // (DBG 4: stores skipped at run time)
        if constexpr (AVR_MLP_TSTORE) {
            // through this wave's 4 KiB of LDS, two tiles (64 columns) at a
            // time: written as the fragments lie (row j, 16-byte chunk
            // 4 (n & 1) + 2 pp + half, XOR-swizzled by row), read back as
            // 8 rows x 128 contiguous bytes per instruction (whole lines)
            char* tr = lds_m + 2 * kMPair + wave * 4096;
#pragma unroll
            for (int m = 0; m < kMN / 2; ++m) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    frag8 f[2];
                    epilogue<E>(acc2[2 * m + u], f);
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp)
                        *reinterpret_cast<frag8*>(tr + j * 128 + (((4 * u + 2 * pp + half) ^ (j & 7)) * 16)) = f[pp];
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int row = 8 * q + (lane >> 3), ch = lane & 7;
                    const frag8 v = *reinterpret_cast<const frag8*>(tr + row * 128 + ((ch ^ (row & 7)) * 16));
                    if (st_on)
                        __builtin_amdgcn_raw_buffer_store_b128(v, yres, ((32 * wave + row) * kMK + 64 * m + 8 * ch) * 2,
                                                               0, 0);
                }
            }
        } else {
            const int rl = 32 * wave + j;
#pragma unroll
            for (int n = 0; n < kMN; ++n) {
                frag8 f[2];
                epilogue<E>(acc2[n], f);
#pragma unroll
                for (int pp = 0; pp < 2; ++pp)
                    if (st_on)
                        __builtin_amdgcn_raw_buffer_store_b128(f[pp], yres,
                                                               (rl * kMK + 32 * n + 16 * pp + 8 * half) * 2, 0, 0);
            }
        }
    };
    // The 64 MFMAs of a pair, layer 1's tile and layer 2's slice alternating
    // (s even: layer-1 k-step s / 2, piece s / 2; s odd: layer-2 column
    // tile n = (s - 1) / 4, k-step (s - 1) / 2 % 2, piece 32 + (s - 1) / 2),
    // the W fragments read D ahead in that order.  `mid` runs at the middle.
#ifndef AVR_MLP_D
#define AVR_MLP_D 6
#endif
    constexpr int D = AVR_MLP_D;  // (8 spills a few registers)
    auto piece = [](int st) { return (st & 1) ? kMKS + (st >> 1) : (st >> 1); };
    auto run_pair = [&](const frag8* ring, f32x16& acc1, bool t1, auto&& mid) {
        frag8 bw[D];
#pragma unroll
        for (int u = 0; u < D; ++u) bw[u] = ring[piece(u) * 64];
#pragma unroll
        for (int st = 0; st < 4 * kMKS / 2; ++st) {
            if ((st & 1) == 0) {
                if (t1) acc1 = mma<E>(bw[st % D], ax[st >> 1], acc1);
            } else {
                const int i = st >> 1;
                acc2[i >> 1] = mma<E>(bw[st % D], bx[i & 1], acc2[i >> 1]);
            }
            if (st + D < 2 * kMKS) bw[st % D] = ring[piece(st + D) * 64];
#if AVR_MLP_SCHED
            // issue order pinned: this step's MFMA, then the read D steps
            // ahead (left to itself the scheduler issues each read just
            // before its MFMA, two or three reads of lead)
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (st + D < 2 * kMKS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#endif
            if (st == kMKS - 1) mid();
        }
    };

    load_rows(blockIdx.x);
    if constexpr (AVR_MLP_DMA) {
        dma_pair(0, 0);
        AVR_MLP_VMCNT(0);
    } else {
        load_half(0, 0);
        write_half(0, 0);
        load_half(0, 1);
        write_half(0, 1);
        load_half(1, 0);
    }
    lds_barrier();
#pragma unroll
    for (int n = 0; n < kMN; ++n) acc2[n] = f32x16{};
    bx[0] = bx[1] = frag8{0u, 0u, 0u, 0u};  // the first pair's layer-2 slice adds zeros

    int q = 0;          // pairs computed so far
    int prev = -1;      // the item whose layer-2 slice 15 is in the next pair 0 (-1: none)
    for (int it = blockIdx.x; it < nitems; it += G) {
        for (int c = 0; c < kMN; ++c, ++q) {
            const frag8* ring = reinterpret_cast<const frag8*>(lds_m + (q & 1) * kMPair) + lane;
            const int slot1 = (q + 1) & 1;  // free: every wave passed pair q - 1's barrier
            // pair q + 1: first half written now (loaded during pair q - 1),
            // second half loaded now and written mid-pair; pair q + 2's first
            // half loaded after that
            if constexpr (AVR_MLP_DMA) {
                // nothing of this wave's in flight on the vector-memory counter
                // (the previous pair's pieces were waited for; the rows and y
                // stores here): the compiler, which cannot count the DMA
                // below, then waits for nothing inside the pair
                AVR_MLP_VMCNT(0);
                if (!(AVR_MLP_DBG & 1)) dma_pair((c + 1) % kMN, slot1);
            } else if (!(AVR_MLP_DBG & 1)) {
                write_half(slot1, 0);
                load_half((c + 1) % kMN, 1);
            }
            f32x16 acc1 = f32x16{};
            run_pair(ring, acc1, true, [&] {
                if constexpr (!AVR_MLP_DMA && !(AVR_MLP_DBG & 1)) {
                    write_half(slot1, 1);
                    load_half((c + 2) % kMN, 0);
                } else {
                    asm volatile("" ::: "memory");  // (the two halves scheduled apart, as with staging)
                }
            });
            if (c == 0 && prev >= 0) {
                store_out(prev);
#pragma unroll
                for (int n = 0; n < kMN; ++n) acc2[n] = f32x16{};
            }
            if constexpr (AVR_MLP_DBG & 8) {  // (timing probe: the raw accumulator bits)
                bx[0] = frag8{__float_as_uint(acc1[0]), __float_as_uint(acc1[1]), __float_as_uint(acc1[2]),
                              __float_as_uint(acc1[3])};
                bx[1] = frag8{__float_as_uint(acc1[4]), __float_as_uint(acc1[5]), __float_as_uint(acc1[6]),
                              __float_as_uint(acc1[7])};
            } else {
                epilogue<E>(acc1, bx);
            }
            if (c == kMN - 1) {
                // the last use of this item's rows was tile 15: the next item's
                const int nxt = it + G;
                // (not scheduled into the pair above: both items' rows live
                // at once would not fit the register file)
                __builtin_amdgcn_sched_barrier(0);
                if (nxt < nitems) load_rows(nxt);
                prev = it;
            }
            if constexpr (AVR_MLP_DMA) {
                // this wave's pieces of pair q + 1 landed: younger are the y
                // stores of pair 0 and the next item's row loads of pair 15
                const int young = (c == 0 && prev >= 0 && !(AVR_MLP_DBG & 4) ? 2 * kMN : 0) +
                                  (c == kMN - 1 && it + G < nitems ? kMKS : 0);
                if (young == 0) AVR_MLP_VMCNT(0);
                else if (young == 2 * kMN) AVR_MLP_VMCNT(2 * kMN);
                else if (young == kMKS) AVR_MLP_VMCNT(kMKS);
                else AVR_MLP_VMCNT(2 * kMN + kMKS);
            }
            if (!(AVR_MLP_DBG & 2)) lds_barrier();
        }
    }
    // layer 2's slice 15 of the last item: the second half of pair 0
    {
        const frag8* ring = reinterpret_cast<const frag8*>(lds_m + (q & 1) * kMPair) + lane;
        f32x16 acc1 = f32x16{};
        run_pair(ring, acc1, false, [] {});
        store_out(prev);
    }
}

// W1, W2 [512][512] -> Wf, 16 pairs of 64 KiB: pair c = layer-1 tile c
// (piece ks: lane (j, h) holds W1[32 c + j][16 ks + 8 h + 0..7]) then layer-2
// slice s = (c + 15) mod 16 (piece 32 + 2 n + kk: W2[32 n + j][16 (2 s + kk) + 8 h + 0..7])
__global__ __launch_bounds__(256) void mlp512_pack_kernel(const uint16_t* __restrict__ W1,
                                                          const uint16_t* __restrict__ W2, frag8* __restrict__ Wf,
                                                          int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int lane = (int)(i & 63), jl = lane & 31, hl = lane >> 5;
        const int piece = (int)((i >> 6) % (2 * kMKS));
        const int c = (int)((i >> 6) / (2 * kMKS));
        const uint16_t* src;
        if (piece < kMKS) {
            src = W1 + (int64_t)(32 * c + jl) * kMK + 16 * piece + 8 * hl;
        } else {
            const int nn = (piece - kMKS) >> 1, kk = (piece - kMKS) & 1, s = (c + kMN - 1) % kMN;
            src = W2 + (int64_t)(32 * nn + jl) * kMK + 16 * (2 * s + kk) + 8 * hl;
        }
        Wf[i] = *reinterpret_cast<const frag8*>(src);
    }
}

}  // namespace

extern "C" int avr_mlp512x2_pack_w(const void* W1, const void* W2, int32_t dtype, void* Wf, void* stream) {
    AVR_REQUIRE(W1 && W2 && Wf, "avr_mlp512x2_pack_w: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_mlp512x2_pack_w: fp16 or bf16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(W1) % 16 == 0 && reinterpret_cast<uintptr_t>(W2) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_mlp512x2_pack_w: W1, W2 and Wf must be 16-byte aligned");
    const int64_t n = (int64_t)kMN * (kMPair / 16);  // fragments of both layers
    hipLaunchKernelGGL(mlp512_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (const uint16_t*)W1, (const uint16_t*)W2, (frag8*)Wf, n);
    return check_launch("avr_mlp512x2_pack_w");
}

extern "C" int avr_mlp512x2_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, void* y, void* stream) {
    AVR_REQUIRE(M >= 1 && x && Wf && y, "avr_mlp512x2_fwd: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_mlp512x2_fwd: fp16 or bf16 operands");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(y) % 16 == 0,
                "avr_mlp512x2_fwd: x, Wf and y must be 16-byte aligned");
    const int64_t items = (M + kMRows - 1) / kMRows;
    AVR_REQUIRE(items < (1ll << 31) && M < (1ll << 40), "avr_mlp512x2_fwd: too many rows");
    const int cus = device_cus();
    const int grid = (int)std::min<int64_t>(items, std::max(cus, 1));
    const size_t lds = 2 * (size_t)kMPair + (AVR_MLP_TSTORE ? 4 * 4096 : 0);
    hipStream_t st = as_stream(stream);
    auto go = [&](auto e_tag) {
        using E = decltype(e_tag);
        auto kern = mlp512x2_kernel<E>;
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, M, (const E*)x, (const frag8*)Wf, (E*)y,
                           (int)items);
    };
    if (dtype == AVR_DTYPE_F16)
        go(__half{});
    else
        go(__hip_bfloat16{});
    return check_launch("avr_mlp512x2_fwd");
}
