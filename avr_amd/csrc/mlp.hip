// Weight gradient of the networks' bias-free linear layers (a6), bf16 MFMA.
//
//   dW[m][k] = sum_n gy[n][m] * x[n][k]      gy [N][M], x [N][K] bf16, dW fp32
//
// The reference trains its MLPs inside tcnn (model.py:21-31, 117-121,
// 176-180); here they are PyTorch GEMMs, and the one shape hipBLASLt serves
// badly is exactly this one: N = B*R*S = 1e5..1e6 rows reduced into a small
// (<= 1600 x 512) output, i.e. a few dozen output tiles for 256 CUs
// (0.15 PFLOP/s measured, tools/mm_probe.py), and batching it as split-K
// costs ~1 ms of host time per call once several shapes alternate.
//
// Split-K MFMA kernel: a 256-thread workgroup owns a 128 x 128 tile of dW and
// a range of n; four waves each compute 64 x 64 with v_mfma_f32_32x32x16_bf16.
// Both operands are stored n-major (the reduction index is the ROW), so
// 32-row slabs are kept row-major in LDS and read back with
// ds_read_b64_tr_b16, the CDNA4 transposing LDS read, which hands each lane
// 4 consecutive rows of one column.  The image is XOR-swizzled per 16-byte
// chunk (cdna_hip_programming.md T10 image (b)) so those reads are
// conflict-free.  The slabs stream into a four-slot LDS ring by LDS-DMA
// (global_load_lds_dwordx4): three slabs in flight per workgroup, one
// barrier per slab (round 5; the round-1..4 form staged one slab through
// registers with two barriers per slab and was bitwise equal and 14-30 %
// slower, tools/bench_wgrad.py).  fp32 partials per n-range are summed in a
// fixed order by a second kernel (deterministic).
#include "common.h"

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

using namespace avr;

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 128;   // dW tile edge (both m and k)
constexpr int kSlab = 32;    // rows of n per LDS slab
constexpr int kImg = kSlab * kTile * 2;  // bytes of one operand image (8 KiB)

// byte offset of 16-byte chunk `ch` (0..15) of image row `row` (0..31)
__device__ __forceinline__ int img_off(int row, int ch) {
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ s16x4 tr_read(const char* lds_base, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds_base + byte_off));
}

// Each DMA instruction fills 4 image rows (1 KiB, lane l at byte 16 l): lane
// l of rows 4j .. 4j+3 fetches the logical chunk that img_off places at its
// physical chunk (the XOR swizzle is an involution).  Rows past the split's
// end read a zero row in device memory.
__device__ __attribute__((aligned(16))) uint32_t g_wgrad_zero_row[64];  // 256 B of zeros (.bss)

__device__ __forceinline__ void wg_dma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// s_waitcnt vmcnt(4 ahead): this wave's DMAs of all but the `ahead` youngest
// slabs landed (4 per slab; expcnt / lgkmcnt not waited on)
#define AVR_WG_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
__device__ __forceinline__ void wg_wait_slabs(int ahead) {
    switch (ahead) {
        case 0: AVR_WG_VMCNT(0); break;
        case 1: AVR_WG_VMCNT(4); break;
        case 2: AVR_WG_VMCNT(8); break;
        case 3: AVR_WG_VMCNT(12); break;
        case 4: AVR_WG_VMCNT(16); break;
        case 5: AVR_WG_VMCNT(20); break;
        default: AVR_WG_VMCNT(24); break;
    }
}

// AVR_WG_SLOTS: ring slots of one slab (A and B images, 16 KiB each);
// AVR_WG_DBG (timing probes, results wrong): bit 0 no DMA, bit 1 no MFMAs,
// bit 2 no barrier
#ifndef AVR_WG_SLOTS
#define AVR_WG_SLOTS 4
#endif
#ifndef AVR_WG_DBG
#define AVR_WG_DBG 0
#endif
constexpr int kWgSlots = AVR_WG_SLOTS;

__global__ __launch_bounds__(256) void linear_wgrad_dma_kernel(int64_t N, int M, int K, int64_t rows_per_split,
                                                                int used, const __hip_bfloat16* __restrict__ gy,
                                                                const __hip_bfloat16* __restrict__ x,
                                                                float* __restrict__ partial) {
    __shared__ __attribute__((aligned(1024))) char lds[kWgSlots * 2 * kImg];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tiles_k = (K + kTile - 1) / kTile;
    const int tiles = tiles_k * ((M + kTile - 1) / kTile);
    const int b = blockIdx.x;
    // block b runs on XCD b % 8; all tiles of a split go to the same XCD, so
    // the split's rows are read from HBM once into that XCD's L2
    const int tile = (b >> 3) % tiles;
    const int split = (b & 7) + 8 * ((b >> 3) / tiles);
    if (split >= used) return;  // padding blocks of the XCD map (block-uniform)
    const int m0 = (tile / tiles_k) * kTile, k0 = (tile % tiles_k) * kTile;
    const int64_t n_begin = (int64_t)split * rows_per_split;
    const int64_t n_end = min(N, n_begin + rows_per_split);
    const int nslab = (int)((n_end - n_begin + kSlab - 1) / kSlab);

    // this wave's DMA instructions: image rows 4j .. 4j+3, j = 2 wave + u, of
    // both operands; lane l -> row 4j + l/16, physical chunk l%16
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    int drow[2], acol[2], bcol[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int row = 4 * (2 * wave + u) + (lane >> 4);
        const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        drow[u] = row;
        // columns past M / K clamped to a valid chunk (never stored)
        acol[u] = min(m0 + 8 * ch, M - 8);
        bcol[u] = min(k0 + 8 * ch, K - 8);
    }
    auto issue = [&](int s) {
        const uint32_t slot = lds_base + (uint32_t)((s % kWgSlots) * 2 * kImg);
        const int64_t n0 = n_begin + (int64_t)s * kSlab;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (AVR_WG_DBG & 1) break;
            const int64_t n = n0 + drow[u];
            const bool ok = n < n_end;
            const void* ga = ok ? (const void*)(gy + n * M + acol[u]) : (const void*)g_wgrad_zero_row;
            const void* gb = ok ? (const void*)(x + n * K + bcol[u]) : (const void*)g_wgrad_zero_row;
            const uint32_t off = (uint32_t)(1024 * (2 * wave + u));
            wg_dma16(ga, __builtin_amdgcn_readfirstlane(slot + off));
            wg_dma16(gb, __builtin_amdgcn_readfirstlane(slot + kImg + off));
        }
    };

    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int wm = wave & 1, wk = wave >> 1;
    auto tr_addr = [&](int colblock, int kh, int second) {
        const int c0 = colblock + 16 * (g & 1);
        const int row = 16 * kh + 8 * (g >> 1) + 4 * second + qq;
        return img_off(row, (c0 >> 3) + (pp >> 1)) + 8 * (pp & 1);
    };
    int aoff[2][2][2], boff[2][2][2];  // [block][kh][second]
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int sc = 0; sc < 2; ++sc) {
                aoff[blk][kh][sc] = tr_addr(64 * wm + 32 * blk, kh, sc);
                boff[blk][kh][sc] = tr_addr(64 * wk + 32 * blk, kh, sc) + kImg;
            }

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    for (int s = 0; s < kWgSlots - 1 && s < nslab; ++s) issue(s);
    for (int s = 0; s < nslab; ++s) {
        // this wave's DMA of slab s landed (slabs s+1, s+2 may still fly);
        // the barrier makes every wave's landed and frees slot (s-1) % 4
        wg_wait_slabs(min(kWgSlots - 2, nslab - 1 - s));
        if (!(AVR_WG_DBG & 4)) __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
        if (s + kWgSlots - 1 < nslab) issue(s + kWgSlots - 1);
        const char* img = lds + (s % kWgSlots) * 2 * kImg;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            bf16x8 av[2], bv[2];
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                const s16x4 a0 = tr_read(img, aoff[blk][kh][0]), a1 = tr_read(img, aoff[blk][kh][1]);
                const s16x4 b0 = tr_read(img, boff[blk][kh][0]), b1 = tr_read(img, boff[blk][kh][1]);
                const s16x8 a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const s16x8 bb = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                av[blk] = __builtin_bit_cast(bf16x8, a);
                bv[blk] = __builtin_bit_cast(bf16x8, bb);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (AVR_WG_DBG & 2) {  // keep the reads: fold them into one register
                        acc[i][j][0] += (float)av[i][0] + (float)bv[j][0];
                        continue;
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
                }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    float* out = partial + (int64_t)split * M * K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = k0 + 64 * wk + 32 * j + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (m < M && k < K) out[(int64_t)m * K + k] = acc[i][j][r];
            }
        }
}

// dW = sum over splits of the partials.  A workgroup covers Q = 256/G
// consecutive 16-byte output quads; its G thread groups each sum the splits
// g, g+G, g+2G, ... of every quad in order (consecutive threads read
// consecutive quads of one split: coalesced), then the G partial sums are
// added in group order through LDS.  G grows (up to 64) while the grid is too
// small to fill the chip, so a small layer split many ways does not become a
// long serial chain.  The order is fixed, so the result is deterministic.
__global__ __launch_bounds__(256) void wgrad_finalize_kernel(int64_t MK, int splits, int G,
                                                              const float* __restrict__ partial,
                                                              float* __restrict__ out) {
    __shared__ f32x4 red[256];
    const int Q = 256 / G;
    const int q = threadIdx.x % Q, g = threadIdx.x / Q;
    const int64_t i = ((int64_t)blockIdx.x * Q + q) * 4;
    f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
    if (i < MK) {
#pragma unroll 4
        for (int k = g; k < splits; k += G)
            s += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(partial + (int64_t)k * MK + i));
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (g == 0 && i < MK) {
        for (int h = 1; h < G; ++h) s += red[h * Q + q];
        *reinterpret_cast<f32x4*>(out + i) = s;
    }
}

// ------------------------------------------- a layer with ONE output (a6)
// The sigma decoder's last layer (model.py:117-121, 259-262: tcnn network
// to 1 output), y[n] = sum_k x[n][k] w[k], x [N][K] 16-bit, K % 8 == 0,
// K <= 512.  As a GEMM it is an N x 1 output tile stream at a fraction of
// HBM speed (22-27 us for 21 MB at config 3); here a row is K/8 lanes of 16
// bytes, summed in fp32 per lane and then over the row's lanes by a fixed
// butterfly, rounded once to the 16-bit type.
template <typename E>
__global__ __launch_bounds__(256) void linear_out1_fwd_kernel(int64_t N, int K, const E* __restrict__ x,
                                                               const E* __restrict__ w, E* __restrict__ y) {
    const int L = K / 8;  // lanes per row (a power of two: 1 .. 64)
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n = i / L;
    const int c = (int)(i % L);
    float acc = 0.0f;
    if (n < N) {
        const u32x4 xv = *reinterpret_cast<const u32x4*>(x + n * K + 8 * c);
        const u32x4 wv = *reinterpret_cast<const u32x4*>(w + 8 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc = fmaf(unpack16<E>(xv[e], 0), unpack16<E>(wv[e], 0), acc);
            acc = fmaf(unpack16<E>(xv[e], 1), unpack16<E>(wv[e], 1), acc);
        }
    }
    for (int m = 1; m < L; m <<= 1) acc += __shfl_xor(acc, m);
    if (n < N && c == 0) store_f(y, n, acc);
}

// Backward of the same layer in one pass over x: gx[n][k] = gy[n] w[k]
// (one product, rounded: the broadcast multiply's arithmetic) and, per
// workgroup, the fp32 partial sum_n gy[n] x[n][k] over its rows; the
// partials are summed in workgroup order by wgrad_finalize_kernel.
template <typename E>
__global__ __launch_bounds__(256) void linear_out1_bwd_kernel(int64_t N, int K, int64_t rows_per_block,
                                                               const E* __restrict__ x, const E* __restrict__ w,
                                                               const E* __restrict__ gy, E* __restrict__ gx,
                                                               float* __restrict__ partial) {
    __shared__ f32x4 red[2][256];
    const int L = K / 8, rpi = 256 / L;  // lanes per row, rows per pass
    const int c = threadIdx.x % L, r0 = threadIdx.x / L;
    const int64_t nb = (int64_t)blockIdx.x * rows_per_block, ne = min(N, nb + rows_per_block);
    const u32x4 wv = *reinterpret_cast<const u32x4*>(w + 8 * c);
    float wf[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        wf[2 * e] = unpack16<E>(wv[e], 0);
        wf[2 * e + 1] = unpack16<E>(wv[e], 1);
    }
    float acc[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int64_t n = nb + r0; n < ne; n += rpi) {
        const float g = load_f(gy, n);
        const u32x4 xv = *reinterpret_cast<const u32x4*>(x + n * K + 8 * c);
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc[2 * e] = fmaf(g, unpack16<E>(xv[e], 0), acc[2 * e]);
            acc[2 * e + 1] = fmaf(g, unpack16<E>(xv[e], 1), acc[2 * e + 1]);
            o[e] = pack16<E>(g * wf[2 * e], g * wf[2 * e + 1]);
        }
        *reinterpret_cast<u32x4*>(gx + n * K + 8 * c) = o;
    }
    // the rpi row groups' sums of each lane column, added in group order
    red[0][threadIdx.x] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    red[1][threadIdx.x] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    __syncthreads();
    if (threadIdx.x < L) {
        f32x4 a = red[0][threadIdx.x], b = red[1][threadIdx.x];
        for (int q = 1; q < rpi; ++q) {
            a += red[0][q * L + threadIdx.x];
            b += red[1][q * L + threadIdx.x];
        }
        float* out = partial + (int64_t)blockIdx.x * K + 8 * threadIdx.x;
        *reinterpret_cast<f32x4*>(out) = a;
        *reinterpret_cast<f32x4*>(out + 4) = b;
    }
}

// ------------------------------- narrow layers: Y = act(X Bt^T), C <= 256
// The sigma networks' layers (model.py:117-121, 259-262: widths 80 .. 256)
// at the training step's 83,200 .. 147,712 rows.  As hipBLASLt GEMMs they
// run at 1-3 TB/s (the N x C output is a stream of small tiles), and a ReLU
// layer's data gradient adds a threshold pass.  Here the whole of Bt
// [C][R] (<= 256 x 256, 16-bit) sits in LDS (rows padded by 16 B: the
// fragment reads are conflict-free), each wave takes 32 rows of X and forms
// Y^T = Bt X^T tile by tile (v_mfma_f32_32x32x16: A = Bt fragment from LDS,
// B = 16 bytes of an X row straight from memory), so a lane ends with one
// row's 4-column groups.  ACT: 0 none, 1 ReLU (the forward's epilogue),
// 2 mask (0 where Mk <= 0, NaN keeps: a data gradient with the input ReLU's
// backward, threshold_backward's selection).  One rounding of the fp32 sum.
typedef uint32_t frag4u __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

template <typename E>
__device__ __forceinline__ f32x16 mfma16(frag4u a, frag4u b, f32x16 c) {
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

template <typename E>
__device__ __forceinline__ uint32_t narrow_keep(uint32_t v, uint32_t m) {
    constexpr uint32_t kInf = std::is_same<E, __half>::value ? 0x7c00u : 0x7f80u;
    const uint32_t lo = m & 0xffffu, hi = m >> 16;
    const bool zlo = lo == 0u || lo - 0x8000u <= kInf, zhi = hi == 0u || hi - 0x8000u <= kInf;
    return (zlo ? 0u : (v & 0xffffu)) | (zhi ? 0u : (v & 0xffff0000u));
}

constexpr int kNarrowRows = 128;  // rows per workgroup tile (4 waves x 32)
#ifndef AVR_NARROW_STAGE
#define AVR_NARROW_STAGE 1
#endif

// STAGE: the tile's X rows land in LDS first (coalesced 16-byte loads, rows
// padded by 16 B like Bt), and the fragments are read from there; otherwise
// each lane loads its row's 16-byte pieces straight from memory (32 rows x
// 32 B per wave instruction).
template <typename E, int NCT, int NKS, int ACT, bool STAGE>
__global__ __launch_bounds__(256, 2) void narrow_mm_kernel(int64_t N, int R, int C, const E* __restrict__ X,
                                                         const E* __restrict__ Bt, const E* __restrict__ Mk,
                                                         E* __restrict__ Y) {
    extern __shared__ frag4u bl[];  // [NCT * 32][R / 8 + 1] 16-byte pieces, then (STAGE) X [128][R / 8 + 1]
    const int pieces = R / 8, stride = pieces + 1;
    frag4u* xs = bl + NCT * 32 * stride;
    for (int i = threadIdx.x; i < NCT * 32 * pieces; i += 256) {
        const int c = i / pieces, p = i % pieces;
        bl[c * stride + p] = c < C ? *reinterpret_cast<const frag4u*>(Bt + (int64_t)c * R + 8 * p) : frag4u{};
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
    const int64_t ntiles = (N + kNarrowRows - 1) / kNarrowRows;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t n = tile * kNarrowRows + 32 * wave + j;
        const bool ok = n < N;
        frag4u xf[NKS];
        if constexpr (STAGE) {
            constexpr int kP = 2 * NKS;  // pieces per row
            frag4u v[NKS];               // 128 kP pieces over 256 threads: kP / 2 each
#pragma unroll
            for (int i = 0; i < NKS; ++i) {
                const int idx = threadIdx.x + 256 * i, row = idx / kP, p = idx % kP;
                const int64_t nn = tile * kNarrowRows + row;
                v[i] = nn < N ? *reinterpret_cast<const frag4u*>(X + nn * R + 8 * p) : frag4u{};
            }
            __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
            for (int i = 0; i < NKS; ++i) {
                const int idx = threadIdx.x + 256 * i, row = idx / kP, p = idx % kP;
                xs[row * stride + p] = v[i];
            }
            __syncthreads();
#pragma unroll
            for (int s = 0; s < NKS; ++s) xf[s] = xs[(32 * wave + j) * stride + 2 * s + h];
        } else {
            const E* xr = X + (ok ? n : 0) * R + 8 * h;
#pragma unroll
            for (int s = 0; s < NKS; ++s) xf[s] = ok ? *reinterpret_cast<const frag4u*>(xr + 16 * s) : frag4u{};
        }
        f32x16 acc[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] = f32x16{};
        // Bt fragments one k-step ahead of the MFMAs that use them (the
        // fences keep hipcc from hoisting every k-step's reads at once)
        frag4u af[2][NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) af[0][ct] = bl[(32 * ct + j) * stride + h];
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            if (s + 1 < NKS) {
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) af[(s + 1) & 1][ct] = bl[(32 * ct + j) * stride + 2 * (s + 1) + h];
            }
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) acc[ct] = mfma16<E>(af[s & 1][ct], xf[s], acc[ct]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (!ok) continue;  // (STAGE: no barrier follows in this tile)
        // lane (j, h) holds Y[n][32 ct + 8 q + 4 h + i] in acc[ct][4 q + i]
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int c0 = 32 * ct + 8 * q + 4 * h;
                if (c0 >= C) continue;
                const f32x16& v = acc[ct];
                float a0 = v[4 * q], a1 = v[4 * q + 1], a2 = v[4 * q + 2], a3 = v[4 * q + 3];
                if (ACT == 1) {
                    a0 = __builtin_elementwise_maximum(a0, 0.0f);
                    a1 = __builtin_elementwise_maximum(a1, 0.0f);
                    a2 = __builtin_elementwise_maximum(a2, 0.0f);
                    a3 = __builtin_elementwise_maximum(a3, 0.0f);
                }
                u32x2v o = {pack16<E>(a0, a1), pack16<E>(a2, a3)};
                if (ACT == 2) {
                    const u32x2v m = *reinterpret_cast<const u32x2v*>(Mk + n * C + c0);
                    o[0] = narrow_keep<E>(o[0], m[0]);
                    o[1] = narrow_keep<E>(o[1], m[1]);
                }
                *reinterpret_cast<u32x2v*>(Y + n * C + c0) = o;
            }
    }
}

constexpr int kOut1Blocks = 512;  // backward workgroups (partials of K floats each)

// Workgroups aimed for: two per CU for the width-512 layers (16 tiles and
// more), one per CU below, where the fp32 partials (splits x M x K x 4
// bytes, written and read back) are a large share of the traffic: e.g.
// 128 x 128 at 83,200 rows 19.7 -> 16.5 us (tools/xbench_wgrad.py).
// AVR_WG_TARGET overrides both; AVR_WG_PCAP keeps the partials below
// 1 / AVR_WG_PCAP of the operand bytes (N (M + K) x 2), 0 = no cap.
#ifndef AVR_WG_TARGET
#define AVR_WG_TARGET 0
#endif
#ifndef AVR_WG_PCAP
#define AVR_WG_PCAP 0
#endif
int wgrad_splits(int64_t N, int M, int K) {
    const int tiles = ((M + kTile - 1) / kTile) * ((K + kTile - 1) / kTile);
    const int target = AVR_WG_TARGET > 0 ? AVR_WG_TARGET : (tiles >= 16 ? 512 : 256);
    int splits = (target + tiles - 1) / tiles;
    const int64_t max_by_rows = N / 256 > 1 ? N / 256 : 1;  // >= 8 slabs per split
    if (splits > max_by_rows) splits = (int)max_by_rows;
    if (AVR_WG_PCAP > 0) {
        const int64_t cap = N * (M + K) * 2 / ((int64_t)AVR_WG_PCAP * M * K * 4);
        if (splits > cap) splits = (int)(cap > 8 ? cap : 8);
    }
    return splits;
}

}  // namespace

extern "C" int avr_linear_wgrad_splits(int64_t N, int32_t M, int32_t K, int32_t* splits) {
    AVR_REQUIRE(N >= 1 && M >= 8 && K >= 8 && splits, "avr_linear_wgrad_splits: bad args");
    *splits = wgrad_splits(N, M, K);
    return 0;
}

extern "C" int avr_linear_wgrad(int64_t N, int32_t M, int32_t K, const void* grad_y, const void* x,
                                float* workspace, int32_t splits, float* grad_w, void* stream) {
    AVR_REQUIRE(N >= 1 && M >= 8 && K >= 8 && grad_y && x && workspace && grad_w && splits >= 1,
                "avr_linear_wgrad: bad args");
    AVR_REQUIRE(M % 8 == 0 && K % 8 == 0, "avr_linear_wgrad: M and K must be multiples of 8");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(grad_y) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(x) % 16 == 0,
                "avr_linear_wgrad: operands must be 16-byte aligned");
    int64_t rows = (N + splits - 1) / splits;
    rows = (rows + kSlab - 1) / kSlab * kSlab;
    const int used = (int)((N + rows - 1) / rows);
    hipStream_t st = as_stream(stream);
    const int tiles = ((K + kTile - 1) / kTile) * ((M + kTile - 1) / kTile);
    // all tiles of a split on one XCD (its rows re-read from that L2): block
    // b runs on XCD b % 8, split = b % 8 + 8 * (b / 8 / tiles)
    const int64_t blocks = (int64_t)tiles * ((used + 7) / 8 * 8);
    hipLaunchKernelGGL(linear_wgrad_dma_kernel, dim3((unsigned)blocks), dim3(256), 0, st, N, (int)M, (int)K, rows,
                       used, (const __hip_bfloat16*)grad_y, (const __hip_bfloat16*)x, workspace);
    if (int e = check_launch("avr_linear_wgrad")) return e;
    const int64_t MK = (int64_t)M * K;
    int G = 1;
    while (G < 64 && 2 * G <= used && (MK / 4) * G < 131072) G *= 2;
    const int64_t quads_per_block = 256 / G;
    hipLaunchKernelGGL(wgrad_finalize_kernel, dim3((unsigned)((MK / 4 + quads_per_block - 1) / quads_per_block)),
                       dim3(256), 0, st, MK, used, G, workspace, grad_w);
    return check_launch("avr_linear_wgrad_finalize");
}

namespace {
int out1_check(int64_t N, int32_t K, int32_t dtype, const char* who) {
    if (!(N >= 1 && K >= 8 && K <= 512 && (K & (K - 1)) == 0))
        return fail(AVR_E_ARG, std::string(who) + ": N >= 1 and K a power of two in [8, 512]");
    if (!(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16))
        return fail(AVR_E_ARG, std::string(who) + ": fp16 or bf16 operands");
    return 0;
}
}  // namespace

extern "C" int avr_linear_out1_fwd(int64_t N, int32_t K, const void* x, const void* w, int32_t dtype, void* y,
                                   void* stream) {
    if (int e = out1_check(N, K, dtype, "avr_linear_out1_fwd")) return e;
    AVR_REQUIRE(x && w && y && reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0,
                "avr_linear_out1_fwd: x and w must be non-null and 16-byte aligned");
    const int64_t threads = N * (K / 8);
    const dim3 grid((unsigned)((threads + 255) / 256));
    hipStream_t st = as_stream(stream);
    if (dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(linear_out1_fwd_kernel<__half>, grid, dim3(256), 0, st, N, (int)K, (const __half*)x,
                           (const __half*)w, (__half*)y);
    else
        hipLaunchKernelGGL(linear_out1_fwd_kernel<__hip_bfloat16>, grid, dim3(256), 0, st, N, (int)K,
                           (const __hip_bfloat16*)x, (const __hip_bfloat16*)w, (__hip_bfloat16*)y);
    return check_launch("avr_linear_out1_fwd");
}

extern "C" int avr_linear_out1_workspace(int32_t K, int64_t* floats) {
    AVR_REQUIRE(floats && K >= 8, "avr_linear_out1_workspace: bad args");
    *floats = (int64_t)kOut1Blocks * K;
    return 0;
}

extern "C" int avr_linear_out1_bwd(int64_t N, int32_t K, const void* x, const void* w, const void* grad_y,
                                   int32_t dtype, void* grad_x, float* workspace, float* grad_w, void* stream) {
    if (int e = out1_check(N, K, dtype, "avr_linear_out1_bwd")) return e;
    AVR_REQUIRE(x && w && grad_y && grad_x && workspace && grad_w && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(w) % 16 == 0 && reinterpret_cast<uintptr_t>(grad_x) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(workspace) % 16 == 0 && reinterpret_cast<uintptr_t>(grad_w) % 16 == 0,
                "avr_linear_out1_bwd: operands must be non-null and 16-byte aligned");
    const int64_t rows = (N + kOut1Blocks - 1) / kOut1Blocks;
    const int used = (int)((N + rows - 1) / rows);
    hipStream_t st = as_stream(stream);
    if (dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(linear_out1_bwd_kernel<__half>, dim3(used), dim3(256), 0, st, N, (int)K, rows,
                           (const __half*)x, (const __half*)w, (const __half*)grad_y, (__half*)grad_x, workspace);
    else
        hipLaunchKernelGGL(linear_out1_bwd_kernel<__hip_bfloat16>, dim3(used), dim3(256), 0, st, N, (int)K, rows,
                           (const __hip_bfloat16*)x, (const __hip_bfloat16*)w, (const __hip_bfloat16*)grad_y,
                           (__hip_bfloat16*)grad_x, workspace);
    if (int e = check_launch("avr_linear_out1_bwd")) return e;
    int G = 1;
    while (G < 64 && 2 * G <= used && (K / 4) * G < 131072) G *= 2;
    const int64_t quads_per_block = 256 / G;
    hipLaunchKernelGGL(wgrad_finalize_kernel, dim3((unsigned)((K / 4 + quads_per_block - 1) / quads_per_block)),
                       dim3(256), 0, st, (int64_t)K, used, G, workspace, grad_w);
    return check_launch("avr_linear_out1_finalize");
}

extern "C" int avr_narrow_mm(int64_t N, int32_t R, int32_t C, const void* X, const void* Bt, int32_t dtype,
                             int32_t act, const void* mask, void* Y, void* stream) {
    AVR_REQUIRE(N >= 1 && (R == 80 || R == 128 || R == 256) && C >= 65 && C <= 256 && C % 4 == 0 &&
                    (R < 256 || C <= 128),
                "avr_narrow_mm: R in {80, 128, 256}, C a multiple of 4 in [68, 256] (<= 128 for R = 256)");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_narrow_mm: fp16 or bf16 operands");
    AVR_REQUIRE(act >= 0 && act <= 2 && (act != 2 || mask), "avr_narrow_mm: act 0 (none), 1 (ReLU), 2 (mask)");
    AVR_REQUIRE(X && Bt && Y && reinterpret_cast<uintptr_t>(X) % 16 == 0 && reinterpret_cast<uintptr_t>(Bt) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(Y) % 8 == 0 && (!mask || reinterpret_cast<uintptr_t>(mask) % 8 == 0),
                "avr_narrow_mm: X, Bt 16-byte and Y, mask 8-byte aligned");
    const int nct = (C + 31) / 32;
    const int64_t ntiles = (N + kNarrowRows - 1) / kNarrowRows;
    const int cus = device_cus();
    const int64_t grid = std::min<int64_t>(ntiles, 2 * (int64_t)cus);
    hipStream_t st = as_stream(stream);
    // the staged form where Bt and the X tile fit two workgroups per CU
    const size_t bt_lds = (size_t)(nct == 3 ? 3 : nct == 4 ? 4 : 8) * 32 * (R / 8 + 1) * 16;
    const size_t x_lds = (size_t)kNarrowRows * (R / 8 + 1) * 16;
    const bool stage = AVR_NARROW_STAGE && bt_lds + x_lds <= 80 * 1024;
    auto go = [&](auto e_tag, auto n_tag, auto a_tag) {
        using E = decltype(e_tag);
        constexpr int kN = decltype(n_tag)::value, kA = decltype(a_tag)::value;
        // (R = 256 only with C <= 128: the 8-tile form would not fit 256 registers)
        constexpr int kN16 = kN == 8 ? 8 : 16;
        auto pick = [&](auto st_tag) {
            constexpr bool kS = decltype(st_tag)::value;
            return R == 80 ? narrow_mm_kernel<E, kN, 5, kA, kS>
                           : (R == 128 ? narrow_mm_kernel<E, kN, 8, kA, kS> : narrow_mm_kernel<E, kN, kN16, kA, kS>);
        };
        auto kern = stage ? pick(std::true_type{}) : pick(std::false_type{});
        const size_t lds = bt_lds + (stage ? x_lds : 0);
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, st, N, (int)R, (int)C, (const E*)X,
                           (const E*)Bt, (const E*)mask, (E*)Y);
    };
    auto by_act = [&](auto e_tag, auto n_tag) {
        if (act == 0) go(e_tag, n_tag, std::integral_constant<int, 0>{});
        else if (act == 1) go(e_tag, n_tag, std::integral_constant<int, 1>{});
        else go(e_tag, n_tag, std::integral_constant<int, 2>{});
    };
    auto by_n = [&](auto e_tag) {
        if (nct == 3) by_act(e_tag, std::integral_constant<int, 3>{});
        else if (nct == 4) by_act(e_tag, std::integral_constant<int, 4>{});
        else by_act(e_tag, std::integral_constant<int, 8>{});
    };
    if (dtype == AVR_DTYPE_F16)
        by_n(__half{});
    else
        by_n(__hip_bfloat16{});
    return check_launch("avr_narrow_mm");
}
