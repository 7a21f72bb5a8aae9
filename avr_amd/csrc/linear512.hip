// A width-512 hidden layer of the signal network at inference (model.py:
// 176-180: tcnn CutlassMLP, ReLU, no bias), y = relu(x W^T) for x [M][512],
// W [512][512], y [M][512], 16-bit operands, fp32 accumulation, one rounding
// of the output (the unfused layer's arithmetic; the sum order is this
// kernel's own).
//
// An output-tiled GEMM shaped for two waves per SIMD: a workgroup (8 waves)
// owns a 256-row x 256-column output tile (one of the two column halves),
// each wave 128 rows x 64 columns = 8 accumulators of v_mfma_f32_32x32x16
// (128 registers).  The product is formed transposed, C^T = W x^T (A = W
// fragment, B = x fragment), so a lane ends with one row's columns.
//
// K = 512 runs in 8 chunks of 64.  A chunk (x: 256 rows x 128 B, W: the
// half's 256 rows x 128 B; 64 KiB) lands by LDS-DMA (global_load_lds_dwordx4)
// in one of two LDS slots while the other is computed.  x arrives row-major,
// 8 rows x 128 B per DMA instruction (whole lines), its 16-byte pieces
// XOR-swizzled by row (lswz) so the fragment reads are conflict-free; W is
// pre-packed in fragment order (avr_linear512_pack_w), 1 KiB per
// instruction.  One barrier per chunk.  Per k-step a wave reads 6 fragments
// (2 W, 4 x) for 8 MFMAs.
//
// Persistent workgroups take tiles t = blockIdx.x + G k; tile t covers row
// tile (t / 16) * 8 + t % 8 and column half (t / 8) % 2, so the two halves
// of a row tile run at the same time on one XCD (blocks b and b + 8) and the
// second reads x from that XCD's L2.  The chunk stream runs on across tiles
// (the next tile's first chunks are in flight during the last ones), and a
// tile's output leaves after those DMAs are issued, through a per-wave 4 KiB
// LDS transpose as whole 128-byte lines: the stores are then younger than
// the DMAs the next chunks wait for, so no wait covers them.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kLK = 512;                  // K = N = 512
constexpr int kLKC = 64;                  // k per chunk
constexpr int kLChunks = kLK / kLKC;
constexpr int kLSlots = 2;                // two 64 KiB slots: one chunk in flight
constexpr int kLAhead = kLSlots - 1;      // chunks in flight
constexpr int kLKS = kLKC / 16;           // k-steps per chunk
constexpr int kLPieces = kLKC / 8;        // 16-byte pieces of a row's chunk
constexpr int kLRowsPerOp = 64 / kLPieces;  // x rows per DMA instruction
constexpr int kLTileRows = 256, kLTileCols = 256;
constexpr int kLXBytes = kLTileRows * kLKC * 2;   // x rows of the chunk
constexpr int kLSlot = 2 * kLXBytes;              // + the W fragments (same size)
constexpr int kLStage = 4096;                     // per-wave transpose area
constexpr int kLLds = kLSlots * kLSlot + 8 * kLStage;  // 160 KiB
constexpr int kLOpsPerChunk = 2 * kLXBytes / 1024 / 8;  // DMA instructions per wave and chunk
static_assert(kLKC == 32 || kLKC == 64, "chunk");

// slot of piece p of row r (XOR swizzle: conflict-free fragment reads)
__host__ __device__ constexpr int lswz(int r, int p) {
    return kLPieces == 8 ? p ^ ((r >> 1) & 7) : p ^ ((r >> 2) & 3);
}

template <typename E>
__device__ __forceinline__ f32x16 mma(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

// lane i's 16 bytes at g land at LDS byte lds + 16 i (issued as inline asm:
// the compiler neither counts it nor treats it as an LDS write; completion is
// waited for with explicit, counted vmcnt before the chunk's barrier)
__device__ __forceinline__ void ldma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g) : "memory", "m0");
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// s_waitcnt vmcnt(n) (gfx9 encoding) for the few counts the chunk loop uses
#define AVR_L512_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
__device__ __forceinline__ void wait_vm_l(int n) {
    switch (n) {
        case 0: AVR_L512_VMCNT(0); break;
        case 4: AVR_L512_VMCNT(4); break;
        case 8: AVR_L512_VMCNT(8); break;
        case 16: AVR_L512_VMCNT(16); break;
        case 20: AVR_L512_VMCNT(20); break;
        case 24: AVR_L512_VMCNT(24); break;
        case 32: AVR_L512_VMCNT(32); break;
        default: AVR_L512_VMCNT(0); break;  // (longer than needed, never shorter)
    }
}

// rectified (IEEE maximum: NaN kept), rounded in pairs to E
template <typename E>
__device__ __forceinline__ uint32_t relu_pack(float a, float b) {
    return pack16<E>(__builtin_elementwise_maximum(a, 0.0f), __builtin_elementwise_maximum(b, 0.0f));
}

// v's 16-bit halves where m's are not <= 0 (threshold_backward's test,
// `m <= 0 ? 0 : v`: +0, -0 and the negatives down to -inf zero it; positives,
// +inf and every NaN keep v)
template <typename E>
__device__ __forceinline__ uint32_t keep_where_positive(uint32_t v, uint32_t m) {
    constexpr uint32_t kInf = std::is_same<E, __half>::value ? 0x7c00u : 0x7f80u;
    const uint32_t lo = m & 0xffffu, hi = m >> 16;
    const bool zlo = lo == 0u || lo - 0x8000u <= kInf, zhi = hi == 0u || hi - 0x8000u <= kInf;
    return (zlo ? 0u : (v & 0xffffu)) | (zhi ? 0u : (v & 0xffff0000u));
}

// kMask = false: y = relu(x W^T).  kMask = true: y = (x W^T) where
// mask > 0, else 0 (mask [M][512] of E, y's shape): a ReLU layer's data
// gradient with the input ReLU's backward fused, gx = (g W) . [x > 0], with
// Wf packed from W^T (avr_linear512_pack_w with transpose = 1)
template <typename E, bool kMask>
__global__ __launch_bounds__(512, 1) void linear512_relu_kernel(int64_t M, const E* __restrict__ x,
                                                                const frag8* __restrict__ Wf, E* __restrict__ y,
                                                                int ntiles, int nrt, const E* __restrict__ mask) {
    extern __shared__ __attribute__((aligned(16))) char lds_l[];
    const int lane = threadIdx.x & 63, half = lane >> 5, j = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wc = wave & 3;  // rows 128 wr.., columns 64 wc.. of the tile
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds_l;
    char* stage = lds_l + kLSlots * kLSlot + wave * kLStage;

    auto tile_rc = [&](int t, int& rt, int& nh) {
        rt = (t / 16) * 8 + (t % 8);
        nh = (t / 8) % 2;
    };
    // the workgroup's tiles in order (the mapping pads to groups of 8 row
    // tiles: skip the padding)
    auto next_tile = [&](int t) {
        while (t < ntiles) {
            int rt, nh;
            tile_rc(t, rt, nh);
            if (rt < nrt) break;
            t += gridDim.x;
        }
        return t;
    };
    // chunk c of tile t into slot: this wave's share of the W fragments
    // (contiguous in Wf) and of the x instructions (kLRowsPerOp rows of the
    // chunk's row segment each; lane l: row kLRowsPerOp q + l / kLPieces,
    // the piece that lands in slot l % kLPieces, lswz)
    auto issue_chunk = [&](int t, int c, int slot) {
        int rt, nh;
        tile_rc(t, rt, nh);
        const uint32_t base = lds0 + slot * kLSlot;
        constexpr int kW = kLXBytes / 1024 / 8;  // per wave
        const char* wsrc = reinterpret_cast<const char*>(Wf) +
                           ((int64_t)(nh * kLChunks + c) * (kLXBytes / 1024)) * 1024 + 16 * lane;
#pragma unroll
        for (int i = 0; i < kW; ++i) {
            const int p = kW * wave + i;
            ldma16(wsrc + p * 1024, base + kLXBytes + p * 1024);
        }
#pragma unroll
        for (int i = 0; i < kW; ++i) {
            const int q = kW * wave + i;
            const int r = kLRowsPerOp * q + lane / kLPieces;
            const int piece = lswz(r, lane % kLPieces);
            const int64_t row = std::min<int64_t>((int64_t)rt * kLTileRows + r, M - 1);
            ldma16(x + row * kLK + kLKC * c + 8 * piece, base + q * 1024);
        }
    };

    int t = next_tile(blockIdx.x);
    if (t >= ntiles) return;
    // prologue: the first kLAhead chunks of the first tile
    for (int a = 0; a < kLAhead; ++a) issue_chunk(t, a, a);
    wait_vm_l((kLAhead - 1) * kLOpsPerChunk);  // chunk 0 landed
    lds_barrier();
    int g = 0;  // chunks computed so far (the slot of chunk g is g % kLSlots)
    while (t < ntiles) {
        int rt, nh;
        tile_rc(t, rt, nh);
        const int tn = next_tile(t + gridDim.x);
        f32x16 acc[2][4];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[a][q] = f32x16{};
        for (int c = 0; c < kLChunks; ++c, ++g) {
            const int slot = g % kLSlots;
            // chunk c + kLAhead (of this tile or the next) into the slot chunk
            // c - 1 left: every wave passed the barrier that ended it
            const int ca = c + kLAhead;
            const bool issued = ca < kLChunks || tn < ntiles;
            if (ca < kLChunks) issue_chunk(t, ca, (g + kLAhead) % kLSlots);
            else if (tn < ntiles) issue_chunk(tn, ca - kLChunks, (g + kLAhead) % kLSlots);
            const char* sb = lds_l + slot * kLSlot;
            auto read_frags = [&](int s, frag8 (&wfr)[2], frag8 (&xfr)[4]) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    wfr[a] = *reinterpret_cast<const frag8*>(sb + kLXBytes + (8 * s + 2 * wc + a) * 1024 + 16 * lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = 32 * (4 * wr + q) + j, pc = 2 * s + half;
                    xfr[q] = *reinterpret_cast<const frag8*>(sb + r * (2 * kLKC) + lswz(r, pc) * 16);
                }
            };
            // k-step s + 1's fragments read during k-step s's MFMAs, in a
            // ring of three: the reads of k-step s + 1 go into the registers
            // of k-step s - 2, whose MFMAs issued a whole k-step earlier (the
            // program order fixed by sched_barrier; the fragments of k-steps
            // s - 1 and s used once more at the end of k-step s), so no read
            // lands on a B register an MFMA may still wait to read (common.h)
            frag8 wfr[3][2], xfr[3][4];
            read_frags(0, wfr[0], xfr[0]);
#pragma unroll
            for (int s = 0; s < kLKS; ++s) {
                const int b = s % 3;
                if (s + 1 < kLKS) read_frags(s + 1, wfr[(s + 1) % 3], xfr[(s + 1) % 3]);
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[a][q] = mma<E>(wfr[b][a], xfr[b][q], acc[a][q]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    keep_live(xfr[b][q]);
                    if (s >= 1) keep_live(xfr[(s + 2) % 3][q]);
                }
            }
            mfma_queue_wait();
#pragma unroll
            for (int q = 0; q < 4; ++q) keep_live(xfr[(kLKS - 1) % 3][q]);
            // (scheduling fences: hipcc would otherwise sink the chunk's MFMAs
            // below the wait and the barrier)
            __builtin_amdgcn_sched_barrier(0);
            // chunk g + 1 landed: younger are the chunks issued after it
            // (kLAhead - 1 of them while the stream runs; none at its end)
            wait_vm_l(issued ? (kLAhead - 1) * kLOpsPerChunk : 0);
            lds_barrier();
            __builtin_amdgcn_sched_barrier(0);
        }

        // epilogue: 32 rows x 64 columns per pass through the wave's 4 KiB
        // (16-byte chunks XOR-swizzled by row), stored as 8 rows x 128 B
        const int64_t r0 = (int64_t)rt * kLTileRows + 128 * wr;
        const int64_t nrows = std::max<int64_t>(0, std::min<int64_t>(128, M - r0));
        const __amdgpu_buffer_rsrc_t yres = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(y + r0 * kLK), (short)0, (int)(nrows * kLK * 2), 0x00020000);
        __amdgpu_buffer_rsrc_t mres;
        if constexpr (kMask)
            mres = __builtin_amdgcn_make_buffer_rsrc((void*)(mask + r0 * kLK), (short)0, (int)(nrows * kLK * 2),
                                                     0x00020000);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            frag8 mk[4];
            if constexpr (kMask) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int row = 8 * u + (lane >> 3), ch = lane & 7;
                    mk[u] = __builtin_amdgcn_raw_buffer_load_b128(
                        mres, ((32 * q + row) * kLK + kLTileCols * nh + 64 * wc + 8 * ch) * 2, 0, 0);
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a) {
#pragma unroll
                for (int gg = 0; gg < 4; ++gg) {
                    const f32x16& v = acc[a][q];
                    uint32_t w0, w1;
                    if constexpr (kMask) {
                        w0 = pack16<E>(v[4 * gg], v[4 * gg + 1]);
                        w1 = pack16<E>(v[4 * gg + 2], v[4 * gg + 3]);
                    } else {
                        w0 = relu_pack<E>(v[4 * gg], v[4 * gg + 1]);
                        w1 = relu_pack<E>(v[4 * gg + 2], v[4 * gg + 3]);
                    }
                    const int ch = (4 * a + gg) ^ (j & 7);
                    *reinterpret_cast<u32x2*>(stage + j * 128 + ch * 16 + 8 * half) = u32x2{w0, w1};
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int row = 8 * u + (lane >> 3), ch = lane & 7;
                frag8 v = *reinterpret_cast<const frag8*>(stage + row * 128 + ((ch ^ (row & 7)) * 16));
                if constexpr (kMask) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = keep_where_positive<E>(v[e], mk[u][e]);
                }
                __builtin_amdgcn_raw_buffer_store_b128(
                        v, yres, ((32 * q + row) * kLK + kLTileCols * nh + 64 * wc + 8 * ch) * 2, 0, 0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        t = tn;
    }
}

// W [512][512] -> Wf: for column half nh, chunk c (kLKC k), k-step s and
// 32-column tile ct, the 64 lanes' A fragments of v_mfma_f32_32x32x16 (lane
// (j, half): W[256 nh + 32 ct + j][kLKC c + 16 s + 8 half + 0..7]) contiguous
__global__ __launch_bounds__(256) void linear512_pack_kernel(const uint16_t* __restrict__ W, frag8* __restrict__ Wf,
                                                             int64_t n, int transpose) {
    for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int lane = (int)(i & 63);
        const int64_t f = i >> 6;  // fragment index ((nh * kLChunks + c) * kLKS + s) * 8 + ct
        const int ct = (int)(f & 7), s = (int)((f >> 3) % kLKS), c = (int)((f >> 3) / kLKS % kLChunks),
                  nh = (int)(f >> 8);
        const int row = 256 * nh + 32 * ct + (lane & 31), k = kLKC * c + 16 * s + 8 * (lane >> 5);
        if (transpose) {  // fragments of W^T: W[k + 0..7][row], gathered
            uint16_t h[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = W[(int64_t)(k + e) * kLK + row];
            Wf[i] = frag8{h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16, h[4] | (uint32_t)h[5] << 16,
                          h[6] | (uint32_t)h[7] << 16};
        } else {
            Wf[i] = *reinterpret_cast<const frag8*>(W + (int64_t)row * kLK + k);
        }
    }
}

}  // namespace

#ifdef AVR_SHAPE_PROBES
extern "C" int avr_linear512_pack_w(const void* W, int32_t dtype, void* Wf, void* stream) {
    return avr_linear512_pack_w2(W, dtype, 0, Wf, stream);
}
#endif

extern "C" int avr_linear512_pack_w2(const void* W, int32_t dtype, int32_t transpose, void* Wf, void* stream) {
    AVR_REQUIRE(W && Wf && (transpose == 0 || transpose == 1), "avr_linear512_pack_w: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_linear512_pack_w: fp16 or bf16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(W) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_linear512_pack_w: W and Wf must be 16-byte aligned");
    const int64_t n = (int64_t)kLK * kLK / 8;  // 16-byte fragments rows
    hipLaunchKernelGGL(linear512_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (const uint16_t*)W, (frag8*)Wf, n, (int)transpose);
    return check_launch("avr_linear512_pack_w");
}

namespace {
int linear512_launch(int64_t M, const void* x, const void* Wf, int32_t dtype, const void* mask, void* y,
                     void* stream) {
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_linear512_relu_fwd: fp16 or bf16 operands");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(y) % 16 == 0,
                "avr_linear512_relu_fwd: x, Wf and y must be 16-byte aligned");
    const int64_t nrt = (M + kLTileRows - 1) / kLTileRows;
    // tiles enumerated in groups of 8 row tiles x 2 halves (the XCD pairing)
    const int64_t ntiles = 16 * ((nrt + 7) / 8);
    AVR_REQUIRE(ntiles < (1ll << 31) && M * kLK * 2 < (1ll << 47), "avr_linear512_relu_fwd: too many rows");
    AVR_REQUIRE(128 * kLK * 2 < (1ll << 31), "avr_linear512_relu_fwd: tile too large");
    const int cus = device_cus();
    // persistent: one workgroup per CU (160 KiB of LDS), a multiple of 16 so
    // that block b's tiles and block b + 8's are a row tile's two halves
    const int64_t g = std::min<int64_t>(ntiles, std::max(16, cus / 16 * 16));
    hipStream_t st = as_stream(stream);
    auto go = [&](auto e_tag, auto m_tag) {
        using E = decltype(e_tag);
        auto kern = linear512_relu_kernel<E, decltype(m_tag)::value>;
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kLLds);
        hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(512), kLLds, st, M, (const E*)x, (const frag8*)Wf, (E*)y,
                           (int)ntiles, (int)nrt, (const E*)mask);
    };
#ifdef AVR_SHAPE_PROBES
    if (!mask) {
        if (dtype == AVR_DTYPE_F16)
            go(__half{}, std::false_type{});
        else
            go(__hip_bfloat16{}, std::false_type{});
        return check_launch("avr_linear512_relu_fwd");
    }
#endif
    AVR_REQUIRE(mask != nullptr, "avr_linear512: mask required");
    if (dtype == AVR_DTYPE_F16)
        go(__half{}, std::true_type{});
    else
        go(__hip_bfloat16{}, std::true_type{});
    return check_launch("avr_linear512_mask_fwd");
}
}  // namespace

#ifdef AVR_SHAPE_PROBES
// the inference layer relu(x W^T) (not faster than hipBLASLt's tuned
// solution): shapes build only (tools/bench_linear512.py)
extern "C" int avr_linear512_relu_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, void* y,
                                      void* stream) {
    return linear512_launch(M, x, Wf, dtype, nullptr, y, stream);
}
#endif

extern "C" int avr_linear512_mask_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, const void* mask,
                                      void* y, void* stream) {
    AVR_REQUIRE(mask && reinterpret_cast<uintptr_t>(mask) % 16 == 0,
                "avr_linear512_mask_fwd: mask must be non-null and 16-byte aligned");
    return linear512_launch(M, x, Wf, dtype, mask, y, stream);
}
