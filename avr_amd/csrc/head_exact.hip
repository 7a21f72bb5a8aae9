// Fused signal head, output-rounding-exact form.
//
// The reference's signal network returns x = h W^T from a 16-bit network
// (tcnn's fp16, model.py:21-31, 176-180): the render sees every element of x
// ROUNDED to 16 bits (renderer_cpu.py:73,80,90 upcast it with .float()).  The
// linear-algebra head of head.hip sums exact products and never forms x, so
// it cannot reproduce that rounding.  This kernel forms x tile by tile on the
// matrix cores, rounds each element to the MLP's 16-bit type exactly as the
// unfused layer's output does (fp32 accumulation, one round to nearest even),
// and reduces it over rays on the spot:
//
//   z[b,s,t] = sum_{p < cnt[b,s,t]} ws[b,s,p] * round16( sum_k h[b,perm_p,s,k] W[t,k] )
//
// with the column's live rays sorted by delay (avr_head_sort: perm, ws and
// cnt[t] = number of rays with delay <= t), so the masked part of the
// [rays x t] plane is a staircase: a 32-ray x 32-t tile whose first ray
// starts after cnt at the tile's last t is skipped whole.  x never reaches
// HBM; h is read once from HBM (the t-blocks of a column run on one XCD and
// share its rows through that XCD's L2).
//
// Work: one workgroup per (column b*S+s, block of 32*WAVES t).  Wave w owns
// the 32 t of tile w: its W rows are the MFMA B operand, held in registers
// for the whole launch (K/16 fragments of 8 16-bit values).  The A operand,
// 32 sorted rays x K features, is staged per ray tile in LDS (double
// buffered, row stride K*2+16 bytes: ds_read_b128 of 32 rows conflict-free),
// loaded whole-row by all waves one tile ahead.  v_mfma_f32_32x32x16_{f16,bf16}
// over K, then the epilogue rounds, masks (p < cnt[t]), weights and sums the
// tile's rows into a per-lane register in a fixed order (sorted position
// order; the two lane halves added last), so results are deterministic.
// Every (b, s, t) is written by exactly one lane: the output is ONE slab
// [B][S][T] (n_split = 1 for avr_dft_phase_fwd), zero at t >= T-1-shift_s.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));  // 8 packed 16-bit values

template <typename E>
__device__ __forceinline__ f32x16 mfma16(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

// x rounded to the 16-bit type E (round to nearest even) and back: the value
// the unfused layer's 16-bit output holds
template <typename E>
__device__ __forceinline__ float round16(float x) {
    if constexpr (std::is_same<E, __half>::value)
        return __half2float(__float2half(x));
    else
        return __bfloat162float(__float2bfloat16(x));
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: global loads stay in flight
    __builtin_amdgcn_s_barrier();
}

constexpr int kTileRays = 32;

// LDS row stride of the A tile in bytes: K 16-bit values + 16 bytes, so 32
// rows read at one column offset fall on distinct bank quads
__host__ __device__ constexpr int a_row_bytes(int KS) { return KS * 32 + 16; }

template <int KS, int WAVES>
__host__ __device__ constexpr size_t exact_lds_bytes(int R) {
    return 2 * (size_t)kTileRays * a_row_bytes(KS) + 8 * (size_t)((R + kTileRays - 1) / kTileRays * kTileRays);
}

template <typename E, int KS, int WAVES, int DBG = 0>
__global__ __launch_bounds__(64 * WAVES) void head_exact_fwd_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const E* __restrict__ W,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ z, int ntb, int per_xcd) {
    constexpr int NT = 64 * WAVES;
    constexpr int TB = 32 * WAVES;  // t per workgroup
    constexpr int ROWB = a_row_bytes(KS);
    constexpr int CPT = (kTileRays * KS * 2 + NT - 1) / NT;  // 16-byte chunks per thread and tile
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    char* abuf = lds_x;                                                      // [2][32][ROWB]
    int* pl = reinterpret_cast<int*>(lds_x + 2 * kTileRays * ROWB);          // perm of the column [R]
    // ws of the column after the padded perm, 16-byte aligned (read as float4)
    float* wl = reinterpret_cast<float*>(pl + (R + kTileRays - 1) / kTileRays * kTileRays);

    const int T = pp.T, S = pp.n_samples;
    // XCD-aware order: the t-blocks of one column are consecutive on one XCD
    // (workgroup g runs on XCD g % 8), so they share the column's h rows in L2
    const int64_t total = (int64_t)B * S * ntb;
    const int64_t L = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (L >= total) return;
    const int64_t col = L / ntb;
    const int tb = (int)(L % ntb);
    const int s = (int)(col % S), b = (int)(col / S);
    const int lim = tail_limit(pp, s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int half = lane >> 5, j = lane & 31;
    const int t0 = tb * TB + wave * 32;
    const int t = t0 + j;
    float* zcol = z + col * T;
    const int tlast = min(tb * TB + TB, lim) - 1;  // last live t of the block
    if (tlast < tb * TB) {  // the block lies past the tail window
        for (int i = threadIdx.x; i < TB; i += NT)
            if (tb * TB + i < T) zcol[tb * TB + i] = 0.0f;
        return;
    }
    const int* ccol = cnt + col * T;
    const int nblk = ccol[tlast];  // rays live anywhere in the block (cnt is nondecreasing)
    const int cnt_t = (t < lim) ? ccol[t] : 0;
    const int cwave = (t0 < lim) ? ccol[min(t0 + 31, lim - 1)] : 0;  // rays live in this wave's tile

    // B operand: W rows t0..t0+31, k = 16 ks + 8 half + 0..7 (registers for
    // the launch); k-steps past K are zero (loads clamped, then selected)
    frag8 wf[KS];
    const int ks_n = K / 16;
    {
        const E* wrow = W + (int64_t)min(t, T - 1) * K + 8 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const frag8*>(wrow + 16 * min(ks, ks_n - 1));
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            if (ks >= ks_n) wf[ks] = frag8{0u, 0u, 0u, 0u};
    }
    // the column's sorted rays and weights for the block's tiles; positions
    // past nblk repeat a live ray (its rows are masked) with weight 0
    const int ntile = (nblk + kTileRays - 1) / kTileRays;
    for (int p = threadIdx.x; p < ntile * kTileRays; p += NT) {
        const bool in = p < nblk;
        pl[p] = perm[col * R + (in ? p : nblk - 1)];
        wl[p] = in ? ws[col * R + p] : 0.0f;
    }
    // this thread's chunks of a tile: row and 16-byte column, fixed over the
    // tiles (chunks past 32 rows wrap: duplicates of the same values)
    const int cpr = K / 8;
    int crow[CPT], hoff[CPT], aoff[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int ch = (threadIdx.x + NT * c) % (kTileRays * cpr);
        crow[c] = ch / cpr;
        const int cc = ch - crow[c] * cpr;
        hoff[c] = 8 * cc;
        aoff[c] = crow[c] * ROWB + 16 * cc;
    }
    __syncthreads();
    const int64_t hstride = (int64_t)S * K;
    const E* hcol = h + ((int64_t)b * R * S + s) * K;

    // A-tile staging: whole h rows, 16 bytes per lane, loaded unconditionally
    // (no exec-masked load whose result would be waited for in its branch),
    // two tiles in flight ahead of the one the MFMAs read from LDS
    auto issue = [&](frag8 (&ld)[CPT], int tile) {
        const int p0 = tile * kTileRays;
        int ray[CPT];
#pragma unroll
        for (int c = 0; c < CPT; ++c) ray[c] = pl[p0 + crow[c]];
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            // DBG & 2: every tile reads the first row (L2-resident): no HBM stream
            const int64_t off = (DBG & 2) ? (int64_t)hoff[c] : (int64_t)ray[c] * hstride + hoff[c];
            ld[c] = *reinterpret_cast<const frag8*>(hcol + off);
        }
    };
    auto commit = [&](const frag8 (&ld)[CPT], int buf) {
        char* a = abuf + buf * kTileRays * ROWB;
#pragma unroll
        for (int c = 0; c < CPT; ++c) *reinterpret_cast<frag8*>(a + aoff[c]) = ld[c];
    };

    float zl = 0.0f;
    auto compute = [&](int it) {
        const int p0 = it * kTileRays;
        if (p0 >= cwave) return;  // wave-uniform: no live (ray, t) pair of this wave in the tile
        const char* a = abuf + (it & 1) * kTileRays * ROWB + j * ROWB + 16 * half;
        f32x16 acc;
        if constexpr (DBG & 1) {  // no MFMA: the epilogue on the A fragment
            const frag8 v = *reinterpret_cast<const frag8*>(a);
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = __uint_as_float(v[i & 3]);
        } else {
            acc = mfma16<E>(*reinterpret_cast<const frag8*>(a), wf[0], f32x16{});
#pragma unroll
            for (int ks = 1; ks < KS; ++ks)
                acc = mfma16<E>(*reinterpret_cast<const frag8*>(a + 32 * ks), wf[ks], acc);
        }
        // register r holds row (r & 3) + 8 (r >> 2) + 4 half of the tile, column t
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
            const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int p = p0 + e + 8 * g + 4 * half;
                const float wsel = (p < cnt_t) ? w4[e] : 0.0f;
                zl = fmaf(wsel, round16<E>(acc[4 * g + e]), zl);
            }
        }
    };

    frag8 ldA[CPT], ldB[CPT];
    // one iteration: `nxt` holds tile it+1 (in flight), `nn` receives tile it+2
    auto body = [&](int it, frag8 (&nxt)[CPT], frag8 (&nn)[CPT]) {
        if (it + 2 < ntile) issue(nn, it + 2);
        compute(it);
        if (it + 1 < ntile) commit(nxt, (it + 1) & 1);  // waits for tile it+1's loads only
        lds_barrier();  // LDS traffic done; the loads of tile it+2 stay in flight
    };
    if (ntile > 0) {
        issue(ldA, 0);
        if (K < 16 * KS) {  // the k-steps past K read zeros (the commits never write there)
            for (int i = threadIdx.x; i < 2 * kTileRays * ROWB / 16; i += NT)
                reinterpret_cast<frag8*>(abuf)[i] = frag8{0u, 0u, 0u, 0u};
            __syncthreads();
        }
        if (ntile > 1) issue(ldB, 1);
        commit(ldA, 0);
        lds_barrier();
    }
    for (int it = 0; it < ntile; it += 2) {
        body(it, ldB, ldA);
        if (it + 1 < ntile) body(it + 1, ldA, ldB);
    }
    const float other = __shfl_xor(zl, 32, 64);
    if (half == 0 && t < T) zcol[t] = (t < lim) ? zl + other : 0.0f;
}

// One wave per SIMD (4 waves, 128 t per workgroup, up to 512 registers per
// lane): the register file holds the wave's W fragments AND all K/16 A
// fragments of the current ray tile, so a tile's MFMAs issue back to back
// (no per-MFMA LDS wait), and the epilogue of the previous tile is placed in
// the same basic block as the current tile's MFMAs, whose issue gaps it
// fills.  After the barrier that publishes tile it+1 its fragments are read
// at once.  Same arithmetic and summation order as head_exact_fwd_kernel.
template <typename E, int KS, int DBG = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void head_exact_pipe_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const E* __restrict__ W,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ z, int ntb, int per_xcd) {
    constexpr int WAVES = 4;
    constexpr int NT = 64 * WAVES;
    constexpr int TB = 32 * WAVES;
    constexpr int ROWB = a_row_bytes(KS);
    constexpr int CPT = (kTileRays * KS * 2 + NT - 1) / NT;
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    char* abuf = lds_x;
    int* pl = reinterpret_cast<int*>(lds_x + 2 * kTileRays * ROWB);
    float* wl = reinterpret_cast<float*>(pl + (R + kTileRays - 1) / kTileRays * kTileRays);

    const int T = pp.T, S = pp.n_samples;
    const int64_t total = (int64_t)B * S * ntb;
    const int64_t L = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (L >= total) return;
    const int64_t col = L / ntb;
    const int tb = (int)(L % ntb);
    const int s = (int)(col % S), b = (int)(col / S);
    const int lim = tail_limit(pp, s);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int half = lane >> 5, j = lane & 31;
    const int t0 = tb * TB + wave * 32;
    const int t = t0 + j;
    float* zcol = z + col * T;
    const int tlast = min(tb * TB + TB, lim) - 1;
    if (tlast < tb * TB) {
        for (int i = threadIdx.x; i < TB; i += NT)
            if (tb * TB + i < T) zcol[tb * TB + i] = 0.0f;
        return;
    }
    const int* ccol = cnt + col * T;
    const int nblk = ccol[tlast];
    const int cnt_t = (t < lim) ? ccol[t] : 0;
    const int cwave = (t0 < lim) ? ccol[min(t0 + 31, lim - 1)] : 0;
    const int ntile = (nblk + kTileRays - 1) / kTileRays;
    const int wtiles = (cwave + kTileRays - 1) / kTileRays;  // tiles 0..wtiles-1 hold this wave's live pairs

    frag8 wf[KS];
    const int ks_n = K / 16;
    {
        const E* wrow = W + (int64_t)min(t, T - 1) * K + 8 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const frag8*>(wrow + 16 * min(ks, ks_n - 1));
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            if (ks >= ks_n) wf[ks] = frag8{0u, 0u, 0u, 0u};
    }
    for (int p = threadIdx.x; p < ntile * kTileRays; p += NT) {
        const bool in = p < nblk;
        pl[p] = perm[col * R + (in ? p : nblk - 1)];
        wl[p] = in ? ws[col * R + p] : 0.0f;
    }
    const int cpr = K / 8;
    int crow[CPT], hoff[CPT], aoff[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int ch = (threadIdx.x + NT * c) % (kTileRays * cpr);
        crow[c] = ch / cpr;
        const int cc = ch - crow[c] * cpr;
        hoff[c] = 8 * cc;
        aoff[c] = crow[c] * ROWB + 16 * cc;
    }
    __syncthreads();
    const int64_t hstride = (int64_t)S * K;
    const E* hcol = h + ((int64_t)b * R * S + s) * K;

    auto issue = [&](frag8 (&ld)[CPT], int tile) {
        const int p0 = tile * kTileRays;
        int ray[CPT];
#pragma unroll
        for (int c = 0; c < CPT; ++c) ray[c] = pl[p0 + crow[c]];
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int64_t off = (DBG & 2) ? (int64_t)hoff[c] : (int64_t)ray[c] * hstride + hoff[c];
            ld[c] = *reinterpret_cast<const frag8*>(hcol + off);
        }
    };
    auto commit = [&](const frag8 (&ld)[CPT], int buf) {
        char* a = abuf + buf * kTileRays * ROWB;
#pragma unroll
        for (int c = 0; c < CPT; ++c) *reinterpret_cast<frag8*>(a + aoff[c]) = ld[c];
    };
    frag8 af[KS];
    auto read_frags = [&](int buf) {
        const char* a = abuf + buf * kTileRays * ROWB + j * ROWB + 16 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) af[ks] = *reinterpret_cast<const frag8*>(a + 32 * ks);
    };
    float zl = 0.0f;
    auto mfma_tile = [&]() {
        f32x16 acc;
        if constexpr (DBG & 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = __uint_as_float(af[i & 7][i & 3]);
        } else {
            acc = mfma16<E>(af[0], wf[0], f32x16{});
#pragma unroll
            for (int ks = 1; ks < KS; ++ks) acc = mfma16<E>(af[ks], wf[ks], acc);
        }
        return acc;
    };
    auto epilogue = [&](const f32x16& acc, int it) {
        const int p0 = it * kTileRays;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
            const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int p = p0 + e + 8 * g + 4 * half;
                const float wsel = (p < cnt_t) ? w4[e] : 0.0f;
                zl = fmaf(wsel, round16<E>(acc[4 * g + e]), zl);
            }
        }
    };

    frag8 ldA[CPT], ldB[CPT];
    f32x16 accA, accB;
    // iteration it: MFMAs of tile it into `cur` while the epilogue of tile
    // it-1 (`prev`) fills their gaps; then tile it+1 is committed, published
    // by the barrier, and its fragments are read
    auto body = [&](int it, frag8 (&nxt)[CPT], frag8 (&nn)[CPT], f32x16& cur, f32x16& prev) {
        if (it + 2 < ntile) issue(nn, it + 2);
        if (it < wtiles) {
            cur = mfma_tile();
            if (it >= 1) epilogue(prev, it - 1);
        } else if (it == wtiles && it >= 1) {
            epilogue(prev, it - 1);
        }
        if (it + 1 < ntile) commit(nxt, (it + 1) & 1);
        lds_barrier();
        if (it + 1 < ntile) read_frags((it + 1) & 1);
    };
    if (ntile > 0) {
        issue(ldA, 0);
        if (K < 16 * KS) {
            for (int i = threadIdx.x; i < 2 * kTileRays * ROWB / 16; i += NT)
                reinterpret_cast<frag8*>(abuf)[i] = frag8{0u, 0u, 0u, 0u};
            __syncthreads();
        }
        if (ntile > 1) issue(ldB, 1);
        commit(ldA, 0);
        lds_barrier();
        read_frags(0);
    }
    int it = 0;
    for (; it + 1 < ntile; it += 2) {
        body(it, ldB, ldA, accA, accB);
        body(it + 1, ldA, ldB, accB, accA);
    }
    if (it < ntile) {
        body(it, ldB, ldA, accA, accB);
        ++it;
        // the last tile's epilogue (if this wave computed it)
        if (it - 1 < wtiles) epilogue(accA, it - 1);
    } else if (it >= 1 && it - 1 < wtiles) {
        epilogue(accB, it - 1);
    }
    const float other = __shfl_xor(zl, 32, 64);
    if (half == 0 && t < T) zcol[t] = (t < lim) ? zl + other : 0.0f;
}

// LDS-DMA form for K = 512 (the reference networks' width), 8 waves, two
// per SIMD: each 1 KiB h row goes from global memory straight into its
// (padded) LDS row with one global_load_lds_dwordx4 (no staging registers),
// three tile buffers so two tiles are in flight behind the one the MFMAs
// read; the freed registers let more A-fragment reads run ahead of the
// MFMA chain.  Tile it+1's rows are complete when this wave's DMA count
// drops to the tile it+2 rows it issued after them (s_waitcnt vmcnt), and
// visible to every wave after the barrier.  Same arithmetic and order as
// head_exact_fwd_kernel.
// One 16-byte-per-lane LDS-DMA load: lane i's 16 bytes at g land at LDS byte
// address lds + 16 i.  Issued as inline asm so the compiler does not treat
// the in-flight DMA as an LDS write every later ds_read must wait for (with
// the builtin it inserts vmcnt(0) inside the MFMA chain, which drains the
// prefetched tiles); completion is waited for explicitly (wait_dma).
__device__ __forceinline__ void dma_row16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// PERSIST: one workgroup per CU for the whole launch instead of one per
// (column, t-block) item: each workgroup keeps one t-block (its W fragments
// are loaded once, not once per item) and walks columns of its XCD's
// contiguous column range with a stride; the t-blocks of a column run on one
// XCD (its h rows shared through that L2).  Removes the per-item W prologue
// and the workgroup turnover of the one-item form.
template <typename E, int TR, int NBUF, int DBG = 0, bool PERSIST = false, int MP = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void head_exact_dma_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const E* __restrict__ W,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ z, int ntb, int per_xcd) {
    constexpr int KS = 32, WAVES = 8, NT = 512, TB = 256;
    constexpr int PD = NBUF - 1;            // tiles in flight behind the one being computed
    constexpr int ROWB = a_row_bytes(KS);   // 1040
    constexpr int RPW = TR / WAVES;         // rows each wave moves per tile
    static_assert(TR % 32 == 0 && RPW * (NBUF - 2) <= 63 && NBUF <= 4, "tile rays / buffers");
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    char* abuf = lds_x;  // [NBUF][TR][ROWB]
    int* pl = reinterpret_cast<int*>(lds_x + NBUF * TR * ROWB);
    float* wl = reinterpret_cast<float*>(pl + (R + TR - 1) / TR * TR);

    const int T = pp.T, S = pp.n_samples;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int64_t ncol = (int64_t)B * S;
    // this workgroup's items: (first column, column stride, column end, t-block)
    int64_t c_first, c_step, c_end;
    int tb;
    if constexpr (PERSIST) {
        // per_xcd = workgroups per XCD (a multiple of ntb); XCD x owns columns
        // [x * cpx, (x + 1) * cpx)
        const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
        const int nq = per_xcd / ntb;
        const int64_t cpx = (ncol + 7) / 8;
        tb = m % ntb;
        c_first = (int64_t)x * cpx + m / ntb;
        c_step = nq;
        c_end = min(ncol, (int64_t)(x + 1) * cpx);
    } else {
        const int64_t total = ncol * ntb;
        const int64_t L = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= total) return;
        c_first = L / ntb;
        c_step = 1;
        c_end = c_first + 1;
        tb = (int)(L % ntb);
    }
    const int t0 = tb * TB + wave * 32;
    const int t = t0 + j;

    frag8 wf[KS];
    {
        const E* wrow = W + (int64_t)min(t, T - 1) * K + 8 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const frag8*>(wrow + 16 * ks);
        // land them here: otherwise the compiler sinks these loads into the
        // tile loop and waits on them there by vmcnt, which also counts the
        // tile DMAs in flight (it does not see the asm-issued ones)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(wf[ks]));
    }
    const int64_t hstride = (int64_t)S * K;

    // a column's metadata (cnt at this wave's t and, for MP > 0, the sorted
    // rays and their weights: R <= 512 * MP), loaded one column ahead into
    // registers: its loads fly under the previous column's tiles.  MP = 0
    // (more rays than the registers allow) loads the rays in the column.
    constexpr int kMP = MP > 0 ? MP : 1;
    struct Meta {
        int nblk, cnt_t, cwave, cfull;
        int pv[kMP];
        float wv[kMP];
    };
    auto fetch = [&](int64_t c, Meta& m) {
        if (c >= c_end) return;
        const int sc = (int)(c % S);
        const int limc = tail_limit(pp, sc);
        const int tl = min(tb * TB + TB, limc) - 1;
        if (tl < tb * TB) {
            m.nblk = -1;  // nothing live in this t-block
            return;
        }
        const int* cc = cnt + c * T;
        m.nblk = cc[tl];
        m.cnt_t = (t < limc) ? cc[t] : 0;
        m.cwave = (t0 < limc) ? cc[min(t0 + 31, limc - 1)] : 0;
        m.cfull = (t0 + 31 < limc) ? cc[t0] : 0;
        if constexpr (MP > 0) {
#pragma unroll
            for (int jj = 0; jj < kMP; ++jj) {
                const int pq = (int)threadIdx.x + NT * jj;
                if (pq < R) {
                    m.pv[jj] = perm[c * R + pq];
                    m.wv[jj] = ws[c * R + pq];
                }
            }
        }
    };
    Meta m;
    fetch(c_first, m);
    for (int64_t col = c_first; col < c_end; col += c_step) {
        if (PERSIST && col != c_first) __syncthreads();  // the previous column's LDS reads are done
        const int s = (int)(col % S), b = (int)(col / S);
        const int lim = tail_limit(pp, s);
        float* zcol = z + col * T;
        if (m.nblk < 0) {
            for (int i = threadIdx.x; i < TB; i += NT)
                if (tb * TB + i < T) zcol[tb * TB + i] = 0.0f;
            fetch(col + c_step, m);
            continue;
        }
        const int nblk = m.nblk, cnt_t = m.cnt_t, cwave = m.cwave;
        // rays live at EVERY t of this wave's tile (cnt is nondecreasing in t):
        // a 32-ray sub-tile below it needs no mask in its epilogue
        const int cfull = __builtin_amdgcn_readfirstlane(m.cfull);
        const int ntile = (nblk + TR - 1) / TR;
        if constexpr (MP > 0) {
#pragma unroll
            for (int jj = 0; jj < kMP; ++jj) {
                const int pq = (int)threadIdx.x + NT * jj;
                if (pq < nblk) {
                    pl[pq] = m.pv[jj];
                    wl[pq] = m.wv[jj];
                }
            }
        } else {
            for (int pq = threadIdx.x; pq < nblk; pq += NT) {
                pl[pq] = perm[col * R + pq];
                wl[pq] = ws[col * R + pq];
            }
        }
        __syncthreads();
        // rows past the live ones: the last live ray again, weight 0
        for (int pq = nblk + (int)threadIdx.x; pq < ntile * TR; pq += NT) {
            pl[pq] = pl[nblk - 1];
            wl[pq] = 0.0f;
        }
        __syncthreads();
        fetch(col + c_step, m);  // the next column's metadata, under this column's tiles
        const E* hcol = h + ((int64_t)b * R * S + s) * K + 8 * lane;

        // rows wave*RPW .. +RPW-1 of tile `tile` into buffer tile % NBUF; the
        // wave's RPW ray indices come from LDS in one vector read
        auto issue = [&](int tile) {
            const int p0 = tile * TR + wave * RPW;
            char* a = abuf + (tile % NBUF) * TR * ROWB + wave * RPW * ROWB;
            int ray[RPW];
#pragma unroll
            for (int r = 0; r < RPW; ++r) ray[r] = pl[p0 + r];
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int rr = __builtin_amdgcn_readfirstlane(ray[r]);
                const int64_t off = (DBG & 2) ? (int64_t)(r & 7) * hstride : (int64_t)rr * hstride;
                dma_row16(hcol + off, (uint32_t)(uintptr_t)(a + r * ROWB));
            }
        };

        float zl = 0.0f;
        constexpr int kDepth = 8;  // A fragments read this many k-steps ahead of their MFMA
        auto epilogue = [&](const f32x16& acc, int p0) {
            if constexpr (DBG & 4) {  // no epilogue: keep the MFMA result alive only
                zl += acc[0];
                return;
            }
            if (p0 + 32 <= cfull) {  // every (ray, t) pair of the sub-tile is live
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
                    zl = fmaf(wv.x, round16<E>(acc[4 * g + 0]), zl);
                    zl = fmaf(wv.y, round16<E>(acc[4 * g + 1]), zl);
                    zl = fmaf(wv.z, round16<E>(acc[4 * g + 2]), zl);
                    zl = fmaf(wv.w, round16<E>(acc[4 * g + 3]), zl);
                }
                return;
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
                const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int p = p0 + e + 8 * g + 4 * half;
                    const float wsel = (p < cnt_t) ? w4[e] : 0.0f;
                    zl = fmaf(wsel, round16<E>(acc[4 * g + e]), zl);
                }
            }
        };
        // NQ consecutive 32-ray sub-tiles starting at row q0 of the tile in
        // buffer `buf`: their MFMA chains back to back (the fragment reads of the
        // next chain run under the previous one's MFMAs), then their epilogues
        // in sub-tile order (the summation order of the other forms)
        auto chains = [&](auto nq_tag, int buf, int q0, int p0) {
            constexpr int NQ = decltype(nq_tag)::value;
            const char* a = abuf + buf * TR * ROWB + (32 * q0 + j) * ROWB + 16 * half;
            f32x16 acc[NQ];
            if constexpr (DBG & 1) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const frag8 v = *reinterpret_cast<const frag8*>(a + q * 32 * ROWB);
#pragma unroll
                    for (int i = 0; i < 16; ++i) acc[q][i] = __uint_as_float(v[i & 3]);
                }
            } else {
                constexpr int N = NQ * KS;  // k-steps of all chains, in order
                auto frag_at = [&](int n) {
                    return *reinterpret_cast<const frag8*>(a + (n / KS) * 32 * ROWB + 32 * (n % KS));
                };
                frag8 fr[kDepth];
#pragma unroll
                for (int i = 0; i < kDepth; ++i) fr[i] = frag_at(i);
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[q] = f32x16{};
#pragma unroll
                for (int n = 0; n < N; ++n) {
                    acc[n / KS] = mfma16<E>(fr[n % kDepth], wf[n % KS], acc[n / KS]);
                    if (n + kDepth < N) fr[n % kDepth] = frag_at(n + kDepth);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, kDepth, 0);  // the first kDepth DS reads
#pragma unroll
                for (int n = 0; n < N; ++n) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                    if (n + kDepth < N) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // then one DS read
                }
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) epilogue(acc[q], p0 + 32 * q);
        };
        auto compute = [&](int it) {
            const int p0 = it * TR, buf = it % NBUF;
            if constexpr (TR == 64) {
                if (p0 + 32 < cwave)
                    chains(std::integral_constant<int, 2>{}, buf, 0, p0);
                else if (p0 < cwave)
                    chains(std::integral_constant<int, 1>{}, buf, 0, p0);
            } else {
                if (p0 < cwave) chains(std::integral_constant<int, 1>{}, buf, 0, p0);
            }
        };
        // s_waitcnt vmcnt(n) (expcnt / lgkmcnt not waited on; gfx9 encoding)
#define AVR_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
        // this wave's DMAs still allowed in flight once the oldest tile landed:
        // the RPW rows of each younger tile issued (n of them)
        auto wait_vm = [](int n) {
            switch (n) {  // the immediate must be a constant
                case 0: AVR_VMCNT(0); break;
                case 1: AVR_VMCNT(RPW); break;
                case 2: AVR_VMCNT(2 * RPW); break;
                default: AVR_VMCNT(0); break;
            }
        };
#undef AVR_VMCNT
        for (int i = 0; i < PD; ++i)
            if (i < ntile) issue(i);
        if (ntile > 0) {
            wait_vm(min(PD, ntile) - 1);  // tile 0 landed (the younger ones may still fly)
            __builtin_amdgcn_s_barrier();
        }
        if constexpr (DBG & 8) {  // no DMA, no barrier: every tile computed from the tile-0 buffer
            for (int it = 0; it < ((DBG & 16) ? 0 : ntile); ++it) {  // DBG & 16: prologue and output only
                const int p0 = it * TR;
                if (p0 < cwave) chains(std::integral_constant<int, 1>{}, 0, 0, p0);
            }
        } else {
            for (int it = 0; it < ntile; ++it) {
                // into the buffer tile it-1 used: every wave left it at the last barrier
                if (it + PD < ntile) issue(it + PD);
                compute(it);
                if (it + 1 < ntile) {
                    wait_vm(min(PD, ntile - 1 - it) - 1);  // tile it+1's rows from this wave have landed
                    __builtin_amdgcn_s_waitcnt(0xC07F);     // and every LDS read of tile it is done
                    __builtin_amdgcn_s_barrier();
                }
            }
        }
        const float other = __shfl_xor(zl, 32, 64);
        if (half == 0 && t < T) zcol[t] = (t < lim) ? zl + other : 0.0f;
    }
}

// Two t-tiles per wave (AVR_HEAD_EXACT_WAVES 20, K = 512): the persistent
// LDS-DMA form with 4 waves of 64 t instead of 8 waves of 32, one wave per
// SIMD.  Each A fragment read from LDS feeds two MFMAs (one per t-tile), so
// the LDS reads per MFMA halve: in the 8-wave form the row stream (127 us
// alone) and the MFMA chains (119 us alone) add up at config 2 (254 us),
// because the chains' fragment reads keep LDS busy while the next tile's
// DMA wants to land.  W fragments of both tiles stay in registers (256).
template <typename E>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void head_exact_w2_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const E* __restrict__ W,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ z, int ntb, int per_xcd) {
    constexpr int KS = 32, WAVES = 4, NT = 256, TB = 256, TR = 64, RPW = TR / WAVES;
    constexpr int ROWB = a_row_bytes(KS);
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    char* abuf = lds_x;  // [2][TR][ROWB]
    int* pl = reinterpret_cast<int*>(lds_x + 2 * TR * ROWB);
    float* wl = reinterpret_cast<float*>(pl + (R + TR - 1) / TR * TR);

    const int T = pp.T, S = pp.n_samples;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int64_t ncol = (int64_t)B * S;
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int nq = per_xcd / ntb;
    const int64_t cpx = (ncol + 7) / 8;
    const int tb = m % ntb;
    const int64_t c_first = (int64_t)x * cpx + m / ntb, c_step = nq;
    const int64_t c_end = min(ncol, (int64_t)(x + 1) * cpx);
    const int t0 = tb * TB + wave * 64;

    frag8 wf[2][KS];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const E* wrow = W + (int64_t)min(t0 + 32 * q + j, T - 1) * K + 8 * half;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[q][ks] = *reinterpret_cast<const frag8*>(wrow + 16 * ks);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(wf[q][ks]));
    const int64_t hstride = (int64_t)S * K;

    for (int64_t col = c_first; col < c_end; col += c_step) {
        __syncthreads();  // the previous column's LDS reads are done
        const int s = (int)(col % S), b = (int)(col / S);
        const int lim = tail_limit(pp, s);
        float* zcol = z + col * T;
        const int tl = min(tb * TB + TB, lim) - 1;
        if (tl < tb * TB) {
            for (int i = threadIdx.x; i < TB; i += NT)
                if (tb * TB + i < T) zcol[tb * TB + i] = 0.0f;
            continue;
        }
        const int* cc = cnt + col * T;
        const int nblk = cc[tl];
        int cnt_t[2], cwq[2], cfull[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int tq0 = t0 + 32 * q, tq = tq0 + j;
            cnt_t[q] = tq < lim ? cc[tq] : 0;
            cwq[q] = __builtin_amdgcn_readfirstlane(tq0 < lim ? cc[min(tq0 + 31, lim - 1)] : 0);
            cfull[q] = __builtin_amdgcn_readfirstlane(tq0 + 31 < lim ? cc[tq0] : 0);
        }
        const int ntile = (nblk + TR - 1) / TR;
        for (int pq = threadIdx.x; pq < nblk; pq += NT) {
            pl[pq] = perm[col * R + pq];
            wl[pq] = ws[col * R + pq];
        }
        __syncthreads();
        for (int pq = nblk + (int)threadIdx.x; pq < ntile * TR; pq += NT) {
            pl[pq] = pl[nblk - 1];
            wl[pq] = 0.0f;
        }
        __syncthreads();
        const E* hcol = h + ((int64_t)b * R * S + s) * K + 8 * lane;
        auto issue = [&](int tile) {
            const int p0 = tile * TR + wave * RPW;
            char* a = abuf + (tile & 1) * TR * ROWB + wave * RPW * ROWB;
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int rr = __builtin_amdgcn_readfirstlane(pl[p0 + r]);
                dma_row16(hcol + (int64_t)rr * hstride, (uint32_t)(uintptr_t)(a + r * ROWB));
            }
        };
        float zl[2] = {0.0f, 0.0f};
        auto epilogue = [&](const f32x16& acc, int q, int p0) {
            if (p0 + 32 <= cfull[q]) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
                    zl[q] = fmaf(wv.x, round16<E>(acc[4 * g + 0]), zl[q]);
                    zl[q] = fmaf(wv.y, round16<E>(acc[4 * g + 1]), zl[q]);
                    zl[q] = fmaf(wv.z, round16<E>(acc[4 * g + 2]), zl[q]);
                    zl[q] = fmaf(wv.w, round16<E>(acc[4 * g + 3]), zl[q]);
                }
                return;
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
                const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int p = p0 + e + 8 * g + 4 * half;
                    zl[q] = fmaf((p < cnt_t[q]) ? w4[e] : 0.0f, round16<E>(acc[4 * g + e]), zl[q]);
                }
            }
        };
        constexpr int kDepth = 4;
        // one 32-ray sub-tile: both t-tiles' chains from the same fragments
        // (NQ = 2), or only the second's when the first needs none of these rays
        auto chain = [&](auto nq_tag, const char* a, int p0) {
            constexpr int NQ = decltype(nq_tag)::value;
            f32x16 acc[2];
            acc[0] = f32x16{};
            acc[1] = f32x16{};
            frag8 fr[kDepth];
#pragma unroll
            for (int i = 0; i < kDepth; ++i) fr[i] = *reinterpret_cast<const frag8*>(a + 32 * i);
#pragma unroll
            for (int n = 0; n < KS; ++n) {
                if constexpr (NQ == 2) acc[0] = mfma16<E>(fr[n % kDepth], wf[0][n], acc[0]);
                acc[1] = mfma16<E>(fr[n % kDepth], wf[1][n], acc[1]);
                if (n + kDepth < KS) fr[n % kDepth] = *reinterpret_cast<const frag8*>(a + 32 * (n + kDepth));
            }
            if constexpr (NQ == 2) epilogue(acc[0], 0, p0);
            epilogue(acc[1], 1, p0);
        };
        issue(0);
#define AVR_W2VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
        AVR_W2VMCNT(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        for (int it = 0; it < ntile; ++it) {
            if (it + 1 < ntile) issue(it + 1);  // into the buffer tile it - 1 used
            const char* a0 = abuf + (it & 1) * TR * ROWB + j * ROWB + 16 * half;
#pragma unroll
            for (int q0 = 0; q0 < TR / 32; ++q0) {
                const int p0 = it * TR + 32 * q0;
                if (p0 < cwq[0])
                    chain(std::integral_constant<int, 2>{}, a0 + q0 * 32 * ROWB, p0);
                else if (p0 < cwq[1])
                    chain(std::integral_constant<int, 1>{}, a0 + q0 * 32 * ROWB, p0);
            }
            if (it + 1 < ntile) {
                AVR_W2VMCNT(0);                       // tile it + 1's rows from this wave have landed
                __builtin_amdgcn_s_waitcnt(0xC07F);  // and every LDS read of tile it is done
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
        }
#undef AVR_W2VMCNT
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const float other = __shfl_xor(zl[q], 32, 64);
            const int tq = t0 + 32 * q + j;
            if (half == 0 && tq < T) zcol[tq] = (tq < lim) ? zl[q] + other : 0.0f;
        }
    }
}

int exact_shape(const avr_render_params& p, int K, int* KS, int* waves) {
    if (K % 16 != 0 || K < 16 || K > 512) return fail(AVR_E_CONFIG, "exact head: K must be a multiple of 16, <= 512");
    const int ks = K / 16;
    *KS = ks <= 8 ? 8 : (ks <= 16 ? 16 : 32);
    // 0: head_exact_pipe_kernel (one wave per SIMD, 4 waves); 8 / 4: the
    // two-waves-per-SIMD head_exact_fwd_kernel (experiments)
    // default: the persistent LDS-DMA form with 64-ray tiles for K = 512 (the
    // reference networks' width; 243 us against 265 for the one-item form at
    // config 2 fp16), the register-staged form otherwise
    int w = K == 512 ? 19 : 8;
    if (const char* e = getenv("AVR_HEAD_EXACT_WAVES")) {
        const int v = atoi(e);
        w = (v == 4 || v == 8 || (v >= 16 && v <= 20)) ? v : 0;  // 16-20: the LDS-DMA forms (K = 512)
    }
    if (w >= 16 && K != 512) w = 8;
    *waves = w;
    return 0;
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

}  // namespace

extern "C" int avr_head_fwd_exact(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                                  const void* W, int32_t dtype, const int32_t* perm, const float* ws,
                                  const int32_t* cnt, float* z, void* stream) {
    AVR_REQUIRE(p && B >= 1 && h && W && perm && ws && cnt && z, "avr_head_fwd_exact: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_head_fwd_exact: h/W must be fp16 or bf16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0,
                "avr_head_fwd_exact: h and W must be 16-byte aligned");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    AVR_REQUIRE(R >= 1 && R <= 4096 && T >= 2 && S >= 1, "avr_head_fwd_exact: shape out of range");
    int KS, waves;
    if (int e = exact_shape(*p, K, &KS, &waves)) return e;
    const int TB = 32 * (waves == 0 ? 4 : (waves >= 16 ? 8 : waves));
    const int ntb = (T + TB - 1) / TB;
    const int64_t total = (int64_t)B * S * ntb;
    const int per_xcd = (int)((total + 7) / 8);
    const dim3 grid((unsigned)(8 * per_xcd));
    // profiling only: 1 = no MFMA, 2 = no HBM stream, 4 = no epilogue, 5 = the
    // row stream alone (fp16, K = 512, the LDS-DMA forms 16-18)
    const char* dbg_env = getenv("AVR_HEAD_EXACT_DBG");
    const int dbg = dbg_env ? atoi(dbg_env) : 0;
    hipStream_t st = as_stream(stream);
    auto go = [&](auto kern, auto ks_tag, auto w_tag, auto hp) {
        constexpr int KSV = decltype(ks_tag)::value, WV = decltype(w_tag)::value;
        const size_t lds = exact_lds_bytes<KSV, WV>(R);
        allow_lds(kern, lds);
        hipLaunchKernelGGL(kern, grid, dim3(64 * WV), lds, st, *p, (int)B, R, (int)K, hp, (decltype(hp))W,
                           perm, ws, cnt, z, ntb, per_xcd);
    };
    using I32 = std::integral_constant<int, 32>;
    using I8 = std::integral_constant<int, 8>;
    using I4 = std::integral_constant<int, 4>;
    if (waves == 20 && KS == 32 && K == 512) {  // two t-tiles per wave, persistent (one workgroup per CU)
        const size_t lds = 2 * (size_t)64 * a_row_bytes(32) + 8 * (size_t)((R + 63) / 64 * 64);
        int cus = 256, dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const int64_t ncol = (int64_t)B * S;
        const int64_t want = ((ncol + 7) / 8) * ntb;
        int wg_per_xcd = (int)std::min<int64_t>(want, std::max(1, cus / 8));
        wg_per_xcd = std::max(ntb, wg_per_xcd / ntb * ntb);
        auto go_w2 = [&](auto kern, auto hp) {
            allow_lds(kern, lds);
            hipLaunchKernelGGL(kern, dim3((unsigned)(8 * wg_per_xcd)), dim3(256), lds, st, *p, (int)B, R, (int)K, hp,
                               (decltype(hp))W, perm, ws, cnt, z, ntb, wg_per_xcd);
        };
        if (dtype == AVR_DTYPE_F16)
            go_w2(head_exact_w2_kernel<__half>, (const __half*)h);
        else
            go_w2(head_exact_w2_kernel<__hip_bfloat16>, (const __hip_bfloat16*)h);
        return check_launch("avr_head_fwd_exact");
    }
    if (waves >= 16 && KS == 32 && K == 512) {  // LDS-DMA forms (16: 32-ray tiles x 3 buffers, 17: 64 x 2, 18: 32 x 4,
                                                // 19: 64 x 2 persistent)
        const int TRv = (waves == 17 || waves == 19) ? 64 : 32, NB = waves == 16 ? 3 : (waves == 18 ? 4 : 2);
        const size_t lds = (size_t)NB * TRv * a_row_bytes(32) + 8 * (size_t)((R + TRv - 1) / TRv * TRv);
        // persistent: per XCD, as many workgroups as CUs hold (one each at
        // this LDS size), rounded down to whole t-block sets
        int wg_per_xcd = per_xcd;
        if (waves == 19) {
            int cus = 256;
            int dev = 0;
            if (hipGetDevice(&dev) == hipSuccess)
                (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            const int64_t ncol = (int64_t)B * S;
            const int64_t want = ((ncol + 7) / 8) * ntb;  // one workgroup per item of an XCD
            wg_per_xcd = (int)std::min<int64_t>(want, std::max(1, cus / 8));
            wg_per_xcd = std::max(ntb, wg_per_xcd / ntb * ntb);
        }
        const dim3 grid_dma((unsigned)(8 * (waves == 19 ? wg_per_xcd : per_xcd)));
        auto go_dma = [&](auto kern, auto hp) {
            allow_lds(kern, lds);
            hipLaunchKernelGGL(kern, grid_dma, dim3(512), lds, st, *p, (int)B, R, (int)K, hp, (decltype(hp))W, perm,
                               ws, cnt, z, ntb, waves == 19 ? wg_per_xcd : per_xcd);
        };
        if (waves == 19) {  // rays prefetched one column ahead while they fit 2 registers per thread
            if (R <= 1024) {
                if (dtype == AVR_DTYPE_F16)
                    go_dma(head_exact_dma_kernel<__half, 64, 2, 0, true, 2>, (const __half*)h);
                else
                    go_dma(head_exact_dma_kernel<__hip_bfloat16, 64, 2, 0, true, 2>, (const __hip_bfloat16*)h);
            } else {
                if (dtype == AVR_DTYPE_F16)
                    go_dma(head_exact_dma_kernel<__half, 64, 2, 0, true, 0>, (const __half*)h);
                else
                    go_dma(head_exact_dma_kernel<__hip_bfloat16, 64, 2, 0, true, 0>, (const __hip_bfloat16*)h);
            }
            return check_launch("avr_head_fwd_exact");
        }
#define AVR_HD(TRV, NBV)                                                                              \
        if (dtype == AVR_DTYPE_F16) {                                                                 \
            if (dbg == 1) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 1>, (const __half*)h);        \
            else if (dbg == 2) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 2>, (const __half*)h);   \
            else if (dbg == 3) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 3>, (const __half*)h);   \
            else if (dbg == 4) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 4>, (const __half*)h);   \
            else if (dbg == 5) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 5>, (const __half*)h);   \
            else if (dbg == 6) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 6>, (const __half*)h);   \
            else if (dbg == 8) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 8>, (const __half*)h);   \
            else if (dbg == 12) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 12>, (const __half*)h); \
            else if (dbg == 24) go_dma(head_exact_dma_kernel<__half, TRV, NBV, 24>, (const __half*)h); \
            else go_dma(head_exact_dma_kernel<__half, TRV, NBV, 0>, (const __half*)h);                 \
        } else {                                                                                      \
            go_dma(head_exact_dma_kernel<__hip_bfloat16, TRV, NBV, 0>, (const __hip_bfloat16*)h);     \
        }
        if (waves == 16) {
            AVR_HD(32, 3)
        } else if (waves == 17) {
            AVR_HD(64, 2)
        } else {
            AVR_HD(32, 4)
        }
#undef AVR_HD
        return check_launch("avr_head_fwd_exact");
    }
    if (waves == 0) {  // default form
        if (dbg && dtype == AVR_DTYPE_F16 && KS == 32) {
            if (dbg == 1) go(head_exact_pipe_kernel<__half, 32, 1>, I32{}, I4{}, (const __half*)h);
            else if (dbg == 2) go(head_exact_pipe_kernel<__half, 32, 2>, I32{}, I4{}, (const __half*)h);
            else go(head_exact_pipe_kernel<__half, 32, 3>, I32{}, I4{}, (const __half*)h);
            return check_launch("avr_head_fwd_exact");
        }
#define AVR_HP(TY, KSV) \
        if (KS == KSV) go(head_exact_pipe_kernel<TY, KSV>, std::integral_constant<int, KSV>{}, I4{}, (const TY*)h);
        if (dtype == AVR_DTYPE_F16) {
            AVR_HP(__half, 8) AVR_HP(__half, 16) AVR_HP(__half, 32)
        } else {
            AVR_HP(__hip_bfloat16, 8) AVR_HP(__hip_bfloat16, 16) AVR_HP(__hip_bfloat16, 32)
        }
#undef AVR_HP
        return check_launch("avr_head_fwd_exact");
    }
    if (dbg && dtype == AVR_DTYPE_F16 && KS == 32 && waves == 8) {
        if (dbg == 1) go(head_exact_fwd_kernel<__half, 32, 8, 1>, I32{}, I8{}, (const __half*)h);
        else if (dbg == 2) go(head_exact_fwd_kernel<__half, 32, 8, 2>, I32{}, I8{}, (const __half*)h);
        else go(head_exact_fwd_kernel<__half, 32, 8, 3>, I32{}, I8{}, (const __half*)h);
        return check_launch("avr_head_fwd_exact");
    }
#define AVR_HX(TY, KSV, WV)                                                                          \
    if (KS == KSV && waves == WV)                                                                    \
        go(head_exact_fwd_kernel<TY, KSV, WV>, std::integral_constant<int, KSV>{},                   \
           std::integral_constant<int, WV>{}, (const TY*)h);
#define AVR_HX_ALL(TY) AVR_HX(TY, 8, 8) AVR_HX(TY, 16, 8) AVR_HX(TY, 32, 8) AVR_HX(TY, 8, 4) AVR_HX(TY, 16, 4) AVR_HX(TY, 32, 4)
    if (dtype == AVR_DTYPE_F16) {
        AVR_HX_ALL(__half)
    } else {
        AVR_HX_ALL(__hip_bfloat16)
    }
#undef AVR_HX_ALL
#undef AVR_HX
    return check_launch("avr_head_fwd_exact");
}
