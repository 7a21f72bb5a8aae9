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
// cnt[t] = number of rays with delay <= t), so the live part of the
// [rays x t] plane is a staircase.
//
// h stationary, W streamed (round 4).  A work item is (ray block, column):
// 256 consecutive sorted rays of one column (b, s).  Each of the 4 waves (one
// per SIMD) loads the h rows of its 64 rays ONCE, from HBM straight into
// registers: 2 x K/16 MFMA A-fragments (256 VGPRs at K = 512).  The item then
// sweeps t in tiles of 32 from the first ray's delay to the tail limit; W,
// shared by every column and resident in each XCD's L2, streams through a
// 4-tile LDS ring by LDS-DMA in fragment order (avr_head_pack_w_exact), one
// 1 KiB B-fragment per k-step feeding the wave's two 32-ray MFMA chains.
// h crosses HBM exactly once (268 MB at config 2) and only W's 32 KB per
// tile moves through LDS-DMA.  A wave whose 64 rays are not live yet in a
// tile skips its chains (32 x 64 staircase granularity).
//
// Per tile every wave rounds, masks (p < cnt[t], select on the VALUE so an
// overflowed masked product cannot leak 0 * inf) and weights its 32 x 64
// products and sums them per lane in position order; the two lane halves are
// added, then the 4 waves' partials in wave order.  Each item writes its own
// slab zpart[block][b][s][t] (zero outside its live range); avr_dft_phase_fwd
// sums the n_split slabs in a fixed order, so results are deterministic.
// Items are ordered block-major (every column's first block first: the
// longest items start first and the short ones fill the tail).
#include "common.h"
#include "probe.h"
#include "stationary.h"

#include <algorithm>

using namespace avr;

AVR_PROBE_TU(avr_probe_set_exact)

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

// One 16-byte-per-lane LDS-DMA load: lane i's 16 bytes at g land at LDS byte
// address lds + 16 i.  Issued as inline asm so the compiler does not treat
// the in-flight DMA as an LDS write every later ds_read must wait for (with
// the builtin it inserts vmcnt(0) inside the MFMA chain); completion is
// waited for explicitly with counted vmcnt.
__device__ __forceinline__ void dma_row16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt not waited on; gfx9 encoding)
#define AVR_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))

// s_waitcnt vmcnt(n) for a run-time n (one case per value; above 31 the
// wait is for 31, a longer wait than asked)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define AVR_VMC(K) case K: AVR_VMCNT(K); break;
        AVR_VMC(0) AVR_VMC(1) AVR_VMC(2) AVR_VMC(3) AVR_VMC(4) AVR_VMC(5) AVR_VMC(6) AVR_VMC(7)
        AVR_VMC(8) AVR_VMC(9) AVR_VMC(10) AVR_VMC(11) AVR_VMC(12) AVR_VMC(13) AVR_VMC(14) AVR_VMC(15)
        AVR_VMC(16) AVR_VMC(17) AVR_VMC(18) AVR_VMC(19) AVR_VMC(20) AVR_VMC(21) AVR_VMC(22) AVR_VMC(23)
        AVR_VMC(24) AVR_VMC(25) AVR_VMC(26) AVR_VMC(27) AVR_VMC(28) AVR_VMC(29) AVR_VMC(30) AVR_VMC(31)
#undef AVR_VMC
        default: AVR_VMCNT(31); break;
    }
}

// bytes of one 32-t W tile in fragment order: KSM k-steps x 64 lanes x 16 B
__host__ __device__ constexpr int xs_tile_bytes(int KSM) { return KSM * 1024; }
__host__ __device__ constexpr size_t xs_lds_bytes(int KSM, int T, int waves, int rays, int nb, int nc) {
    return (size_t)nb * nc * xs_tile_bytes(KSM) + 4 * (size_t)((T + 3) / 4 * 4) + 4 * (size_t)rays +
           4 * (size_t)(2 * waves * 32 * nc) + 4 * (size_t)waves + 16;
}

// One work item: RAYS consecutive sorted rays of one column (b, s), WAVES
// waves of RPW = RAYS / WAVES rays (NQ = RPW / 32 MFMA A tiles each), a ring
// of NB W tiles.  <8, 256, 4>: one workgroup per CU (two waves per SIMD);
// <4, 128, 2>: half the item and ~70 KB of LDS, so two workgroups share a CU
// and one's prologue and barriers overlap the other's MFMA chains.
template <typename E, int KSM, int WAVES, int RAYS, int NB, int NC>
__global__ __launch_bounds__(64 * WAVES) void head_exact_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const frag8* __restrict__ Wf,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ zpart) {
    constexpr int NT = 64 * WAVES, TILE = NC * xs_tile_bytes(KSM);  // a tile: TT = 32 NC values of t
    constexpr int TT = 32 * NC;
    constexpr int RPW = RAYS / WAVES;    // rays per wave
    constexpr int NQ = RPW / 32;         // 32-ray A tiles per wave
    constexpr int DPW = NC * KSM / WAVES;  // 1 KiB DMAs per wave and tile
    static_assert((NC * KSM) % WAVES == 0 && NQ == 1 && DPW * NB <= 63 && NT >= RAYS, "shape");
    AVR_PROBE_DECL;
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    const int T = pp.T, S = pp.n_samples;
    const int Tp = (T + 3) & ~3;
    char* ring = lds_x;                                         // [NB][TILE]
    int* cl = reinterpret_cast<int*>(lds_x + NB * TILE);        // cnt of the column [Tp]
    float* wl = reinterpret_cast<float*>(cl + Tp);              // weights of the item's rays [RAYS]
    float* zr = wl + RAYS;                                      // wave partials [2][WAVES][TT]
    int* dstart = reinterpret_cast<int*>(zr + 2 * WAVES * TT);  // first live t per wave [WAVES]

    const int64_t ncol = (int64_t)B * S;
    const int64_t col = (int64_t)blockIdx.x % ncol;
    const int blk = (int)((int64_t)blockIdx.x / ncol);
    const int s = (int)(col % S), b = (int)(col / S);
    const int lim = tail_limit(pp, s);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    float* zc = zpart + ((int64_t)blk * ncol + col) * T;
    const int* cc = cnt + col * T;
    const int nk = cc[T - 1];  // kept rays of the column
    const int p0 = blk * RAYS;
    if (p0 >= nk || lim <= 0) {
        for (int t = threadIdx.x; t < T; t += NT) zc[t] = 0.0f;
        return;
    }
    // the wave's rows first: their DMA flies under the metadata work below
    // (positions past the kept rays repeat the last kept ray; masked)
    const int ksn = K / 16;
    const int pw = p0 + RPW * wave;
    const bool dma_rows = KSM == 32 && K == 512 && NQ == 1;
    const E* hrow[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int ray = perm[col * R + min(pw + 32 * q + j, nk - 1)];
        hrow[q] = h + (((int64_t)b * R + ray) * S + s) * K;
    }
    if (dma_rows) {
        stat_issue_round(reinterpret_cast<const uint16_t*>(hrow[0]), ring + wave * 16384, 0);
        stat_issue_round(reinterpret_cast<const uint16_t*>(hrow[0]), ring + wave * 16384, 1);
    }

    // ---- prologue: cnt and the item's weights into LDS; each wave's first live t
    for (int t = threadIdx.x; t < T; t += NT) cl[t] = cc[t];
    if (threadIdx.x < RAYS) {
        const int p = p0 + (int)threadIdx.x;
        wl[threadIdx.x] = p < nk ? ws[col * R + p] : 0.0f;
    }
    if (threadIdx.x < WAVES) dstart[threadIdx.x] = 1 << 30;
    __syncthreads();
    for (int t = threadIdx.x; t < lim; t += NT) {  // the delay of sorted ray p0 + RPW w (a kept ray: < lim)
        const int c = cl[t], cp = t > 0 ? cl[t - 1] : 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const int pw = p0 + RPW * w;
            if (c > pw && cp <= pw) dstart[w] = t;
        }
    }
    __syncthreads();
    AVR_PROBE_MARK(8);
    const int tb = dstart[0] / TT;              // first tile with a live ray of the item
    const int te = (lim + TT - 1) / TT;         // tiles holding t < lim
    const int tw = min(dstart[wave] / TT, te);  // this wave's first live tile
    for (int t = threadIdx.x; t < T; t += NT)
        if (t < TT * tb || t >= TT * te) zc[t] = 0.0f;

    // ---- the wave's rays: A fragments (k = 16 ks + 8 half + 0..7), loaded once
    frag8 a[NQ][KSM];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const E* hr = hrow[q];
        if (dma_rows) {
            // whole rows by LDS-DMA through the (still idle) ring, 16 KiB per wave
            stat_finish_rows512(reinterpret_cast<frag8_t(&)[32]>(a[q]), reinterpret_cast<const uint16_t*>(hr),
                                ring + wave * 16384);
        } else {
#pragma unroll
            for (int ks = 0; ks < KSM; ++ks)
                a[q][ks] = *reinterpret_cast<const frag8*>(hr + 8 * half + 16 * min(ks, ksn - 1));
#pragma unroll
            for (int ks = 0; ks < KSM; ++ks)
                if (ks >= ksn) a[q][ks] = frag8{0u, 0u, 0u, 0u};
#pragma unroll
            for (int ks = 0; ks < KSM; ++ks) asm volatile("" ::"v"(a[q][ks]));
            AVR_VMCNT(0);
        }
    }
    AVR_PROBE_MARK(9);
    __syncthreads();  // every wave is done with the staging area: the ring may fill
    AVR_PROBE_MARK(10);
    const uint32_t ring_lds = (uint32_t)(uintptr_t)ring;
    auto issue = [&](int tau, int slot) {  // W tile tau into ring slot `slot`: this wave's DPW pieces
        const char* src = reinterpret_cast<const char*>(Wf) + (int64_t)tau * TILE + wave * DPW * 1024 + 16 * lane;
        const uint32_t dst = ring_lds + slot * TILE + wave * DPW * 1024;
#pragma unroll
        for (int d = 0; d < DPW; ++d) dma_row16(src + d * 1024, dst + d * 1024);
    };
    for (int i = 0; i < NB - 1; ++i)
        if (tb + i < te) issue(tb + i, i);
    AVR_VMCNT(0);
    __syncthreads();
    AVR_PROBE_MARK(2);

    // the wave's 32 rays against 32-t column group c of the tile in ring slot
    // `slot`: one MFMA chain over K (A from registers, B read from the ring
    // D k-steps ahead), then the epilogue (rounded, masked by value:
    // p < cnt[t], weighted, summed per lane in row order)
    const float* wq = wl + RPW * wave + 4 * half;
    auto group = [&](int slot, int tau, int c) {
        const char* bsrc = ring + slot * TILE + c * xs_tile_bytes(KSM) + 16 * lane;
        constexpr int D = KSM < 8 ? KSM : 8;  // B fragments read ahead
        frag8 bw[D];
#pragma unroll
        for (int u = 0; u < D; ++u) bw[u] = *reinterpret_cast<const frag8*>(bsrc + u * 1024);
        f32x16 acc = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KSM; ++ks) {
            acc = mfma16<E>(a[0][ks], bw[ks % D], acc);
            if (ks + D < KSM) bw[ks % D] = *reinterpret_cast<const frag8*>(bsrc + (ks + D) * 1024);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
#pragma unroll
        for (int ks = 0; ks < KSM; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (ks + D < KSM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        // register r of acc is row (r & 3) + 8 (r >> 2) + 4 half of the wave's
        // rays, column t = TT tau + 32 c + j
        const int t0 = TT * tau + 32 * c;
        const int t = t0 + j;
        const int full = __builtin_amdgcn_readfirstlane((t0 + 31 < lim) ? cl[t0] : 0);
        float z = 0.0f;
        if (pw + 32 <= full) {  // every (ray, t) pair of the group is live
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 w4 = *reinterpret_cast<const float4*>(wq + 8 * g);
                z = fmaf(w4.x, round16<E>(acc[4 * g + 0]), z);
                z = fmaf(w4.y, round16<E>(acc[4 * g + 1]), z);
                z = fmaf(w4.z, round16<E>(acc[4 * g + 2]), z);
                z = fmaf(w4.w, round16<E>(acc[4 * g + 3]), z);
            }
        } else {
            const int ct = t < lim ? cl[min(t, T - 1)] : 0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 w4 = *reinterpret_cast<const float4*>(wq + 8 * g);
                const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = round16<E>(acc[4 * g + e]);
                    z = fmaf(wv[e], (pw + 8 * g + 4 * half + e < ct) ? v : 0.0f, z);
                }
            }
        }
        return z;
    };
    for (int tau = tb; tau < te; ++tau) {
        const int i = tau - tb;
        AVR_PROBE_BEGIN(comp);
        if (tau + NB - 1 < te) issue(tau + NB - 1, (i + NB - 1) % NB);  // the slot tile tau-1 left
        float zl[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            // group c holds a live ray of the wave from the wave's first live t
            // on (cnt is nondecreasing in t), and nothing at or past lim
            const int t0 = TT * tau + 32 * c;
            zl[c] = (t0 + 31 >= dstart[wave] && t0 < lim) ? group(i % NB, tau, c) : 0.0f;
        }
        AVR_PROBE_END(comp, 6);
        // lower + upper lane half (rows 4 half + ...), the same association in every lane
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const auto r =
                __builtin_amdgcn_permlane32_swap(__float_as_uint(zl[c]), __float_as_uint(zl[c]), false, false);
            const float v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
            if (half == 0) zr[(i & 1) * (WAVES * TT) + wave * TT + 32 * c + j] = v;
        }
        AVR_PROBE_BEGIN(dma);
        if (tau + 1 < te) {
            // this wave's pieces of tile tau+1 have landed.  Younger in vmcnt:
            // the ring's later tiles and this wave's partial stores since tile
            // tau+1 was issued (a wave stores after the barrier of iteration m
            // when wave == m % WAVES), so no store in flight is waited for
            int st = 0;
            for (int m = max(0, i + 2 - NB); m < i; ++m) st += (wave == m % WAVES);
            wait_vm(min(NB - 2, te - 2 - tau) * DPW + st);
        }
        AVR_PROBE_END(dma, 4);
        AVR_PROBE_BEGIN(bar);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // every LDS access of tile tau (and the partials) done
        __builtin_amdgcn_s_barrier();
        AVR_PROBE_END(bar, 5);
        if (wave == (i % WAVES) && lane < TT) {  // the wave partials of tile tau, in wave order
            const float* zz = zr + (i & 1) * (WAVES * TT) + lane;
            float v = zz[0];
#pragma unroll
            for (int w = 1; w < WAVES; ++w) v += zz[TT * w];
            const int t = TT * tau + lane;
            if (t < T) zc[t] = v;
        }
    }
    AVR_PROBE_FLUSH(blockIdx.x * WAVES + wave);
}

// W [T][K] -> Wf: for t-tile tau and k-step ks, the 64 lanes' 16-byte B
// fragments of v_mfma_f32_32x32x16 (lane (j, half): W[32 tau + j][16 ks + 8 half
// + 0..7]) contiguous, zero past T and K
template <typename E>
__global__ __launch_bounds__(256) void head_pack_exact_kernel(int T, int K, int KSM, const uint16_t* __restrict__ W,
                                                              frag8* __restrict__ Wf, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int lane = (int)(i & 63);
        const int64_t r = i >> 6;
        const int ks = (int)(r % KSM);
        const int tau = (int)(r / KSM);
        const int t = 32 * tau + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
        frag8 v = frag8{0u, 0u, 0u, 0u};
        if (t < T && k0 < K) v = *reinterpret_cast<const frag8*>(W + (int64_t)t * K + k0);
        Wf[i] = v;
    }
}

int exact_ksm(int K) { return K <= 128 ? 8 : (K <= 256 ? 16 : 32); }

// Work-item shape: 128 rays and two workgroups per CU where the DFT's slab
// count allows (<= 2048 rays) and two ~70 KB LDS images fit (T <= 1024);
// 256 rays, one workgroup per CU, otherwise.  AVR_EXACT_RAYS_PROBE=256 forces
// the latter (probe runs).
int exact_rays(int R, int T) {
    const char* e = getenv("AVR_EXACT_RAYS_PROBE");
    if (e && atoi(e) == 256) return 256;
    return (R <= 16 * 128 && T <= 1024) ? 128 : 256;
}

int exact_check(const avr_render_params* p, int32_t K, int32_t dtype) {
    AVR_REQUIRE(p, "avr_head_fwd_exact: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_head_fwd_exact: h/W must be fp16 or bf16");
    if (K % 16 != 0 || K < 16 || K > 512) return fail(AVR_E_CONFIG, "exact head: K must be a multiple of 16, <= 512");
    const int R = n_rays(*p);
    AVR_REQUIRE(R >= 1 && R <= 16 * 256 && p->T >= 2 && p->T <= 4096 && p->n_samples >= 1,
                "avr_head_fwd_exact: shape out of range (<= 4096 rays per shard, T <= 4096)");
    return 0;
}

int exact_splits(int R, int T) {
    const int rays = exact_rays(R, T);
    const int nb = (R + rays - 1) / rays;
    int n = 1;
    while (n < nb) n *= 2;
    return n;
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

}  // namespace

extern "C" int avr_head_exact_layout(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                                     int32_t* n_split, int64_t* wpack_bytes) {
    AVR_REQUIRE(B >= 1 && n_split && wpack_bytes, "avr_head_exact_layout: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    *n_split = exact_splits(n_rays(*p), p->T);
    // whole 64-t tile pairs (a 64-t tile reads two consecutive 32-t tiles), zero past T
    *wpack_bytes = (int64_t)((p->T + 63) / 64) * 2 * xs_tile_bytes(exact_ksm(K));
    return 0;
}

extern "C" int avr_head_pack_w_exact(const avr_render_params* p, int32_t K, const void* W, int32_t dtype,
                                     void* Wf, void* stream) {
    AVR_REQUIRE(W && Wf, "avr_head_pack_w_exact: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(W) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_head_pack_w_exact: W and Wf must be 16-byte aligned");
    const int T = p->T, KSM = exact_ksm(K);
    const int64_t n = (int64_t)((T + 63) / 64) * 2 * KSM * 64;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(head_pack_exact_kernel<__half>, dim3(blocks), dim3(256), 0, as_stream(stream), T, (int)K,
                       KSM, (const uint16_t*)W, (frag8*)Wf, n);
    return check_launch("avr_head_pack_w_exact");
}

extern "C" int avr_head_fwd_exact(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* Wf,
                                  int32_t dtype, const int32_t* perm, const float* ws, const int32_t* cnt,
                                  int32_t n_split, float* zpart, void* stream) {
    AVR_REQUIRE(p && B >= 1 && h && Wf && perm && ws && cnt && zpart, "avr_head_fwd_exact: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_head_fwd_exact: h and Wf must be 16-byte aligned");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    AVR_REQUIRE(n_split == exact_splits(R, T), "avr_head_fwd_exact: n_split must be avr_head_exact_layout's");
    const int64_t items = (int64_t)n_split * B * S;
    AVR_REQUIRE(items < (1ll << 31), "avr_head_fwd_exact: too many columns");
    const int KSM = exact_ksm(K);
    hipStream_t st = as_stream(stream);
    const bool small = exact_rays(R, T) == 128;
    const char* tte = getenv("AVR_EXACT_TT_PROBE");
    const bool tt64 = !small && tte && atoi(tte) == 64;
    auto run = [&](auto e_tag) {
        using E = decltype(e_tag);
        auto go = [&](auto kern, int ksm, int waves, int rays, int nb, int nc, const void* hv) {
            const size_t lds = xs_lds_bytes(ksm, T, waves, rays, nb, nc);
            allow_lds(kern, lds);
            hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(64 * waves), lds, st, *p, (int)B, R, (int)K,
                               (const E*)hv, (const frag8*)Wf, perm, ws, cnt, zpart);
        };
        if (small) {
            if (KSM == 8) go(head_exact_kernel<E, 8, 4, 128, 2, 1>, 8, 4, 128, 2, 1, h);
            else if (KSM == 16) go(head_exact_kernel<E, 16, 4, 128, 2, 1>, 16, 4, 128, 2, 1, h);
            else go(head_exact_kernel<E, 32, 4, 128, 2, 1>, 32, 4, 128, 2, 1, h);
        } else if (tt64 && KSM == 32) {
            go(head_exact_kernel<E, 32, 8, 256, 2, 2>, 32, 8, 256, 2, 2, h);
        } else {
            if (KSM == 8) go(head_exact_kernel<E, 8, 8, 256, 4, 1>, 8, 8, 256, 4, 1, h);
            else if (KSM == 16) go(head_exact_kernel<E, 16, 8, 256, 4, 1>, 16, 8, 256, 4, 1, h);
            else go(head_exact_kernel<E, 32, 8, 256, 4, 1>, 32, 8, 256, 4, 1, h);
        }
    };
    if (dtype == AVR_DTYPE_F16)
        run(__half{});
    else
        run(__hip_bfloat16{});
    return check_launch("avr_head_fwd_exact");
}
