// Fused signal head, linear form, forward by delay bands (SURVEY.md §8f
// rank 1; the same quantity as head_fwd_kernel in head.hip, for 16-bit h).
//
// The reference renders x = h W^T (model.py:176-180 -> renderer.py:72-115):
//
//   z[b,s,t] = sum_{p < cnt[t]} ws[p] x_p[t],   x_p[t] = h[b,perm_p,s,:] . W[t,:]
//
// with a column's live rays sorted by delay (avr_head_sort: perm, ws, and
// cnt[t] = number of kept rays with delay <= t).  Cut t into tiles of 32 and
// let lo_tau = cnt[32 tau - 1] (0 for tau = 0): the rays before position
// lo_tau have a delay below the tile, so by linearity, for t in tile tau,
//
//   z[t] = W[t] . C_tau + sum_{lo_tau <= p < cnt[t]} ws[p] x_p[t],
//   C_tau = sum_{p < lo_tau} ws[p] h_p                      (a K-vector)
//
// The band [lo_tau, hi_tau) of every live ray is its own tile, so a column
// costs one pass over its rows in sorted order: R x 32 x K band products on
// the matrix cores (v_mfma_f32_32x32x16_{f16,bf16}: rays x t, fp32
// accumulation) plus T x K for the C terms, and reads each h row once, whole.
// head_fwd_kernel instead gathers 64-byte row pieces per lane (3 TB/s).
//
// Work: one workgroup per (column b*S+s, slice of 128 features); the slices
// are the DFT's n_split partials ([n][B][S][T], like head_fwd_kernel).  Four
// waves, 32 features each.  The slice's 256-byte row pieces stream through
// an LDS ring in chunks of 32 sorted positions by LDS-DMA (whole 128-byte
// lines, 4 rows per instruction), NBUF-1 chunks ahead, XOR-swizzled so the 32
// rows of an MFMA fragment read fall on distinct bank quads.  W's fragments
// (the MFMA B operand, 32 t x 32 features per wave) come from L2 straight
// into registers, kD tiles ahead.  Every sum runs in a fixed order: results
// are bitwise reproducible.
//
// Status: the default for 16-bit h; at config 2 fp16 it runs
// 139.4 us against 141.6 us for head_fwd_kernel (warmed up, interleaved), and
// is closer to a float64 sum.  Measured bounds: the streaming skeleton alone
// (no C terms, no band products) takes 63-66 us, the compute adds ~75 us that
// the two or three workgroups per CU do not hide.
#include "common.h"

#include <algorithm>

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));  // 8 packed 16-bit values

constexpr int kSliceK = 128;                    // features per workgroup (WV waves x 128/WV)
constexpr int kRowB = kSliceK * 2;              // 256 bytes of a row per slice
constexpr int kChunkB = 32 * kRowB;             // 8 KiB: 32 rows

template <typename E>
__device__ __forceinline__ f32x16 mfma16(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: the DMAs stay in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS access moves across the barrier
}

// lane i's 16 bytes at g land at LDS byte address lds + 16 i (asm-issued, so
// the compiler never waits on it; see head_exact.hip's dma_row16)
__device__ __forceinline__ void band_dma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// s_waitcnt until at most n of this wave's vector-memory operations are
// outstanding (n rounded down to an encodable step: waiting longer is safe)
#define AVR_BAND_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))
__device__ __forceinline__ void wait_vm_le(int n) {
    if (n >= 24) AVR_BAND_VMCNT(24);
    else if (n >= 20) AVR_BAND_VMCNT(20);
    else if (n >= 16) AVR_BAND_VMCNT(16);
    else if (n >= 14) AVR_BAND_VMCNT(14);
    else if (n >= 12) AVR_BAND_VMCNT(12);
    else if (n >= 10) AVR_BAND_VMCNT(10);
    else if (n >= 8) AVR_BAND_VMCNT(8);
    else if (n >= 6) AVR_BAND_VMCNT(6);
    else if (n >= 4) AVR_BAND_VMCNT(4);
    else if (n >= 2) AVR_BAND_VMCNT(2);
    else AVR_BAND_VMCNT(0);
}
#undef AVR_BAND_VMCNT

// sum over the 16 lanes of a DPP row (every lane gets it; lane-dependent
// association order, fixed for a given lane)
__device__ __forceinline__ float row_sum16(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));  // row_ror:8
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));  // row_ror:4
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));  // row_ror:2
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));  // row_ror:1
    return x;
}

constexpr int kBandWaves = 4;
constexpr int kBandBuf = 4;  // chunk ring: 3 chunks in flight ahead of the one in use

__host__ __device__ constexpr size_t band_lds_bytes(int R, int T, int nbuf = kBandBuf) {
    return (size_t)nbuf * kChunkB + 8 * (size_t)((R + 31) / 32 * 32) + 4 * (size_t)((T + 3) / 4 * 4) +
           4 * 2 * kBandWaves * 32;
}

// sum of x over the two lanes 16 apart (the two DPP rows of a lane half),
// the same association in every lane
__device__ __forceinline__ float swap16_sum(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// lower half + upper half of the wave, in every lane
__device__ __forceinline__ float swap32_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// dbg (AVR_HEAD_BAND_DBG, timing experiments only; results then wrong):
// 1 waits for every DMA, 2 skips the C terms, 8 the band products, 16 the
// chunk barriers, 32 the tile barriers
template <typename E, int NBUF = kBandBuf>
__global__ __launch_bounds__(64 * kBandWaves) void head_band_fwd_kernel(
    avr_render_params pp, int B, int R, int K, int nq, int kbw, const E* __restrict__ h, const E* __restrict__ Wp,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    float* __restrict__ zpart, int dbg) {
    constexpr int PD = NBUF - 1, WV = kBandWaves;
    constexpr int KS = 8 / WV;   // k-steps of 16 per wave
    constexpr int IPW = 8 / WV;  // DMA instructions per wave per 32-row block
    extern __shared__ __attribute__((aligned(16))) char lds_b[];
    const int RP = (R + 31) / 32 * 32;
    char* hbuf = lds_b;                                     // [NBUF][32 rows][256 B]
    int* pl = reinterpret_cast<int*>(hbuf + NBUF * kChunkB);  // [RP] sorted rays
    float* wl = reinterpret_cast<float*>(pl + RP);          // [RP] their weights
    int* cl = reinterpret_cast<int*>(wl + RP);              // [T] cnt
    float* zs = reinterpret_cast<float*>(cl + (pp.T + 3) / 4 * 4);  // [2][WV][32] per-wave z of a tile

    const int T = pp.T, S = pp.n_samples;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, j = lane & 31;
    const int q = (int)(blockIdx.x % nq);
    const int64_t col = blockIdx.x / nq;
    const int s = (int)(col % S), b = (int)(col / S);
    float* zcol = zpart + ((int64_t)q * B * S + col) * T;
    const int limc = min(tail_limit(pp, s), T);
    if (limc <= 0) {
        for (int t = threadIdx.x; t < T; t += 64 * WV) zcol[t] = 0.0f;
        return;
    }
    for (int i = threadIdx.x; i < RP; i += 64 * WV) {
        pl[i] = i < R ? perm[col * R + i] : 0;
        wl[i] = i < R ? ws[col * R + i] : 0.0f;
    }
    for (int i = threadIdx.x; i < T; i += 64 * WV) cl[i] = cnt[col * T + i];
    __syncthreads();
    const int nlive = __builtin_amdgcn_readfirstlane(cl[limc - 1]);
    const int ntl = (limc + 31) / 32;  // t-tiles with a live t
    const int nch = (nlive + 31) / 32;
    const E* hcol = h + ((int64_t)b * R * S + s) * K + q * kSliceK;
    const int64_t hstride = (int64_t)S * K;

    // this wave's two DMA instructions of a 32-row block: instruction ii moves
    // rows 4 ii .. 4 ii + 3; lane L fetches piece (L & 15) ^ (row & 15) of row
    // 4 ii + L / 16 into slot L & 15 of that row
    const int drow0 = 4 * IPW * wave + (lane >> 4);
    auto issue_chunk = [&](int c) {
        char* dst = hbuf + (c % NBUF) * kChunkB;
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
            const int row = drow0 + 4 * i;
            const int ray = pl[min(32 * c + row, nlive - 1)];
            const int piece = (lane & 15) ^ (row & 15);
            band_dma16(hcol + (int64_t)ray * hstride + piece * 8, (uint32_t)(uintptr_t)(dst + (IPW * wave + i) * 1024));
        }
    };
    // byte offset of this lane's fragment for k-step ks in a swizzled 32-row block
    int foff[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) foff[ks] = j * kRowB + (((2 * KS * wave + 2 * ks + half) ^ (j & 15)) * 16);

    // DMA bookkeeping (uniform): instructions issued by this wave and the
    // count right after each pending chunk (FIFO)
    int issued = 0, npend = 0, cur = -1, nxt = 0;
    int fifo[NBUF];
#pragma unroll
    for (int i = 0; i < NBUF; ++i) fifo[i] = 0;
    auto push_chunk = [&]() {
        issue_chunk(nxt);
        ++nxt;
        issued += IPW;
#pragma unroll
        for (int i = 0; i < NBUF; ++i)
            if (i == npend) fifo[i] = issued;
        ++npend;
    };
    auto advance = [&]() {  // make chunk cur + 1 the one in use
        ++cur;
        wait_vm_le((dbg & 1) ? 0 : issued - fifo[0]);
#pragma unroll
        for (int i = 0; i + 1 < NBUF; ++i) fifo[i] = fifo[i + 1];
        --npend;
        if (!(dbg & 16)) lds_barrier();  // chunk cur landed for every wave; every wave is done with chunk cur - 1
        if (nxt < nch) push_chunk();  // into chunk cur - 1's buffer
    };

    for (int i = 0; i < PD; ++i)
        if (nxt < nch) push_chunk();

    // z of tile u: the waves' shares added in wave order (by wave u % 4)
    auto finish = [&](int u) {
        const int t = 32 * u + j;
        if (wave == (u & (WV - 1)) && half == 0 && t < T) {
            const float* zu = zs + (u & 1) * 32 * WV + j;
            float v = zu[0];
#pragma unroll
            for (int w = 1; w < WV; ++w) v += zu[32 * w];
            zcol[t] = t < limc ? v : 0.0f;
        }
    };

    float cs[KS][8];  // this lane's row slot: sum of ws * h over the bands so far
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 8; ++i) cs[ks][i] = 0.0f;

    // one t-tile with the W fragments bw of its 32 t
    auto tile = [&](int tau, const frag8 (&bw)[KS]) {
        const int t = 32 * tau + j;
        const int cnt_t = t < limc ? cl[t] : 0;
        const int lo = tau > 0 ? __builtin_amdgcn_readfirstlane(cl[32 * tau - 1]) : 0;
        const int hi = __builtin_amdgcn_readfirstlane(cl[min(32 * tau + 31, limc - 1)]);
        float zl = 0.0f;
        if (lo > 0 && !(dbg & 2)) {
            // C_tau over this half's features (the 32 row slots summed), dotted
            // with W[t] on the same features
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float c = swap16_sum(row_sum16(cs[ks][i]));
                    zl = fmaf(c, unpack16<E>(bw[ks][i >> 1], i & 1), zl);
                }
        }
        for (int c = lo >> 5; 32 * c < hi; ++c) {
            if (cur < c) advance();
            if (dbg & 8) continue;
            const char* a = hbuf + (c % NBUF) * kChunkB;
            frag8 af[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) af[ks] = *reinterpret_cast<const frag8*>(a + foff[ks]);
            f32x16 acc = {};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) acc = mfma16<E>(af[ks], bw[ks], acc);
            const int p0 = 32 * c;
            // acc[4g + e]: sorted position p0 + 8g + 4 half + e at this lane's t
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 wv = *reinterpret_cast<const float4*>(wl + p0 + 8 * g + 4 * half);
                const float w4[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int p = p0 + 8 * g + 4 * half + e;
                    zl = fmaf((p >= lo && p < cnt_t) ? w4[e] : 0.0f, acc[4 * g + e], zl);
                }
            }
            // this lane's row (position p0 + j) joins C if it lies in the band
            const int pr = p0 + j;
            const float wr = (pr >= lo && pr < hi) ? wl[pr] : 0.0f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int i = 0; i < 8; ++i) cs[ks][i] = fmaf(wr, unpack16<E>(af[ks][i >> 1], i & 1), cs[ks][i]);
        }
        // this wave's features' share of z, summed over the waves in wave
        // order by one wave after the next barrier
        const float zw = swap32_sum(zl);
        if (half == 0) zs[(tau & 1) * 32 * WV + wave * 32 + j] = zw;
    };

    {
        // W fragments straight from memory (L2) into registers, kD
        // tiles ahead, slots rotated by unrolling (compiler-visible loads:
        // the compiler's wait before a slot's first use also covers the
        // LDS-DMAs issued before the younger slots' loads, i.e. chunks issued
        // kD - 1 tiles earlier)
        constexpr int kD = 4;
        frag8 wq[kD][KS];
        auto load_w = [&](int tau, frag8 (&dst)[KS]) {
            const int t = min(32 * tau + j, T - 1);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int k0 = q * kSliceK + 16 * KS * wave + 16 * ks + 8 * half;
                dst[ks] = *reinterpret_cast<const frag8*>(Wp + ((int64_t)(k0 / kbw) * T + t) * kbw + (k0 % kbw));
            }
        };
#pragma unroll
        for (int u = 0; u < kD; ++u)
            if (u < ntl) load_w(u, wq[u]);
        for (int tau0 = 0; tau0 < ntl; tau0 += kD) {
#pragma unroll
            for (int u = 0; u < kD; ++u) {
                const int tau = tau0 + u;
                if (tau < ntl) {
                    if (!(dbg & 32)) lds_barrier();  // the previous tile's z shares are in LDS
                    if (tau > 0) finish(tau - 1);
                    tile(tau, wq[u]);
                    if (tau + kD < ntl) load_w(tau + kD, wq[u]);
                }
            }
        }
    }
    lds_barrier();
    finish(ntl - 1);
    for (int t = 32 * ntl + (int)threadIdx.x; t < T; t += 64 * WV) zcol[t] = 0.0f;
    // every DMA this wave issued has landed before the workgroup ends
    __builtin_amdgcn_s_waitcnt(0);
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

}  // namespace

namespace avr {

// Feature slices of the band forward for this shape (the DFT's n_split), or 0
// when it does not apply: 16-bit h, K a multiple of 128 with K/128 a power of
// two <= 16, W packed in blocks of >= 8 features, <= 4096 rays and T.
// AVR_HEAD_BAND=0 selects head_fwd_kernel (A/B runs, tests).
int head_band_slices(const avr_render_params& p, int K, int es, int kbw) {
    if (const char* e = getenv("AVR_HEAD_BAND"))
        if (atoi(e) == 0) return 0;
    if (es != 2 || K % kSliceK != 0 || kbw % 8 != 0) return 0;
    const int nq = K / kSliceK;
    if (nq > 16 || (nq & (nq - 1)) != 0) return 0;
    if (n_rays(p) > 4096 || p.T > 4096 || p.T < 2) return 0;
    if (band_lds_bytes(n_rays(p), p.T) > 160 * 1024) return 0;
    return nq;
}

int head_band_fwd(const avr_render_params& p, int B, int K, const void* h, const void* Wp, int dtype, int kbw,
                  const int32_t* perm, const float* ws, const int32_t* cnt, int nq, float* zpart,
                  hipStream_t st) {
    const int R = n_rays(p), S = p.n_samples, T = p.T;
    const int64_t items = (int64_t)B * S * nq;
    AVR_REQUIRE(items <= 0x7fffffff, "avr_head_fwd: too many columns");
    const char* dbg_env = getenv("AVR_HEAD_BAND_DBG");  // experiments only
    const int dbg = dbg_env ? atoi(dbg_env) : 0;
    // AVR_HEAD_BAND_BUF=3: a 3-slot chunk ring (experiments)
    const char* buf_env = getenv("AVR_HEAD_BAND_BUF");
    const int nbuf = (buf_env && atoi(buf_env) == 3) ? 3 : kBandBuf;
    const size_t lds = band_lds_bytes(R, T, nbuf);
    auto go = [&](auto kern, auto e) {
        using E = decltype(e);
        allow_lds(kern, lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)items), dim3(64 * kBandWaves), lds, st, p, B, R, K, nq, kbw,
                           (const E*)h, (const E*)Wp, perm, ws, cnt, zpart, dbg);
    };
    if (dtype == AVR_DTYPE_F16) {
        if (nbuf == 3)
            go(head_band_fwd_kernel<__half, 3>, __half{});
        else
            go(head_band_fwd_kernel<__half>, __half{});
    } else {
        if (nbuf == 3)
            go(head_band_fwd_kernel<__hip_bfloat16, 3>, __hip_bfloat16{});
        else
            go(head_band_fwd_kernel<__hip_bfloat16>, __hip_bfloat16{});
    }
    return check_launch("avr_head_fwd (band)");
}

}  // namespace avr
