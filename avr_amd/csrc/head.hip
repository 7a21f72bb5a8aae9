// Fused signal head: the signal network's last,
// bias-free linear layer (model.py:176-180, output_activation None) folded
// into the ray reduction, so the [B,R,S,T] network output never exists.
//
// With h the last hidden activation [B,R,S,K] and W the layer's weight [T,K]
// (x = h W^T is what the reference network returns), the reduction's column
// sum is, by linearity,
//
//   z[b,s,t] = sum_r w[b,r,s] [d_brs <= t < lim_s] x[b,r,s,t]
//            = sum_k W[t,k] P[b,s,k,t],   P[b,s,k,t] = sum_{r: d_brs <= t} w_brs h_brsk
//
// (lim_s = T-1-shift_s).  P is a prefix sum over t of a scatter of w*h into
// delay bins, so a column costs R*K scatter-adds + K*T scan + K*T MACs
// instead of the R*K*T of the layer itself plus an R*T*4-byte round trip.
// Per workgroup: one (b, s) and a group of KG features, processed as LDS
// blocks of KB features x T bins.  The partials of the feature groups are
// the DFT's "n_split" partials (same [n][B][S][T] layout as the reduction).
//
// Backward, with gz = dL/dz (avr_dft_phase_bwd, zero for t >= lim):
//   Q[b,s,k,d] = sum_{t >= d} gz[b,s,t] W[t,k]          (suffix scan over t)
//   dL/dh[b,r,s,k] = w_brs Q[b,s,k,d_brs]   (0 if d_brs >= lim_s)
//   dL/dw[b,r,s]   = sum_k h_brsk Q[b,s,k,d_brs]
//   dL/dW[t,k]     = sum_{b,s} gz[b,s,t] P[b,s,k,t]
// The first two come from head_bwd_h (per (b, s, feature group)), the last
// from head_bwd_w (per (feature block, s group, b), accumulating over its
// samples in registers).  Every sum runs in a fixed order (rays sorted by
// the total order (delay, ray); no float atomics), so renders and gradients
// are bitwise reproducible.
#include "common.h"

using namespace avr;

namespace {

constexpr int kThreads = 256;

// Barrier for LDS-only communication: waits for this thread's LDS traffic but
// leaves its global loads in flight (__syncthreads would drain them), so the
// next block's operands stream in while the current block is scanned.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched (gfx9 encoding)
    __builtin_amdgcn_s_barrier();
}

// KB consecutive elements of a row, held raw (packed) in registers until used
template <typename Th, int KB>
struct Raw {
    static constexpr int NB = KB * (int)sizeof(Th);  // 8..64 bytes
    static constexpr int ND = NB / 4;
    uint32_t d[ND];
    __device__ __forceinline__ void load(const Th* p) {
        if constexpr (NB % 16 == 0) {
#pragma unroll
            for (int c = 0; c < NB / 16; ++c) {
                const u32x4 v = reinterpret_cast<const u32x4*>(p)[c];
                d[4 * c] = v[0];
                d[4 * c + 1] = v[1];
                d[4 * c + 2] = v[2];
                d[4 * c + 3] = v[3];
            }
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(p);
            d[0] = v.x;
            d[1] = v.y;
        }
    }
    __device__ __forceinline__ float operator[](int k) const {
        if constexpr (sizeof(Th) == 2)
            return unpack16<Th>(d[k >> 1], k & 1);
        else
            return __uint_as_float(d[k]);
    }
};

template <typename Th, int KB>
__device__ __forceinline__ void store_block(Th* p, const float* v) {
    if constexpr (sizeof(Th) == 2) {
        uint32_t u[KB / 2];
#pragma unroll
        for (int i = 0; i < KB / 2; ++i) u[i] = pack16<Th>(v[2 * i], v[2 * i + 1]);
        if constexpr (KB >= 8) {
#pragma unroll
            for (int c = 0; c < KB / 8; ++c)
                reinterpret_cast<u32x4*>(p)[c] = u32x4{u[4 * c], u[4 * c + 1], u[4 * c + 2], u[4 * c + 3]};
        } else {
            *reinterpret_cast<uint2*>(p) = make_uint2(u[0], u[1]);
        }
    } else {
#pragma unroll
        for (int c = 0; c < KB / 4; ++c)
            reinterpret_cast<f32x4*>(p)[c] = f32x4{v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
    }
}

// Row stride of Q[KB][qs] in head_bwd_h: T rounded up to 4 floats, so every
// thread's scan segment starts 16-byte aligned.
__host__ __device__ constexpr int q_stride(int T) { return (T + 3) / 4 * 4; }

// In-place inclusive prefix (or suffix) sums of the KB rows of A[KB][qs]:
// 256/KB threads per row, each a contiguous segment of a multiple of 4
// floats read and written as 16-byte vectors (lanes 4*seg4/4 words apart:
// distinct bank quads, conflict-free), segment totals combined by a shuffle
// scan inside the row's lanes (a row's threads share a wave).
template <int KB, bool SUFFIX>
__device__ __forceinline__ void scan_rows(float* A, int T) {
    constexpr int TPR = kThreads / KB;  // 16, 32 or 64 (<= one wave)
    const int row = threadIdx.x / TPR, j = threadIdx.x % TPR;
    const int seg = ((T + TPR - 1) / TPR + 3) / 4 * 4;
    float* a = A + row * q_stride(T);
    const int lo = min(T, j * seg), hi = min(T, lo + seg);
    const int nfull = (hi - lo) / 4;  // whole 16-byte chunks; the tail (< 4) only in the last segment
    f32x4* a4 = reinterpret_cast<f32x4*>(a + lo);
    float run = 0.0f;
    if (!SUFFIX) {
        for (int c = 0; c < nfull; ++c) {
            f32x4 v = a4[c];
            v[0] += run;
            v[1] += v[0];
            v[2] += v[1];
            v[3] += v[2];
            run = v[3];
            a4[c] = v;
        }
        for (int t = lo + 4 * nfull; t < hi; ++t) {
            run += a[t];
            a[t] = run;
        }
    } else {
        for (int t = hi - 1; t >= lo + 4 * nfull; --t) {
            run += a[t];
            a[t] = run;
        }
        for (int c = nfull - 1; c >= 0; --c) {
            f32x4 v = a4[c];
            v[3] += run;
            v[2] += v[3];
            v[1] += v[2];
            v[0] += v[1];
            run = v[0];
            a4[c] = v;
        }
    }
    // exclusive scan of the segment totals over the TPR lanes of this row
    // (inclusive shuffle scan, then shifted by one lane: no subtraction)
    float x = run, off;
    if (!SUFFIX) {
#pragma unroll
        for (int d = 1; d < TPR; d <<= 1) {
            const float y = __shfl_up(x, d, 64);
            if (j >= d) x += y;
        }
        off = __shfl_up(x, 1, 64);
        if (j == 0) off = 0.0f;
    } else {
#pragma unroll
        for (int d = 1; d < TPR; d <<= 1) {
            const float y = __shfl_down(x, d, 64);
            if (j + d < TPR) x += y;
        }
        off = __shfl_down(x, 1, 64);
        if (j == TPR - 1) off = 0.0f;
    }
    if (off != 0.0f) {
        for (int c = 0; c < nfull; ++c) {
            f32x4 v = a4[c];
            v[0] += off;
            v[1] += off;
            v[2] += off;
            v[3] += off;
            a4[c] = v;
        }
        for (int t = lo + 4 * nfull; t < hi; ++t) a[t] += off;
    }
}

// The RPT rays a thread owns (r = tid + 256*u) and their w / delay
template <int RPT>
struct Rays {
    float w[RPT];
    int d[RPT];
    __device__ __forceinline__ void load(const float* __restrict__ wp, const int32_t* __restrict__ dp,
                                         int b, int s, int R, int S) {
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int r = threadIdx.x + kThreads * u;
            const int64_t i = ((int64_t)b * R + min(r, R - 1)) * S + s;
            w[u] = wp[i];
            d[u] = r < R ? dp[i] : 0x7fffffff;  // spare slots are never live
        }
    }
};

template <typename Th, int KB, int RPT>
__device__ __forceinline__ void load_rows(Raw<Th, KB> (&v)[RPT], const Th* __restrict__ h, int64_t hrow0,
                                          int64_t hstride, int k0, int R) {
#pragma unroll
    for (int u = 0; u < RPT; ++u)
        v[u].load(h + hrow0 + (int64_t)min((int)threadIdx.x + kThreads * u, R - 1) * hstride + k0);
}

// W rows t of feature block k0 / KB from the forward's packed layout
// Wp[K/KB][T][KB] (avr_head_pack_w): a wave-instruction reads 64 consecutive
// t, i.e. 64*KB contiguous elements, instead of 64 rows K elements apart.
template <typename Th, int KB, int NT>
__device__ __forceinline__ void load_wpacked(Raw<Th, KB> (&v)[NT], const Th* __restrict__ Wp, int k0, int T) {
#pragma unroll
    for (int i = 0; i < NT; ++i)
        v[i].load(Wp + ((int64_t)(k0 / KB) * T + min((int)threadIdx.x + kThreads * i, T - 1)) * KB);
}

// Runs of equal keys over the lanes of a wavefront (consecutive rays have
// slowly changing delays): the run's first lane, last lane and whether this
// lane ends its run.
struct Run {
    int first, last;
    bool tail;
};
__device__ __forceinline__ Run lane_run(int key) {
    const int lane = threadIdx.x & 63;
    const int prev = __shfl_up(key, 1, 64);
    const bool head = lane == 0 || prev != key;
    const unsigned long long heads = __ballot(head);
    const unsigned long long upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
    Run r;
    r.first = 63 - __clzll(heads & upto);
    const unsigned long long later = heads & ~upto;
    r.last = later ? (__ffsll((long long)later) - 2) : 63;
    r.tail = r.last == lane;
    return r;
}

// In-place inclusive prefix sum of cnt[0..T) (ints): contiguous segments per
// thread, segment totals scanned through the wavefronts and 4 LDS slots.
__device__ __forceinline__ void block_inclusive_scan(int* cnt, int T, int* wtot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = (T + kThreads - 1) / kThreads;
    const int lo = threadIdx.x * seg, hi = min(T, lo + seg);
    int tot = 0;
    for (int t = lo; t < hi; ++t) tot += cnt[t];
    int x = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    lds_barrier();
    int off = x - tot;  // exact for ints
    for (int w = 0; w < wave; ++w) off += wtot[w];
    for (int t = lo; t < hi; ++t) {
        off += cnt[t];
        cnt[t] = off;
    }
}

// Smallest power of two >= R (the bitonic sort's key array)
__host__ __device__ constexpr int pow2_ceil(int R) {
    int n = 1;
    while (n < R) n <<= 1;
    return n;
}

// Ascending bitonic sort of keys[0..n) (n a power of two) in LDS.  The keys
// are distinct, so the result (and everything summed in its order) does not
// depend on how the waves are scheduled.
__device__ __forceinline__ void bitonic_sort(uint32_t* keys, int n) {
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < (n >> 1); i += kThreads) {
                const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                const int hi = lo + j;
                const uint32_t a = keys[lo], c = keys[hi];
                if ((a > c) == ((lo & k) == 0)) {
                    keys[lo] = c;
                    keys[hi] = a;
                }
            }
            lds_barrier();
        }
    }
}

// The same bitonic network with the keys in registers: thread t holds
// positions t*KPT .. t*KPT+KPT-1 (n = 256*KPT).  Exchange distances below
// KPT stay inside a thread, those below 64*KPT cross lanes of one wave
// (ds_bpermute shuffles, no barrier); only the distances that cross waves
// go through LDS.  At n = 1024 that is 3 barrier-separated LDS passes
// instead of 55.  Same compare-exchanges, so the same sorted keys.
template <int KPT>
__device__ __forceinline__ void bitonic_sort_regs(uint32_t* keys) {
    constexpr int n = kThreads * KPT;
    constexpr int kWaveSpan = 64 * KPT;  // distances below this stay in a wave
    const int t = threadIdx.x;
    uint32_t v[KPT];
#pragma unroll
    for (int e = 0; e < KPT; ++e) v[e] = keys[t * KPT + e];
#pragma unroll
    for (int k = 2; k <= n; k <<= 1) {
        if ((k >> 1) >= kWaveSpan) {  // cross-wave distances through LDS
#pragma unroll
            for (int e = 0; e < KPT; ++e) keys[t * KPT + e] = v[e];
            lds_barrier();
            for (int j = k >> 1; j >= kWaveSpan; j >>= 1) {
                for (int i = t; i < (n >> 1); i += kThreads) {
                    const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                    const int hi = lo + j;
                    const uint32_t a = keys[lo], c = keys[hi];
                    if ((a > c) == ((lo & k) == 0)) {
                        keys[lo] = c;
                        keys[hi] = a;
                    }
                }
                lds_barrier();
            }
#pragma unroll
            for (int e = 0; e < KPT; ++e) v[e] = keys[t * KPT + e];
            lds_barrier();  // every read done before the next LDS write
        }
#pragma unroll
        for (int j = ((k >> 1) < kWaveSpan ? (k >> 1) : kWaveSpan >> 1); j >= KPT; j >>= 1) {
#pragma unroll
            for (int e = 0; e < KPT; ++e) {
                const int i = t * KPT + e;
                const uint32_t p = (uint32_t)__shfl_xor((int)v[e], j / KPT, 64);
                const bool keep_min = ((i & k) == 0) == ((i & j) == 0);
                v[e] = keep_min ? min(v[e], p) : max(v[e], p);
            }
        }
#pragma unroll
        for (int j = ((k >> 1) < KPT ? (k >> 1) : KPT >> 1); j >= 1; j >>= 1) {
#pragma unroll
            for (int e = 0; e < KPT; ++e) {
                if (e & j) continue;
                const int i = t * KPT + e;  // lower of the pair (e, e ^ j)
                const uint32_t a = v[e], c = v[e ^ j];
                const bool asc = (i & k) == 0;
                v[e] = asc ? min(a, c) : max(a, c);
                v[e ^ j] = asc ? max(a, c) : min(a, c);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < KPT; ++e) keys[t * KPT + e] = v[e];
    lds_barrier();
}

// Rays of column (b, s) with a non-empty window (d < lim), sorted by
// (delay, ray) -- a total order, so the sort is deterministic: keys
// (d << 12 | r) in LDS through a bitonic sort; afterwards cnt[t] = number of
// live rays with delay <= t (integer histogram + scan, order-free) and
// keys[p] & 0xfff is the p-th ray.  Returns the number of live rays.
template <int RPT>
__device__ __forceinline__ int sort_rays(const Rays<RPT>& rays, int lim, int T, int R, int* cnt, float* wr,
                                         uint32_t* keys, int nk, int* wtot) {
    for (int t = threadIdx.x; t < T; t += kThreads) cnt[t] = 0;
    for (int i = threadIdx.x; i < nk; i += kThreads) keys[i] = 0xffffffffu;
    lds_barrier();
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int r = threadIdx.x + kThreads * u;
        const int d = rays.d[u];
        const bool live = d < lim;
        if (r < R) wr[r] = rays.w[u];
        if (live) keys[r] = ((uint32_t)d << 12) | (uint32_t)r;
        const Run run = lane_run(live ? d : -1);
        if (run.tail && live) atomicAdd(&cnt[d], run.last - run.first + 1);  // integer: order-free
    }
    lds_barrier();
    block_inclusive_scan(cnt, T, wtot);
    // the scan does not end with a barrier; the sorts below only hide that
    // for nk >= 2 (a one-ray shard runs no sort pass)
    lds_barrier();
    if (nk == 1024)
        bitonic_sort_regs<4>(keys);
    else if (nk == 2048)
        bitonic_sort_regs<8>(keys);
    else if (nk == 4096)
        bitonic_sort_regs<16>(keys);
    else
        bitonic_sort(keys, nk);
    return T > 0 ? cnt[T - 1] : 0;
}

// Row stride of C: C[k][j] sits at k*RS + 3 + j, so the slots j = p0+1 ..
// p0+RPT a thread owns (p0 = tid*RPT) start 16-byte aligned, and a thread
// whose last owned slot runs past the row's n rays stays inside the row.
__host__ __device__ constexpr int cs_stride(int R) { return ((R + 22) / 4) * 4; }

// DPP operand of a wave-wide scan step (VALU cross-lane move, no LDS trip)
template <int CTRL, int ROW_MASK, bool BOUND>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xf, BOUND));
}

// Inclusive scan over the 64 lanes: row_shr 1,2,4,8 inside each 16-lane row,
// then row_bcast:15 / row_bcast:31 carry the row totals forward.
__device__ __forceinline__ float wave_scan_incl(float x) {
    x += dpp<0x111, 0xf, true>(x);
    x += dpp<0x112, 0xf, true>(x);
    x += dpp<0x114, 0xf, true>(x);
    x += dpp<0x118, 0xf, true>(x);
    x += dpp<0x142, 0xa, false>(x);
    x += dpp<0x143, 0xc, false>(x);
    return x;
}

// C[k][j] = sum of w h[k] over the first j sorted rays, i.e.
// P[k][t] = C[k][cnt[t]].  Thread i owns sorted positions i*spt ..
// i*spt+spt-1; its h rows (hv, already loaded) are summed locally, the
// per-thread totals scanned across the block (DPP inside a wave, 4 LDS slots
// across waves).  When a thread owns RPT positions (spt == RPT) its slots are
// written as 16-byte vectors.
template <typename Th, int KB, int RPT>
__device__ __forceinline__ void build_cumsum(float* C, int R, int n, int spt, const float (&wr)[RPT],
                                             const Raw<Th, KB> (&hv)[RPT], float* wtotf) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int RS = cs_stride(R);
    const int p0 = threadIdx.x * spt;
    // local totals first; the local prefixes are recomputed (same fmaf
    // chain, bit-identical) while C is written, instead of held in RPT*KB
    // registers across the scan
    float run[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) run[k] = 0.0f;
#pragma unroll
    for (int u = 0; u < RPT; ++u)
#pragma unroll
        for (int k = 0; k < KB; ++k) run[k] = fmaf(wr[u], hv[u][k], run[k]);
    // exclusive scan of run[k] over the 256 threads
    float off[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
        const float x = wave_scan_incl(run[k]);
        off[k] = dpp<0x138, 0xf, true>(x);  // wave_shr:1 (lane 0 reads 0): exclusive
        if (lane == 63) wtotf[wave * KB + k] = x;
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < KB; ++k) {
        float o = 0.0f;
        for (int w = 0; w < wave; ++w) o += wtotf[w * KB + k];
        off[k] += o;
    }
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < KB; ++k) C[k * RS + 3] = 0.0f;
    if (RPT % 4 == 0 && spt == RPT) {
        if (p0 < n)
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                float r = 0.0f;
#pragma unroll
                for (int c = 0; c < RPT / 4; ++c) {
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        r = fmaf(wr[4 * c + e], hv[4 * c + e][k], r);
                        v[e] = off[k] + r;
                    }
                    *reinterpret_cast<f32x4*>(C + k * RS + 4 + p0 + 4 * c) = f32x4{v[0], v[1], v[2], v[3]};
                }
            }
    } else {
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            float r = 0.0f;
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                r = fmaf(wr[u], hv[u][k], r);
                if (u < spt && p0 + u < n) C[k * RS + 4 + p0 + u] = off[k] + r;
            }
        }
    }
}

// The sorted positions a thread owns (p = tid*spt + u, u < spt): the ray and
// its weight (0 for positions past n), from the avr_head_sort tables.
template <int RPT>
struct Owned {
    int ray[RPT];
    float w[RPT];
    int n, spt;
    __device__ __forceinline__ void load(const int* __restrict__ perm, const float* __restrict__ ws,
                                         const int* __restrict__ cnt, int T) {
        n = cnt[T - 1];
        spt = (n + kThreads - 1) / kThreads;  // <= RPT
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int p = threadIdx.x * spt + u;
            const bool ok = u < spt && p < n;
            ray[u] = ok ? perm[p] : 0;
            w[u] = ok ? ws[p] : 0.0f;
        }
    }
};

template <typename Th, int KB, int RPT>
__device__ __forceinline__ void load_sorted_rows(Raw<Th, KB> (&v)[RPT], const Th* __restrict__ h, int64_t hrow0,
                                                 int64_t hstride, int k0, const Owned<RPT>& own) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) v[u].load(h + hrow0 + (int64_t)own.ray[u] * hstride + k0);
}

// LDS of the cumulative-sum kernels: C[KB][cs_stride(R)] | wave totals
__host__ __device__ constexpr size_t cumsum_lds_bytes(int R, int KB) {
    return 4 * ((size_t)KB * cs_stride(R) + 4 * (size_t)KB);
}

// Counting sort of the rays of every column (b, s) by delay (rays with an
// empty window, d >= lim, dropped): perm / ws [B][S][R] and
// cnt[B][S][T] = number of kept rays with delay <= t.  Shared by the forward
// feature groups and by both backward kernels.
template <int RPT>
__global__ __launch_bounds__(kThreads) void head_sort_kernel(avr_render_params pp, int R,
                                                             const float* __restrict__ w,
                                                             const int32_t* __restrict__ delay,
                                                             int* __restrict__ perm_out,
                                                             float* __restrict__ ws_out,
                                                             int* __restrict__ cnt_out) {
    extern __shared__ float lds_f[];
    const int T = pp.T, S = pp.n_samples;
    const int s = blockIdx.x, b = blockIdx.y;
    const int nk = pow2_ceil(R);
    int* cnt = reinterpret_cast<int*>(lds_f);
    float* wr = reinterpret_cast<float*>(cnt + T);
    uint32_t* keys = reinterpret_cast<uint32_t*>(wr + R);
    int* wtot = reinterpret_cast<int*>(keys + nk);
    Rays<RPT> rays;
    rays.load(w, delay, b, s, R, S);
    const int n = sort_rays<RPT>(rays, tail_limit(pp, s), T, R, cnt, wr, keys, nk, wtot);
    const int64_t col = (int64_t)b * S + s;
    for (int p = threadIdx.x; p < R; p += kThreads) {
        const int r = p < n ? (int)(keys[p] & 0xfffu) : 0;
        perm_out[col * R + p] = r;
        ws_out[col * R + p] = p < n ? wr[r] : 0.0f;
    }
    for (int t = threadIdx.x; t < T; t += kThreads) cnt_out[col * T + t] = cnt[t];
}

// W [T][K] -> Wp[K/KB][T][KB] (the forward's feature-block-major layout)
template <typename Th>
__global__ __launch_bounds__(kThreads) void head_pack_w_kernel(int T, int K, int KB, const Th* __restrict__ W,
                                                               Th* __restrict__ Wp) {
    const int64_t n = (int64_t)T * K;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const int j = (int)(i % KB);
        const int64_t r = i / KB;  // = kb * T + t
        const int t = (int)(r % T), kb = (int)(r / T);
        Wp[i] = W[(int64_t)t * K + kb * KB + j];
    }
}

// ------------------------------------------------------------------ forward
// Per (feature group, s, b): rays counting-sorted by delay once; per feature
// block, cumulative sums over the sorted rays (no float atomics), then
// z[t] += sum_k W[t,k] C[k][cnt[t]].  The next block's h rows and W rows are
// loaded as soon as the current ones are consumed (LDS-only barriers keep
// them in flight).
//
// SB > 1: each ray's h is loaded SB feature blocks at a time (64 bytes for
// 16-bit h with SB = 2), the next such super-block in flight under the current
// one's SB blocks.  A 128-byte line of a row holds 64 16-bit features: loaded
// one 32-byte block at a time it is requested 4 times, spread over 4 block
// iterations, and with ~64 workgroups per XCD each holding 1024 such lines
// it has left L2 by then (PMC: 1.08 GB fetched for the 268 MB h at config 2).
// W here is the packed Wp[K/KB][T][KB] of avr_head_pack_w.
template <typename Th, int KB, int NT, int RPT, int SB>
__global__ __launch_bounds__(kThreads) void head_fwd_kernel(avr_render_params pp, int B, int R, int K,
                                                            int KG, const Th* __restrict__ h,
                                                            const Th* __restrict__ W,
                                                            const int* __restrict__ perm,
                                                            const float* __restrict__ ws,
                                                            const int* __restrict__ cnt,
                                                            float* __restrict__ zpart) {
    extern __shared__ float lds_f[];
    const int T = pp.T, S = pp.n_samples;
    const int kg = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
    float* C = lds_f;                  // [KB][RS]
    const int RS = cs_stride(R);
    float* wtotf = C + KB * RS;        // [4][KB]
    const int lim = tail_limit(pp, s);
    const int64_t col = (int64_t)b * S + s;
    const int64_t hrow0 = ((int64_t)b * R * S + s) * K;
    const int64_t hstride = (int64_t)S * K;
    const int kbeg = kg * KG, kend = kbeg + KG;
    Raw<Th, KB> wt[NT];
    load_wpacked<Th, KB, NT>(wt, W, kbeg, T);
    Owned<RPT> own;
    own.load(perm + col * R, ws + col * R, cnt + col * T, T);
    int ct[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) ct[i] = cnt[col * T + min((int)threadIdx.x + kThreads * i, T - 1)];
    float zacc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) zacc[i] = 0.0f;
    auto contract = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < lim) {
                float a = zacc[i];
#pragma unroll
                for (int k = 0; k < KB; ++k) a = fmaf(wt[i][k], C[k * RS + 3 + ct[i]], a);
                zacc[i] = a;
            }
        }
        if (k0 + KB < kend) load_wpacked<Th, KB, NT>(wt, W, k0 + KB, T);
        lds_barrier();  // C and wtotf are rewritten by the next block
    };
    if constexpr (SB == 1) {
        Raw<Th, KB> hv[RPT];
        load_sorted_rows<Th, KB, RPT>(hv, h, hrow0, hstride, kbeg, own);
        for (int k0 = kbeg; k0 < kend; k0 += KB) {
            build_cumsum<Th, KB, RPT>(C, R, own.n, own.spt, own.w, hv, wtotf);
            if (k0 + KB < kend) load_sorted_rows<Th, KB, RPT>(hv, h, hrow0, hstride, k0 + KB, own);
            lds_barrier();
            contract(k0);
        }
    } else {
        constexpr int ND = Raw<Th, KB>::ND;
        Raw<Th, KB * SB> nxt[RPT];
        auto load_sb = [&](int k0) { load_sorted_rows<Th, KB * SB, RPT>(nxt, h, hrow0, hstride, k0, own); };
        load_sb(kbeg);
        for (int k0 = kbeg; k0 < kend; k0 += KB * SB) {
            Raw<Th, KB * SB> big[RPT];
#pragma unroll
            for (int u = 0; u < RPT; ++u) big[u] = nxt[u];
            if (k0 + KB * SB < kend) load_sb(k0 + KB * SB);
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                Raw<Th, KB> hv[RPT];
#pragma unroll
                for (int u = 0; u < RPT; ++u)
#pragma unroll
                    for (int d = 0; d < ND; ++d) hv[u].d[d] = big[u].d[sb * ND + d];
                build_cumsum<Th, KB, RPT>(C, R, own.n, own.spt, own.w, hv, wtotf);
                lds_barrier();
                contract(k0 + sb * KB);
            }
        }
    }
    float* out = zpart + (((int64_t)kg * B + b) * S + s) * T;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = threadIdx.x + kThreads * i;
        if (t < T) out[t] = t < lim ? zacc[i] : 0.0f;
    }
}

// ------------------------------------------------- backward: dL/dh, dL/dw
// relu_mask: h is a ReLU output consumed only by the head, and grad_h leaves
// with that ReLU's backward applied, threshold_backward(grad_h, h, 0)'s
// selection (0 where h <= 0; NaN keeps), on the rounded value
__device__ __forceinline__ bool relu_keeps(float hv) { return !(hv <= 0.0f); }

// SB > 1 (16-bit h): each ray's h is loaded and its grad_h stored SB feature
// blocks at a time (32 bytes per row for SB = 2) instead of 16 bytes per
// block; the grad_h of the SB blocks waits packed in registers.
template <typename Th, int KB, int NT, int RPT, int SB = 1>
__global__ __launch_bounds__(kThreads) void head_bwd_h_kernel(avr_render_params pp, int B, int R, int K,
                                                              int KG, const Th* __restrict__ h,
                                                              const Th* __restrict__ W,
                                                              const float* __restrict__ w,
                                                              const int32_t* __restrict__ delay,
                                                              const float* __restrict__ gz,
                                                              Th* __restrict__ grad_h,
                                                              float* __restrict__ gw_part, int relu_mask) {
    extern __shared__ float Q[];  // [KB][QS]
    const int T = pp.T, S = pp.n_samples;
    const int QS = q_stride(T);
    const int kg = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
    const int lim = tail_limit(pp, s);
    const int64_t hrow0 = ((int64_t)b * R * S + s) * K;
    const int64_t hstride = (int64_t)S * K;
    const int kbeg = kg * KG, kend = kbeg + KG;
    Rays<RPT> rays;
    rays.load(w, delay, b, s, R, S);
    const float* gzr = gz + ((int64_t)b * S + s) * T;
    float g[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = threadIdx.x + kThreads * i;
        const float v = gzr[min(t, T - 1)];
        g[i] = t < lim ? v : 0.0f;
    }
    Raw<Th, KB> wt[NT];
    load_wpacked<Th, KB, NT>(wt, W, kbeg, T);  // W packed [K/KB][T][KB] by avr_head_bwd
    float gw[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) gw[u] = 0.0f;
    // Q[k][t] = suffix sum over t of gz[t] W[t][k] for feature block kk
    auto build_q = [&](int kk) {
        lds_barrier();
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < T)
#pragma unroll
                for (int k = 0; k < KB; ++k) Q[k * QS + t] = g[i] * wt[i][k];
        }
        if (kk + KB < kend) load_wpacked<Th, KB, NT>(wt, W, kk + KB, T);
        lds_barrier();
        scan_rows<KB, true>(Q, T);
        lds_barrier();
    };
    if constexpr (SB == 1) {
        Raw<Th, KB> hv[RPT];
        load_rows<Th, KB, RPT>(hv, h, hrow0, hstride, kbeg, R);
        for (int k0 = kbeg; k0 < kend; k0 += KB) {
            build_q(k0);
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int r = threadIdx.x + kThreads * u;
                if (r < R) {
                    const int d = rays.d[u];
                    float gh[KB];
                    if (d < lim) {
                        const float wr = rays.w[u];
                        float acc = gw[u];
#pragma unroll
                        for (int k = 0; k < KB; ++k) {
                            const float q = Q[k * QS + d];
                            gh[k] = (!relu_mask || relu_keeps(hv[u][k])) ? wr * q : 0.0f;
                            acc = fmaf(hv[u][k], q, acc);
                        }
                        gw[u] = acc;
                    } else {
#pragma unroll
                        for (int k = 0; k < KB; ++k) gh[k] = 0.0f;
                    }
                    store_block<Th, KB>(grad_h + hrow0 + (int64_t)r * hstride + k0, gh);
                }
            }
            if (k0 + KB < kend) load_rows<Th, KB, RPT>(hv, h, hrow0, hstride, k0 + KB, R);
        }
    } else {
        static_assert(sizeof(Th) == 2, "super-blocks are for 16-bit h");
        constexpr int NDW = KB * SB / 2;  // dwords of SB blocks of one row
        Raw<Th, KB * SB> hv[RPT];
        load_rows<Th, KB * SB, RPT>(hv, h, hrow0, hstride, kbeg, R);
        for (int k0 = kbeg; k0 < kend; k0 += KB * SB) {
            uint32_t ghp[RPT][NDW];
#pragma unroll
            for (int sb = 0; sb < SB; ++sb) {
                build_q(k0 + sb * KB);
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    const int d = rays.d[u];
                    const bool live = d < lim && (int)threadIdx.x + kThreads * u < R;
                    const float wr = rays.w[u];
                    float acc = gw[u];
#pragma unroll
                    for (int k = 0; k < KB; k += 2) {
                        const float q0 = live ? Q[k * QS + d] : 0.0f;
                        const float q1 = live ? Q[(k + 1) * QS + d] : 0.0f;
                        acc = fmaf(hv[u][sb * KB + k], q0, acc);
                        acc = fmaf(hv[u][sb * KB + k + 1], q1, acc);
                        const bool k0 = live && (!relu_mask || relu_keeps(hv[u][sb * KB + k]));
                        const bool k1 = live && (!relu_mask || relu_keeps(hv[u][sb * KB + k + 1]));
                        ghp[u][sb * KB / 2 + k / 2] = pack16<Th>(k0 ? wr * q0 : 0.0f, k1 ? wr * q1 : 0.0f);
                    }
                    if (live) gw[u] = acc;
                }
            }
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int r = threadIdx.x + kThreads * u;
                if (r < R) {
                    u32x4* dst = reinterpret_cast<u32x4*>(grad_h + hrow0 + (int64_t)r * hstride + k0);
#pragma unroll
                    for (int c = 0; c < NDW / 4; ++c)
                        dst[c] = u32x4{ghp[u][4 * c], ghp[u][4 * c + 1], ghp[u][4 * c + 2], ghp[u][4 * c + 3]};
                }
            }
            if (k0 + KB * SB < kend) load_rows<Th, KB * SB, RPT>(hv, h, hrow0, hstride, k0 + KB * SB, R);
        }
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int r = threadIdx.x + kThreads * u;
        if (r < R) gw_part[(((int64_t)kg * B + b) * R + r) * S + s] = gw[u];
    }
}

// ------------------------------------ backward: dL/dh, dL/dw by block sums
// The scan form above builds Q[k][t] for every t of every feature block in
// LDS (three barriers per 8 features) although each ray reads Q only at its
// own delay.  Here Q at a delay is assembled from sums computed once per
// column (blk = ceil(d / kHbBlk)):
//   Q[k](d) = sum_{d <= t < min(kHbBlk blk, lim)} gz[t] W[t,k]    (< kHbBlk terms)
//           + L[k](blk)        (suffix from kHbBlk blk within its kHbSeg-t segment)
//           + C[k](segment)    (the totals of the later segments)
// head_bwd_suffix writes L every kHbBlk t and the segment totals (one wave
// per 128 features x segment x column, walking t downward); head_bwd_carry
// turns the totals into C; head_bwd_h_blk gives every ray 16 lanes of 8
// features, reads its L and C rows and up to kHbBlk - 1 W rows, and writes
// grad_h and its dL/dw partial (16-lane sum).  Every sum is in a fixed order
// (bitwise reproducible); the rays need no sort.  Config 3 (bf16, K = 512,
// T = 1600): 99 us per step against 207 for the scan form and its W pack
// (block of 8 t and 128-t segments measured against 4 / 16 t and 64 / 256 t).
constexpr int kHbBlk = 8;    // t between stored block sums
constexpr int kHbSeg = 128;  // t per suffix segment (a multiple of kHbBlk)
constexpr int kHbFeat = 128; // features per workgroup (16 lanes x 8)

__host__ __device__ inline int hb_nblk(int T) { return (T + kHbBlk - 1) / kHbBlk + 1; }
__host__ __device__ inline int hb_nseg(int T) { return (T + kHbSeg - 1) / kHbSeg; }

template <typename Th>
__global__ __launch_bounds__(64) void head_bwd_suffix_kernel(avr_render_params pp, int K, const Th* __restrict__ W,
                                                             const float* __restrict__ gz, float* __restrict__ L,
                                                             float* __restrict__ segtot) {
    const int T = pp.T, S = pp.n_samples;
    const int seg = blockIdx.y, col = blockIdx.z, s = col % S;
    const int nblk = hb_nblk(T), nseg = hb_nseg(T);
    const int k = blockIdx.x * kHbFeat + 2 * threadIdx.x;  // this lane's two features
    const int lim = tail_limit(pp, s);
    const int t0 = seg * kHbSeg, t1 = min(t0 + kHbSeg, lim);
    const bool on = k < K;
    const int kc = on ? k : 0;  // (lanes past K load a valid pair and store nothing)
    const float* g = gz + (int64_t)col * T;
    float a0 = 0.0f, a1 = 0.0f;
    // t downward in batches of 16 (the batch's W rows and gz loaded first;
    // t below the segment clamped to its first t and masked out of the sums)
    for (int tb = t1 - 1; tb >= t0; tb -= 16) {
        float wv0[16], wv1[16], gv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int t = max(tb - j, t0);
            gv[j] = tb - j >= t0 ? g[t] : 0.0f;
            if constexpr (sizeof(Th) == 2) {
                const uint32_t u = *reinterpret_cast<const uint32_t*>(W + (int64_t)t * K + kc);
                wv0[j] = unpack16<Th>(u, 0);
                wv1[j] = unpack16<Th>(u, 1);
            } else {
                const float2 v = *reinterpret_cast<const float2*>(W + (int64_t)t * K + kc);
                wv0[j] = v.x;
                wv1[j] = v.y;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int t = tb - j;
            // (gv is 0 below the segment: a0 + 0 * w is a0 for finite W)
            if (t >= t0) {
                a0 = fmaf(gv[j], wv0[j], a0);
                a1 = fmaf(gv[j], wv1[j], a1);
            }
            if (t >= t0 && t % kHbBlk == 0 && on)
                *reinterpret_cast<float2*>(L + ((int64_t)col * nblk + t / kHbBlk) * K + k) = make_float2(a0, a1);
        }
    }
    if (on) *reinterpret_cast<float2*>(segtot + ((int64_t)col * nseg + seg) * K + k) = make_float2(a0, a1);
}

// C[col][seg][k] = sum of the totals of the segments after seg (last first)
__global__ __launch_bounds__(256) void head_bwd_carry_kernel(int T, int K, int64_t n, const float* __restrict__ segtot,
                                                             float* __restrict__ C) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (col, k)
    if (i >= n) return;
    const int nseg = hb_nseg(T);
    const int64_t col = i / K, k = i - col * K;
    float c = 0.0f;
    for (int sg = nseg - 1; sg >= 0; --sg) {
        const int64_t at = (col * nseg + sg) * K + k;
        C[at] = c;
        c += segtot[at];
    }
}

template <typename Th>
__global__ __launch_bounds__(256) void head_bwd_h_blk_kernel(avr_render_params pp, int B, int R, int K,
                                                             const Th* __restrict__ h, const Th* __restrict__ W,
                                                             const float* __restrict__ w,
                                                             const int32_t* __restrict__ delay,
                                                             const float* __restrict__ gz,
                                                             const float* __restrict__ L,
                                                             const float* __restrict__ C,
                                                             Th* __restrict__ grad_h, float* __restrict__ gw_part,
                                                             int relu_mask) {
    const int T = pp.T, S = pp.n_samples;
    const int fg = blockIdx.x, col = blockIdx.z, b = col / S, s = col % S;
    const int r = blockIdx.y * 16 + (threadIdx.x >> 4), sub = threadIdx.x & 15;
    if (r >= R) return;  // (a whole 16-lane group)
    const int nblk = hb_nblk(T), nseg = hb_nseg(T);
    const int k = fg * kHbFeat + 8 * sub;
    const bool on = k < K;
    const int lim = tail_limit(pp, s);
    const int64_t idx = ((int64_t)b * R + r) * S + s;
    const int d = delay[idx];
    float gwv = 0.0f;
    if (d >= lim) {  // empty window: no gradient
        float z[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        if (on) store_block<Th, 8>(grad_h + idx * K + k, z);
    } else {
        const float wr = w[idx];
        Raw<Th, 8> hv;
        if (on) hv.load(h + idx * K + k);
        const int blk = (d + kHbBlk - 1) / kHbBlk;
        const int te = min(blk * kHbBlk, lim);
        const float* g = gz + (int64_t)col * T;
        const int kc = on ? k : 0;  // (lanes past K load valid rows and store nothing)
        float q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = 0.0f;
        // the partial block, t downward from te - 1 to d (at most kHbBlk - 1
        // terms): every load issued first, from clamped t, masked by value
        float gt[kHbBlk - 1];
        Raw<Th, 8> wv[kHbBlk - 1];
#pragma unroll
        for (int j = 0; j < kHbBlk - 1; ++j) {
            const int t = max(te - 1 - j, d);
            gt[j] = g[t];
            wv[j].load(W + (int64_t)t * K + kc);
        }
#pragma unroll
        for (int j = 0; j < kHbBlk - 1; ++j)
            if (te - 1 - j >= d) {
#pragma unroll
                for (int i = 0; i < 8; ++i) q[i] = fmaf(gt[j], wv[j][i], q[i]);
            }
        if (blk * kHbBlk < lim) {
            const f32x4* lp = reinterpret_cast<const f32x4*>(L + ((int64_t)col * nblk + blk) * K + kc);
            const f32x4* cp =
                reinterpret_cast<const f32x4*>(C + ((int64_t)col * nseg + blk * kHbBlk / kHbSeg) * K + kc);
            const f32x4 l0 = lp[0], l1 = lp[1], c0 = cp[0], c1 = cp[1];
            q[0] += l0[0]; q[1] += l0[1]; q[2] += l0[2]; q[3] += l0[3];
            q[4] += l1[0]; q[5] += l1[1]; q[6] += l1[2]; q[7] += l1[3];
            q[0] += c0[0]; q[1] += c0[1]; q[2] += c0[2]; q[3] += c0[3];
            q[4] += c1[0]; q[5] += c1[1]; q[6] += c1[2]; q[7] += c1[3];
        }
        if (on) {
            float gh[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                gwv = fmaf(hv[i], q[i], gwv);
                gh[i] = (!relu_mask || relu_keeps(hv[i])) ? wr * q[i] : 0.0f;
            }
            store_block<Th, 8>(grad_h + idx * K + k, gh);
        }
    }
    // the ray's dL/dw partial over this workgroup's features: 16-lane sum
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) gwv += __shfl_xor(gwv, off, 16);
    if (sub == 0) gw_part[((int64_t)fg * B + b) * R * S + (int64_t)r * S + s] = gwv;
}

// ---------------------------------------------------- backward: dL/dW
// One workgroup per (feature block, sample group, b): for each of its
// samples, sort the rays, build the cumulative sums C (as the forward) and
// accumulate gz[t] C[k][cnt[t]] in registers; one [T][KB] partial per
// workgroup.  The next sample's rays and gz are loaded during the current one.
template <typename Th, int KB, int NT, int RPT>
__global__ __launch_bounds__(kThreads) void head_bwd_w_kernel(avr_render_params pp, int B, int R, int K,
                                                              int s_per_group,
                                                              const Th* __restrict__ h,
                                                              const int* __restrict__ perm,
                                                              const float* __restrict__ ws,
                                                              const int* __restrict__ cnt,
                                                              const float* __restrict__ gz,
                                                              float* __restrict__ gW_part) {
    extern __shared__ float lds_f[];
    const int T = pp.T, S = pp.n_samples;
    const int kb = blockIdx.x, sg = blockIdx.y, b = blockIdx.z;
    const int k0 = kb * KB;
    float* C = lds_f;
    const int RS = cs_stride(R);
    float* wtotf = C + KB * RS;
    const int64_t hstride = (int64_t)S * K;
    float acc[NT][KB];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int k = 0; k < KB; ++k) acc[i][k] = 0.0f;
    const int s_lo = sg * s_per_group, s_hi = min(S, s_lo + s_per_group);
    Owned<RPT> own;
    Raw<Th, KB> hv[RPT];
    float g[NT];
    int ct[NT];
    auto prefetch = [&](int s) {
        const int64_t col = (int64_t)b * S + s;
        own.load(perm + col * R, ws + col * R, cnt + col * T, T);
        load_sorted_rows<Th, KB, RPT>(hv, h, ((int64_t)b * R * S + s) * K, hstride, k0, own);
        const float* gzr = gz + col * T;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int tc = min((int)threadIdx.x + kThreads * i, T - 1);
            g[i] = gzr[tc];
            ct[i] = cnt[col * T + tc];
        }
    };
    if (s_lo < s_hi) prefetch(s_lo);
    for (int s = s_lo; s < s_hi; ++s) {
        const int lim = tail_limit(pp, s);
        lds_barrier();  // the previous sample is done with C
        build_cumsum<Th, KB, RPT>(C, R, own.n, own.spt, own.w, hv, wtotf);
        float gc[NT];
        int cc[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            gc[i] = g[i];
            cc[i] = ct[i];
        }
        if (s + 1 < s_hi) prefetch(s + 1);
        lds_barrier();
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < lim) {
#pragma unroll
                for (int k = 0; k < KB; ++k) acc[i][k] = fmaf(gc[i], C[k * RS + 3 + cc[i]], acc[i][k]);
            }
        }
    }
    float* out = gW_part + ((int64_t)b * gridDim.y + sg) * (int64_t)T * K;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = threadIdx.x + kThreads * i;
        if (t < T) store_block<float, KB>(out + (int64_t)t * K + k0, acc[i]);
    }
}

// out[i] = sum_p part[p][i], fixed order
__global__ __launch_bounds__(256) void sum_parts_kernel(int64_t n, int parts, const float* __restrict__ part,
                                                        float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float s = 0.0f;
    int p = 0;
    for (; p + 4 <= parts; p += 4) {
        const float a = part[(int64_t)p * n + i], b2 = part[(int64_t)(p + 1) * n + i];
        const float c = part[(int64_t)(p + 2) * n + i], d = part[(int64_t)(p + 3) * n + i];
        s += a;
        s += b2;
        s += c;
        s += d;
    }
    for (; p < parts; ++p) s += part[(int64_t)p * n + i];
    out[i] = s;
}

// ----------------------------------------------------------- launch shapes
struct HeadShape {
    int rpt;            // rays per thread (4, 8 or 16)
    int nt;             // t slots per thread (4, 8 or 16)
    int kb;             // features per block (4, 8 or 16)
    int n_kg;           // forward feature groups = DFT partials (power of two <= 16)
    int kg;             // features per group
    size_t lds_q;       // head_bwd_h: Q[kb][q_stride(T)]
    size_t lds_c;       // head_fwd / head_bwd_w: C[kb][R+1]
    size_t lds_sort;    // head_sort: cnt[T], wr[R], keys[pow2_ceil(R)]
};

int head_shape(const avr_render_params& p, int B, int R, int K, int es, HeadShape* hs) {
    const int T = p.T, S = p.n_samples;
    if (T > kThreads * 16) return fail(AVR_E_CONFIG, "fused head: T > 4096 not supported");
    if (R > kThreads * 16) return fail(AVR_E_CONFIG, "fused head: more than 4096 rays per shard");
    const int nt = T <= 1024 ? 4 : (T <= 2048 ? 8 : 16);
    // feature block: prefetched W rows in registers (kb*nt <= 64), the
    // backward's Q[kb][T] in <= 80 KiB of LDS (two workgroups per CU), and
    // the cumulative sums C[kb][R] within the 150 KiB budget (many rays)
    int kb = 16;
    while (kb > 4 && ((size_t)kb * q_stride(T) * 4 > 80 * 1024 || kb * nt > 64 ||
                      cumsum_lds_bytes(R, kb) > 150 * 1024))
        kb /= 2;
    const size_t lds_sort = 4 * ((size_t)T + (size_t)R + (size_t)pow2_ceil(R) + 4);
    if ((size_t)kb * q_stride(T) * 4 > 150 * 1024 || cumsum_lds_bytes(R, kb) > 150 * 1024 ||
        lds_sort > 150 * 1024)
        return fail(AVR_E_CONFIG, "fused head: T x rays too large for LDS");
    if (K % kb != 0 || (kb * es) % 8 != 0)
        return fail(AVR_E_CONFIG, "fused head: hidden width must be a multiple of the feature block");
    int n = 1;
    const int64_t cols = (int64_t)B * S;
    while (n < 16 && cols * n < 1024 && (K / (2 * n)) % kb == 0 && K % (2 * n) == 0) n *= 2;
    hs->rpt = R <= 4 * kThreads ? 4 : (R <= 8 * kThreads ? 8 : 16);
    hs->nt = nt;
    hs->kb = kb;
    hs->n_kg = n;
    hs->kg = K / n;
    hs->lds_q = (size_t)kb * q_stride(T) * 4;
    hs->lds_c = cumsum_lds_bytes(R, kb);
    hs->lds_sort = lds_sort;
    return 0;
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

int elem_size(int dtype) { return dtype == AVR_DTYPE_F32 ? 4 : 2; }

int head_check(const avr_render_params* p, int B, int K, const void* h, const void* W, int dtype) {
    AVR_REQUIRE(p && B >= 1 && K >= 4 && h && W, "fused head: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F32 || dtype == AVR_DTYPE_BF16 || dtype == AVR_DTYPE_F16,
                "fused head: h/W must be fp32, bf16 or fp16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0,
                "fused head: h and W must be 16-byte aligned");
    return 0;
}

// dW workgroups: (feature block, sample group, b), ~1024 of them
#ifndef AVR_HEAD_DW_TARGET
#define AVR_HEAD_DW_TARGET 512  // head_bwd_w workgroups aimed for (1024: 4 us slower per config-3 step, plus 3 us of partial sums)
#endif
void dw_groups(const HeadShape& hs, int B, int S, int K, int* n_sg, int* s_per) {
    const int nkb = K / hs.kb;
    int n = 1;
    while (n < S && (int64_t)nkb * n * B < AVR_HEAD_DW_TARGET) n *= 2;
    *s_per = (S + n - 1) / n;
    *n_sg = (S + *s_per - 1) / *s_per;
}

// Forward-only block shape for 16-bit h (tools/probe_head.py sweep, MI355X):
// feature blocks of <= 8 (C[kb][RS] of 33 KB: 4 workgroups per CU instead of
// 2) and SB blocks per row load (4 while the t slots leave the registers:
// NT <= 4, else 2): config 2 0.36 -> 0.24 ms, config 3 0.17 -> 0.16 ms for
// the render with the head.
void fwd_block(const HeadShape& hs, int dtype, int* kb, int* sb) {
    int kbf = hs.kb, s = 1;
    if (elem_size(dtype) == 2 && hs.rpt <= 8) {
        kbf = hs.kb > 8 ? 8 : hs.kb;
        s = hs.nt <= 4 ? 4 : 2;
        if (hs.kg % (s * kbf) != 0) s = 1;
    }
    *kb = kbf;
    *sb = s;
}

}  // namespace

extern "C" int avr_head_pack_w(const avr_render_params* p, int32_t B, int32_t K, const void* W, int32_t dtype,
                               void* Wp, void* stream) {
    if (int e = head_check(p, B, K, W, W, dtype)) return e;
    AVR_REQUIRE(Wp && reinterpret_cast<uintptr_t>(Wp) % 16 == 0, "avr_head_pack_w: Wp must be 16-byte aligned");
    HeadShape hs;
    if (int e = head_shape(*p, B, n_rays(*p), K, elem_size(dtype), &hs)) return e;
    int kbf, sb;
    fwd_block(hs, dtype, &kbf, &sb);
    const int T = p->T;
    const int64_t n = (int64_t)T * K;
    const int blocks = (int)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096);
    hipStream_t st = as_stream(stream);
    if (dtype == AVR_DTYPE_BF16)
        hipLaunchKernelGGL(head_pack_w_kernel<__hip_bfloat16>, dim3(blocks), dim3(kThreads), 0, st, T, (int)K, kbf,
                           (const __hip_bfloat16*)W, (__hip_bfloat16*)Wp);
    else if (dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(head_pack_w_kernel<__half>, dim3(blocks), dim3(kThreads), 0, st, T, (int)K, kbf,
                           (const __half*)W, (__half*)Wp);
    else
        hipLaunchKernelGGL(head_pack_w_kernel<float>, dim3(blocks), dim3(kThreads), 0, st, T, (int)K, kbf,
                           (const float*)W, (float*)Wp);
    return check_launch("avr_head_pack_w");
}

extern "C" int avr_head_splits(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                               int32_t* n_split) {
    AVR_REQUIRE(p && n_split, "avr_head_splits: bad args");
    HeadShape hs;
    if (int e = head_shape(*p, B, n_rays(*p), K, elem_size(dtype), &hs)) return e;
    *n_split = hs.n_kg;
    return 0;
}

extern "C" int avr_head_sort(const avr_render_params* p, int32_t B, const float* w, const int32_t* delay,
                             int32_t* perm, float* ws, int32_t* cnt, void* stream) {
    AVR_REQUIRE(p && B >= 1 && w && delay && perm && ws && cnt, "avr_head_sort: bad args");
    const int R = n_rays(*p);
    HeadShape hs;
    if (int e = head_shape(*p, B, R, 16, 4, &hs)) return e;
    hipStream_t st = as_stream(stream);
    const dim3 grid(p->n_samples, B);
    auto go = [&](auto kern) {
        allow_lds(kern, hs.lds_sort);
        hipLaunchKernelGGL(kern, grid, dim3(kThreads), hs.lds_sort, st, *p, R, w, delay, perm, ws, cnt);
    };
    if (hs.rpt == 4)
        go(head_sort_kernel<4>);
    else if (hs.rpt == 8)
        go(head_sort_kernel<8>);
    else
        go(head_sort_kernel<16>);
    return check_launch("avr_head_sort");
}

extern "C" int avr_head_fwd(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                            const void* W, int32_t dtype, const int32_t* perm, const float* ws,
                            const int32_t* cnt, int32_t n_split, float* zpart, void* stream) {
    if (int e = head_check(p, B, K, h, W, dtype)) return e;
    AVR_REQUIRE(perm && ws && cnt && zpart, "avr_head_fwd: bad args");
    const int R = n_rays(*p);
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, elem_size(dtype), &hs)) return e;
    hipStream_t st = as_stream(stream);
    int kbf, sb;
    fwd_block(hs, dtype, &kbf, &sb);
    AVR_REQUIRE(n_split == hs.n_kg, "avr_head_fwd: n_split must come from avr_head_splits");
    const dim3 grid(hs.n_kg, p->n_samples, B);
    HeadShape hf = hs;
    hf.kb = kbf;
    hf.lds_c = cumsum_lds_bytes(R, kbf);
    auto go = [&](auto kern, auto hp, auto wp) {
        allow_lds(kern, hf.lds_c);
        hipLaunchKernelGGL(kern, grid, dim3(kThreads), hf.lds_c, st, *p, (int)B, R, (int)K, hf.kg, hp, wp,
                           perm, ws, cnt, zpart);
    };
#define AVR_HF(TH, KBV, NTV, RP)                                                                   \
    if (hf.kb == KBV && hf.nt == NTV && hf.rpt == RP) {                                            \
        constexpr bool kSb = sizeof(TH) == 2 && RP <= 8;                                            \
        if (kSb && sb == 2)                                                                         \
            go(head_fwd_kernel<TH, KBV, NTV, RP, kSb ? 2 : 1>, (const TH*)h, (const TH*)W);         \
        else if (kSb && sb == 4)                                                                    \
            go(head_fwd_kernel<TH, KBV, NTV, RP, kSb ? 4 : 1>, (const TH*)h, (const TH*)W);         \
        else                                                                                        \
            go(head_fwd_kernel<TH, KBV, NTV, RP, 1>, (const TH*)h, (const TH*)W);                   \
    }
#define AVR_HF_R(TH, KBV, NTV) AVR_HF(TH, KBV, NTV, 4) AVR_HF(TH, KBV, NTV, 8) AVR_HF(TH, KBV, NTV, 16)
#define AVR_HF_ALL(TH)                                                                             \
    AVR_HF_R(TH, 4, 4) AVR_HF_R(TH, 4, 8) AVR_HF_R(TH, 4, 16) AVR_HF_R(TH, 8, 4) AVR_HF_R(TH, 8, 8) \
    AVR_HF_R(TH, 16, 4)
    if (dtype == AVR_DTYPE_BF16) {
        AVR_HF_ALL(__hip_bfloat16)
    } else if (dtype == AVR_DTYPE_F16) {
        AVR_HF_ALL(__half)
    } else {
        AVR_HF_ALL(float)
    }
#undef AVR_HF_R
#undef AVR_HF_ALL
#undef AVR_HF
    return check_launch("avr_head_fwd");
}

// the block-sum form of dL/dh (head_bwd_h_blk) serves K % 8 == 0; its dL/dw
// partials are per 128 features, the scan form's per feature group
// (columns B * S are the grids' z dimension)
bool hb_blk_ok(int B, int S, int K) { return K % 8 == 0 && (int64_t)B * S <= 65535; }
int hb_parts(const HeadShape& hs, int B, int S, int K) {
    return hb_blk_ok(B, S, K) ? std::max(hs.n_kg, (K + kHbFeat - 1) / kHbFeat) : hs.n_kg;
}
int64_t hb_sum_floats(int B, int S, int T, int K) {
    return hb_blk_ok(B, S, K) ? (int64_t)B * S * (hb_nblk(T) + 2 * hb_nseg(T)) * K : 0;
}

extern "C" int avr_head_bwd_workspace(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                                      int64_t* bytes) {
    AVR_REQUIRE(p && bytes, "avr_head_bwd_workspace: bad args");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, elem_size(dtype), &hs)) return e;
    int n_sg, s_per;
    dw_groups(hs, B, S, K, &n_sg, &s_per);
    // fp32 partials, then W packed in the backward's feature blocks (16-B
    // aligned), then the block sums of head_bwd_h_blk
    *bytes = ((int64_t)hb_parts(hs, B, S, K) * B * R * S + (int64_t)B * n_sg * T * K) * 4 + 16 +
             (int64_t)T * K * (elem_size(dtype)) + hb_sum_floats(B, S, T, K) * 4 + 16;
    return 0;
}

extern "C" int avr_head_bwd(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                            const void* W, int32_t dtype, const float* w, const int32_t* delay,
                            const int32_t* perm, const float* ws, const int32_t* cnt, const float* gz,
                            void* grad_h, float* grad_w, float* grad_W, float* workspace,
                            int64_t workspace_bytes, void* stream) {
    return avr_head_bwd2(p, B, K, h, W, dtype, w, delay, perm, ws, cnt, gz, 0, grad_h, grad_w, grad_W, workspace,
                         workspace_bytes, stream);
}

extern "C" int avr_head_bwd2(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                             const void* W, int32_t dtype, const float* w, const int32_t* delay,
                             const int32_t* perm, const float* ws, const int32_t* cnt, const float* gz,
                             int32_t relu_mask, void* grad_h, float* grad_w, float* grad_W, float* workspace,
                             int64_t workspace_bytes, void* stream) {
    if (int e = head_check(p, B, K, h, W, dtype)) return e;
    AVR_REQUIRE(relu_mask == 0 || relu_mask == 1, "avr_head_bwd: relu_mask must be 0 or 1");
    AVR_REQUIRE(w && delay && perm && ws && cnt && gz && grad_h && grad_w && grad_W && workspace,
                "avr_head_bwd: bad args");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, elem_size(dtype), &hs)) return e;
    int n_sg, s_per;
    dw_groups(hs, B, S, K, &n_sg, &s_per);
    const bool blk = hb_blk_ok(B, S, K);
    const int n_parts = blk ? (K + kHbFeat - 1) / kHbFeat : hs.n_kg;  // dL/dw partials written
    const int64_t gw_elems = (int64_t)hb_parts(hs, B, S, K) * B * R * S;
    const int64_t gW_elems = (int64_t)B * n_sg * T * K;
    const int64_t es = elem_size(dtype);
    const int64_t sum_floats = hb_sum_floats(B, S, T, K);
    if (workspace_bytes < (gw_elems + gW_elems) * 4 + 16 + (int64_t)T * K * es + sum_floats * 4 + 16)
        return fail(AVR_E_ARG, "avr_head_bwd: workspace too small");
    float* gw_part = workspace;
    float* gW_part = workspace + gw_elems;
    // W [T][K] -> [K/kb][T][kb]: head_bwd_h then reads 1 KB per wave-instruction
    char* wp_raw = reinterpret_cast<char*>(gW_part + gW_elems);
    void* Wb = wp_raw + ((16 - (reinterpret_cast<uintptr_t>(wp_raw) & 15)) & 15);
    // block sums of the block-sum form: L [B*S][nblk][K], segment totals and
    // the later segments' carries [B*S][nseg][K] each
    char* ls_raw = static_cast<char*>(Wb) + (int64_t)T * K * es;
    float* Lsum = reinterpret_cast<float*>(ls_raw + ((16 - (reinterpret_cast<uintptr_t>(ls_raw) & 15)) & 15));
    float* Ssum = Lsum + (int64_t)B * S * hb_nblk(T) * K;
    float* Csum = Ssum + (int64_t)B * S * hb_nseg(T) * K;
    hipStream_t st = as_stream(stream);
    if (!blk) {  // (the scan form's packed W)
        const int64_t n = (int64_t)T * K;
        const int blocks = (int)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096);
        if (dtype == AVR_DTYPE_BF16)
            hipLaunchKernelGGL(head_pack_w_kernel<__hip_bfloat16>, dim3(blocks), dim3(kThreads), 0, st, T,
                               (int)K, hs.kb, (const __hip_bfloat16*)W, (__hip_bfloat16*)Wb);
        else if (dtype == AVR_DTYPE_F16)
            hipLaunchKernelGGL(head_pack_w_kernel<__half>, dim3(blocks), dim3(kThreads), 0, st, T,
                               (int)K, hs.kb, (const __half*)W, (__half*)Wb);
        else
            hipLaunchKernelGGL(head_pack_w_kernel<float>, dim3(blocks), dim3(kThreads), 0, st, T, (int)K, hs.kb,
                               (const float*)W, (float*)Wb);
    }
    // 16-bit h: h loads / grad_h stores 2 feature blocks (32 B) per row
    const int bsb = (elem_size(dtype) == 2 && hs.kg % (2 * hs.kb) == 0) ? 2 : 1;
    auto go_h = [&](auto kern, auto hp, auto wp, auto gp) {
        if (blk) return;  // (the block-sum form below)
        allow_lds(kern, hs.lds_q);
        hipLaunchKernelGGL(kern, dim3(hs.n_kg, S, B), dim3(kThreads), hs.lds_q, st, *p, (int)B, R, (int)K,
                           hs.kg, hp, wp, w, delay, gz, gp, gw_part, (int)relu_mask);
    };
    auto go_w = [&](auto kern, auto hp) {
        allow_lds(kern, hs.lds_c);
        hipLaunchKernelGGL(kern, dim3(K / hs.kb, n_sg, B), dim3(kThreads), hs.lds_c, st, *p, (int)B, R,
                           (int)K, s_per, hp, perm, ws, cnt, gz, gW_part);
    };
#define AVR_HB(TH, KBV, NTV, RP)                                                                   \
    if (hs.kb == KBV && hs.nt == NTV && hs.rpt == RP) {                                            \
        if constexpr (sizeof(TH) == 2 && RP <= 8) {                                                \
            if (bsb == 2)                                                                           \
                go_h(head_bwd_h_kernel<TH, KBV, NTV, RP, 2>, (const TH*)h, (const TH*)Wb, (TH*)grad_h); \
            else                                                                                    \
                go_h(head_bwd_h_kernel<TH, KBV, NTV, RP, 1>, (const TH*)h, (const TH*)Wb, (TH*)grad_h); \
        } else {                                                                                    \
            go_h(head_bwd_h_kernel<TH, KBV, NTV, RP, 1>, (const TH*)h, (const TH*)Wb, (TH*)grad_h);   \
        }                                                                                           \
        go_w(head_bwd_w_kernel<TH, KBV, NTV, RP>, (const TH*)h);                                   \
    }
#define AVR_HB_R(TH, KBV, NTV) AVR_HB(TH, KBV, NTV, 4) AVR_HB(TH, KBV, NTV, 8) AVR_HB(TH, KBV, NTV, 16)
#define AVR_HB_ALL(TH)                                                                             \
    AVR_HB_R(TH, 4, 4) AVR_HB_R(TH, 4, 8) AVR_HB_R(TH, 4, 16) AVR_HB_R(TH, 8, 4) AVR_HB_R(TH, 8, 8) \
    AVR_HB_R(TH, 16, 4)
    if (dtype == AVR_DTYPE_BF16) {
        AVR_HB_ALL(__hip_bfloat16)
    } else if (dtype == AVR_DTYPE_F16) {
        AVR_HB_ALL(__half)
    } else {
        AVR_HB_ALL(float)
    }
#undef AVR_HB_R
#undef AVR_HB_ALL
#undef AVR_HB
    if (int e = check_launch("avr_head_bwd")) return e;
    if (blk) {
        const unsigned nfg = (unsigned)((K + kHbFeat - 1) / kHbFeat);
        const dim3 gs(nfg, (unsigned)hb_nseg(T), (unsigned)(B * S));
        const dim3 gh(nfg, (unsigned)((R + 15) / 16), (unsigned)(B * S));
        const int64_t nck = (int64_t)B * S * K;
#define AVR_HBLK(TH)                                                                                        \
    hipLaunchKernelGGL(head_bwd_suffix_kernel<TH>, gs, dim3(64), 0, st, *p, (int)K, (const TH*)W, gz, Lsum, Ssum); \
    hipLaunchKernelGGL(head_bwd_carry_kernel, dim3((unsigned)((nck + 255) / 256)), dim3(256), 0, st, T, (int)K,   \
                       nck, Ssum, Csum);                                                                     \
    hipLaunchKernelGGL(head_bwd_h_blk_kernel<TH>, gh, dim3(256), 0, st, *p, (int)B, R, (int)K, (const TH*)h,     \
                       (const TH*)W, w, delay, gz, Lsum, Csum, (TH*)grad_h, gw_part, (int)relu_mask);
        if (dtype == AVR_DTYPE_BF16) {
            AVR_HBLK(__hip_bfloat16)
        } else if (dtype == AVR_DTYPE_F16) {
            AVR_HBLK(__half)
        } else {
            AVR_HBLK(float)
        }
#undef AVR_HBLK
        if (int e = check_launch("avr_head_bwd")) return e;
    }
    const int64_t n1 = (int64_t)B * R * S, n2 = (int64_t)T * K;
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st, n1,
                       n_parts, gw_part, grad_w);
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, n2,
                       (int)(B * n_sg), gW_part, grad_W);
    return check_launch("avr_head_bwd_sum");
}
