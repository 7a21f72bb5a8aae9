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
// samples in registers).  Scatter-adds into LDS are float atomics: the
// summation order, and so the last bits, can vary from run to run.
#include "common.h"

using namespace avr;

namespace {

constexpr int kThreads = 256;

// KB consecutive elements of a row as floats (16-byte aligned when KB*es >= 16)
template <typename Th, int KB>
__device__ __forceinline__ void load_block(const Th* p, float* o) {
    if constexpr (sizeof(Th) == 2) {
        static_assert(KB % 4 == 0, "KB");
        if constexpr (KB >= 8) {
#pragma unroll
            for (int c = 0; c < KB / 8; ++c) {
                const u32x4 v = reinterpret_cast<const u32x4*>(p)[c];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    o[8 * c + 2 * i] = bf16_lo(v[i]);
                    o[8 * c + 2 * i + 1] = bf16_hi(v[i]);
                }
            }
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(p);
            o[0] = bf16_lo(v.x);
            o[1] = bf16_hi(v.x);
            o[2] = bf16_lo(v.y);
            o[3] = bf16_hi(v.y);
        }
    } else {
#pragma unroll
        for (int c = 0; c < KB / 4; ++c) {
            const f32x4 v = reinterpret_cast<const f32x4*>(p)[c];
            o[4 * c] = v[0];
            o[4 * c + 1] = v[1];
            o[4 * c + 2] = v[2];
            o[4 * c + 3] = v[3];
        }
    }
}

template <typename Th, int KB>
__device__ __forceinline__ void store_block(Th* p, const float* v) {
    if constexpr (sizeof(Th) == 2) {
        uint32_t u[KB / 2];
#pragma unroll
        for (int i = 0; i < KB / 2; ++i) {
            const __hip_bfloat16 a = __float2bfloat16(v[2 * i]);
            const __hip_bfloat16 b = __float2bfloat16(v[2 * i + 1]);
            u[i] = (uint32_t)(*reinterpret_cast<const uint16_t*>(&a)) |
                   ((uint32_t)(*reinterpret_cast<const uint16_t*>(&b)) << 16);
        }
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

// In-place inclusive prefix (or suffix) sums of the KB rows of A[KB][T]:
// 256/KB threads per row, each a contiguous segment, segment totals combined
// by a shuffle scan inside the row's lanes (a row's threads share a wave).
template <int KB, bool SUFFIX>
__device__ __forceinline__ void scan_rows(float* A, int T) {
    constexpr int TPR = kThreads / KB;  // 16, 32 or 64 (<= one wave)
    const int row = threadIdx.x / TPR, j = threadIdx.x % TPR;
    const int seg = (T + TPR - 1) / TPR;
    float* a = A + row * T;
    const int lo = j * seg, hi = min(T, lo + seg);
    float run = 0.0f;
    if (!SUFFIX) {
#pragma unroll 8
        for (int t = lo; t < hi; ++t) {
            run += a[t];
            a[t] = run;
        }
    } else {
#pragma unroll 8
        for (int t = hi - 1; t >= lo; --t) {
            run += a[t];
            a[t] = run;
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
#pragma unroll 8
        for (int t = lo; t < hi; ++t) a[t] += off;
    }
}

constexpr int kRB = 4;  // rays per thread per batch: their global loads are issued together

// w / delay of the rays of column (b, s) into LDS
__device__ __forceinline__ void stage_rays(const float* __restrict__ w, const int32_t* __restrict__ delay,
                                           int b, int s, int R, int S, float* wl, int* dl) {
    for (int rb = 0; rb < R; rb += kThreads * kRB) {
        float wv[kRB];
        int dv[kRB];
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
            const int rc = min(rb + (int)threadIdx.x + kThreads * u, R - 1);
            const int64_t i = ((int64_t)b * R + rc) * S + s;
            wv[u] = w[i];
            dv[u] = delay[i];
        }
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
            const int r = rb + threadIdx.x + kThreads * u;
            if (r < R) {
                wl[r] = wv[u];
                dl[r] = dv[u];
            }
        }
    }
}

// A[k][t] = sum_{r: d_r = t < lim} w_r h[r, k0+k]  (LDS float atomics), then
// the inclusive prefix over t.  The kRB rays of a thread are loaded together.
template <typename Th, int KB>
__device__ __forceinline__ void build_prefix(const Th* __restrict__ h, int64_t hrow0, int64_t hstride,
                                             int k0, int R, int lim, const float* wl, const int* dl,
                                             float* A, int T) {
    for (int i = threadIdx.x; i < KB * T; i += kThreads) A[i] = 0.0f;
    __syncthreads();
    for (int rb = 0; rb < R; rb += kThreads * kRB) {
        float v[kRB][KB];
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
            const int rc = min(rb + (int)threadIdx.x + kThreads * u, R - 1);
            load_block<Th, KB>(h + hrow0 + (int64_t)rc * hstride + k0, v[u]);
        }
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
            const int r = rb + threadIdx.x + kThreads * u;
            if (r < R) {
                const int d = dl[r];
                if (d < lim) {
                    const float wr = wl[r];
#pragma unroll
                    for (int k = 0; k < KB; ++k) atomicAdd(&A[k * T + d], wr * v[u][k]);
                }
            }
        }
    }
    __syncthreads();
    scan_rows<KB, false>(A, T);
    __syncthreads();
}

constexpr int kMaxTPer = 16;  // T <= 4096: t slots per thread NT in {4, 8, 16}

// ------------------------------------------------------------------ forward
template <typename Th, int KB, int NT>
__global__ __launch_bounds__(kThreads) void head_fwd_kernel(avr_render_params pp, int B, int R, int K,
                                                            int KG, const Th* __restrict__ h,
                                                            const Th* __restrict__ W,
                                                            const float* __restrict__ w,
                                                            const int32_t* __restrict__ delay,
                                                            float* __restrict__ zpart) {
    extern __shared__ float lds_h[];
    const int T = pp.T, S = pp.n_samples;
    const int kg = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
    float* A = lds_h;                        // [KB][T]
    float* wl = lds_h + KB * T;              // [R]
    int* dl = reinterpret_cast<int*>(wl + R);
    const int lim = tail_limit(pp, s);
    stage_rays(w, delay, b, s, R, S, wl, dl);
    float zacc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) zacc[i] = 0.0f;
    const int64_t hrow0 = ((int64_t)b * R * S + s) * K;
    const int64_t hstride = (int64_t)S * K;
    for (int k0 = kg * KG; k0 < (kg + 1) * KG; k0 += KB) {
        // this block's W rows, in flight while the prefix is built
        float wt[NT][KB];
#pragma unroll
        for (int i = 0; i < NT; ++i)
            load_block<Th, KB>(W + (int64_t)min((int)threadIdx.x + kThreads * i, T - 1) * K + k0, wt[i]);
        __syncthreads();
        build_prefix<Th, KB>(h, hrow0, hstride, k0, R, lim, wl, dl, A, T);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < lim) {
                float a = zacc[i];
#pragma unroll
                for (int k = 0; k < KB; ++k) a = fmaf(wt[i][k], A[k * T + t], a);
                zacc[i] = a;
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
template <typename Th, int KB, int NT>
__global__ __launch_bounds__(kThreads) void head_bwd_h_kernel(avr_render_params pp, int B, int R, int K,
                                                              int KG, const Th* __restrict__ h,
                                                              const Th* __restrict__ W,
                                                              const float* __restrict__ w,
                                                              const int32_t* __restrict__ delay,
                                                              const float* __restrict__ gz,
                                                              Th* __restrict__ grad_h,
                                                              float* __restrict__ gw_part) {
    extern __shared__ float lds_h[];
    const int T = pp.T, S = pp.n_samples;
    const int kg = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
    float* Q = lds_h;                        // [KB][T]
    float* wl = lds_h + KB * T;              // [R]
    int* dl = reinterpret_cast<int*>(wl + R);
    float* gwl = wl + 2 * R;                 // [R] dL/dw partial (each ray owned by one thread)
    const int lim = tail_limit(pp, s);
    stage_rays(w, delay, b, s, R, S, wl, dl);
    for (int r = threadIdx.x; r < R; r += kThreads) gwl[r] = 0.0f;
    const float* gzr = gz + ((int64_t)b * S + s) * T;
    float g[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int t = threadIdx.x + kThreads * i;
        const float v = gzr[min(t, T - 1)];
        g[i] = t < lim ? v : 0.0f;
    }
    const int64_t hrow0 = ((int64_t)b * R * S + s) * K;
    const int64_t hstride = (int64_t)S * K;
    for (int k0 = kg * KG; k0 < (kg + 1) * KG; k0 += KB) {
        float wt[NT][KB];
#pragma unroll
        for (int i = 0; i < NT; ++i)
            load_block<Th, KB>(W + (int64_t)min((int)threadIdx.x + kThreads * i, T - 1) * K + k0, wt[i]);
        __syncthreads();
        // u[k][t] = gz[t] W[t][k], then the suffix sum over t
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < T)
#pragma unroll
                for (int k = 0; k < KB; ++k) Q[k * T + t] = g[i] * wt[i][k];
        }
        __syncthreads();
        scan_rows<KB, true>(Q, T);
        __syncthreads();
        for (int rb = 0; rb < R; rb += kThreads * kRB) {
            float hv[kRB][KB];
#pragma unroll
            for (int u = 0; u < kRB; ++u) {
                const int rc = min(rb + (int)threadIdx.x + kThreads * u, R - 1);
                load_block<Th, KB>(h + hrow0 + (int64_t)rc * hstride + k0, hv[u]);
            }
#pragma unroll
            for (int u = 0; u < kRB; ++u) {
                const int r = rb + threadIdx.x + kThreads * u;
                if (r < R) {
                    const int d = dl[r];
                    float gh[KB];
                    if (d < lim) {
                        const float wr = wl[r];
                        float acc = 0.0f;
#pragma unroll
                        for (int k = 0; k < KB; ++k) {
                            const float q = Q[k * T + d];
                            gh[k] = wr * q;
                            acc = fmaf(hv[u][k], q, acc);
                        }
                        gwl[r] += acc;
                    } else {
#pragma unroll
                        for (int k = 0; k < KB; ++k) gh[k] = 0.0f;
                    }
                    store_block<Th, KB>(grad_h + hrow0 + (int64_t)r * hstride + k0, gh);
                }
            }
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < R; r += kThreads)
        gw_part[(((int64_t)kg * B + b) * R + r) * S + s] = gwl[r];
}

// ---------------------------------------------------- backward: dL/dW
// One workgroup per (feature block, sample group, b): for each of its
// samples, rebuild P (as the forward) and accumulate gz[t] * P[k][t] in
// registers; one [T][KB] partial per workgroup.
template <typename Th, int KB, int NT>
__global__ __launch_bounds__(kThreads) void head_bwd_w_kernel(avr_render_params pp, int B, int R, int K,
                                                              int s_per_group,
                                                              const Th* __restrict__ h,
                                                              const float* __restrict__ w,
                                                              const int32_t* __restrict__ delay,
                                                              const float* __restrict__ gz,
                                                              float* __restrict__ gW_part) {
    extern __shared__ float lds_h[];
    const int T = pp.T, S = pp.n_samples;
    const int kb = blockIdx.x, sg = blockIdx.y, b = blockIdx.z;
    const int k0 = kb * KB;
    float* A = lds_h;
    float* wl = lds_h + KB * T;
    int* dl = reinterpret_cast<int*>(wl + R);
    float acc[NT][KB];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int k = 0; k < KB; ++k) acc[i][k] = 0.0f;
    const int s_lo = sg * s_per_group, s_hi = min(S, s_lo + s_per_group);
    for (int s = s_lo; s < s_hi; ++s) {
        const int lim = tail_limit(pp, s);
        const float* gzr = gz + ((int64_t)b * S + s) * T;
        float g[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) g[i] = gzr[min((int)threadIdx.x + kThreads * i, T - 1)];
        __syncthreads();
        stage_rays(w, delay, b, s, R, S, wl, dl);
        __syncthreads();
        build_prefix<Th, KB>(h, ((int64_t)b * R * S + s) * K, (int64_t)S * K, k0, R, lim, wl, dl, A, T);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int t = threadIdx.x + kThreads * i;
            if (t < lim) {
#pragma unroll
                for (int k = 0; k < KB; ++k) acc[i][k] = fmaf(g[i], A[k * T + t], acc[i][k]);
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
    int nt;      // t slots per thread (4, 8 or 16)
    int kb;      // features per LDS block (4, 8 or 16)
    int n_kg;    // feature groups = DFT partials (power of two <= 16)
    int kg;      // features per group
    size_t lds;  // bytes
};

int head_shape(const avr_render_params& p, int B, int R, int K, int es, HeadShape* hs) {
    const int T = p.T, S = p.n_samples;
    if (T > kThreads * kMaxTPer) return fail(AVR_E_CONFIG, "fused head: T > 4096 not supported");
    if (R > kThreads * 16) return fail(AVR_E_CONFIG, "fused head: more than 4096 rays per shard");
    const size_t ray_bytes = (size_t)R * 12;  // w, delay (+ dL/dw in the backward)
    int kb = 16;
    // two workgroups per CU when the block fits 80 KiB; 16-byte row loads
    const int nt = T <= 1024 ? 4 : (T <= 2048 ? 8 : 16);
    while (kb > 4 && ((size_t)kb * T * 4 + ray_bytes > 80 * 1024 || kb * nt > 64)) kb /= 2;
    if ((size_t)kb * T * 4 + ray_bytes > 150 * 1024)
        return fail(AVR_E_CONFIG, "fused head: T x rays too large for LDS");
    if (K % kb != 0 || (kb * es) % 8 != 0)
        return fail(AVR_E_CONFIG, "fused head: hidden width must be a multiple of the feature block");
    int n = 1;
    const int64_t cols = (int64_t)B * S;
    while (n < 16 && cols * n < 1024 && (K / (2 * n)) % kb == 0 && K % (2 * n) == 0) n *= 2;
    hs->nt = nt;
    hs->kb = kb;
    hs->n_kg = n;
    hs->kg = K / n;
    hs->lds = (size_t)kb * T * 4 + ray_bytes;
    return 0;
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

int head_check(const avr_render_params* p, int B, int K, const void* h, const void* W, int dtype) {
    AVR_REQUIRE(p && B >= 1 && K >= 4 && h && W, "fused head: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F32 || dtype == AVR_DTYPE_BF16,
                "fused head: h/W must be fp32 or bf16");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 && reinterpret_cast<uintptr_t>(W) % 16 == 0,
                "fused head: h and W must be 16-byte aligned");
    return 0;
}

}  // namespace

extern "C" int avr_head_splits(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                               int32_t* n_split) {
    AVR_REQUIRE(p && n_split, "avr_head_splits: bad args");
    HeadShape hs;
    const int es = dtype == AVR_DTYPE_BF16 ? 2 : 4;
    if (int e = head_shape(*p, B, n_rays(*p), K, es, &hs)) return e;
    *n_split = hs.n_kg;
    return 0;
}

extern "C" int avr_head_fwd(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                            const void* W, int32_t dtype, const float* w, const int32_t* delay,
                            int32_t n_split, float* zpart, void* stream) {
    if (int e = head_check(p, B, K, h, W, dtype)) return e;
    AVR_REQUIRE(w && delay && zpart, "avr_head_fwd: bad args");
    const int R = n_rays(*p);
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, dtype == AVR_DTYPE_BF16 ? 2 : 4, &hs)) return e;
    AVR_REQUIRE(n_split == hs.n_kg, "avr_head_fwd: n_split must come from avr_head_splits");
    const dim3 grid(hs.n_kg, p->n_samples, B);
    hipStream_t st = as_stream(stream);
    auto go = [&](auto kern, auto hp, auto wp) {
        allow_lds(kern, hs.lds);
        hipLaunchKernelGGL(kern, grid, dim3(kThreads), hs.lds, st, *p, (int)B, R, (int)K, hs.kg, hp, wp, w,
                           delay, zpart);
    };
#define AVR_HF(TH, KBV, NTV)                                                                       \
    if (hs.kb == KBV && hs.nt == NTV) go(head_fwd_kernel<TH, KBV, NTV>, (const TH*)h, (const TH*)W);
#define AVR_HF_ALL(TH)                                                                             \
    AVR_HF(TH, 4, 4) AVR_HF(TH, 4, 8) AVR_HF(TH, 4, 16) AVR_HF(TH, 8, 4) AVR_HF(TH, 8, 8)          \
    AVR_HF(TH, 16, 4)
    if (dtype == AVR_DTYPE_BF16) {
        AVR_HF_ALL(__hip_bfloat16)
    } else {
        AVR_HF_ALL(float)
    }
#undef AVR_HF_ALL
#undef AVR_HF
    return check_launch("avr_head_fwd");
}

extern "C" int avr_head_bwd(const avr_render_params* p, int32_t B, int32_t K, const void* h,
                            const void* W, int32_t dtype, const float* w, const int32_t* delay,
                            const float* gz, void* grad_h, float* grad_w, float* grad_W,
                            float* workspace, int64_t workspace_bytes, void* stream) {
    if (int e = head_check(p, B, K, h, W, dtype)) return e;
    AVR_REQUIRE(w && delay && gz && grad_h && grad_w && grad_W && workspace, "avr_head_bwd: bad args");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, dtype == AVR_DTYPE_BF16 ? 2 : 4, &hs)) return e;
    // dW: (feature block, sample group, b) workgroups, ~1024 of them
    const int nkb = K / hs.kb;
    int n_sg = 1;
    while (n_sg < S && (int64_t)nkb * n_sg * B < 1024) n_sg *= 2;
    const int s_per = (S + n_sg - 1) / n_sg;
    n_sg = (S + s_per - 1) / s_per;
    int64_t need = 0;
    AVR_REQUIRE(workspace_bytes >= 0, "avr_head_bwd: bad workspace size");
    const int64_t gw_elems = (int64_t)hs.n_kg * B * R * S;
    const int64_t gW_elems = (int64_t)B * n_sg * T * K;
    need = (gw_elems + gW_elems) * 4;
    if (workspace_bytes < need) return fail(AVR_E_ARG, "avr_head_bwd: workspace too small");
    float* gw_part = workspace;
    float* gW_part = workspace + gw_elems;
    hipStream_t st = as_stream(stream);
    auto go_h = [&](auto kern, auto hp, auto wp, auto gp) {
        const size_t lds_h = hs.lds + (size_t)R * 4;  // + the per-ray dL/dw accumulators
        allow_lds(kern, lds_h);
        hipLaunchKernelGGL(kern, dim3(hs.n_kg, S, B), dim3(kThreads), lds_h, st, *p, (int)B, R, (int)K,
                           hs.kg, hp, wp, w, delay, gz, gp, gw_part);
    };
    auto go_w = [&](auto kern, auto hp) {
        allow_lds(kern, hs.lds);
        hipLaunchKernelGGL(kern, dim3(nkb, n_sg, B), dim3(kThreads), hs.lds, st, *p, (int)B, R, (int)K,
                           s_per, hp, w, delay, gz, gW_part);
    };
#define AVR_HB(TH, KBV, NTV)                                                                       \
    if (hs.kb == KBV && hs.nt == NTV) {                                                            \
        go_h(head_bwd_h_kernel<TH, KBV, NTV>, (const TH*)h, (const TH*)W, (TH*)grad_h);            \
        go_w(head_bwd_w_kernel<TH, KBV, NTV>, (const TH*)h);                                       \
    }
#define AVR_HB_ALL(TH)                                                                             \
    AVR_HB(TH, 4, 4) AVR_HB(TH, 4, 8) AVR_HB(TH, 4, 16) AVR_HB(TH, 8, 4) AVR_HB(TH, 8, 8)          \
    AVR_HB(TH, 16, 4)
    if (dtype == AVR_DTYPE_BF16) {
        AVR_HB_ALL(__hip_bfloat16)
    } else {
        AVR_HB_ALL(float)
    }
#undef AVR_HB_ALL
#undef AVR_HB
    if (int e = check_launch("avr_head_bwd")) return e;
    const int64_t n1 = (int64_t)B * R * S, n2 = (int64_t)T * K;
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st, n1,
                       hs.n_kg, gw_part, grad_w);
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, n2,
                       (int)(B * n_sg), gW_part, grad_W);
    return check_launch("avr_head_bwd_sum");
}

extern "C" int avr_head_bwd_workspace(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                                      int64_t* bytes) {
    AVR_REQUIRE(p && bytes, "avr_head_bwd_workspace: bad args");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    HeadShape hs;
    if (int e = head_shape(*p, B, R, K, dtype == AVR_DTYPE_BF16 ? 2 : 4, &hs)) return e;
    const int nkb = K / hs.kb;
    int n_sg = 1;
    while (n_sg < S && (int64_t)nkb * n_sg * B < 1024) n_sg *= 2;
    const int s_per = (S + n_sg - 1) / n_sg;
    n_sg = (S + s_per - 1) / s_per;
    *bytes = ((int64_t)hs.n_kg * B * R * S + (int64_t)B * n_sg * T * K) * 4;
    return 0;
}
