// Backward of the render hot path (a14): torch autograd through
// renderer.py:86-121 restated as three kernels.
//
//   forward:  out[b,f] = sum_s phase[s,f] * sum_t z[b,s,t] * e^{-2 pi i f t/T}
//             z[b,s,t] = pl[s,t]*tail[s,t] * sum_r w[b,r,s]*[t>=delay]*x[b,r,s,t]
//   dft_phase_bwd:  gz[b,s,t] = pl*tail * dL/dz            (fp32 MFMA GEMM over f)
//   ray_reduce_bwd: dL/dx = w*[t>=delay]*gz ;  dL/dw = sum_t [t>=delay]*gz*x
//   weights_bwd:    adjoint of w = T_s*alpha_s (suffix affine scan) and of
//                   alpha = 1-exp(-attn*dist)
#include "common.h"

using namespace avr;

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

// ----------------------------------------------------- adjoint DFT (MFMA)
// gz[s,t] = sum_f U[s,f]*cos(2pi f t/T) + V[s,f]*sin(2pi f t/T), with
//   U = gr*pc + gi*ps,  V = gr*ps - gi*pc   (g = dL/dout[b,f], ph = phase[s,f])
// v_mfma_f32_16x16x4_f32: lane l feeds A[s=l&15][k=l>>4], B[k=l>>4][t=l&15];
// the 4 k-slots of one instruction are (f, cos), (f, sin), (f+1, cos),
// (f+1, sin).  A tile (U, V for 16 samples x 32 bins) is built in LDS; the
// twiddle is gathered from the T-entry table by (t*f) mod T.
constexpr int kBwdThreads = 256;
constexpr int kFc = 32;  // bins per LDS stage

__global__ __launch_bounds__(kBwdThreads) void dft_phase_bwd_kernel(
    avr_render_params pp, const float2* __restrict__ gout, const float* __restrict__ pl,
    const float2* __restrict__ phase, const float2* __restrict__ twg, float* __restrict__ gz, int B,
    int S, int T) {
    extern __shared__ float2 tw[];         // [T]  (cos, -sin)
    __shared__ float Au[16][kFc + 1];      // U
    __shared__ float Av[16][kFc + 1];      // -V  (pairs with the -sin table entry)
    const int F = T / 2 + 1;
    const int b = blockIdx.z;
    const int s0 = blockIdx.y * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 64 + wave * 16 + (lane & 15);
    const int tm = (t < T) ? t : 0;
    const int kq = lane >> 4;            // 0..3
    const int fo = kq >> 1, comp = kq & 1;
    // staging: thread -> (row = tid / 16, cols 2*(tid % 16) + {0,1}) of the 16 x 32 tile
    const int srow = threadIdx.x >> 4, scol = 2 * (threadIdx.x & 15);
    const int ss = min(s0 + srow, S - 1);
    float2 ph_raw[2], g_raw[2];
    auto issue = [&](int fc) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int f = min(fc + scol + q, F - 1);
            g_raw[q] = gout[(int64_t)b * F + f];
            ph_raw[q] = phase[(int64_t)ss * F + f];
        }
    };
    auto commit = [&](int fc) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const bool ok = (s0 + srow) < S && (fc + scol + q) < F;
            const float2 g = g_raw[q], ph = ph_raw[q];
            Au[srow][scol + q] = ok ? g.x * ph.x + g.y * ph.y : 0.0f;
            Av[srow][scol + q] = ok ? -(g.x * ph.y - g.y * ph.x) : 0.0f;
        }
    };
    issue(0);
    stage_table<kBwdThreads>(tw, twg, T);
    floatx4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const int inc = (int)((2LL * tm) % T);
    for (int fc = 0; fc < F; fc += kFc) {
        __syncthreads();
        commit(fc);
        __syncthreads();
        if (fc + kFc < F) issue(fc + kFc);  // next tile's loads fly under the MFMAs
        int idx = (int)(((int64_t)(fc + fo) * tm) % T);
#pragma unroll 4
        for (int ff = 0; ff < kFc; ff += 2) {
            const int r = lane & 15;
            const float a = comp ? Av[r][ff + fo] : Au[r][ff + fo];
            const float2 c = tw[idx];
            const float bv = comp ? c.y : c.x;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
            idx += inc;
            if (idx >= T) idx -= T;
        }
    }
    // C layout: col t = lane&15, rows s = 4*(lane>>4) + reg.  shift[s]
    // recomputed (renderer.py:79-80, identical to the table); the 4
    // path-loss gathers are issued together.
    float g4[4];
    int sh4[4];
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int s = min(s0 + 4 * kq + reg, S - 1);
        sh4[reg] = receiver_shift(pp, s);
        g4[reg] = pl[sh4[reg] + min(tm, T - 1)];
    }
    if (t < T) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int s = s0 + 4 * kq + reg;
            if (s < S) {
                const float v = (t < T - 1 - sh4[reg]) ? acc[reg] * g4[reg] : 0.0f;
                gz[((int64_t)b * S + s) * T + t] = v;
            }
        }
    }
}

// -------------------------------------------------- ray reduce backward
constexpr int kMaxRbThreads = 1024;
constexpr int kMaxRbRays = 4096;  // G * rays per split

// The forward reduction's twin: one workgroup per (ray split, column group of
// G samples, b) streams the group's contiguous super-rows ray by ray.  Each
// lane keeps gz for its fixed (g, t) chunk slots in registers, reads the
// signal chunk once, writes grad_x = w*[t>=delay]*gz with 16-byte stores
// (masked scalar stores only where a chunk leaves the super-row) and adds
// its share of grad_w = sum_t [t>=delay]*gz*x, reduced per ray by a wave
// shuffle tree and one LDS atomic per wave.  Four rays' loads are issued
// before any of them is consumed.
template <typename Tin, bool VECTOR, int CPT, int G, int MAXT, bool NTS>
__global__ __launch_bounds__(MAXT) void ray_reduce_bwd_kernel(
    avr_render_params pp, const Tin* __restrict__ sig, const float* __restrict__ gz, const float* __restrict__ w,
    const int32_t* __restrict__ delay, Tin* __restrict__ gsig, float* __restrict__ gw, int B,
    int R, int S, int T, int rays_per_split, int64_t total) {
    constexpr int VEC = VECTOR ? Vec16<Tin>::N : 1;
    extern __shared__ float lds_rb[];  // w_l[G][nr], d_l[G][nr], dot_l[G][nr]
    const int nthreads = blockDim.x, lane = threadIdx.x & 63;
    const int split = blockIdx.x, s0 = blockIdx.y * G, b = blockIdx.z;
    const int gcount = min(G, S - s0);
    const int r0 = split * rays_per_split;
    const int nr = max(0, min(R, r0 + rays_per_split) - r0);
    const int stride_l = G * max(nr, 1);
    float* w_l = lds_rb;
    int* d_l = reinterpret_cast<int*>(lds_rb + stride_l);
    float* dot_l = lds_rb + 2 * stride_l;
    for (int i = threadIdx.x; i < G * nr; i += nthreads) {
        const int g = i / nr, rr = i - g * nr;
        dot_l[i] = 0.0f;
        if (g < gcount) {
            const int64_t idx = ((int64_t)b * R + r0 + rr) * S + s0 + g;
            w_l[i] = w[idx];
            d_l[i] = delay[idx];
        } else {
            w_l[i] = 0.0f;
            d_l[i] = 0x7fffffff;
        }
    }
    const int64_t row0 = (((int64_t)b * R + r0) * S + s0) * (int64_t)T;
    const int L = gcount * T;
    const int phase = (int)(row0 % VEC);
    const int nchunks = (L + phase + VEC - 1) / VEC;
    const int64_t row_stride = (int64_t)S * T;

    float gv[CPT][VEC];
    int tk[CPT][VEC];  // t of each slot (-1: outside the super-row)
    int tm[CPT][VEC];  // t if inside the tail window t < T-1-shift[s], else -1
    int gk[CPT][VEC];
    int tmax[CPT][G];  // per chunk and column: largest tm (-1: no live slot)
    int lim[G];
    bool full[CPT];  // chunk lies inside the super-row: vector store allowed
    const float* gzc = gz + ((int64_t)b * S + s0) * T;  // gz rows of the group are contiguous
#pragma unroll
    for (int g = 0; g < G; ++g) lim[g] = tail_limit(pp, min(s0 + g, S - 1));
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int j = threadIdx.x + c * nthreads;
        const int ebase = j * VEC - phase;
        full[c] = j < nchunks && ebase >= 0 && ebase + VEC <= L;
#pragma unroll
        for (int g = 0; g < G; ++g) tmax[c][g] = -1;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int e = ebase + k;
            const bool ok = j < nchunks && e >= 0 && e < L;
            const int g = (G == 1) ? 0 : (ok ? e / T : 0);
            gk[c][k] = g;
            tk[c][k] = ok ? e - g * T : -1;
            gv[c][k] = ok ? gzc[e] : 0.0f;
            int l = lim[0];
#pragma unroll
            for (int q = 1; q < G; ++q)
                if (g == q) l = lim[q];
            tm[c][k] = (tk[c][k] >= 0 && tk[c][k] < l) ? tk[c][k] : -1;
#pragma unroll
            for (int q = 0; q < G; ++q)
                if (g == q) tmax[c][q] = max(tmax[c][q], tm[c][k]);
        }
    }
    __syncthreads();

    // chunk c of ray r is live if any slot t satisfies delay <= t < T-1-shift;
    // a dead chunk's signal is not needed (its grad_x is 0, its grad_w term 0)
    auto live = [&](int r, int c) {
        bool any = false;
#pragma unroll
        for (int g = 0; g < G; ++g) any |= tmax[c][g] >= d_l[g * nr + r];
        return any;
    };
    auto load_chunk = [&](int64_t rowbase, int c, bool need, float* x) {
        const int j = threadIdx.x + c * nthreads;
        if constexpr (VECTOR) {
            // S*T % VEC == 0 (host check), rowbase VEC-aligned: chunks lie
            // inside the tensor; dead chunks / spare lanes read zeros for free
            load16_masked(sig + rowbase, (uint32_t)nchunks * 16u,
                          need ? (uint32_t)j * 16u : kSkip, x);
        } else {
            const int64_t e0 = rowbase + j;
            x[0] = (need && j < nchunks && e0 < total) ? load_f(sig, e0) : 0.0f;
        }
    };
    auto finish = [&](int r, int64_t rowbase, float (*x)[VEC]) {
        float wg[G], dotg[G];
        int dg[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            wg[g] = w_l[g * nr + r];
            dg[g] = d_l[g * nr + r];
            dotg[g] = 0.0f;
        }
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            float o[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                float ws = wg[0];
                int ds = dg[0];
#pragma unroll
                for (int g = 1; g < G; ++g)
                    if (gk[c][k] == g) {
                        ws = wg[g];
                        ds = dg[g];
                    }
                const float gm = (tm[c][k] >= ds) ? gv[c][k] : 0.0f;
                o[k] = ws * gm;
                const float pd = gm * x[c][k];
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (gk[c][k] == g) dotg[g] += pd;
            }
            const int j = threadIdx.x + c * nthreads;
            const int64_t e0 = rowbase + (int64_t)j * VEC;
            if (VECTOR && full[c]) {
                if constexpr (VECTOR) {
                    if constexpr (NTS)
                        store16_nt(gsig + e0, o);
                    else
                        store16(gsig + e0, o);
                }
            } else {
#pragma unroll
                for (int k = 0; k < VEC; ++k)
                    if (tk[c][k] >= 0) store_f(gsig, e0 + k, o[k]);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float v = dotg[g];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (lane == 0) atomicAdd(&dot_l[g * nr + r], v);
        }
    };

    constexpr int U = 4;  // rays in flight per lane
    int r = 0;
    for (; r + U <= nr; r += U) {
        float x[U][CPT][VEC];
        bool need[U][CPT];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < CPT; ++c) need[u][c] = live(r + u, c);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t bu = row0 + (int64_t)(r + u) * row_stride - phase;
#pragma unroll
            for (int c = 0; c < CPT; ++c) load_chunk(bu, c, need[u][c], x[u][c]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) finish(r + u, row0 + (int64_t)(r + u) * row_stride - phase, x[u]);
    }
    for (; r < nr; ++r) {
        float xa[CPT][VEC];
        const int64_t ba = row0 + (int64_t)r * row_stride - phase;
#pragma unroll
        for (int c = 0; c < CPT; ++c) load_chunk(ba, c, live(r, c), xa[c]);
        finish(r, ba, xa);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * nr; i += nthreads) {
        const int g = i / nr, rr = i - g * nr;
        if (g < gcount) gw[((int64_t)b * R + r0 + rr) * S + s0 + g] = dot_l[i];
    }
}

// --------------------------------------------------- weights backward
// Per ray (one wavefront), with f_k = (1-alpha_k)+1e-6, T_s = prod_{k<s} f_k:
//   dL/dalpha_s = T_s * (gw_s - U_s),  U_s = sum_{j>s} gw_j alpha_j prod_{s<k<j} f_k
//   U_{s-1} = gw_s alpha_s + f_s U_s  -> reverse affine scan over lanes
//   dL/dattn_s = dL/dalpha_s * exp(-attn_s*dist_s) * dist_s
template <typename Ta>
__global__ void weights_bwd_kernel(avr_render_params p, int B, const Ta* __restrict__ attn,
                                   const float* __restrict__ d_vals,
                                   const float* __restrict__ grad_w, Ta* __restrict__ grad_attn,
                                   int waves_per_block) {
    extern __shared__ float lds[];
    const int R = n_rays(p), S = p.n_samples;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * waves_per_block + wave;
    const bool active = ray < (int64_t)B * R;
    float* alpha = lds + (int64_t)wave * 4 * S;
    float* gwl = alpha + S;
    float* ex = gwl + S;     // exp(-attn*dist)
    float* dist = ex + S;
    const int64_t base = ray * S;
    if (active) {
        for (int s = lane; s < S; s += 64) {
            const float a = load_f(attn, base + s);
            const float d = d_vals[s];
            const float gap = (s + 1 < S) ? d_vals[s + 1] - d : 1e10f;
            const float e = expf(-a * gap);
            alpha[s] = 1.0f - e;
            ex[s] = e;
            dist[s] = gap;
            gwl[s] = grad_w[base + s];
        }
    }
    __syncthreads();
    if (!active) return;
    const int per = (S + 63) / 64;
    const int s0 = min(S, lane * per), s1 = min(S, s0 + per);
    // forward exclusive transmittance at the chunk start
    float run = 1.0f;
    for (int s = s0; s < s1; ++s) run = run * ((1.0f - alpha[s]) + 1e-6f);
    float incl = run;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float v = __shfl_up(incl, off, 64);
        if (lane >= off) incl = incl * v;
    }
    float trans0 = __shfl_up(incl, 1, 64);
    if (lane == 0) trans0 = 1.0f;
    // chunk composite of u -> a_s + m_s*u over s in [s0, s1), applied from the top
    float ca = 0.0f, cm = 1.0f;
    for (int s = s1 - 1; s >= s0; --s) {
        const float a_s = gwl[s] * alpha[s];
        const float m_s = (1.0f - alpha[s]) + 1e-6f;
        ca = a_s + m_s * ca;
        cm = m_s * cm;
    }
    // suffix composition over lanes: cur = mine o next o ... (shfl_down)
    float qa = ca, qm = cm;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float na = __shfl_down(qa, off, 64);
        const float nm = __shfl_down(qm, off, 64);
        if (lane + off < 64) {
            qa = qa + qm * na;
            qm = qm * nm;
        }
    }
    float q = __shfl_down(qa, 1, 64);  // Q at s1 (value of U_{s1-1})
    if (lane == 63) q = 0.0f;
    // local transmittance for each s needs a forward walk; store per-s T in ex? keep
    // a second pass: walk forward computing T_s, walk backward computing U_s.
    // Use the gwl slot to hold dL/dalpha after the backward walk.
    for (int s = s1 - 1; s >= s0; --s) {
        const float u_s = q;  // U_s
        q = gwl[s] * alpha[s] + ((1.0f - alpha[s]) + 1e-6f) * q;
        gwl[s] = gwl[s] - u_s;  // (gw_s - U_s)
    }
    float tr = trans0;
    for (int s = s0; s < s1; ++s) {
        const float galpha = tr * gwl[s];
        const float gatt = (galpha * ex[s]) * dist[s];
        store_f(grad_attn, base + s, gatt);
        tr = tr * ((1.0f - alpha[s]) + 1e-6f);
    }
}

}  // namespace

// ======================================================================
// C-ABI
// ======================================================================
extern "C" int avr_dft_phase_bwd(const avr_render_params* p, int32_t B, const float* grad_out,
                                 const float* pl_table, const int32_t* shift, const float* phase,
                                 const float* twiddle, float* gz, void* stream) {
    AVR_REQUIRE(p && B >= 1 && grad_out && pl_table && shift && phase && twiddle && gz,
                "avr_dft_phase_bwd: bad args");
    const int S = p->n_samples, T = p->T;
    AVR_REQUIRE(T >= 2 && T <= 16384, "avr_dft_phase_bwd: T out of range");
    const dim3 grid((T + 63) / 64, (S + 15) / 16, B);
    const size_t lds = (size_t)T * sizeof(float2);
    (void)shift;
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)dft_phase_bwd_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dft_phase_bwd_kernel, grid, dim3(kBwdThreads), lds, as_stream(stream), *p,
                       reinterpret_cast<const float2*>(grad_out), pl_table,
                       reinterpret_cast<const float2*>(phase),
                       reinterpret_cast<const float2*>(twiddle), gz, (int)B, S, T);
    return check_launch("avr_dft_phase_bwd");
}

namespace {
template <typename Tin, bool VECTOR>
int launch_rb(const avr_render_params* p, int B, const void* sig, const float* gz, const float* w,
              const int32_t* delay, void* gsig, float* gw, hipStream_t st) {
    constexpr int VEC = VECTOR ? Vec16<Tin>::N : 1;
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    // same super-row shape rule as the forward reduction
    int G = 1;
    const int max_chunks = (VEC == 8) ? 256 : 512;
    while (G < 4 && 2 * G * T <= max_chunks * VEC && 2 * G <= S) G *= 2;
    int max_phase = 0;
    for (int s0 = 0; s0 < S && s0 < VEC * G; s0 += G)
        max_phase = max(max_phase, (int)(((int64_t)s0 * T) % VEC));
    const int nch = (G * T + max_phase + VEC - 1) / VEC;
    int cpt = 1;
    while ((nch + cpt - 1) / cpt > kMaxRbThreads) ++cpt;
    const int threads = max(64, ((nch + cpt - 1) / cpt + 63) / 64 * 64);
    const int groups = (S + G - 1) / G;
    // rays per split within the LDS slab, at least 4 per split
    int n = 1;
    const int64_t wps = (int64_t)groups * B * (threads / 64);
    // no partials in the backward, so splits cost only a gz re-read from L2:
    // take many (best at the 256-split cap, profiles/r01_tune_bwd_*.jsonl)
    const int64_t waves_target = 262144;
    auto rps_of = [&](int k) { return (R + k - 1) / k; };
    while (n < 256 && (n * wps < waves_target || rps_of(n) * G > kMaxRbRays) && rps_of(2 * n) >= 4) n *= 2;
    const int rps = rps_of(n);
    if (rps * G > kMaxRbRays) return fail(AVR_E_CONFIG, "ray_reduce_bwd: too many rays per split");
    const int64_t total = (int64_t)B * R * S * T;
    const dim3 grid((R + rps - 1) / rps, groups, B);
    const size_t lds = (size_t)3 * G * max(rps, 1) * 4;
    const Tin* x = (const Tin*)sig;
    Tin* gx = (Tin*)gsig;
    const bool nts = true;  // streaming grad_x stores (profiles/r01_tune_bwd_*.jsonl)
#define AVR_RB_L(C, GG, MT, NTS)                                                                   \
    hipLaunchKernelGGL((ray_reduce_bwd_kernel<Tin, VECTOR, C, GG, MT, NTS>), grid, dim3(threads),  \
                       lds, st, *p, x, gz, w, delay, gx, gw, B, R, S, T, rps, total)
#define AVR_RB(C, GG)                                                                              \
    if (cpt == C && G == GG) {                                                                     \
        if (threads <= 512) {                                                                      \
            if (nts)                                                                               \
                AVR_RB_L(C, GG, 512, true);                                                        \
            else                                                                                   \
                AVR_RB_L(C, GG, 512, false);                                                       \
        } else {                                                                                   \
            if (nts)                                                                               \
                AVR_RB_L(C, GG, 1024, true);                                                       \
            else                                                                                   \
                AVR_RB_L(C, GG, 1024, false);                                                      \
        }                                                                                          \
        return check_launch("avr_ray_reduce_bwd");                                                 \
    }
    AVR_RB(1, 1) AVR_RB(1, 2) AVR_RB(1, 4) AVR_RB(2, 1) AVR_RB(2, 2) AVR_RB(2, 4) AVR_RB(3, 1)
    AVR_RB(4, 1)
#undef AVR_RB_L
#undef AVR_RB
    return fail(AVR_E_CONFIG, "ray_reduce_bwd: T too long for this build");
}
}  // namespace

extern "C" int avr_ray_reduce_bwd(const avr_render_params* p, int32_t B, const void* signal,
                                  int32_t sig_dtype, const float* gz, const float* w,
                                  const int32_t* delay, void* grad_signal, float* grad_w,
                                  void* stream) {
    AVR_REQUIRE(p && B >= 1 && signal && gz && w && delay && grad_signal && grad_w,
                "avr_ray_reduce_bwd: bad args");
    AVR_REQUIRE(p->T >= 2 && p->T <= 16384, "avr_ray_reduce_bwd: T out of range");
    const int64_t st = (int64_t)p->n_samples * p->T;
    const bool aligned = (reinterpret_cast<uintptr_t>(signal) % 16) == 0 &&
                         (reinterpret_cast<uintptr_t>(grad_signal) % 16) == 0;
    hipStream_t s = as_stream(stream);
    if (sig_dtype == AVR_DTYPE_F32) {
        if (aligned && st % 4 == 0)
            return launch_rb<float, true>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
        return launch_rb<float, false>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
    }
    if (sig_dtype == AVR_DTYPE_F16) {
        if (aligned && st % 8 == 0)
            return launch_rb<__half, true>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
        return launch_rb<__half, false>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
    }
    if (sig_dtype == AVR_DTYPE_BF16) {
        if (aligned && st % 8 == 0)
            return launch_rb<__hip_bfloat16, true>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
        return launch_rb<__hip_bfloat16, false>(p, B, signal, gz, w, delay, grad_signal, grad_w, s);
    }
    return fail(AVR_E_ARG, "avr_ray_reduce_bwd: unknown signal dtype");
}

extern "C" int avr_weights_bwd(const avr_render_params* p, int32_t B, const void* attn,
                               int32_t attn_dtype, const float* d_vals, const float* grad_w,
                               void* grad_attn, void* stream) {
    AVR_REQUIRE(p && B >= 1 && attn && d_vals && grad_w && grad_attn, "avr_weights_bwd: bad args");
    const int S = p->n_samples;
    AVR_REQUIRE(S >= 1 && S <= 8192, "avr_weights_bwd: n_samples out of range");
    const int wpb = (S <= 1024) ? 4 : 1;
    const int64_t rays = (int64_t)B * n_rays(*p);
    const dim3 grid((unsigned)((rays + wpb - 1) / wpb));
    const size_t lds = (size_t)wpb * 4 * S * sizeof(float);
    if (lds > 65536) {
        if (attn_dtype == AVR_DTYPE_F32)
            (void)hipFuncSetAttribute((const void*)weights_bwd_kernel<float>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        else if (attn_dtype == AVR_DTYPE_F16)
            (void)hipFuncSetAttribute((const void*)weights_bwd_kernel<__half>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        else
            (void)hipFuncSetAttribute((const void*)weights_bwd_kernel<__hip_bfloat16>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (attn_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(weights_bwd_kernel<float>, grid, dim3(64 * wpb), lds, as_stream(stream),
                           *p, (int)B, (const float*)attn, d_vals, grad_w, (float*)grad_attn, wpb);
    else if (attn_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(weights_bwd_kernel<__half>, grid, dim3(64 * wpb), lds,
                           as_stream(stream), *p, (int)B, (const __half*)attn, d_vals, grad_w,
                           (__half*)grad_attn, wpb);
    else if (attn_dtype == AVR_DTYPE_BF16)
        hipLaunchKernelGGL(weights_bwd_kernel<__hip_bfloat16>, grid, dim3(64 * wpb), lds,
                           as_stream(stream), *p, (int)B, (const __hip_bfloat16*)attn, d_vals, grad_w,
                           (__hip_bfloat16*)grad_attn, wpb);
    else
        return fail(AVR_E_ARG, "avr_weights_bwd: unknown attn dtype");
    return check_launch("avr_weights_bwd");
}
