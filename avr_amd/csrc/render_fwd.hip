// Forward render hot path for MI355X (gfx950): tables, ray generation,
// network-input sampling, compositing weights, the HBM ray-reduction stream,
// the fp32-MFMA DFT with fused phase epilogue, and the irfft to the IR.
//
// Reference: renderer.py:31-193 (AVRRender.forward, ray_directions,
// acoustic_render) and utils/criterion.py:71 (irfft).  See DESIGN.md for the
// reordering (sum over rays in the time domain before the transform) and the
// roofline of each kernel.
#include "common.h"

#include <cstdlib>

using namespace avr;

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr double kTwoPi = 6.283185307179586476925286766559;

// ------------------------------------------------------------------ tables
// d_vals/frac/shift: renderer.py:54, 79-80.  Path loss: renderer.py:95-98
// (arange/fs*speed + 1e-3, then pathloss * reciprocal, the near-field entries
// copied from index near_clamp+1).  Phase: renderer.py:108, theta =
// fp32(fp32(c*f)*frac[s]), exp(i*theta).  Twiddles in double, rounded once.
__global__ void tables_kernel(avr_render_params p, float* __restrict__ d_vals,
                              float* __restrict__ frac, int32_t* __restrict__ shift,
                              float* __restrict__ pl, float2* __restrict__ phase,
                              float2* __restrict__ tw) {
    const int S = p.n_samples, T = p.T, F = T / 2 + 1;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = gid; i < S; i += stride) {
        const float d = linspace_at(0.0f, 1.0f, S, (int)i) * p.depth_scale + p.depth_offset;
        const float fr = (p.fs * d) / p.speed;
        d_vals[i] = d;
        frac[i] = fr;
        shift[i] = (int32_t)rintf(fr);
    }
    for (int64_t i = gid; i < p.pl_len; i += stride) {
        const int k = (i < p.near_clamp) ? p.near_clamp + 1 : (int)i;
        const float dist = ((float)k / p.fs) * p.speed;
        const float den = dist + 1e-3f;
        pl[i] = p.pathloss * (1.0f / den);
    }
    for (int64_t i = gid; i < (int64_t)S * F; i += stride) {
        const int s = (int)(i / F), f = (int)(i % F);
        const float d = linspace_at(0.0f, 1.0f, S, s) * p.depth_scale + p.depth_offset;
        const float fr = (p.fs * d) / p.speed;
        const float cf = p.phase_c * (float)f;
        const float th = cf * fr;
        phase[i] = make_float2((float)cos((double)th), (float)sin((double)th));
    }
    for (int64_t k = gid; k < T; k += stride) {
        const double a = kTwoPi * (double)k / (double)T;
        tw[k] = make_float2((float)cos(a), (float)(-sin(a)));
    }
}

__global__ void depth_samples_kernel(avr_render_params p, float* __restrict__ d_vals) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < p.n_samples)
        d_vals[s] = linspace_at(0.0f, 1.0f, p.n_samples, s) * p.depth_scale + p.depth_offset;
}

__global__ void ir_twiddle_kernel(int n, float2* __restrict__ tw) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const double a = kTwoPi * (double)k / (double)n;
        tw[k] = make_float2((float)cos(a), (float)sin(a));
    }
}

// ------------------------------------------------------------- a2: rays
// renderer.py:147-165: azimuth linspace + jitter, elevation acos ring,
// meshgrid(ij) azimuth-major, then the two poles.  Trig in double, rounded
// once (the reference uses SLEEF u10; components may differ by 1 ulp).
__device__ __forceinline__ void ray_direction(const avr_render_params& p, float u, int r,
                                              float* out) {
    const int grid = p.n_azi * p.n_ele;
    if (r < grid) {
        const int ia = r / p.n_ele, ie = r % p.n_ele;
        const float base = linspace_at(0.0f, p.two_pi, p.n_azi + 1, ia);
        const float jit = p.azi_jitter * u;
        const float azi = base + jit;
        const float el_lin = linspace_at(0.0f, 1.0f, p.n_ele + 2, ie + 1);
        const float el_arg = 2.0f * el_lin - 1.0f;
        const float ele = (float)acos((double)el_arg);
        const float se = (float)sin((double)ele);
        out[0] = (float)cos((double)azi) * se;
        out[1] = (float)sin((double)azi) * se;
        out[2] = (float)cos((double)ele);
    } else {
        out[0] = 0.0f;
        out[1] = 0.0f;
        out[2] = (r == grid) ? 1.0f : -1.0f;
    }
}

__global__ void ray_directions_kernel(avr_render_params p, const float* __restrict__ u_azi,
                                      float* __restrict__ dirs) {
    const int R = grid_rays(p);
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    float d[3];
    ray_direction(p, r < p.n_azi * p.n_ele ? u_azi[r / p.n_ele] : 0.0f, r, d);
    dirs[r * 3 + 0] = d[0];
    dirs[r * 3 + 1] = d[1];
    dirs[r * 3 + 2] = d[2];
}

// ------------------------------------------------- a3/a4: network inputs
// renderer.py:54-62: pts = norm(o + dir*d), view = -dir, tx = norm(tx),
// dir_tx broadcast.  One thread per ray-sample, [B][R*S][3] outputs.
__global__ void sample_points_kernel(avr_render_params p, int B, const float* __restrict__ rays_o,
                                     const float* __restrict__ pos_tx,
                                     const float* __restrict__ dir_tx,
                                     const float* __restrict__ dirs,
                                     const float* __restrict__ d_vals, float* __restrict__ net_pts,
                                     float* __restrict__ net_view, float* __restrict__ net_tx,
                                     float* __restrict__ net_dir_tx) {
    const int R = n_rays(p), S = p.n_samples;
    const int64_t n = (int64_t)B * R * S;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)(i % S);
        const int64_t br = i / S;
        const int r = (int)(br % R);
        const int b = (int)(br / R);
        const float d = d_vals[s];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float dc = dirs[r * 3 + c];
            const float world = rays_o[b * 3 + c] + dc * d;
            net_pts[i * 3 + c] = to_unit(world, p.lo, p.span);
            net_view[i * 3 + c] = -dc;
            net_tx[i * 3 + c] = to_unit(pos_tx[b * 3 + c], p.lo, p.span);
            if (dir_tx) net_dir_tx[i * 3 + c] = dir_tx[b * 3 + c];
        }
    }
}

// Fused a2+a3+a4 for the hot path: the azimuth jitter arrives by value in the
// kernel arguments (no host->device copy), every wave derives its ray's
// direction and depth itself, and the shard's directions are written once
// for the weights kernel.  One launch instead of three plus a copy.
struct AziJitter {
    float u[AVR_MAX_AZI];
};

constexpr int kSampleThreads = 256;

__global__ __launch_bounds__(kSampleThreads) void sample_rays_kernel(
    avr_render_params p, int B, AziJitter jit, const float* __restrict__ jit_dev, int r_begin,
    const float* __restrict__ rays_o, const float* __restrict__ pos_tx, const float* __restrict__ dir_tx,
    float* __restrict__ dirs, float* __restrict__ net_pts, float* __restrict__ net_view,
    float* __restrict__ net_tx, float* __restrict__ net_dir_tx, float* __restrict__ pose_out) {
    if (pose_out && blockIdx.x == 0) {  // staged pose -> device copy for the later kernels
        for (int i = threadIdx.x; i < 3 * B; i += kSampleThreads) {
            pose_out[i] = rays_o[i];
            pose_out[3 * B + i] = pos_tx[i];
            if (dir_tx) pose_out[6 * B + i] = dir_tx[i];
        }
    }
    // directions of the (at most 256/S + 2) rays this block touches, once each
    __shared__ float sdir[kSampleThreads + 1][3];
    const int R = n_rays(p), S = p.n_samples;
    const int64_t n = (int64_t)B * R * S;
    const int64_t i0 = (int64_t)blockIdx.x * kSampleThreads;
    const int64_t br0 = i0 / S;
    const int64_t br1 = (min(n, i0 + kSampleThreads) - 1) / S;
    for (int k = threadIdx.x; k <= (int)(br1 - br0); k += kSampleThreads) {
        const int r = r_begin + (int)((br0 + k) % R);
        const float u = r < p.n_azi * p.n_ele ? (jit_dev ? jit_dev[r / p.n_ele] : jit.u[r / p.n_ele]) : 0.0f;
        ray_direction(p, u, r, sdir[k]);
    }
    // the poses of the (at most 256/(R*S) + 2) listeners this block touches,
    // read once per block (a staged pose lives in host memory: one bus read
    // per block, not per sample)
    __shared__ float spose[kSampleThreads + 1][9];
    const int64_t b0 = br0 / R, b1 = br1 / R;
    for (int k = threadIdx.x; k <= (int)(b1 - b0); k += kSampleThreads) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            spose[k][c] = rays_o[(b0 + k) * 3 + c];
            spose[k][3 + c] = pos_tx[(b0 + k) * 3 + c];
            spose[k][6 + c] = dir_tx ? dir_tx[(b0 + k) * 3 + c] : 0.0f;
        }
    }
    __syncthreads();
    // stage the block's 256 x 3 outputs per tensor in LDS, then write them
    // as coalesced 4-byte rows (one 1 KiB wave store instead of 12-byte strides)
    __shared__ float obuf[4][kSampleThreads * 3];
    const int64_t i = i0 + threadIdx.x;
    const bool live = i < n;
    if (live) {
        const int s = (int)(i % S);
        const int64_t br = i / S;
        const int rl = (int)(br % R);
        const int b = (int)(br / R);
        const float* dir = sdir[br - br0];
        const float* pose = spose[b - b0];
        const float d = linspace_at(0.0f, 1.0f, S, s) * p.depth_scale + p.depth_offset;
        if (b == 0 && s == 0) {
            dirs[rl * 3 + 0] = dir[0];
            dirs[rl * 3 + 1] = dir[1];
            dirs[rl * 3 + 2] = dir[2];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float world = pose[c] + dir[c] * d;
            obuf[0][threadIdx.x * 3 + c] = to_unit(world, p.lo, p.span);
            obuf[1][threadIdx.x * 3 + c] = -dir[c];
            obuf[2][threadIdx.x * 3 + c] = to_unit(pose[3 + c], p.lo, p.span);
            obuf[3][threadIdx.x * 3 + c] = pose[6 + c];
        }
    }
    __syncthreads();
    const int64_t lim = (n - i0) * 3;  // valid floats in this block
    float* outs[4] = {net_pts, net_view, net_tx, net_dir_tx};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q == 3 && !dir_tx) break;
        float* o = outs[q] + i0 * 3;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int e = threadIdx.x + k * kSampleThreads;
            if (e < lim) o[e] = obuf[q][e];
        }
    }
}

// ------------------------------------- a8 + a11: delays and the weights
// One ray per wavefront; samples strided over the 64 lanes for coalesced
// attn loads, alpha staged in LDS, then each lane owns a contiguous run of
// samples for the exclusive transmittance product (renderer.py:185-192):
//   alpha = 1 - exp(-attn*dist), dist = d[s+1]-d[s] (last 1e10)
//   T_s = prod_{k<s} ((1-alpha_k) + 1e-6), w = T_s * alpha_s
// The cross-lane part is a multiplicative shuffle scan (6 steps).
template <typename Ta>
__global__ __launch_bounds__(256) void weights_fwd_kernel(
    avr_render_params p, int B, const Ta* __restrict__ attn, const float* __restrict__ rays_o,
    const float* __restrict__ pos_tx, const float* __restrict__ dirs,
    const float* __restrict__ d_vals, float* __restrict__ w_out, int32_t* __restrict__ delay) {
    extern __shared__ float lds_alpha[];
    const int R = n_rays(p), S = p.n_samples;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wave;  // flattened (b, r)
    const bool active = ray < (int64_t)B * R;
    float* alpha = lds_alpha + wave * S;
    if (active) {
        const int b = (int)(ray / R), r = (int)(ray % R);
        float o[3], txn[3], dir[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            o[c] = rays_o[b * 3 + c];
            txn[c] = to_unit(pos_tx[b * 3 + c], p.lo, p.span);
            dir[c] = dirs[r * 3 + c];
        }
        const int64_t base = ray * S;
        // rounds of 8 coalesced attn loads per lane, all in flight before use
        for (int s0 = 0; s0 < S; s0 += 8 * 64) {
            float av[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) av[j] = load_f(attn, base + min(s0 + j * 64 + lane, S - 1));
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int s = s0 + j * 64 + lane;
                if (s < S) {
                    const float d = linspace_at(0.0f, 1.0f, S, s) * p.depth_scale + p.depth_offset;
                    const float dn =
                        linspace_at(0.0f, 1.0f, S, s + 1) * p.depth_scale + p.depth_offset;
                    const float gap = (s + 1 < S) ? dn - d : 1e10f;
                    alpha[s] = 1.0f - expf(-av[j] * gap);
                    delay[base + s] = source_delay(p, o, txn, dir, d);
                }
            }
        }
    }
    __syncthreads();
    const int64_t base = ray * S;
    if (active) {
        const int per = (S + 63) / 64;
        const int s0 = min(S, lane * per), s1 = min(S, s0 + per);
        float run = 1.0f;
        for (int s = s0; s < s1; ++s) run = run * ((1.0f - alpha[s]) + 1e-6f);
        // inclusive multiplicative scan over lanes, then shift to exclusive
        float incl = run;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float v = __shfl_up(incl, off, 64);
            if (lane >= off) incl = incl * v;
        }
        float trans = __shfl_up(incl, 1, 64);
        if (lane == 0) trans = 1.0f;
        for (int s = s0; s < s1; ++s) {
            const float al = alpha[s];
            alpha[s] = trans * al;  // w_s, written back in place
            trans = trans * ((1.0f - al) + 1e-6f);
        }
    }
    __syncthreads();
    if (active)
        for (int s = lane; s < S; s += 64) w_out[base + s] = alpha[s];  // coalesced
}

// --------------------------------------------- the HBM stream: ray reduce
// part[k][b][s][t] = sum_{r in split k} w[b,r,s] * [delay[b,r,s] <= t < T-1-shift[s]] * x[b,r,s,t]
// i.e. both masks of renderer.py:72-78 (the tail mask is applied again,
// redundantly, by the DFT stage).  Each row (b,r,s) of T contiguous elements
// is read at most once with 16-byte loads, and only its LIVE window
// [delay, T-1-shift) is read at all: a 16-byte chunk whose slots are all
// masked is never loaded (its product with the mask is zero for any finite
// signal).  Because S*T is a multiple of VEC, every row of one (b,s) column
// has the same alignment phase, so a lane's register accumulators always see
// the same t indices.  The per-ray w/delay of the split are gathered into
// LDS once.
constexpr int kMaxReduceThreads = 1024;
constexpr int kMaxGroupRays = 4096;  // G * rays_per_split (LDS: 32 KiB of w/delay)

// One workgroup per (ray split, column group, b).  A column group is G
// consecutive samples s0..s0+G-1 whose rows are contiguous in memory for
// every ray (the sample index is the second-fastest), so the workgroup
// streams one "super-row" of G*T elements per ray with 16-byte loads.  G is
// chosen so a super-row is ~256*VEC elements (short rows: fp16 or small T);
// the block size is chosen so every lane owns CPT chunks of it.  Lane slots
// have fixed (g, t) coordinates, so the accumulators need no shuffling.
template <typename Tin, bool VECTOR, int CPT, int kUnroll, int G, int MAXT>
__global__ __launch_bounds__(MAXT) void ray_reduce_fwd_kernel(
    avr_render_params pp, const Tin* __restrict__ sig, const float* __restrict__ w,
    const int32_t* __restrict__ delay, float* __restrict__ part, int B, int R, int S, int T,
    int rays_per_split, int64_t total) {
    constexpr int VEC = VECTOR ? Vec16<Tin>::N : 1;
    extern __shared__ float lds_wd[];  // w_l[G][nr], then d_l[G][nr]
    const int nthreads = blockDim.x;
    const int split = blockIdx.x, s0 = blockIdx.y * G, b = blockIdx.z;
    const int gcount = min(G, S - s0);
    const int r0 = split * rays_per_split;
    const int nr = max(0, min(R, r0 + rays_per_split) - r0);
    float* w_l = lds_wd;
    int* d_l = reinterpret_cast<int*>(lds_wd + G * max(nr, 1));
    for (int i = threadIdx.x; i < G * nr; i += nthreads) {
        const int g = i / nr, rr = i - g * nr;
        if (g < gcount) {
            const int64_t idx = ((int64_t)b * R + r0 + rr) * S + s0 + g;
            w_l[i] = w[idx];
            d_l[i] = delay[idx];
        } else {
            w_l[i] = 0.0f;
            d_l[i] = 0x7fffffff;
        }
    }
    __syncthreads();
    // an empty split (nr == 0) falls through both loops and writes zeros
    const int64_t row0 = (((int64_t)b * R + r0) * S + s0) * (int64_t)T;
    const int L = gcount * T;  // super-row length
    const int phase = (int)(row0 % VEC);
    const int nchunks = (L + phase + VEC - 1) / VEC;
    const int64_t row_stride = (int64_t)S * T;

    float acc[CPT][VEC];
    int tk[CPT][VEC];  // t of each slot (-1: outside the super-row)
    int tm[CPT][VEC];  // t if inside the tail window t < T-1-shift[s], else -1
    int gk[CPT][VEC];  // column of each slot within the group
    int tmax[CPT][G];  // per chunk and column: largest tm (-1: no live slot)
    int lim[G];
#pragma unroll
    for (int g = 0; g < G; ++g) lim[g] = tail_limit(pp, min(s0 + g, S - 1));
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
#pragma unroll
        for (int g = 0; g < G; ++g) tmax[c][g] = -1;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            acc[c][k] = 0.0f;
            const int e = (threadIdx.x + c * nthreads) * VEC + k - phase;
            const bool ok = e >= 0 && e < L;
            const int g = (G == 1) ? 0 : (ok ? e / T : 0);
            gk[c][k] = g;
            tk[c][k] = ok ? e - g * T : -1;
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

    // chunk c of ray r is live if any slot t satisfies delay <= t < T-1-shift
    auto live = [&](int r, int c) {
        bool any = false;
#pragma unroll
        for (int g = 0; g < G; ++g) any |= tmax[c][g] >= d_l[g * nr + r];
        return any;
    };
    auto load_chunk = [&](int64_t rowbase, int c, bool need, float* x) {
        const int j = threadIdx.x + c * nthreads;
        if constexpr (VECTOR) {
            // S*T % VEC == 0 (host check) and rowbase is VEC-aligned: the
            // super-row's chunks lie inside the tensor.  Dead chunks and lanes
            // past the last chunk read zeros without touching memory.
            load16_masked(sig + rowbase, (uint32_t)nchunks * 16u,
                          need ? (uint32_t)j * 16u : kSkip, x);
        } else {
            const int64_t e0 = rowbase + j;
            x[0] = (need && j < nchunks && e0 < total) ? load_f(sig, e0) : 0.0f;
        }
    };
    auto accumulate = [&](int r, float (*x)[VEC]) {
        float wg[G];
        int dg[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            wg[g] = w_l[g * nr + r];
            dg[g] = d_l[g * nr + r];
        }
#pragma unroll
        for (int c = 0; c < CPT; ++c)
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
                const float wm = (tm[c][k] >= ds) ? ws : 0.0f;
                acc[c][k] = fmaf(wm, x[c][k], acc[c][k]);
            }
    };

    int r = 0;
    for (; r + kUnroll <= nr; r += kUnroll) {
        float x[kUnroll][CPT][VEC];
        bool need[kUnroll][CPT];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
#pragma unroll
            for (int c = 0; c < CPT; ++c) need[u][c] = live(r + u, c);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t rowbase = row0 + (int64_t)(r + u) * row_stride - phase;
#pragma unroll
            for (int c = 0; c < CPT; ++c) load_chunk(rowbase, c, need[u][c], x[u][c]);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) accumulate(r + u, x[u]);
    }
    for (; r < nr; ++r) {
        const int64_t rowbase = row0 + (int64_t)r * row_stride - phase;
        float x[CPT][VEC];
#pragma unroll
        for (int c = 0; c < CPT; ++c) load_chunk(rowbase, c, live(r, c), x[c]);
        accumulate(r, x);
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const int t = tk[c][k];
            if (t >= 0) part[(((int64_t)split * B + b) * S + s0 + gk[c][k]) * T + t] = acc[c][k];
        }
}

// ------------------------------- DFT + phase + sum over samples (MFMA f32)
// C[s, (f,re|im)] = sum_t z[b,s,t] * tw[(t*f) mod T]  with v_mfma_f32_32x32x2_f32
// (exact fp32 FMA chain).  A = z tile staged in LDS (32 samples x 64 t),
// built on the fly from the ray-reduce partials with path loss and the tail
// mask applied; B = twiddles gathered from a 1-D table of T complex values
// in LDS by the index (t*f) mod T, advanced incrementally.  Epilogue: rotate
// by phase[s,f] and reduce the 32 sample rows; partials per (s-tile, k-slice)
// are summed by avr_spectrum_finalize.
constexpr int kDftThreads = 256;
constexpr int kKc = 64;  // t per LDS stage

// A-tile staging (see `stage` below): thread owns column t = kc + (tid & 63)
// of rows (tid >> 6) + 4i, i < 8.  Addresses are clamped to valid locations
// and masked afterwards, so all 8*NS partial loads (+ 8 path-loss loads)
// issue back to back with no per-element branch, and the next tile's loads
// are in flight while the MFMAs consume the current one.
template <int NS>
__global__ __launch_bounds__(kDftThreads) void dft_phase_fwd_kernel(
    avr_render_params pp, const float* __restrict__ part, const float* __restrict__ pl,
    const int32_t* __restrict__ shift, const float2* __restrict__ phase,
    const float2* __restrict__ twg, float2* __restrict__ spart, int B, int S, int T, int KS,
    int kchunk, int xcd_order) {
    extern __shared__ float2 tw[];           // [T]
    __shared__ float As[32][kKc + 1];
    const int F = T / 2 + 1;
    const int P = ((S + 31) / 32) * KS;
    // XCD-aware order: every workgroup of one s-tile (its k-slices x F-blocks)
    // runs on one XCD (dispatch goes round-robin over the 8 XCDs by
    // workgroup id), so the tile's z rows and phase rows are fetched into
    // that XCD's L2 once instead of once per k-slice / F-block.  With fewer
    // than 8 s-tiles (S < 225: configs 3 and 4) that order would leave XCDs
    // idle, so the tile's workgroups are spread over all of them instead.
    (void)P;
    const int nfb = (F + 127) / 128, nst = (S + 31) / 32;
    const int per = KS * nfb;  // workgroups of one s-tile
    int stile, q;
    if (xcd_order) {
        const int L = blockIdx.x, xcd = L & 7;
        q = L >> 3;
        stile = (q / per) * 8 + xcd;
        if (stile >= nst) return;  // padding workgroups of the 8-way split
    } else {
        stile = blockIdx.x / per;
        q = blockIdx.x;
    }
    const int ks = (q % per) / nfb, fblk = (q % per) % nfb;
    const int b = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int fbase = fblk * 128 + wave * 32;
    const int f = fbase + (lane & 31);
    const int fm = (f < F) ? f : 0;
    const int half = lane >> 5;
    // this thread's staging rows; shift[s] recomputed (renderer.py:79-80),
    // identical to the table, so the path-loss gather is not a dependent load
    const int col = threadIdx.x & 63, row0 = threadIdx.x >> 6;
    int sh[8];
    bool srow[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int s = stile * 32 + row0 + 4 * i;
        srow[i] = s < S;
        sh[i] = receiver_shift(pp, min(s, S - 1));
    }
    (void)shift;
    const int64_t slab = (int64_t)B * S * T;
    // rows beyond S are clamped to row S-1 (masked by srow)
    const int s_first = min(stile * 32 + row0, S - 1);
    const int64_t rowbase0 = ((int64_t)b * S + s_first) * T;
    const int64_t max_row_off = ((int64_t)b * S + (S - 1)) * T;

    const int k0 = ks * kchunk;
    const int k1 = min(T, k0 + kchunk);
    floatx16 acc_re, acc_im;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc_re[i] = 0.0f;
        acc_im[i] = 0.0f;
    }
    const int inc = (int)((2LL * fm) % T);
    // raw loads of one tile (NS partial slabs + path loss), kept in registers
    // until the tile is committed to LDS, so the next tile's loads stay in
    // flight under the current tile's MFMAs
    float raw[NS][8], g[8];
    auto issue = [&](int kc) {
        const int tc = min(kc + col, T - 1);
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int64_t ro = min(rowbase0 + (int64_t)(4 * i) * T, max_row_off);
                raw[k][i] = part[k * slab + ro + tc];
            }
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = pl[sh[i] + tc];
    };
    auto commit = [&](int kc) {
        const int t = kc + col;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float sum = raw[0][i];
#pragma unroll
            for (int k = 1; k < NS; ++k) sum += raw[k][i];
            const bool ok = srow[i] && t < k1 && t < T - 1 - sh[i];
            As[row0 + 4 * i][col] = ok ? sum * g[i] : 0.0f;
        }
    };
    if (k0 < k1) issue(k0);
    stage_table<kDftThreads>(tw, twg, T);  // its loads overlap the first tile's
    for (int kc = k0; kc < k1; kc += kKc) {
        __syncthreads();
        commit(kc);
        __syncthreads();
        if (kc + kKc < k1) issue(kc + kKc);  // next tile's loads fly under the MFMAs
        int idx = (int)(((int64_t)(kc + half) * fm) % T);
#pragma unroll 8
        for (int kk = 0; kk < kKc; kk += 2) {
            const float a = As[lane & 31][kk + half];
            float2 c = tw[idx];
            asm volatile("" : "+v"(c.x), "+v"(c.y));
            acc_re = __builtin_amdgcn_mfma_f32_32x32x2f32(a, c.x, acc_re, 0, 0, 0);
            acc_im = __builtin_amdgcn_mfma_f32_32x32x2f32(a, c.y, acc_im, 0, 0, 0);
            idx += inc;
            if (idx >= T) idx -= T;
        }
    }
    // epilogue: rows (reg&3) + 8*(reg>>2) + 4*half, column lane&31; the 16
    // phase loads are issued together (clamped, masked after)
    float re = 0.0f, im = 0.0f;
    {
        float2 ph[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int s = stile * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * half;
            ph[reg] = phase[(int64_t)min(s, S - 1) * F + fm];
        }
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) asm volatile("" ::"v"(ph[reg].x), "v"(ph[reg].y));
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int s = stile * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * half;
            if (s < S) {
                const float zr = acc_re[reg], zi = acc_im[reg];
                re += zr * ph[reg].x - zi * ph[reg].y;
                im += zr * ph[reg].y + zi * ph[reg].x;
            }
        }
    }
    re += __shfl_xor(re, 32, 64);
    im += __shfl_xor(im, 32, 64);
    if (half == 0 && f < F) {
        spart[((int64_t)b * P + stile * KS + ks) * F + f] = make_float2(re, im);
    }
}

// out[b,f] = sum_p spart[b,p,f]: 16 partial-groups x 16 bins per block; each
// thread's loads of a round (4 partials) are issued together, then the 16
// groups are combined in LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void spectrum_finalize_kernel(int B, int P, int F,
                                                                const float2* __restrict__ spart,
                                                                float2* __restrict__ out) {
    __shared__ float2 red[16][17];
    const int b = blockIdx.y;
    const int g = threadIdx.x >> 4, j = threadIdx.x & 15;
    const int f = blockIdx.x * 16 + j;
    const int fc = min(f, F - 1);
    const float2* src = spart + (int64_t)b * P * F + fc;
    float ax = 0.f, ay = 0.f;
    for (int q0 = 0; q0 < P; q0 += 64) {
        float2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[(int64_t)min(q0 + g + 16 * u, P - 1) * F];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (q0 + g + 16 * u < P) {
                ax += v[u].x;
                ay += v[u].y;
            }
    }
    red[g][j] = make_float2(ax, ay);
    __syncthreads();
    if (g == 0 && f < F) {
        float2 r = red[0][j];
        for (int k = 1; k < 16; ++k) {
            r.x += red[k][j].x;
            r.y += red[k][j].y;
        }
        out[(int64_t)b * F + f] = r;
    }
}

// -------------------------------------------------- a13: irfft -> IR
// torch.fft.irfft semantics (n = 2(F-1), backward norm 1/n, imaginary parts
// of the DC and Nyquist bins ignored):
//   ir[t] = (X0 + (-1)^t X_{n/2} + 2 sum_{k=1}^{n/2-1} Re(X_k e^{2 pi i k t/n})) / n
// Block = 32 output samples x 8 bin-slices; each thread walks bins
// k = 1 + slice + 8j with four independent index chains (ILP over the LDS
// latency), then the 8 slices are combined in LDS in a fixed order.
// Rows b >= B1 come from (spec2, ir2): the criterion transforms the
// predicted and measured spectra in one launch.
__global__ __launch_bounds__(256) void irfft_kernel(int F, int B1, const float2* __restrict__ spec,
                                                    const float2* __restrict__ spec2,
                                                    const float2* __restrict__ twg,
                                                    float* __restrict__ ir, float* __restrict__ ir2) {
    extern __shared__ float2 lds[];
    __shared__ float red[8][33];
    const int n = 2 * (F - 1);
    float2* X = lds;       // [F]
    float2* tw = lds + F;  // [n]
    int b = blockIdx.y;
    if (b >= B1) {
        b -= B1;
        spec = spec2;
        ir = ir2;
    }
    stage_table<256>(X, spec + (int64_t)b * F, F);
    stage_table<256>(tw, twg, n);
    __syncthreads();
    const int tl = threadIdx.x & 31, slice = threadIdx.x >> 5;
    const int t = blockIdx.x * 32 + tl;
    const int tm = (t < n) ? t : 0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int idx[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) idx[c] = (int)(((int64_t)(1 + slice + 8 * c) * tm) % n);
    const int step4 = (int)((32LL * tm) % n);
    int k = 1 + slice;
    for (; k + 24 < F - 1; k += 32) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float2 w = tw[idx[c]];
            const float2 x = X[k + 8 * c];
            acc[c] += x.x * w.x - x.y * w.y;
            idx[c] += step4;
            if (idx[c] >= n) idx[c] -= n;
        }
    }
    for (; k < F - 1; k += 8) {
        // tail bins of this slice
        const int id = (int)(((int64_t)k * tm) % n);
        const float2 w = tw[id];
        const float2 x = X[k];
        acc[0] += x.x * w.x - x.y * w.y;
    }
    red[slice][tl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (slice == 0 && t < n) {
        float s = 0.0f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s += red[q][tl];
        const float nyq = (t & 1) ? -X[F - 1].x : X[F - 1].x;
        const float v = (X[0].x + nyq) + 2.0f * s;
        ir[(int64_t)b * n + t] = v / (float)n;
    }
}

// Adjoint irfft (torch's c2r backward): for bin k with weight c_k (1 at DC
// and Nyquist, 2 inside),
//   grad[k] = c_k / n * ( sum_t g[t] cos(2 pi k t/n), -sum_t g[t] sin(2 pi k t/n) )
// and a zero imaginary part at DC / Nyquist.  Block = 32 bins x 8 t-slices;
// each thread walks t = slice + 8j with the twiddle index advanced
// incrementally, the 8 slices combined in LDS in a fixed order.
__global__ __launch_bounds__(256) void irfft_bwd_kernel(int F, const float* __restrict__ gir,
                                                        const float2* __restrict__ twg,
                                                        float2* __restrict__ grad) {
    extern __shared__ float lds_irb[];
    __shared__ float2 red[8][33];
    const int n = 2 * (F - 1);
    const int b = blockIdx.y;
    float2* tw = reinterpret_cast<float2*>(lds_irb);  // [n]
    float* g = lds_irb + 2 * n;                       // [n]
    stage_table<256>(tw, twg, n);
    for (int i = threadIdx.x; i < n; i += 256) g[i] = gir[(int64_t)b * n + i];
    __syncthreads();
    const int kl = threadIdx.x & 31, sl = threadIdx.x >> 5;
    const int k = blockIdx.x * 32 + kl;
    const int km = k < F ? k : 0;
    int idx = (int)(((int64_t)km * sl) % n);
    const int step = (int)(((int64_t)km * 8) % n);
    float ac = 0.f, as = 0.f;
    for (int t = sl; t < n; t += 8) {
        const float2 c = tw[idx];
        ac = fmaf(g[t], c.x, ac);
        as = fmaf(g[t], c.y, as);
        idx += step;
        if (idx >= n) idx -= n;
    }
    red[sl][kl] = make_float2(ac, as);
    __syncthreads();
    if (sl == 0 && k < F) {
        float2 r = red[0][kl];
        for (int q = 1; q < 8; ++q) {
            r.x += red[q][kl].x;
            r.y += red[q][kl].y;
        }
        const bool edge = (k == 0) || (k == F - 1);
        const float c = (edge ? 1.0f : 2.0f) / (float)n;
        grad[(int64_t)b * F + k] = make_float2(c * r.x, edge ? 0.0f : -c * r.y);
    }
}

int pick_blocks(int64_t n, int threads, int cap = 4096) {
    int64_t g = (n + threads - 1) / threads;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

int validate(const avr_render_params* p) {
    if (!p) return fail(AVR_E_ARG, "null params");
    if (p->n_azi < 1 || p->n_ele < 1 || p->n_samples < 1 || p->T < 2)
        return fail(AVR_E_CONFIG, "n_azi, n_ele, n_samples must be >=1 and T >= 2");
    if (p->T > 16384) return fail(AVR_E_CONFIG, "T > 16384 not supported");
    if (p->n_rays < 1 || p->n_rays > grid_rays(*p))
        return fail(AVR_E_CONFIG, "n_rays must be in [1, n_azi*n_ele+2]");
    if (p->n_samples > 8192) return fail(AVR_E_CONFIG, "n_samples > 8192 not supported");
    return 0;
}

}  // namespace

// ======================================================================
// C-ABI
// ======================================================================
extern "C" int avr_tables(const avr_render_params* p, float* d_vals, float* frac, int32_t* shift,
                          float* pl_table, float* phase, float* twiddle, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(d_vals && frac && shift && pl_table && phase && twiddle, "avr_tables: null pointer");
    const int64_t work = (int64_t)p->n_samples * (p->T / 2 + 1);
    hipLaunchKernelGGL(tables_kernel, dim3(pick_blocks(work, 256, 1024)), dim3(256), 0,
                       as_stream(stream), *p, d_vals, frac, shift, pl_table,
                       reinterpret_cast<float2*>(phase), reinterpret_cast<float2*>(twiddle));
    return check_launch("avr_tables");
}

extern "C" int avr_depth_samples(const avr_render_params* p, float* d_vals, void* stream) {
    AVR_REQUIRE(p && p->n_samples >= 1 && d_vals, "avr_depth_samples: bad args");
    hipLaunchKernelGGL(depth_samples_kernel, dim3((p->n_samples + 255) / 256), dim3(256), 0,
                       as_stream(stream), *p, d_vals);
    return check_launch("avr_depth_samples");
}

extern "C" int avr_ir_twiddle(int32_t n, float* tw, void* stream) {
    AVR_REQUIRE(n >= 2 && tw, "avr_ir_twiddle: bad args");
    hipLaunchKernelGGL(ir_twiddle_kernel, dim3(pick_blocks(n, 256, 256)), dim3(256), 0,
                       as_stream(stream), n, reinterpret_cast<float2*>(tw));
    return check_launch("avr_ir_twiddle");
}

extern "C" int avr_ray_directions(const avr_render_params* p, const float* u_azi, float* dirs,
                                  void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(u_azi && dirs, "avr_ray_directions: null pointer");
    const int R = grid_rays(*p);
    hipLaunchKernelGGL(ray_directions_kernel, dim3((R + 255) / 256), dim3(256), 0,
                       as_stream(stream), *p, u_azi, dirs);
    return check_launch("avr_ray_directions");
}

extern "C" int avr_sample_points(const avr_render_params* p, int32_t B, const float* rays_o,
                                 const float* pos_tx, const float* dir_tx, const float* dirs,
                                 const float* d_vals, float* net_pts, float* net_view,
                                 float* net_tx, float* net_dir_tx, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && rays_o && pos_tx && dirs && d_vals && net_pts && net_view && net_tx,
                "avr_sample_points: bad args");
    AVR_REQUIRE(!dir_tx || net_dir_tx, "avr_sample_points: dir_tx given without net_dir_tx");
    const int64_t n = (int64_t)B * n_rays(*p) * p->n_samples;
    hipLaunchKernelGGL(sample_points_kernel, dim3(pick_blocks(n, 256, 8192)), dim3(256), 0,
                       as_stream(stream), *p, (int)B, rays_o, pos_tx, dir_tx, dirs, d_vals,
                       net_pts, net_view, net_tx, dir_tx ? net_dir_tx : nullptr);
    return check_launch("avr_sample_points");
}

extern "C" int avr_sample_rays(const avr_render_params* p, int32_t B, const float* u_azi_host,
                               int32_t ray_begin, const float* rays_o, const float* pos_tx,
                               const float* dir_tx, float* dirs, float* net_pts, float* net_view,
                               float* net_tx, float* net_dir_tx, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && u_azi_host && rays_o && pos_tx && dirs && net_pts && net_view && net_tx,
                "avr_sample_rays: bad args");
    AVR_REQUIRE(!dir_tx || net_dir_tx, "avr_sample_rays: dir_tx given without net_dir_tx");
    AVR_REQUIRE(p->n_azi <= AVR_MAX_AZI, "avr_sample_rays: n_azi > AVR_MAX_AZI (use avr_ray_directions)");
    AVR_REQUIRE(ray_begin >= 0 && ray_begin + p->n_rays <= grid_rays(*p),
                "avr_sample_rays: ray range outside the sphere");
    AziJitter jit;
    for (int i = 0; i < AVR_MAX_AZI; ++i) jit.u[i] = (i < p->n_azi) ? u_azi_host[i] : 0.0f;
    const int64_t n = (int64_t)B * n_rays(*p) * p->n_samples;
    hipLaunchKernelGGL(sample_rays_kernel, dim3((unsigned)((n + kSampleThreads - 1) / kSampleThreads)),
                       dim3(kSampleThreads), 0,
                       as_stream(stream), *p, (int)B, jit, (const float*)nullptr, (int)ray_begin, rays_o,
                       pos_tx, dir_tx, dirs, net_pts, net_view, net_tx, dir_tx ? net_dir_tx : nullptr,
                       (float*)nullptr);
    return check_launch("avr_sample_rays");
}

// Same launch with the jitter read from DEVICE memory when the kernel runs
// (graph replay: avr_amd.graph.GraphedRender refreshes the buffer per pose).
extern "C" int avr_sample_rays_dev(const avr_render_params* p, int32_t B, const float* u_azi_dev,
                                   int32_t ray_begin, const float* rays_o, const float* pos_tx,
                                   const float* dir_tx, float* dirs, float* net_pts, float* net_view,
                                   float* net_tx, float* net_dir_tx, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && u_azi_dev && rays_o && pos_tx && dirs && net_pts && net_view && net_tx,
                "avr_sample_rays_dev: bad args");
    AVR_REQUIRE(!dir_tx || net_dir_tx, "avr_sample_rays_dev: dir_tx given without net_dir_tx");
    AVR_REQUIRE(ray_begin >= 0 && ray_begin + p->n_rays <= grid_rays(*p),
                "avr_sample_rays_dev: ray range outside the sphere");
    AziJitter jit{};
    const int64_t n = (int64_t)B * n_rays(*p) * p->n_samples;
    hipLaunchKernelGGL(sample_rays_kernel, dim3((unsigned)((n + kSampleThreads - 1) / kSampleThreads)),
                       dim3(kSampleThreads), 0,
                       as_stream(stream), *p, (int)B, jit, u_azi_dev, (int)ray_begin, rays_o, pos_tx, dir_tx,
                       dirs, net_pts, net_view, net_tx, dir_tx ? net_dir_tx : nullptr, (float*)nullptr);
    return check_launch("avr_sample_rays_dev");
}

extern "C" int avr_sample_rays_staged(const avr_render_params* p, int32_t B, const float* staged,
                                      int32_t has_dir_tx, int32_t ray_begin, float* pose_out, float* dirs,
                                      float* net_pts, float* net_view, float* net_tx, float* net_dir_tx,
                                      void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && staged && pose_out && dirs && net_pts && net_view && net_tx,
                "avr_sample_rays_staged: bad args");
    AVR_REQUIRE(!has_dir_tx || net_dir_tx, "avr_sample_rays_staged: dir_tx without net_dir_tx");
    AVR_REQUIRE(ray_begin >= 0 && ray_begin + p->n_rays <= grid_rays(*p),
                "avr_sample_rays_staged: ray range outside the sphere");
    AziJitter jit{};
    const float* ro = staged;
    const float* tx = ro + 3 * B;
    const float* dtx = has_dir_tx ? tx + 3 * B : nullptr;
    const float* u = staged + 9 * B;
    const int64_t n = (int64_t)B * n_rays(*p) * p->n_samples;
    hipLaunchKernelGGL(sample_rays_kernel, dim3((unsigned)((n + kSampleThreads - 1) / kSampleThreads)),
                       dim3(kSampleThreads), 0, as_stream(stream), *p, (int)B, jit, u, (int)ray_begin,
                       ro, tx, dtx, dirs, net_pts, net_view, net_tx, dtx ? net_dir_tx : nullptr, pose_out);
    return check_launch("avr_sample_rays_staged");
}

extern "C" int avr_weights_fwd(const avr_render_params* p, int32_t B, const void* attn,
                               int32_t attn_dtype, const float* rays_o, const float* pos_tx,
                               const float* dirs, const float* d_vals, float* w, int32_t* delay,
                               void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && attn && rays_o && pos_tx && dirs && d_vals && w && delay,
                "avr_weights_fwd: bad args");
    const int64_t rays = (int64_t)B * n_rays(*p);
    const dim3 grid((unsigned)((rays + 3) / 4));
    const size_t lds = 4 * (size_t)p->n_samples * sizeof(float);
    if (lds > 65536) {
        (void)hipFuncSetAttribute((const void*)weights_fwd_kernel<float>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)weights_fwd_kernel<__half>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)weights_fwd_kernel<__hip_bfloat16>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (attn_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(weights_fwd_kernel<float>, grid, dim3(256), lds, as_stream(stream), *p,
                           (int)B, (const float*)attn, rays_o, pos_tx, dirs, d_vals, w, delay);
    else if (attn_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(weights_fwd_kernel<__half>, grid, dim3(256), lds, as_stream(stream),
                           *p, (int)B, (const __half*)attn, rays_o, pos_tx, dirs, d_vals, w, delay);
    else if (attn_dtype == AVR_DTYPE_BF16)
        hipLaunchKernelGGL(weights_fwd_kernel<__hip_bfloat16>, grid, dim3(256), lds,
                           as_stream(stream), *p, (int)B, (const __hip_bfloat16*)attn, rays_o,
                           pos_tx, dirs, d_vals, w, delay);
    else
        return fail(AVR_E_ARG, "avr_weights_fwd: unknown attn dtype");
    return check_launch("avr_weights_fwd");
}


namespace {
// Streaming variant of the reduction: 4 rows in flight per lane with
// non-temporal loads, the best of the sweeps (profiles/r01_tune*; 8 rows is
// variant 3).
int reduce_variant() { return 2; }

struct ReduceShape {
    int G, cpt, threads;
};

// Column group, chunks per lane and block size for one (T, VEC, S).
template <int VEC>
ReduceShape reduce_shape(int S, int T) {
    ReduceShape sh;
    // one sample per column group: G = 1 beat G = 2 (and G = 2 beat G = 4)
    // on configs 2 (fp32 and fp16) and 3 in every interleaved round of the
    // round-2 sweeps (profiles/r02_sweepG_*.jsonl: config 2 fp32 111.8 vs
    // 115.7 us per launch); fewer w/delay selects per loaded element
    sh.G = 1;
    int max_phase = 0;  // group starts are s0 = multiples of G; S*T % VEC == 0
    for (int s0 = 0; s0 < S && s0 < VEC * sh.G; s0 += sh.G)
        max_phase = max(max_phase, (int)(((int64_t)s0 * T) % VEC));
    const int nch = (sh.G * T + max_phase + VEC - 1) / VEC;
    sh.cpt = 1;
    while ((nch + sh.cpt - 1) / sh.cpt > kMaxReduceThreads) ++sh.cpt;
    const int need = (nch + sh.cpt - 1) / sh.cpt;
    sh.threads = max(64, (need + 63) / 64 * 64);
    return sh;
}

// Variants: rows in flight per lane (4 or 8) x launch
// bound (512 threads leaves 256 VGPRs per lane, 1024 only 128).
template <typename Tin, bool VECTOR, int C, int G>
void launch_reduce_v(dim3 grid, dim3 block, size_t lds, hipStream_t st, const avr_render_params& pp,
                     const Tin* s, const float* w,
                     const int32_t* delay, float* part, int B, int R, int S, int T, int rps,
                     int64_t total) {
    const bool u8 = reduce_variant() == 3;
    if (block.x <= 512) {
        if (u8)
            hipLaunchKernelGGL((ray_reduce_fwd_kernel<Tin, VECTOR, C, 8, G, 512>), grid, block,
                               lds, st, pp, s, w, delay, part, B, R, S, T, rps, total);
        else
            hipLaunchKernelGGL((ray_reduce_fwd_kernel<Tin, VECTOR, C, 4, G, 512>), grid, block,
                               lds, st, pp, s, w, delay, part, B, R, S, T, rps, total);
    } else {
        if (u8)
            hipLaunchKernelGGL((ray_reduce_fwd_kernel<Tin, VECTOR, C, 8, G, 1024>), grid, block,
                               lds, st, pp, s, w, delay, part, B, R, S, T, rps, total);
        else
            hipLaunchKernelGGL((ray_reduce_fwd_kernel<Tin, VECTOR, C, 4, G, 1024>), grid, block,
                               lds, st, pp, s, w, delay, part, B, R, S, T, rps, total);
    }
}

template <typename Tin, bool VECTOR>
int launch_reduce(const avr_render_params* p, int B, const void* sig, const float* w,
                  const int32_t* delay, int n_split, float* part, hipStream_t st) {
    constexpr int VEC = VECTOR ? Vec16<Tin>::N : 1;
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    const int rps = (R + n_split - 1) / n_split;
    const ReduceShape sh = reduce_shape<VEC>(S, T);
    if (sh.G * rps > kMaxGroupRays)
        return fail(AVR_E_ARG, "avr_ray_reduce_fwd: too many rays per split (raise n_split)");
    const int64_t total = (int64_t)B * R * S * T;
    const dim3 grid(n_split, (S + sh.G - 1) / sh.G, B);
    const dim3 block(sh.threads);
    const size_t lds = (size_t)sh.G * max(rps, 1) * 8;
    const Tin* s = (const Tin*)sig;
#define AVR_RR(C, GG)                                                                              \
    if (sh.cpt == C && sh.G == GG)                                                                 \
        return launch_reduce_v<Tin, VECTOR, C, GG>(grid, block, lds, st, *p, s, w, delay, part, B, R, S, \
                                                   T, rps, total),                                 \
               check_launch("avr_ray_reduce_fwd");
    AVR_RR(1, 1) AVR_RR(1, 2) AVR_RR(1, 4) AVR_RR(2, 1) AVR_RR(2, 2) AVR_RR(2, 4) AVR_RR(3, 1)
    AVR_RR(4, 1)
#undef AVR_RR
    return fail(AVR_E_CONFIG, "ray_reduce: T too long for this build");
}
}  // namespace

extern "C" int avr_reduce_splits(const avr_render_params* p, int32_t B, int32_t sig_dtype,
                                 int32_t* n_split) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && n_split, "avr_reduce_splits: bad args");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    const int vec = (sig_dtype == AVR_DTYPE_F16 || sig_dtype == AVR_DTYPE_BF16) ? 8 : 4;
    const ReduceShape sh = vec == 8 ? reduce_shape<8>(S, T) : reduce_shape<4>(S, T);
    const int groups = (S + sh.G - 1) / sh.G;
    auto rps = [&](int k) { return (R + k - 1) / k; };
    if (const char* f = getenv("AVR_NSPLIT")) {  // validated tuning knob: 1, 2, 4, 8 or 16 ray splits
        const int v = atoi(f);
        if ((v == 1 || v == 2 || v == 4 || v == 8 || v == 16) && v <= R && rps(v) * sh.G <= kMaxGroupRays) {
            *n_split = v;
            return 0;
        }
    }
    // power of two <= 16 (the DFT staging is templated on it) giving ~8 (fp32)
    // or ~16 (fp16: twice the VALU work per byte) resident waves per CU, and
    // a split's w/delay within the 32 KiB LDS slab.  Sweeps:
    // profiles/r01_sweep_*.jsonl.
    const int64_t waves_target = (vec == 8) ? 4096 : 1536;
    const int64_t waves_per_split = (int64_t)groups * B * (sh.threads / 64);
    int n = 1;
    while (n < 16 && (n * waves_per_split < waves_target || rps(n) * sh.G > kMaxGroupRays) &&
           rps(2 * n) >= 8)
        n *= 2;
    if (rps(n) * sh.G > kMaxGroupRays) return fail(AVR_E_CONFIG, "avr_reduce_splits: too many rays");
    *n_split = n;
    return 0;
}

extern "C" int avr_ray_reduce_fwd(const avr_render_params* p, int32_t B, const void* signal,
                                  int32_t sig_dtype, const float* w, const int32_t* delay,
                                  int32_t n_split, float* part, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && signal && w && delay && part, "avr_ray_reduce_fwd: null pointer");
    const int R = n_rays(*p);
    AVR_REQUIRE(n_split >= 1 && n_split <= R, "avr_ray_reduce_fwd: n_split out of range");
    AVR_REQUIRE((R + n_split - 1) / n_split <= kMaxGroupRays,
                "avr_ray_reduce_fwd: too many rays per split (raise n_split)");
    const int64_t st = (int64_t)p->n_samples * p->T;
    const bool aligned = (reinterpret_cast<uintptr_t>(signal) % 16) == 0;
    hipStream_t s = as_stream(stream);
    if (sig_dtype == AVR_DTYPE_F32) {
        if (aligned && st % 4 == 0) return launch_reduce<float, true>(p, B, signal, w, delay, n_split, part, s);
        return launch_reduce<float, false>(p, B, signal, w, delay, n_split, part, s);
    }
    if (sig_dtype == AVR_DTYPE_F16) {
        if (aligned && st % 8 == 0) return launch_reduce<__half, true>(p, B, signal, w, delay, n_split, part, s);
        return launch_reduce<__half, false>(p, B, signal, w, delay, n_split, part, s);
    }
    if (sig_dtype == AVR_DTYPE_BF16) {
        if (aligned && st % 8 == 0)
            return launch_reduce<__hip_bfloat16, true>(p, B, signal, w, delay, n_split, part, s);
        return launch_reduce<__hip_bfloat16, false>(p, B, signal, w, delay, n_split, part, s);
    }
    return fail(AVR_E_ARG, "avr_ray_reduce_fwd: unknown signal dtype");
}

extern "C" int avr_dft_phase_fwd(const avr_render_params* p, int32_t B, const float* part,
                                 int32_t n_split, const float* pl_table, const int32_t* shift,
                                 const float* phase, const float* twiddle, int32_t k_split,
                                 float* spart, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && part && pl_table && shift && phase && twiddle && spart,
                "avr_dft_phase_fwd: null pointer");
    const int S = p->n_samples, T = p->T, F = T / 2 + 1;
    const int nkc = (T + kKc - 1) / kKc;
    AVR_REQUIRE(k_split >= 1 && k_split <= nkc, "avr_dft_phase_fwd: k_split out of range");
    const int kchunk = ((nkc + k_split - 1) / k_split) * kKc;
    // one dimension of (s-tile, k-slice, F-block) workgroups in the XCD-aware
    // order the kernel decodes (8 XCDs x ceil(s-tiles / 8) x k-slices x
    // F-blocks; padding ones exit)
    const int nst = (S + 31) / 32;
    const int xcd_order = nst >= 8;
    const int per = k_split * ((F + 127) / 128);
    const dim3 grid((unsigned)(xcd_order ? 8 * ((nst + 7) / 8) * per : nst * per), 1, B);
    const size_t lds = (size_t)T * sizeof(float2);
    auto go = [&](auto kern) {
        if (lds > 65536)
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds);
        hipLaunchKernelGGL(kern, grid, dim3(kDftThreads), lds, as_stream(stream), *p, part, pl_table,
                           shift, reinterpret_cast<const float2*>(phase),
                           reinterpret_cast<const float2*>(twiddle),
                           reinterpret_cast<float2*>(spart), (int)B, S, T, (int)k_split, kchunk, xcd_order);
    };
    switch (n_split) {
        case 1: go(dft_phase_fwd_kernel<1>); break;
        case 2: go(dft_phase_fwd_kernel<2>); break;
        case 4: go(dft_phase_fwd_kernel<4>); break;
        case 8: go(dft_phase_fwd_kernel<8>); break;
        case 16: go(dft_phase_fwd_kernel<16>); break;
        default: return fail(AVR_E_ARG, "avr_dft_phase_fwd: n_split must be 1, 2, 4, 8 or 16");
    }
    return check_launch("avr_dft_phase_fwd");
}

extern "C" int avr_spectrum_finalize(int32_t B, int32_t P, int32_t F, const float* spart,
                                     float* out, void* stream) {
    AVR_REQUIRE(B >= 1 && P >= 1 && F >= 1 && spart && out, "avr_spectrum_finalize: bad args");
    hipLaunchKernelGGL(spectrum_finalize_kernel, dim3((unsigned)((F + 15) / 16), B), dim3(256), 0,
                       as_stream(stream), (int)B, (int)P, (int)F,
                       reinterpret_cast<const float2*>(spart), reinterpret_cast<float2*>(out));
    return check_launch("avr_spectrum_finalize");
}

namespace avr {
int launch_irfft(int B, int F, const float* spec, const float* spec2, const float* tw, float* ir,
                 float* ir2, void* stream) {
    AVR_REQUIRE(B >= 1 && F >= 2 && spec && tw && ir, "avr_irfft: bad args");
    const int n = 2 * (F - 1);
    AVR_REQUIRE(n <= 16384, "avr_irfft: n too large");
    const size_t lds = (size_t)(F + n) * sizeof(float2);
    const int rows = spec2 ? 2 * B : B;
    hipLaunchKernelGGL(irfft_kernel, dim3((n + 31) / 32, rows), dim3(256), lds, as_stream(stream),
                       (int)F, (int)B, reinterpret_cast<const float2*>(spec),
                       reinterpret_cast<const float2*>(spec2 ? spec2 : spec),
                       reinterpret_cast<const float2*>(tw), ir, ir2 ? ir2 : ir);
    return check_launch("avr_irfft");
}
}  // namespace avr

extern "C" int avr_irfft(int32_t B, int32_t F, const float* spec, const float* tw, float* ir,
                         void* stream) {
    return avr::launch_irfft(B, F, spec, nullptr, tw, ir, nullptr, stream);
}

extern "C" int avr_irfft_bwd(int32_t B, int32_t F, const float* grad_ir, const float* tw,
                             float* grad_spec, void* stream) {
    AVR_REQUIRE(B >= 1 && F >= 2 && grad_ir && tw && grad_spec, "avr_irfft_bwd: bad args");
    const int n = 2 * (F - 1);
    const size_t lds = (size_t)n * (sizeof(float2) + sizeof(float));
    AVR_REQUIRE(lds <= 160 * 1024, "avr_irfft_bwd: n too large for LDS");
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)irfft_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
    hipLaunchKernelGGL(irfft_bwd_kernel, dim3((F + 31) / 32, B), dim3(256), lds, as_stream(stream), (int)F,
                       grad_ir, reinterpret_cast<const float2*>(tw), reinterpret_cast<float2*>(grad_spec));
    return check_launch("avr_irfft_bwd");
}

// ---------------------------------------------------- one-call render core
// weights -> ray reduction -> DFT + phase -> finalize [-> irfft] with one
// host call: the stages above in order on one stream, sized by
// avr_render_core_layout.  Cuts the host issue cost of a pose to one
// ctypes call (the Python path otherwise issues four, each with its own
// allocation and argument marshalling).
namespace {
struct CoreLayout {
    int64_t w, delay, part, spart, bytes;
    int32_t n_split, k_split, P;
};

CoreLayout core_layout(const avr_render_params* p, int B, int sig_dtype) {
    CoreLayout L{};
    const int64_t R = n_rays(*p), S = p->n_samples, T = p->T, F = T / 2 + 1;
    int32_t ns = 1;
    avr_reduce_splits(p, B, sig_dtype, &ns);
    L.n_split = ns;
    const int nkc = (int)((T + kKc - 1) / kKc);
    int ks = 1;
    if (const char* f = getenv("AVR_KSPLIT")) {  // validated tuning knob: DFT k-slices, clamped to [1, T/kKc]
        ks = atoi(f);
    } else {
        const int64_t base = ((F + 127) / 128) * ((S + 31) / 32) * B;
        ks = (int)((256 + (base > 0 ? base : 1) - 1) / (base > 0 ? base : 1));
    }
    if (ks < 1) ks = 1;
    if (ks > nkc) ks = nkc;
    L.k_split = ks;
    L.P = (int32_t)(((S + 31) / 32) * ks);
    auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    int64_t o = 0;
    L.w = o;
    o += al((int64_t)B * R * S * 4);
    L.delay = o;
    o += al((int64_t)B * R * S * 4);
    L.part = o;
    o += al((int64_t)ns * B * S * T * 4);
    L.spart = o;
    o += al((int64_t)B * L.P * F * 8);
    L.bytes = o;
    return L;
}
}  // namespace

extern "C" int avr_render_core_layout(const avr_render_params* p, int32_t B, int32_t sig_dtype,
                                      int64_t* offsets /*[5]: w, delay, part, spart, bytes*/,
                                      int32_t* splits /*[2]: n_split, k_split*/) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(B >= 1 && offsets && splits, "avr_render_core_layout: bad args");
    const CoreLayout L = core_layout(p, B, sig_dtype);
    offsets[0] = L.w;
    offsets[1] = L.delay;
    offsets[2] = L.part;
    offsets[3] = L.spart;
    offsets[4] = L.bytes;
    splits[0] = L.n_split;
    splits[1] = L.k_split;
    return 0;
}

extern "C" int avr_render_core_fwd(const avr_render_params* p, int32_t B, const void* attn,
                                   int32_t attn_dtype, const void* signal, int32_t sig_dtype,
                                   const float* rays_o, const float* pos_tx, const float* dirs,
                                   const avr_table_ptrs* tab, void* workspace,
                                   int64_t workspace_bytes, float* out, float* ir, void* ev_begin,
                                   void* ev_end, void* stream) {
    if (int e = validate(p)) return e;
    AVR_REQUIRE(tab && workspace && out, "avr_render_core_fwd: null pointer");
    const CoreLayout L = core_layout(p, B, sig_dtype);
    AVR_REQUIRE(workspace_bytes >= L.bytes, "avr_render_core_fwd: workspace too small");
    char* ws = reinterpret_cast<char*>(workspace);
    float* w = reinterpret_cast<float*>(ws + L.w);
    int32_t* delay = reinterpret_cast<int32_t*>(ws + L.delay);
    float* part = reinterpret_cast<float*>(ws + L.part);
    float* spart = reinterpret_cast<float*>(ws + L.spart);
    if (int e = avr_weights_fwd(p, B, attn, attn_dtype, rays_o, pos_tx, dirs, tab->d_vals, w, delay, stream))
        return e;
    hipStream_t s = as_stream(stream);
    if (ev_begin) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s);
    if (int e = avr_ray_reduce_fwd(p, B, signal, sig_dtype, w, delay, L.n_split, part, stream))
        return e;
    if (ev_end) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s);
    // DFT + phase, then the fixed-order sum of its partials.  The finalize
    // folded into the DFT's last workgroup per F-block (round 4) was slower in
    // both the serial and the pipelined renders
    if (int e = avr_dft_phase_fwd(p, B, part, L.n_split, tab->pl_table, tab->shift, tab->phase, tab->twiddle,
                                  L.k_split, spart, stream))
        return e;
    if (int e = avr_spectrum_finalize(B, L.P, p->T / 2 + 1, spart, out, stream)) return e;
    if (ir) {
        AVR_REQUIRE(tab->ir_twiddle, "avr_render_core_fwd: ir requested without ir_twiddle");
        return avr_irfft(B, p->T / 2 + 1, out, tab->ir_twiddle, ir, stream);
    }
    return 0;
}
