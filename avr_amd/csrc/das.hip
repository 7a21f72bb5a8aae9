// das.hip — the delay-and-sum (DAS) direction terms of the training loss
// (utils/criterion.py:35-67 compute_beamforming_power, :100-122 losses) on
// gfx950, forward and backward.
//
// Input: the 8 channels' impulse responses pred_time / ori_time [8][n]
// (irfft of the rendered / measured spectra, the criterion's first launch).
//   X[m][f]    = rfft(time[m], n=512)[f], f < 257   (truncated / zero-padded)
//   beam[k][f] = sum_m X[m][f] * steer[k][m][f] / 8   (k = 360 look directions)
//   bp = |beam|^2,  bpn[k][f] = bp / (sum_k bp + 1e-8),  power[k] = sum_f bpn
//   ce  = cross_entropy(power_pred, argmax power_ori) * w_ce
//   reg = (|sin a_p - sin a_o| + |cos a_p - cos a_o|) * w_reg,
//         a = sum_k softmax(beta * power)_k * theta_k
// steer[k][m][f] = exp(-i 2 pi delay[k][m] freq[f]) is a host-built table
// (the reference's own torch ops, criterion.py:55-60), cached per device.
//
// Launches: das_spectrum_kernel (16 workgroups: one per channel and signal),
// das_power_kernel (one workgroup per 16 frequencies and signal: all 360
// directions, partial powers), das_loss_kernel (one workgroup).  Backward:
// das_bwd_beam_kernel (dL/dX per frequency tile) and das_bwd_time_kernel
// (adjoint rfft).  Fixed summation orders throughout.
#include <math.h>

#include "common.h"

using namespace avr;

namespace {

constexpr int kMics = 8;      // criterion.py:41 asserts M == 8
constexpr int kDirs = 360;    // criterion.py:24, one-degree look directions
constexpr int kNfft = 512;    // criterion.py:43
constexpr int kBins = kNfft / 2 + 1;
constexpr int kFTile = 16;
constexpr int kFTiles = (kBins + kFTile - 1) / kFTile;  // 17
constexpr int kThreads = 256;

struct DasWs {
    float2* X;      // [2][8][257]
    float* ppart;   // [2][kFTiles][360]
    float* power;   // [2][360]
    float2* GX;     // [8][257]
    int64_t bytes;
};

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

DasWs carve(void* base) {
    DasWs W{};
    char* p = reinterpret_cast<char*>(base);
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        char* r = p ? p + o : nullptr;
        o += align16(bytes);
        return r;
    };
    W.X = reinterpret_cast<float2*>(take(2 * kMics * kBins * sizeof(float2)));
    W.ppart = reinterpret_cast<float*>(take(2 * kFTiles * kDirs * 4));
    W.power = reinterpret_cast<float*>(take(2 * kDirs * 4));
    W.GX = reinterpret_cast<float2*>(take(kMics * kBins * sizeof(float2)));
    W.bytes = o;
    return W;
}

__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }

// X[s][m][f] = sum_{t < min(n, 512)} time[m][t] e^{-2 pi i f t / 512}
__global__ __launch_bounds__(kThreads) void das_spectrum_kernel(int n,
                                                                const float* __restrict__ ptime,
                                                                const float* __restrict__ otime,
                                                                const float2* __restrict__ tw,
                                                                DasWs W) {
    __shared__ float2 stw[kNfft];
    __shared__ float x[kNfft];
    const int m = blockIdx.x, s = blockIdx.y;
    const float* src = (s ? otime : ptime) + (int64_t)m * n;
    const int L = min(n, kNfft);
    for (int i = threadIdx.x; i < kNfft; i += kThreads) {
        stw[i] = tw[i];
        x[i] = i < L ? src[i] : 0.f;
    }
    __syncthreads();
    for (int f = threadIdx.x; f < kBins; f += kThreads) {
        float re = 0.f, im = 0.f;
        int j = 0;
        for (int t = 0; t < L; ++t) {
            const float2 c = stw[j];
            re = fmaf(x[t], c.x, re);
            im = fmaf(-x[t], c.y, im);
            j = (j + f) & (kNfft - 1);
        }
        W.X[((int64_t)s * kMics + m) * kBins + f] = make_float2(re, im);
    }
}

// beam power for 16 frequencies x 360 directions of one signal, normalised
// over directions per frequency, summed over the tile's frequencies.
__global__ __launch_bounds__(kThreads) void das_power_kernel(const float2* __restrict__ steer,
                                                             DasWs W) {
    __shared__ float2 xs[kMics][kFTile];
    __shared__ float bp[kDirs][kFTile + 1];
    __shared__ float inv[kFTile];
    const int tile = blockIdx.x, s = blockIdx.y;
    const int f0 = tile * kFTile;
    const int nf = min(kFTile, kBins - f0);
    for (int i = threadIdx.x; i < kMics * kFTile; i += kThreads) {
        const int m = i / kFTile, j = i % kFTile;
        xs[m][j] = j < nf ? W.X[((int64_t)s * kMics + m) * kBins + f0 + j] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kDirs * kFTile; i += kThreads) {
        const int k = i / kFTile, j = i % kFTile;
        float re = 0.f, im = 0.f;
        if (j < nf) {
#pragma unroll
            for (int m = 0; m < kMics; ++m) {
                const float2 a = xs[m][j];
                const float2 b = steer[((int64_t)k * kMics + m) * kBins + f0 + j];
                re += a.x * b.x - a.y * b.y;
                im += a.x * b.y + a.y * b.x;
            }
            re /= (float)kMics;
            im /= (float)kMics;
        }
        const float mag = hypotf(re, im);
        bp[k][j] = mag * mag;
    }
    __syncthreads();
    if (threadIdx.x < kFTile) {
        const int j = threadIdx.x;
        float sum = 0.f;
        for (int k = 0; k < kDirs; ++k) sum += bp[k][j];
        inv[j] = sum + 1e-8f;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kDirs; k += kThreads) {
        float p = 0.f;
        for (int j = 0; j < nf; ++j) p += bp[k][j] / inv[j];
        W.ppart[((int64_t)s * kFTiles + tile) * kDirs + k] = p;
    }
}

__device__ __forceinline__ float block_max(float v, float* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int st = 256; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int st = 256; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}

struct DasStats {
    int target;           // argmax power_ori (first maximum)
    float lse_ce;         // logsumexp(power_pred)
    float mx_p, sum_p;    // softmax(beta * power_pred) normaliser
    float a_p, a_o;       // softmax-weighted angles
};

// All 512 lanes: power = sum of tile partials, then the statistics of both
// loss terms.  theta_k = deg2rad(k) from the host table `angles`.
__device__ DasStats das_stats(const DasWs& W, const float* __restrict__ angles, float beta,
                              float* pw /*[2][360] LDS*/, float* red, int* redi) {
    for (int i = threadIdx.x; i < 2 * kDirs; i += blockDim.x) {
        const int s = i / kDirs, k = i % kDirs;
        float p = 0.f;
        for (int t = 0; t < kFTiles; ++t) p += W.ppart[((int64_t)s * kFTiles + t) * kDirs + k];
        pw[i] = p;
    }
    __syncthreads();
    DasStats st;
    const int k = threadIdx.x;
    const bool live = k < kDirs;
    // argmax of power_ori, first index among equal maxima
    const float vo = live ? pw[kDirs + k] : -INFINITY;
    const float mo = block_max(vo, red);
    redi[threadIdx.x] = (live && vo == mo) ? k : kDirs;
    __syncthreads();
    for (int s2 = 256; s2 > 0; s2 >>= 1) {
        if ((int)threadIdx.x < s2) redi[threadIdx.x] = min(redi[threadIdx.x], redi[threadIdx.x + s2]);
        __syncthreads();
    }
    st.target = redi[0];
    __syncthreads();
    // log-sum-exp of power_pred (cross entropy)
    const float vp = live ? pw[k] : -INFINITY;
    const float mp = block_max(vp, red);
    const float se = block_sum(live ? expf(vp - mp) : 0.f, red);
    st.lse_ce = mp + logf(se);
    // softmax(beta * power) angle averages
    const float zp = live ? beta * pw[k] : -INFINITY;
    const float zo = live ? beta * pw[kDirs + k] : -INFINITY;
    st.mx_p = block_max(zp, red);
    const float mxo = block_max(zo, red);
    const float ep = live ? expf(zp - st.mx_p) : 0.f;
    const float eo = live ? expf(zo - mxo) : 0.f;
    st.sum_p = block_sum(ep, red);
    const float so = block_sum(eo, red);
    const float th = live ? angles[k] : 0.f;
    st.a_p = block_sum(ep / st.sum_p * th, red);
    st.a_o = block_sum(eo / so * th, red);
    return st;
}

__global__ __launch_bounds__(512) void das_loss_kernel(const float* __restrict__ angles,
                                                       float beta, float w_reg, float w_ce,
                                                       DasWs W, float* __restrict__ losses) {
    __shared__ float pw[2 * kDirs];
    __shared__ float red[512];
    __shared__ int redi[512];
    const DasStats st = das_stats(W, angles, beta, pw, red, redi);
    if (threadIdx.x < 2 * kDirs) W.power[threadIdx.x] = pw[threadIdx.x];
    if (threadIdx.x == 0) {
        const float ce = st.lse_ce - pw[st.target];
        const float reg = fabsf(sinf(st.a_p) - sinf(st.a_o)) + fabsf(cosf(st.a_p) - cosf(st.a_o));
        losses[0] = w_reg > 0.f ? reg * w_reg : 0.f;
        losses[1] = w_ce > 0.f ? ce * w_ce : 0.f;
    }
}

// dL/dpower_pred[k] for upstream grads g[0] (reg) and g[1] (ce).
__device__ __forceinline__ float dpower(const DasStats& st, const float* pw, int k,
                                        const float* angles, float beta, float w_reg, float w_ce,
                                        const float* g) {
    float d = 0.f;
    if (w_ce > 0.f) {
        const float sm = expf(pw[k] - st.lse_ce);
        d += g[1] * w_ce * (sm - (k == st.target ? 1.f : 0.f));
    }
    if (w_reg > 0.f) {
        const float da = g[0] * w_reg *
                         (sgnf(sinf(st.a_p) - sinf(st.a_o)) * cosf(st.a_p) -
                          sgnf(cosf(st.a_p) - cosf(st.a_o)) * sinf(st.a_p));
        const float sk = expf(beta * pw[k] - st.mx_p) / st.sum_p;
        d += da * beta * sk * (angles[k] - st.a_p);
    }
    return d;
}

// dL/dX_pred[m][f] for the tile's frequencies (recomputes the beams).
__global__ __launch_bounds__(512) void das_bwd_beam_kernel(const float2* __restrict__ steer,
                                                           const float* __restrict__ angles,
                                                           float beta, float w_reg, float w_ce,
                                                           const float* __restrict__ g, DasWs W) {
    __shared__ float pw[2 * kDirs];
    __shared__ float red[512];
    __shared__ int redi[512];
    __shared__ float gp[kDirs];
    __shared__ float2 xs[kMics][kFTile];
    __shared__ float2 beam[kDirs][kFTile];
    __shared__ float sinv[kFTile], dot[kFTile];
    const DasStats st = das_stats(W, angles, beta, pw, red, redi);
    const float gl[2] = {g[0], g[1]};
    for (int k = threadIdx.x; k < kDirs; k += blockDim.x)
        gp[k] = dpower(st, pw, k, angles, beta, w_reg, w_ce, gl);
    const int tile = blockIdx.x;
    const int f0 = tile * kFTile;
    const int nf = min(kFTile, kBins - f0);
    for (int i = threadIdx.x; i < kMics * kFTile; i += blockDim.x) {
        const int m = i / kFTile, j = i % kFTile;
        xs[m][j] = j < nf ? W.X[(int64_t)m * kBins + f0 + j] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kDirs * kFTile; i += blockDim.x) {
        const int k = i / kFTile, j = i % kFTile;
        float re = 0.f, im = 0.f;
        if (j < nf) {
#pragma unroll
            for (int m = 0; m < kMics; ++m) {
                const float2 a = xs[m][j];
                const float2 b = steer[((int64_t)k * kMics + m) * kBins + f0 + j];
                re += a.x * b.x - a.y * b.y;
                im += a.x * b.y + a.y * b.x;
            }
            re /= (float)kMics;
            im /= (float)kMics;
        }
        beam[k][j] = make_float2(re, im);
    }
    __syncthreads();
    if (threadIdx.x < kFTile) {
        const int j = threadIdx.x;
        float sum = 0.f, d = 0.f;
        for (int k = 0; k < kDirs; ++k) {
            const float mag = hypotf(beam[k][j].x, beam[k][j].y);
            sum += mag * mag;
        }
        const float S = sum + 1e-8f;
        for (int k = 0; k < kDirs; ++k) {
            const float mag = hypotf(beam[k][j].x, beam[k][j].y);
            d += gp[k] * (mag * mag / S);
        }
        sinv[j] = 1.0f / S;
        dot[j] = d;
    }
    __syncthreads();
    // dL/dbp[k][f] = (gp[k] - sum_j gp[j] bpn[j][f]) / S_f;  dL/dbeam = 2 dL/dbp beam;
    // dL/dX[m][f] = sum_k dL/dbeam[k][f] conj(steer[k][m][f]) / 8
    for (int i = threadIdx.x; i < kMics * kFTile; i += blockDim.x) {
        const int m = i / kFTile, j = i % kFTile;
        if (j >= nf) continue;
        float re = 0.f, im = 0.f;
        for (int k = 0; k < kDirs; ++k) {
            const float gbp = (gp[k] - dot[j]) * sinv[j];
            const float2 bm = beam[k][j];
            const float gr = 2.f * gbp * bm.x, gi = 2.f * gbp * bm.y;
            const float2 b = steer[((int64_t)k * kMics + m) * kBins + f0 + j];
            // (gr + i gi) * conj(b)
            re += gr * b.x + gi * b.y;
            im += gi * b.x - gr * b.y;
        }
        W.GX[(int64_t)m * kBins + f0 + j] = make_float2(re / (float)kMics, im / (float)kMics);
    }
}

// grad_time[m][t] = sum_f Re(GX) cos(2 pi f t/512) - Im(GX) sin(...), t < 512
__global__ __launch_bounds__(kThreads) void das_bwd_time_kernel(int n,
                                                                const float2* __restrict__ tw,
                                                                DasWs W,
                                                                float* __restrict__ grad_time) {
    __shared__ float2 stw[kNfft];
    __shared__ float2 gx[kBins];
    const int m = blockIdx.x;
    for (int i = threadIdx.x; i < kNfft; i += kThreads) stw[i] = tw[i];
    for (int i = threadIdx.x; i < kBins; i += kThreads) gx[i] = W.GX[(int64_t)m * kBins + i];
    __syncthreads();
    for (int t = threadIdx.x; t < n; t += kThreads) {
        float acc = 0.f;
        if (t < kNfft) {
            int j = 0;
            for (int f = 0; f < kBins; ++f) {
                const float2 c = stw[j];
                acc = fmaf(gx[f].x, c.x, acc);
                acc = fmaf(-gx[f].y, c.y, acc);
                j = (j + t) & (kNfft - 1);
            }
        }
        grad_time[(int64_t)m * n + t] = acc;
    }
}

}  // namespace

extern "C" int avr_das_workspace(int64_t* bytes) {
    AVR_REQUIRE(bytes, "avr_das_workspace: null bytes");
    *bytes = carve(nullptr).bytes;
    return 0;
}

extern "C" int avr_das_fwd(int32_t n, const float* pred_time, const float* ori_time,
                           const float* steer, const float* angles, const float* tw512,
                           float beta, float w_reg, float w_ce, float* losses, void* ws,
                           int64_t ws_bytes, void* stream) {
    AVR_REQUIRE(n >= 2 && pred_time && ori_time && steer && angles && tw512 && losses && ws,
                "avr_das_fwd: bad args");
    DasWs W = carve(ws);
    AVR_REQUIRE(ws_bytes >= W.bytes, "avr_das_fwd: workspace too small");
    hipLaunchKernelGGL(das_spectrum_kernel, dim3(kMics, 2), dim3(kThreads), 0, as_stream(stream),
                       (int)n, pred_time, ori_time, reinterpret_cast<const float2*>(tw512), W);
    if (int e = check_launch("das_spectrum_kernel")) return e;
    hipLaunchKernelGGL(das_power_kernel, dim3(kFTiles, 2), dim3(kThreads), 0, as_stream(stream),
                       reinterpret_cast<const float2*>(steer), W);
    if (int e = check_launch("das_power_kernel")) return e;
    hipLaunchKernelGGL(das_loss_kernel, dim3(1), dim3(512), 0, as_stream(stream), angles, beta,
                       w_reg, w_ce, W, losses);
    return check_launch("das_loss_kernel");
}

extern "C" int avr_das_bwd(int32_t n, const float* steer, const float* angles,
                           const float* tw512, float beta, float w_reg, float w_ce,
                           const float* grad_losses, void* ws, int64_t ws_bytes,
                           float* grad_pred_time, void* stream) {
    AVR_REQUIRE(n >= 2 && steer && angles && tw512 && grad_losses && ws && grad_pred_time,
                "avr_das_bwd: bad args");
    DasWs W = carve(ws);
    AVR_REQUIRE(ws_bytes >= W.bytes, "avr_das_bwd: workspace too small");
    hipLaunchKernelGGL(das_bwd_beam_kernel, dim3(kFTiles), dim3(512), 0, as_stream(stream),
                       reinterpret_cast<const float2*>(steer), angles, beta, w_reg, w_ce,
                       grad_losses, W);
    if (int e = check_launch("das_bwd_beam_kernel")) return e;
    hipLaunchKernelGGL(das_bwd_time_kernel, dim3(kMics), dim3(kThreads), 0, as_stream(stream),
                       (int)n, reinterpret_cast<const float2*>(tw512), W, grad_pred_time);
    return check_launch("das_bwd_time_kernel");
}
