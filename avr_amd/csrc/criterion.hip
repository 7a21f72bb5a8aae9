// criterion.hip — the training loss of the reference (utils/criterion.py:69-98)
// on gfx950, forward and backward, for the rendered spectra [B][F][2].
//
// Terms (weights w_* from the `train:` config, criterion.py:11-16):
//   spec   = (L1(Re p, Re o) + L1(Im p, Im o)) * w_spec          (:85-87)
//   amp    = L1(|p|, |o|) * w_amp                                 (:89)
//   angle  = (L1(cos∠p, cos∠o) + L1(sin∠p, sin∠o)) * w_angle      (:91-92)
//   time   = L1(irfft o, irfft p) * w_time                        (:71-72, 94)
//   energy = L1(EDC(o), EDC(p)) * w_energy, EDC = log10 of the reversed
//            cumulative sum of squared |STFT_256|^2 frame energies (:74-83, 96)
//   mrstft = auraloss MultiResolutionSTFTLoss(ori_time, pred_time) * w_mr (:33, 98)
//            (fft 512/256/128/64, hann 300/150/75/30, hop 60/30/8/4;
//             sc + log-mag L1 + lin-mag L1 per resolution, mean of the four)
//
// Launches: forward = irfft (both spectra, one launch) + crit_stft_kernel
// (all five STFTs of both signals: direct DFT of each frame against a
// 512-entry twiddle table in LDS, per-tile partial sums of the MR-STFT terms
// and per-frame energies, fixed-order) + crit_reduce_kernel (one workgroup:
// spectral/time sums, per-item norms, energy decay curves, final losses, and
// the unit gradient of the energy term).  Backward = crit_bwd_frames_kernel
// (dL/dX per STFT bin, then each frame's adjoint DFT) + crit_bwd_time_kernel
// (overlap-add of the frame adjoints through the reflect padding, plus the
// time term) + crit_bwd_spec_kernel (adjoint irfft plus the spectral terms).
// Every sum is in a fixed order: results are deterministic.
#include <math.h>

#include "common.h"

using namespace avr;

namespace {

constexpr int kNRes = 5;    // 4 MR-STFT resolutions + the energy STFT (criterion.py:74)
constexpr int kEnergy = 4;  // index of the energy STFT
constexpr int kTw = 512;    // twiddle table length; every n_fft divides it
constexpr int kThreads = 256;
constexpr float kMagEps = 1e-8f;  // auraloss STFTLoss eps

// criterion.py:33 and :74 (torch.stft defaults: hop n_fft/4, rectangular window)
constexpr int kNfft[kNRes] = {512, 256, 128, 64, 256};
constexpr int kWin[kNRes] = {300, 150, 75, 30, 256};
constexpr int kHop[kNRes] = {60, 30, 8, 4, 64};
// frames per workgroup: forward ~2 (frame, bin) items per lane, backward ~2
// (frame, tap) items per lane
constexpr int kFptF[kNRes] = {2, 4, 8, 16, 4};
constexpr int kFptB[kNRes] = {1, 3, 6, 17, 2};
constexpr int kSpanMax = 576;   // max (fpt_f-1)*hop + n_fft
constexpr int kItemsF = 528;    // max fpt_f * K
constexpr int kItemsG = 561;    // max fpt_b * K
constexpr int kWinMax = 300;

struct CritRes {
    int N, win, hop, off, K, M;
    int fpt_f, tile_f;  // forward tiles of this resolution start at tile_f
    int fpt_b, tile_b;  // backward tiles
    int xoff;           // offset of this resolution in a signal's X row
    int yoff;           // offset in a signal's Y row
    int woff;           // offset in the window table
};

struct CritPlan {
    int B, F, n;
    int tiles_f, tiles_b;  // per signal
    int NX, NY, M4;
    float w[6];  // spec, amp, angle, time, energy, mrstft weights
    CritRes r[kNRes];
};

struct CritWs {
    float2* X;     // [2][B][NX] STFT bins of pred (0) and ori (1)
    float* Y;      // [B][NY] frame adjoints
    float* e;      // [2][B][M4] energy-STFT frame energies
    float* part;   // [B][tiles_f(MR)][4] MR-STFT partial sums
    float* stat;   // [B][4][4] MR-STFT sums per (item, resolution)
    float* ge;     // [B][M4] d energy_loss / d e_pred (unit upstream)
    float* gtime;  // [B][n] d loss / d pred_time
    int64_t bytes;
};

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

int make_plan(int B, int F, const float* w, CritPlan* P) {
    AVR_REQUIRE(B >= 1 && F >= 2, "avr_criterion: B >= 1 and F >= 2 required");
    const int n = 2 * (F - 1);
    AVR_REQUIRE(n <= 12288, "avr_criterion: IR length must be <= 12288");
    // torch.stft(center=True) reflect-pads n_fft/2 samples on each side
    if (n <= kNfft[0] / 2)
        return fail(AVR_E_CONFIG,
                    "avr_criterion: Padding size should be less than the corresponding input "
                    "dimension (IR length must exceed 256 for the 512-point STFT)");
    P->B = B;
    P->F = F;
    P->n = n;
    int tf = 0, tb = 0, nx = 0, ny = 0, wo = 0;
    for (int q = 0; q < kNRes; ++q) {
        CritRes& r = P->r[q];
        r.N = kNfft[q];
        r.win = kWin[q];
        r.hop = kHop[q];
        r.off = (r.N - r.win) / 2;  // torch.stft centres a short window in n_fft
        r.K = r.N / 2 + 1;
        r.M = 1 + n / r.hop;
        r.fpt_f = kFptF[q];
        r.tile_f = tf;
        tf += (r.M + r.fpt_f - 1) / r.fpt_f;
        r.fpt_b = kFptB[q];
        r.tile_b = tb;
        tb += (r.M + r.fpt_b - 1) / r.fpt_b;
        r.xoff = nx;
        nx += r.K * r.M;
        r.yoff = ny;
        ny += r.M * r.win;
        r.woff = wo;
        wo += r.win;
    }
    P->tiles_f = tf;
    P->tiles_b = tb;
    P->NX = nx;
    P->NY = ny;
    P->M4 = P->r[kEnergy].M;
    for (int i = 0; i < 6; ++i) P->w[i] = w ? w[i] : 1.0f;
    return 0;
}

// Window table length (concatenated hann windows of the MR resolutions and
// the rectangular energy window).
int window_len() {
    int s = 0;
    for (int q = 0; q < kNRes; ++q) s += kWin[q];
    return s;
}

CritWs carve(const CritPlan& P, void* base) {
    CritWs W{};
    char* p = reinterpret_cast<char*>(base);
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        char* r = p ? p + o : nullptr;
        o += align16(bytes);
        return r;
    };
    const int64_t B = P.B;
    const int mr_tiles = P.r[kEnergy].tile_f;
    W.X = reinterpret_cast<float2*>(take(2 * B * P.NX * (int64_t)sizeof(float2)));
    W.Y = reinterpret_cast<float*>(take(B * P.NY * 4));
    W.e = reinterpret_cast<float*>(take(2 * B * P.M4 * 4));
    W.part = reinterpret_cast<float*>(take(B * mr_tiles * 4 * 4));
    W.stat = reinterpret_cast<float*>(take(B * 16 * 4));
    W.ge = reinterpret_cast<float*>(take(B * P.M4 * 4));
    W.gtime = reinterpret_cast<float*>(take(B * (int64_t)P.n * 4));
    W.bytes = o;
    return W;
}

__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }

__device__ __forceinline__ int find_res(const CritPlan& P, int tile, bool fwd) {
    int q = 0;
#pragma unroll
    for (int i = 1; i < kNRes; ++i)
        if (tile >= (fwd ? P.r[i].tile_f : P.r[i].tile_b)) q = i;
    return q;
}

// reflect padding of torch.stft(center=True): padded index j -> sample index
__device__ __forceinline__ int reflect(int j, int pad, int n) {
    int t = j - pad;
    if (t < 0) t = -t;
    if (t >= n) t = 2 * (n - 1) - t;
    return t;
}

template <int N>
__device__ __forceinline__ void block_sum(float (*red)[kThreads], float* v) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int c = 0; c < N; ++c) red[c][tid] = v[c];
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if (tid < s) {
#pragma unroll
            for (int c = 0; c < N; ++c) red[c][tid] += red[c][tid + s];
        }
        __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = red[c][0];
}

// ---------------------------------------------------------------- forward
// One workgroup = fpt_f consecutive frames of one resolution of item b, for
// the predicted and the measured signal together (the MR terms need both
// magnitudes of a bin).  Lanes own (frame, bin) items; each walks the
// window taps with an incremental twiddle index (k*(tap+off)) mod n_fft.
__global__ __launch_bounds__(kThreads) void crit_stft_kernel(CritPlan P,
                                                             const float* __restrict__ ptime,
                                                             const float* __restrict__ otime,
                                                             const float* __restrict__ wtab,
                                                             const float2* __restrict__ tw,
                                                             CritWs W) {
    __shared__ float2 stw[kTw];
    __shared__ float swin[kWinMax > 256 ? kWinMax : 256];
    __shared__ float xs[2][kSpanMax];
    __shared__ float en[2][kItemsF];
    __shared__ float red[4][kThreads];
    const int tid = threadIdx.x;
    const int b = blockIdx.y, tile = blockIdx.x;
    const int q = find_res(P, tile, true);
    const CritRes R = P.r[q];
    const int n = P.n, B = P.B;
    const int m0 = (tile - R.tile_f) * R.fpt_f;
    const int nf = min(R.fpt_f, R.M - m0);
    const int span = (nf - 1) * R.hop + R.N;
    const int j0 = m0 * R.hop;
    const int pad = R.N / 2;
    for (int i = tid; i < kTw; i += kThreads) stw[i] = tw[i];
    for (int i = tid; i < R.win; i += kThreads) swin[i] = wtab[R.woff + i];
    for (int i = tid; i < 2 * span; i += kThreads) {
        const int s = i >= span, j = i - s * span;
        xs[s][j] = (s ? otime : ptime)[(int64_t)b * n + reflect(j0 + j, pad, n)];
    }
    __syncthreads();
    const int stride = kTw / R.N;
    const int items = nf * R.K;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int it = tid; it < items; it += kThreads) {
        const int mi = it / R.K, k = it - mi * R.K;
        const int base = mi * R.hop + R.off;
        const int step = (k * stride) & (kTw - 1);
        int jj = (k * R.off * stride) & (kTw - 1);
        float pr = 0.f, pi = 0.f, orr = 0.f, oi = 0.f;
        for (int t = 0; t < R.win; ++t) {
            const float wv = swin[t];
            const float vp = wv * xs[0][base + t];
            const float vo = wv * xs[1][base + t];
            const float2 c = stw[jj];
            pr = fmaf(vp, c.x, pr);
            pi = fmaf(-vp, c.y, pi);
            orr = fmaf(vo, c.x, orr);
            oi = fmaf(-vo, c.y, oi);
            jj = (jj + step) & (kTw - 1);
        }
        const int64_t xi = R.xoff + (int64_t)(m0 + mi) * R.K + k;
        W.X[(int64_t)b * P.NX + xi] = make_float2(pr, pi);
        W.X[((int64_t)B + b) * P.NX + xi] = make_float2(orr, oi);
        const float sp = pr * pr + pi * pi;
        const float so = orr * orr + oi * oi;
        if (q < kEnergy) {
            // auraloss: mag = sqrt(clamp(re^2 + im^2, min=eps)); x = ori, y = pred
            const float p = sqrtf(sp < kMagEps ? kMagEps : sp);
            const float o = sqrtf(so < kMagEps ? kMagEps : so);
            const float d = p - o;
            acc[0] += d * d;
            acc[1] += p * p;
            acc[2] += fabsf(logf(o) - logf(p));
            acc[3] += fabsf(o - p);
        } else {
            en[0][it] = sp;
            en[1][it] = so;
        }
    }
    if (q < kEnergy) {
        block_sum<4>(red, acc);
        if (tid < 4) W.part[((int64_t)b * P.r[kEnergy].tile_f + tile) * 4 + tid] = acc[tid];
    } else {
        __syncthreads();
        if (tid < 2 * nf) {
            const int s = tid / nf, mi = tid - s * nf;
            float sum = 0.f;
            for (int k = 0; k < R.K; ++k) sum += en[s][mi * R.K + k];
            W.e[((int64_t)s * B + b) * P.M4 + m0 + mi] = sum;
        }
    }
}

// One workgroup of 1024 lanes: every remaining sum, the losses, and the
// statistics the backward needs.  losses[6] = spec, amp, angle, time,
// energy, mrstft (weighted as criterion.py does).
constexpr int kRedThreads = 1024;
__global__ __launch_bounds__(kRedThreads) void crit_reduce_kernel(CritPlan P,
                                                                  const float2* __restrict__ pred,
                                                                  const float2* __restrict__ ori,
                                                                  const float* __restrict__ pt,
                                                                  const float* __restrict__ ot,
                                                                  CritWs W,
                                                                  float* __restrict__ losses,
                                                                  float* __restrict__ total) {
    __shared__ float red[6][kRedThreads];
    __shared__ float qsum[4][3];
    const int tid = threadIdx.x;
    const int B = P.B, F = P.F, n = P.n;
    // ---- spectral and time-domain L1 sums
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = tid; i < B * F; i += kRedThreads) {
        const float2 p = pred[i], o = ori[i];
        s[0] += fabsf(p.x - o.x);
        s[1] += fabsf(p.y - o.y);
        s[2] += fabsf(hypotf(p.x, p.y) - hypotf(o.x, o.y));
        const float tp = atan2f(p.y, p.x), to = atan2f(o.y, o.x);
        s[3] += fabsf(cosf(tp) - cosf(to));
        s[4] += fabsf(sinf(tp) - sinf(to));
    }
    for (int i = tid; i < B * n; i += kRedThreads) s[5] += fabsf(ot[i] - pt[i]);
#pragma unroll
    for (int c = 0; c < 6; ++c) red[c][tid] = s[c];
    __syncthreads();
    for (int st = kRedThreads / 2; st > 0; st >>= 1) {
        if (tid < st) {
#pragma unroll
            for (int c = 0; c < 6; ++c) red[c][tid] += red[c][tid + st];
        }
        __syncthreads();
    }
    float tot[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) tot[c] = red[c][0];
    __syncthreads();
    // ---- MR-STFT: per (item, resolution) sums over that pair's tiles
    const int mr_tiles = P.r[kEnergy].tile_f;
    if (tid < 4 * B) {
        const int b = tid >> 2, q = tid & 3;
        const int t0 = P.r[q].tile_f, t1 = P.r[q + 1].tile_f;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        for (int t = t0; t < t1; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] += W.part[((int64_t)b * mr_tiles + t) * 4 + c];
#pragma unroll
        for (int c = 0; c < 4; ++c) W.stat[(b * 4 + q) * 4 + c] = a[c];
    }
    __threadfence_block();
    __syncthreads();
    if (tid < 4) {
        const int q = tid;
        float sc = 0.f, lg = 0.f, ln = 0.f;
        for (int b = 0; b < B; ++b) {
            const float* st = W.stat + (b * 4 + q) * 4;
            sc += sqrtf(st[0]) / sqrtf(st[1]);
            lg += st[2];
            ln += st[3];
        }
        const float cnt = (float)B * (float)P.r[q].K * (float)P.r[q].M;
        qsum[q][0] = sc / (float)B;
        qsum[q][1] = lg / cnt;
        qsum[q][2] = ln / cnt;
    }
    // ---- energy decay curves (criterion.py:80-83), one lane per item
    const int M = P.M4;
    if (tid < B) {
        const int b = tid;
        const float* ep = W.e + (int64_t)b * M;
        const float* eo = W.e + ((int64_t)B + b) * M;
        float* g = W.ge + (int64_t)b * M;  // scratch: reversed cumsums, then grads
        // C_m = sum_{j>=m} e_j^2, accumulated from the end (flip, cumsum, flip)
        float cp = 0.f, co = 0.f;
        float* cbuf = W.gtime + (int64_t)b * P.n;  // [2][M] scratch (gtime is free until bwd)
        for (int m = M - 1; m >= 0; --m) {
            cp += ep[m] * ep[m];
            co += eo[m] * eo[m];
            cbuf[m] = cp;
            cbuf[M + m] = co;
        }
        const float lp0 = log10f(cbuf[0] + 1e-9f), lo0 = log10f(cbuf[M] + 1e-9f);
        float sum = 0.f, ssum = 0.f;
        const float inv = 1.0f / ((float)B * (float)M);
        for (int m = 0; m < M; ++m) {
            const float Ep = log10f(cbuf[m] + 1e-9f) - lp0;
            const float Eo = log10f(cbuf[M + m] + 1e-9f) - lo0;
            sum += fabsf(Eo - Ep);
            const float sm = sgnf(Ep - Eo) * inv;
            g[m] = sm;  // d loss / d E_m
            ssum += sm;
        }
        // dL/dL_j = s_j - [j == 0] * sum_m s_m;  dL/dC_m = that / ((C_m + 1e-9) ln 10)
        // dL/d(e_j^2) = sum_{m <= j} dL/dC_m;  dL/de_j = 2 e_j * that
        const float ln10 = 2.302585092994046f;
        float run = 0.f;
        for (int m = 0; m < M; ++m) {
            const float gl = g[m] - (m == 0 ? ssum : 0.f);
            run += gl / ((cbuf[m] + 1e-9f) * ln10);
            g[m] = 2.0f * ep[m] * run;
        }
        cbuf[0] = sum;  // per-item energy L1 sum, combined below in item order
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {
        float esum_all = 0.f;
        for (int b = 0; b < B; ++b) esum_all += W.gtime[(int64_t)b * P.n];
        const float nbf = (float)B * (float)F;
        float l[8];
        l[0] = (tot[0] / nbf + tot[1] / nbf) * P.w[0];
        l[1] = (tot[2] / nbf) * P.w[1];
        l[2] = (tot[3] / nbf + tot[4] / nbf) * P.w[2];
        l[3] = (tot[5] / ((float)B * (float)n)) * P.w[3];
        l[4] = (esum_all / ((float)B * (float)M)) * P.w[4];
        float mr = 0.f;
        for (int q = 0; q < 4; ++q) mr += (qsum[q][0] + qsum[q][1]) + qsum[q][2];
        l[5] = (mr / 4.0f) * P.w[5];
        l[6] = 0.f;  // DAS terms (criterion.py:101-102), filled by the DAS kernels
        l[7] = 0.f;
        float t = l[0];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            losses[i] = l[i];
            if (i > 0) t += l[i];  // left to right, as avr_runner.py:187 adds them
        }
        if (total) *total = t;
    }
}

// --------------------------------------------------------------- backward
// dL/dX for every bin of fpt_b frames, then each frame's adjoint DFT:
//   Y[m][t] = win[t] * sum_k Re(G_k) cos(2 pi k (t+off)/N) - Im(G_k) sin(...)
__global__ __launch_bounds__(kThreads) void crit_bwd_frames_kernel(
    CritPlan P, const float* __restrict__ wtab, const float2* __restrict__ tw,
    const float* __restrict__ gloss, CritWs W) {
    __shared__ float2 stw[kTw];
    __shared__ float swin[kWinMax > 256 ? kWinMax : 256];
    __shared__ float2 sg[kItemsG];
    const int tid = threadIdx.x;
    const int b = blockIdx.y, tile = blockIdx.x;
    const int q = find_res(P, tile, false);
    const CritRes R = P.r[q];
    const int B = P.B;
    const int m0 = (tile - R.tile_b) * R.fpt_b;
    const int nf = min(R.fpt_b, R.M - m0);
    for (int i = tid; i < kTw; i += kThreads) stw[i] = tw[i];
    for (int i = tid; i < R.win; i += kThreads) swin[i] = wtab[R.woff + i];
    float c_sc1 = 0.f, c_sc2 = 0.f, c_n = 0.f, gm = 0.f;
    if (q < kEnergy) {
        const float* st = W.stat + (b * 4 + q) * 4;
        const float A = sqrtf(st[0]), Bn = sqrtf(st[1]);
        gm = gloss[5] * P.w[5] / 4.0f;
        // d(A/Bn)/dp = (p-o)/(A Bn) - A p / Bn^3, averaged over items
        c_sc1 = A > 0.f ? 1.0f / (A * Bn * (float)B) : 0.f;
        c_sc2 = A / (Bn * Bn * Bn * (float)B);
        c_n = 1.0f / ((float)B * (float)R.K * (float)R.M);
    }
    const float gE = gloss[4] * P.w[4];
    for (int it = tid; it < nf * R.K; it += kThreads) {
        const int mi = it / R.K, k = it - mi * R.K;
        const int64_t xi = R.xoff + (int64_t)(m0 + mi) * R.K + k;
        const float2 xp = W.X[(int64_t)b * P.NX + xi];
        float2 g;
        if (q < kEnergy) {
            const float2 xo = W.X[((int64_t)B + b) * P.NX + xi];
            const float sp = xp.x * xp.x + xp.y * xp.y;
            const float so = xo.x * xo.x + xo.y * xo.y;
            const float p = sqrtf(sp < kMagEps ? kMagEps : sp);
            const float o = sqrtf(so < kMagEps ? kMagEps : so);
            float dp = (p - o) * c_sc1 - p * c_sc2;
            dp += sgnf(logf(p) - logf(o)) * c_n / p;
            dp += sgnf(p - o) * c_n;
            dp *= gm;
            // sqrt(clamp(s, eps)): the clamp passes the gradient where s >= eps
            const float f = sp >= kMagEps ? dp / p : 0.f;
            g = make_float2(xp.x * f, xp.y * f);
        } else {
            const float f = 2.0f * W.ge[(int64_t)b * P.M4 + m0 + mi] * gE;
            g = make_float2(xp.x * f, xp.y * f);
        }
        sg[it] = g;
    }
    __syncthreads();
    const int stride = kTw / R.N;
    for (int it = tid; it < nf * R.win; it += kThreads) {
        const int mi = it / R.win, t = it - mi * R.win;
        const int step = ((t + R.off) * stride) & (kTw - 1);
        int jj = 0;
        float acc = 0.f;
        const float2* gm_row = sg + mi * R.K;
        for (int k = 0; k < R.K; ++k) {
            const float2 c = stw[jj];
            const float2 g = gm_row[k];
            acc = fmaf(g.x, c.x, acc);
            acc = fmaf(-g.y, c.y, acc);
            jj = (jj + step) & (kTw - 1);
        }
        W.Y[(int64_t)b * P.NY + R.yoff + (int64_t)(m0 + mi) * R.win + t] = swin[t] * acc;
    }
}

// dL/dpred_time[b,t]: time term + upstream grad of pred_time + the frame
// adjoints of every STFT overlapping t (through the reflect padding).
__global__ __launch_bounds__(kThreads) void crit_bwd_time_kernel(CritPlan P,
                                                                 const float* __restrict__ ptime,
                                                                 const float* __restrict__ otime,
                                                                 const float* __restrict__ gloss,
                                                                 const float* __restrict__ gpt,
                                                                 CritWs W) {
    const int b = blockIdx.y;
    const int t = blockIdx.x * kThreads + threadIdx.x;
    const int n = P.n, B = P.B;
    if (t >= n) return;
    const float pt = ptime[(int64_t)b * n + t];
    const float ot = otime[(int64_t)b * n + t];
    float g = gloss[3] * P.w[3] * sgnf(pt - ot) / ((float)B * (float)n);
    if (gpt) g += gpt[(int64_t)b * n + t];
    const float* Yb = W.Y + (int64_t)b * P.NY;
    for (int q = 0; q < kNRes; ++q) {
        const CritRes R = P.r[q];
        const int pad = R.N / 2;
        int js[3];
        int nj = 0;
        js[nj++] = pad + t;
        if (t >= 1 && t <= pad) js[nj++] = pad - t;
        if (t >= n - 1 - pad && t <= n - 2) js[nj++] = pad + 2 * n - 2 - t;
        for (int u = 0; u < nj; ++u) {
            const int rel = js[u] - R.off;
            if (rel < 0) continue;
            const int hi = min(R.M - 1, rel / R.hop);
            const int lo_num = rel - R.win + 1;
            const int lo = lo_num <= 0 ? 0 : (lo_num + R.hop - 1) / R.hop;
            for (int m = lo; m <= hi; ++m) g += Yb[R.yoff + (int64_t)m * R.win + (rel - m * R.hop)];
        }
    }
    W.gtime[(int64_t)b * n + t] = g;
}

// grad_pred[b,k] = adjoint irfft of dL/dpred_time + the spectral terms.
// Block = 32 bins x 8 time slices, gtime and the twiddle table in LDS.
__global__ __launch_bounds__(kThreads) void crit_bwd_spec_kernel(CritPlan P,
                                                                 const float2* __restrict__ pred,
                                                                 const float2* __restrict__ ori,
                                                                 const float2* __restrict__ irtw,
                                                                 const float* __restrict__ gloss,
                                                                 CritWs W,
                                                                 float2* __restrict__ grad) {
    extern __shared__ float lds_f[];
    __shared__ float2 red[8][33];
    const int n = P.n, F = P.F, B = P.B;
    const int b = blockIdx.y;
    float2* tw = reinterpret_cast<float2*>(lds_f);  // [n]
    float* gt = lds_f + 2 * n;                      // [n]
    stage_table<kThreads>(tw, irtw, n);
    for (int i = threadIdx.x; i < n; i += kThreads) gt[i] = W.gtime[(int64_t)b * n + i];
    __syncthreads();
    const int kl = threadIdx.x & 31, sl = threadIdx.x >> 5;
    const int k = blockIdx.x * 32 + kl;
    const int km = k < F ? k : 0;
    int idx = (int)(((int64_t)km * sl) % n);
    const int step = (int)(((int64_t)km * 8) % n);
    float ac = 0.f, as = 0.f;
    for (int t = sl; t < n; t += 8) {
        const float2 c = tw[idx];
        ac = fmaf(gt[t], c.x, ac);
        as = fmaf(gt[t], c.y, as);
        idx += step;
        if (idx >= n) idx -= n;
    }
    red[sl][kl] = make_float2(ac, as);
    __syncthreads();
    if (sl != 0 || k >= F) return;
    float sc = 0.f, ss = 0.f;
    for (int u = 0; u < 8; ++u) {
        sc += red[u][kl].x;
        ss += red[u][kl].y;
    }
    const bool edge = (k == 0) || (k == F - 1);
    float dre = (edge ? 1.0f : 2.0f) * sc / (float)n;
    float dim = edge ? 0.f : -2.0f * ss / (float)n;
    const int64_t i = (int64_t)b * F + k;
    const float2 p = pred[i], o = ori[i];
    const float inv = 1.0f / ((float)B * (float)F);
    const float gs = gloss[0] * P.w[0] * inv;
    dre += gs * sgnf(p.x - o.x);
    dim += gs * sgnf(p.y - o.y);
    const float ap = hypotf(p.x, p.y), ao = hypotf(o.x, o.y);
    if (ap > 0.f) {
        const float f = gloss[1] * P.w[1] * inv * sgnf(ap - ao) / ap;
        dre += f * p.x;
        dim += f * p.y;
        const float tp = atan2f(p.y, p.x), to = atan2f(o.y, o.x);
        const float dth = gloss[2] * P.w[2] * inv *
                          (-sinf(tp) * sgnf(cosf(tp) - cosf(to)) + cosf(tp) * sgnf(sinf(tp) - sinf(to)));
        const float r2 = p.x * p.x + p.y * p.y;
        dre += -dth * p.y / r2;
        dim += dth * p.x / r2;
    }
    grad[i] = make_float2(dre, dim);
}

}  // namespace

extern "C" int avr_criterion_window_len(void) { return window_len(); }

extern "C" int avr_criterion_workspace(int32_t B, int32_t F, int64_t* bytes) {
    CritPlan P;
    if (int e = make_plan(B, F, nullptr, &P)) return e;
    AVR_REQUIRE(bytes, "avr_criterion_workspace: null bytes");
    *bytes = carve(P, nullptr).bytes;
    return 0;
}

extern "C" int avr_criterion_fwd(int32_t B, int32_t F, const float* weights, const float* pred,
                                 const float* ori, const float* wtab, const float* tw512,
                                 const float* irtw, float* pred_time, float* ori_time,
                                 float* losses, void* ws, int64_t ws_bytes, void* stream) {
    return avr_criterion_fwd2(B, F, weights, pred, ori, wtab, tw512, irtw, pred_time, ori_time, losses, nullptr,
                              ws, ws_bytes, stream);
}

extern "C" int avr_criterion_fwd2(int32_t B, int32_t F, const float* weights, const float* pred,
                                  const float* ori, const float* wtab, const float* tw512,
                                  const float* irtw, float* pred_time, float* ori_time,
                                  float* losses, float* total, void* ws, int64_t ws_bytes, void* stream) {
    CritPlan P;
    if (int e = make_plan(B, F, weights, &P)) return e;
    AVR_REQUIRE(pred && ori && wtab && tw512 && irtw && pred_time && ori_time && losses && ws,
                "avr_criterion_fwd: null pointer");
    CritWs W = carve(P, ws);
    AVR_REQUIRE(ws_bytes >= W.bytes, "avr_criterion_fwd: workspace too small");
    AVR_REQUIRE(B <= 256, "avr_criterion_fwd: at most 256 items per call");
    if (int e = launch_irfft(B, F, pred, ori, irtw, pred_time, ori_time, stream))
        return e;
    hipLaunchKernelGGL(crit_stft_kernel, dim3(P.tiles_f, B), dim3(kThreads), 0, as_stream(stream),
                       P, pred_time, ori_time, wtab, reinterpret_cast<const float2*>(tw512), W);
    if (int e = check_launch("crit_stft_kernel")) return e;
    hipLaunchKernelGGL(crit_reduce_kernel, dim3(1), dim3(kRedThreads), 0, as_stream(stream), P,
                       reinterpret_cast<const float2*>(pred), reinterpret_cast<const float2*>(ori),
                       pred_time, ori_time, W, losses, total);
    return check_launch("crit_reduce_kernel");
}

extern "C" int avr_criterion_bwd(int32_t B, int32_t F, const float* weights, const float* pred,
                                 const float* ori, const float* pred_time, const float* ori_time,
                                 const float* grad_losses,
                                 const float* grad_pred_time, const float* wtab,
                                 const float* tw512, const float* irtw, void* ws, int64_t ws_bytes,
                                 float* grad_pred, void* stream) {
    CritPlan P;
    if (int e = make_plan(B, F, weights, &P)) return e;
    AVR_REQUIRE(pred && ori && pred_time && ori_time && grad_losses && wtab && tw512 && irtw && ws && grad_pred,
                "avr_criterion_bwd: null pointer");
    CritWs W = carve(P, ws);
    AVR_REQUIRE(ws_bytes >= W.bytes, "avr_criterion_bwd: workspace too small");
    hipLaunchKernelGGL(crit_bwd_frames_kernel, dim3(P.tiles_b, B), dim3(kThreads), 0,
                       as_stream(stream), P, wtab, reinterpret_cast<const float2*>(tw512),
                       grad_losses, W);
    if (int e = check_launch("crit_bwd_frames_kernel")) return e;
    hipLaunchKernelGGL(crit_bwd_time_kernel, dim3((P.n + kThreads - 1) / kThreads, B),
                       dim3(kThreads), 0, as_stream(stream), P, pred_time, ori_time, grad_losses,
                       grad_pred_time, W);
    if (int e = check_launch("crit_bwd_time_kernel")) return e;
    const size_t lds = (size_t)P.n * 3 * sizeof(float);
    hipLaunchKernelGGL(crit_bwd_spec_kernel, dim3((F + 31) / 32, B), dim3(kThreads), lds,
                       as_stream(stream), P, reinterpret_cast<const float2*>(pred),
                       reinterpret_cast<const float2*>(ori),
                       reinterpret_cast<const float2*>(irtw), grad_losses, W,
                       reinterpret_cast<float2*>(grad_pred));
    return check_launch("crit_bwd_spec_kernel");
}
