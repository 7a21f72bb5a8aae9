/*
 * avr_hip.h — C-ABI of the MI355X (gfx950) acoustic volume render hot path.
 *
 * The reference (KMASAHIRO/AVR) is pure Python; its hot path is
 * `AVRRender.forward` (renderer.py:31-124, identical math in
 * renderer_cpu.py:23-102) plus the hash-grid encodings it calls through
 * tinycudann (model.py:66-68, 258-264) and the irfft in
 * utils/criterion.py:71.  There is no FFI in the reference: each entry point
 * below replaces one stage of that Python code, and the Python host package
 * `avr_amd` (the drop-in `AVRRender`) binds them with ctypes — see
 * INTEGRATION.md for the binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - All pointers are DEVICE pointers allocated by the caller (PyTorch's
 *     caching allocator); the library never allocates or frees memory and
 *     keeps no global mutable state, so it is reentrant (nn.DataParallel
 *     calls forward from several host threads, avr_runner.py:63).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).
 *   - Every function returns 0 on success, otherwise a nonzero code
 *     (AVR_E_* or a hipError_t value); `avr_last_error()` returns a
 *     thread-local message for the last failure on the calling thread.
 *   - Layouts are row-major, innermost index last.
 *     B = poses, R = n_azi*n_ele+2 rays, S = n_samples, T = signal length,
 *     F = T/2+1 bins.
 */
#ifndef AVR_HIP_H
#define AVR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVR_ABI_VERSION 2

/* element types of network outputs / gradients */
#define AVR_DTYPE_F32 0
#define AVR_DTYPE_F16 1
#define AVR_DTYPE_BF16 2  /* network outputs of bf16 MLPs (render kernels only) */

/* error codes besides hipError_t values */
#define AVR_E_ARG 1001      /* bad argument / shape / alignment */
#define AVR_E_CONFIG 1002   /* render config outside supported range */

/*
 * Render scalars, rounded on the host exactly the way the reference's torch
 * ops round them (Python double arithmetic first, fp32 at the tensor op):
 * AVRRender.__init__ (renderer.py:16-29) reads the same keys.
 */
typedef struct avr_render_params {
    int32_t n_azi;        /* azimuth rays */
    int32_t n_ele;        /* elevation rings */
    int32_t n_samples;    /* S */
    int32_t T;            /* signal_output_dim */
    int32_t n_rays;       /* rays handled by the render-core kernels: n_azi*n_ele+2,
                             or the size of this rank's contiguous ray shard */
    float depth_scale;    /* fp32(far - near)            renderer.py:54 */
    float depth_offset;   /* fp32(near)                  renderer.py:54 */
    float lo;             /* fp32(xyz_min)               renderer.py:128 */
    float span;           /* fp32(xyz_max - xyz_min)     renderer.py:128 */
    float fs;             /* fp32(fs) */
    float speed;          /* fp32(speed) */
    float pathloss;       /* fp32(pathloss)              renderer.py:98 */
    float azi_jitter;     /* fp32(2*pi / n_azi)          renderer.py:149 */
    float two_pi;         /* fp32(2*pi): linspace end    renderer.py:148 */
    float phase_c;        /* fp32(-2*pi/T)               renderer.py:108 */
    int32_t near_clamp;   /* int(0.1/speed*fs)           renderer.py:96 */
    int32_t pl_len;       /* len(arange(0, 2.5*T))       renderer.py:97 */
} avr_render_params;

const char* avr_last_error(void);
int avr_abi_version(void);

/* Host memory the GPU reads directly (pinned, mapped, fine-grained coherent:
 * every device read goes over the bus, no stale cache lines).  Used for
 * per-call scalars a captured HIP graph reads at replay (the azimuth jitter
 * of avr_sample_rays_dev), so a replay needs no host-to-device copy.
 * *dev_ptr is the address kernels use. */
int avr_pinned_alloc(int64_t bytes, void** host_ptr, void** dev_ptr);
int avr_pinned_free(void* host_ptr);

/* Launch an instantiated HIP graph (hipGraphExec_t) on a stream: the replay
 * of a captured render (avr_amd.graph.GraphedRender) without the host work
 * torch's CUDAGraph.replay adds for device-RNG state.  Valid only for graphs
 * that draw no device random numbers (the render path draws on the CPU). */
int avr_graph_launch(void* graph_exec, void* stream);

/* ---- pose-independent tables (cached per device by the host) ----------
 * d_vals[S], frac[S] (= pts2rx_idx), shift[S] (int), pl_table[pl_len],
 * phase[S][F][2] (cos, sin of the fractional-delay phase),
 * twiddle[T][2] = (cos, -sin)(2*pi*k/T).
 * Replaces renderer.py:54, 79-80, 95-99, 108. */
int avr_tables(const avr_render_params* p, float* d_vals, float* frac, int32_t* shift,
               float* pl_table, float* phase, float* twiddle, void* stream);

/* d_vals[S] alone (needs only n_samples/depth_*), for sampling before the
 * network has revealed T. */
int avr_depth_samples(const avr_render_params* p, float* d_vals, void* stream);

/* irfft twiddle for length n: tw[n][2] = (cos, sin)(2*pi*k/n). */
int avr_ir_twiddle(int32_t n, float* tw, void* stream);

/* ---- a2: spherical ray directions (renderer.py:133-165) ----------------
 * u_azi[n_azi] are the CPU-generator U[0,1) draws (renderer.py:149);
 * writes all n_azi*n_ele+2 directions dirs[..][3] (ignores p->n_rays). */
int avr_ray_directions(const avr_render_params* p, const float* u_azi, float* dirs,
                       void* stream);

/* ---- a3/a4: samples and network inputs (renderer.py:54-62) ------------
 * rays_o, pos_tx, dir_tx: [B][3] (dir_tx may be NULL); dirs points at the
 * first of the p->n_rays directions to sample.  Writes the four network
 * inputs [B][R*S][3] (R = p->n_rays); net_dir_tx unused when dir_tx is NULL. */
int avr_sample_points(const avr_render_params* p, int32_t B, const float* rays_o,
                      const float* pos_tx, const float* dir_tx, const float* dirs,
                      const float* d_vals, float* net_pts, float* net_view, float* net_tx,
                      float* net_dir_tx, void* stream);

/* ---- a2+a3+a4 fused (the hot path's single launch before the network) --
 * u_azi_host: HOST pointer to the n_azi jitter draws, passed by value in the
 * kernel arguments (n_azi <= AVR_MAX_AZI).  Samples rays
 * [ray_begin, ray_begin + p->n_rays) of the sphere, writes their directions
 * dirs[p->n_rays][3] and the four network inputs [B][n_rays*S][3]. */
#define AVR_MAX_AZI 512
int avr_sample_rays(const avr_render_params* p, int32_t B, const float* u_azi_host,
                    int32_t ray_begin, const float* rays_o, const float* pos_tx,
                    const float* dir_tx, float* dirs, float* net_pts, float* net_view,
                    float* net_tx, float* net_dir_tx, void* stream);
/* The same with u_azi_dev a DEVICE pointer to the n_azi jitter draws, read
 * when the kernel runs (HIP-graph replay; any n_azi). */
int avr_sample_rays_dev(const avr_render_params* p, int32_t B, const float* u_azi_dev,
                        int32_t ray_begin, const float* rays_o, const float* pos_tx,
                        const float* dir_tx, float* dirs, float* net_pts, float* net_view,
                        float* net_tx, float* net_dir_tx, void* stream);
/* The same with the jitter AND the pose read from one staged block when the
 * kernel runs: staged = [rays_o (B*3) | pos_tx (B*3) | dir_tx (B*3, read if
 * has_dir_tx) | u_azi (n_azi)], typically device-mapped pinned host memory
 * (avr_pinned_alloc) that a HIP-graph replay refreshes from the host with no
 * copy.  The pose is also published to device memory for the later kernels:
 * pose_out[0..3B) = rays_o, [3B..6B) = pos_tx, [6B..9B) = dir_tx. */
int avr_sample_rays_staged(const avr_render_params* p, int32_t B, const float* staged,
                           int32_t has_dir_tx, int32_t ray_begin, float* pose_out, float* dirs,
                           float* net_pts, float* net_view, float* net_tx, float* net_dir_tx,
                           void* stream);

/* ---- a8 + a11: source delays and compositing weights -------------------
 * attn [B][R*S] (dtype), writes w[B][R][S] fp32 and delay[B][R][S] int32.
 * One ray per wavefront, samples strided over lanes, transmittance by a
 * wavefront shuffle scan.  Replaces renderer.py:86-88, 181-190. */
int avr_weights_fwd(const avr_render_params* p, int32_t B, const void* attn, int32_t attn_dtype,
                    const float* rays_o, const float* pos_tx, const float* dirs,
                    const float* d_vals, float* w, int32_t* delay, void* stream);

/* ---- a7-a12 (time-domain half): ray reduction --------------------------
 * part[n_split][B][S][T] = sum over the rays of split k of
 *   w[b,r,s] * [delay[b,r,s] <= t < T-1-shift[s]] * signal[b,r,s,t]
 * (both masks of renderer.py:72-78; shift[s] = round(fs*d_s/speed)).
 * signal [B][R][S][T] (dtype).  The HBM stream of the forward pass; only the
 * live window [delay, T-1-shift) of each row is read, so non-finite values
 * outside it do not propagate (the reference multiplies them by 0). */
int avr_ray_reduce_fwd(const avr_render_params* p, int32_t B, const void* signal,
                       int32_t sig_dtype, const float* w, const int32_t* delay,
                       int32_t n_split, float* part, void* stream);

/* Number of ray splits avr_ray_reduce_fwd should use for this shape (a power
 * of two <= 16); the caller sizes `part` with it. */
int avr_reduce_splits(const avr_render_params* p, int32_t B, int32_t sig_dtype, int32_t* n_split);

/* ---- a9/a10/a11/a12 (frequency half): DFT + phase + sum over samples ---
 * z[b,s,t] = pl[shift[s]+t] * [t < T-1-shift[s]] * sum_k part[k,b,s,t]
 * spart[B][P][F][2], P = ceil(S/32) * k_split: partial spectra
 *   sum_{s in tile} phase[s,f] * sum_{t in slice} z[b,s,t] * twiddle[(t*f)%T]
 * computed as an fp32 MFMA GEMM [B*S, T] x [T, 2F]. */
int avr_dft_phase_fwd(const avr_render_params* p, int32_t B, const float* part,
                      int32_t n_split, const float* pl_table, const int32_t* shift,
                      const float* phase, const float* twiddle, int32_t k_split,
                      float* spart, void* stream);

/* out[B][F][2] = sum_p spart[B][p][F][2] (fixed order, deterministic). */
int avr_spectrum_finalize(int32_t B, int32_t P, int32_t F, const float* spart, float* out,
                          void* stream);

/* ---- a13: IR synthesis, torch.fft.irfft (utils/criterion.py:71) --------
 * spec[B][F][2] -> ir[B][n], n = 2*(F-1), tw = avr_ir_twiddle(n). */
int avr_irfft(int32_t B, int32_t F, const float* spec, const float* tw, float* ir,
              void* stream);
/* Adjoint of avr_irfft (torch's irfft backward: 1/n, the interior bins
 * doubled, zero imaginary gradient at DC and Nyquist):
 * grad_ir[B][n] -> grad_spec[B][F][2].  Differentiates the IR the loss is
 * taken on (utils/criterion.py:71-72). */
int avr_irfft_bwd(int32_t B, int32_t F, const float* grad_ir, const float* tw, float* grad_spec,
                  void* stream);

/* ---- a7-a13 in one host call -------------------------------------------
 * The pose-independent tables of avr_tables / avr_ir_twiddle. */
typedef struct avr_table_ptrs {
    const float* d_vals;      /* [S] */
    const int32_t* shift;     /* [S] */
    const float* pl_table;    /* [pl_len] */
    const float* phase;       /* [S][F][2] */
    const float* twiddle;     /* [T][2] */
    const float* ir_twiddle;  /* [2(F-1)][2], only needed when ir is requested */
} avr_table_ptrs;

/* Workspace layout of avr_render_core_fwd for this shape: byte offsets of
 * w [B][R][S] fp32, delay [B][R][S] int32, the ray-reduction partials and
 * the spectrum partials, then the total size (offsets[5]); the ray splits
 * and DFT k-slices it uses (splits[2]). */
int avr_render_core_layout(const avr_render_params* p, int32_t B, int32_t sig_dtype,
                           int64_t* offsets, int32_t* splits);

/* avr_weights_fwd -> avr_ray_reduce_fwd -> avr_dft_phase_fwd ->
 * avr_spectrum_finalize [-> avr_irfft when ir != NULL] on one stream.
 * out [B][F][2]; w and delay stay in the workspace for the backward.
 * ev_begin / ev_end: optional hipEvent_t recorded around the ray-reduction
 * launch (benchmark instrumentation; NULL otherwise).
 * Replaces renderer.py:74-124 + utils/criterion.py:71. */
int avr_render_core_fwd(const avr_render_params* p, int32_t B, const void* attn,
                        int32_t attn_dtype, const void* signal, int32_t sig_dtype,
                        const float* rays_o, const float* pos_tx, const float* dirs,
                        const avr_table_ptrs* tables, void* workspace, int64_t workspace_bytes,
                        float* out, float* ir, void* ev_begin, void* ev_end, void* stream);

/* ---- a14: backward ------------------------------------------------------
 * grad_out[B][F][2] -> gz[B][S][T] = pl*tail * d out / d z   (adjoint DFT) */
int avr_dft_phase_bwd(const avr_render_params* p, int32_t B, const float* grad_out,
                      const float* pl_table, const int32_t* shift, const float* phase,
                      const float* twiddle, float* gz, void* stream);

/* gz, signal, w, delay -> grad_signal[B][R][S][T] (sig dtype) and
 * grad_w[B][R][S] = sum_t m gz[b,s,t] * signal[b,r,s,t], where
 * m = [delay[b,r,s] <= t < T-1-shift[s]] as in avr_ray_reduce_fwd;
 * grad_signal = w * m * gz.  Reads only the live window of the signal. */
int avr_ray_reduce_bwd(const avr_render_params* p, int32_t B, const void* signal,
                       int32_t sig_dtype, const float* gz, const float* w,
                       const int32_t* delay, void* grad_signal, float* grad_w, void* stream);

/* grad_w -> grad_attn[B][R*S] (attn dtype): adjoint of the transmittance
 * scan and of alpha = 1 - exp(-attn*dist). */
int avr_weights_bwd(const avr_render_params* p, int32_t B, const void* attn, int32_t attn_dtype,
                    const float* d_vals, const float* grad_w, void* grad_attn, void* stream);

/* ---- a5: multiresolution hash-grid encoding (tcnn GridEncoding) --------
 * x[N][3] in [0,1]; params = concatenated level tables [sum_l size_l][2];
 * level_offset[L+1] (entries), level_scale[L] (fp32), level_res[L] are HOST
 * arrays (passed by value in the kernel arguments);
 * out[N][L*2] (out_dtype).  model.py:66-68, 191, 219-220, 315-324. */
int avr_hashgrid_fwd(int64_t N, int32_t n_levels, const float* x, const void* params,
                     int32_t param_dtype, const int64_t* level_offset, const float* level_scale,
                     const int32_t* level_res, void* out, int32_t out_dtype, void* stream);

/* Same encoding, level-major output out[L][N][2] (inference: the blocks in
 * flight share one level's table, which then stays in L2). */
int avr_hashgrid_fwd_lm(int64_t N, int32_t n_levels, const float* x, const void* params,
                        int32_t param_dtype, const int64_t* level_offset, const float* level_scale,
                        const int32_t* level_res, void* out, int32_t out_dtype, void* stream);
/* The same for points in [-1, 1]: encodes (x + 1) / 2 (model.py:187-189),
 * mapped on load as 0.5 + 0.5 x (exact halving, one rounding: bit-identical
 * to the separate elementwise map). */
int avr_hashgrid_fwd_lm_unit(int64_t N, int32_t n_levels, const float* x, const void* params,
                             int32_t param_dtype, const int64_t* level_offset, const float* level_scale,
                             const int32_t* level_res, void* out, int32_t out_dtype, void* stream);

/* AVRModel inference: the signal network's first-layer bias of every ray,
 * from the per-ray view direction and the per-pose tx position (model.py:221
 * concatenates both encodings to every sample):
 *   e_dir = mlp(enc(dir_grid((view[b][r*S] + 1) / 2))), e_tx likewise from
 *   tx[b][0];  bias[b*R + r][o] = sum_k e_dir[k] w_dir[k][o] + sum_k e_tx[k] w_tx[k][o]
 * view, tx [B][R*S][3] fp32 (network inputs in [-1, 1]); both grids' tables
 * in param_dtype; enc_dtype (F16/F32) the encodings' output rounding;
 * mlp_dtype (BF16/F16) the MLP input rounding mlp(.);
 * w_dir [2*dir_levels][n_out], w_tx [2*tx_levels][n_out] fp32; bias
 * [B*R][n_out] fp32.  Level arrays are HOST pointers as above. */
int avr_ray_pose_bias(int32_t B, int32_t R, int32_t S, const float* view, const float* tx,
                      int32_t dir_levels, const void* dir_params, const int64_t* dir_offset,
                      const float* dir_scale, const int32_t* dir_res, int32_t tx_levels,
                      const void* tx_params, const int64_t* tx_offset, const float* tx_scale,
                      const int32_t* tx_res, int32_t param_dtype, int32_t enc_dtype,
                      int32_t mlp_dtype, const float* w_dir, const float* w_tx, int32_t n_out,
                      float* bias, void* stream);

/* grad_out[N][L*2] -> grad_params (fp32, accumulated with atomics; zero it
 * first). */
int avr_hashgrid_bwd(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                     int32_t grad_dtype, const int64_t* level_offset, const float* level_scale,
                     const int32_t* level_res, float* grad_params, void* stream);

/* The same gradient without global atomics (what training uses): the merged
 * corner contributions are counted and scattered by table partition (8192
 * entries of one level) into `workspace`, then one block per partition sums
 * them in LDS and adds the partition to grad_params (fp32, += : zero it first
 * for a plain gradient).  grad_params 16-byte aligned; workspace 256-byte
 * aligned, of avr_hashgrid_bwd_workspace bytes (12 B per possible
 * contribution, N * n_levels * 8).  Level sizes must be multiples of 8. */
int avr_hashgrid_bwd_workspace(int64_t N, int32_t n_levels, const int64_t* level_offset, int64_t* bytes);
int avr_hashgrid_bwd_partitioned(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                                 int32_t grad_dtype, const int64_t* level_offset, const float* level_scale,
                                 const int32_t* level_res, float* grad_params, void* workspace,
                                 int64_t workspace_bytes, void* stream);
/* The same, writing the gradient instead of adding it (=, not +=): every
 * entry of grad_params is written, zeros where no point contributes, so the
 * caller skips clearing the table and the pass skips reading it (the
 * training step's grids). */
int avr_hashgrid_bwd_partitioned_set(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                                     int32_t grad_dtype, const int64_t* level_offset, const float* level_scale,
                                     const int32_t* level_res, float* grad_params, void* workspace,
                                     int64_t workspace_bytes, void* stream);

/* ---- a6: weight gradient of the networks' bias-free linear layers -------
 * grad_w[M][K] (fp32) = sum_n grad_y[n][M] * x[n][K], both operands bf16,
 * row-major, 16-byte aligned, M and K multiples of 8.  Replaces the wgrad
 * GEMM tcnn runs inside its MLP backward (model.py:21-31, 176-180 through
 * avr_runner.py:190).  Split-K over n: `workspace` holds splits*M*K fp32
 * partials (splits from avr_linear_wgrad_splits), summed deterministically. */
int avr_linear_wgrad_splits(int64_t N, int32_t M, int32_t K, int32_t* splits);
/* A bias-free layer with ONE output (the sigma decoder's last, model.py:
 * 117-121, 259-262), 16-bit x [N][K] and w [K] (fp16 / bf16), K a power of
 * two in [8, 512], fp32 sums:
 *   fwd: y[n] = round16(sum_k x[n][k] w[k])                 (y [N])
 *   bwd: grad_x[n][k] = round16(grad_y[n] w[k]), grad_w[k] = sum_n grad_y[n]
 *        x[n][k] (fp32, deterministic; `workspace` holds
 *        avr_linear_out1_workspace() floats).
 * Replaces the N x 1 GEMM, its broadcast-multiply data gradient and its
 * weight-gradient GEMM (x @ w^T, gy * w, gy^T @ x). */
/* A narrow bias-free layer product, Y[N][C] = act(X[N][R] Bt[C][R]^T), 16-bit
 * operands, fp32 sums rounded once: R in {80, 128, 256}, C a multiple of 4
 * in [68, 256] (<= 128 when R = 256); act 0 none, 1 ReLU, 2 mask (0 where
 * mask[N][C] <= 0, NaN keeps: threshold_backward's selection).  The sigma
 * networks' layers in training (model.py:117-121, 259-262): forward
 * relu(x W^T) with Bt = W, data gradient (g W) with Bt = W^T, the input
 * ReLU's backward fused with act 2 (mask = the layer's input).  X, Bt
 * 16-byte aligned, Y and mask 8-byte aligned. */
int avr_narrow_mm(int64_t N, int32_t R, int32_t C, const void* X, const void* Bt, int32_t dtype, int32_t act,
                  const void* mask, void* Y, void* stream);
int avr_linear_out1_fwd(int64_t N, int32_t K, const void* x, const void* w, int32_t dtype, void* y, void* stream);
int avr_linear_out1_workspace(int32_t K, int64_t* floats);
int avr_linear_out1_bwd(int64_t N, int32_t K, const void* x, const void* w, const void* grad_y, int32_t dtype,
                        void* grad_x, float* workspace, float* grad_w, void* stream);
/* The packed weight of avr_linear512_mask_fwd: W [512][512] (16-bit,
 * 16-byte aligned) in MFMA fragment order into Wf (512 KiB, 16-byte
 * aligned); transpose = 1 packs W^T (for a data gradient, g W = g (W^T)^T). */
int avr_linear512_pack_w2(const void* W, int32_t dtype, int32_t transpose, void* Wf, void* stream);
/* The data gradient of a ReLU layer whose input x is itself a ReLU output
 * consumed only by this layer, with that ReLU's backward fused:
 * y = 0 where mask <= 0, else x Wf^T (threshold_backward's selection: NaN
 * keeps the value; mask, y [M][512], mask = the layer's
 * input activation, Wf packed from W^T).  Replaces `grad @ W` (hipBLASLt) +
 * threshold_backward(., x, 0) in the MLP backward (tcnn's fused MLP
 * backward, model.py:21-31, through avr_runner.py:190). */
int avr_linear512_mask_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, const void* mask, void* y,
                           void* stream);

#ifdef AVR_SHAPE_PROBES
/* Experiments kept for tools/ (the shapes build, make -C avr_amd/csrc
 * shapes), measured slower than the tuned hipBLASLt layers they would
 * replace and not in libavr_hip.so:
 * one width-512 ReLU layer at inference, y = relu(x W^T) (x, y [M][512], W
 * packed by avr_linear512_pack_w = avr_linear512_pack_w2 with transpose 0),
 * and two consecutive ones in one launch, y = relu(relu(x W1^T) W2^T)
 * (csrc/mlp512.hip; avr_mlp512x2_pack_w packs both weights). */
int avr_linear512_pack_w(const void* W, int32_t dtype, void* Wf, void* stream);
int avr_linear512_relu_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, void* y, void* stream);
int avr_mlp512x2_pack_w(const void* W1, const void* W2, int32_t dtype, void* Wf, void* stream);
int avr_mlp512x2_fwd(int64_t M, const void* x, const void* Wf, int32_t dtype, void* y, void* stream);
#endif
int avr_linear_wgrad(int64_t N, int32_t M, int32_t K, const void* grad_y, const void* x,
                     float* workspace, int32_t splits, float* grad_w, void* stream);

/* ---- a5/a6: fused sigma networks (inference) ---------------------------
 * The width-128 bias-free ReLU MLPs the reference runs as tcnn
 * FullyFusedMLP (sigma encoder + decoder, model.py:117-121, 146-150, 199-216
 * for AVRModel; 267-277, 314-317 for AVRModel_complex) and the concatenation
 * of the signal network's input (model.py:221, 325) in one launch:
 *   AVR_SIGMA_MESHRIR: input[0] = pos_enc [N][40];
 *     base[n][0:128] = sigma_feat, attn[n] = |leaky_relu(decoder(relu(sigma_feat)))|
 *     (encoder 40-128-128-128-128, decoder 128-128-128-128-1)
 *   AVR_SIGMA_RAF: input[0] = pos_e [N][40], input[1] = tx_pos_e (per pose);
 *     base[n][0:256] = relu(sigma_feature), attn as above with leaky_slope
 *     (encoder 80-128-128-128-256, decoder 256-128-1)
 * then base[n][out:...] = the extra sources in order (bf16).  Source rows:
 * sample n reads row n / rows_div (1 per sample, S per ray, R*S per pose).
 * wpack = avr_sigma_pack_bytes bytes of bf16 MFMA fragments laid out by
 * avr_amd/sigma.py (pack_sigma_weights).  base, attn are bf16. */
#define AVR_SIGMA_MESHRIR 0
#define AVR_SIGMA_RAF 1
/* AVR_SIGMA_MESHRIR_H1: AVR_SIGMA_MESHRIR followed by the signal network's
 * first layer on the per-sample features (model.py:176-180, 221):
 *   base[n][0:512] = relu(W1[:, :128] sigma_feat[n] + bias[n / bias_div])
 * with bias[g] = W1[:, 128:] [dir_enc | tx_enc] of the group (per ray), so
 * ldb = 512 and no extras; the signal network continues from layer 2. */
#define AVR_SIGMA_MESHRIR_H1 2
#define AVR_SIGMA_MAX_EXTRA 4
typedef struct {
    const void* data; /* [rows][width] (row-major) or [width/2][rows][2] (level-major,
                         avr_hashgrid_fwd_lm output), fp16 or fp32, 16-byte aligned */
    int32_t dtype;    /* AVR_DTYPE_F16 / AVR_DTYPE_F32 */
    int32_t rows_div;
    int64_t lm_rows;  /* 0: row-major; > 0: level-major with this many rows */
} avr_feat_src;

typedef struct {
    int32_t variant;  /* AVR_SIGMA_* */
    int32_t tile_cfg; /* 0 = default tiling (tuning knob, 0..8; anything else is AVR_E_ARG) */
    int64_t n_samples;
    float leaky_slope;
    avr_feat_src input[2];
    int32_t n_extra;
    avr_feat_src extra[AVR_SIGMA_MAX_EXTRA];
    int32_t extra_width[AVR_SIGMA_MAX_EXTRA];
    const float* bias; /* AVR_SIGMA_MESHRIR_H1: [groups][512] fp32 */
    int32_t bias_div;  /* sample n uses bias row n / bias_div */
    int32_t dtype;     /* MLP dtype: AVR_DTYPE_BF16 or AVR_DTYPE_F16 (tcnn's); packed
                          weights, activations, base and attn are in it */
} avr_sigma_desc;

int avr_sigma_pack_bytes(int32_t variant, int64_t* bytes);
int avr_sigma_desc_size(void); /* sizeof(avr_sigma_desc), for binding checks */
int avr_sigma_fwd(const avr_sigma_desc* d, const void* wpack, void* base, int32_t ldb, void* attn,
                  void* stream);

/* ---- a6: grouped feature concatenation (training path) ------------------
 * out[n][col_i + c] = src_i[n / rows_div_i][c] (cast to out_dtype), the
 * sources side by side in order (col_0 = 0); the inputs of the sigma
 * encoder and of the signal network (model.py:199-221, 314-325) with the
 * per-ray / per-pose encodings read per group instead of expanded.
 * Backward: grad_i[r][c] = sum over the rows_div rows of group r of
 * grad_out[n][col_i + c], fp32 sums in a fixed order, stored in src dtype
 * (skipped where grad is NULL); with split > 1 the group is summed in two
 * passes (rows_div/split rows, then split partials) through `workspace`
 * (fp32, N / (rows_div/split) * width floats).  Widths multiples of 8,
 * total <= 512, pointers 16-byte aligned. */
#define AVR_CONCAT_MAX_SRC 8
typedef struct {
    const void* data;
    void* grad;
    int32_t dtype;  /* AVR_DTYPE_F32 / F16 / BF16 */
    int32_t rows_div;
    int32_t width;
    int32_t split;
} avr_concat_src;

int avr_concat_fwd(int64_t N, int32_t n_src, const avr_concat_src* src, void* out, int32_t out_dtype,
                   void* stream);
int avr_concat_bwd(int64_t N, int32_t n_src, const avr_concat_src* src, const void* grad_out,
                   int32_t grad_dtype, float* workspace, void* stream);

/* ---- §8f rank 1: fused signal head -------------------------------------
 * The signal network's last bias-free linear layer (model.py:176-180,
 * output_activation None) folded into the ray reduction:
 *   zpart[n][B][S][T], summed over n = avr_ray_reduce_fwd's `part` for
 *   signal[b,r,s,t] = sum_k h[b,r,s,k] * W[t,k]
 * without materialising the signal.  h [B][R][S][K] (post-activation hidden
 * features) and W [T][K] are fp32 or bf16 (dtype), 16-byte aligned.  n_split
 * (a power of two <= 16, for avr_dft_phase_fwd) comes from avr_head_splits.
 * T <= 4096 and <= 4096 rays per shard. */
int avr_head_splits(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                    int32_t* n_split);
/* Counting sort of each column's rays by delay (rays with d >= T-1-shift
 * dropped): perm, ws [B][S][R] (ray index, weight) and cnt [B][S][T] (number
 * of kept rays with delay <= t).  Input to avr_head_fwd and avr_head_bwd. */
int avr_head_sort(const avr_render_params* p, int32_t B, const float* w, const int32_t* delay,
                  int32_t* perm, float* ws, int32_t* cnt, void* stream);
/* W [T][K] -> Wp (same size) in the forward's feature-block-major layout
 * [K/kb][T][kb] (kb chosen from p, B, K, dtype as in avr_head_fwd): one
 * wave-instruction of the forward then reads 64 consecutive t of a block
 * contiguously.  Wp is avr_head_fwd's W argument. */
int avr_head_pack_w(const avr_render_params* p, int32_t B, int32_t K, const void* W, int32_t dtype,
                    void* Wp, void* stream);
/* W: the packed weight from avr_head_pack_w (same p, B, K, dtype); the
 * linear-algebra head (exact products, no per-element rounding). */
int avr_head_fwd(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* W,
                 int32_t dtype, const int32_t* perm, const float* ws, const int32_t* cnt,
                 int32_t n_split, float* zpart, void* stream);
/* Output-rounding-exact forward for 16-bit networks (fp16 / bf16 h and W,
 * K a multiple of 16, <= 512; T <= 4096, <= 4096 rays per shard): every
 * element of x = h W^T is formed on the matrix cores and rounded to the
 * 16-bit type, as the unfused layer's (the reference network's) output is,
 * before the masked weighted ray sum (csrc/head_exact.hip).
 * avr_head_exact_layout gives n_split (the number of 256-ray slabs, a power
 * of two <= 16, for avr_dft_phase_fwd) and the size of the packed weight;
 * avr_head_pack_w_exact packs W [T][K] into Wf (MFMA B-fragment order, once
 * per weight update); avr_head_fwd_exact writes zpart [n_split][B][S][T],
 * zero for t >= T-1-shift_s.  perm / ws / cnt from avr_head_sort, delay
 * [B][R][S] the integer delays avr_head_sort was given; queue: 256 int32 of
 * device scratch (the kernel's work-queue counters, zeroed on the stream by
 * the call), not shared with a concurrent call. */
int avr_head_exact_layout(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                          int32_t* n_split, int64_t* wpack_bytes);
int avr_head_pack_w_exact(const avr_render_params* p, int32_t K, const void* W, int32_t dtype, void* Wf,
                          void* stream);
int avr_head_fwd_exact(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* Wf,
                       int32_t dtype, const int32_t* perm, const float* ws, const int32_t* cnt,
                       const int32_t* delay, int32_t n_split, float* zpart, int32_t* queue, void* stream);
/* Backward: gz [B][S][T] (avr_dft_phase_bwd) -> grad_h [B][R][S][K] (dtype),
 * grad_w [B][R][S] fp32 (to avr_weights_bwd) and grad_W [T][K] fp32.
 * `workspace` holds avr_head_bwd_workspace() bytes of fp32 partials. */
int avr_head_bwd_workspace(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                           int64_t* bytes);
int avr_head_bwd(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* W,
                 int32_t dtype, const float* w, const int32_t* delay, const int32_t* perm,
                 const float* ws, const int32_t* cnt, const float* gz, void* grad_h,
                 float* grad_w, float* grad_W, float* workspace, int64_t workspace_bytes,
                 void* stream);
/* avr_head_bwd with relu_mask = 1: h is the last hidden layer's ReLU output
 * and the head its only consumer (model.py:176-180, tcnn's MLP backward);
 * grad_h leaves with that ReLU's backward applied (0 where h <= 0, NaN
 * keeps: threshold_backward's selection), so the layer skips its own.
 * relu_mask = 0 is avr_head_bwd. */
int avr_head_bwd2(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* W,
                  int32_t dtype, const float* w, const int32_t* delay, const int32_t* perm,
                  const float* ws, const int32_t* cnt, const float* gz, int32_t relu_mask, void* grad_h,
                  float* grad_w, float* grad_W, float* workspace, int64_t workspace_bytes, void* stream);

/* ---- §8f rank 2: training criterion (utils/criterion.py:69-98) ---------
 * pred, ori: spectra [B][F][2] fp32 (the renderer's output and the measured
 * spectrum); IR length n = 2(F-1) must exceed 256 (torch.stft reflect pad of
 * the 512-point resolution) and be <= 12288; B <= 256.
 * weights[6] (HOST) = spec, amplitude, angle, time, energy, multistft loss
 * weights (criterion.py:11-16).  wtab[avr_criterion_window_len()] = the
 * hann windows torch.hann_window(300), (150), (75), (30) then 256 ones,
 * concatenated; tw512 = avr_ir_twiddle(512); irtw = avr_ir_twiddle(n).
 * Forward writes pred_time, ori_time [B][n] (irfft of each,
 * criterion.py:71-72) and losses[8] = spec, amplitude, angle, time, energy
 * and multi-STFT losses, weighted as the reference returns them
 * (criterion.py:85-98), then two zeros (the DAS terms, criterion.py:101-102).  The workspace (avr_criterion_workspace bytes) holds
 * the STFT bins and statistics the backward reuses: pass the same one.
 * Backward: grad_losses[6] (DEVICE) = upstream grads of the six losses,
 * grad_pred_time [B][n] (DEVICE, may be NULL) = upstream grad of pred_time;
 * writes grad_pred [B][F][2] = dL/dRe, dL/dIm of pred. */
int avr_criterion_window_len(void);
int avr_criterion_workspace(int32_t B, int32_t F, int64_t* bytes);
int avr_criterion_fwd(int32_t B, int32_t F, const float* weights, const float* pred,
                      const float* ori, const float* wtab, const float* tw512, const float* irtw,
                      float* pred_time, float* ori_time, float* losses, void* workspace,
                      int64_t workspace_bytes, void* stream);
/* As avr_criterion_fwd, and total[1] (DEVICE, may be NULL) = losses[0] +
 * losses[1] + ... + losses[7] added left to right, the training loop's
 * total_loss (avr_runner.py:187) in the same kernel (the reference sums the
 * eight scalars with seven torch adds). */
int avr_criterion_fwd2(int32_t B, int32_t F, const float* weights, const float* pred,
                       const float* ori, const float* wtab, const float* tw512, const float* irtw,
                       float* pred_time, float* ori_time, float* losses, float* total, void* workspace,
                       int64_t workspace_bytes, void* stream);
int avr_criterion_bwd(int32_t B, int32_t F, const float* weights, const float* pred,
                      const float* ori, const float* pred_time, const float* ori_time,
                      const float* grad_losses,
                      const float* grad_pred_time, const float* wtab, const float* tw512,
                      const float* irtw, void* workspace, int64_t workspace_bytes,
                      float* grad_pred, void* stream);

/* DAS direction terms (criterion.py:35-67, 100-122) for 8 channels:
 * pred_time, ori_time [8][n]; steer [360][8][257][2] = the reference's
 * steering vectors exp(-i 2 pi delay freq) and angles [360] (radians), both
 * built by the host with the reference's torch ops; tw512 = avr_ir_twiddle(512).
 * Forward writes losses[2] = das_reg * w_reg, das_ce * w_ce (0 for a zero
 * weight).  Backward: grad_losses[2] (DEVICE) -> grad_pred_time [8][n]
 * (overwritten).  Same workspace for both. */
int avr_das_workspace(int64_t* bytes);
int avr_das_fwd(int32_t n, const float* pred_time, const float* ori_time, const float* steer,
                const float* angles, const float* tw512, float beta, float w_reg, float w_ce,
                float* losses, void* workspace, int64_t workspace_bytes, void* stream);
int avr_das_bwd(int32_t n, const float* steer, const float* angles, const float* tw512, float beta,
                float w_reg, float w_ce, const float* grad_losses, void* workspace,
                int64_t workspace_bytes, float* grad_pred_time, void* stream);

/* ---- training-loop gradient post-processing (avr_runner.py:190-196) -----
 * For each of n_tensors fp32 gradients (HOST arrays of device pointers and
 * element counts): g = isfinite(g * coef) ? g * coef : 0, where coef is a
 * DEVICE scalar (clip_grad_norm_'s clamped coefficient; NULL = 1).  One
 * launch per 32 tensors. */
int avr_scale_sanitize(int32_t n_tensors, float* const* ptrs, const int64_t* sizes,
                       const float* coef, void* stream);
/* clip_grad_norm_'s total 2-norm over n_tensors fp32 gradients (HOST arrays
 * of device pointers and element counts) and its clamped coefficient
 * min(max_norm / (total + 1e-6), 1), written to the DEVICE scalars total and
 * coef without a host sync (the coef argument of avr_scale_sanitize /
 * avr_adam_step).  One launch per 32 tensors + 1: partial sums of squares
 * in fixed slots of `workspace` (avr_grad_clip_workspace bytes), summed in a
 * fixed order (run to run identical; within fp32 rounding of torch's
 * foreach norm).  A NaN / Inf element makes total NaN / Inf as in torch. */
int avr_grad_clip_workspace(int32_t n_tensors, const int64_t* sizes, int64_t* bytes);
int avr_grad_clip_coef(int32_t n_tensors, const float* const* ptrs, const int64_t* sizes, float max_norm,
                       void* workspace, int64_t workspace_bytes, float* total, float* coef, void* stream);
/* The same post-processing fused with torch.optim.Adam's update (amsgrad
 * off, L2 weight_decay; avr_runner.py:67-69, 190-200), one pass per element:
 *   g = finite(g*coef) ? g*coef : 0;  g += weight_decay * p;
 *   m += (1-b1) (g - m);  v = v b2 + (1-b2) g g;
 *   p -= step_size[i] * (m / (sqrt(v) / bc2_sqrt[i] + eps))
 * (the fp32 operation order of torch.optim.Adam's default foreach step)
 * with step_size = lr / (1 - b1^step), bc2_sqrt = sqrt(1 - b2^step) per
 * tensor (host arrays).  params, grads, exp_avg, exp_avg_sq: HOST arrays of
 * fp32 device pointers; the gradient is read, not written. */
int avr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads,
                  float* const* exp_avg, float* const* exp_avg_sq, const int64_t* sizes,
                  const float* step_size, const float* bc2_sqrt, double beta1, double beta2,
                  float eps, float weight_decay, const float* coef, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AVR_HIP_H */
