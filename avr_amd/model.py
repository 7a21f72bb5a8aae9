"""Networks the renderer drives: `AVRModel` (MeshRIR / Simu / Real_env) and
`AVRModel_complex` (RAF), model.py:63-235 and 238-331 of the reference.

Encodings are the HIP hash grid (`avr_amd.encoding`); the MLPs are plain
`nn.Linear(bias=False)` stacks with ReLU (tcnn FullyFusedMLP / CutlassMLP
have no biases), run by PyTorch-ROCm (hipBLASLt GEMMs) so autograd covers
them.  `mlp_dtype` selects the GEMM precision (tcnn runs its MLPs in fp16;
bf16 is the MI355X MFMA-native choice).  The channel-embedding ablations of
AVRModel (model.py:71-181, "injection"/"concat") are outside the hot path
and not provided.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import os

from . import sigma as _sigma
from .concat import grouped_concat
from .encoding import HashGridEncoding
from .options import DEFAULT, KernelOptions, resolve
from .wcache import cache_lookup, cache_store, capturing, cast_weight

_WGRAD_ROWS = 4096  # rows per split of the weight-gradient GEMM
# split only the large weights (KernelOptions.wgrad_min): every distinct
# batched-GEMM shape in a step costs ~1 ms of host time in hipBLASLt's
# solution lookup once more than a few alternate (tools/mm_probe.py --interleave)


def _wgrad_hip(gy, x):
    """dW = gy^T x on the HIP split-K MFMA kernel (bf16 operands, fp32 out)."""
    import ctypes

    from . import _lib

    N, M = gy.shape
    K = x.size(1)
    sp = ctypes.c_int32(0)
    _lib.call("avr_linear_wgrad_splits", N, M, K, ctypes.byref(sp))
    ws = torch.empty(sp.value * M * K, dtype=torch.float32, device=gy.device)
    out = torch.empty(M, K, dtype=torch.float32, device=gy.device)
    _lib.call("avr_linear_wgrad", N, M, K, ctypes.c_void_p(gy.data_ptr()),
              ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(ws.data_ptr()), sp.value,
              ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(gy.device).cuda_stream))
    return out


def _hip_wgrad_ok(gy, x):
    return (gy.is_cuda and gy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and gy.size(1) % 8 == 0 and x.size(1) % 8 == 0 and gy.size(1) >= 8 and x.size(1) >= 8
            and gy.is_contiguous() and x.is_contiguous()
            and gy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def _wgrad(gy, x, opts=DEFAULT):
    """dW = gy^T x for gy [N, out], x [N, in] with N >> out, in.

    A single GEMM with a K dimension of N = B*R*S (1e5..1e6) and a 512x512
    output has only a few dozen output tiles, far too few for 256 CUs (it
    measured 0.14 PFLOP/s).  Split K into chunks of _WGRAD_ROWS rows,
    batch them (one output tile set per chunk) and sum the fp32 partials."""
    if _hip_wgrad_ok(gy, x):
        return _wgrad_hip(gy, x)
    M = gy.size(1)
    if M < 8 and gy.is_cuda and gy.dtype == torch.bfloat16:
        # a 1-wide output layer (the sigma decoder's last): as a GEMM its
        # [M, K] output has a few tiles for a K of N = B*R*S rows (86 us at
        # config 3 for 42 MB of x); zero-padded to 8 rows it runs split-K on
        # the HIP kernel at the speed of reading x
        gp = torch.zeros(gy.size(0), 8, dtype=gy.dtype, device=gy.device)
        gp[:, :M] = gy
        if _hip_wgrad_ok(gp, x):
            return _wgrad_hip(gp, x)[:M].contiguous()
    N = gy.size(0)
    k = N // _WGRAD_ROWS
    if k < 2 or gy.size(1) * x.size(1) < opts.wgrad_min:
        return (gy.t() @ x).float()
    m = k * _WGRAD_ROWS
    a = gy[:m].view(k, _WGRAD_ROWS, -1).transpose(1, 2)
    b = x[:m].view(k, _WGRAD_ROWS, -1)
    part = torch.bmm(a, b)
    gw = part.sum(0, dtype=torch.float32)
    if m < N:
        gw += (gy[m:].t() @ x[m:]).float()
    return gw


class _Linear(torch.autograd.Function):
    """y = x W^T with W kept in fp32 (master) and cast to the GEMM dtype;
    the weight gradient uses the split-K GEMM above and is returned in fp32."""

    @staticmethod
    def forward(ctx, x, w_master, dtype, cache=False, opts=DEFAULT):
        w = cast_weight(w_master, dtype, cache)
        ctx.save_for_backward(x, w)
        ctx.opts = opts
        return _mm_dgrad(x, w.t(), opts)  # (a g @ W-shaped GEMM: the tuned file's "NN" entries)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            # one output (sigma decoder's last layer): the K = 1 GEMM is an
            # outer product; the broadcast multiply rounds the same exact
            # fp32 products once, at write speed (hipBLASLt's K=1 tile: 2 TB/s)
            gx = gy * w if w.size(0) == 1 else _mm_dgrad(gy, w, ctx.opts)
        gw = _wgrad(gy, x, ctx.opts) if ctx.needs_input_grad[1] else None
        return gx, gw, None, None, None


class _LinearOut1(torch.autograd.Function):
    """A layer with one output, y = x w^T for w [1, K] (the sigma decoder's
    last), on csrc/mlp.hip's `avr_linear_out1_*`: one pass over x forward,
    one pass over x backward for both gradients (the N x 1 GEMM, the
    broadcast-multiply data gradient and the weight-gradient GEMM took
    ~75 us at config 3's 83,200 rows for 21 MB of x)."""

    @staticmethod
    def forward(ctx, x, w_master, dtype, cache=False):
        import ctypes

        from . import _lib

        w = cast_weight(w_master, dtype, cache).contiguous()
        x = x.contiguous()
        N, K = x.shape
        y = torch.empty(N, 1, dtype=dtype, device=x.device)
        code = _lib.DTYPE_F16 if dtype == torch.float16 else _lib.DTYPE_BF16
        _lib.call("avr_linear_out1_fwd", N, K, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()), code,
                  ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        import ctypes

        from . import _lib

        x, w = ctx.saved_tensors
        N, K = x.shape
        gy = gy.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        nf = ctypes.c_int64(0)
        _lib.call("avr_linear_out1_workspace", K, ctypes.byref(nf))
        ws = torch.empty(nf.value, dtype=torch.float32, device=x.device)
        gw = torch.empty(1, K, dtype=torch.float32, device=x.device)
        code = _lib.DTYPE_F16 if x.dtype == torch.float16 else _lib.DTYPE_BF16
        _lib.call("avr_linear_out1_bwd", N, K, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()),
                  ctypes.c_void_p(gy.data_ptr()), code, ctypes.c_void_p(gx.data_ptr()),
                  ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(gw.data_ptr()),
                  ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        return (gx if ctx.needs_input_grad[0] else None), (gw if ctx.needs_input_grad[1] else None), None, None


def _out1_ok(h, w_master, dtype, opts=DEFAULT):
    K = h.size(-1)
    return (opts.out1 and h.is_cuda and torch.is_grad_enabled() and dtype in (torch.float16, torch.bfloat16)
            and w_master.size(0) == 1 and h.dim() == 2 and 8 <= K <= 512 and K & (K - 1) == 0)


_ZERO_BIAS: dict = {}


def _zero_bias(n, dtype, device):
    key = (n, dtype, device)
    z = _ZERO_BIAS.get(key)
    if z is None:
        z = torch.zeros(n, dtype=dtype, device=device)
        _ZERO_BIAS[key] = z
    return z


# hipBLASLt / rocBLAS solutions picked by PyTorch TunableOp over every
# candidate on MI355X (tools/tune_gemms.sh; bit-identical output to the
# default solution, which only changes tiling): the width-512 layers at
# config-2 and config-5 inference (0.12 vs 0.16-0.21 ms per layer at 262,144
# rows, 0.99 vs 1.27 ms at 2,097,152; C5=1) and the MLP GEMMs of the config-3
# and -4 training steps, forward and data gradient (TRAIN=1; e.g. the
# 128 -> 80 data gradient 23 vs 40 us, 512 -> 416 73 vs 102 us at 83,200 rows).
# TunableOp is process-global state, so it is switched on only for the
# duration of one of the file's own GEMM shapes (`_tuned_window`) and left as
# the caller had it afterwards: every other GEMM of the process keeps the
# default heuristic, nothing is tuned or recorded, and no results file is
# written at exit (TunableOp writes one only while it is enabled).  Not used
# when the process runs TunableOp itself, off with KernelOptions(tunableop=False).
_TUNED_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")
_TUNED = [None]  # None: not loaded yet; then True (entries loaded) or False


def _tuned_shapes(path=_TUNED_FILE):
    """The file's GEMMs as (kind, torch dtype, rows, out, in):
    kind "relu": `GemmAndBiasTunableOp_<dtype>_TN,tn_<out>_<rows>_<in>_...`,
    y[rows, out] = relu(x[rows, in] W^T) (`_addmm_activation`);
    kind "dgrad": `GemmTunableOp_<dtype>_NN,nn_<in>_<rows>_<out>_...`,
    gx[rows, in] = g[rows, out] W[out, in] (`g @ W`)."""
    names = {"Half": torch.float16, "BFloat16": torch.bfloat16}
    out = set()
    if not os.path.exists(path):
        return out
    for line in open(path):
        f = line.strip().split(",")
        if len(f) < 3 or f[2] == "Default":
            continue
        if f[0].startswith("GemmAndBiasTunableOp_") and f[1].startswith("tn_"):
            dt = names.get(f[0][len("GemmAndBiasTunableOp_"):].rsplit("_", 1)[0])
            n, m, k = (int(v) for v in f[1].split("_")[1:4])
            if dt is not None:
                out.add(("relu", dt, m, n, k))
        elif f[0].startswith("GemmTunableOp_") and f[0].endswith("_NN") and f[1].startswith("nn_"):
            dt = names.get(f[0][len("GemmTunableOp_"):].rsplit("_", 1)[0])
            m, n, k = (int(v) for v in f[1].split("_")[1:4])
            if dt is not None:
                out.add(("dgrad", dt, n, k, m))
    return out


_TUNED_SHAPES = _tuned_shapes()


class _tuned_window:
    """TunableOp on (tuning and untuned-recording off) inside the block; the
    caller's enable / tuning / recording state and results file name
    restored on exit, whatever the block raised.  (TunableOp's first use
    initialises its results manager, which sets the default file name; that
    is put back too, so a process that never used TunableOp sees '' still.)"""

    def __enter__(self):
        import torch.cuda.tunable as tun

        self.prev = (tun.is_enabled(), tun.tuning_is_enabled(), tun.record_untuned_is_enabled(),
                     tun.get_filename())
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        tun.enable(True)
        return self

    def __exit__(self, *exc):
        import torch.cuda.tunable as tun

        tun.enable(self.prev[0])
        tun.tuning_enable(self.prev[1])
        tun.record_untuned_enable(self.prev[2])
        if tun.get_filename() != self.prev[3]:
            tun.set_filename(self.prev[3])
        return False


def _enable_tuned_gemms(device):
    """Load the shipped TunableOp results once, read-only; True when they
    loaded (the file's validators — library versions, gfx950 — make
    TunableOp reject it anywhere else, and then it is not used)."""
    if _TUNED[0] is not None:
        return _TUNED[0]
    _TUNED[0] = False
    if not _TUNED_SHAPES:
        return False
    import torch.cuda.tunable as tun

    if tun.is_enabled() or "gfx950" not in torch.cuda.get_device_properties(device).gcnArchName:
        return False
    with _tuned_window():
        ok = bool(tun.read_file(_TUNED_FILE))
        loaded = {r[1] for r in tun.get_results()} if ok else set()
    _TUNED[0] = ok and len(loaded) > 0
    return _TUNED[0]


def _tuned_gemm(x, w, opts=DEFAULT):
    """True when relu(x W^T) is one of the shipped tuned shapes and the
    results loaded: the caller then runs the GEMM inside `_tuned_window`."""
    return (opts.tunableop and ("relu", x.dtype, x.size(0), w.size(0), x.size(1)) in _TUNED_SHAPES and x.is_cuda
            and _enable_tuned_gemms(x.device))


def _tuned_dgrad(g, w, opts=DEFAULT):
    """As `_tuned_gemm` for the data gradient g @ W (g [rows, out], W [out, in])."""
    return (opts.tunableop and ("dgrad", g.dtype, g.size(0), w.size(0), w.size(1)) in _TUNED_SHAPES and g.is_cuda
            and _enable_tuned_gemms(g.device))


def _mm_dgrad(g, w, opts=DEFAULT):
    """g @ W, inside the TunableOp window for the file's shapes."""
    if _tuned_dgrad(g, w, opts):
        with _tuned_window():
            return g @ w
    return g @ w


# The data gradient of a width-512 ReLU layer whose input is the previous
# layer's ReLU output, with that ReLU's backward fused into the GEMM's
# epilogue (csrc/linear512.hip, `avr_linear512_mask_fwd`);
# KernelOptions(fused_dgrad=False) keeps hipBLASLt + threshold_backward.
def _dgrad512_ok(x, w_master, dtype, opts=DEFAULT):
    """x: the chain's input (device and grad mode); the layer's own input is
    512 wide when its weight is 512 x 512."""
    return (opts.fused_dgrad and x.is_cuda and torch.is_grad_enabled() and dtype in (torch.float16, torch.bfloat16)
            and x.dim() == 2 and tuple(w_master.shape) == (512, 512))


def _dgrad512_masked(g, w, x):
    """(g W) where x > 0, else 0, for g, x [N, 512] and W [512, 512] of the
    16-bit type: threshold_backward(g @ W, x, 0) in one launch."""
    import ctypes

    from . import _lib

    if tuple(w.shape) != (512, 512) or g.dim() != 2 or g.size(1) != 512 or x.shape != g.shape:
        raise ValueError("_dgrad512_masked: g, x [N, 512] and W [512, 512] required")
    code = _lib.DTYPE_F16 if w.dtype == torch.float16 else _lib.DTYPE_BF16
    st = ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    w = w.contiguous()
    wf = torch.empty(512, 512, dtype=w.dtype, device=g.device)
    _lib.call("avr_linear512_pack_w2", ctypes.c_void_p(w.data_ptr()), code, 1, ctypes.c_void_p(wf.data_ptr()), st)
    g = g.contiguous()
    x = x.contiguous()
    out = torch.empty_like(g)
    _lib.call("avr_linear512_mask_fwd", g.size(0), ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(wf.data_ptr()),
              code, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), st)
    return out


# The sigma networks' narrow layers (widths 80 .. 256) in training on
# csrc/mlp.hip's `avr_narrow_mm` (forward with the ReLU, data gradient with
# the input ReLU's backward).  Timed against the tuned hipBLASLt solutions
# (tools/bench_narrow.py, GPU time behind a spin): faster only where a side
# is 80 wide (the RAF sigma encoder's first layer: 13.3 vs 17.9 us forward,
# 14.4 vs 19.2 data gradient at 83,200 rows), slower at 128 / 256 (e.g.
# 15.7 vs 14.0, and 32.6 vs 26.6 for the masked data gradient against
# hipBLASLt + threshold_backward).  KernelOptions.narrow: "80" (default)
# those shapes only, "all" every shape it takes, "off" none.
def _narrow_ok(x, R, C, dtype, opts=DEFAULT, in_backward=False):
    """Y[N, C] = act(X[N, R] Bt[C, R]^T) fits avr_narrow_mm (training only:
    grad mode on, or called from a backward)."""
    if opts.narrow == "off" or (opts.narrow != "all" and 80 not in (R, C)):
        return False
    return (x.is_cuda and x.dim() == 2 and (in_backward or torch.is_grad_enabled())
            and dtype in (torch.float16, torch.bfloat16)
            and R in (80, 128, 256) and 68 <= C <= 256 and C % 4 == 0 and (R < 256 or C <= 128))


def _narrow(x, bt, act, mask=None):
    """act(x bt^T) on avr_narrow_mm: act 0 none, 1 ReLU, 2 zero where mask <= 0."""
    import ctypes

    from . import _lib

    x = x.contiguous()
    bt = bt.contiguous()
    N, R = x.shape
    C = bt.size(0)
    y = torch.empty(N, C, dtype=x.dtype, device=x.device)
    code = _lib.DTYPE_F16 if x.dtype == torch.float16 else _lib.DTYPE_BF16
    m = ctypes.c_void_p(mask.contiguous().data_ptr()) if mask is not None else None
    _lib.call("avr_narrow_mm", N, R, C, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(bt.data_ptr()), code, act, m,
              ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    return y


def _fuse_dgrad_ok(x, w_master, dtype, opts=DEFAULT):
    """The layer's data gradient can carry its input ReLU's backward: the
    width-512 kernel or the narrow one fits (x: the chain's input)."""
    return _dgrad512_ok(x, w_master, dtype, opts) or _narrow_ok(x, w_master.size(0), w_master.size(1), dtype, opts)


class _LinearReLU(torch.autograd.Function):
    """y = relu(x W^T) with the ReLU in the GEMM epilogue: hipBLASLt's
    `_addmm_activation` with a zero bias (one kernel instead of GEMM + an
    elementwise pass over the [N, width] activation, bit-identical output).
    The backward is ReLU's own (threshold on the saved output), then the
    same data / weight gradients as `_Linear`.

    In a chain of such layers (`MLP.hidden`) two flags move each ReLU's
    backward into the GEMM that produces its gradient: `mask_gx` (x is the
    previous layer's ReLU output and this layer its only consumer) returns
    the data gradient already masked by x > 0 (`_dgrad512_masked` for the
    512 -> 512 layers, `_narrow` with its mask epilogue where that applies), and
    `gy_masked` (the consumer of y did so) skips the threshold.  The mask is
    the same selection threshold_backward makes (y > 0 with y = the next
    layer's x), applied to the same rounded values.  `link` (the last layer
    of `MLP.hidden`): a one-element list the output's consumer sets when it
    applies the mask itself (the fused head).  The data-gradient kernel is
    chosen in the forward (ctx.dgrad: "narrow", "512" or "gemm") from the
    shapes it was built for, so the backward never reaches a kernel whose
    shape checks the forward did not make."""

    @staticmethod
    def forward(ctx, x, w_master, dtype, cache=False, mask_gx=False, gy_masked=False, link=None, opts=DEFAULT):
        w = cast_weight(w_master, dtype, cache)
        # (grad mode is off inside forward: training is "an input needs grad")
        training = any(ctx.needs_input_grad[:2])
        if (x.is_cuda and training and _narrow_ok(x, w.size(1), w.size(0), dtype, opts, True)
                and x.dtype == dtype):
            y = _narrow(x, w, 1)
        elif x.is_cuda:
            bias = _zero_bias(w.size(0), dtype, x.device)
            if _tuned_gemm(x, w, opts):
                with _tuned_window():
                    y = torch._addmm_activation(bias, x, w.t(), use_gelu=False)
            else:
                y = torch._addmm_activation(bias, x, w.t(), use_gelu=False)
        else:
            y = torch.relu(x @ w.t())
        ctx.save_for_backward(x, w, y)
        ctx.gy_masked, ctx.link, ctx.opts = gy_masked, link, opts
        # the data gradient g [N, out] @ W [out, in]: narrow kernel, the
        # width-512 masked one (only with mask_gx, for a 512 x 512 weight and
        # a 2-D 16-bit input), or the GEMM (+ threshold_backward if masked)
        dg = "gemm"
        if x.is_cuda and x.dtype == dtype and _narrow_ok(x, w.size(0), w.size(1), dtype, opts, True):
            dg = "narrow"
        elif (mask_gx and x.is_cuda and x.dim() == 2 and x.dtype == dtype and tuple(w.shape) == (512, 512)
              and dtype in (torch.float16, torch.bfloat16) and opts.fused_dgrad):
            dg = "512"
        ctx.dgrad, ctx.mask_gx = dg, mask_gx
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        masked = ctx.gy_masked or (ctx.link is not None and ctx.link[0])
        g = gy.contiguous() if masked else torch.ops.aten.threshold_backward(gy, y, 0).contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            narrow = ctx.dgrad == "narrow" and g.dtype == w.dtype
            if narrow:
                gx = _narrow(g, w.t(), 2 if ctx.mask_gx else 0, x if ctx.mask_gx else None)
            elif ctx.dgrad == "512" and g.dtype == w.dtype:
                gx = _dgrad512_masked(g, w, x)
            else:
                gx = _mm_dgrad(g, w, ctx.opts)
                if ctx.mask_gx:
                    gx = torch.ops.aten.threshold_backward(gx, x, 0)
        gw = _wgrad(g, x, ctx.opts) if ctx.needs_input_grad[1] else None
        return gx, gw, None, None, None, None, None, None


class MLP(nn.Module):
    """tcnn.Network(n_in, n_out, {n_neurons, n_hidden_layers, activation ReLU,
    output_activation None}) without biases."""

    def __init__(self, n_in, n_out, cfg, dtype=torch.float32, options=None):
        super().__init__()
        self.options = resolve(options)
        width = int(cfg["n_neurons"])
        depth = int(cfg["n_hidden_layers"])
        if cfg.get("activation", "ReLU") != "ReLU":
            raise ValueError("only ReLU MLPs are used by the reference configs")
        dims = [n_in] + [width] * depth + [n_out]
        self.layers = nn.ModuleList(nn.Linear(a, b, bias=False) for a, b in zip(dims[:-1], dims[1:]))
        self.dtype = dtype
        self.n_output_dims = n_out

    def hidden(self, x, link=None):
        """All layers but the last (each followed by ReLU): the features the
        output layer is applied to.  `link` (a one-element list, False): the
        last layer's backward skips its ReLU mask once a consumer that
        applies it sets link[0] (the fused head, renderer.FusedHeadCore)."""
        return self._chain(x, list(self.layers[:-1]), link)

    def _chain(self, x, hid, link=None):
        """ReLU layers `hid` in order on x."""
        x = x.to(self.dtype).contiguous()
        # layer i >= 1 takes layer i-1's ReLU output only: its data gradient
        # can carry that ReLU's backward (_LinearReLU's flags)
        o = self.options
        fuse = [i > 0 and _fuse_dgrad_ok(x, lin.weight, self.dtype, o) for i, lin in enumerate(hid)]
        for i, lin in enumerate(hid):
            x = _LinearReLU.apply(x, lin.weight, self.dtype, not torch.is_grad_enabled(), fuse[i],
                                  i + 1 < len(hid) and fuse[i + 1], link if i + 1 == len(hid) else None, o)
        return x

    def hidden_from(self, x, start):
        """Hidden layers start .. n-2 (each followed by ReLU) on x, the
        rectified output of layer start-1."""
        x = x.to(self.dtype).contiguous()
        for lin in self.layers[start:-1]:
            x = _LinearReLU.apply(x, lin.weight, self.dtype, not torch.is_grad_enabled(), False, False, None,
                                  self.options)
        return x

    def last(self, h):
        """The bias-free output layer (output_activation None); a one-output
        layer in training on `_LinearOut1`."""
        w = self.layers[-1].weight
        if _out1_ok(h, w, self.dtype, self.options):
            return _LinearOut1.apply(h.to(self.dtype), w, self.dtype, False)
        return _Linear.apply(h.contiguous(), w, self.dtype, not torch.is_grad_enabled(), self.options)

    def forward(self, x, out_relu=False):
        """The network; `out_relu=True` returns relu(output) with the ReLU in
        the last GEMM's epilogue (for callers that only use the rectified
        output, model.py:316, 323)."""
        if out_relu:  # the output layer joins the ReLU chain
            return self._chain(x, list(self.layers))
        return self.last(self.hidden(x))


class _Broadcast(torch.autograd.Function):
    """e [G, E] -> [B, R, S, E] broadcast over each group's rows; the backward
    sums the group's row gradients in fp32 (autograd's own expand backward
    would sum them in the feature dtype, fp16 for AVRModel's grids)."""

    @staticmethod
    def forward(ctx, e, view_shape, shape):
        ctx.view_shape = view_shape
        return e.view(view_shape).expand(shape).contiguous()

    @staticmethod
    def backward(ctx, g):
        dims = tuple(i for i, n in enumerate(ctx.view_shape) if n == 1)
        gs = g.sum(dim=dims, keepdim=True, dtype=torch.float32)
        return gs.to(g.dtype).view(-1, g.size(-1)), None, None


def _grouped(enc, x, layout, per):
    """Encode rows that repeat over a known group and broadcast the result.

    x is the full [B*R*S, 3] network input.  With the renderer's layout
    (B, R, S), `per="ray"` rows are constant over the S samples of a ray
    (the view direction) and `per="pose"` rows over all R*S samples of a
    pose (tx position / orientation): the grid is evaluated once per group
    (bit-identical features) and expanded, so its backward scatters one
    summed gradient per group instead of R*S contended atomics.  Returns a
    [B, R, S, E] tensor."""
    if layout is None:
        return enc(x)
    B, R, S = layout
    if per == "sample":
        return enc(x).view(B, R, S, -1)
    if per == "ray":
        e = enc(x.view(B, R, S, 3)[:, :, 0].reshape(B * R, 3))
        return _Broadcast.apply(e, (B, R, 1, e.size(-1)), (B, R, S, e.size(-1)))
    e = enc(x.view(B, R * S, 3)[:, 0].contiguous())
    return _Broadcast.apply(e, (B, 1, 1, e.size(-1)), (B, R, S, e.size(-1)))


def _fused_sigma_ok(model, pts, layout, variant):
    """Inference with the renderer's ray layout on a GPU and the sigma
    networks in the shapes `csrc/sigma.hip` implements: run the fused
    kernel.  Training (autograd recording) keeps the per-layer path, whose
    saved activations the backward needs."""
    return (layout is not None and pts.is_cuda and not torch.is_grad_enabled()
            and model.options.fused_sigma and _sigma.variant_of(model) == variant)


def _concat_ok(pts, layout, opts=DEFAULT):
    """Grouped concatenation on the HIP path (renderer layout, GPU tensors)."""
    return layout is not None and pts.is_cuda and opts.grouped_concat


_HALF = torch.tensor(0.5)


def _unit(x):
    """(x + 1) / 2 (model.py:187-189) as ONE elementwise kernel: 0.5 + 0.5 x.
    Halving is exact, so round(0.5 x + 0.5) == round(x + 1) / 2 bit for bit
    (tests/test_gpu_model.py::test_unit_map_is_bit_identical)."""
    return torch.add(_HALF, x, alpha=0.5)


def _per_ray(x, layout):
    """The first sample's row of each ray.  Callers select before mapping
    to [0, 1] ((x + 1) / 2 is elementwise): the map then runs on B*R rows."""
    B, R, S = layout
    return x.reshape(B, R, S, 3)[:, :, 0].reshape(B * R, 3)


def _per_pose(x, layout):
    B, R, S = layout
    return x.reshape(B, R * S, 3)[:, 0].contiguous()


def _bias_columns(w1, dtype=torch.bfloat16):
    """The signal network's first-layer columns that act per ray (dir
    encoding, 128:168) and per pose (tx encoding, 168:208), rounded to the
    MLP dtype as the unfused GEMM reads them, in fp32 and transposed; kept on
    the weight until it changes (version counter), like wcache.cast_weight."""
    key = (w1.data_ptr(), w1._version, dtype)
    hit = None if capturing() else cache_lookup(w1, "_avr_bias_cols", key)
    if hit is not None:
        return hit
    wb = cast_weight(w1, dtype, True).float()
    cols = (wb[:, 128:168].t().contiguous(), wb[:, 168:208].t().contiguous())
    return cols if capturing() else cache_store(w1, "_avr_bias_cols", key, cols)


def _ray_pose_bias(dir_enc, tx_enc, view, tx, wd, wt, layout, mlp_dtype=torch.bfloat16):
    """The first-layer bias of every ray in one launch (`avr_ray_pose_bias`):
    the per-ray direction and per-pose tx encodings, rounded as the unfused
    path rounds them, times their weight columns.  None when the grids do
    not fit the kernel (the caller then runs the torch ops)."""
    B, R, S = layout
    if not (view.is_cuda and dir_enc.dtype == tx_enc.dtype and dir_enc.param_dtype == tx_enc.param_dtype
            and dir_enc.n_levels <= 32 and tx_enc.n_levels <= 32
            and wd.size(0) == dir_enc.n_output_dims and wt.size(0) == tx_enc.n_output_dims):
        return None
    from . import _lib
    from .encoding import _code
    v = view.reshape(B, R * S, 3).float().contiguous()
    t = tx.reshape(B, R * S, 3).float().contiguous()
    cache = not torch.is_grad_enabled()
    dtab, ttab = dir_enc.table(cache), tx_enc.table(cache)
    bias = torch.empty(B * R, wd.size(1), dtype=torch.float32, device=view.device)
    st = torch.cuda.current_stream(view.device).cuda_stream
    _lib.call("avr_ray_pose_bias", B, R, S, v.data_ptr(), t.data_ptr(),
              dir_enc.n_levels, dtab.data_ptr(), dir_enc._off.ctypes.data, dir_enc._scale.ctypes.data,
              dir_enc._res.ctypes.data, tx_enc.n_levels, ttab.data_ptr(), tx_enc._off.ctypes.data,
              tx_enc._scale.ctypes.data, tx_enc._res.ctypes.data, _code(dtab.dtype), _code(dir_enc.dtype),
              _lib.DTYPE_F16 if mlp_dtype == torch.float16 else _lib.DTYPE_BF16,
              wd.data_ptr(), wt.data_ptr(), wd.size(1), bias.data_ptr(), st)
    return bias


def _sigma_params(model):
    return _sigma.network_layers(model._model_encoder_sigma) + _sigma.network_layers(model._model_decoder_sigma)


def _cat_features(parts, layout):
    """Concatenate per-sample features ([N, E] or [B, R, S, E] views) into
    one contiguous [N, sum E] MLP input."""
    if layout is None:
        return torch.cat(parts, -1)
    return torch.cat(parts, -1).view(-1, sum(p.size(-1) for p in parts))


class AVRModel(nn.Module):
    """model.py:63-235 without channel embedding: pos/dir/tx hash grids,
    sigma encoder (-> 128) and decoder (-> 1), signal network (-> T).
    `options`: the kernel selection (avr_amd.KernelOptions; defaults are the
    shipped paths)."""

    def __init__(self, cfg, mlp_dtype=torch.float32, enc_dtype=torch.float16, options=None):
        super().__init__()
        o = self.options = resolve(options)
        self._pos_encoding = HashGridEncoding(3, cfg["pos_encoding_sigma"], dtype=enc_dtype, seed=1, options=o)
        self._dir_encoding = HashGridEncoding(3, cfg["dir_encoding_sig"], dtype=enc_dtype, seed=2, options=o)
        self._tx_encoding = HashGridEncoding(3, cfg["tx_encoding_sig"], dtype=enc_dtype, seed=3, options=o)
        self.signal_output_dim = int(cfg["signal_output_dim"])
        self._model_encoder_sigma = MLP(self._pos_encoding.n_output_dims, 128,
                                        cfg["sigma_encoder_network"], mlp_dtype, o)
        self._model_decoder_sigma = MLP(128, 1, cfg["sigma_decoder_network"], mlp_dtype, o)
        sig_in = 128 + self._dir_encoding.n_output_dims + self._tx_encoding.n_output_dims
        self._model_signal = MLP(sig_in, self.signal_output_dim, cfg["signal_network"], mlp_dtype, o)
        self._sigma_pack = _sigma.SigmaWeights()

    # AVRRender passes ray_layout=(B, R, S) to networks that declare this
    accepts_ray_layout = True
    # ... and folds the signal network's last layer into the render
    # (forward_fused / finish_signal) for networks that declare this
    supports_fused_head = True
    # no dropout or other device RNG: a captured render replays without
    # torch's RNG prologue (avr_amd.graph)
    draws_no_device_rng = True

    def _trunk(self, pts, view, tx, ch_idx, ray_layout):
        """Everything up to the signal network's input: (attn, features)."""
        if ch_idx is not None:
            raise NotImplementedError("channel-embedding variants are not provided")
        bs, n = pts.size(0), pts.size(1)
        L = ray_layout
        if _fused_sigma_ok(self, pts, L, _sigma.MESHRIR):
            return self._trunk_fused(pts, view, tx, L)
        pos_enc = self._pos_encoding(_unit(pts.reshape(-1, 3)))
        sigma_feat = self._model_encoder_sigma(pos_enc)
        attn = self._model_decoder_sigma(F.relu(sigma_feat))
        if _concat_ok(pts, L, self.options):
            B, R, S = L
            dir_e = self._dir_encoding(_unit(_per_ray(view.reshape(-1, 3), L)))
            tx_e = self._tx_encoding(_unit(_per_pose(tx.reshape(-1, 3), L)))
            base = grouped_concat([(sigma_feat, 1), (dir_e, S), (tx_e, R * S)], bs * n, sigma_feat.dtype,
                                  splits=[1, 1, R])
            return torch.abs(F.leaky_relu(attn)).view(bs, n, 1), base
        dir_enc = _grouped(self._dir_encoding, _unit(view.reshape(-1, 3)), L, "ray")
        tx_enc = _grouped(self._tx_encoding, _unit(tx.reshape(-1, 3)), L, "pose")
        dt = sigma_feat.dtype
        sf = sigma_feat if L is None else sigma_feat.view(*L, -1)
        base = _cat_features([sf, dir_enc.to(dt), tx_enc.to(dt)], L)
        attn = torch.abs(F.leaky_relu(attn)).view(bs, n, 1)
        return attn, base

    def _trunk_fused(self, pts, view, tx, L):
        """Encodings (per sample / ray / pose) + one `avr_sigma_fwd` launch:
        attn [B, N, 1] and the signal network's input [N, 208] (bf16)."""
        B, R, S = L
        bs, n = pts.size(0), pts.size(1)
        pos_enc = self._pos_encoding.forward_level_major(pts.reshape(-1, 3), unit_map=True)
        dir_e = self._dir_encoding(_unit(_per_ray(view.reshape(-1, 3), L)))
        tx_e = self._tx_encoding(_unit(_per_pose(tx.reshape(-1, 3), L)))
        packed = self._sigma_pack.get(_sigma.MESHRIR, _sigma_params(self), self._model_encoder_sigma.dtype)
        attn, base = _sigma.sigma_fwd(_sigma.MESHRIR, packed, bs * n, [(pos_enc, 1)],
                                      [(dir_e, S), (tx_e, R * S)], 128, 0.01)
        return attn.view(bs, n, 1), base

    def _trunk_fused_h1(self, pts, view, tx, L):
        """Inference: encodings + one `avr_sigma_fwd` (MESHRIR_H1) launch that
        also applies the signal network's first layer to sigma_feat; the
        layer's dir / tx columns act per ray, as a bias computed here once per
        ray (model.py:221 concatenates them to every sample).  Returns attn
        and h1 = relu(layer 1) [N, 512] bf16."""
        B, R, S = L
        bs, n = pts.size(0), pts.size(1)
        pos_enc = self._pos_encoding.forward_level_major(pts.reshape(-1, 3), unit_map=True)
        w1 = self._model_signal.layers[0].weight
        dt = self._model_encoder_sigma.dtype
        wd, wt = _bias_columns(w1, dt)
        bias = _ray_pose_bias(self._dir_encoding, self._tx_encoding, view, tx, wd, wt, L, dt)
        if bias is None:
            dir_e = self._dir_encoding(_unit(_per_ray(view.reshape(-1, 3), L)))
            tx_e = self._tx_encoding(_unit(_per_pose(tx.reshape(-1, 3), L)))
            bias = dir_e.to(dt).float() @ wd
            bias = (bias.view(B, R, -1) + (tx_e.to(dt).float() @ wt).view(B, 1, -1))
            bias = bias.reshape(B * R, -1).contiguous()
        params = _sigma_params(self) + [w1[:, :128]]
        packed = self._sigma_pack.get(_sigma.MESHRIR_H1, params, dt)
        attn, h1 = _sigma.sigma_fwd(_sigma.MESHRIR_H1, packed, bs * n, [(pos_enc, 1)], [], 512, 0.01,
                                    bias=bias, bias_div=S)
        return attn.view(bs, n, 1), h1

    def _signal_hidden(self, pts, view, tx, ch_idx, ray_layout):
        """(attn, h): h the signal network's last hidden activation."""
        if (ch_idx is None and _fused_sigma_ok(self, pts, ray_layout, _sigma.MESHRIR)
                and self.options.fused_h1 and _sigma.h1_ok(self)):
            attn, h1 = self._trunk_fused_h1(pts, view, tx, ray_layout)
            return attn, self._model_signal.hidden_from(h1, 1)
        attn, base = self._trunk(pts, view, tx, ch_idx, ray_layout)
        return attn, self._model_signal.hidden(base)

    def forward(self, pts, view, tx, ch_idx=None, ray_layout=None):
        attn, h = self._signal_hidden(pts, view, tx, ch_idx, ray_layout)
        signal = self._model_signal.last(h)
        return attn, signal.view(pts.size(0), pts.size(1), self.signal_output_dim)

    def forward_fused(self, pts, view, tx, ch_idx=None, ray_layout=None):
        """(attn, h, W, dtype) with signal = h @ W^T left to the renderer."""
        attn, h = self._signal_hidden(pts, view, tx, ch_idx, ray_layout)
        return (attn, h.view(pts.size(0), pts.size(1), -1), self._model_signal.layers[-1].weight,
                self._model_signal.dtype)

    def finish_signal(self, h):
        """The output layer forward_fused left out: [B, N, K] -> [B, N, T]."""
        return self._model_signal.last(h.reshape(-1, h.size(-1))).view(h.size(0), h.size(1), -1)


class AVRModel_complex(nn.Module):  # noqa: N801  (reference name)
    """model.py:238-331: six hash grids (pos/tx for sigma and for signal,
    view and tx orientation), sigma encoder (-> 256) / decoder, signal MLP."""

    def __init__(self, cfg, mlp_dtype=torch.float32, enc_dtype=torch.float32, options=None):
        super().__init__()
        o = self.options = resolve(options)
        self.leaky_relu = cfg["leaky_relu"]
        self.signal_output_dim = int(cfg["signal_output_dim"])
        E = lambda key, seed: HashGridEncoding(3, cfg[key], dtype=enc_dtype, seed=seed, options=o)  # noqa: E731
        self._pos_encoding = E("pos_encoding_sigma", 11)
        self._pos_signal_encoding = E("pos_encoding_sig", 12)
        self._tx_pos_encoding = E("tx_pos_encoding_sigma", 13)
        self._tx_pos_signal_encoding = E("tx_pos_encoding_sig", 14)
        self._dir_encoding = E("dir_encoding_sig", 15)
        self._tx_dir_encoding = E("tx_dir_encoding_sig", 16)
        n_in = self._pos_encoding.n_output_dims + self._tx_pos_encoding.n_output_dims
        self._model_encoder_sigma = MLP(n_in, 256, cfg["sigma_encoder_network"], mlp_dtype, o)
        self._model_decoder_sigma = MLP(256, 1, cfg["sigma_decoder_network"], mlp_dtype, o)
        n_sig = (256 + self._dir_encoding.n_output_dims + self._tx_dir_encoding.n_output_dims
                 + self._pos_signal_encoding.n_output_dims + self._tx_pos_signal_encoding.n_output_dims)
        self._model_signal = MLP(n_sig, self.signal_output_dim, cfg["signal_network"], mlp_dtype, o)
        self._sigma_pack = _sigma.SigmaWeights()

    accepts_ray_layout = True
    supports_fused_head = True
    draws_no_device_rng = True

    def forward(self, pts, view, tx, tx_view, ray_layout=None):
        attn, base = self._trunk(pts, view, tx, tx_view, ray_layout)
        signal = self._model_signal(base)
        return attn, signal.reshape(pts.size(0), pts.size(1), self.signal_output_dim)

    def forward_fused(self, pts, view, tx, tx_view, ray_layout=None):
        attn, base = self._trunk(pts, view, tx, tx_view, ray_layout)
        link = [False]  # the fused head may take over h's ReLU backward (MLP.hidden)
        h = self._model_signal.hidden(base, link)
        if torch.is_grad_enabled() and len(self._model_signal.layers) > 1:
            self._relu_link = link
        return (attn, h.view(pts.size(0), pts.size(1), -1), self._model_signal.layers[-1].weight,
                self._model_signal.dtype)

    finish_signal = AVRModel.finish_signal

    def _trunk(self, pts, view, tx, tx_view, ray_layout):
        bs, n = pts.size(0), pts.size(1)
        L = ray_layout
        if _fused_sigma_ok(self, pts, L, _sigma.RAF):
            return self._trunk_fused(pts, view, tx, tx_view, L)
        pts = _unit(pts.reshape(-1, 3))
        view = _unit(view.reshape(-1, 3))
        tx = _unit(tx.reshape(-1, 3))
        tx_view = _unit(tx_view.reshape(-1, 3))
        if _concat_ok(pts, L, self.options):
            return self._trunk_grouped(pts, view, tx, tx_view, L)
        pos_e = _grouped(self._pos_encoding, pts, L, "sample")
        txp_e = _grouped(self._tx_pos_encoding, tx, L, "pose")
        # the sigma feature is only used rectified (model.py:316, 323)
        rf = self._model_encoder_sigma(_cat_features([pos_e, txp_e], L), out_relu=True)
        attn = self._model_decoder_sigma(rf)
        dt = rf.dtype
        parts = [rf if L is None else rf.view(*L, -1),
                 _grouped(self._dir_encoding, view, L, "ray").to(dt),
                 _grouped(self._tx_dir_encoding, tx_view, L, "pose").to(dt),
                 _grouped(self._pos_signal_encoding, pts, L, "sample").to(dt),
                 _grouped(self._tx_pos_signal_encoding, tx, L, "pose").to(dt)]
        attn = torch.abs(F.leaky_relu(attn, negative_slope=self.leaky_relu)).view(bs, n, 1)
        return attn, _cat_features(parts, L)

    def _trunk_grouped(self, pts, view, tx, tx_view, L):
        """Training path with the renderer's layout: per-ray / per-pose
        encodings evaluated once per group and concatenated by
        `avr_concat_fwd` (backward: fixed-order group sums)."""
        B, R, S = L
        N = B * R * S
        t = _per_pose(tx, L)
        txp_e = self._tx_pos_encoding(t)
        enc_in = grouped_concat([(self._pos_encoding(pts), 1), (txp_e, R * S)], N,
                                self._model_encoder_sigma.dtype, splits=[1, R])
        rf = self._model_encoder_sigma(enc_in, out_relu=True)
        attn = self._model_decoder_sigma(rf)
        base = grouped_concat(
            [(rf, 1), (self._dir_encoding(_per_ray(view, L)), S),
             (self._tx_dir_encoding(_per_pose(tx_view, L)), R * S),
             (self._pos_signal_encoding(pts), 1), (self._tx_pos_signal_encoding(t), R * S)],
            N, rf.dtype, splits=[1, 1, R, 1, R])
        attn = torch.abs(F.leaky_relu(attn, negative_slope=self.leaky_relu)).view(B, R * S, 1)
        return attn, base

    def _trunk_fused(self, pts, view, tx, tx_view, L):
        """Six encodings at their own granularity + one `avr_sigma_fwd`
        launch: attn [B, N, 1] and the signal network's input [N, 416]."""
        B, R, S = L
        bs, n = pts.size(0), pts.size(1)
        p = pts.reshape(-1, 3)  # (the per-sample grids map (x + 1) / 2 on load)
        t = _unit(_per_pose(tx.reshape(-1, 3), L))
        v = _unit(_per_ray(view.reshape(-1, 3), L))
        tv = _unit(_per_pose(tx_view.reshape(-1, 3), L))
        packed = self._sigma_pack.get(_sigma.RAF, _sigma_params(self), self._model_encoder_sigma.dtype)
        attn, base = _sigma.sigma_fwd(
            _sigma.RAF, packed, bs * n,
            [(self._pos_encoding.forward_level_major(p, unit_map=True), 1), (self._tx_pos_encoding(t), R * S)],
            [(self._dir_encoding(v), S), (self._tx_dir_encoding(tv), R * S),
             (self._pos_signal_encoding.forward_level_major(p, unit_map=True), 1),
             (self._tx_pos_signal_encoding(t), R * S)],
            256, self.leaky_relu)
        return attn.view(bs, n, 1), base
