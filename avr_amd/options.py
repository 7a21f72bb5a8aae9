"""Kernel selection of the drop-in, as constructor arguments.

The reference's callers build `AVRModel(cfg)` / `AVRModel_complex(cfg)` and
`AVRRender(networks_fn=..., **cfg['render'])` (avr_runner.py:60-63, 168);
they never see process environment, so the kernel choices are keyword
arguments: `AVRModel(cfg, mlp_dtype, options=KernelOptions(...))`, and
`AVRRender(..., head_relu_link=True)` for the renderer's own switch.  The
defaults are the measured-fastest paths, every one parity-tested against
the alternative it replaces (INTEGRATION.md §5 lists them).

Process environment is read in exactly two places of the package:
* `KernelOptions.from_env()`, which tools/ call explicitly to A/B a
  switch without editing code (`AVR_OPT_<FIELD>=value`); the product never
  calls it;
* the two validated tuning knobs of the render core, AVR_NSPLIT (ray splits
  of the reduction) and AVR_KSPLIT (t-slices of the DFT), read by the C
  library itself (csrc/render_fwd.hip) and by `tuning_env()` below so that
  cached layouts follow them; tests/test_gpu_knobs.py renders the golden
  vectors under every value, so neither can change a result.
"""
from __future__ import annotations

import dataclasses
import os

TUNING_ENV = ("AVR_NSPLIT", "AVR_KSPLIT")


@dataclasses.dataclass(frozen=True)
class KernelOptions:
    # inference: the sigma networks (+ the signal network's first layer and
    # the concatenated input) in one csrc/sigma.hip launch
    fused_sigma: bool = True
    fused_h1: bool = True
    # the per-ray / per-pose encodings concatenated by csrc/concat.hip
    grouped_concat: bool = True
    # training: a width-512 ReLU layer's data gradient with the input ReLU's
    # backward fused (csrc/linear512.hip, avr_linear512_mask_fwd)
    fused_dgrad: bool = True
    # training: narrow layers on csrc/mlp.hip's avr_narrow_mm: "80" where a
    # side is 80 wide (the only shapes it wins), "all", or "off"
    narrow: str = "80"
    # training: one-output layers on avr_linear_out1_* (one pass over x)
    out1: bool = True
    # the shipped TunableOp solutions for the file's GEMM shapes
    tunableop: bool = True
    # weight gradients split over rows only for weights with at least this
    # many elements (hipBLASLt fallback path)
    wgrad_min: int = 512 * 512
    # hash-grid backward: "partitioned" (deterministic, no atomics),
    # "partitioned_add" (accumulates into the existing gradient), "atomic"
    hashgrid_bwd: str = "partitioned"

    def __post_init__(self):
        if self.narrow not in ("80", "all", "off"):
            raise ValueError(f"KernelOptions.narrow must be '80', 'all' or 'off', not {self.narrow!r}")
        if self.hashgrid_bwd not in ("partitioned", "partitioned_add", "atomic"):
            raise ValueError("KernelOptions.hashgrid_bwd must be 'partitioned', 'partitioned_add' or 'atomic'")

    def replace(self, **kw) -> "KernelOptions":
        return dataclasses.replace(self, **kw)

    @classmethod
    def from_env(cls, base: "KernelOptions | None" = None) -> "KernelOptions":
        """For tools/ only: fields overridden by AVR_OPT_<FIELD> variables
        (booleans as 0/1)."""
        base = base or cls()
        kw = {}
        for f in dataclasses.fields(cls):
            v = os.environ.get("AVR_OPT_" + f.name.upper())
            if v is None:
                continue
            if f.type in ("bool", bool):
                kw[f.name] = v not in ("0", "false", "False", "")
            elif f.type in ("int", int):
                kw[f.name] = int(v)
            else:
                kw[f.name] = v
        return dataclasses.replace(base, **kw)


DEFAULT = KernelOptions()


def resolve(options) -> KernelOptions:
    if options is None:
        return DEFAULT
    if not isinstance(options, KernelOptions):
        raise TypeError("options must be an avr_amd.KernelOptions")
    return options


def tuning_env() -> tuple:
    """The values of the render core's tuning knobs (part of layout cache keys)."""
    return tuple(os.environ.get(k) for k in TUNING_ENV)


def apply(module, options: KernelOptions):
    """Set `options` on `module` and every submodule that carries kernel
    options (an existing model switched to another selection); returns it."""
    options = resolve(options)
    for m in module.modules():
        if hasattr(m, "options"):
            m.options = options
    return module
