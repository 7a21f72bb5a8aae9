"""avr_amd — MI355X-native acoustic volume renderer (hot path of KMASAHIRO/AVR).

`AVRRender` is a drop-in for the reference's `renderer.AVRRender`; the render
core, ray generation, sampling, hash-grid encoding and IR synthesis run in
hand-written HIP kernels for gfx950 behind the C-ABI in `include/avr_hip.h`.
"""
from .renderer import (  # noqa: F401
    AVRRender,
    RenderCore,
    denormalize_points,
    normalize_points,
    ray_directions,
    spectrum_to_ir,
)
from .criterion import Criterion  # noqa: F401
from .options import KernelOptions  # noqa: F401
from . import workloads  # noqa: F401

__version__ = "0.1.0"
