"""Per-parameter cache of the GEMM-dtype copy of an fp32 master weight.

Every linear layer casts its fp32 weight to the GEMM dtype (bf16) per call
(one small elementwise launch per layer, ~10 per pose at inference).  The
copy is kept on the parameter and reused until the parameter changes
(storage pointer or version counter: an optimizer step bumps the version, so
training recasts each step exactly as before).  Used only where no autograd
graph is recorded (callers pass cache=not torch.is_grad_enabled()): writes
through `param.data` do not bump the version counter, so code that edits
weights that way between inference calls must call `clear(module)`."""
from __future__ import annotations

import torch


def cast_weight(w: torch.Tensor, dtype: torch.dtype, cache: bool = True) -> torch.Tensor:
    """w.to(dtype).contiguous(), cached on `w` while it is unchanged."""
    if w.dtype == dtype and w.is_contiguous():
        return w
    if not cache:
        return w.to(dtype).contiguous()
    key = (w.data_ptr(), w._version, dtype, w.device)
    hit = getattr(w, "_avr_cast", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    c = w.detach().to(dtype).contiguous()
    try:
        w._avr_cast = (key, c)
    except AttributeError:  # plain tensors created by some callers: no cache
        pass
    return c


def clear(module: torch.nn.Module) -> None:
    """Drop the cached casts (and derived weight copies) of a module's parameters."""
    for p in module.parameters():
        for attr in ("_avr_cast", "_avr_bias_cols", "_avr_headpack"):
            if hasattr(p, attr):
                delattr(p, attr)
