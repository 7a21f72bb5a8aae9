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

_CACHE_ATTRS = ("_avr_cast", "_avr_bias_cols", "_avr_headpack", "_avr_exactpack", "_avr_linpack")


def capturing() -> bool:
    """True while the current stream records a HIP graph: nothing is read
    from or written to the caches then, so the captured graph recomputes the
    derived copies from the master weights at every replay (an optimizer step
    between replays is seen) and holds no pointer into a cache entry that a
    later eager call could replace and free."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _tensors(v):
    if isinstance(v, torch.Tensor):
        yield v
    elif isinstance(v, (tuple, list)):
        for x in v:
            yield from _tensors(x)


def cache_lookup(owner, attr, key):
    """The value cached on `owner.attr` under `key`, or None.

    Cross-stream safe (nn.DataParallel threads, bench streams): an entry made
    on another stream makes the current stream wait for the producing
    stream's event, and its tensors are marked used on the current stream so
    the caching allocator does not hand their blocks out early."""
    hit = getattr(owner, attr, None)
    if hit is None or hit[0] != key:
        return None
    value, stream, event = hit[1], hit[2], hit[3]
    if event is not None:
        cur = torch.cuda.current_stream()
        if cur.cuda_stream != stream:
            cur.wait_event(event)
            for t in _tensors(value):
                if t.is_cuda:
                    t.record_stream(cur)
    return value


def cache_store(owner, attr, key, value):
    """Keep `value` on `owner.attr` under `key` (with the producing stream's
    event for cache_lookup); silently skipped where attributes cannot be set."""
    stream = event = None
    if any(t.is_cuda for t in _tensors(value)):
        cur = torch.cuda.current_stream()
        stream = cur.cuda_stream
        event = torch.cuda.Event()
        event.record(cur)
    try:
        setattr(owner, attr, (key, value, stream, event))
    except AttributeError:  # plain tensors created by some callers: no cache
        pass
    return value


def cast_weight(w: torch.Tensor, dtype: torch.dtype, cache: bool = True) -> torch.Tensor:
    """w.to(dtype).contiguous(), cached on `w` while it is unchanged."""
    if w.dtype == dtype and w.is_contiguous():
        return w
    if not cache or capturing():
        return w.to(dtype).contiguous()
    key = (w.data_ptr(), w._version, dtype, w.device)
    hit = cache_lookup(w, "_avr_cast", key)
    if hit is not None:
        return hit
    return cache_store(w, "_avr_cast", key, w.detach().to(dtype).contiguous())


def clear(module: torch.nn.Module) -> None:
    """Drop the cached casts (and derived weight copies) of a module's parameters."""
    for p in module.parameters():
        for attr in _CACHE_ATTRS:
            if hasattr(p, attr):
                delattr(p, attr)
