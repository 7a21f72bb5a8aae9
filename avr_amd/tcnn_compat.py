"""State-dict interchange with the reference's tiny-cuda-nn modules.

The reference networks are `tcnn.Encoding` / `tcnn.Network` modules
(model.py:21-31, 43-53, 66-68, 117-121, 146-150, 176-180, 258-289), each of
which holds ONE flat fp32 parameter named `params`; avr_runner.py:148-153
saves them under `network_fn.<module>.params`.  Here:

* the hash-grid encodings (`HashGridEncoding`) already hold one flat
  `params` vector in tcnn's GridEncoding order (level tables concatenated,
  [entries][features] per level), so their keys and values carry over as
  they are;
* an `MLP` holds one bias-free `nn.Linear` per layer.  tcnn's FullyFusedMLP
  and CutlassMLP store the layers' weight matrices back to back, each
  row-major [out][in], with the network's input width and output width
  padded to multiples of 16 (the padded rows/columns are zero and unused).
  `mlp_to_tcnn` / `mlp_from_tcnn` convert one network; `to_reference` /
  `from_reference` convert whole state dicts, so a checkpoint written by the
  reference loads into `avr_amd` models and vice versa
  (`TrainStep.load_checkpoint` detects the layout).

Parity unpinned: tinycudann is not in /root/reference and no reference
checkpoint exists, so the matrix order above is restated from upstream
tiny-cuda-nn (network weights as `GPUMatrix<T, RM>` of (padded) out x in,
first layer first) and checked only by round trips (tests/test_tcnn_compat.py).
"""
from __future__ import annotations

import torch

from .model import MLP

_ALIGN = 16  # tcnn's tensor-core width: input / output padding


def _pad(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def tcnn_shapes(mlp: MLP):
    """[(rows, cols)] of the stored matrices: (width, pad(n_in)), hidden
    (width, width)..., (pad(n_out), width)."""
    ws = [lin.weight for lin in mlp.layers]
    shapes = []
    for i, w in enumerate(ws):
        out, inp = w.shape
        rows = _pad(out) if i == len(ws) - 1 else out
        cols = _pad(inp) if i == 0 else inp
        shapes.append((rows, cols))
    return shapes


def tcnn_n_params(mlp: MLP) -> int:
    return sum(r * c for r, c in tcnn_shapes(mlp))


def mlp_to_tcnn(mlp: MLP) -> torch.Tensor:
    """The network's weights as tcnn's flat `params` (fp32, padding zero)."""
    parts = []
    for (rows, cols), lin in zip(tcnn_shapes(mlp), mlp.layers):
        w = lin.weight.detach().float()
        m = torch.zeros(rows, cols, dtype=torch.float32, device=w.device)
        m[:w.size(0), :w.size(1)] = w
        parts.append(m.reshape(-1))
    return torch.cat(parts)


def mlp_from_tcnn(mlp: MLP, params: torch.Tensor) -> None:
    """Load tcnn's flat `params` into the network's layers (in place)."""
    params = params.detach().reshape(-1)
    need = tcnn_n_params(mlp)
    if params.numel() != need:
        raise ValueError(f"tcnn params: {params.numel()} values, this network needs {need} "
                         f"(layers {[tuple(l.weight.shape) for l in mlp.layers]}, padding to {_ALIGN})")
    off = 0
    with torch.no_grad():
        for (rows, cols), lin in zip(tcnn_shapes(mlp), mlp.layers):
            m = params[off:off + rows * cols].view(rows, cols)
            off += rows * cols
            lin.weight.copy_(m[:lin.weight.size(0), :lin.weight.size(1)].to(lin.weight))


def _mlps(module):
    return {name: m for name, m in module.named_modules() if isinstance(m, MLP)}


def to_reference(module) -> dict:
    """`module.state_dict()` with every MLP's per-layer weights replaced by
    tcnn's flat `<mlp>.params` (what the reference's modules hold)."""
    sd = module.state_dict()
    for name, mlp in _mlps(module).items():
        pre = name + "." if name else ""
        for k in [k for k in sd if k.startswith(pre + "layers.")]:
            del sd[k]
        sd[pre + "params"] = mlp_to_tcnn(mlp).to(next(iter(mlp.parameters())).device)
    return sd


def is_reference_layout(module, state_dict) -> bool:
    """True when the state dict holds tcnn-style `<mlp>.params` for the
    module's MLPs (a checkpoint written by the reference)."""
    names = list(_mlps(module))
    return bool(names) and all(((n + ".") if n else "") + "params" in state_dict for n in names)


def from_reference(module, state_dict, strict: bool = True):
    """Load a reference-layout state dict (tcnn flat `params` per network)
    into `module`: encodings by key, MLP layers by `mlp_from_tcnn`."""
    sd = dict(state_dict)
    mlps = _mlps(module)
    for name, mlp in mlps.items():
        key = ((name + ".") if name else "") + "params"
        if key not in sd:
            if strict:
                raise KeyError(f"reference state dict has no {key!r}")
            continue
        mlp_from_tcnn(mlp, sd.pop(key))
    own = module.state_dict()
    rest = {k: v for k, v in sd.items() if k in own}
    unexpected = [k for k in sd if k not in own]
    missing = [k for k in own if k not in rest and not any(
        k.startswith(((n + ".") if n else "") + "layers.") for n in mlps)]
    if strict and (unexpected or missing):
        raise KeyError(f"reference state dict: unexpected {unexpected}, missing {missing}")
    module.load_state_dict(rest, strict=False)
    return missing, unexpected
