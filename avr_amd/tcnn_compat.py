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


# --------------------------------------------------------------------------
# Adam state over the reference's parameters (avr_runner.py:121-124, 148-153)
# --------------------------------------------------------------------------
def _mlp_of(module, name):
    """Name of the MLP whose layer `name` is, or None."""
    for n in _mlps(module):
        if name.startswith(((n + ".") if n else "") + "layers."):
            return n
    return None


def param_units(module):
    """`module.parameters()` grouped as the reference's modules hold them:
    [(mlp name or None, [parameter indices])] in parameter order -- one unit
    per encoding (its flat `params`), one per MLP (all its layers, which tcnn
    stores as ONE flat `params`).  Our modules are registered in the
    reference's order (model.py:66-180, 258-289), so unit j is the
    reference optimizer's parameter j."""
    units = []
    for i, (name, _) in enumerate(module.named_parameters()):
        owner = _mlp_of(module, name)
        if owner is not None and units and units[-1][0] == owner:
            units[-1][1].append(i)
        else:
            units.append((owner, [i]))
    return units


def _flat_like_tcnn(mlp, tensors):
    """Per-layer tensors shaped like the MLP's weights -> tcnn's flat layout
    (padded rows/columns zero), as mlp_to_tcnn lays out the weights."""
    parts = []
    for (rows, cols), t in zip(tcnn_shapes(mlp), tensors):
        m = torch.zeros(rows, cols, dtype=t.dtype, device=t.device)
        m[:t.size(0), :t.size(1)] = t
        parts.append(m.reshape(-1))
    return torch.cat(parts)


def _split_from_tcnn(mlp, flat):
    out, off = [], 0
    for (rows, cols), lin in zip(tcnn_shapes(mlp), mlp.layers):
        m = flat.reshape(-1)[off:off + rows * cols].view(rows, cols)
        off += rows * cols
        out.append(m[:lin.weight.size(0), :lin.weight.size(1)].clone())
    return out


_MOMENTS = ("exp_avg", "exp_avg_sq", "max_exp_avg_sq")


def optimizer_state_to_reference(module, opt_state):
    """torch.optim.Adam state_dict over `module.parameters()` -> the same
    state over the reference's parameters (one flat tensor per tcnn module),
    which the reference's `optimizer.load_state_dict` accepts after its
    `load_state_dict` of the converted weights (avr_runner.py:121-124)."""
    if len(opt_state["param_groups"]) != 1:
        raise NotImplementedError("reference-layout optimizer state: one parameter group expected")
    mlps = _mlps(module)
    units = param_units(module)
    state = opt_state["state"]
    new_state = {}
    for j, (owner, idx) in enumerate(units):
        if owner is None:
            if idx[0] in state:
                new_state[j] = state[idx[0]]
            continue
        sts = [state.get(i) for i in idx]
        if all(s is None for s in sts):
            continue
        if any(s is None for s in sts):
            raise ValueError(f"optimizer state covers only some layers of {owner!r}")
        entry = {k: v for k, v in sts[0].items() if k not in _MOMENTS}
        for k in _MOMENTS:
            if k in sts[0]:
                entry[k] = _flat_like_tcnn(mlps[owner], [s[k] for s in sts])
        new_state[j] = entry
    group = dict(opt_state["param_groups"][0])
    group["params"] = list(range(len(units)))
    return {"state": new_state, "param_groups": [group]}


def optimizer_state_from_reference(module, ref_state, own_groups):
    """The inverse of optimizer_state_to_reference: a reference Adam
    state_dict (flat tcnn parameters) -> a state_dict for an optimizer over
    `module.parameters()` whose param_groups are `own_groups` (that
    optimizer's own state_dict()["param_groups"]; hyper-parameters are
    taken from the reference).  Raises ValueError when the reference state
    does not match this model's parameters (count or sizes)."""
    mlps = _mlps(module)
    units = param_units(module)
    params = list(module.parameters())
    groups = ref_state["param_groups"]
    if len(groups) != 1 or len(own_groups) != 1:
        raise ValueError("reference optimizer state: one parameter group expected")
    if len(groups[0]["params"]) != len(units):
        raise ValueError(f"reference optimizer has {len(groups[0]['params'])} parameters, "
                         f"this model's reference layout {len(units)}")
    pos = {p: j for j, p in enumerate(groups[0]["params"])}
    new_state = {}
    for key, st in ref_state["state"].items():
        j = pos.get(key, key)
        if not isinstance(j, int) or j >= len(units):
            raise ValueError(f"reference optimizer state index {key} out of range")
        owner, idx = units[j]
        if owner is None:
            for k in _MOMENTS:
                if k in st and st[k].shape != params[idx[0]].shape:
                    raise ValueError(f"reference state {k} of parameter {j}: shape {tuple(st[k].shape)}, "
                                     f"expected {tuple(params[idx[0]].shape)}")
            new_state[idx[0]] = st
            continue
        need = tcnn_n_params(mlps[owner])
        parts = {}
        for k in _MOMENTS:
            if k in st:
                if st[k].numel() != need:
                    raise ValueError(f"reference state {k} of {owner!r}: {st[k].numel()} values, "
                                     f"expected {need}")
                parts[k] = _split_from_tcnn(mlps[owner], st[k])
        for n, i in enumerate(idx):
            entry = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items() if k not in _MOMENTS}
            for k, v in parts.items():
                entry[k] = v[n]
            new_state[i] = entry
    group = dict(groups[0])
    group["params"] = list(own_groups[0]["params"])
    return {"state": new_state, "param_groups": [group]}
