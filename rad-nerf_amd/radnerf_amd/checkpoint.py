"""Checkpoint interchange with the reference.

The reference trains `MNGP` + `Ray_Gate` inside a Lightning module
(train_ml.py:74-78) and loads weights with utils/util.py:8-31
(`extract_model_state_dict` / `load_ckpt`: a 'state_dict' of keys
'model.<name>' / 'gating_net.<name>').  Its learnable tensors are tcnn flat
parameter vectors:

  model.xyz_encoder.params   hash table, level-major, entries x F=2
  model.geo_net_{i}.params   FullyFusedMLP 32 -> 64 -> 17(pad 32)
  model.rgb_net_{i}.params   FullyFusedMLP 32 -> 64 -> 64 -> 3(pad 16)
  gating_net.encoder.params  FullyFusedMLP 6(pad 16) -> 64 x4 -> K(pad 16)

plus the buffers center, xyz_min, xyz_max, half_size, grid_coords,
density_bitfield_{i}, density_grid_{i} under their own names.  The single
NGP (networks.py:17-126, train.py) uses un-indexed names: geo_net.params,
rgb_net.params (CUTLASSMLP, same no-bias padded RM convention),
density_bitfield, density_grid.

Layout of a FullyFusedMLP vector (upstream tiny-cuda-nn convention; the
dependency is absent here and unpinned, so this mapping is "parity unpinned"):
the weight matrices one after another, each row-major [out, in] (tcnn's
`GPUMatrix<T, RM>` weights), input width padded to a multiple of 16 and the
output layer padded to 16 rows; no biases.  Padded rows/columns are dropped on
import and written as zeros on export.  The hash-table vector is taken as is
when its length equals this build's table (the level sizes come
from tcnn's f32 level-scale arithmetic); any other length raises.

Only loaders that execute nothing from the file are used (`torch.load(...,
weights_only=True)`).
"""
import numpy as np
import torch

from . import layout as LY

GEO_PADDED = [(64, 32), (32, 64)]
RGB_PADDED = [(64, 32), (64, 64), (16, 64)]
GATE_PADDED = [(64, 16), (64, 64), (64, 64), (64, 64), (16, 64)]
MODEL_BUFFERS = ("center", "xyz_min", "xyz_max", "half_size", "grid_coords")


def _split(vec, shapes, what):
    n = sum(r * c for r, c in shapes)
    if vec.numel() != n:
        raise ValueError(f"{what}: expected {n} tcnn parameters, got {vec.numel()}")
    out, o = [], 0
    for r, c in shapes:
        out.append(vec[o:o + r * c].reshape(r, c))
        o += r * c
    return out


def _join(mats, shapes):
    out = []
    for m, (r, c) in zip(mats, shapes):
        p = torch.zeros(r, c, dtype=torch.float32)
        p[:m.shape[0], :m.shape[1]] = m
        out.append(p.reshape(-1))
    return torch.cat(out)


def _field_from_tcnn(geo, rgb):
    g1, g2 = _split(geo.float().cpu().reshape(-1), GEO_PADDED, "geo_net")
    r1, r2, r3 = _split(rgb.float().cpu().reshape(-1), RGB_PADDED, "rgb_net")
    flat = torch.zeros(LY.FIELD_PARAMS)
    m = LY.split_field_params(flat)
    m["g1"].copy_(g1[:, :32]); m["g2"].copy_(g2[:17, :])
    m["r1"].copy_(r1[:, :32]); m["r2"].copy_(r2); m["r3"].copy_(r3[:3, :])
    return flat


def _field_to_tcnn(flat):
    m = LY.split_field_params(flat.detach().float().cpu())
    return (_join([m["g1"], m["g2"]], GEO_PADDED),
            _join([m["r1"], m["r2"], m["r3"]], RGB_PADDED))


def _gate_from_tcnn(vec, K):
    w = _split(vec.float().cpu().reshape(-1), GATE_PADDED, "gating_net")
    flat = torch.zeros(LY.gate_params(K))
    m = LY.split_gate_params(flat, K)
    m["w0"].copy_(w[0][:, :6])
    for i in (1, 2, 3):
        m[f"w{i}"].copy_(w[i])
    m["w4"].copy_(w[4][:K, :])
    return flat


def _gate_to_tcnn(flat, K):
    m = LY.split_gate_params(flat.detach().float().cpu(), K)
    return _join([m["w0"], m["w1"], m["w2"], m["w3"], m["w4"]], GATE_PADDED)


def extract_model_state_dict(state, model_name="model", prefixes_to_ignore=()):
    """utils/util.py:8-22 on an in-memory checkpoint dict."""
    if "state_dict" in state:
        state = state["state_dict"]
    out = {}
    for k, v in state.items():
        if not k.startswith(model_name + "."):
            continue
        k = k[len(model_name) + 1:]
        if any(k.startswith(p) for p in prefixes_to_ignore):
            continue
        out[k] = v
    return out


@torch.no_grad()
def load_reference_state(model, gating_net=None, state=None, path=None):
    """Load a reference checkpoint (Lightning 'state_dict' or the flat dict
    utils/util.py:slim_ckpt writes) into MNGP / NGP (+ Ray_Gate)."""
    if state is None:
        state = torch.load(path, map_location="cpu", weights_only=True)
    sd = extract_model_state_dict(state, "model")
    enc = sd["xyz_encoder.params"].float().reshape(-1)
    if enc.numel() != model.xyz_encoder.params.numel():
        raise ValueError(f"xyz_encoder.params: {enc.numel()} values, this build's table has "
                         f"{model.xyz_encoder.params.numel()}")
    model.xyz_encoder.params.copy_(enc.to(model.xyz_encoder.params.device))
    single = model.size == 1 and "geo_net.params" in sd
    nm = (lambda n, i: n) if single else (lambda n, i: f"{n}_{i}")
    for i in range(model.size):
        flat = _field_from_tcnn(sd[nm("geo_net", i) + ".params"], sd[nm("rgb_net", i) + ".params"])
        model.mlp_params[i].copy_(flat.to(model.mlp_params.device))
    for name in MODEL_BUFFERS:
        if name in sd:
            getattr(model, name).copy_(sd[name].to(getattr(model, name).device))
    for i in range(model.size):
        for n in ("density_bitfield", "density_grid"):
            if nm(n, i) in sd:
                buf = getattr(model, f"{n}_{i}")
                buf.copy_(sd[nm(n, i)].reshape(buf.shape).to(buf.device))
    if hasattr(model, "_set_box_host"):
        model._set_box_host()
    if gating_net is not None:
        gd = extract_model_state_dict(state, "gating_net")
        flat = _gate_from_tcnn(gd["encoder.params"], gating_net.out_dim)
        gating_net.params.copy_(flat.to(gating_net.params.device))


@torch.no_grad()
def reference_state_dict(model, gating_net=None, dtype=torch.float16):
    """Export in the reference's key names and tcnn flat layouts (the inverse of
    load_reference_state); tcnn keeps parameters in f16."""
    from .networks import NGP
    single = isinstance(model, NGP)
    nm = (lambda n, i: n) if single else (lambda n, i: f"{n}_{i}")
    sd = {"model.xyz_encoder.params": model.xyz_encoder.params.detach().cpu().to(dtype)}
    for i in range(model.size):
        geo, rgb = _field_to_tcnn(model.mlp_params[i])
        sd[f"model.{nm('geo_net', i)}.params"] = geo.to(dtype)
        sd[f"model.{nm('rgb_net', i)}.params"] = rgb.to(dtype)
        sd[f"model.{nm('density_bitfield', i)}"] = getattr(model, f"density_bitfield_{i}").cpu()
        sd[f"model.{nm('density_grid', i)}"] = getattr(model, f"density_grid_{i}").cpu()
    for name in MODEL_BUFFERS:
        sd[f"model.{name}"] = getattr(model, name).detach().cpu()
    if gating_net is not None:
        sd["gating_net.encoder.params"] = _gate_to_tcnn(gating_net.params,
                                                        gating_net.out_dim).to(dtype)
    return {"state_dict": sd}
