"""ORACLE — test infrastructure only.  torch-CPU fp32 restatement of the Rad-NeRF
field and gate (models/networks.py:214-328 MNGP, :1070-1093 Ray_Gate) with the
tinycudann semantics of networks.py:229-289 (hash grid L=16 F=2, SH degree 4,
FullyFusedMLP without bias).  Autograd provides the backward reference.

f16 rounding points are the ones the HIP kernels use:
weights f16; encoding, hidden activations and geo outputs 1..16 rounded to f16;
sigma = exp(fp32 geo output 0); rgb = sigmoid(fp32 pre-activation) in fp32;
gate input and weights f16, hidden activations / logits fp32, softmax fp32.

Deviation from tcnn's own numerics (wider everywhere, allowed by north_star):
upstream tiny-cuda-nn accumulates the 8-corner trilinear sum in __half
(`result` of type T in kernel_grid), runs FullyFusedMLP with half accumulator
fragments, emits the network output (sigma pre-activation, rgb) as f16, and
accumulates the grid gradient with half2 atomics.  This restatement (and the
HIP kernels) accumulate the trilinear sum, every MLP layer and the grid
gradient in fp32, and keep sigma / rgb in fp32.  tcnn is an absent, unpinned dependency, so this
restatement is "parity unpinned" against tcnn itself.
"""
import math

import numpy as np
import torch


def grid_levels(scale, log2_hashmap_size=19, n_levels=16, n_min=16):
    """tcnn GridEncodingTemplated level table, restated independently of the
    product: per_level_scale b = exp(log(2048*scale/N_min)/(L-1)) as f32
    (networks.py:230), grid_scale = exp2f(l*log2f(b))*N_min - 1,
    resolution = ceil(scale)+1, params_in_level = min(next_multiple(res^3, 8), T)
    for hashed levels (res^3 > T)."""
    b = np.float32(np.exp(np.log(2048 * scale / n_min) / (n_levels - 1)))
    lg = np.float32(math.log2(float(b)))
    T = 1 << log2_hashmap_size
    off, hs, res, sc = [], [], [], []
    o = 0
    for l in range(n_levels):
        s = np.float32(np.float32(2.0 ** float(np.float32(l) * lg)) * np.float32(n_min) - np.float32(1))
        r = int(math.ceil(float(s))) + 1
        p = min((r ** 3 + 7) // 8 * 8, T)
        off.append(o); hs.append(p); res.append(r); sc.append(s)
        o += p
    return {"offset": np.array(off, np.int64), "hsize": np.array(hs, np.int64),
            "res": np.array(res, np.int64), "scale": np.array(sc, np.float32), "n_entries": o}


class _RoundF16(torch.autograd.Function):
    """Forward: round to f16 and back; backward: identity (kernel grads are
    separately rounded, compared with a tolerance)."""

    @staticmethod
    def forward(ctx, x):
        return x.half().float()

    @staticmethod
    def backward(ctx, g):
        return g


def r16(x):
    return _RoundF16.apply(x)


def _fma_f32(a, b, c):
    """Emulate fmaf on fp32 tensors via fp64 (exact product)."""
    return (a.double() * b.double() + c.double()).float()


def grid_index(lv, l, gx, gy, gz):
    """tcnn grid_index: dense when res^3 <= hashmap_size else coherent prime hash."""
    res = int(lv["res"][l])
    hs = int(lv["hsize"][l])
    if res ** 3 <= hs:
        idx = gx + gy * res + gz * res * res
    else:
        idx = gx ^ ((gy * 2654435761) & 0xFFFFFFFF) ^ ((gz * 805459861) & 0xFFFFFFFF)
    idx = idx & 0xFFFFFFFF
    return idx % hs


def unit_coords(x, xyz_min, xyz_max):
    """networks.py:300-301"""
    ext = (xyz_max - xyz_min).float()
    return ((x - xyz_min) / ext).clamp(0.0, 1.0)


def hash_encode(u, grid_params, lv):
    """u (N,3) in [0,1]; grid_params (E,2) fp32 holding f16-representable values
    (requires_grad allowed).  Returns (N,32) fp32 features (before f16 rounding)."""
    feats = []
    offs = lv["offset"]
    for l in range(16):
        sc = torch.tensor(float(lv["scale"][l]), dtype=torch.float64)
        pos = (sc * u.double() + 0.5).float()          # fmaf(scale, x, 0.5)
        g = torch.floor(pos)
        f = pos - g
        gi = g.long()
        acc0 = torch.zeros(len(u))
        acc1 = torch.zeros(len(u))
        for c in range(8):
            bx, by, bz = c & 1, (c >> 1) & 1, (c >> 2) & 1
            w = torch.ones(len(u))
            w = w * (f[:, 0] if bx else 1.0 - f[:, 0])
            w = w * (f[:, 1] if by else 1.0 - f[:, 1])
            w = w * (f[:, 2] if bz else 1.0 - f[:, 2])
            idx = grid_index(lv, l, gi[:, 0] + bx, gi[:, 1] + by, gi[:, 2] + bz) + int(offs[l])
            v = grid_params[idx]
            acc0 = _fma_f32(w, v[:, 0], acc0)
            acc1 = _fma_f32(w, v[:, 1], acc1)
        feats += [acc0, acc1]
    return torch.stack(feats, 1)


def sh4(d):
    """tcnn SphericalHarmonics degree 4 on (d/|d| + 1)/2 (networks.py:324-325)."""
    n = torch.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])
    x = (d[:, 0] / n + 1.0) / 2.0 * 2.0 - 1.0
    y = (d[:, 1] / n + 1.0) / 2.0 * 2.0 - 1.0
    z = (d[:, 2] / n + 1.0) / 2.0 * 2.0 - 1.0
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    o = [torch.full_like(x, 0.28209479177387814),
         -0.48860251190291987 * y,
         0.48860251190291987 * z,
         -0.48860251190291987 * x,
         1.0925484305920792 * xy,
         -1.0925484305920792 * yz,
         0.94617469575755997 * z2 - 0.31539156525251999,
         -1.0925484305920792 * xz,
         0.54627421529603959 * x2 - 0.54627421529603959 * y2,
         0.59004358992664352 * y * (-3.0 * x2 + y2),
         2.8906114426405538 * xy * z,
         0.45704579946446572 * y * (1.0 - 5.0 * z2),
         0.3731763325901154 * z * (5.0 * z2 - 3.0),
         0.45704579946446572 * x * (1.0 - 5.0 * z2),
         1.4453057213202769 * z * (x2 - y2),
         0.59004358992664352 * x * (-x2 + 3.0 * y2)]
    return torch.stack(o, 1)


class TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173"""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


def field_forward(x, d, grid_params, mlp, lv, xyz_min, xyz_max):
    """MNGP.forward for one sub-NeRF.  mlp: dict g1,g2,r1,r2,r3 of fp32 [out,in]
    masters (rounded to f16 here).  Returns sigma (N), rgb (N,3) fp32."""
    u = unit_coords(x, xyz_min, xyz_max)
    e = r16(hash_encode(u, grid_params, lv))
    W = {k: r16(v) for k, v in mlp.items()}
    h1 = r16(torch.relu(e @ W["g1"].t()))
    g32 = h1 @ W["g2"].t()
    g = r16(g32)
    sigma = TruncExp.apply(g32[:, 0])
    sh = r16(sh4(d))
    r1 = r16(torch.relu(torch.cat([sh, g[:, 1:]], 1) @ W["r1"].t()))
    r2 = r16(torch.relu(r1 @ W["r2"].t()))
    out = r2 @ W["r3"].t()
    rgb = torch.sigmoid(out)
    return sigma, rgb


def density_forward(x, grid_params, mlp, lv, xyz_min, xyz_max):
    """MNGP.density(x, ind, return_feat=True) (networks.py:291-309): sigma (N)
    and the geo features h[:, 1:17] (f16 values) of one sub-NeRF."""
    u = unit_coords(x, xyz_min, xyz_max)
    e = r16(hash_encode(u, grid_params, lv))
    W = {k: r16(v) for k, v in mlp.items()}
    h1 = r16(torch.relu(e @ W["g1"].t()))
    g32 = h1 @ W["g2"].t()
    return TruncExp.apply(g32[:, 0]), r16(g32)[:, 1:]


def gate_forward(x6, gate_w):
    """Ray_Gate.forward: softmax(MLP(x6)) with f16 input and weights (tcnn) and
    fp32 hidden activations / logits.  tcnn rounds those to f16; at scale 16
    (|rays_o| up to 24) a rounding flip moves the gate by ~2e-3 against any
    other accumulation order, so both sides evaluate them wider."""
    W = {k: r16(v) for k, v in gate_w.items()}
    h = r16(x6)
    for n in ("w0", "w1", "w2", "w3"):
        h = torch.relu(h @ W[n].t())
    logit = h @ W["w4"].t()
    return torch.softmax(logit, 1)
