"""ORACLE — test infrastructure only.  CPU restatement of one Rad-NeRF training
step of the hot path (forward + backward), as in models/ml_rendering.py:11-78
and :158-202 with train_ml.py:82-105 providing the inputs:

  gate = Ray_Gate(cat(rays_o, rays_d))                 ml_rendering.py:31-36
  for each sub-NeRF i:
     hits = RayAABBIntersector(...); near clamp         :48-50
     RayMarcher (jitter noise[i])                       :174-179
     sigma, rgb = MNGP.forward(xyzs, dirs, i)           :183
     VolumeRenderer(...) ; rgb_i += bg*(1-opacity_i)    :186-200
     rgb += rgb_i*g_i ; opacity += O_i*g_i ; depth[:,i] = D_i   :66-68

March / composite run in the C restatement (oracle/vren_oracle.c); field,
gate and the gated combine run in torch-CPU fp32 with autograd.
"""
import numpy as np
import torch

import oracle
from oracle import field_oracle as fo

NEAR_DISTANCE = 0.01
MAX_SAMPLES = 1024


def _split_field(flat):
    sizes = {"g1": (64, 32), "g2": (17, 64), "r1": (64, 32), "r2": (64, 64), "r3": (3, 64)}
    offs = {"g1": 0, "g2": 2048, "r1": 3136, "r2": 5184, "r3": 9280}
    return {n: flat[offs[n]:offs[n] + r * c].view(r, c) for n, (r, c) in sizes.items()}


def _split_gate(flat, K):
    sizes = {"w0": (64, 6), "w1": (64, 64), "w2": (64, 64), "w3": (64, 64), "w4": (K, 64)}
    offs = {"w0": 0, "w1": 384, "w2": 4480, "w3": 8576, "w4": 12672}
    return {n: flat[offs[n]:offs[n] + r * c].view(r, c) for n, (r, c) in sizes.items()}


def ml_train_step(rays_o, rays_d, bitfields, noise, grid_master, mlp_master, gate_master,
                  scale, seeds=None, bg=None, T_threshold=1e-4, log2_T=19, grid_size=128,
                  input_grads=False, gate_in2=None):
    """One fwd (+ bwd if seeds) step.  All inputs numpy / CPU tensors.

    input_grads: also differentiate w.r.t. rays_o / rays_d (--optimize_ext,
    train_ml.py:90-93): through the gate input, the field's positions and
    directions (autograd over the field restatement) and RayMarcher.backward
    (custom_functions.py:102-112: per-ray sums of dL/dxyz and dL/dxyz * t +
    dL/ddir).  Adds "drays_o", "drays_d" (B, 3) and per-sample "dxyzs",
    "ddirs" lists (one per sub-NeRF) to the result.

    grid_master (E,2) fp32, mlp_master (K,9472) fp32, gate_master (12672+64K,)
    fp32.  seeds = (dL_drgb (B,3), dL_dopacity (B), dL_ddepth (B,K)).
    Returns dict with outputs, per-model intermediates and gradients.
    """
    K = bitfields.shape[0]
    B = len(rays_o)
    cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    if bg is None:
        bg = np.ones(3, np.float32) if esf == 0 else np.zeros(3, np.float32)
    lv = fo.grid_levels(scale, log2_T)
    xyz_min = torch.full((1, 3), -float(scale))
    xyz_max = torch.full((1, 3), float(scale))
    center = np.zeros(3, np.float32)
    half = np.full(3, scale, np.float32)

    o_t = torch.from_numpy(np.asarray(rays_o, np.float32).copy()).requires_grad_(input_grads)
    d_t = torch.from_numpy(np.asarray(rays_d, np.float32).copy()).requires_grad_(input_grads)
    grid_p = torch.tensor(np.asarray(grid_master, np.float32)).half().float().requires_grad_(True)
    mlp_p = torch.tensor(np.asarray(mlp_master, np.float32)).requires_grad_(True)
    gate_p = torch.tensor(np.asarray(gate_master, np.float32)).requires_grad_(True)

    # gate input: cat(rays_o, rays_d), or cat(rays_o, imgs_d) for gate_type
    # "image" (ml_rendering.py:31-36)
    second = d_t if gate_in2 is None else torch.from_numpy(np.asarray(gate_in2, np.float32))
    gate = fo.gate_forward(torch.cat([o_t, second], 1), _split_gate(gate_p, K))

    counts, starts, xyzs, ts, deltas, total = oracle.ml_march(
        rays_o, rays_d, center, half, noise, bitfields, cascades, scale, esf, grid_size,
        MAX_SAMPLES, NEAR_DISTANCE)
    ray_of = np.repeat(np.tile(np.arange(B), K), counts.reshape(-1))
    res = {"counts": counts, "starts": starts, "xyzs": xyzs, "ts": ts, "deltas": deltas,
           "total": total, "gate": gate.detach().numpy(), "ray_of": ray_of}

    sig_l, rgb_l, Ok, Dk, RGBk, ws_l, used_l, ra_l, x_l = [], [], [], [], [], [], [], [], []
    for k in range(K):
        base = int(starts[k, 0]) if B > 0 else 0
        n_k = int(counts[k].sum())
        sl = slice(base, base + n_k)
        x = torch.from_numpy(xyzs[sl].copy()).requires_grad_(input_grads)
        d = d_t[torch.from_numpy(ray_of[sl])]
        sigma, rgb = fo.field_forward(x, d, grid_p, _split_field(mlp_p[k]), lv, xyz_min, xyz_max)
        rays_a = np.stack([np.arange(B), starts[k] - base, counts[k]], 1).astype(np.int64)
        total_k, O, D, RGB, ws = oracle.composite_train_fw(
            sigma.detach().numpy(), rgb.detach().numpy(), deltas[sl], ts[sl], rays_a, T_threshold)
        sig_l.append(sigma); rgb_l.append(rgb); ra_l.append(rays_a); x_l.append(x)
        Ok.append(O); Dk.append(D); RGBk.append(RGB); ws_l.append(ws); used_l.append(total_k)

    O_t = torch.tensor(np.stack(Ok), requires_grad=True)       # (K,B)
    D_t = torch.tensor(np.stack(Dk), requires_grad=True)
    C_t = torch.tensor(np.stack(RGBk), requires_grad=True)      # (K,B,3)
    bg_t = torch.from_numpy(np.asarray(bg, np.float32))
    rgb_out = torch.zeros(B, 3)
    op_out = torch.zeros(B)
    depth_out = torch.zeros(B, K)
    for k in range(K):
        rgb_k = C_t[k] + bg_t * (1 - O_t[k])[:, None]
        rgb_out = rgb_out + rgb_k * gate[:, k][:, None]
        op_out = op_out + O_t[k] * gate[:, k]
        depth_out[:, k] = D_t[k]
    res.update({"rgb": rgb_out.detach().numpy(), "opacity": op_out.detach().numpy(),
                "depth": depth_out.detach().numpy(), "sigmas": [s.detach().numpy() for s in sig_l],
                "rgbs": [c.detach().numpy() for c in rgb_l], "opacity_k": np.stack(Ok),
                "depth_k": np.stack(Dk), "rgb_k": np.stack(RGBk), "ws": ws_l, "used": used_l})
    if seeds is None:
        return res

    g_rgb, g_op, g_depth = (torch.from_numpy(np.asarray(s, np.float32)) for s in seeds)
    torch.autograd.backward([rgb_out, op_out, depth_out], [g_rgb, g_op, g_depth])
    dsig_l, drgb_l = [], []
    for k in range(K):
        base = int(starts[k, 0]) if B > 0 else 0
        n_k = int(counts[k].sum())
        sl = slice(base, base + n_k)
        dsig, drgb = oracle.composite_train_bw(
            O_t.grad[k].numpy(), D_t.grad[k].numpy(), C_t.grad[k].numpy(), np.zeros(n_k, np.float32),
            sig_l[k].detach().numpy(), rgb_l[k].detach().numpy(), ws_l[k], deltas[sl], ts[sl],
            ra_l[k], Ok[k], Dk[k], RGBk[k], T_threshold)
        dsig_l.append(dsig); drgb_l.append(drgb)
        if n_k:
            torch.autograd.backward([sig_l[k], rgb_l[k]],
                                    [torch.from_numpy(dsig), torch.from_numpy(drgb)])
    if input_grads:
        # RayMarcher.backward: segment sums over each ray's samples (fp64)
        go = np.zeros((B, 3)) if o_t.grad is None else o_t.grad.numpy().astype(np.float64)
        gd = np.zeros((B, 3)) if d_t.grad is None else d_t.grad.numpy().astype(np.float64)
        dx_l = []
        for k in range(K):
            base = int(starts[k, 0]) if B > 0 else 0
            n_k = int(counts[k].sum())
            gx = np.zeros((n_k, 3)) if x_l[k].grad is None else x_l[k].grad.numpy().astype(np.float64)
            rk = ray_of[base:base + n_k]
            np.add.at(go, rk, gx)
            np.add.at(gd, rk, gx * ts[base:base + n_k, None].astype(np.float64))
            dx_l.append(gx)
        res.update({"drays_o": go, "drays_d": gd, "dxyzs": dx_l})
    res.update({"dsigmas": dsig_l, "drgbs": drgb_l,
                "grid_grad": grid_p.grad.numpy() if grid_p.grad is not None else None,
                "mlp_grad": mlp_p.grad.numpy() if mlp_p.grad is not None else None,
                "gate_grad": gate_p.grad.numpy() if gate_p.grad is not None else None,
                "dgate": None})
    return res


def _hits(rays_o, rays_d, scale):
    """ml_rendering.py:48-50: AABB hits + NEAR_DISTANCE clamp, (B, 2)."""
    c = np.zeros((1, 3), np.float32)
    h = np.full((1, 3), scale, np.float32)
    _, ht, _ = oracle.ray_aabb_intersect(rays_o, rays_d, c, h, 1)
    ht = np.ascontiguousarray(ht[:, 0])
    m = (ht[:, 0] >= 0) & (ht[:, 0] < NEAR_DISTANCE)
    ht[m, 0] = NEAR_DISTANCE
    return ht


def ml_render_test(rays_o, rays_d, bitfields, grid_master, mlp_master, gate_master, scale,
                   gate_in2=None, T_threshold=1e-4, log2_T=19, grid_size=128):
    """ml_render(test_time=True): the gate, then per sub-NeRF the host-driven
    progressive-compaction loop of __render_rays_test (ml_rendering.py:81-155:
    raymarching_test with in-place hits_t, the field on the valid samples,
    composite_test_fw, drop converged rays, N_samples = max(min(N/N_alive, 64),
    min_samples)), background, gate-weighted combine (:41-78)."""
    K = bitfields.shape[0]
    B = len(rays_o)
    cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    lv = fo.grid_levels(scale, log2_T)
    xyz_min = torch.full((1, 3), -float(scale))
    xyz_max = torch.full((1, 3), float(scale))
    o = np.ascontiguousarray(rays_o, np.float32)
    d = np.ascontiguousarray(rays_d, np.float32)
    second = d if gate_in2 is None else np.ascontiguousarray(gate_in2, np.float32)
    grid_p = torch.tensor(np.asarray(grid_master, np.float32)).half().float()
    mlp_p = torch.tensor(np.asarray(mlp_master, np.float32))
    with torch.no_grad():
        gate = fo.gate_forward(torch.from_numpy(np.concatenate([o, second], 1)),
                               _split_gate(torch.tensor(np.asarray(gate_master, np.float32)), K)).numpy()
    bg = np.ones(3, np.float32) if esf == 0 else np.zeros(3, np.float32)
    rgb_acc = np.zeros((B, 3), np.float32)
    op_acc = np.zeros(B, np.float32)
    depth_all = np.zeros((B, K), np.float32)
    min_samples = 1 if esf == 0 else 4
    for k in range(K):
        ht = _hits(o, d, scale)
        opacity = np.zeros(B, np.float32)
        depth = np.zeros(B, np.float32)
        rgb = np.zeros((B, 3), np.float32)
        alive = np.arange(B, dtype=np.int64)
        samples = 0
        while samples < MAX_SAMPLES:
            n_alive = len(alive)
            if n_alive == 0:
                break
            ns = max(min(B // n_alive, 64), min_samples)
            samples += ns
            xyzs, dirs, deltas, ts, n_eff = oracle.raymarching_test(
                o, d, ht, alive, bitfields[k], cascades, scale, esf, grid_size, MAX_SAMPLES, ns)
            xyzs = xyzs.reshape(-1, 3)
            dirs = dirs.reshape(-1, 3)
            valid = ~np.all(dirs == 0, axis=1)
            if valid.sum() == 0:
                break
            sig = np.zeros(len(xyzs), np.float32)
            col = np.zeros((len(xyzs), 3), np.float32)
            with torch.no_grad():
                s_v, c_v = fo.field_forward(torch.from_numpy(xyzs[valid]), torch.from_numpy(dirs[valid]),
                                            grid_p, _split_field(mlp_p[k]), lv, xyz_min, xyz_max)
            sig[valid] = s_v.numpy()
            col[valid] = c_v.numpy()
            oracle.composite_test_fw(sig.reshape(-1, ns), col.reshape(-1, ns, 3), deltas, ts, alive,
                                     T_threshold, n_eff, opacity, depth, rgb)
            alive = np.ascontiguousarray(alive[alive >= 0])
        rgb_k = rgb + bg * (1 - opacity)[:, None]
        rgb_acc = rgb_acc + rgb_k * gate[:, k][:, None]
        op_acc = op_acc + opacity * gate[:, k]
        depth_all[:, k] = depth
    return {"rgb": rgb_acc, "opacity": op_acc, "depth": depth_all, "gate": gate}
