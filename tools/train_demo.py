"""Training convergence on a synthetic scene (dev tool / evidence).

trainer.Trainer runs train_ml.py's step (training_step :172-193 + FusedAdam
:138-153; occupancy-grid update every 16 steps, warm-up sweeps for the first
256): fused render -> fused NeRFLoss -> merged backward -> Adam.  The scene is
analytic, so every ray has an exact target: a sphere of radius 0.25 at the
origin coloured 0.5 + 0.5 * normal, in front of the white background that
train_ml.py uses at scale 0.5 (ml_rendering.py:192-198).  Every step draws a
fresh batch of rays (origins on the radius-1.5 sphere, aimed into
[-0.4, 0.4]^3).  The same initialisation and ray stream run twice: with the
fixed-point grid gradient (the default) and with fp32 atomics, and the tool
reports both loss curves, the PSNR of the rgb term and how many steps the
fixed-point path redid in fp32.

    python tools/train_demo.py [steps] [rays] [K] [scale]      -> one JSON line
"""
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402

from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402
from radnerf_amd.trainer import Trainer  # noqa: E402

R_SPHERE = 0.25


def batch(gen, n, dev, bg=1.0):
    """rays + analytic targets (sphere hit -> 0.5 + 0.5 n, miss -> bg)"""
    u = torch.randn(n, 3, generator=gen, device=dev)
    o = 1.5 * u / u.norm(dim=1, keepdim=True)
    p = (torch.rand(n, 3, generator=gen, device=dev) * 2 - 1) * 0.4
    d = p - o
    d = d / d.norm(dim=1, keepdim=True)
    b = (o * d).sum(1)
    c = (o * o).sum(1) - R_SPHERE ** 2
    disc = b * b - c
    t = -b - torch.sqrt(disc.clamp_min(0))
    hit = (disc > 0) & (t > 0)
    nrm = o + t[:, None] * d
    nrm = nrm / nrm.norm(dim=1, keepdim=True)
    target = torch.where(hit[:, None], 0.5 + 0.5 * nrm, torch.full_like(nrm, bg))
    return o.contiguous(), d.contiguous(), target.contiguous()


def run(steps, B, K, grid_fx, dev, scale=0.5):
    torch.manual_seed(0)
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    tr = Trainer(m, g, B, lr=1e-2, lambda_cv_importance=1e-2)
    tr.renderer.grid_fx = grid_fx
    # $FX_F32_LEVELS="4,5,6,7,8": those levels by fp32 atomics (fused.fx_f32_levels)
    tr.renderer.fx_f32_levels = tuple(int(x) for x in os.environ.get("FX_F32_LEVELS", "").split(",")
                                      if x)
    # $BIN_F32_LEVELS=n: the binned form's fp32 coarse levels (default: the renderer's)
    if os.environ.get("BIN_F32_LEVELS"):
        tr.renderer.bin_f32_levels = int(os.environ["BIN_F32_LEVELS"])
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(os.environ.get("DEMO_SEED", 1234)))
    curve, redo_steps = [], 0
    acc_rgb, n_acc = 0.0, 0
    tail, tail_n = 0.0, 0                # the last 200 steps' mean rgb loss
    torch.cuda.synchronize()
    t0 = time.time()
    for s in range(steps):
        # train_ml.py's background: white at scale 0.5, black beyond (esf > 0)
        o, d, target = batch(gen, B, dev, 1.0 if scale <= 0.5 else 0.0)
        terms = tr.step(o, d, d, target)
        if grid_fx and getattr(tr.renderer.ws, "_fx", None) is not None:
            redo_steps += int(tr.renderer.ws._fx[3].item())
        acc_rgb += float(terms["rgb"])
        n_acc += 1
        if s >= steps - 200:
            tail += float(terms["rgb"])
            tail_n += 1
        if (s + 1) % 50 == 0:
            mse = acc_rgb / n_acc
            curve.append({"step": s + 1, "rgb_mse": round(mse, 6),
                          "psnr": round(-10 * math.log10(max(mse, 1e-12)), 2),
                          "opacity": round(float(terms["opacity"]), 5)})
            acc_rgb, n_acc = 0.0, 0
    torch.cuda.synchronize()
    params = torch.cat([m.xyz_encoder.params.detach().view(-1), m.mlp_params.detach().view(-1)])
    return {"grid_fx": grid_fx, "binned": bool(grid_fx and tr.renderer.grid_bin),
            "seconds": round(time.time() - t0, 2), "curve": curve,
            "fx_redo_steps": redo_steps if grid_fx else None,
            "final_psnr": curve[-1]["psnr"],
            "psnr_last200": round(-10 * math.log10(max(tail / max(tail_n, 1), 1e-12)), 3),
            "params": params}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    scale = float(sys.argv[4]) if len(sys.argv) > 4 else 0.5
    dev = torch.device("cuda")
    a = run(steps, B, K, True, dev, scale)
    b = run(steps, B, K, False, dev, scale)
    pa, pb = a.pop("params"), b.pop("params")
    rel = float((pa - pb).norm() / pb.norm().clamp_min(1e-30))
    print(json.dumps({"scene": f"sphere r={R_SPHERE} coloured 0.5+0.5n, "
                               f"{'white' if scale <= 0.5 else 'black'} background, "
                               "fresh random rays every step",
                      "steps": steps, "rays": B, "models": K, "scale": scale, "fixed_point": a, "fp32_atomics": b,
                      "param_rel_l2_fx_vs_fp32": round(rel, 6)}))


if __name__ == "__main__":
    main()
