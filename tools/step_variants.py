"""Whole-step timing of renderer options on the bench workload (dev tool, GPU):
fwd+bwd steps with no per-launch events, variants interleaved round by round
(rule 24 of cdna_hip_programming.md §5.4); prints median ms per step.

usage: [STEP_K=K] [STEP_B=B] [STEP_SCALE=S] python tools/step_variants.py [attr=value[,attr=value]] ...
  e.g. gate_bwd_at=field gate_bwd_at=early gate_bwd_at=main
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def parse(tok):
    out = {}
    for kv in tok.split(","):
        k, v = kv.split("=")
        out[k] = int(v) if v.lstrip("-").isdigit() else v
    return out


def main():
    variants = sys.argv[1:] or ["gate_bwd_at=field", "gate_bwd_at=early", "gate_bwd_at=main"]
    dev = torch.device("cuda")
    B, K, steps = int(os.environ.get("STEP_B", 8192)), int(os.environ.get("STEP_K", 2)), 10
    scale = float(os.environ.get("STEP_SCALE", 0.5))
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, m.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=0))
    nz = torch.from_numpy(S.noise(K, B, seed=2)).to(dev)
    sd = [torch.from_numpy(a).to(dev) for a in S.loss_seeds(B, K, seed=4)]
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    gg = torch.zeros_like(m.xyz_encoder.params)
    mg = torch.zeros_like(m.mlp_params)
    ag = torch.zeros_like(g.params)
    defaults = {k: getattr(r, k) for v in variants for k in parse(v)}

    def step():
        _, _, _, gt, _ = r.forward(o, d, d, nz, bg, 1e-4, esf)
        r.backward(o, d, d, gt, bg, *sd, None, 1e-4, gg, mg, ag)

    times = {v: [] for v in variants}
    for rnd in range(6):
        for v in variants:
            for k, val in defaults.items():
                setattr(r, k, val)
            for k, val in parse(v).items():
                setattr(r, k, val)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            if rnd:
                times[v].append((time.perf_counter() - t0) / steps * 1e3)
    print(json.dumps({v: round(float(np.median(t)), 4) for v, t in times.items()}))


if __name__ == "__main__":
    main()
