"""Timing probe (dev tool): the fused march (rn_ml_march_count) at a bench
shape with and without the exponential-step t chain (debug bit 24: t taken
as tb + j * dt(tb), wrong samples, timing only) -- the chain's share of the
march.  usage: python tools/march_probe.py K scale rays"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd._lib import lib, use_ablation_build  # noqa: E402

use_ablation_build()        # rn_set_debug_flags switches live only in librn_abl.so
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def main():
    K, scale, B = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
    dev = torch.device("cuda")
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, m.cascades, p=0.5)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale))
    nz = torch.from_numpy(S.noise(K, B)).to(dev)
    bg = torch.zeros(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    r.trace = {"march"}
    L = lib()
    out = {}
    for name, flag in (("chain", 0), ("no_chain", 1 << 24), ("chain2", 0)):
        L.set_debug_flags(flag)
        r.events = {}
        for _ in range(8):
            r.forward(o, d, d, nz, bg, 1e-4, esf)
        t = r.kernel_times_ms()["march"][2:]
        out[name] = round(float(np.median(t)), 4)
    L.set_debug_flags(0)
    print(json.dumps({"K": K, "scale": scale, "rays": B, "march_ms": out}))


if __name__ == "__main__":
    main()
