"""Stage timing of MNGP.update_density_grid on the bench workload (dev tool, GPU)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402

from radnerf_amd import dist as rdist  # noqa: E402
from radnerf_amd import vren  # noqa: E402
from radnerf_amd.networks import MNGP  # noqa: E402


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e3, 3)


def main():
    dev = torch.device("cuda")
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    m = MNGP(scale, size=K, seed=3).to(dev)
    thr = 0.01 * 1024 / 3 ** 0.5
    rdist.update_density_grid(m, thr, 0, warmup=True)
    if len(sys.argv) > 2:       # occupied fraction of a trained scene: densities above thr
        occ = float(sys.argv[2])
        with torch.no_grad():
            for i in range(m.size):
                d = getattr(m, f"density_grid_{i}")
                d.copy_(torch.where(torch.rand_like(d) < occ, 2 * thr, 0.5 * thr))
    g = rdist.step_generator(dev, 0, 1)
    M = 128 ** 3 // 4
    dg = m.density_grid_0
    saved = {n: b.clone() for n, b in m.named_buffers() if "density" in n}

    def restore():
        with torch.no_grad():
            for n, b in m.named_buffers():
                if n in saved:
                    b.copy_(saved[n])

    def sampled():
        restore()
        rdist.update_density_grid(m, thr, 1, warmup=False)

    out = {"restore": t(restore),
           "sampled": t(sampled),
           "randint": t(lambda: torch.randint(128, (M, 3), dtype=torch.int32, device=dev, generator=g)),
           "nonzero": t(lambda: torch.nonzero(dg[0] > thr)[:, 0]),
           "cells": t(lambda: m.sample_uniform_and_occupied_cells(M, thr, 0, g)),
           "density_1M": t(lambda: m.density(torch.rand(2 * M, 3, device=dev) - 0.5, 0)),
           "occupied_frac": float((dg > thr).float().mean()),
           "warmup": t(lambda: rdist.update_density_grid(m, thr, 0, warmup=True))}
    print(out)


if __name__ == "__main__":
    main()
