"""Per-entry diagnosis of the fixed-point grid gradient vs fp32 atomics (dev
tool, round 5): for each level, how many entries differ in sign (or are zero
on one side only), how large those entries are relative to the level's largest
|gradient|, and the relative error of the others; plus the same for a second
fp32 run with the rays in reverse order (summation-order noise).

    python tools/fx_entry_diag.py [B] [K] [scale]      -> one JSON line
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd.fused import get_renderer, ml_render_fused  # noqa: E402
from test_gpu_ml import _run, _setup  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    scale = float(sys.argv[3]) if len(sys.argv) > 3 else 16.0
    esf = 1 / 256 if scale > 0.5 else 0.0
    cuda = torch.device("cuda")
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    lv = LY.grid_levels(scale)
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    unit = (1.0 / r.ws._fx[1][r.ws.fx_i].abs().clamp_min(1e-30)).cpu().numpy()
    _, gfx = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.grid_fx = False
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    rev = (o[::-1].copy(), d[::-1].copy(), noise[:, ::-1].copy(), tuple(x[::-1].copy() for x in seeds))
    _, g32r = _run(ml_render_fused, m, g, *rev, cuda, esf)
    r.grid_fx = True
    out = {"shape": [B, K, scale], "binned": bool(r.grid_bin), "levels": []}
    A, Bv, C = (x[0].view(-1, 2).cpu().numpy().astype(np.float64) for x in (gfx, g32, g32r))
    for l in range(16):
        a0, n = int(lv["offset"][l]), int(lv["hsize"][l])
        a, b, c = A[a0:a0 + n].ravel(), Bv[a0:a0 + n].ravel(), C[a0:a0 + n].ravel()
        mx = float(np.abs(b).max()) or 1.0

        def stats(x, y):
            flip = (np.sign(x) != np.sign(y))
            nz = y != 0
            rel = np.abs(x - y)[nz & ~flip] / np.abs(y[nz & ~flip])
            fy = np.abs(y[flip]) / mx
            return {"flip": int(flip.sum()), "nz": int(nz.sum()),
                    "flip_mag_q": [float(np.quantile(fy, q)) for q in (0.5, 0.9, 0.99)] if flip.any() else None,
                    "rel_q": [float(np.quantile(rel, q)) for q in (0.5, 0.9, 0.99, 0.999)] if rel.size else None,
                    "zero_one_side": int(((x == 0) != (y == 0)).sum())}
        out["levels"].append({"l": l, "unit_rel_max": float(unit[l]) / mx, "max": mx,
                              "fx": stats(a, b), "fp32_reordered": stats(c, b)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
