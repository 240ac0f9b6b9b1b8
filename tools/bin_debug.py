"""Debug: the binned backward's page pool after each step (dev tool, GPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tests")]
from radnerf_amd.fused import get_renderer, ml_render_fused  # noqa: E402
from test_gpu_ml import _run, _setup  # noqa: E402

cuda = torch.device("cuda:0")
B, K, scale = 1024, 4, 16.0
m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
r = get_renderer(m, g, B)
print("grid_fx", r.grid_fx, "grid_bin", r.grid_bin, "feat_cache", r.feat_cache,
      "int_grad", r.int_grad, "merged_bwd", r.merged_bwd)
for step in range(3):
    _, gr = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    torch.cuda.synchronize()
    w = r.ws
    acc, scales, stats, redo = w._fx
    pool = getattr(w, "_bin", None)
    print("step", step, "fx_i", w.fx_i, "redo", int(redo[0]), "scales", scales.cpu().tolist())
    if pool is not None:
        print("  pool pages", pool["pages"], "ctl", pool["ctl"][:18].cpu().tolist())
        print("  meta[:8]", pool["meta"][:8].cpu().tolist())
    print("  stats vmax", stats[:16].cpu().tolist())
    print("  grad norm", float(gr[0].norm()))
