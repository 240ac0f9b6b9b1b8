"""Dev probe: rn_render_test on a few rays vs the host loop (fused=False)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch
from radnerf_amd import synthetic as S
from radnerf_amd.networks import NGP
from radnerf_amd.rendering import render
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda")
m = NGP(0.5, seed=3).to(dev)
bits = S.bitfields(1, m.cascades, p=0.3, seed=1)
with torch.no_grad():
    m.density_bitfield_0.copy_(torch.from_numpy(bits[0]))
o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, 0.5))
with torch.no_grad():
    lp = render(m, o, d, test_time=True, fused=False)
    torch.cuda.synchronize()
    print("loop ok", lp["opacity"][:4].tolist(), flush=True)
    from radnerf_amd import rendering as R
    hits = R._near_far(m, o, d)
    print("hits", hits[:, 0].tolist(), flush=True)
    te = render(m, o, d, test_time=True)
    torch.cuda.synchronize()
    print("fused ok", te["opacity"][:4].tolist(), int(te["total_samples"]), flush=True)
    print("max diff", float((te["rgb"] - lp["rgb"]).abs().max()), flush=True)
