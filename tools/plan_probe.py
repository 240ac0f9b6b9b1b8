"""Per-ray sample counts of the merged plan at a bench shape (dev tool): the
distribution of a ray's samples over all K models (k_bwd_plan_multi stages a
ray in LDS up to 2048 samples, longer rays rank by global binary searches).
Workload from ABL_K / ABL_SCALE / ABL_RAYS (default C5)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("ABL_RAYS", 8192))
    K = int(os.environ.get("ABL_K", 8))
    scale = float(os.environ.get("ABL_SCALE", 16.0))
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, m.cascades, p=0.5)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale))
    nz = torch.from_numpy(S.noise(K, B)).to(dev)
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    r.forward(o, d, d, nz, bg, 1e-4, esf)
    torch.cuda.synchronize()
    cnt = r.ws.counts.cpu().numpy().astype(np.int64)[:K, :B]
    tot = cnt.sum(0)
    q = np.percentile(tot, [50, 90, 99, 99.9, 100]).tolist()
    print(json.dumps({"K": K, "rays": B, "scale": scale, "mean": float(tot.mean()),
                      "pct_50_90_99_999_100": q, "over_2048": int((tot > 2048).sum()),
                      "per_model_max": int(cnt.max())}))


if __name__ == "__main__":
    main()
