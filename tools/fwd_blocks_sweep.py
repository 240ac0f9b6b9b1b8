"""Forward launch-shape sweep (dev tool, GPU): field_fwd per-model kernel vs
the merged (chunked, models interleaved) kernel at several grid / block
shapes on the bench workload; prints median ms per configuration."""
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
    B, K = 8192, 2
    m = MNGP(0.5, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, 1, p=0.5)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B))
    nz = torch.from_numpy(S.noise(K, B)).to(dev)
    bg = torch.ones(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    r.forward(o, d, d, nz, bg)
    st = torch.cuda.current_stream().cuda_stream
    cfgs = [("s2048", False, 2048, 0, 0)] + [
        (f"m{b}x{t}", True, 0, b, t) for b in (256, 512) for t in (256, 512, 768, 1024)]
    res = {}
    for _ in range(3):
        for name, mf, fb, mb, mt in cfgs:
            r.merged_fwd = mf
            if mf:
                r.merged_fwd_blocks, r.merged_fwd_threads = mb, mt
            else:
                r.fwd_blocks = fb
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            r._field(True, o, d, st)
            b.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(a.elapsed_time(b))
    print(json.dumps({k: float(np.median(v)) for k, v in res.items()}))


if __name__ == "__main__":
    main()
