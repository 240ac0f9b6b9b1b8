"""Diagnostic (dev tool): per hashed level, the exact sum of the fixed-point
int32 entries (torch, int64) vs the kernel's record sum (FxStats.qsum) of one
C3 merged backward, captured just before rn_grid_fx_fold."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd._lib import lib  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def main():
    B, K, scale = int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 2, 0.5
    # usage: fx_diag.py [B] [steps] [adam]
    dev = torch.device("cuda", 0)
    model = MNGP(scale, size=K, seed=3).to(dev)
    gate = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, model.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=0))
    noise = torch.from_numpy(S.noise(K, B, seed=2)).to(dev)
    g_rgb, g_op, g_depth = (torch.from_numpy(s).to(dev) for s in S.loss_seeds(B, K, seed=4))
    bg = torch.ones(3, device=dev)
    r = FusedMLRenderer(model, gate, B)
    L = lib()
    orig = L.grid_fx_fold
    cap = {}

    def fold(*args):
        acc_p, stats_p = args[3], args[6]
        w = r.ws
        acc, scales, stats, redo = w._fx
        assert acc.data_ptr() == acc_p and stats.data_ptr() == stats_p
        cap["acc"] = acc.clone()
        cap["stats"] = stats.clone()
        cap["scale"] = scales[w.fx_i].clone()
        return orig(*args)

    L.grid_fx_fold = fold
    lv = LY.grid_levels(scale)
    from radnerf_amd.optim import FusedAdam
    params = [model.xyz_encoder.params, model.mlp_params, gate.params]
    opt = FusedAdam(params, lr=1e-2, eps=1e-15) if "adam" in sys.argv else None
    n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for step in range(n_steps):
        gg = torch.zeros_like(model.xyz_encoder.params)
        mg = torch.zeros_like(model.mlp_params)
        ag = torch.zeros_like(gate.params)
        _, _, _, gt, _ = r.forward(o, d, d, noise, bg, 1e-4, 0.0)
        r.backward(o, d, d, gt, bg, g_rgb, g_op, g_depth, None, 1e-4, gg, mg, ag)
        if opt is not None:
            for p_, g_ in zip(params, (gg, mg, ag)):
                p_.grad = g_
            opt.step()
        torch.cuda.synchronize()
        st = cap["stats"]
        qsum = st[32:64].view(torch.int64)
        acc = cap["acc"].view(-1, 2).long()
        print(f"step {step}: redo {int(r.ws._fx[3][0])}")
        for l in range(16):
            a, n = int(lv["offset"][l]), int(lv["hsize"][l])
            es = int(acc[a:a + n].sum())
            mx = int(acc[a:a + n].abs().max())
            print(f"  level {l:2d} scale {float(cap['scale'][l]):.3g}: entries {es} records "
                  f"{int(qsum[l])} diff {es - int(qsum[l])}; max |entry| 2^{np.log2(max(mx, 1)):.1f} units")


if __name__ == "__main__":
    main()
