"""Diagnostics for the fused step vs the CPU oracle (GPU box; test tooling).

Prints, for one (scale, K, B) setup of tests/test_gpu_ml.py:
  * per (sub-NeRF, MLP layer): gradient norms of the oracle / fused path and
    their relative error, plus the same with the oracle's field backward fed
    the GPU's own composite seeds (isolates the field backward);
  * the rays whose rgb is furthest from the oracle, with their samples.

    python tools/diag_parity.py 16 8 256
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tests")]

from oracle import field_oracle as fo  # noqa: E402
from oracle import ml_oracle  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd.fused import get_renderer, ml_render_fused  # noqa: E402
from test_gpu_ml import LAYERS, _run, _setup  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main(scale, K, B):
    cuda = torch.device("cuda:0")
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, scale=scale, K=K)
    rf, gf = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    w = get_renderer(m, g, B).ws
    gm = m.xyz_encoder.params.detach().cpu().view(-1, 2)
    mp = m.mlp_params.detach().cpu()
    ores = ml_oracle.ml_train_step(o, d, bits, noise, gm, mp, g.params.detach().cpu(), scale,
                                   seeds=seeds)
    gate = rf["gating_code"].detach().cpu().numpy()
    cnt = w.counts.cpu().numpy()
    off = w.offsets.cpu().numpy()
    print(f"scale {scale} K {K} B {B}: samples per model {cnt.sum(1).tolist()}")
    print("gate mean per model", np.round(gate.mean(0), 4).tolist(),
          "min", np.round(gate.min(0), 6).tolist())
    # GPU composite seeds mapped to the oracle's sample order
    dsig = w.dsigma.cpu().numpy()
    drgb = w.drgb.cpu().numpy()
    lv = fo.grid_levels(scale)
    mg = gf[1].cpu().numpy()
    for k in range(K):
        idx = np.concatenate([np.arange(off[k, r], off[k, r] + cnt[k, r]) for r in range(B)])
        a = int(ores["starts"][k, 0])
        sl = slice(a, a + int(cnt[k].sum()))
        e_ds = np.abs(dsig[idx] - ores["dsigmas"][k]).max() if len(idx) else 0
        e_dr = np.abs(drgb[idx] - ores["drgbs"][k]).max() if len(idx) else 0
        # oracle field backward with the GPU seeds
        x = torch.from_numpy(ores["xyzs"][sl])
        dd = torch.from_numpy(d)[torch.from_numpy(ores["ray_of"][sl])]
        gp = gm.half().float().clone().requires_grad_(True)
        mk = mp[k].clone().requires_grad_(True)
        sig, rgb = fo.field_forward(x, dd, gp, ml_oracle._split_field(mk), lv,
                                    torch.full((1, 3), -float(scale)), torch.full((1, 3), float(scale)))
        torch.autograd.backward([sig, rgb], [torch.from_numpy(dsig[idx]), torch.from_numpy(drgb[idx])])
        og = ores["mlp_grad"][k]
        line = [f"k{k}: |dsig| {np.abs(ores['dsigmas'][k]).max():.2e} (gpu-oracle {e_ds:.1e}) "
                f"|drgb| {np.abs(ores['drgbs'][k]).max():.2e} ({e_dr:.1e})"]
        for name, (a0, b0) in LAYERS.items():
            line.append(f"  {name}: |o| {np.linalg.norm(og[a0:b0]):.2e} |f| {np.linalg.norm(mg[k, a0:b0]):.2e}"
                        f" rel {rel(mg[k, a0:b0], og[a0:b0]):.1e}"
                        f" same-seeds {rel(mg[k, a0:b0], mk.grad.numpy()[a0:b0]):.1e}")
        print("\n".join(line))
        # samples dominating the layer gradients
        sg = np.abs(dsig[idx] * sig.detach().numpy())
        top = np.argsort(-sg)[:3]
        print("   top |dsig*sigma| samples:", [(int(t), float(sg[t]), float(sig[t])) for t in top])
    # worst rgb rays
    e = np.abs(rf["rgb"].detach().cpu().numpy() - ores["rgb"]).max(1)
    for r in np.argsort(-e)[:3]:
        print(f"ray {r}: rgb err {e[r]:.2e} gate {np.round(gate[r], 4).tolist()} gate err "
              f"{np.abs(gate[r] - ores['gate'][r]).max():.2e}; rgb_k err "
              f"{np.abs(w.rgb_k.cpu().numpy()[:, r] - ores['rgb_k'][:, r]).max(1).tolist()} O_k err "
              f"{np.abs(w.opacity_k.cpu().numpy()[:, r] - ores['opacity_k'][:, r]).tolist()}")
        for k in range(K):
            n = cnt[k, r]
            if n == 0:
                continue
            gi = np.arange(off[k, r], off[k, r] + n)
            a = int(ores["starts"][k, r]) - int(ores["starts"][k, 0])
            orgb = ores["rgbs"][k][a:a + n]
            osig = ores["sigmas"][k][a:a + n]
            ws = ores["ws"][k][a:a + n]
            grgb = w.rgb.cpu().numpy()[gi]
            gsig = w.sigma.cpu().numpy()[gi]
            de = np.abs(grgb - orgb).max(1)
            j = np.argsort(-(de * ws))[:3]
            print(f"  k{k}: n {n} used {int(ores['used'][k][r])} "
                  f"max|drgb_s| {de.max():.2e} max w {ws.max():.3f}; worst w*drgb:",
                  [(int(i), float(ws[i]), float(de[i]), float(gsig[i]), float(osig[i])) for i in j])


if __name__ == "__main__":
    sc, k, b = float(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    main(sc, k, b)
