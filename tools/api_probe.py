"""Probe (dev tool): the C3 step through the renderer directly (as bench.py's
headline) vs through ml_render()'s autograd API, per-step time and, under
rocprofv3 --kernel-trace, the kernels each issues.

usage: python tools/api_probe.py [direct|api|dropin|both|bench] [K] [steps]
(bench: the bench's leg order direct, train (FusedAdam), dropin, api)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, NGP, Ray_Gate  # noqa: E402
from radnerf_amd.rendering import ml_render, render  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    B, scale = 8192, 0.5
    dev = torch.device("cuda", 0)
    model = (NGP(scale, seed=3) if K == 1 else MNGP(scale, size=K, seed=3)).to(dev)
    gate = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, model.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=0))
    noise = torch.from_numpy(S.noise(K, B, seed=2)).to(dev)
    g_rgb, g_op, g_depth = (torch.from_numpy(s).to(dev) for s in S.loss_seeds(B, K, seed=4))
    bg = torch.ones(3, device=dev)

    def direct(r):
        gg = torch.zeros_like(model.xyz_encoder.params)
        mg = torch.zeros_like(model.mlp_params)
        ag = torch.zeros_like(gate.params)
        _, _, _, gt, _ = r.forward(o, d, d, noise, bg, 1e-4, 0.0)
        r.backward(o, d, d, gt, bg, g_rgb, g_op, g_depth, None, 1e-4, gg, mg, ag)

    def api(_r):
        model.zero_grad(set_to_none=True)
        gate.zero_grad(set_to_none=True)
        if K == 1:
            res = render(model, o, d, noise=noise[0])
            torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]],
                                    [g_rgb, g_op, g_depth[:, 0]])
        else:
            res = ml_render(model, gate, o, d, d, noise=noise)
            torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]],
                                    [g_rgb, g_op, g_depth])

    def dropin(_r):
        model.zero_grad(set_to_none=True)
        gate.zero_grad(set_to_none=True)
        res = ml_render(model, gate, o, d, d, noise=noise, fused=False)
        torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]],
                                [g_rgb, g_op, g_depth])

    opt = None

    def train(r):
        nonlocal opt
        from radnerf_amd import dist as rdist
        from radnerf_amd.optim import FusedAdam
        if opt is None:
            train.ar = rdist.GradAllReduce([model.xyz_encoder.params, model.mlp_params,
                                            gate.params], dev)
            for p_, v_ in zip([model.xyz_encoder.params, model.mlp_params, gate.params],
                              train.ar.views):
                p_.grad = v_
            opt = FusedAdam([model.xyz_encoder.params, model.mlp_params, gate.params], lr=1e-2,
                            eps=1e-15)
        ar = train.ar
        ar.zero()
        tgt = torch.rand(B, 3, device=dev)
        r.train_step(o, d, d, tgt, noise, bg, 1e-3, 1e-2, 5e-2, 1e-4, 0.0, ar.views[0],
                     ar.views[1], ar.views[2])
        ar.reduce_and_step(opt)

    r = FusedMLRenderer(model, gate, B)
    seq = {"both": ("direct", "api"), "bench": ("direct", "train", "dropin", "api")}.get(mode, (mode,))
    fns = {"direct": direct, "api": api, "dropin": dropin, "train": train}
    for name in seq:
        fn = fns[name]
        for _ in range(3):
            fn(r)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn(r)
        torch.cuda.synchronize()
        fx = getattr(r.ws, "_fx", None)
        print(f"{name}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/step"
              f" (direct renderer's last redo flag {int(fx[3][0]) if fx is not None else None})",
              flush=True)


if __name__ == "__main__":
    main()
