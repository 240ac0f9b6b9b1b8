"""Regenerate the golden fixtures from the CPU oracle (test infrastructure).

The reference ships no golden vectors and cannot run here, so
these fixtures are produced by oracle/ (the restatement pinned by the KATs in
tests/test_oracle.py) on the seeded synthetic inputs of radnerf_amd.synthetic.
They pin the oracle against regressions (CPU test) and are the fixed
input/output vectors the HIP path is checked against on the GPU.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]

import oracle  # noqa: E402
from oracle import ml_oracle  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402


def hits(o, d, scale):
    c = np.zeros((1, 3), np.float32)
    h = np.full((1, 3), scale, np.float32)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    ht = ht[:, 0].copy()
    m = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
    ht[m, 0] = 0.01
    return ht


def march_case(scale, n=48, p=0.5):
    o, d = S.rays(n, scale, seed=10)
    cascades = LY.cascades_for_scale(scale)
    esf = 1 / 256 if scale > 0.5 else 0.0
    bits = S.bitfields(1, cascades, p=p, seed=11)[0]
    nz = S.noise(1, n, seed=12)[0]
    ht = hits(o, d, scale)
    ra, xyz, dirs, dl, ts, tot = oracle.raymarching_train(o, d, ht, bits, cascades, scale, esf, nz)
    return dict(rays_o=o, rays_d=d, hits_t=ht, bitfield=bits, noise=nz, rays_a=ra, xyzs=xyz,
                deltas=dl, ts=ts, cascades=cascades, scale=scale, esf=esf)


def composite_case():
    rng = np.random.default_rng(13)
    counts = np.array([0, 1, 5, 64, 65, 200, 3, 128], np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    N = int(counts.sum())
    sig = rng.gamma(1.0, 15.0, N).astype(np.float32)
    rgbs = rng.random((N, 3), dtype=np.float32)
    dl = np.full(N, 0.004, np.float32)
    ts = rng.random(N, dtype=np.float32)
    ra = np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)
    tot, op, de, rgb, ws = oracle.composite_train_fw(sig, rgbs, dl, ts, ra)
    g = rng.normal(0, 1, (len(counts), 5)).astype(np.float32)
    gws = rng.normal(0, 1, N).astype(np.float32)
    dsig, drgb = oracle.composite_train_bw(g[:, 0], g[:, 1], g[:, 2:5], gws, sig, rgbs, ws, dl, ts,
                                           ra, op, de, rgb)
    return dict(sigmas=sig, rgbs=rgbs, deltas=dl, ts=ts, rays_a=ra, total=tot, opacity=op,
                depth=de, rgb=rgb, ws=ws, g=g, gws=gws, dsig=dsig, drgb=drgb)


def ml_case(B=24, K=2, scale=0.5):
    o, d = S.rays(B, scale, seed=20)
    bits = S.bitfields(K, LY.cascades_for_scale(scale), p=0.5, seed=21)
    nz = S.noise(K, B, seed=22)
    lv = LY.grid_levels(scale)
    gp = S.grid_params(lv["n_entries"], seed=23)
    mp = S.mlp_params(K, LY.FIELD_PARAMS, seed=24)
    ap = S.mlp_params(1, LY.gate_params(K), seed=25)[0]
    sd = S.loss_seeds(B, K, seed=26, std=1.0)
    r = ml_oracle.ml_train_step(o, d, bits, nz, gp, mp, ap, scale, seeds=sd)
    gg = r["grid_grad"]
    touched = np.nonzero(np.abs(gg).sum(1))[0][:512]
    return dict(rays_o=o, rays_d=d, bitfields=bits, noise=nz, seeds_rgb=sd[0], seeds_op=sd[1],
                seeds_depth=sd[2], rgb=r["rgb"], opacity=r["opacity"], depth=r["depth"],
                gate=r["gate"], counts=r["counts"], mlp_grad=r["mlp_grad"],
                gate_grad=r["gate_grad"], grid_idx=touched, grid_grad=gg[touched],
                grid_grad_norm=np.float64(np.linalg.norm(gg)), scale=scale)


def main():
    np.savez_compressed(os.path.join(HERE, "march_s0p5.npz"), **march_case(0.5))
    np.savez_compressed(os.path.join(HERE, "march_s16.npz"), **march_case(16.0, p=0.05))
    np.savez_compressed(os.path.join(HERE, "composite.npz"), **composite_case())
    np.savez_compressed(os.path.join(HERE, "ml_step.npz"), **ml_case())
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
