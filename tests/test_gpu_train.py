"""GPU: §8(f) rows 2-3 -- the fused NeRFLoss (rn_nerf_loss) and the Adam step
(rn_adam) against the reference formulas evaluated with torch autograd / torch
optimizers on the same inputs, and the fused train step (render -> loss ->
backward) against autograd through ml_render_fused + the reference loss."""
import numpy as np
import pytest
import torch

from radnerf_amd import layout as LY
from radnerf_amd import synthetic as S
from radnerf_amd.fused import get_renderer, ml_render_fused
from radnerf_amd.losses import NeRFLoss, fused_nerf_loss
from radnerf_amd.networks import MNGP, Ray_Gate
from radnerf_amd.optim import FusedAdam

pytestmark = pytest.mark.gpu

LAMBDAS = dict(lambda_opacity=1e-3, lambda_cv_importance=1e-2, lambda_depth_mutual=5e-2)


def _results(cuda, B, K, seed=0):
    g = torch.Generator().manual_seed(seed)
    gate = torch.softmax(torch.randn(B, K, generator=g), 1)
    res = {"rgb": torch.rand(B, 3, generator=g), "opacity": torch.rand(B, generator=g),
           "depth": torch.rand(B, K, generator=g) * 3, "gating_code": gate,
           "gating_importance": gate.sum(0)}
    target = {"rgb": torch.rand(B, 3, generator=g)}
    return res, target


@pytest.mark.parametrize("K", [1, 2, 4])
def test_fused_loss_matches_reference_formula(cuda, K):
    B = 3000
    res, target = _results(cuda, B, K)
    # reference: losses.py NeRFLoss + train_ml.py sum of means, autograd on CPU fp64
    leaves = {k: v.double().requires_grad_(True) for k, v in res.items() if k != "gating_importance"}
    leaves_res = dict(leaves, gating_importance=leaves["gating_code"].sum(0))
    ld = NeRFLoss()(leaves_res, {"rgb": target["rgb"].double()}, **LAMBDAS)
    total = sum(v.mean() for v in ld.values())
    total.backward()
    c = lambda t: t.to(cuda)
    terms, (d_rgb, d_op, d_depth, d_gate) = fused_nerf_loss(
        c(res["rgb"]), c(target["rgb"]), c(res["opacity"]), c(res["depth"]),
        c(res["gating_code"]), c(res["gating_importance"]), **LAMBDAS)
    assert set(terms) == set(ld)
    for k in ld:
        assert abs(float(terms[k]) - float(ld[k].mean().detach())) <= 1e-5 * max(1.0, abs(float(ld[k].mean().detach()))), k
    def close(a, b):
        b = torch.zeros(a.shape, dtype=torch.float64) if b is None else b   # term absent
        return torch.allclose(a.cpu().double(), b, rtol=1e-4, atol=1e-9)
    assert close(d_rgb, leaves["rgb"].grad)
    assert close(d_op, leaves["opacity"].grad)
    assert close(d_depth, leaves["depth"].grad)
    # the reference's gate gradient from the loss: CV^2 through gating_importance
    # and the (detached) depth-mutual mean contributes nothing
    assert close(d_gate, leaves["gating_code"].grad)


@pytest.mark.parametrize("betas", [(0.9, 0.99), None])
def test_fused_adam_matches_torch_adam(cuda, betas):
    """betas=None: constructed as train_ml.py:143 constructs apex.FusedAdam
    (lr and eps only), against torch.optim.Adam's defaults (0.9, 0.999)."""
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(100_003, generator=g)
    grads = [torch.randn(100_003, generator=g) * 1e-2 for _ in range(5)]
    ref = torch.nn.Parameter(p0.clone())
    kw = {} if betas is None else {"betas": betas}
    opt_ref = torch.optim.Adam([ref], lr=1e-2, eps=1e-15, **kw)
    ours = torch.nn.Parameter(p0.clone().to(cuda))
    opt = FusedAdam([ours], lr=1e-2, eps=1e-15, **kw)
    assert opt.defaults["betas"] == opt_ref.defaults["betas"]
    for gr in grads:
        ref.grad = gr.clone()
        opt_ref.step()
        ours.grad = gr.to(cuda)
        opt.step()
    assert torch.allclose(ours.detach().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    st, st_ref = opt.state[ours], opt_ref.state[ref]
    assert torch.allclose(st["exp_avg"].cpu(), st_ref["exp_avg"], rtol=1e-5, atol=1e-9)
    assert torch.allclose(st["exp_avg_sq"].cpu(), st_ref["exp_avg_sq"], rtol=1e-5, atol=1e-12)


def _setup(cuda, B, K, scale=0.5):
    m = MNGP(scale, size=K, seed=3)
    g = Ray_Gate(K, seed=2)
    with torch.no_grad():
        m.xyz_encoder.params.copy_(torch.from_numpy(S.grid_params(m.xyz_encoder.n_entries)).view(-1))
        m.mlp_params.copy_(torch.from_numpy(S.mlp_params(K, LY.FIELD_PARAMS)))
        g.params.copy_(torch.from_numpy(S.mlp_params(1, LY.gate_params(K), seed=6)[0]))
        bits = S.bitfields(K, m.cascades, p=0.5)
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    return m.to(cuda), g.to(cuda)


@pytest.mark.parametrize("B,K,scale", [(512, 2, 0.5), (512, 4, 16.0)])
def test_fused_train_step_matches_autograd(cuda, B, K, scale):
    """(512, 4, 16): config C4's branch -- K = 4 with depth-mutual, exp step
    1/256, 6 cascades, black background (scripts/rad_360v2.sh:3-7)."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g = _setup(cuda, B, K, scale)
    o, d = (torch.from_numpy(a).to(cuda) for a in S.rays(B, scale))
    nz = torch.from_numpy(S.noise(K, B)).to(cuda)
    tgt = torch.rand(B, 3, generator=torch.Generator().manual_seed(5)).to(cuda)
    # reference structure: render (autograd) -> NeRFLoss -> sum of means -> backward
    m.zero_grad(); g.zero_grad()
    res = ml_render_fused(m, g, o, d, d, noise=nz, exp_step_factor=esf)
    ld = NeRFLoss()(res, {"rgb": tgt}, **LAMBDAS)
    assert "depth_mutual" in ld or K == 1
    sum(v.mean() for v in ld.values()).backward()
    ref = [m.xyz_encoder.params.grad.clone(), m.mlp_params.grad.clone(), g.params.grad.clone()]
    # fused train step
    r = get_renderer(m, g, B)
    bg = torch.ones(3, device=cuda) if esf == 0 else torch.zeros(3, device=cuda)
    terms, grads = r.train_step(o, d, d, tgt, nz, bg, exp_step_factor=esf, **LAMBDAS)
    for k in ld:
        assert abs(float(terms[k]) - float(ld[k].mean().detach())) <= 1e-5 * max(1.0, abs(float(ld[k].mean().detach()))), k
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))
    for a, b in zip(grads, ref):
        assert rel(a, b) <= 1e-3, rel(a, b)


def test_adam_refreshes_derived_caches(cuda):
    """After an in-place kernel update the f16 table mirror is current and the
    MLP fragments are repacked (no stale weights in the next forward)."""
    B, K = 256, 2
    m, g = _setup(cuda, B, K)
    o, d = (torch.from_numpy(a).to(cuda) for a in S.rays(B, 0.5))
    nz = torch.from_numpy(S.noise(K, B)).to(cuda)
    ml_render_fused(m, g, o, d, d, noise=nz)                    # builds the caches
    opt = FusedAdam([m.xyz_encoder.params, m.mlp_params, g.params], lr=1e-2)
    for p in (m.xyz_encoder.params, m.mlp_params, g.params):
        p.grad = torch.randn_like(p) * 1e-3
    opt.step()
    f16 = m.xyz_encoder.params_f16()
    assert torch.equal(f16, m.xyz_encoder.params.detach().half())
    frags = m.packed_frags().clone()
    with torch.no_grad():
        m.mlp_params.add_(0)                                      # forces a fresh repack
    assert torch.equal(m.packed_frags(), frags)


def test_batch_rays_match_reference_formula(cuda):
    """train_ml.py:84-96 / ray_utils.py:45-70 restated in torch (CPU fp64)."""
    from radnerf_amd.rays import batch_rays, get_rays
    g = torch.Generator().manual_seed(9)
    H, W, n_img, n = 40, 50, 7, 4096
    dirs = torch.stack([torch.rand(H * W, generator=g) - 0.5, torch.rand(H * W, generator=g) - 0.5,
                        torch.ones(H * W)], -1)
    q, _ = torch.linalg.qr(torch.randn(n_img, 3, 3, generator=g))
    poses = torch.cat([q, torch.randn(n_img, 3, 1, generator=g)], 2)
    img = torch.randint(n_img, (n,), generator=g)
    pix = torch.randint(H * W, (n,), generator=g)
    ro, rd, imd = batch_rays(dirs.to(cuda), poses.to(cuda), img.to(cuda), pix.to(cuda))
    P = poses.double()[img]
    ref_d = (dirs.double()[pix][:, None, :] @ P[..., :3].transpose(1, 2))[:, 0]
    ref_i = (dirs.double().mean(0)[None, None, :].expand(n, 1, 3) @ P[..., :3].transpose(1, 2))[:, 0]
    assert torch.allclose(rd.cpu().double(), ref_d, atol=1e-6)
    assert torch.equal(ro.cpu(), poses[img][..., 3])
    assert torch.allclose(imd.cpu().double(), ref_i, atol=1e-6)
    # single-pose form of get_rays
    o1, d1 = get_rays(dirs.to(cuda), poses[0].to(cuda))
    assert torch.allclose(d1.cpu().double(), dirs.double() @ poses[0, :, :3].double().T, atol=1e-6)
    assert torch.equal(o1.cpu(), poses[0, :, 3].expand(H * W, 3))


def test_trainer_converges_fixed_point_like_fp32(cuda):
    """End to end: trainer.Trainer (density updates with warm-up, fused render,
    fused loss, merged backward, Adam) learns an analytic scene -- a coloured
    sphere before the white background, fresh rays every step -- and the
    fixed-point grid gradient trains like fp32 atomics (same init and rays).
    tools/train_demo.py runs the long form (1000 steps: 35.9 vs 35.8 dB,
    profiles/r03/train_demo_r03.json)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "train_demo", os.path.join(os.path.dirname(__file__), "..", "tools", "train_demo.py"))
    td = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(td)
    fx = td.run(300, 4096, 2, True, cuda)
    f32 = td.run(300, 4096, 2, False, cuda)
    first, last = fx["curve"][0]["psnr"], fx["final_psnr"]
    assert last > first + 10 and last > 28, fx["curve"]
    assert abs(last - f32["final_psnr"]) < 0.5, (last, f32["final_psnr"])
    assert fx["fx_redo_steps"] == 0
