"""GPU parity of the auxiliary vren ops against the CPU oracle (whose
definitions tests/test_oracle_aux.py pins):

  * ray_sphere_intersect: counts / indices bit-exact, t within 1 ulp-scale
    (1e-6 relative; both sides use IEEE div/sqrt, no contraction);
  * distortion_loss_fw/bw: the kernel's wave prefix sums add in a different
    order than the reference's serial thrust scans, and the scan form of the
    loss cancels (2*(wts_incl*ws_excl - ws_incl*wts_excl)): the f32 oracle is
    itself 5e-5 relative off the f64 definition at 400 samples/ray.  Bars:
    loss and scans 2e-4 relative; dL/dws 1e-3 relative + 1e-5 of its scale;
  * RayMarcher backward (segment sums): 1e-5 relative, through the autograd
    Function on a real march.
"""
import numpy as np
import pytest
import torch

import oracle
from radnerf_amd import synthetic as S
from radnerf_amd import vren
from radnerf_amd.custom_functions import RayMarcher
from radnerf_amd.losses import DistortionLoss

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _rows(counts):
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    return np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)


@pytest.mark.parametrize("max_hits", [1, 3])
def test_ray_sphere(cuda, max_hits):
    o, d = S.rays(4096, 0.5)
    d[::5] = -d[::5]
    rng = np.random.default_rng(3)
    c = rng.uniform(-0.4, 0.4, (4, 3)).astype(np.float32)
    r = rng.uniform(0.05, 0.3, 4).astype(np.float32)
    cnt, ht, hi = vren.ray_sphere_intersect(_t(o, cuda), _t(d, cuda), _t(c, cuda), _t(r, cuda),
                                            max_hits)
    ocnt, oht, ohi = oracle.ray_sphere_intersect(o, d, c, r, max_hits)
    assert np.array_equal(cnt.cpu().numpy(), ocnt)
    assert np.array_equal(hi.cpu().numpy(), ohi)
    np.testing.assert_allclose(ht.cpu().numpy(), oht, rtol=1e-6, atol=1e-7)
    assert (ocnt == 0).any() and (ocnt >= 1).any()


def _dist_inputs(n_rays=3000, seed=5):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 400, n_rays)
    counts[:4] = [0, 1, 64, 65]
    N = int(counts.sum())
    ws = rng.uniform(0, 0.02, N).astype(np.float32)
    deltas = rng.uniform(1e-3, 5e-3, N).astype(np.float32)
    ts = np.zeros(N, np.float32)
    o = 0
    for c in counts:   # increasing t along each ray, as the march emits
        ts[o:o + c] = np.cumsum(rng.uniform(1e-3, 5e-3, c)) + rng.uniform(0.5, 1.0)
        o += c
    return _rows(counts), ws, deltas, ts


def test_distortion_fw_bw(cuda):
    ra, ws, deltas, ts = _dist_inputs()
    loss, wi, wti = vren.distortion_loss_fw(_t(ws, cuda), _t(deltas, cuda), _t(ts, cuda),
                                            _t(ra, cuda))
    oloss, owi, owti = oracle.distortion_loss_fw(ws, deltas, ts, ra)
    np.testing.assert_allclose(loss.cpu().numpy(), oloss, rtol=2e-4, atol=1e-7)
    np.testing.assert_allclose(wi.cpu().numpy(), owi, rtol=2e-4, atol=1e-7)
    np.testing.assert_allclose(wti.cpu().numpy(), owti, rtol=2e-4, atol=1e-7)
    g = np.random.default_rng(6).normal(size=len(ra)).astype(np.float32)
    dws = vren.distortion_loss_bw(_t(g, cuda), wi, wti, _t(ws, cuda), _t(deltas, cuda),
                                  _t(ts, cuda), _t(ra, cuda))
    odws = oracle.distortion_loss_bw(g, owi, owti, ws, deltas, ts, ra)
    np.testing.assert_allclose(dws.cpu().numpy(), odws, rtol=1e-3,
                               atol=1e-5 * np.abs(odws).max())


def test_distortion_autograd(cuda):
    ra, ws, deltas, ts = _dist_inputs(500, seed=7)
    w = _t(ws, cuda).requires_grad_(True)
    loss = DistortionLoss.apply(w, _t(deltas, cuda), _t(ts, cuda), _t(ra, cuda))
    loss.mean().backward()
    _, owi, owti = oracle.distortion_loss_fw(ws, deltas, ts, ra)
    g = np.full(len(ra), 1.0 / len(ra), np.float32)
    odws = oracle.distortion_loss_bw(g, owi, owti, ws, deltas, ts, ra)
    np.testing.assert_allclose(w.grad.cpu().numpy(), odws, rtol=1e-3,
                               atol=1e-5 * np.abs(odws).max())


def test_raymarcher_backward(cuda):
    n, scale = 1024, 0.5
    o, d = S.rays(n, scale)
    bits = S.bitfields(1, 1, p=0.5)[0]
    nz = S.noise(1, n)[0]
    c = np.zeros((1, 3), np.float32)
    h = np.full((1, 3), scale, np.float32)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    ht = ht[:, 0].copy()
    m = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
    ht[m, 0] = 0.01
    ro = _t(o, cuda).requires_grad_(True)
    rd = _t(d, cuda).requires_grad_(True)
    rays_a, xyzs, dirs, deltas, ts, total = RayMarcher.apply(
        ro, rd, _t(ht, cuda), _t(bits, cuda), 1, scale, 0.0, 128, 1024, _t(nz, cuda))
    rng = np.random.default_rng(8)
    gx = rng.normal(size=tuple(xyzs.shape)).astype(np.float32)
    gd = rng.normal(size=tuple(dirs.shape)).astype(np.float32)
    torch.autograd.backward([xyzs, dirs], [_t(gx, cuda), _t(gd, cuda)])
    go, gdir = oracle.raymarching_train_bw(gx, gd, ts.detach().cpu().numpy(),
                                           rays_a.cpu().numpy())
    np.testing.assert_allclose(ro.grad.cpu().numpy(), go, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(rd.grad.cpu().numpy(), gdir, rtol=1e-5, atol=1e-4)
