"""GPU parity: HIP path (through the C ABI via radnerf_amd) vs the CPU oracle.

Bars (BASELINE.json north_star):
  * ray/AABB, march counts, sample t/dt/xyz, Morton, packbits: bit-exact;
  * composite rgb/depth/opacity: |diff| <= 1e-4 (fp32; the kernel folds T as
    a wave prefix product, the oracle serially; both evaluate exp(-sigma*dt)
    with the same deterministic sequence, rn_exp_det / det_expf), and the
    termination (which samples get weights) bit-exact;
  * field (f16 MFMA, fp32 accumulate) vs the torch fp32 oracle with the same
    f16 rounding points: tolerances stated per test.
"""
import numpy as np
import pytest
import torch

import oracle
from radnerf_amd import synthetic as S
from radnerf_amd import vren

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-4


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _hits(o, d, scale, dev):
    c = np.zeros((1, 3), np.float32)
    h = np.full((1, 3), scale, np.float32)
    cnt, ht, hi = vren.ray_aabb_intersect(_t(o, dev), _t(d, dev), _t(c, dev), _t(h, dev), 1)
    ocnt, oht, ohi = oracle.ray_aabb_intersect(o, d, c, h, 1)
    return cnt, ht, hi, ocnt, oht, ohi


@pytest.mark.parametrize("scale", [0.5, 16.0])
def test_ray_aabb_bit_exact(cuda, scale):
    o, d = S.rays(4096, scale)
    # include misses: flip some directions away from the box
    d[::7] = -d[::7]
    cnt, ht, hi, ocnt, oht, ohi = _hits(o, d, scale, cuda)
    assert np.array_equal(cnt.cpu().numpy(), ocnt)
    assert np.array_equal(ht.cpu().numpy().view(np.uint32), oht.view(np.uint32))
    assert np.array_equal(hi.cpu().numpy(), ohi)
    assert (ocnt == 0).any() and (ocnt == 1).any()


def test_ray_aabb_multi_box(cuda):
    o, d = S.rays(512, 0.5)
    rng = np.random.default_rng(7)
    c = rng.uniform(-0.5, 0.5, (5, 3)).astype(np.float32)
    h = rng.uniform(0.05, 0.3, (5, 3)).astype(np.float32)
    cnt, ht, hi = vren.ray_aabb_intersect(_t(o, cuda), _t(d, cuda), _t(c, cuda), _t(h, cuda), 3)
    ocnt, oht, ohi = oracle.ray_aabb_intersect(o, d, c, h, 3)
    assert np.array_equal(cnt.cpu().numpy(), ocnt)
    assert np.array_equal(ht.cpu().numpy(), oht)
    assert np.array_equal(hi.cpu().numpy(), ohi)


def _near_clamp(ht):
    ht = ht.copy()
    m = (ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01)
    ht[m, 0, 0] = 0.01
    return ht


@pytest.mark.parametrize("scale,p,esf,max_samples", [
    (0.5, 0.5, None, 1024), (0.5, 0.1, None, 1024), (16.0, 0.5, None, 1024),
    (0.5, 1.0, None, 1024), (0.5, 0.0, None, 1024),
    # full grid, constant dt, box diagonal 3.5: rays hit the 1024-sample cap
    (1.0, 1.0, 0.0, 1024),
    # a cap that falls inside a 64-step chunk of the wave march
    (1.0, 0.7, 0.0, 100)])
def test_raymarching_train_bit_exact(cuda, scale, p, esf, max_samples):
    n = 2048
    o, d = S.rays(n, scale)
    cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
    if esf is None:
        esf = 1 / 256 if scale > 0.5 else 0.0
    bits = S.bitfields(1, cascades, p=p)[0]
    nz = S.noise(1, n)[0]
    _, ht, _, _, oht, _ = _hits(o, d, scale, cuda)
    ht_np = _near_clamp(oht)
    h2 = np.ascontiguousarray(ht_np[:, 0])
    rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
        _t(o, cuda), _t(d, cuda), _t(h2, cuda), _t(bits, cuda), cascades, scale, esf,
        _t(nz, cuda), 128, max_samples)
    ora, oxyz, odir, odl, ots, otot = oracle.raymarching_train(o, d, h2, bits, cascades, scale,
                                                               esf, nz, 128, max_samples)
    assert int(counter[0]) == otot and int(counter[1]) == n
    assert np.array_equal(rays_a.cpu().numpy(), ora)
    for a, b in ((xyzs, oxyz), (dirs, odir), (deltas, odl), (ts, ots)):
        assert np.array_equal(a.cpu().numpy().view(np.uint32), b.view(np.uint32))
    if p == 0.0:
        assert otot == 0
    if p == 1.0:
        assert ora[:, 2].max() <= max_samples and otot > 0
    if esf == 0.0 and scale == 1.0:
        assert ora[:, 2].max() == max_samples       # the cap is exercised


def test_raymarching_test_bit_exact(cuda):
    n, scale = 1024, 16.0
    o, d = S.rays(n, scale)
    cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
    bits = S.bitfields(1, cascades, p=0.3)[0]
    _, _, _, _, oht, _ = _hits(o, d, scale, cuda)
    h2 = np.ascontiguousarray(_near_clamp(oht)[:, 0])
    alive = np.arange(0, n, 3, dtype=np.int64)
    g_h = _t(h2, cuda)
    res = vren.raymarching_test(_t(o, cuda), _t(d, cuda), g_h, _t(alive, cuda), _t(bits, cuda),
                                cascades, scale, 1 / 256, 128, 1024, 8)
    o_h = h2.copy()
    ores = oracle.raymarching_test(o, d, o_h, alive, bits, cascades, scale, 1 / 256, 128, 1024, 8)
    for a, b in zip(res, ores):
        assert np.array_equal(a.cpu().numpy(), b)
    assert np.array_equal(g_h.cpu().numpy(), o_h)


def _march_for_composite(n, seed=11):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 300, n)
    counts[::17] = 0
    counts[5] = 1024
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    N = int(counts.sum())
    sig = rng.gamma(1.0, 20.0, N).astype(np.float32)
    sig[rng.random(N) < 0.3] = 0.0
    rgbs = rng.random((N, 3), dtype=np.float32)
    deltas = np.full(N, np.sqrt(3) / 1024, np.float32) * rng.uniform(0.5, 2, N).astype(np.float32)
    ts = np.concatenate([np.cumsum(deltas[s:s + c]) for s, c in zip(starts, counts)]).astype(
        np.float32) if N else np.zeros(0, np.float32)
    perm = rng.permutation(n)           # rays_a rows in arbitrary order, like the reference
    rays_a = np.stack([perm, starts[perm], counts[perm]], 1).astype(np.int64)
    return sig, rgbs, deltas, ts, rays_a


def test_composite_train_fw_bw(cuda):
    n = 3000
    sig, rgbs, deltas, ts, rays_a = _march_for_composite(n)
    g = lambda a: _t(a, cuda)
    tot, op, de, rgb, ws = vren.composite_train_fw(g(sig), g(rgbs), g(deltas), g(ts), g(rays_a),
                                                   1e-4)
    otot, oop, ode, orgb, ows = oracle.composite_train_fw(sig, rgbs, deltas, ts, rays_a, 1e-4)
    assert np.abs(rgb.cpu().numpy() - orgb).max() <= RGB_TOL
    assert np.abs(op.cpu().numpy() - oop).max() <= RGB_TOL
    assert np.abs(de.cpu().numpy() - ode).max() <= RGB_TOL
    assert np.abs(ws.cpu().numpy() - ows).max() <= 1e-5
    # transmittance folds in the reference's serial order with the exponent
    # shared with the oracle (rn_exp_det / det_expf): termination is bit-exact
    assert np.array_equal(tot.cpu().numpy(), otot)
    assert np.array_equal(ws.cpu().numpy() == 0, ows == 0)
    rng = np.random.default_rng(3)
    gO, gD = rng.normal(0, 1, n).astype(np.float32), rng.normal(0, 1, n).astype(np.float32)
    gR = rng.normal(0, 1, (n, 3)).astype(np.float32)
    gW = rng.normal(0, 1, len(sig)).astype(np.float32)
    dsig, drgb = vren.composite_train_bw(g(gO), g(gD), g(gR), g(gW), g(sig), g(rgbs), ws, g(deltas),
                                         g(ts), g(rays_a), op, de, rgb, 1e-4)
    odsig, odrgb = oracle.composite_train_bw(gO, gD, gR, gW, sig, rgbs, ows, deltas, ts, rays_a,
                                             oop, ode, orgb, 1e-4)
    assert np.abs(drgb.cpu().numpy() - odrgb).max() <= 1e-4
    err = np.abs(dsig.cpu().numpy() - odsig)
    assert err.max() <= 1e-4 * max(1.0, np.abs(odsig).max())


def test_composite_test_fw(cuda):
    n_alive, ns, n_rays = 700, 8, 1000
    rng = np.random.default_rng(5)
    sig = rng.gamma(1.0, 30.0, (n_alive, ns)).astype(np.float32)
    rgbs = rng.random((n_alive, ns, 3), dtype=np.float32)
    deltas = np.full((n_alive, ns), 0.01, np.float32)
    ts = np.cumsum(deltas, 1).astype(np.float32)
    n_eff = rng.integers(0, ns + 1, n_alive).astype(np.int32)
    alive = rng.choice(n_rays, n_alive, replace=False).astype(np.int64)
    op = rng.uniform(0, 0.5, n_rays).astype(np.float32)
    de = rng.random(n_rays, dtype=np.float32)
    rgb = rng.random((n_rays, 3), dtype=np.float32)
    g = lambda a: _t(a, cuda)
    g_alive, g_op, g_de, g_rgb = g(alive), g(op), g(de), g(rgb)
    hits = g(np.zeros((n_rays, 2), np.float32))
    vren.composite_test_fw(g(sig), g(rgbs), g(deltas), g(ts), hits, g_alive, 1e-4, g(n_eff), g_op,
                           g_de, g_rgb)
    oracle.composite_test_fw(sig, rgbs, deltas, ts, alive, 1e-4, n_eff, op, de, rgb)
    assert np.array_equal(g_alive.cpu().numpy(), alive)
    assert (alive == -1).sum() > 50            # enough rays terminate to exercise the break
    assert np.abs(g_op.cpu().numpy() - op).max() <= RGB_TOL
    assert np.abs(g_rgb.cpu().numpy() - rgb).max() <= RGB_TOL
    assert np.abs(g_de.cpu().numpy() - de).max() <= RGB_TOL


def test_morton_packbits(cuda):
    rng = np.random.default_rng(0)
    coords = rng.integers(0, 128, (10000, 3)).astype(np.int32)
    m = vren.morton3D(_t(coords, cuda)).cpu().numpy()
    assert np.array_equal(m, oracle.morton3d(coords))
    inv = vren.morton3D_invert(_t(m, cuda)).cpu().numpy()
    assert np.array_equal(inv, coords)
    grid = rng.random(2 * 128 ** 3, dtype=np.float32)
    bits = torch.zeros(2 * 128 ** 3 // 8, dtype=torch.uint8, device=cuda)
    vren.packbits(_t(grid, cuda), 0.3, bits)
    assert np.array_equal(bits.cpu().numpy(), oracle.packbits(grid, 0.3))


def test_composite_termination_at_threshold(cuda):
    """Segments built so the serial transmittance lands within a few ulps of
    T_threshold at a chosen sample (both sides): the tree-order product cannot
    decide these, the serial fallback must, and the break (total_samples and
    the samples that get weights / gradients) equals the oracle's."""
    rng = np.random.default_rng(7)
    thr = np.float32(1e-4)
    n_seg = 240
    sig_l, dl_l, counts = [], [], []
    for i in range(n_seg):
        k = int(rng.integers(0, 400))
        n = k + int(rng.integers(1, 40))
        dl = (np.float32(np.sqrt(3) / 1024) * rng.uniform(0.5, 2, n)).astype(np.float32)
        # samples before k leave T well above thr: total optical depth ~ 7
        sig = (rng.uniform(0.2, 1.8, n) * 7.0 / max(1, k) / dl).astype(np.float32)
        sig[k + 1:] = rng.uniform(0, 50, n - k - 1).astype(np.float32)
        # serial T before sample k, with the shared exponent
        E = oracle.det_expf(-sig[:k] * dl[:k])
        T = np.float32(1.0)
        for e in E:
            T = np.float32(T * np.float32(np.float32(1.0) - np.float32(np.float32(1.0) - e)))
        if T <= thr:
            continue
        Ek = np.float64(thr) / np.float64(T)
        s = np.float32(-np.log(Ek) / np.float64(dl[k]))
        sig[k] = np.float32(s) + np.float32(np.spacing(s)) * np.float32(rng.integers(-4, 5))
        sig_l.append(sig); dl_l.append(dl); counts.append(n)
    counts = np.array(counts, np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    sig = np.concatenate(sig_l).astype(np.float32)
    dl = np.concatenate(dl_l).astype(np.float32)
    N = len(sig)
    rgbs = rng.random((N, 3), dtype=np.float32)
    ts = np.cumsum(dl).astype(np.float32)
    rays_a = np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)
    g = lambda a: _t(a, cuda)
    tot, op, de, rgb, ws = vren.composite_train_fw(g(sig), g(rgbs), g(dl), g(ts), g(rays_a), 1e-4)
    otot, oop, ode, orgb, ows = oracle.composite_train_fw(sig, rgbs, dl, ts, rays_a, 1e-4)
    assert np.array_equal(tot.cpu().numpy(), otot)
    assert (otot < counts).sum() > len(counts) // 4        # many break at the threshold sample
    assert np.array_equal(ws.cpu().numpy() == 0, ows == 0)
    assert np.abs(rgb.cpu().numpy() - orgb).max() <= RGB_TOL
    gO = rng.normal(0, 1, len(counts)).astype(np.float32)
    gD = rng.normal(0, 1, len(counts)).astype(np.float32)
    gR = rng.normal(0, 1, (len(counts), 3)).astype(np.float32)
    gW = np.zeros(N, np.float32)
    dsig, drgb = vren.composite_train_bw(g(gO), g(gD), g(gR), g(gW), g(sig), g(rgbs), ws, g(dl),
                                         g(ts), g(rays_a), op, de, rgb, 1e-4)
    odsig, odrgb = oracle.composite_train_bw(gO, gD, gR, gW, sig, rgbs, ows, dl, ts, rays_a,
                                             oop, ode, orgb, 1e-4)
    assert np.array_equal(drgb.cpu().numpy() == 0, odrgb == 0)
    assert np.abs(drgb.cpu().numpy() - odrgb).max() <= 1e-4


def test_scatter_max_duplicates(cuda):
    """rn_scatter_max: the density update's tmp[c, indices] = sigma with
    duplicate cells resolved by their max (numpy reference), deterministic."""
    from radnerf_amd._lib import lib
    rng = np.random.default_rng(4)
    n, m = 300000, 50000
    idx = rng.integers(0, m, n).astype(np.int64)
    val = rng.gamma(1.0, 2.0, n).astype(np.float32)
    ref = np.zeros(m, np.float32)
    np.maximum.at(ref, idx, val)
    outs = []
    for _ in range(2):
        out = torch.zeros(m, device=cuda)
        gi, gv = _t(idx, cuda), _t(val, cuda)
        lib().scatter_max(gi.data_ptr(), gv.data_ptr(), n, out.data_ptr(),
                          torch.cuda.current_stream(cuda).cuda_stream)
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], ref) and np.array_equal(outs[1], ref)
