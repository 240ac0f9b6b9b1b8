"""CPU: known-answer tests pinning the oracle (oracle/vren_oracle.c) to the
reference formulas.  The reference ships no tests or golden vectors for this
path, so these analytic KATs (SURVEY.md §8c list) are the pin:

  KAT1 fully occupied grid, exp_step_factor 0: per-ray count = #steps of
       sqrt(3)/1024 from t1 + dt*noise while t < t2, capped at 1024
  KAT2 empty bitfield: no samples; composite opacity 0
  KAT3 constant sigma / colour along a ray: opacity = 1 - exp(-sigma * sum(dt))
       up to the T <= 1e-4 termination
  KAT4 single-sample backward formula
  KAT5 Morton round trip
  KAT6 a ray that misses the AABB: hits_t = -1, zero samples
plus a finite-difference check of composite_train_bw against composite_train_fw.
"""
import numpy as np
import pytest

import oracle
from radnerf_amd import synthetic as S

SQRT3 = np.float32(1.73205080757)


def _hits(o, d, scale):
    c = np.zeros((1, 3), np.float32)
    h = np.full((1, 3), scale, np.float32)
    cnt, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    ht = ht[:, 0].copy()
    m = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
    ht[m, 0] = 0.01
    return cnt, ht


def test_kat5_morton_roundtrip():
    g = np.arange(128, dtype=np.int32)
    coords = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    idx = oracle.morton3d(coords)
    assert len(np.unique(idx)) == 128 ** 3 and idx.min() == 0 and idx.max() == 128 ** 3 - 1
    assert np.array_equal(oracle.morton3d_invert(idx), coords)
    # bit interleave: x -> bit 0, y -> bit 1, z -> bit 2
    assert oracle.morton3d(np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [2, 0, 0]], np.int32)).tolist() == [1, 2, 4, 8]


def test_packbits():
    rng = np.random.default_rng(0)
    g = rng.random(8 * 1000, dtype=np.float32)
    bits = oracle.packbits(g, 0.5)
    ref = np.packbits((g > 0.5).reshape(-1, 8), axis=1, bitorder="little").reshape(-1)
    assert np.array_equal(bits, ref)


def test_kat6_miss():
    o = np.array([[2.0, 2.0, 2.0]], np.float32)
    d = np.array([[1.0, 0.0, 0.0]], np.float32)     # moving away, never enters [-0.5,0.5]^3
    cnt, ht = _hits(o, d, 0.5)
    assert cnt[0] == 0 and np.all(ht == -1)
    bits = np.full(128 ** 3 // 8, 255, np.uint8)
    ra, xyz, _, _, _, tot = oracle.raymarching_train(o, d, ht, bits, 1, 0.5, 0.0, np.zeros(1, np.float32))
    assert tot == 0 and ra[0, 2] == 0


def test_kat1_full_grid_counts():
    o, d = S.rays(300)
    _, ht = _hits(o, d, 0.5)
    nz = S.noise(1, 300)[0]
    bits = np.full(128 ** 3 // 8, 255, np.uint8)
    ra, xyz, _, dl, ts, tot = oracle.raymarching_train(o, d, ht, bits, 1, 0.5, 0.0, nz)
    dt = SQRT3 / np.float32(1024)
    for r in range(300):
        t1, t2 = ht[r]
        if t1 < 0:
            assert ra[r, 2] == 0
            continue
        t = np.float32(float(dt) * float(nz[r]) + float(t1))       # exact fmaf via fp64
        n = 0
        while 0 <= t < t2 and n < 1024:
            t = np.float32(t + dt)
            n += 1
        assert ra[r, 2] == n
    assert np.all(dl == dt)
    # samples are evenly spaced along each ray and lie inside the box
    assert np.all(np.abs(xyz) <= 0.5 + 1e-5)


def test_kat2_empty_grid():
    o, d = S.rays(200)
    _, ht = _hits(o, d, 0.5)
    bits = np.zeros(128 ** 3 // 8, np.uint8)
    ra, _, _, _, _, tot = oracle.raymarching_train(o, d, ht, bits, 1, 0.5, 0.0,
                                                   S.noise(1, 200)[0])
    assert tot == 0 and np.all(ra[:, 2] == 0)
    total, op, de, rgb, ws = oracle.composite_train_fw(np.zeros(0), np.zeros((0, 3)), np.zeros(0),
                                                       np.zeros(0), ra)
    assert np.all(op == 0) and np.all(rgb == 0) and np.all(total == 0)


def test_kat3_constant_medium():
    n, sigma, dt = 400, 3.0, 0.01
    ra = np.array([[0, 0, n]], np.int64)
    sig = np.full(n, sigma, np.float32)
    rgbs = np.tile(np.array([[0.2, 0.5, 0.9]], np.float32), (n, 1))
    dl = np.full(n, dt, np.float32)
    ts = (np.arange(n) * dt).astype(np.float32)
    total, op, de, rgb, ws = oracle.composite_train_fw(sig, rgbs, dl, ts, ra, 1e-4)
    # T_k = exp(-sigma*dt*k); termination after the first k with T_k <= 1e-4
    k_stop = int(np.ceil(np.log(1e-4) / (-sigma * dt)))
    assert total[0] == k_stop - 1
    assert abs(op[0] - (1 - np.exp(-sigma * dt * k_stop))) < 1e-5
    assert np.allclose(rgb[0], op[0] * np.array([0.2, 0.5, 0.9]), atol=1e-5)
    assert np.all(ws[k_stop:] == 0)


def test_kat4_single_sample_backward():
    sig = np.array([2.0], np.float32)
    rgbs = np.array([[0.3, 0.6, 0.9]], np.float32)
    dl = np.array([0.1], np.float32)
    ts = np.array([1.5], np.float32)
    ra = np.array([[0, 0, 1]], np.int64)
    _, op, de, rgb, ws = oracle.composite_train_fw(sig, rgbs, dl, ts, ra)
    gO, gD, gR = np.array([0.7], np.float32), np.array([-0.2], np.float32), np.array([[0.1, -0.3, 0.5]], np.float32)
    dsig, drgb = oracle.composite_train_bw(gO, gD, gR, np.zeros(1, np.float32), sig, rgbs, ws, dl,
                                           ts, ra, op, de, rgb)
    a = 1 - np.exp(-2.0 * 0.1)
    T1 = 1 - a
    # volumerendering.cu:140-147 with r=R, d=D after one sample
    expect = 0.1 * (np.sum(gR[0] * (rgbs[0] * T1 - 0)) + gO[0] * (1 - a) + gD[0] * (1.5 * T1 - 0))
    assert abs(dsig[0] - expect) < 1e-6
    assert np.allclose(drgb[0], gR[0] * a, atol=1e-7)


def test_composite_bw_finite_difference():
    rng = np.random.default_rng(2)
    n = 60
    sig = rng.gamma(1.0, 5.0, n).astype(np.float32)
    rgbs = rng.random((n, 3), dtype=np.float32)
    dl = np.full(n, 0.02, np.float32)
    ts = np.cumsum(dl).astype(np.float32)
    ra = np.array([[0, 0, n]], np.int64)
    gO, gD = np.array([0.3], np.float32), np.array([0.2], np.float32)
    gR = np.array([[0.5, -0.4, 0.8]], np.float32)

    def loss(s, c):
        _, op, de, rgb, _ = oracle.composite_train_fw(s, c, dl, ts, ra, 0.0)
        return float(gO[0] * op[0] + gD[0] * de[0] + (gR[0] * rgb[0]).sum())

    _, op, de, rgb, ws = oracle.composite_train_fw(sig, rgbs, dl, ts, ra, 0.0)
    dsig, drgb = oracle.composite_train_bw(gO, gD, gR, np.zeros(n, np.float32), sig, rgbs, ws, dl,
                                           ts, ra, op, de, rgb, 0.0)
    eps = 1e-2
    for i in (0, 7, 30, 59):
        sp, sm = sig.copy(), sig.copy()
        sp[i] += eps; sm[i] -= eps
        fd = (loss(sp, rgbs) - loss(sm, rgbs)) / (2 * eps)
        assert abs(fd - dsig[i]) < 2e-3 * max(1, abs(fd))
        cp = rgbs.copy(); cp[i, 1] += eps
        fd = (loss(sig, cp) - loss(sig, rgbs)) / eps
        assert abs(fd - drgb[i, 1]) < 1e-3


def test_raymarching_test_matches_train_without_jitter():
    """With exp_step_factor 0 the test-time march (incl. its calc_dt(cascades)
    quirk, raymarching.cu:370,399) visits the same samples as the training
    march with zero jitter."""
    n = 256
    o, d = S.rays(n)
    _, ht = _hits(o, d, 0.5)
    bits = S.bitfields(1, 1, p=0.4)[0]
    ra, xyz, _, dl, ts, tot = oracle.raymarching_train(o, d, ht, bits, 1, 0.5, 0.0,
                                                       np.zeros(n, np.float32))
    h = ht.copy()
    alive = np.arange(n, dtype=np.int64)
    txyz, _, tdl, tts, ne = oracle.raymarching_test(o, d, h, alive, bits, 1, 0.5, 0.0, 128, 1024, 1024)
    for r in range(n):
        k = ra[r, 2]
        assert ne[r] == k
        assert np.array_equal(tts[r, :k], ts[ra[r, 1]:ra[r, 1] + k])
        assert np.array_equal(txyz[r, :k], xyz[ra[r, 1]:ra[r, 1] + k])


def test_multiscale_cascades_exp_step():
    """scale 16: 6 cascades, exp_step_factor 1/256; dt grows with t and is
    clamped to [sqrt3/1024, sqrt3*2*16/128]."""
    o, d = S.rays(200, scale=16.0)
    _, ht = _hits(o, d, 16.0)
    bits = S.bitfields(1, 6, p=0.5)[0]
    ra, xyz, _, dl, ts, tot = oracle.raymarching_train(o, d, ht, bits, 6, 16.0, 1 / 256,
                                                       S.noise(1, 200)[0])
    assert tot > 0
    lo, hi = SQRT3 / np.float32(1024), SQRT3 * np.float32(2 * 16.0) / np.float32(128)
    assert dl.min() >= lo and dl.max() <= hi
    exp = np.clip(ts * np.float32(1 / 256), lo, hi)
    assert np.array_equal(dl, exp.astype(np.float32))


def test_det_expf_accuracy():
    """The compositing exponent shared by the oracle and the kernels
    (det_expf / rn_exp_det, a fixed IEEE operation sequence in place of CUDA's
    __expf) is within 1 ulp of exp over the compositing range."""
    rng = np.random.default_rng(0)
    x = np.concatenate([-rng.exponential(2.0, 20000), -rng.uniform(0, 87, 5000),
                        [0.0, -1e-30, -1e-7, -0.5, -0.6931472, -1.0, -20.0, -86.9]]).astype(np.float32)
    got = oracle.det_expf(x)
    ref = np.exp(x.astype(np.float64))
    ulp = np.spacing(np.float32(ref).astype(np.float32))
    err = np.abs(got.astype(np.float64) - ref) / ulp
    assert err.max() <= 1.0, err.max()
    assert oracle.det_expf([0.0])[0] == 1.0 and oracle.det_expf([-100.0])[0] == 0.0


def test_ml_march_threads_invariant(monkeypatch):
    """The OpenMP oracle march (count, ray-order starts, write) equals its
    sequential form: the totals and per-segment starts are the prefix sums."""
    o, d = S.rays(300, 16.0, seed=4)
    bits = S.bitfields(3, 6, p=0.3, seed=5)
    nz = S.noise(3, 300, seed=6)
    c = np.zeros(3, np.float32); h = np.full(3, 16.0, np.float32)
    counts, starts, xyzs, ts, dl, total = oracle.ml_march(o, d, c, h, nz, bits, 6, 16.0, 1 / 256)
    flat = counts.reshape(-1).astype(np.int64)
    assert total == flat.sum()
    assert np.array_equal(starts.reshape(-1), np.concatenate([[0], np.cumsum(flat)[:-1]]))
    for g in range(0, len(flat), 37):
        seg = ts[starts.reshape(-1)[g]:starts.reshape(-1)[g] + flat[g]]
        assert np.all(np.diff(seg) > 0)
