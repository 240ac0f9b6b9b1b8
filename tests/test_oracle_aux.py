"""CPU: known-answer tests pinning the oracle's restatement of the reference's
auxiliary vren ops (distortion loss, ray/sphere, RayMarcher backward) to their
published definitions.  The reference ships no fixtures for them.

  distortion  Mip-NeRF 360 eq. 15 / DVGO-v2 eq. 2, the definition the scan form
              of losses.cu:9-110 computes:
                L = sum_ij w_i w_j |t_i - t_j| + 1/3 sum_i w_i^2 delta_i
              (evaluated in float64 by the O(n^2) double sum), and its
              gradient by central differences of that definition;
  sphere      analytic entry/exit of axis-aligned rays through a sphere;
  march bw    segment sums against numpy.
"""
import numpy as np

import oracle


def _rows(counts):
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    return np.stack([np.arange(len(counts)), starts, counts], 1).astype(np.int64)


def _dist_def(w, t, d):
    w, t, d = (np.asarray(a, np.float64) for a in (w, t, d))
    return (w[:, None] * w[None, :] * np.abs(t[:, None] - t[None, :])).sum() \
        + (w * w * d).sum() / 3


def _ray_data(rng, counts):
    N = int(sum(counts))
    ws = rng.uniform(0, 0.05, N).astype(np.float32)
    deltas = rng.uniform(1e-3, 5e-3, N).astype(np.float32)
    ts = np.zeros(N, np.float32)
    o = 0
    for c in counts:   # increasing t per ray
        ts[o:o + c] = np.cumsum(rng.uniform(1e-3, 5e-3, c)) + rng.uniform(0.5, 1.0)
        o += c
    return ws, deltas, ts


def test_distortion_fw_matches_definition():
    rng = np.random.default_rng(0)
    counts = np.array([0, 1, 2, 7, 64, 65, 300])
    ws, deltas, ts = _ray_data(rng, counts)
    ra = _rows(counts)
    loss, wi, wti = oracle.distortion_loss_fw(ws, deltas, ts, ra)
    for n, (_, s, c) in enumerate(ra):
        ref = _dist_def(ws[s:s + c], ts[s:s + c], deltas[s:s + c]) if c else 0.0
        assert abs(loss[n] - ref) <= 1e-5 * max(1.0, abs(ref)) + 1e-9, (n, loss[n], ref)
        if c:
            assert np.allclose(wi[s:s + c], np.cumsum(ws[s:s + c].astype(np.float64)), rtol=1e-5)


def test_distortion_bw_matches_finite_differences():
    rng = np.random.default_rng(1)
    counts = np.array([1, 5, 40])
    ws, deltas, ts = _ray_data(rng, counts)
    ra = _rows(counts)
    g = rng.normal(size=len(counts)).astype(np.float32)
    _, wi, wti = oracle.distortion_loss_fw(ws, deltas, ts, ra)
    dws = oracle.distortion_loss_bw(g, wi, wti, ws, deltas, ts, ra)
    eps = 1e-4
    for n, (_, s, c) in enumerate(ra):
        for i in range(s, s + c):
            wp, wm = ws.astype(np.float64), ws.astype(np.float64)
            wp = wp.copy(); wm = wm.copy()
            wp[i] += eps; wm[i] -= eps
            fd = g[n] * (_dist_def(wp[s:s + c], ts[s:s + c], deltas[s:s + c])
                         - _dist_def(wm[s:s + c], ts[s:s + c], deltas[s:s + c])) / (2 * eps)
            assert abs(dws[i] - fd) <= 1e-4 * max(1.0, abs(fd)), (i, dws[i], fd)


def test_ray_sphere_analytic():
    # rays along +x at height y through a sphere of radius 1 centred at (3,0,0)
    y = np.array([0.0, 0.5, 0.99, 1.5], np.float32)
    o = np.stack([np.zeros(4), y, np.zeros(4)], 1).astype(np.float32)
    d = np.tile(np.array([[1, 0, 0]], np.float32), (4, 1))
    cnt, ht, hi = oracle.ray_sphere_intersect(o, d, np.array([[3, 0, 0]], np.float32),
                                              np.ones(1, np.float32), 1)
    h = np.sqrt(np.maximum(1 - y.astype(np.float64) ** 2, 0))
    assert cnt.tolist() == [1, 1, 1, 0]
    assert np.allclose(ht[:3, 0, 0], 3 - h[:3], atol=1e-5)
    assert np.allclose(ht[:3, 0, 1], 3 + h[:3], atol=1e-5)
    assert ht[3].tolist() == [[-1.0, -1.0]] and hi[3, 0] == -1
    # origin inside the sphere: t_near clamps to 0; sphere behind: no hit
    cnt, ht, _ = oracle.ray_sphere_intersect(np.array([[3, 0, 0], [5, 0, 0]], np.float32),
                                             d[:2], np.array([[3, 0, 0]], np.float32),
                                             np.ones(1, np.float32), 1)
    assert cnt.tolist() == [1, 0] and ht[0, 0, 0] == 0.0 and abs(ht[0, 0, 1] - 1) < 1e-6


def test_ray_sphere_sorted_by_near():
    o = np.zeros((1, 3), np.float32)
    d = np.array([[1, 0, 0]], np.float32)
    c = np.array([[9, 0, 0], [3, 0, 0], [6, 0, 0]], np.float32)
    cnt, ht, hi = oracle.ray_sphere_intersect(o, d, c, np.full(3, 0.5, np.float32), 3)
    assert cnt[0] == 3 and hi[0].tolist() == [1, 2, 0]
    assert np.allclose(ht[0, :, 0], [2.5, 5.5, 8.5])
    # max_hits 4 with 3 hits: the -1 slot sorts first, as torch::sort does
    cnt, ht, hi = oracle.ray_sphere_intersect(o, d, c, np.full(3, 0.5, np.float32), 4)
    assert hi[0].tolist() == [-1, 1, 2, 0]


def test_march_bw_segment_sums():
    rng = np.random.default_rng(2)
    counts = np.array([0, 3, 64, 129])
    ra = _rows(counts)
    N = int(counts.sum())
    gx = rng.normal(size=(N, 3)).astype(np.float32)
    gd = rng.normal(size=(N, 3)).astype(np.float32)
    ts = rng.uniform(0, 2, N).astype(np.float32)
    go, gdir = oracle.raymarching_train_bw(gx, gd, ts, ra)
    for n, (_, s, c) in enumerate(ra):
        assert np.allclose(go[n], gx[s:s + c].sum(0), atol=1e-4)
        assert np.allclose(gdir[n], (gx[s:s + c] * ts[s:s + c, None] + gd[s:s + c]).sum(0),
                           atol=1e-4)
