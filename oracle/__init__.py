"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
cpu_baseline).  Never imported by the product package rad-nerf_amd/.

CPU restatement of the reference path of thu-nics/Rad-NeRF:
  * vren_oracle.c  — raymarching.cu / volumerendering.cu / intersection.cu
                     restated serially in C (ctypes wrappers below);
  * field_oracle.py — MNGP / Ray_Gate (models/networks.py) over tcnn semantics,
                      torch-CPU fp32 with the f16 rounding points of the kernels;
  * ml_oracle.py    — ml_render (models/ml_rendering.py) train step fwd + bwd.

Parity unpinned: the reference holds no tests/fixtures for this path and its
CUDA extension is unbuildable here.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        _lib = ctypes.CDLL(_SO)
        _lib.oracle_raymarching_train.restype = ctypes.c_int64
        _lib.oracle_ml_march.restype = ctypes.c_int64
        _lib.oracle_morton3d_one.restype = ctypes.c_uint32
        _lib.oracle_morton3d_invert_one.restype = ctypes.c_uint32
        _lib.oracle_det_expf.restype = ctypes.c_float
        _lib.oracle_det_expf.argtypes = [ctypes.c_float]
    return _lib


def set_threads(n):
    """OpenMP threads of the C loops (bench.py's CPU-baseline thread sweep)."""
    lib().oracle_set_threads(ctypes.c_int(int(n)))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


I64 = ctypes.c_int64
I32 = ctypes.c_int32
F32 = ctypes.c_float


def det_expf(x):
    """The compositing exponent (vren_oracle.c det_expf), elementwise."""
    f = lib().oracle_det_expf
    x = np.asarray(x, np.float32).reshape(-1)
    return np.array([f(float(v)) for v in x], np.float32)


def morton3d(coords):
    c = np.ascontiguousarray(coords, dtype=np.int32)
    out = np.zeros(len(c), np.int32)
    lib().oracle_morton3d(_p(c), I64(len(c)), _p(out))
    return out


def morton3d_invert(idx):
    i = np.ascontiguousarray(idx, dtype=np.int32)
    out = np.zeros((len(i), 3), np.int32)
    lib().oracle_morton3d_invert(_p(i), I64(len(i)), _p(out))
    return out


def packbits(grid, thr):
    g = _f32(grid).reshape(-1)
    out = np.zeros(len(g) // 8, np.uint8)
    lib().oracle_packbits(_p(g), I64(len(out)), F32(thr), _p(out))
    return out


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    o, d, c, h = map(_f32, (rays_o, rays_d, centers, half_sizes))
    n = len(o)
    cnt = np.zeros(n, np.int32)
    ht = np.zeros((n, max_hits, 2), np.float32)
    hi = np.zeros((n, max_hits), np.int64)
    lib().oracle_ray_aabb_intersect(_p(o), _p(d), _p(c), _p(h), I64(n), I64(len(c)),
                                    I32(max_hits), _p(cnt), _p(ht), _p(hi))
    return cnt, ht, hi


def raymarching_train(rays_o, rays_d, hits_t, bitfield, cascades, scale, esf, noise,
                      grid_size=128, max_samples=1024):
    """Returns rays_a (B,3) i64, xyzs, dirs, deltas, ts (exact size), total."""
    o, d, ht, nz = map(_f32, (rays_o, rays_d, hits_t, noise))
    bits = np.ascontiguousarray(bitfield, dtype=np.uint8)
    n = len(o)
    rays_a = np.zeros((n, 3), np.int64)
    L = lib()
    args = (_p(o), _p(d), _p(ht), _p(bits), I32(cascades), F32(scale), F32(esf), _p(nz),
            I32(grid_size), I32(max_samples), I64(n))
    total = L.oracle_raymarching_train(*args, I64(0), _p(rays_a), None, None, None, None)
    xyzs = np.zeros((total, 3), np.float32)
    dirs = np.zeros((total, 3), np.float32)
    deltas = np.zeros(total, np.float32)
    ts = np.zeros(total, np.float32)
    L.oracle_raymarching_train(*args, I64(total), _p(rays_a), _p(xyzs), _p(dirs), _p(deltas),
                               _p(ts))
    return rays_a, xyzs, dirs, deltas, ts, int(total)


def raymarching_test(rays_o, rays_d, hits_t, alive, bitfield, cascades, scale, esf, grid_size,
                     max_samples, n_samples):
    """hits_t (B,2) float32 numpy array is advanced IN PLACE (reference semantics)."""
    o, d = _f32(rays_o), _f32(rays_d)
    assert hits_t.dtype == np.float32 and hits_t.flags.c_contiguous
    al = np.ascontiguousarray(alive, dtype=np.int64)
    bits = np.ascontiguousarray(bitfield, dtype=np.uint8)
    na = len(al)
    xyzs = np.zeros((na, n_samples, 3), np.float32)
    dirs = np.zeros((na, n_samples, 3), np.float32)
    deltas = np.zeros((na, n_samples), np.float32)
    ts = np.zeros((na, n_samples), np.float32)
    ne = np.zeros(na, np.int32)
    lib().oracle_raymarching_test(_p(o), _p(d), _p(hits_t), _p(al), I64(na), _p(bits),
                                  I32(cascades), F32(scale), F32(esf), I32(grid_size),
                                  I32(max_samples), I32(n_samples), _p(xyzs), _p(dirs),
                                  _p(deltas), _p(ts), _p(ne))
    return xyzs, dirs, deltas, ts, ne


def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold=1e-4):
    s, c, dl, t = map(_f32, (sigmas, rgbs, deltas, ts))
    ra = np.ascontiguousarray(rays_a, dtype=np.int64)
    nr = len(ra)
    total = np.zeros(nr, np.int64)
    op = np.zeros(nr, np.float32)
    de = np.zeros(nr, np.float32)
    rgb = np.zeros((nr, 3), np.float32)
    ws = np.zeros(len(s), np.float32)
    lib().oracle_composite_train_fw(_p(s), _p(c), _p(dl), _p(t), _p(ra), I64(nr),
                                    F32(T_threshold), _p(total), _p(op), _p(de), _p(rgb), _p(ws))
    return total, op, de, rgb, ws


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts,
                       rays_a, opacity, depth, rgb, T_threshold=1e-4):
    arrs = list(map(_f32, (dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts)))
    ra = np.ascontiguousarray(rays_a, dtype=np.int64)
    op, de, rg = map(_f32, (opacity, depth, rgb))
    n = len(arrs[4])
    dsig = np.zeros(n, np.float32)
    drgb = np.zeros((n, 3), np.float32)
    lib().oracle_composite_train_bw(*[_p(a) for a in arrs], _p(ra), I64(len(ra)), _p(op), _p(de),
                                    _p(rg), F32(T_threshold), _p(dsig), _p(drgb))
    return dsig, drgb


def composite_test_fw(sigmas, rgbs, deltas, ts, alive, T_threshold, n_eff, opacity, depth, rgb):
    """alive / opacity / depth / rgb are numpy arrays updated IN PLACE."""
    s, c, dl, t = map(_f32, (sigmas, rgbs, deltas, ts))
    ne = np.ascontiguousarray(n_eff, dtype=np.int32)
    na, ns = s.shape
    lib().oracle_composite_test_fw(_p(s), _p(c), _p(dl), _p(t), I64(na), I32(ns), _p(alive),
                                   F32(T_threshold), _p(ne), _p(opacity), _p(depth), _p(rgb))


def ml_march(rays_o, rays_d, center, half_size, noise, bitfields, cascades, scale, esf,
             grid_size=128, max_samples=1024, near_distance=0.01):
    """Fused K-model march.  Returns counts [K,B] i32, starts [K,B] i64 (dense,
    model-major), xyzs, ts, deltas for all samples, total."""
    o, d, c, h = map(_f32, (rays_o, rays_d, center, half_size))
    nz = _f32(noise)
    bf = np.ascontiguousarray(bitfields, dtype=np.uint8)
    K, nbytes = bf.shape
    B = len(o)
    counts = np.zeros((K, B), np.int32)
    starts = np.zeros((K, B), np.int64)
    L = lib()
    args = (_p(o), _p(d), _p(c), _p(h), F32(near_distance), _p(nz), _p(bf), I64(nbytes), I32(K),
            I32(cascades), F32(scale), F32(esf), I32(grid_size), I32(max_samples), I64(B))
    total = L.oracle_ml_march(*args, I64(0), _p(counts), _p(starts), None, None, None)
    xyzs = np.zeros((total, 3), np.float32)
    ts = np.zeros(total, np.float32)
    deltas = np.zeros(total, np.float32)
    L.oracle_ml_march(*args, I64(total), _p(counts), _p(starts), _p(xyzs), _p(ts), _p(deltas))
    return counts, starts, xyzs, ts, deltas, int(total)


def ray_sphere_intersect(rays_o, rays_d, centers, radii, max_hits):
    o, d, c, r = map(_f32, (rays_o, rays_d, centers, radii))
    n = len(o)
    cnt = np.zeros(n, np.int32)
    ht = np.zeros((n, max_hits, 2), np.float32)
    hi = np.zeros((n, max_hits), np.int64)
    lib().oracle_ray_sphere_intersect(_p(o), _p(d), _p(c), _p(r), I64(n), I64(len(c)),
                                      I32(max_hits), _p(cnt), _p(ht), _p(hi))
    return cnt, ht, hi


def distortion_loss_fw(ws, deltas, ts, rays_a):
    """losses.cu:62-110 -> loss (N_rays), ws_inclusive_scan, wts_inclusive_scan."""
    w, dl, t = map(_f32, (ws, deltas, ts))
    ra = np.ascontiguousarray(rays_a, dtype=np.int64)
    loss = np.zeros(len(ra), np.float32)
    wi = np.zeros(len(w), np.float32)
    wti = np.zeros(len(w), np.float32)
    lib().oracle_distortion_loss_fw(_p(w), _p(dl), _p(t), _p(ra), I64(len(ra)), _p(loss),
                                    _p(wi), _p(wti))
    return loss, wi, wti


def distortion_loss_bw(dL_dloss, ws_incl, wts_incl, ws, deltas, ts, rays_a):
    g, wi, wti, w, dl, t = map(_f32, (dL_dloss, ws_incl, wts_incl, ws, deltas, ts))
    ra = np.ascontiguousarray(rays_a, dtype=np.int64)
    out = np.zeros(len(w), np.float32)
    lib().oracle_distortion_loss_bw(_p(g), _p(wi), _p(wti), _p(w), _p(dl), _p(t), _p(ra),
                                    I64(len(ra)), _p(out))
    return out


def raymarching_train_bw(dL_dxyzs, dL_ddirs, ts, rays_a):
    gx, gd, t = map(_f32, (dL_dxyzs, dL_ddirs, ts))
    ra = np.ascontiguousarray(rays_a, dtype=np.int64)
    go = np.zeros((len(ra), 3), np.float32)
    gdir = np.zeros((len(ra), 3), np.float32)
    lib().oracle_raymarching_train_bw(_p(gx), _p(gd), _p(t), _p(ra), I64(len(ra)), _p(go),
                                      _p(gdir))
    return go, gdir
