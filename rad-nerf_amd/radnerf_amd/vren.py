"""Drop-in replacement of the reference's `vren` CUDA extension
(models/csrc/binding.cpp:234-251) on the HIP library librn.so.

Same function names, positional arguments, dtypes, return arity and in-place
semantics as the reference pybind module, so models/custom_functions.py and
models/ml_rendering.py run unchanged with `import vren` resolving here.
Differences (documented in DESIGN.md §boundary):
  * raymarching_train returns exactly-sized xyzs/dirs/deltas/ts (the caller
    slices to counter[0] anyway, custom_functions.py:91-96) and rays_a rows in
    ray order (the reference's row order is atomicAdd-random);
  * kernels run on torch's current stream (the reference uses the legacy
    default stream).
Errors follow utils.h:4-6: non-CUDA or non-contiguous inputs raise
RuntimeError("<name> must be a CUDA tensor" / "must be contiguous").
"""
import torch

from ._lib import lib


def _check(name, t):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _check_f32(name, t):
    _check(name, t)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """binding.cpp:4-16 -> [hit_cnt i32 (N), hits_t f32 (N,max_hits,2), hits_voxel_idx i64]"""
    for n, t in (("rays_o", rays_o), ("rays_d", rays_d), ("centers", centers),
                 ("half_sizes", half_sizes)):
        _check_f32(n, t)
    n_rays, n_vox = rays_o.shape[0], centers.shape[0]
    dev = rays_o.device
    hit_cnt = torch.empty(n_rays, dtype=torch.int32, device=dev)
    hits_t = torch.empty(n_rays, max_hits, 2, dtype=torch.float32, device=dev)
    hits_idx = torch.empty(n_rays, max_hits, dtype=torch.int64, device=dev)
    lib().ray_aabb_intersect(_p(rays_o), _p(rays_d), _p(centers), _p(half_sizes), n_rays, n_vox,
                             int(max_hits), _p(hit_cnt), _p(hits_t), _p(hits_idx),
                             _stream(rays_o))
    return [hit_cnt, hits_t, hits_idx]


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale,
                      exp_step_factor, noise, grid_size, max_samples):
    """binding.cpp:60-81 -> [rays_a i64 (N,3), xyzs, dirs, deltas, ts, counter i32 (2)]"""
    for n, t in (("rays_o", rays_o), ("rays_d", rays_d), ("hits_t", hits_t), ("noise", noise)):
        _check_f32(n, t)
    _check("density_bitfield", density_bitfield)
    n_rays = rays_o.shape[0]
    dev = rays_o.device
    st = _stream(rays_o)
    L = lib()
    counts = torch.empty(n_rays, dtype=torch.int32, device=dev)
    offsets = torch.empty(n_rays, dtype=torch.int32, device=dev)
    seg = torch.empty(4, dtype=torch.int32, device=dev)
    args = (_p(rays_o), _p(rays_d), _p(hits_t), _p(density_bitfield), int(cascades),
            float(scale), float(exp_step_factor), _p(noise), int(grid_size), int(max_samples),
            n_rays)
    L.raymarching_train_count(*args, _p(counts), st)
    L.scan_segments(_p(counts), 1, n_rays, 1, _p(offsets), _p(seg), _p(seg[1:]), _p(seg[2:]), st)
    total = int(seg[3].item()) if n_rays > 0 else 0     # the reference's counter[0] sync
    rays_a = torch.empty(n_rays, 3, dtype=torch.int64, device=dev)
    xyzs = torch.empty(total, 3, device=dev)
    dirs = torch.empty(total, 3, device=dev)
    deltas = torch.empty(total, device=dev)
    ts = torch.empty(total, device=dev)
    L.raymarching_train_write(*args, _p(counts), _p(offsets), _p(rays_a), _p(xyzs), _p(dirs),
                              _p(deltas), _p(ts), st)
    counter = torch.tensor([total, n_rays], dtype=torch.int32, device=dev)
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale,
                     exp_step_factor, grid_size, max_samples, N_samples):
    """binding.cpp:84-106 -> [xyzs, dirs, deltas, ts, N_eff_samples]; hits_t advanced in place"""
    for n, t in (("rays_o", rays_o), ("rays_d", rays_d), ("hits_t", hits_t)):
        _check_f32(n, t)
    _check("alive_indices", alive_indices)
    _check("density_bitfield", density_bitfield)
    if alive_indices.dtype != torch.int64:
        raise RuntimeError("alive_indices must be int64")
    n = alive_indices.shape[0]
    dev = rays_o.device
    xyzs = torch.zeros(n, N_samples, 3, device=dev)
    dirs = torch.zeros(n, N_samples, 3, device=dev)
    deltas = torch.zeros(n, N_samples, device=dev)
    ts = torch.zeros(n, N_samples, device=dev)
    n_eff = torch.empty(n, dtype=torch.int32, device=dev)
    lib().raymarching_test(_p(rays_o), _p(rays_d), _p(hits_t), _p(alive_indices), n,
                           _p(density_bitfield), int(cascades), float(scale),
                           float(exp_step_factor), int(grid_size), int(max_samples),
                           int(N_samples), _p(xyzs), _p(dirs), _p(deltas), _p(ts), _p(n_eff),
                           _stream(rays_o))
    return [xyzs, dirs, deltas, ts, n_eff]


def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold):
    """binding.cpp:109-126 -> [total_samples i64 (N_rays), opacity, depth, rgb, ws]"""
    for n, t in (("sigmas", sigmas), ("rgbs", rgbs), ("deltas", deltas), ("ts", ts)):
        _check_f32(n, t)
    _check("rays_a", rays_a)
    n_rows = rays_a.shape[0]
    dev = sigmas.device
    total = torch.zeros(n_rows, dtype=torch.int64, device=dev)
    opacity = torch.zeros(n_rows, device=dev)
    depth = torch.zeros(n_rows, device=dev)
    rgb = torch.zeros(n_rows, 3, device=dev)
    ws = torch.empty(sigmas.shape[0], device=dev)
    lib().composite_train_fw(_p(sigmas), _p(rgbs), _p(deltas), _p(ts), _p(rays_a), n_rows,
                             float(T_threshold), _p(total), _p(opacity), _p(depth), _p(rgb),
                             _p(ws), _stream(sigmas))
    return [total, opacity, depth, rgb, ws]


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts,
                       rays_a, opacity, depth, rgb, T_threshold):
    """binding.cpp:129-163 -> [dL_dsigmas, dL_drgbs]"""
    for n, t in (("dL_dopacity", dL_dopacity), ("dL_ddepth", dL_ddepth), ("dL_drgb", dL_drgb),
                 ("dL_dws", dL_dws), ("sigmas", sigmas), ("rgbs", rgbs), ("ws", ws),
                 ("deltas", deltas), ("ts", ts), ("opacity", opacity), ("depth", depth),
                 ("rgb", rgb)):
        _check_f32(n, t)
    _check("rays_a", rays_a)
    n = sigmas.shape[0]
    dsig = torch.empty(n, device=sigmas.device)
    drgb = torch.empty(n, 3, device=sigmas.device)
    lib().composite_train_bw(_p(dL_dopacity), _p(dL_ddepth), _p(dL_drgb), _p(dL_dws), _p(sigmas),
                             _p(rgbs), _p(ws), _p(deltas), _p(ts), _p(rays_a), rays_a.shape[0],
                             _p(opacity), _p(depth), _p(rgb), float(T_threshold), _p(dsig),
                             _p(drgb), _stream(sigmas))
    return [dsig, drgb]


def composite_test_fw(sigmas, rgbs, deltas, ts, hits_t, alive_indices, T_threshold,
                      N_eff_samples, opacity, depth, rgb):
    """binding.cpp:166-194; updates alive_indices/opacity/depth/rgb in place"""
    for n, t in (("sigmas", sigmas), ("rgbs", rgbs), ("deltas", deltas), ("ts", ts),
                 ("opacity", opacity), ("depth", depth), ("rgb", rgb)):
        _check_f32(n, t)
    _check("alive_indices", alive_indices)
    _check("N_eff_samples", N_eff_samples)
    n_alive, n_samples = sigmas.shape[0], sigmas.shape[1]
    lib().composite_test_fw(_p(sigmas), _p(rgbs), _p(deltas), _p(ts), n_alive, n_samples,
                            _p(alive_indices), float(T_threshold), _p(N_eff_samples), _p(opacity),
                            _p(depth), _p(rgb), _stream(sigmas))


def morton3D(coords):
    """raymarching.cu:72-88 -> int32 Morton codes"""
    _check("coords", coords)
    c = coords.to(torch.int32).contiguous()
    out = torch.empty(c.shape[0], dtype=torch.int32, device=c.device)
    lib().morton3d(_p(c), c.shape[0], _p(out), _stream(c))
    return out


def morton3D_invert(indices):
    """raymarching.cu:103-119 -> int32 coords (N,3)"""
    _check("indices", indices)
    i = indices.to(torch.int32).contiguous()
    out = torch.empty(i.shape[0], 3, dtype=torch.int32, device=i.device)
    lib().morton3d_invert(_p(i), i.shape[0], _p(out), _stream(i))
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    """raymarching.cu:143-161; writes density_bitfield in place"""
    _check_f32("density_grid", density_grid)
    _check("density_bitfield", density_bitfield)
    lib().packbits(_p(density_grid), density_bitfield.numel(), float(density_threshold),
                   _p(density_bitfield), _stream(density_grid))


def distortion_loss_fw(ws, deltas, ts, rays_a):
    """binding.cpp:197-209, losses.cu:62-110 -> [loss (N_rays), ws_inclusive_scan (N),
    wts_inclusive_scan (N)]; loss is indexed by rays_a[:, 0]."""
    for n, t in (("ws", ws), ("deltas", deltas), ("ts", ts)):
        _check_f32(n, t)
    _check("rays_a", rays_a)
    n_rows, N = rays_a.shape[0], ws.shape[0]
    dev = ws.device
    loss = torch.zeros(n_rows, device=dev)
    ws_incl = torch.zeros(N, device=dev)
    wts_incl = torch.zeros(N, device=dev)
    lib().distortion_loss_fw(_p(ws), _p(deltas), _p(ts), _p(rays_a), n_rows, _p(loss),
                             _p(ws_incl), _p(wts_incl), _stream(ws))
    return [loss, ws_incl, wts_incl]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    """binding.cpp:212-231, losses.cu:113-150 -> dL_dws (N)"""
    for n, t in (("dL_dloss", dL_dloss), ("ws_inclusive_scan", ws_inclusive_scan),
                 ("wts_inclusive_scan", wts_inclusive_scan), ("ws", ws), ("deltas", deltas),
                 ("ts", ts)):
        _check_f32(n, t)
    _check("rays_a", rays_a)
    dL_dws = torch.zeros(ws.shape[0], device=ws.device)
    lib().distortion_loss_bw(_p(dL_dloss), _p(ws_inclusive_scan), _p(wts_inclusive_scan),
                             _p(ws), _p(deltas), _p(ts), _p(rays_a), rays_a.shape[0],
                             _p(dL_dws), _stream(ws))
    return dL_dws


def ray_sphere_intersect(rays_o, rays_d, centers, radii, max_hits):
    """binding.cpp:19-31, intersection.cu:153-197 -> [hit_cnt i32 (N), hits_t f32
    (N,max_hits,2), hits_sphere_idx i64 (N,max_hits)]"""
    for n, t in (("rays_o", rays_o), ("rays_d", rays_d), ("centers", centers),
                 ("radii", radii)):
        _check_f32(n, t)
    n_rays, n_sph = rays_o.shape[0], centers.shape[0]
    dev = rays_o.device
    hit_cnt = torch.empty(n_rays, dtype=torch.int32, device=dev)
    hits_t = torch.empty(n_rays, max_hits, 2, dtype=torch.float32, device=dev)
    hits_idx = torch.empty(n_rays, max_hits, dtype=torch.int64, device=dev)
    lib().ray_sphere_intersect(_p(rays_o), _p(rays_d), _p(centers), _p(radii), n_rays, n_sph,
                               int(max_hits), _p(hit_cnt), _p(hits_t), _p(hits_idx),
                               _stream(rays_o))
    return [hit_cnt, hits_t, hits_idx]


def raymarching_train_bw(dL_dxyzs, dL_ddirs, ts, rays_a):
    """RayMarcher.backward's segment_csr pair (custom_functions.py:107-110) in one
    launch -> [dL_drays_o (N_rows,3), dL_drays_d (N_rows,3)].  Not a reference vren
    export: the reference calls torch_scatter here."""
    for n, t in (("dL_dxyzs", dL_dxyzs), ("dL_ddirs", dL_ddirs), ("ts", ts)):
        _check_f32(n, t)
    _check("rays_a", rays_a)
    n_rows = rays_a.shape[0]
    go = torch.empty(n_rows, 3, device=ts.device)
    gd = torch.empty(n_rows, 3, device=ts.device)
    lib().raymarching_train_bw(_p(dL_dxyzs), _p(dL_ddirs), _p(ts), _p(rays_a), n_rows, _p(go),
                               _p(gd), _stream(ts))
    return [go, gd]
