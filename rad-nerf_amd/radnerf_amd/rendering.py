"""Renderer glue (drop-in for models/rendering.py and models/ml_rendering.py).

`render(model, rays_o, rays_d, **kw)`            rendering.py:12-46 (single NGP)
`ml_render(model, gating_net, rays_o, rays_d, imgs_d, warmup=False, **kw)`
                                                  ml_rendering.py:11-78 (Rad-NeRF)
Both return the reference's result keys.  A training render (test_time
False) of ml_render runs the fused single-chain path (radnerf_amd.fused): the
same outputs and gradients (tests/test_gpu_ml.py: outputs within 1e-5,
gradients within 1e-3) with fewer launches and no host synchronisation, 988 vs
578 M samples/s on C3.  `fused=False` keeps the reference's op-by-op autograd
structure (RayAABBIntersector -> RayMarcher -> model(x, d, i) ->
VolumeRenderer per sub-NeRF, then background and the gate-weighted combine).

Test-time rendering (test_time=True) runs rn_render_test by default: one
wave per ray marches, evaluates and composites its samples 32 at a time until
the transmittance threshold, all sub-NeRFs in one launch, no host loop
(render.hip).  `fused=False` keeps the host-driven compaction loop of
ml_rendering.py:81-155 / rendering.py:113-189 (vren.raymarching_test + field +
vren.composite_test_fw per round); both give the same per-ray results up to
float rounding (tests/test_gpu_render.py).
"""
import torch

from . import vren
from ._lib import lib
from .custom_functions import RayAABBIntersector, RayMarcher, VolumeRenderer
from .fused import grad_unsupported

MAX_SAMPLES = 1024
NEAR_DISTANCE = 0.01


def _near_far(model, rays_o, rays_d):
    """AABB hits with the NEAR_DISTANCE clamp (ml_rendering.py:48-50)."""
    _, hits_t, _ = RayAABBIntersector.apply(rays_o, rays_d, model.center, model.half_size, 1)
    near = hits_t[:, 0, 0]
    clamp = (near >= 0) & (near < NEAR_DISTANCE)
    hits_t[clamp, 0, 0] = NEAR_DISTANCE
    return hits_t


def _background(exp_step_factor, random_bg, device):
    """rendering.py:226-233 / ml_rendering.py:192-198"""
    if exp_step_factor == 0:
        return torch.ones(3, device=device)
    if random_bg:
        return torch.rand(3, device=device)
    return torch.zeros(3, device=device)


def _train_rays(model, rays_o, rays_d, hits_t, bitfield, call_model, kw):
    """One model's training render (ml_rendering.py:158-202)."""
    esf = kw.get("exp_step_factor", 0.0)
    out = {}
    rays_a, xyzs, dirs, deltas, ts, n_march = RayMarcher.apply(
        rays_o, rays_d, hits_t[:, 0], bitfield, model.cascades, model.scale, esf,
        model.grid_size, MAX_SAMPLES, kw.get("noise"))
    out["deltas"], out["ts"], out["rm_samples"] = deltas, ts, n_march
    sigmas, rgbs = call_model(xyzs, dirs)
    vr, opacity, depth, rgb, ws = VolumeRenderer.apply(
        sigmas, rgbs.contiguous(), deltas, ts, rays_a, kw.get("T_threshold", 1e-4))
    bg = _background(esf, kw.get("random_bg", False), rays_o.device)
    out.update({"vr_samples": vr, "opacity": opacity, "depth": depth, "ws": ws,
                "rays_a": rays_a, "rgb": rgb + bg * (1 - opacity)[:, None]})
    return out


@torch.no_grad()
def _test_rays(model, rays_o, rays_d, hits_t, bitfield, call_model, kw):
    """Progressive-compaction inference (ml_rendering.py:81-155)."""
    esf = kw.get("exp_step_factor", 0.0)
    n_rays, dev = rays_o.shape[0], rays_o.device
    opacity = torch.zeros(n_rays, device=dev)
    depth = torch.zeros(n_rays, device=dev)
    rgb = torch.zeros(n_rays, 3, device=dev)
    alive = torch.arange(n_rays, device=dev)
    min_samples = 1 if esf == 0 else 4
    taken, total = 0, 0
    deltas = None
    hits0 = hits_t[:, 0].contiguous()
    while taken < kw.get("max_samples", MAX_SAMPLES):
        n_alive = alive.shape[0]
        if n_alive == 0:
            break
        step = max(min(n_rays // n_alive, 64), min_samples)
        taken += step
        xyzs, dirs, deltas, ts, n_eff = vren.raymarching_test(
            rays_o, rays_d, hits0, alive, bitfield, model.cascades, model.scale, esf,
            model.grid_size, MAX_SAMPLES, step)
        total += n_eff.sum()
        xyzs = xyzs.reshape(-1, 3)
        dirs = dirs.reshape(-1, 3)
        valid = ~torch.all(dirs == 0, dim=1)
        if valid.sum() == 0:
            break
        sig = torch.zeros(xyzs.shape[0], device=dev)
        col = torch.zeros(xyzs.shape[0], 3, device=dev)
        s_v, c_v = call_model(xyzs[valid], dirs[valid])
        sig[valid] = s_v.float()
        col[valid] = c_v.float()
        vren.composite_test_fw(sig.view(-1, step), col.view(-1, step, 3), deltas, ts, hits0,
                               alive, kw.get("T_threshold", 1e-4), n_eff, opacity, depth, rgb)
        alive = alive[alive >= 0]
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    return {"opacity": opacity, "depth": depth, "rgb": rgb + bg * (1 - opacity)[:, None],
            "total_samples": total, "deltas": deltas}


@torch.no_grad()
def _test_fused(model, rays_o, rays_d, hits_t, kw):
    """Test-time renders of all model.size sub-NeRFs in one rn_render_test
    launch; a list of per-sub-NeRF results with _test_rays' keys ('deltas' is
    None: there are no per-round sample buffers)."""
    K, B, dev = model.size, rays_o.shape[0], rays_o.device
    esf = kw.get("exp_step_factor", 0.0)
    bf = [getattr(model, f"density_bitfield_{i}") for i in range(K)]
    nb = bf[0].numel()
    bits = torch.stack([b.view(-1) for b in bf]).contiguous()
    opacity = torch.empty(K, B, device=dev)
    depth = torch.empty(K, B, device=dev)
    rgb = torch.empty(K, B, 3, device=dev)
    n_smp = torch.empty(K, B, device=dev, dtype=torch.int32)
    hits = hits_t[:, 0].contiguous()
    enc = model.xyz_encoder
    lo, lh, lr, ls = enc.level_ptrs()
    # 4 waves per block, ~2 blocks per CU and sub-NeRF in flight; rays go
    # round-robin over the waves, so the grid only needs to fill the chip
    blocks = max(1, min((B + 3) // 4, 512 // K))
    if B > 0:
        lib().render_test(rays_o.data_ptr(), rays_d.data_ptr(), hits.data_ptr(), B, K,
                          bits.data_ptr(), nb, model.cascades, float(model.scale), float(esf),
                          model.grid_size, int(kw.get("max_samples", MAX_SAMPLES)),
                          enc.params_f16().data_ptr(), lo, lh, lr, ls, model._h_min.ctypes.data,
                          model._h_ext.ctypes.data, model.packed_frags().data_ptr(),
                          float(kw.get("T_threshold", 1e-4)), opacity.data_ptr(), depth.data_ptr(), rgb.data_ptr(), n_smp.data_ptr(),
                          blocks, torch.cuda.current_stream(dev).cuda_stream)
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    return [{"opacity": opacity[i], "depth": depth[i],
             "rgb": rgb[i] + bg * (1 - opacity[i])[:, None],
             "total_samples": n_smp[i].sum(), "deltas": None} for i in range(K)]


class _SingleGate:
    """Gate of a single NGP for the fused renderer: softmax over one model is
    exactly 1, so the renderer skips the gate MLP (no parameters)."""
    out_dim = 1
    type = "ray"

    def __init__(self, device):
        self.params = torch.zeros(0, device=device)


def _single_gate(model):
    g = getattr(model, "_fused_single_gate", None)
    if g is None or g.params.device != model.mlp_params.device:
        g = _SingleGate(model.mlp_params.device)
        model._fused_single_gate = g
    return g


class _TrainResults(dict):
    """render()'s training result on the fused chain.  rgb / opacity / depth
    are there at once; the per-sample keys of __render_rays_train
    (rendering.py:207-239: rays_a, ws, deltas, ts, rm_samples, vr_samples) are
    copied out of the renderer's workspace on first access (one read-back of
    the sample count), so a training step that only reads rgb / opacity pays
    nothing for them.  Reading them after another forward has reused the
    workspace raises.  ws carries no gradient through the fused chain: a
    loss on it (e.g. a distortion loss) raises at backward."""
    LAZY = ("rays_a", "ws", "deltas", "ts", "rm_samples", "vr_samples")

    def __init__(self, base, renderer, anchor):
        super().__init__(base)
        self._r, self._gen, self._anchor = renderer, renderer.ws.generation, anchor

    def __contains__(self, key):
        return super().__contains__(key) or key in self.LAZY

    def __missing__(self, key):
        if key not in self.LAZY:
            raise KeyError(key)
        w = self._r.ws
        if w.generation != self._gen:
            raise RuntimeError(f"render(): '{key}' read after another forward reused the "
                               "renderer's workspace; read it before the next render")
        n = int(w.meta[1])                      # K = 1: segment 0 starts at 0
        if key == "rays_a":
            v = torch.stack((torch.arange(w.B, device=w.device, dtype=torch.int32),
                             w.offsets[0], w.counts[0]), 1)
        elif key == "ws":
            v = grad_unsupported(w.ws[:n], self._anchor, "render() ws")
        elif key == "deltas":
            v = w.deltas[:n].clone()
        elif key == "ts":
            v = w.ts[:n].clone()
        elif key == "rm_samples":
            v = w.meta[1].clone()
        else:
            v = w.used.sum()
        self[key] = v
        return v

    # the lazy keys are keys of the result for every dict access path, not
    # only [] / in: get, iteration, keys / values / items, len,
    # dict(res) and copies materialise them like [] does
    def get(self, key, default=None):
        return self[key] if key in self else default

    def _all(self):
        for k in self.LAZY:
            if not dict.__contains__(self, k):
                self[k]
        return self

    def keys(self):
        return dict.keys(self._all())

    def values(self):
        return dict.values(self._all())

    def items(self):
        return dict.items(self._all())

    def __iter__(self):
        return dict.__iter__(self._all())

    def __len__(self):
        return dict.__len__(self) + sum(1 for k in self.LAZY if not dict.__contains__(self, k))

    def copy(self):
        return dict(self.items())


def _train_fused(model, rays_o, rays_d, kw):
    """rendering.py:192-239 on the fused K = 1 chain (radnerf_amd.fused):
    march, field, composite and background as one launch chain forward and
    backward, merged fixed-point grid-gradient scatter, no host sync."""
    from .fused import get_renderer, ml_render_fused
    gate = _single_gate(model)
    kw = dict(kw)
    noise = kw.pop("noise", None)
    if noise is not None:
        kw["noise"] = noise.reshape(1, -1)
    res = ml_render_fused(model, gate, rays_o, rays_d, rays_d, **kw)
    r = get_renderer(model, gate, rays_o.shape[0], grad=torch.is_grad_enabled())
    return _TrainResults({"rgb": res["rgb"], "opacity": res["opacity"],
                          "depth": res["depth"][:, 0]}, r,
                         (model.mlp_params, model.xyz_encoder.params))


def render(model, rays_o, rays_d, **kwargs):
    """rendering.py:12-46 for a single NGP model.  Training renders take the
    fused chain (fused=True, the default); fused=False keeps the reference's
    op-by-op autograd structure (RayMarcher -> model -> VolumeRenderer)."""
    fused = kwargs.pop("fused", True)
    if fused and not kwargs.get("test_time", False):
        return _to_host(_train_fused(model, rays_o, rays_d, kwargs), kwargs)
    with torch.autocast("cuda"):
        rays_o, rays_d = rays_o.contiguous(), rays_d.contiguous()
        hits_t = _near_far(model, rays_o, rays_d)
        if kwargs.get("test_time", False) and fused:
            return _to_host(_test_fused(model, rays_o, rays_d, hits_t, kwargs)[0], kwargs)
        fn = _test_rays if kwargs.get("test_time", False) else _train_rays
        call = lambda x, d: model(x, d)
        res = fn(model, rays_o, rays_d, hits_t, model.density_bitfield, call, kwargs)
        return _to_host(res, kwargs)


def _to_host(res, kw):
    if kw.get("to_cpu", False):
        if isinstance(res, _TrainResults):
            for k in _TrainResults.LAZY:         # materialise before copying out
                res[k]
        res = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in res.items()}
        if kw.get("to_numpy", False):
            res = {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in res.items()}
    return res


def ml_render(model, gating_net, rays_o, rays_d, imgs_d, warmup=False, **kwargs):
    """ml_rendering.py:11-78: gate, K sub-NeRF renders, gate-weighted combine.
    fused (default: training renders) routes to radnerf_amd.fused."""
    fused = kwargs.pop("fused", True)
    if fused and not kwargs.get("test_time", False):
        from .fused import ml_render_fused
        return ml_render_fused(model, gating_net, rays_o, rays_d, imgs_d, warmup, **kwargs)
    with torch.autocast("cuda"):
        rays_o, rays_d = rays_o.contiguous(), rays_d.contiguous()
        second = imgs_d.contiguous() if gating_net.type == "image" else rays_d
        gate, importance, _ = gating_net(torch.cat((rays_o, second), 1), warmup)
        B, K, dev = rays_o.shape[0], model.size, rays_o.device
        rgb_acc = torch.zeros(B, 3, device=dev)
        op_acc = torch.zeros(B, device=dev)
        depth_all = torch.zeros(B, K, device=dev)
        singles, total_k = [], []
        noise = kwargs.pop("noise", None)
        fn = _test_rays if kwargs.get("test_time", False) else _train_rays
        test_fused = None
        if kwargs.get("test_time", False) and fused:
            # every sub-NeRF's test-time render in one launch (the same AABB
            # interval for all of them, as the per-model _near_far below)
            test_fused = _test_fused(model, rays_o, rays_d, _near_far(model, rays_o, rays_d),
                                     kwargs)
        for i in range(K):
            if test_fused is not None:
                r = _to_host(test_fused[i], kwargs)
            else:
                hits_t = _near_far(model, rays_o, rays_d)
                kw = dict(kwargs)
                if noise is not None:
                    kw["noise"] = noise[i]
                call = lambda x, d, i=i: model(x, d, i)
                r = fn(model, rays_o, rays_d, hits_t, getattr(model, f"density_bitfield_{i}"),
                       call, kw)
                r = _to_host(r, kwargs)
            singles.append(r["rgb"])
            total_k.append(r["total_samples"] if "total_samples" in r else 0)
            rgb_acc = rgb_acc + r["rgb"] * gate[:, i][:, None]
            depth_all[:, i] = r["depth"]
            op_acc = op_acc + r["opacity"] * gate[:, i]
        out = {"rgb": rgb_acc, "independent_rgbs": singles, "depth": depth_all,
               "opacity": op_acc, "gating_code": gate, "gating_importance": importance}
        if kwargs.get("test_time", False):
            # samples composited over all sub-NeRFs (a device scalar)
            out["total_samples"] = sum(total_k)
        return out
