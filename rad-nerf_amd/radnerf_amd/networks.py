"""Field and gate modules of Rad-NeRF on the HIP kernels.

Mirrors the reference modules' interface (models/networks.py):
  * MNGP(scale, rgb_act='Sigmoid', size=2, t=19)     networks.py:214-421
      forward(x, d, ind) -> (sigmas (N) f32, rgbs (N,3) f32)
      density(x, ind, return_feat=False) -> sigmas
      update_density_grid(...) / sample_uniform_and_occupied_cells / get_all_cells
      buffers center, xyz_min, xyz_max, half_size, grid_coords,
              density_bitfield_{i}, density_grid_{i}; attrs scale, cascades, grid_size, size
  * NGP(scale, rgb_act='Sigmoid', t=19)               networks.py:17-211 (single model)
  * Ray_Gate(out_dim, type='ray')                     networks.py:1070-1097
      forward(x (B,6), warmup=False) -> (gate (B,K), importance (K), None)

Parameters are fp32 masters: `xyz_encoder.params` (hash table, (entries*2,)),
`mlp_params` (size, 9472) and `Ray_Gate.params`.  The kernels read f16 copies
(hash table) and f16 MFMA fragments (MLPs) packed from the masters by HIP
kernels whenever the master changed (tracked with the tensor version counter).
tcnn's own flat-parameter ordering is not reproduced (unpinned dependency).
"""
import functools
import math

import numpy as np
import torch
from torch import nn

from . import layout as LY
from . import vren
from ._lib import lib

RGB_ACTS = ("Sigmoid",)


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _xavier_(mat, gen):
    fan_out, fan_in = mat.shape
    bound = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        mat.uniform_(-bound, bound, generator=gen)


class _DeviceTables:
    """Per-device cache of the int index tables (layout.py)."""
    _cache = {}

    @classmethod
    def get(cls, key, device, builder):
        k = (key, str(device))
        if k not in cls._cache:
            cls._cache[k] = torch.from_numpy(builder()).to(device)
        return cls._cache[k]


class HashGridEncoding(nn.Module):
    """tcnn Grid/Hash encoding parameters (networks.py:234-247): L=16, F=2,
    T=2^t, N_min=16, per_level_scale = exp(log(2048*scale/16)/15)."""

    def __init__(self, scale, log2_T=19, generator=None):
        super().__init__()
        self.levels = LY.grid_levels(scale, log2_T)
        self.n_entries = int(self.levels["n_entries"])
        self.n_levels, self.n_output_dims = LY.N_LEVELS, LY.N_LEVELS * LY.N_FEATURES
        p = torch.empty(self.n_entries * 2)
        p.uniform_(-1e-4, 1e-4, generator=generator)
        self.params = nn.Parameter(p)
        self._f16 = None
        self._f16_ver = None
        # host copies handed to the kernels
        self.h_offset = np.ascontiguousarray(self.levels["offset"], np.uint32)
        self.h_hsize = np.ascontiguousarray(self.levels["hsize"], np.uint32)
        self.h_res = np.ascontiguousarray(self.levels["res"], np.uint32)
        self.h_scale = np.ascontiguousarray(self.levels["scale"], np.float32)

    def level_ptrs(self):
        return (self.h_offset.ctypes.data, self.h_hsize.ctypes.data, self.h_res.ctypes.data,
                self.h_scale.ctypes.data)

    def params_f16(self):
        """f16 copy of the table (tcnn keeps the table in f16), refreshed when
        the fp32 master changes.  radnerf_amd.optim.FusedAdam refreshes it in
        its own pass and marks it current (p._rn_f16_key)."""
        p = self.params
        key = _param_key(p)
        if self._f16 is not None and getattr(p, "_rn_f16_key", None) == key:
            self._f16_ver = key
        if self._f16 is None or self._f16.device != p.device or self._f16_ver != key:
            if self._f16 is None or self._f16.device != p.device:
                self._f16 = torch.empty(p.numel(), dtype=torch.float16, device=p.device)
                p._rn_f16 = self._f16
            lib().to_f16(p.data_ptr(), p.numel(), self._f16.data_ptr(), _stream(p.device))
            self._f16_ver = key
        return self._f16


def _param_key(p):
    """Version key of a parameter's derived caches: torch's in-place version
    plus the epoch radnerf_amd.optim.FusedAdam bumps after its kernel update."""
    return (p._version, getattr(p, "_rn_epoch", 0))


class _FieldFn(torch.autograd.Function):
    """MNGP.forward(x, d, ind) on rn_field_fwd / rn_field_bwd."""

    @staticmethod
    def forward(ctx, xyzs, dirs, grid_params, mlp_params, model, ind, want_cache=True):
        xyzs = xyzs.float().contiguous()
        dirs = dirs.float().contiguous()
        n = xyzs.shape[0]
        dev = xyzs.device
        sigma = torch.empty(n, device=dev)
        rgb = torch.empty(n, 3, device=dev)
        # encoding cache for the backward (64 B/sample): only when a gradient
        # will be asked for.  needs_input_grad reflects the parameters'
        # requires_grad even under no_grad, and inside Function.forward grad
        # mode is always off, so the caller's grad mode comes in as want_cache
        # (no_grad renders and density-grid updates skip the cache)
        feat = None
        if n > 0 and want_cache and any(ctx.needs_input_grad[:4]):
            feat = torch.empty((n + 31) // 32 * 32, 32, device=dev, dtype=torch.float16)
        if n > 0:
            model._launch_field(True, xyzs, dirs, ind, sigma=sigma, rgb=rgb, feat=feat)
        ctx.save_for_backward(xyzs, dirs)
        ctx.feat = feat
        ctx.model, ctx.ind = model, ind
        return sigma, rgb

    @staticmethod
    def backward(ctx, dsigma, drgb):
        xyzs, dirs = ctx.saved_tensors
        model, ind = ctx.model, ctx.ind
        dev = xyzs.device
        n = xyzs.shape[0]
        need_x, need_d, need_g, need_w = ctx.needs_input_grad[:4]
        grid_grad = torch.zeros_like(model.xyz_encoder.params) if need_g else None
        dw = torch.zeros_like(model.mlp_params) if need_w else None
        dx = torch.zeros_like(xyzs) if need_x else None
        dd = torch.zeros_like(dirs) if need_d else None
        if n > 0:
            ds = torch.zeros(n, device=dev) if dsigma is None else dsigma.float().contiguous()
            dr = torch.zeros(n, 3, device=dev) if drgb is None else drgb.float().contiguous()
            if need_g or need_w:
                gg = grid_grad if grid_grad is not None else torch.zeros_like(model.xyz_encoder.params)
                ww = dw if dw is not None else torch.zeros_like(model.mlp_params)
                model._launch_field(False, xyzs, dirs, ind, dsigma=ds, drgb=dr, grid_grad=gg,
                                    dw=ww, feat=ctx.feat)
            if need_x or need_d:
                # tcnn's modules back-propagate into their inputs (with
                # --optimize_ext, train_ml.py:90-93): positions and directions
                xg = dx if dx is not None else torch.empty_like(xyzs)
                dg = dd if dd is not None else torch.empty_like(dirs)
                model._launch_dinput(xyzs, dirs, ind, ds, dr, xg, dg, feat=ctx.feat)
        ctx.feat = None
        return dx, dd, grid_grad, dw, None, None, None


class _DensityFn(torch.autograd.Function):
    """MNGP.density on rn_field_density.  Backward: the sigma path through the
    full field backward (rgb seeds zero) and, for x, rn_field_dinput.  The
    geo features are returned detached (non-differentiable): in the reference
    only forward() consumes them with a gradient, and forward() here runs the
    whole field in one kernel."""

    @staticmethod
    def forward(ctx, x, grid_params, mlp_params, model, ind, return_feat):
        x = x.float().contiguous()
        n = x.shape[0]
        sigma = torch.empty(n, device=x.device)
        feat = torch.empty(n, 16, device=x.device) if return_feat else None
        if n > 0:
            model._launch_density(x, ind, sigma, feat)
        ctx.save_for_backward(x)
        ctx.model, ctx.ind = model, ind
        if feat is None:
            feat = torch.empty(0, 16, device=x.device)
        ctx.mark_non_differentiable(feat)
        return sigma, feat

    @staticmethod
    def backward(ctx, dsigma, dfeat):
        (x,) = ctx.saved_tensors
        model, ind = ctx.model, ctx.ind
        n = x.shape[0]
        need_x, need_g, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gg = torch.zeros_like(model.xyz_encoder.params) if need_g else None
        ww = torch.zeros_like(model.mlp_params) if need_w else None
        dx = torch.zeros_like(x) if need_x else None
        if n > 0 and dsigma is not None:
            ds = dsigma.float().contiguous()
            d = torch.ones_like(x)                      # no rgb seed: directions unused
            dr = torch.zeros(n, 3, device=x.device)
            if need_g or need_w:
                model._launch_field(False, x, d, ind, dsigma=ds, drgb=dr,
                                    grid_grad=gg if gg is not None else torch.zeros_like(model.xyz_encoder.params),
                                    dw=ww if ww is not None else torch.zeros_like(model.mlp_params))
            if need_x:
                model._launch_dinput(x, d, ind, ds, dr, dx, torch.empty_like(x))
        return dx, gg, ww, None, None, None


class MNGP(nn.Module):
    """networks.py:214-421 on the HIP field kernels."""

    def __init__(self, scale, rgb_act="Sigmoid", size=2, t=19, seed=None):
        super().__init__()
        if rgb_act not in RGB_ACTS:
            raise ValueError(f"rgb_act {rgb_act} not supported (only {RGB_ACTS})")
        self.rgb_act = rgb_act
        self.scale = scale
        self.register_buffer("center", torch.zeros(1, 3))
        self.register_buffer("xyz_min", -torch.ones(1, 3) * scale)
        self.register_buffer("xyz_max", torch.ones(1, 3) * scale)
        self.register_buffer("half_size", (self.xyz_max - self.xyz_min) / 2)
        self.size = size
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.xyz_encoder = HashGridEncoding(scale, t, gen)
        self.cascades = LY.cascades_for_scale(scale)
        self.grid_size = 128
        g = torch.arange(self.grid_size, dtype=torch.int32)
        coords = torch.stack(torch.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
        # kornia create_meshgrid3d(..., False) order: (x fastest) -> coords[:, (2,1,0)]
        self.register_buffer("grid_coords", coords[:, [2, 1, 0]].contiguous())
        for i in range(size):
            self.register_buffer(f"density_bitfield_{i}",
                                 torch.zeros(self.cascades * self.grid_size ** 3 // 8,
                                             dtype=torch.uint8))
            self.register_buffer(f"density_grid_{i}",
                                 torch.zeros(self.cascades, self.grid_size ** 3))
        mlp = torch.empty(size, LY.FIELD_PARAMS)
        for i in range(size):
            for name, mat in LY.split_field_params(mlp[i]).items():
                _xavier_(mat, gen)
        self.mlp_params = nn.Parameter(mlp)
        self._frags = None
        self._frags_ver = None
        self._set_box_host()

    # ---------------------------------------------------------------- plumbing
    def _set_box_host(self):
        mn = self.xyz_min.detach().float().cpu().numpy().reshape(3)
        mx = self.xyz_max.detach().float().cpu().numpy().reshape(3)
        self._h_min = np.ascontiguousarray(mn, np.float32)
        self._h_ext = np.ascontiguousarray((mx - mn).astype(np.float32))

    def packed_frags(self):
        """f16 MFMA fragments of all sub-NeRFs, (size, 46*512) halfs."""
        p = self.mlp_params
        if self._frags is None or self._frags.device != p.device or self._frags_ver != _param_key(p):
            idx = _DeviceTables.get("field_frags", p.device, LY.field_frag_index)
            if self._frags is None or self._frags.device != p.device:
                self._frags = torch.empty(self.size, idx.numel(), dtype=torch.float16,
                                          device=p.device)
            lib().pack_f16(p.data_ptr(), LY.FIELD_PARAMS, idx.data_ptr(), idx.numel(), self.size,
                           idx.numel(), self._frags.data_ptr(), _stream(p.device))
            self._frags_ver = _param_key(p)
        return self._frags

    def packed_dinput_frags(self):
        """f16 fragments of every sub-NeRF's rgb-net SH columns, transposed
        (K, 4*512) halfs: the input-gradient kernel's dL/dSH."""
        p = self.mlp_params
        if (getattr(self, "_dfrags", None) is None or self._dfrags.device != p.device
                or self._dfrags_ver != _param_key(p)):
            idx = _DeviceTables.get("field_dinput_frags", p.device, LY.field_dinput_frag_index)
            if getattr(self, "_dfrags", None) is None or self._dfrags.device != p.device:
                self._dfrags = torch.empty(self.size, idx.numel(), dtype=torch.float16,
                                           device=p.device)
            lib().pack_f16(p.data_ptr(), LY.FIELD_PARAMS, idx.data_ptr(), idx.numel(), self.size,
                           idx.numel(), self._dfrags.data_ptr(), _stream(p.device))
            self._dfrags_ver = _param_key(p)
        return self._dfrags

    def _launch_dinput(self, xyzs, dirs, ind, dsigma, drgb, dxyz, ddir, feat=None):
        """dL/dxyzs, dL/ddirs of forward(xyzs, dirs, ind) (rn_field_dinput)."""
        frags = self.packed_frags()
        dfr = self.packed_dinput_frags()
        grid16 = self.xyz_encoder.params_f16()
        lo, lh, lr, ls = self.xyz_encoder.level_ptrs()
        n = xyzs.shape[0]
        nb = max(1, min(2048, (n + 127) // 128))
        lib().field_dinput(xyzs.data_ptr(), dirs.data_ptr(), n, None, None, None, None, None, None,
                           1, grid16.data_ptr(), lo, lh, lr, ls, self._h_min.ctypes.data,
                           self._h_ext.ctypes.data,
                           frags.data_ptr() + ind * frags.shape[1] * 2,
                           dfr.data_ptr() + ind * dfr.shape[1] * 2, dsigma.data_ptr(),
                           drgb.data_ptr(), None if feat is None else feat.data_ptr(),
                           dxyz.data_ptr(), ddir.data_ptr(), nb, _stream(xyzs.device))

    def _launch_field(self, fwd, xyzs, dirs, ind, sigma=None, rgb=None, dsigma=None, drgb=None,
                      grid_grad=None, dw=None, blocks=None, feat=None):
        dev = xyzs.device
        frags = self.packed_frags()
        grid16 = self.xyz_encoder.params_f16()
        fptr = frags.data_ptr() + ind * frags.shape[1] * 2
        lo, lh, lr, ls = self.xyz_encoder.level_ptrs()
        n = xyzs.shape[0]
        if fwd:
            nb = blocks or max(1, min(2048, (n + 127) // 128))
            lib().field_fwd(xyzs.data_ptr(), dirs.data_ptr(), n, None, None, None, None, None,
                            None, 1, grid16.data_ptr(), lo, lh, lr, ls, self._h_min.ctypes.data,
                            self._h_ext.ctypes.data, fptr, sigma.data_ptr(), rgb.data_ptr(),
                            None if feat is None else feat.data_ptr(), nb, _stream(dev))
        else:
            nb = blocks or max(1, min(256, (n + 255) // 256))
            lib().field_bwd(xyzs.data_ptr(), dirs.data_ptr(), n, None, None, None, None, None,
                            None, 1, grid16.data_ptr(), lo, lh, lr, ls, self._h_min.ctypes.data,
                            self._h_ext.ctypes.data, fptr, dsigma.data_ptr(), drgb.data_ptr(),
                            grid_grad.data_ptr(), dw.data_ptr() + ind * LY.FIELD_PARAMS * 4,
                            None if feat is None else feat.data_ptr(), nb, _stream(dev))

    # ------------------------------------------------------------ reference API
    def density(self, x, ind, return_feat=False):
        """networks.py:291-309: hash grid + geo MLP only (rn_field_density);
        returns sigmas (N), and with return_feat also h[:, 1:17] (N, 16), the
        geo features the rgb net takes (fp32 of tcnn's f16 values)."""
        sigma, feat = _DensityFn.apply(x, self.xyz_encoder.params, self.mlp_params, self, ind,
                                       bool(return_feat))
        return (sigma, feat) if return_feat else sigma

    def _launch_density(self, x, ind, sigma, feat):
        frags = self.packed_frags()
        lo, lh, lr, ls = self.xyz_encoder.level_ptrs()
        lib().field_density(x.data_ptr(), x.shape[0], self.xyz_encoder.params_f16().data_ptr(),
                            lo, lh, lr, ls, self._h_min.ctypes.data, self._h_ext.ctypes.data,
                            frags.data_ptr() + ind * frags.shape[1] * 2, sigma.data_ptr(),
                            None if feat is None else feat.data_ptr(), _stream(x.device))

    def forward(self, x, d, ind, **kwargs):
        """networks.py:311-328 -> sigmas (N), rgbs (N,3)"""
        return _FieldFn.apply(x, d, self.xyz_encoder.params, self.mlp_params, self, ind,
                              torch.is_grad_enabled())

    @torch.no_grad()
    def get_all_cells(self):
        """networks.py:330-343"""
        indices = vren.morton3D(self.grid_coords).long()
        return [(indices, self.grid_coords)] * self.cascades

    @torch.no_grad()
    def sample_uniform_and_occupied_cells(self, M, density_threshold, ind, generator=None):
        """networks.py:345-372 as an API: per cascade, (Morton indices, coords)
        of M uniform cells followed by M cells drawn with replacement among
        those denser than the threshold (none when no cell is).  The update
        itself no longer draws explicit cells (rn_density_update_sampled
        decides per cell whether it is hit, with the same hit rates)."""
        grid = getattr(self, f"density_grid_{ind}")
        draw = functools.partial(torch.randint, device=grid.device, generator=generator)
        out = []
        for c in range(self.cascades):
            coords = draw(self.grid_size, (M, 3), dtype=torch.int32)
            dense = torch.flatnonzero(grid[c] > density_threshold)
            if dense.numel():
                picked = dense[draw(dense.numel(), (M,))].int()
                coords = torch.cat([coords, vren.morton3D_invert(picked)])
            out.append((vren.morton3D(coords).long(), coords))
        return out

    @torch.no_grad()
    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=False,
                            generator=None, seed=None):
        """networks.py:375-409 on the device, every sub-NeRF and cascade in one
        rn_density_update_sampled call (warm-up: every cell; otherwise the
        cells hit by the uniform and the occupied draws, each evaluated once at
        a jittered point, as the reference's index_put keeps one draw per cell).
        The draws and jitters come from a counter-based hash of `seed`; without
        one, the seed is drawn from `generator` (a torch.Generator: ranks that
        seed it identically keep bit-identical grids and bitfields with no
        collective, radnerf_amd.dist) or from torch's default generator (as the
        reference's torch.randint / rand_like).  sigma comes from the density
        kernel (hash grid + geo MLP, networks.py:393-394).  `erode` (off in
        train_ml.py) is not supported."""
        if erode:
            raise NotImplementedError("update_density_grid(erode=True): not used by train_ml.py")
        if seed is None:
            dev = generator.device if generator is not None else torch.device("cpu")
            seed = int(torch.randint(1 << 62, (1,), generator=generator, device=dev))
        return self._update_sampled_device(density_threshold, decay, seed, all_cells=warmup)

    @torch.no_grad()
    def _update_sampled_device(self, density_threshold, decay, seed, all_cells=False):
        """The update of every sub-NeRF in one rn_density_update_sampled call;
        the density grids and bitfields are updated in place."""
        K, C, G = self.size, self.cascades, self.grid_size
        dev = self.mlp_params.device
        n = K * C * G ** 3
        du = getattr(self, "_du", None)
        if du is None or du["tmp"].numel() != n or du["tmp"].device != dev:
            du = {"tmp": torch.empty(n, device=dev),
                  "occ": torch.empty(n, device=dev, dtype=torch.int32),
                  # per-block occupied counts | per-block draw counts (scanned in place)
                  "blk": torch.empty(2 * (n // 1024 + 1), device=dev, dtype=torch.int32),
                  "part": torch.empty(K * 1024, device=dev),
                  "thr": torch.empty(K, device=dev)}
            self._du = du
        grids = [getattr(self, f"density_grid_{i}") for i in range(K)]
        bits = [getattr(self, f"density_bitfield_{i}") for i in range(K)]
        for i, g in enumerate(grids):
            if not (g.is_contiguous() and g.dtype == torch.float32 and g.numel() == C * G ** 3):
                g = g.float().contiguous()
                setattr(self, f"density_grid_{i}", g)
                grids[i] = g
        ptrs = torch.tensor([g.data_ptr() for g in grids] + [b.data_ptr() for b in bits],
                            dtype=torch.int64).to(dev, non_blocking=True)
        lo, lh, lr, ls = self.xyz_encoder.level_ptrs()
        lib().density_update_sampled(
            ptrs.data_ptr(), ptrs.data_ptr() + 8 * K, K, C, G, float(self.scale),
            float(density_threshold), float(decay), int(seed) & 0xFFFFFFFFFFFFFFFF,
            self.xyz_encoder.params_f16().data_ptr(), lo, lh, lr, ls, self._h_min.ctypes.data,
            self._h_ext.ctypes.data, self.packed_frags().data_ptr(), du["tmp"].data_ptr(),
            du["occ"].data_ptr(), du["blk"].data_ptr(), du["part"].data_ptr(),
            du["thr"].data_ptr(), int(bool(all_cells)), _stream(dev))
        self._du_ptrs = ptrs          # keep the pointer array alive until the launch ran
        return du

    @torch.no_grad()
    def register_bbox(self, bbox):
        """networks.py:413-422: scene box from a (2, 3) [min, max] array; resets
        the cascades and every sub-NeRF's density grid / bitfield."""
        bbox = np.asarray(bbox, dtype=np.float32)
        dev = self.xyz_min.device
        self.xyz_min = torch.from_numpy(bbox[0][None, :]).float().to(dev)
        self.xyz_max = torch.from_numpy(bbox[1][None, :]).float().to(dev)
        self.half_size = torch.from_numpy((bbox[1] - bbox[0]) / 2)[None, :].float().to(dev)
        self.center = torch.from_numpy(np.mean(bbox, axis=0))[None, :].float().to(dev)
        self.cascades = max(1 + int(np.ceil(np.log2(2 * float(self.half_size.max())))), 1)
        for i in range(self.size):
            setattr(self, f"density_bitfield_{i}",
                    torch.zeros(self.cascades * self.grid_size ** 3 // 8, dtype=torch.uint8,
                                device=dev))
            setattr(self, f"density_grid_{i}",
                    torch.zeros(self.cascades, self.grid_size ** 3, device=dev))
        self._set_box_host()

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._set_box_host()
        return out


class NGP(MNGP):
    """networks.py:17-211: single model; forward(x, d) and buffer
    `density_bitfield`.  (The reference's CUTLASSMLP and FullyFusedMLP share
    the no-bias ReLU f16 MLP semantics restated here.)"""

    def __init__(self, scale, rgb_act="Sigmoid", t=19, seed=None):
        super().__init__(scale, rgb_act, size=1, t=t, seed=seed)

    @property
    def density_bitfield(self):
        return self.density_bitfield_0

    @property
    def density_grid(self):
        return self.density_grid_0

    def density(self, x, return_feat=False, ind=0):
        return super().density(x, 0, return_feat)

    def forward(self, x, d, *args, **kwargs):
        return super().forward(x, d, 0)

    @torch.no_grad()
    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=False,
                            generator=None, seed=None):
        return super().update_density_grid(density_threshold, warmup, decay, erode, generator,
                                           seed)


class _GateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, params, gate_mod):
        x = x.float().contiguous()
        B = x.shape[0]
        K = gate_mod.out_dim
        dev = x.device
        gate = torch.empty(B, K, device=dev)
        imp = torch.zeros(K, device=dev)
        if B > 0:
            frags = gate_mod.packed_frags()
            nb = max(1, min(256, (B + 127) // 128))
            lib().gate_fwd(x.data_ptr(), x.data_ptr() + 12, 6, B, K, frags.data_ptr(),
                           gate.data_ptr(), imp.data_ptr(), nb, _stream(dev))
        ctx.save_for_backward(x)
        ctx.gate_mod = gate_mod
        ctx.mark_non_differentiable(imp)
        return gate, imp

    @staticmethod
    def backward(ctx, dgate, dimp):
        (x,) = ctx.saved_tensors
        g = ctx.gate_mod
        dw = torch.zeros_like(g.params)
        B = x.shape[0]
        # tcnn's Network back-propagates into its input when it requires grad
        # (rays_o / rays_d under --optimize_ext)
        dx = torch.zeros_like(x) if ctx.needs_input_grad[0] else None
        if B > 0 and dgate is not None:
            frags = g.packed_frags()
            dfr = g.packed_dinput_frags() if dx is not None else None
            nb = max(1, min(128, (B + 127) // 128))
            lib().gate_bwd(x.data_ptr(), x.data_ptr() + 12, 6, B, g.out_dim, frags.data_ptr(),
                           dgate.float().contiguous().data_ptr(), dw.data_ptr(), dw.numel(),
                           None if dfr is None else dfr.data_ptr(),
                           None if dx is None else dx.data_ptr(), nb, _stream(x.device))
        return dx, dw, None


class Ray_Gate(nn.Module):
    """networks.py:1070-1097: FullyFusedMLP 6 -> 64x4 -> K (ReLU, no bias) +
    softmax(dim=1); importance = gate.sum(0); top_k_indices = None.
    Gradients flow into the input x when it requires grad, as through tcnn."""

    def __init__(self, out_dim, type="ray", seed=None):
        super().__init__()
        if not 1 <= out_dim <= 16:
            raise ValueError("Ray_Gate supports 1..16 sub-NeRFs")
        self.out_dim = out_dim
        self.type = type
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        p = torch.empty(LY.gate_params(out_dim))
        for _, mat in LY.split_gate_params(p, out_dim).items():
            _xavier_(mat, gen)
        self.params = nn.Parameter(p)
        self._frags = None
        self._frags_ver = None

    def packed_frags(self):
        p = self.params
        if self._frags is None or self._frags.device != p.device or self._frags_ver != _param_key(p):
            idx = _DeviceTables.get(f"gate_frags_{self.out_dim}", p.device,
                                    lambda: LY.gate_frag_index(self.out_dim))
            if self._frags is None or self._frags.device != p.device:
                self._frags = torch.empty(idx.numel(), dtype=torch.float16, device=p.device)
            lib().pack_f16(p.data_ptr(), p.numel(), idx.data_ptr(), idx.numel(), 1, idx.numel(),
                           self._frags.data_ptr(), _stream(p.device))
            self._frags_ver = _param_key(p)
        return self._frags

    def packed_dinput_frags(self):
        """f16 A fragments of W0^T (the input gradient of rn_gate_bwd)."""
        p = self.params
        if (getattr(self, "_dfrags", None) is None or self._dfrags.device != p.device
                or self._dfrags_ver != _param_key(p)):
            idx = _DeviceTables.get(f"gate_dinput_frags_{self.out_dim}", p.device,
                                    lambda: LY.gate_dinput_frag_index(self.out_dim))
            if getattr(self, "_dfrags", None) is None or self._dfrags.device != p.device:
                self._dfrags = torch.empty(idx.numel(), dtype=torch.float16, device=p.device)
            lib().pack_f16(p.data_ptr(), p.numel(), idx.data_ptr(), idx.numel(), 1, idx.numel(),
                           self._dfrags.data_ptr(), _stream(p.device))
            self._dfrags_ver = _param_key(p)
        return self._dfrags

    def forward(self, x, warmup=False):
        gate, _ = _GateFn.apply(x, self.params, self)
        # importance feeds only the CV^2 loss (losses.py:67-69); keep it on the
        # autograd graph like the reference's gate.sum(0)
        return gate, gate.sum(0), None

    def freeze_dict(self):
        for _, p in self.named_parameters():
            p.requires_grad_(False)
