"""Autograd surface of the reference (models/custom_functions.py:8-173) on the
HIP library: RayAABBIntersector, RayMarcher, VolumeRenderer, TruncExp.

Identical class names, `apply` signatures, fp32 autocast casting and return
tuples.  One addition: RayMarcher.apply takes an optional trailing `noise`
tensor (test-only override of the torch.rand_like jitter drawn at
custom_functions.py:83) so parity tests can feed identical jitter.
"""
import torch
from torch.amp import custom_bwd, custom_fwd

from . import vren


class RayAABBIntersector(torch.autograd.Function):
    """custom_functions.py:8-29"""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, center, half_size, max_hits):
        return vren.ray_aabb_intersect(rays_o, rays_d, center, half_size, max_hits)


class RayMarcher(torch.autograd.Function):
    """custom_functions.py:55-112"""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, hits_t, density_bitfield, cascades, scale,
                exp_step_factor, grid_size, max_samples, noise=None):
        if noise is None:
            noise = torch.rand_like(rays_o[:, 0])
        rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
            rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor,
            noise.contiguous(), grid_size, max_samples)
        total_samples = counter[0]
        ctx.save_for_backward(rays_a, ts)
        return rays_a, xyzs, dirs, deltas, ts, total_samples

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_drays_a, dL_dxyzs, dL_ddirs, dL_ddeltas, dL_dts, dL_dtotal_samples):
        # segment_csr over rays_a's [start, start+count) segments (torch_scatter
        # in the reference, custom_functions.py:107-110); only live with
        # --optimize_ext.  rays_a here is in ray order, so segments are sorted.
        rays_a, ts = ctx.saved_tensors
        z = lambda g: torch.zeros(ts.shape[0], 3, device=ts.device) if g is None \
            else g.float().contiguous()
        dL_drays_o, dL_drays_d = vren.raymarching_train_bw(z(dL_dxyzs), z(dL_ddirs), ts, rays_a)
        return dL_drays_o, dL_drays_d, None, None, None, None, None, None, None, None


class VolumeRenderer(torch.autograd.Function):
    """custom_functions.py:115-159"""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, sigmas, rgbs, deltas, ts, rays_a, T_threshold):
        total_samples, opacity, depth, rgb, ws = vren.composite_train_fw(
            sigmas.contiguous(), rgbs.contiguous(), deltas, ts, rays_a, T_threshold)
        ctx.save_for_backward(sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws)
        ctx.T_threshold = T_threshold
        return total_samples.sum(), opacity, depth, rgb, ws

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_dtotal_samples, dL_dopacity, dL_ddepth, dL_drgb, dL_dws):
        sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws = ctx.saved_tensors
        dL_dsigmas, dL_drgbs = vren.composite_train_bw(
            dL_dopacity.contiguous(), dL_ddepth.contiguous(), dL_drgb.contiguous(),
            dL_dws.contiguous(), sigmas.contiguous(), rgbs.contiguous(), ws, deltas, ts, rays_a,
            opacity, depth, rgb, ctx.T_threshold)
        return dL_dsigmas, dL_drgbs, None, None, None, None


class TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173 (used standalone; the fused field applies it
    inside the HIP kernels)."""

    @staticmethod
    @custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    @custom_bwd(device_type="cuda")
    def backward(ctx, dL_dout):
        x = ctx.saved_tensors[0]
        return dL_dout * torch.exp(x.clamp(-15, 15))
