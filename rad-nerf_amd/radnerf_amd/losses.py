"""NeRFLoss of the reference (losses.py:39-76) in two forms.

`NeRFLoss`         the reference module: a dict of loss tensors built from torch
                   ops (autograd), for callers that keep the reference training
                   loop (`loss = sum(l.mean() for l in loss_d.values())`).
`fused_nerf_loss`  one HIP pass (rn_nerf_loss) that returns the per-term means
                   AND the seeds dL/drgb, dL/dopacity, dL/ddepth, dL/dgate of
                   `sum(term.mean())`; FusedMLRenderer.train_step feeds them
                   straight into the fused backward (no autograd graph).

`DistortionLoss`    the reference autograd Function (losses.py:6-36) on the HIP
                   distortion kernels (vren.distortion_loss_fw / _bw).
"""
import torch
from torch import nn

from . import vren
from ._lib import lib


class DistortionLoss(torch.autograd.Function):
    """losses.py:6-36: Mip-NeRF 360 distortion loss (DVGO-v2 form) per ray.
    Inputs ws, deltas, ts (N) and rays_a (N_rays, 3); output loss (N_rays)."""

    @staticmethod
    def forward(ctx, ws, deltas, ts, rays_a):
        loss, ws_incl, wts_incl = vren.distortion_loss_fw(
            ws.float().contiguous(), deltas.float().contiguous(), ts.float().contiguous(),
            rays_a.contiguous())
        ctx.save_for_backward(ws_incl, wts_incl, ws, deltas, ts, rays_a)
        return loss

    @staticmethod
    def backward(ctx, dL_dloss):
        ws_incl, wts_incl, ws, deltas, ts, rays_a = ctx.saved_tensors
        dL_dws = vren.distortion_loss_bw(dL_dloss.float().contiguous(), ws_incl, wts_incl,
                                         ws.float().contiguous(), deltas.float().contiguous(),
                                         ts.float().contiguous(), rays_a.contiguous())
        return dL_dws, None, None, None


class NeRFLoss(nn.Module):
    """losses.py:39-76."""

    def __init__(self, lambda_opacity=1e-3):
        super().__init__()

    def forward(self, results, target, lambda_opacity=1e-3, lambda_distortion=0, lambda_disp=0,
                lambda_cv_importance=0, lambda_depth_mutual=0):
        loss = {}
        loss["rgb"] = (results["rgb"] - target["rgb"]) ** 2
        o = results["opacity"] + 1e-10
        loss["opacity"] = lambda_opacity * (-o * torch.log(o))
        if lambda_disp > 0:
            loss["disp"] = lambda_disp * results["disp"] ** 2
        K = results["gating_code"].shape[-1]
        if lambda_distortion > 0:
            # per sub-NeRF keys ws_i / deltas_i / ts_i / rays_a_i (losses.py:63-67)
            loss["distortion"] = 0
            for i in range(K):
                loss["distortion"] += lambda_distortion * DistortionLoss.apply(
                    results[f"ws_{i}"], results[f"deltas_{i}"], results[f"ts_{i}"],
                    results[f"rays_a_{i}"]).mean()
        if lambda_cv_importance > 0 and K > 1:
            imp = results["gating_importance"].float()
            loss["cv_importance"] = lambda_cv_importance * imp.var() / (imp.mean() ** 2 + 1e-10)
        if lambda_depth_mutual > 0 and K > 1:
            d = results["depth"]
            loss["depth_mutual"] = lambda_depth_mutual * (
                (d - torch.sum(d * results["gating_code"], 1, keepdim=True).detach()) ** 2)
        return loss


def fused_nerf_loss(rgb, target_rgb, opacity, depth, gate, importance, lambda_opacity=1e-3,
                    lambda_cv_importance=0.0, lambda_depth_mutual=0.0):
    """Returns ({term: mean (0-d tensor)}, (dL_drgb, dL_dopacity, dL_ddepth, dL_dgate))
    for loss = sum of the term means.  All inputs fp32 CUDA, contiguous."""
    B, K = gate.shape
    dev = rgb.device
    f = lambda *s: torch.empty(*s, device=dev, dtype=torch.float32)
    out = f(4)
    d_rgb, d_op, d_depth, d_gate = f(B, 3), f(B), f(B, K), f(B, K)
    c = lambda t: t.float().contiguous()
    rgb, target_rgb, opacity, depth, gate, importance = map(
        c, (rgb, target_rgb, opacity, depth, gate, importance))
    lib().nerf_loss(rgb.data_ptr(), target_rgb.data_ptr(), opacity.data_ptr(), depth.data_ptr(),
                    gate.data_ptr(), importance.data_ptr(), B, K, float(lambda_opacity),
                    float(lambda_cv_importance), float(lambda_depth_mutual), out.data_ptr(),
                    d_rgb.data_ptr(), d_op.data_ptr(), d_depth.data_ptr(), d_gate.data_ptr(),
                    torch.cuda.current_stream(dev).cuda_stream)
    terms = {"rgb": out[0] / (3 * B), "opacity": out[1] / B}
    if lambda_cv_importance > 0 and K > 1:
        terms["cv_importance"] = out[2]
    if lambda_depth_mutual > 0 and K > 1:
        terms["depth_mutual"] = out[3] / (B * K)
    return terms, (d_rgb, d_op, d_depth, d_gate)
