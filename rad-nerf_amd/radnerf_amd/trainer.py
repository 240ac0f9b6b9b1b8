"""The training step of train_ml.py (training_step :172-193 + the optimizer of
:138-153) on the fused renderer, data-parallel over torch.distributed: one
process per GPU, each rank renders its own ray batch (dist.shard_rays) with
full replicas; one flat-gradient all-reduce (RCCL over xGMI) per step, then
the fused Adam; the occupancy grids are updated every `update_interval`
steps with a rank-consistent random stream (dist.update_density_grid), so
parameters, density grids and bitfields stay bit-identical across ranks.

    tr = Trainer(model, gate, n_rays=8192, lr=1e-2, lambda_cv_importance=1e-2)
    for step in range(n):
        terms = tr.step(rays_o, rays_d, imgs_d, target_rgb)

Out of scope: datasets, the Lightning loop, the cosine lr
schedule (set `tr.opt.param_groups[0]["lr"]` per epoch), logging.
"""
import torch

from . import dist as rdist
from .fused import FusedMLRenderer
from .optim import FusedAdam

MAX_SAMPLES = 1024


class Trainer:
    def __init__(self, model, gating_net, n_rays, lr=1e-2, lambda_opacity=1e-3,
                 lambda_cv_importance=0.0, lambda_depth_mutual=0.0, exp_step_factor=None,
                 random_bg=False, update_interval=16, warmup_steps=256, seed=0,
                 bucketed=True):
        self.model, self.gate = model, gating_net
        self.device = model.mlp_params.device
        self.renderer = FusedMLRenderer(model, gating_net, n_rays)
        # train_ml.py:101-102: exp step 1/256 beyond scale 0.5
        self.esf = (1 / 256 if model.scale > 0.5 else 0.0) if exp_step_factor is None \
            else float(exp_step_factor)
        self.random_bg = random_bg
        self.lambdas = dict(lambda_opacity=lambda_opacity,
                            lambda_cv_importance=lambda_cv_importance,
                            lambda_depth_mutual=lambda_depth_mutual)
        params = [model.xyz_encoder.params, model.mlp_params, gating_net.params]
        # gradients live in one flat buffer: one collective per step
        self.grads = rdist.GradAllReduce(params, self.device)
        for p, v in zip(params, self.grads.views):
            p.grad = v
        self.opt = FusedAdam(params, lr=lr, eps=1e-15)      # train_ml.py:143
        self.update_interval, self.warmup_steps, self.seed = update_interval, warmup_steps, seed
        # Adam as the epilogue of a bucketed all-reduce (dist.GradAllReduce.
        # reduce_and_step); False: one collective, a division, then Adam
        self.bucketed = bucketed
        self.global_step = 0

    def _bg(self):
        """ml_rendering.py:192-198"""
        if self.esf == 0:
            return torch.ones(3, device=self.device)
        if self.random_bg:
            return torch.rand(3, device=self.device)
        return torch.zeros(3, device=self.device)

    def step(self, rays_o, rays_d, imgs_d, target_rgb, noise=None):
        """One training step on this rank's rays; returns {term: mean} (this rank)."""
        if self.global_step % self.update_interval == 0:
            rdist.update_density_grid(self.model, 0.01 * MAX_SAMPLES / 3 ** 0.5,
                                      self.global_step,
                                      warmup=self.global_step < self.warmup_steps,
                                      seed=self.seed)
        B, K = rays_o.shape[0], self.model.size
        if noise is None:
            noise = torch.rand(K, B, device=self.device)
        second = imgs_d if self.gate.type == "image" else rays_d
        self.grads.zero()
        v = self.grads.views
        terms, _ = self.renderer.train_step(rays_o, rays_d, second, target_rgb, noise, self._bg(),
                                            exp_step_factor=self.esf, grid_grad=v[0],
                                            mlp_grad=v[1], gate_grad=v[2], **self.lambdas)
        if self.bucketed:
            self.grads.reduce_and_step(self.opt)
        else:
            self.grads.reduce()
            self.opt.step()
        self.global_step += 1
        return terms
