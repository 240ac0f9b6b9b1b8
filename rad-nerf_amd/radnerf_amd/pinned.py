"""Sub-NeRF-per-GPU training render (variant C5: model_zoo_size=8
on 8 GPUs, "sub-NeRFs pinned one-per-GPU with gate-weighted RCCL reduce").

The reference is single-GPU: `ml_rendering.ml_render` loops over the K
sub-NeRFs (models/ml_rendering.py:30-78) and gates their per-ray outputs
(:158-202).  Here rank r of P owns the sub-NeRFs [r K/P, (r+1) K/P): their
MLPs and occupancy bitfields.  Every rank holds the shared hash grid and the
gate, and every rank sees all B rays.

  forward : gate_fwd (all K, identical on every rank)
            | march -> field_fwd -> composite_fw of the OWN sub-NeRFs, all B rays
            -> all-gather of the per-ray (opacity, depth, rgb) = 20 B x B x K/P
               per rank (RCCL; the only exchange of the forward)
            -> gated combine of all K (identical on every rank)
  backward: combine_bw (all K) -> composite_bw + field_bwd of the own sub-NeRFs
            -> gate_bwd on rank 0 only
            -> one summed all-reduce of the flat gradient (dist.GradAllReduce,
               average=False): the shared grid's partial gradients add up,
               each MLP gradient is non-zero on its owner only, the gate's on
               rank 0 only.

The loss sees identical (rgb, opacity, depth, gate) on every rank, so its seeds
are identical too; nothing else is exchanged.  The grid all-reduce stays (the
grid is shared), as SURVEY.md §8(e) notes.
"""
import torch
import torch.distributed as dist

from .fused import FusedMLRenderer


class ModelSlice:
    """Sub-NeRFs [k0, k1) of an MNGP as the renderer sees them: the shared
    hash grid, their own MLPs (contiguous rows of `mlp_params` and of the
    packed fragments) and their own bitfields."""

    def __init__(self, model, k0, k1):
        if not 0 <= k0 < k1 <= model.size:
            raise ValueError(f"bad sub-NeRF range [{k0}, {k1}) of {model.size}")
        self.full, self.k0, self.k1, self.size = model, k0, k1, k1 - k0

    def __getattr__(self, name):
        if name.startswith("density_bitfield_") or name.startswith("density_grid_"):
            base, i = name.rsplit("_", 1)
            return getattr(self.full, f"{base}_{self.k0 + int(i)}")
        return getattr(self.full, name)

    @property
    def mlp_params(self):
        return self.full.mlp_params[self.k0:self.k1]

    def packed_frags(self):
        return self.full.packed_frags()[self.k0:self.k1]


def owned_range(n_models, rank, world):
    """Sub-NeRFs [k0, k1) of `rank`: contiguous blocks of K/P."""
    if n_models % world:
        raise ValueError(f"model_zoo_size {n_models} must be a multiple of the {world} ranks")
    per = n_models // world
    return rank * per, (rank + 1) * per


class PinnedMLRenderer(FusedMLRenderer):
    """FusedMLRenderer over this rank's sub-NeRFs; forward/backward/train_step
    take and return the same full-K tensors (noise (K, B), gate (B, K), depth
    (B, K)).  Gradients: pass the views of a dist.GradAllReduce over
    [grid, mlp_params, gate] and call reduce(average=False) after backward."""

    def __init__(self, model, gating_net, n_rays, group=None, device=None, sim=None, **kw):
        """sim=(rank, world): run rank `rank`'s share of a `world`-rank layout
        in this one process (bench.py --pinned-sim: its sub-NeRFs over all B
        rays, the gate backward if rank 0), the all-gather replaced by local
        copies of this rank's rows (the other ranks' rows are stand-ins)."""
        self.group = group
        self.simulated = sim is not None
        if self.simulated:
            rank, world = sim
        elif dist.is_initialized():
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        else:
            rank, world = 0, 1
        self.rank, self.world = rank, world
        self.k0, self.k1 = owned_range(model.size, rank, world)
        super().__init__(ModelSlice(model, self.k0, self.k1), gating_net, n_rays, device=device,
                         **kw)
        self.full_model = model
        self.gate_grad_here = rank == 0
        B, K = n_rays, model.size
        f = dict(device=self.device, dtype=torch.float32)
        kl = self.k1 - self.k0
        # packed per-ray outputs: one row per sub-NeRF, [opacity B | depth B | rgb 3B]
        self._pack = torch.empty(kl, 5 * B, **f)
        self._gathered = torch.empty(K, 5 * B, **f)
        self.opacity_all = torch.empty(K, B, **f)
        self.depth_all = torch.empty(K, B, **f)
        self.rgb_all = torch.empty(K, B, 3, **f)
        self._dgate_all = torch.empty(B, K, **f)

    def forward(self, rays_o, rays_d, gate_in2, noise, bg, T_threshold=1e-4, exp_step_factor=0.0):
        return super().forward(rays_o, rays_d, gate_in2, noise[self.k0:self.k1], bg, T_threshold,
                               exp_step_factor)

    def _model_outputs(self):
        if self.world == 1:
            return super()._model_outputs()
        return self.opacity_all, self.depth_all, self.rgb_all

    def _gather_model_outputs(self):
        w, B = self.ws, self.ws.B
        if self.world == 1:
            return w.opacity_k, w.depth_k, w.rgb_k
        pk = self._pack
        pk[:, :B].copy_(w.opacity_k)
        pk[:, B:2 * B].copy_(w.depth_k)
        pk[:, 2 * B:].copy_(w.rgb_k.view(-1, 3 * B))
        if self.simulated:
            # one process stands in for all ranks: every rank's rows = ours
            self._gathered.view(self.world, *pk.shape).copy_(
                pk.unsqueeze(0).expand(self.world, *pk.shape))
        else:
            all_gather_rows(self._gathered, pk, self.group)
        g = self._gathered
        self.opacity_all.copy_(g[:, :B])
        self.depth_all.copy_(g[:, B:2 * B])
        self.rgb_all.view(-1, 3 * B).copy_(g[:, 2 * B:])
        return self.opacity_all, self.depth_all, self.rgb_all

    def _local_cols(self, x):
        if self.world == 1:
            return x
        return x[:, self.k0:self.k1].contiguous()

    def _dgate(self, B, G):
        return self.ws.dgate if self.world == 1 else self._dgate_all

    def backward(self, rays_o, rays_d, gate_in2, gate, bg, dL_drgb, dL_dopacity, dL_ddepth,
                 dL_dgate_ext=None, T_threshold=1e-4, grid_grad=None, mlp_grad=None,
                 gate_grad=None):
        """mlp_grad: the full (K, FIELD_PARAMS) buffer; this rank adds its rows."""
        if self.input_grad:
            # each rank would hold the ray gradients of its own sub-NeRFs only
            raise NotImplementedError(
                "PinnedMLRenderer: gradients into rays_o / rays_d (--optimize_ext) are not "
                "supported in the sub-NeRF-per-GPU layout; use the data-parallel renderer")
        m = self.full_model
        grid_grad = torch.zeros_like(m.xyz_encoder.params) if grid_grad is None else grid_grad
        mlp_grad = torch.zeros_like(m.mlp_params) if mlp_grad is None else mlp_grad
        gate_grad = torch.zeros_like(self.gate.params) if gate_grad is None else gate_grad
        super().backward(rays_o, rays_d, gate_in2, gate, bg, dL_drgb, dL_dopacity, dL_ddepth,
                         dL_dgate_ext, T_threshold, grid_grad, mlp_grad[self.k0:self.k1],
                         gate_grad)
        return grid_grad, mlp_grad, gate_grad


def all_gather_rows(out, rows, group=None):
    """out[r * n:(r + 1) * n] = rows of rank r (n = rows.shape[0]).  RCCL:
    one all_gather_into_tensor; gloo (the CPU tests, or rehearsing several
    ranks on one GPU): the list form."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, rows, group=group)
    else:
        n = rows.shape[0]
        dist.all_gather([out[i * n:(i + 1) * n] for i in range(out.shape[0] // n)], rows,
                        group=group)
    return out
