"""GPU worker of tests/test_gpu_dist.py::test_data_parallel_training_stays_identical
(not a test module): one rank of radnerf_amd.trainer.Trainer rehearsed with 2
ranks on ONE GPU over gloo.  Each rank trains on its own rays for N steps
(density-grid updates every 4 steps, warm-up updates over every cell first,
Adam; argv[2] the scale, 16: the binned grid scatter); at the end the ranks
compare SHA-256 digests of their parameters, density grids and bitfields and
rank 0 writes the result to argv[1]."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radnerf_amd import dist as rdist  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402
from radnerf_amd.trainer import Trainer  # noqa: E402


def digest(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def main(out_path, scale=0.5):
    rank, _, world = rdist.init(backend="gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    B, K, n_steps = 1024, 2, 14
    model = MNGP(scale, size=K, seed=3)
    gate = Ray_Gate(K, seed=4)
    with torch.no_grad():
        model.xyz_encoder.params.copy_(torch.from_numpy(S.grid_params(model.xyz_encoder.n_entries, seed=5)).view(-1))
        model.mlp_params.copy_(torch.from_numpy(S.mlp_params(K, LY.FIELD_PARAMS, seed=6)))
    model, gate = model.to(dev), gate.to(dev)
    tr = Trainer(model, gate, B, lr=1e-2, lambda_cv_importance=1e-2, lambda_depth_mutual=1e-2,
                 update_interval=4, warmup_steps=6, seed=7)
    bits0 = [getattr(model, f"density_bitfield_{i}").clone() for i in range(K)]
    losses = []
    g = torch.Generator().manual_seed(100 + rank)
    for step in range(n_steps):
        o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=1000 * rank + step))
        tgt = torch.rand(B, 3, generator=g).to(dev)
        nz = torch.rand(K, B, generator=g).to(dev)
        terms = tr.step(o, d, d, tgt, noise=nz)
        losses.append(float(sum(v for v in terms.values())))
    torch.cuda.synchronize()
    state = {"grid": model.xyz_encoder.params, "mlp": model.mlp_params, "gate": gate.params}
    for i in range(K):
        state[f"bitfield_{i}"] = getattr(model, f"density_bitfield_{i}")
        state[f"density_grid_{i}"] = getattr(model, f"density_grid_{i}")
    mine = {k: digest(v) for k, v in state.items()}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        changed = [bool((getattr(model, f"density_bitfield_{i}") != bits0[i]).any()) for i in range(K)]
        occ = [float(getattr(model, f"density_bitfield_{i}").float().mean()) for i in range(K)]
        res = {"world": world, "identical": {k: all(a[k] == mine[k] for a in allr) for k in mine},
               "bitfields_changed": changed, "occupancy_byte_mean": occ, "losses": losses,
               "finite": bool(all(torch.isfinite(v.float()).all() for v in state.values())),
               "grid_bin": bool(tr.renderer.grid_bin and tr.renderer.grid_fx),
               "bin_pages": (int(tr.renderer.ws._bin["ctl"][0])
                             if getattr(tr.renderer.ws, "_bin", None) else 0)}
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
