"""GPU worker of tests/test_gpu_dist.py (not a test module): one rank of the
ray-batch data-parallel step (radnerf_amd/dist.py, bench.py --gpus N)
rehearsed on ONE GPU over gloo.  Rank r renders its own rays; the flat
gradient is averaged over the ranks.  Rank 0 also renders every rank's rays
in one process, averages those gradients and writes the comparison to the
JSON path in argv[1]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radnerf_amd import dist as rdist  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def inputs(rank, B, K, scale, dev):
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=1000 * rank))
    nz = torch.from_numpy(S.noise(K, B, seed=2 + 7919 * rank)).to(dev)
    sd = [torch.from_numpy(s).to(dev) for s in S.loss_seeds(B, K, seed=4 + rank)]
    return o, d, nz, sd


def step(r, o, d, nz, sd, bg, views):
    _, _, _, g_out, _ = r.forward(o, d, d, nz, bg, 1e-4, 0.0)
    r.backward(o, d, d, g_out, bg, *sd, None, 1e-4, grid_grad=views[0], mlp_grad=views[1],
               gate_grad=views[2])


def hooked_split_schedule(rank, dev, stream_ordered=True, force=False):
    """bench.py's N > 1 schedule through the renderer's own hooks, at scale 16
    (binned fold split into fine / coarse sum launches):
    the MLP + gate bucket after field_bwd, levels [8, 16) after their sum
    pass, levels [0, 8) after the backward -- comm-stream launches, forced over
    gloo.  Each range's local values are copied (main stream) just before its
    collective starts; the result must equal one plain all-reduce of those
    local values, bit for bit.  Steps 1-2 set the fixed-point scales; step 3
    is checked (binned, no redo).  (tests/rccl_worker.py runs the same over a
    one-rank RCCL group: stream_ordered=None picks the backend's form, force
    issues the collectives with one rank.)"""
    B, K, scale = 512, 2, 16.0
    model = MNGP(scale, size=K, seed=5).to(dev)
    gate = Ray_Gate(K, seed=6).to(dev)
    bits = S.bitfields(K, model.cascades, p=0.5, seed=7)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    bg = torch.zeros(3, device=dev)
    r = FusedMLRenderer(model, gate, B)
    r.grid_fx = r.grid_bin = True            # (512 x 2 rays: fp32 by the renderer's choice)
    ar = rdist.GradAllReduce([model.xyz_encoder.params, model.mlp_params, gate.params], dev)
    off = model.xyz_encoder.h_offset
    rg = rdist.step_ranges(ar, off, r.grid_split_level)
    pending, cut, splits, local = [], [None], [], {}

    def launch(a, b, n):
        local[(a, b)] = ar.flat[a:b].clone()          # main stream: the local values
        pending.append(ar.launch_range(a, b, n, stream_ordered=stream_ordered, force=force))

    def mlp_bucket():
        # (the gate backward ran on the renderer's side stream, as in bench.py)
        torch.cuda.current_stream(dev).wait_stream(r._side(dev))
        launch(*rg["rest"], 1)

    def lv(split):
        a, b = rdist.step_ranges(ar, off, split)["fine"]
        launch(a, b, 4)
        cut[0] = a
        splits.append(split)

    r.after_field_bwd = mlp_bucket
    r.after_grid_levels = lv
    o, d, nz, sd = inputs(rank, B, K, scale, dev)
    for _ in range(3):
        ar.zero()
        pending.clear()
        local.clear()
        cut[0] = None
        _, _, _, g_out, _ = r.forward(o, d, d, nz, bg, 1e-4, 1 / 256)
        r.backward(o, d, d, g_out, bg, *sd, None, 1e-4, grid_grad=ar.views[0],
                   mlp_grad=ar.views[1], gate_grad=ar.views[2])
        g0 = ar.param_range(0, 1)[0]
        if cut[0] is not None and cut[0] > g0:
            launch(g0, cut[0], 1)
        for h in pending:
            ar.finish(h)
    torch.cuda.synchronize()
    ref = torch.zeros_like(ar.flat)
    covered = torch.zeros(ar.flat.numel(), dtype=torch.int32, device=dev)
    for (a, b), v in local.items():
        ref[a:b] = v
        covered[a:b] += 1
    dist.all_reduce(ref)
    ref.div_(dist.get_world_size())
    r.after_field_bwd = r.after_grid_levels = None
    return {"equal": bool(torch.equal(ar.flat, ref)), "splits": splits,
            "cuda": [bool(h["cuda"]) for h in ar.timed[-len(local):]] if ar.timed else [],
            "covered_once": bool((covered == 1).all()), "n_ranges": len(local),
            "redo": int(r.ws._fx[3][0]), "pages": int(r.ws._bin["ctl"][0]),
            "finite": bool(torch.isfinite(ar.flat).all()), "nonzero": bool(ar.flat.abs().max() > 0)}


def main(out_path):
    rank, _, world = rdist.init(backend="gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    B, K, scale = 1024, 2, 0.5
    model = MNGP(scale, size=K, seed=3).to(dev)
    gate = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, model.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    bg = torch.ones(3, device=dev)
    params = [model.xyz_encoder.params, model.mlp_params, gate.params]
    r = FusedMLRenderer(model, gate, B)
    ar = rdist.GradAllReduce(params, dev)
    ar.zero()
    o, d, nz, sd = inputs(rank, B, K, scale, dev)
    step(r, o, d, nz, sd, bg, ar.views)
    ar.reduce()
    torch.cuda.synchronize()
    result = ar.flat.clone()
    # the staged form bench.py uses over RCCL (comm stream, events, the MLP +
    # gate bucket then the grid in 4 buckets), forced here over gloo, on one
    # more step's local gradient: the same averaged buffer as reduce() of the
    # same gradient, and its timing fields
    ar.zero()
    ar.reset_timing()
    step(r, o, d, nz, sd, bg, ar.views)
    torch.cuda.synchronize()
    local = ar.flat.clone()
    hs = [ar.launch_range(*ar.param_range(1), 1, stream_ordered=True),
          ar.launch_range(*ar.param_range(0, 1), 4, stream_ordered=True)]
    for h in hs:
        ar.finish(h)
    torch.cuda.synchronize()
    staged = ar.flat.clone()
    stats = ar.comm_stats(1)
    ar.flat.copy_(local)
    ar.reduce()
    torch.cuda.synchronize()
    staged_equal = bool(torch.equal(staged, ar.flat))
    ar.flat.copy_(result)
    hooked = hooked_split_schedule(rank, dev)
    if rank == 0:
        ref = rdist.GradAllReduce(params, dev)      # not reduced: a local buffer
        ref.zero()
        for q in range(world):
            step(r, *inputs(q, B, K, scale, dev), bg, ref.views)
        ref.flat.div_(world)
        torch.cuda.synchronize()
        res = {"world": world, "grid_rel": rel(ar.views[0], ref.views[0]),
               "mlp_rel": rel(ar.views[1], ref.views[1]),
               "gate_rel": rel(ar.views[2], ref.views[2]),
               "staged_equal": staged_equal, "staged_stats": stats,
               "staged_cuda": all(h["cuda"] for h in hs), "n_flat": ar.flat.numel(),
               "hooked": hooked}
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
