#!/usr/bin/env python
"""Headline benchmark: million samples/s fwd+bwd of the Rad-NeRF hot path.

Workload (BASELINE.json configs[2], "C3"): Rad-NeRF train_ml.py with
model_zoo_size K=2, gate_type=ray, B=8192 rays per GPU, scale 0.5 (1 cascade,
exp_step_factor 0), on synthetic rays through a random-init 128^3 occupancy
grid (Bernoulli p=0.5 per cell, one grid per sub-NeRF) and random-init
parameters (tcnn-style: hash table U(-1e-4,1e-4), Xavier MLPs).
A step = gate fwd + K x (AABB + march + field fwd + composite fw) + gated
combine, then the full backward (combine bw, composite bw, field bw with hash
grid + MLP weight gradients, gate bw) seeded with N(0,1e-3) loss gradients;
at N>1 plus one RCCL all-reduce of all gradients (weak scaling: every rank
renders its own 8192 rays).  Optimizer / density-grid update excluded, as in
the metric definition.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` without a torchrun environment starts the N ranks itself (a
`torch.distributed.run` child process, before this process touches the GPU)
and exits with its status; under torchrun every rank checks that the world
size equals --gpus and the JSON line reports the ranks it saw.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "rad-nerf_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "million samples/s fwd+bwd, 8192 rays, model_zoo_size=2; rgb L∞ vs ref"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
# algorithmic bytes per sample of the field backward kernel:
#   dL/dsigma + dL/drgb read 16 + sample position/direction re-read 24 +
#   hash-grid gradient scatter 1024 (16 levels x 8 corners x 2 fp32) = 1064 B
FIELD_BWD_BYTES_PER_SAMPLE = 16 + 24 + 1024
# field forward: read 24 + hash gather 512 + sigma/rgb write 16
FIELD_FWD_BYTES_PER_SAMPLE = 24 + 512 + 16
# whole path fwd+bwd: 612 + 1112
PATH_BYTES_PER_SAMPLE = 1724
MLP_FLOP_PER_SAMPLE = 56832          # fwd + bwd, SURVEY.md §8(d)
MFMA_F16_PEAK_TFLOPS = 2500.0        # MI355X dense f16/bf16 (MI355X_MICROARCH.md)
# MI355X_MICROARCH.md "Global float atomics": ~1.3 TB/s of added bytes at four
# 64-B requests per 256-B wave instruction = 20.3 G requests/s chip-wide
ATOMIC_PEAK_GREQ = 1.3e12 / 64 / 1e9
# u32 atomics (the fixed-point hashed levels): 26.6 G requests/s measured
# (tools/atomic_probe.hip, profiles/r01/atomic_probe.json); the guide gives no
# integer figure
ATOMIC_U32_PEAK_GREQ = 26.6


# BASELINE.json configs by (sub-NeRFs, scale): C1/C2 single NGP (C1 is the
# reference's CPU case at 1024 rays), C3 K=2, C4 K=4 scale 16, C5 K=8 scale 16
def config_label(K, scale, rays):
    if K == 1:
        return "C1" if rays <= 1024 else "C2"
    if K == 2 and scale <= 0.5:
        return "C3"
    if K == 4 and scale >= 16:
        return "C4"
    if K == 8 and scale >= 16:
        return "C5"
    return "custom"


def mfma_measured(key, path=os.path.join(ROOT, "profiles", "mfma.json")):
    """MFMA busy fraction and achieved TFLOP/s per kernel from the committed
    counter pass of this workload (tools/gpu/mfma_r04.sh), or None."""
    try:
        with open(path) as f:
            return json.load(f).get("workloads", {}).get(key)
    except (OSError, ValueError):
        return None


def workload_key(K, scale, rays, occupancy, binned=False):
    """Key of a workload's PMC pass in profiles/traffic.json (tools/pmc_traffic.py);
    "_bin" when the grid gradient went through the binned scatter (its own pass:
    the walk's page stores replace the atomics)."""
    return f"K{K}_s{float(scale):g}_B{rays}_p{float(occupancy):.2f}" + ("_bin" if binned else "")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=8192, help="rays per GPU")
    ap.add_argument("--models", type=int, default=2)
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--occupancy", type=float, default=0.5)
    ap.add_argument("--cpu-rays", type=int, default=512,
                    help="rays in the bounded CPU-oracle sample: CPU baseline timing and the "
                         "rgb L_inf check (0 = skip)")
    ap.add_argument("--cpu-sample-rays", type=int, default=256,
                    help="rays of the workload in the timed CPU-baseline sample")
    ap.add_argument("--cpu-reps", type=int, default=10,
                    help="timed CPU-baseline steps (median; after 3 warm-up steps)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--train-step", type=int, default=1,
                    help="also time the full train step (loss + Adam); 0 = skip")
    ap.add_argument("--dropin-step", type=int, default=1,
                    help="also time the step through the drop-in rendering.ml_render chain; 0 = skip")
    ap.add_argument("--test-time-rays", type=int, default=640000,
                    help="rays of the test-time render leg (one 800x800 image; 0 = skip)")
    ap.add_argument("--density-update", type=int, default=1,
                    help="also time the occupancy-grid update (warm-up and sampled); 0 = skip")
    ap.add_argument("--split-bwd", action="store_true",
                    help="backward with one model per block (rn_field_bwd) instead of the "
                         "merged per-ray grid scatter (rn_field_bwd_merged)")
    ap.add_argument("--grid-fx", type=int, default=None,
                    help="fixed-point grid-gradient accumulation: 1 on, 0 fp32 atomics "
                         "(default: the renderer's choice)")
    ap.add_argument("--grid-bin", type=int, default=None,
                    help="binned (store + sum) grid-gradient scatter 1/0 (default: the "
                         "renderer's choice by shape)")
    ap.add_argument("--level-fwd", type=int, default=None,
                    help="level-partitioned field forward (rn_field_fwd_levels): 1 on, 0 the "
                         "merged forward (default: the renderer's choice)")
    ap.add_argument("--max-chunk", type=int, default=None,
                    help="merged backward: largest chunk of merged samples per queue grab "
                         "(default: the renderer's, by rays x sub-NeRFs)")
    ap.add_argument("--enc-blocks", type=int, default=None,
                    help="level-partitioned forward: encode workgroups (a multiple of 8; "
                         "default: the renderer's, 4096)")
    ap.add_argument("--mlp-blocks", type=int, default=None,
                    help="level-partitioned forward: MLP-tile workgroups (default 256)")
    ap.add_argument("--min-chunk", type=int, default=None,
                    help="merged backward: chunk of the last 1/8 of the work (default: the "
                         "renderer's, 512)")
    ap.add_argument("--plan-prep", type=int, default=None,
                    help="timing studies: 0 = the level forward's per-position input by its "
                         "own pass instead of from rn_bwd_plan")
    ap.add_argument("--balance-chunks", type=int, default=None,
                    help="merged backward: 1 = big chunks a multiple of the persistent "
                         "blocks in number (the renderer's default), 0 = max_chunk each")
    ap.add_argument("--head-chunk", type=int, default=None,
                    help="merged backward: the blocks' first chunks ramp from ~0 to this many "
                         "merged samples (0 = none; default: the renderer's, max_chunk at "
                         "scale 0.5)")
    ap.add_argument("--pinned", action="store_true",
                    help="sub-NeRF-per-GPU layout (SURVEY.md §8(e) C5): rank r renders ALL rays "
                         "for its K/N sub-NeRFs, per-ray outputs all-gathered (strong scaling)")
    ap.add_argument("--pinned-sim", type=int, default=0,
                    help="one GPU: time rank 0's share of the pinned layout over this many "
                         "ranks (its K/P sub-NeRFs over all rays + the gate backward; the "
                         "all-gather replaced by local copies, no collectives)")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend (auto: RCCL on GPUs); gloo only to rehearse the "
                         "multi-rank path on one GPU")
    ap.add_argument("--buckets", type=int, default=4,
                    help="N>1: the gradient all-reduce as this many asynchronous bucket "
                         "collectives, each averaged behind its own wait (1 = one collective)")
    ap.add_argument("--grid-split", type=int, default=8, choices=range(16), metavar="[0-15]",
                    help="N>1, binned fold: the grid levels [this, 16) are summed first and "
                         "their all-reduce starts while levels [0, this) are summed")
    ap.add_argument("--fx-f32-levels", default="",
                    help="comma-separated hash levels whose grid gradient goes in by fp32 "
                         "atomics instead of fixed point (e.g. 4,5,6,7,8; default none)")
    ap.add_argument("--bin-f32-levels", type=int, default=None, choices=range(17), metavar="[0-16]",
                    help="binned scatter: the coarse levels [0, n) by fp32 atomics instead of page "
                         "records (default: the renderer's choice by shape)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check the world size, print the ranks seen and exit "
                         "(no GPU work; with --backend gloo it runs on CPU)")
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def self_launch(args):
    """--gpus N > 1 with no torchrun environment: run this script under
    torch.distributed.run with N ranks (one process per GPU) as a child
    process and return its exit status; None when this process is a rank
    (or N = 1).  Runs before anything initialises the GPU in this process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def ranks_seen(rank, local, world, backend, dev_index):
    """(rank, local rank, host, device) of every rank, gathered on all ranks."""
    me = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": dev_index}
    if world == 1:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def check_world(args, world):
    if world != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but the process group has {world} "
                         f"rank(s)\n")
        sys.exit(3)


def launch_check(args, rank, local, world):
    """--launch-check: the launcher's contract without GPU work."""
    check_world(args, world)
    seen = ranks_seen(rank, local, world, None, None)
    # the headline N > 1 step's collective schedule on CPU tensors of the C3
    # gradient shapes (grid 45.7 MB, MLP, gate): the early MLP + gate bucket,
    # then the grid in args.buckets buckets, timed like the GPU run
    comm = None
    if world > 1:
        from radnerf_amd import dist as rdist
        from radnerf_amd import layout as LY
        n_grid = 2 * int(LY.grid_levels(0.5)["n_entries"])
        ar = rdist.GradAllReduce([torch.zeros(n_grid), torch.zeros(2, LY.FIELD_PARAMS),
                                  torch.zeros(LY.gate_params(2))], "cpu")
        for i, v in enumerate(ar.views):
            v.copy_(torch.randn(v.shape, generator=torch.Generator().manual_seed(rank * 10 + i)))
        local = ar.flat.clone()
        # the step's schedule: MLP + gate, the fine levels, the coarse levels
        rg = rdist.step_ranges(ar, LY.grid_levels(0.5)["offset"], args.grid_split)
        hs = [ar.launch_range(*rg["rest"], 1), ar.launch_range(*rg["fine"], args.buckets),
              ar.launch_range(*rg["coarse"], 1)]
        for h in hs:
            ar.finish(h)
        comm = ar.comm_stats(1)
        # the same local gradients through one plain all-reduce: equal within
        # rounding (bit-identical at world 2; with more ranks the ring's
        # summation order follows the bucket bounds), and the same bits on
        # every rank
        ref = local.clone()
        dist.all_reduce(ref)
        ref.div_(world)
        r0 = ar.flat.clone()
        dist.broadcast(r0, 0)
        same = torch.tensor([int(torch.equal(ar.flat, r0))])
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        comm["mean_bit_identical"] = bool(torch.equal(ar.flat, ref))
        comm["rank_consistent"] = bool(same.item())
        comm["mean_ok"] = bool(torch.allclose(ar.flat, ref, rtol=1e-6, atol=1e-6)) \
            and comm["rank_consistent"]
        comm["ranges"] = {k: list(v) for k, v in rg.items()}
        comm["backend"] = dist.get_backend()
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world,
                          "backend": dist.get_backend() if world > 1 else None,
                          "comm": comm, "ranks_seen": seen}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    from radnerf_amd import dist as rdist
    from radnerf_amd import synthetic as S
    from radnerf_amd.fused import FusedMLRenderer
    from radnerf_amd.networks import MNGP, Ray_Gate

    backend = None if args.backend == "auto" else args.backend
    if args.launch_check:
        rank, local, world = rdist.init(backend=backend or "gloo")
        return launch_check(args, rank, local, world)
    rank, local, world = rdist.init(backend=backend)
    check_world(args, world)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    local = rdist.device_index(local)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, K, scale = args.rays, args.models, args.scale
    esf = 1.0 / 256 if scale > 0.5 else 0.0

    if K == 1:
        # single NGP (C1 / C2): the model render() takes (density_bitfield)
        from radnerf_amd.networks import NGP
        model = NGP(scale, seed=3).to(dev)
    else:
        model = MNGP(scale, size=K, seed=3).to(dev)
    gate = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, model.cascades, p=args.occupancy, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    # data parallel: every rank its own rays; pinned: the same rays on every rank
    rs = 0 if (args.pinned or args.pinned_sim) else rank
    o_np, d_np = S.rays(B, scale, seed=1000 * rs)
    rays_o = torch.from_numpy(o_np).to(dev)
    rays_d = torch.from_numpy(d_np).to(dev)
    noises = [torch.from_numpy(S.noise(K, B, seed=2 + 7919 * rs + i)).to(dev) for i in range(4)]
    seeds_np = S.loss_seeds(B, K, seed=4 + rs)
    g_rgb, g_op, g_depth = (torch.from_numpy(s).to(dev) for s in seeds_np)
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)

    if args.pinned_sim:
        if world != 1:
            raise SystemExit("--pinned-sim runs on one process")
        from radnerf_amd.pinned import PinnedMLRenderer
        r = PinnedMLRenderer(model, gate, B, sim=(0, args.pinned_sim))
    elif args.pinned:
        from radnerf_amd.pinned import PinnedMLRenderer
        r = PinnedMLRenderer(model, gate, B)
    else:
        r = FusedMLRenderer(model, gate, B)
    r.merged_bwd = r.merged_bwd and not args.split_bwd
    if args.grid_fx is not None:
        r.grid_fx = bool(args.grid_fx)
    if args.bin_f32_levels is not None:
        r.bin_f32_levels = args.bin_f32_levels
    if args.fx_f32_levels:
        r.fx_f32_levels = tuple(int(x) for x in args.fx_f32_levels.split(","))
    if args.grid_bin is not None:
        r.grid_bin = bool(args.grid_bin) and r.grid_fx
    if args.level_fwd is not None:
        r.level_fwd = bool(args.level_fwd)
    if args.max_chunk:
        r.max_chunk = args.max_chunk
    if args.head_chunk is not None:
        r.head_chunk = args.head_chunk
    if args.min_chunk:
        r.min_chunk = args.min_chunk
    if args.enc_blocks:
        r.level_enc_blocks = args.enc_blocks
    if args.mlp_blocks:
        r.level_mlp_blocks = args.mlp_blocks
    if args.balance_chunks is not None:
        r.balance_chunks = bool(args.balance_chunks)
    if args.plan_prep is not None:
        r.plan_prep = bool(args.plan_prep)
    ar = rdist.GradAllReduce([model.xyz_encoder.params, model.mlp_params, gate.params], dev)
    samples_acc = torch.zeros((), dtype=torch.int64, device=dev)

    # data parallel: the MLP + gate gradients (one small bucket) go out as soon
    # as field_bwd has written them, beside the grid gradient's fold (or bin
    # + sum); the grid gradient in args.buckets buckets after the backward.
    # Both on a comm stream, bracketed by events there (comm fields below).
    r.grid_split_level = args.grid_split
    rng = rdist.step_ranges(ar, model.xyz_encoder.h_offset, r.grid_split_level)
    comm_on = [world > 1]
    pending = []
    grid_early = [None]             # the grid range already launched this step
    # gloo's collectives on device tensors block the host until they complete:
    # launched from inside the backward they stall the launch queue mid-step
    # (the 2-rank gloo rehearsal on one GPU fell from 476 to 80 Msamples/s),
    # so with gloo every bucket goes out after the backward
    early_ok = world > 1 and dist.get_backend() == "nccl"

    def early_bucket():
        if comm_on[0] and early_ok:
            main = torch.cuda.current_stream(dev)
            main.wait_stream(r._side(dev))       # the gate backward ran on the side stream
            pending.append(ar.launch_range(*rng["rest"], 1))

    def grid_levels_ready(split):
        # binned fold: levels [split, 16) are summed, [0, split) not yet (split
        # 0: the whole grid is final) -- their collective overlaps the rest
        if comm_on[0] and early_ok:
            a, b = rdist.step_ranges(ar, model.xyz_encoder.h_offset, split)["fine"]
            pending.append(ar.launch_range(a, b, args.buckets))
            grid_early[0] = a

    r.after_field_bwd = early_bucket
    # (one rank: no collective to overlap, the fold sums every level in one launch)
    r.after_grid_levels = grid_levels_ready if world > 1 else None

    def step(i):
        ar.zero()
        _, _, _, gt, _ = r.forward(rays_o, rays_d, rays_d, noises[i % 4], bg, 1e-4, esf)
        samples_acc.add_(r.ws.meta[1])
        grid_early[0] = None
        r.backward(rays_o, rays_d, rays_d, gt, bg, g_rgb, g_op, g_depth, None, 1e-4,
                   grid_grad=ar.views[0], mlp_grad=ar.views[1], gate_grad=ar.views[2])
        if comm_on[0]:
            if not pending:                      # (no merged backward: no early bucket)
                pending.append(ar.launch_range(*rng["rest"], 1))
            g0, g1 = ar.param_range(0, 1)
            if grid_early[0] is None:            # gloo: the whole grid after the backward
                pending.append(ar.launch_range(g0, g1, args.buckets))
            elif grid_early[0] > g0:             # the coarse levels, summed last
                pending.append(ar.launch_range(g0, grid_early[0], 1))
            for h in pending:                    # pinned: partial gradients add up
                ar.finish(h, average=not args.pinned)
            pending.clear()

    log(f"rank {rank}/{world}: warm-up ({args.warmup} steps)")
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    samples_acc.zero_()
    ar.reset_timing()
    # timed region: HIP events only around the roofline kernel (an event pair
    # per launch costs ~5 us of queue time; all twelve would add ~2.5 %)
    binned_run = bool(getattr(r, "grid_bin", False) and r.grid_fx and not args.split_bwd)
    # (binned scatter: the fold's two event spans too -- the roofline covers
    # field_bwd + bin + sum)
    r.trace = {"field_bwd", "fx_bin", "fx_sum"} if binned_run else {"field_bwd"}
    r.events = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    live = r.kernel_times_ms()
    bwd_live = live["field_bwd"]
    comm = None
    if world > 1:
        # the collectives of the timed steps, then the same steps without them:
        # exposed = what the all-reduce adds to the step (max over ranks)
        comm = ar.comm_stats(args.steps)
        comm_on[0] = False
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        dist.barrier()
        no_comm = torch.tensor(time.perf_counter() - t1, device=dev, dtype=torch.float64)
        with_comm = torch.tensor(elapsed, device=dev, dtype=torch.float64)
        dist.all_reduce(no_comm, op=dist.ReduceOp.MAX)
        dist.all_reduce(with_comm, op=dist.ReduceOp.MAX)
        comm_on[0] = True
        comm.update({
            "ms_per_step_without": round(float(no_comm) / args.steps * 1e3, 4),
            "exposed_ms": round((float(with_comm) - float(no_comm)) / args.steps * 1e3, 4),
            "backend": dist.get_backend(),
            "schedule": ("MLP+gate bucket after field_bwd (beside the grid fold); binned fold: "
                         f"grid levels [{args.grid_split}, 16) in {args.buckets} buckets once "
                         "summed (beside the coarse levels' sum), levels "
                         f"[0, {args.grid_split}) after it; int32 fold: the grid in "
                         f"{args.buckets} buckets after the fold; comm stream events"
                         if early_ok else
                         f"gloo: MLP+gate bucket and the grid in {args.buckets} buckets after the "
                         "backward (host-blocking collectives); comm stream events")})
    # per-kernel breakdown: the same steps again with every launch traced
    # (after the timed region; not part of `value`)
    r.trace = True
    r.events = {}
    saved = samples_acc.clone()
    for i in range(args.steps):
        step(i)
    samples_acc.copy_(saved)
    r.trace = False
    kt = r.kernel_times_ms()
    kt["field_bwd"] = bwd_live
    for k_ in ("fx_bin", "fx_sum"):             # the binned fold, timed in the headline region
        if k_ in live:
            kt[k_] = live[k_]
    # gate_bwd runs on a side stream beside field_bwd (hidden there, but its
    # events then span the wait for CUs): its own duration, in line
    at = r.gate_bwd_at
    r.gate_bwd_at, r.trace, r.events = "main", {"gate_bwd"}, {}
    for i in range(3):
        step(i)
    samples_acc.copy_(saved)
    r.gate_bwd_at, r.trace = at, False
    gt_ms = r.kernel_times_ms().get("gate_bwd")
    if gt_ms:                       # (one sub-NeRF: no gate MLP at all)
        kt["gate_bwd"] = gt_ms

    # forward-only rate (north_star's forward target), timed after the headline
    # region with the same barrier/sync bracketing; not part of `value`
    fwd_acc = torch.zeros((), dtype=torch.int64, device=dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        r.forward(rays_o, rays_d, rays_d, noises[i % 4], bg, 1e-4, esf)
        fwd_acc.add_(r.ws.meta[1])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    fwd_elapsed = torch.tensor(time.perf_counter() - t0, device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(fwd_acc)
        dist.all_reduce(fwd_elapsed, op=dist.ReduceOp.MAX)
    fwd_only = {"value": round(int(fwd_acc) / float(fwd_elapsed) / 1e6, 2), "unit": "Msamples/s",
                "ms_per_step": round(float(fwd_elapsed) / args.steps * 1e3, 4)}

    # full training step of train_ml.py: render ->
    # fused NeRFLoss (opacity 1e-3, CV^2 1e-2, depth-mutual 5e-2) -> backward ->
    # (all-reduce) -> FusedAdam; synthetic target colours.  Not part of `value`.
    train = None
    if args.train_step:
        log("train step leg")
        from radnerf_amd.optim import FusedAdam
        params = [model.xyz_encoder.params, model.mlp_params, gate.params]
        for p_, v_ in zip(params, ar.views):
            p_.grad = v_
        r.after_field_bwd = None        # reduce_and_step launches every bucket itself
        r.after_grid_levels = None
        opt = FusedAdam(params, lr=1e-2, eps=1e-15)   # train_ml.py:143 (apex defaults)
        tgt = torch.rand(B, 3, generator=torch.Generator().manual_seed(7 + rank)).to(dev)

        def tstep(i):
            ar.zero()
            r.train_step(rays_o, rays_d, rays_d, tgt, noises[i % 4], bg, 1e-3, 1e-2, 5e-2,
                         1e-4, esf, ar.views[0], ar.views[1], ar.views[2])
            # all-reduce with Adam as its epilogue (one rank: plain Adam)
            ar.reduce_and_step(opt, average=not args.pinned)

        for i in range(2):
            tstep(i)
        tr_acc = torch.zeros((), dtype=torch.int64, device=dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            tstep(i)
            tr_acc.add_(r.ws.meta[1])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tr_el = torch.tensor(time.perf_counter() - t0, device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tr_acc)
            dist.all_reduce(tr_el, op=dist.ReduceOp.MAX)
        train = {"value": round(int(tr_acc) / float(tr_el) / 1e6, 2), "unit": "Msamples/s",
                 "ms_per_step": round(float(tr_el) / args.steps * 1e3, 4),
                 "includes": "render + fused loss + backward + (bucketed all-reduce with) FusedAdam"}
    # the same step through the drop-in path (rendering.ml_render: the
    # reference's op-by-op autograd structure, vren ops + field autograd on the
    # same kernels), for the callers that keep ml_rendering.py; rank 0 at N=1.
    # Same rays and noise cycle as the headline, so the same samples per step.
    dropin, api_step = None, None
    if args.dropin_step and world == 1:
        log("drop-in / API legs")
        from radnerf_amd.rendering import ml_render, render

        def dstep(i, fused=False):
            model.zero_grad(set_to_none=True)
            gate.zero_grad(set_to_none=True)
            if K == 1:
                # train.py:118 -> rendering.render (single NGP)
                res = render(model, rays_o, rays_d, noise=noises[i % 4][0], exp_step_factor=esf,
                             fused=fused)
                torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]],
                                        [g_rgb, g_op, g_depth[:, 0]])
            else:
                res = ml_render(model, gate, rays_o, rays_d, rays_d, noise=noises[i % 4],
                                exp_step_factor=esf, fused=fused)
                torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]],
                                        [g_rgb, g_op, g_depth])

        def timed(fused):
            for i in range(2):
                dstep(i, fused)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                dstep(i, fused)
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        fn = "rendering.render" if K == 1 else "rendering.ml_render"
        d_el = timed(False)
        dropin = {"value": round(int(samples_acc) / d_el / 1e6, 2), "unit": "Msamples/s",
                  "ms_per_step": round(d_el / args.steps * 1e3, 4),
                  "path": f"{fn}(fused=False) (drop-in op-by-op autograd chain), fwd+bwd"}
        # the caller's own API with its default (fused) training render
        a_el = timed(True)
        api_step = {"value": round(int(samples_acc) / a_el / 1e6, 2), "unit": "Msamples/s",
                    "ms_per_step": round(a_el / args.steps * 1e3, 4),
                    "path": f"{fn}() default (fused chain through autograd), fwd+bwd"}
    # occupancy-grid maintenance (train_ml.py:174-177;
    # every 16 steps, outside the metric): the warm-up update over all
    # 128^3 x cascades cells of every sub-NeRF, and the regular update over
    # 128^3/4 uniform + 128^3/4 occupied cells, rank-consistent stream
    density = None
    if args.density_update:
        log("density-update leg")
        thr = 0.01 * 1024 / 3 ** 0.5
        dms = {}
        # the update rewrites the occupancy buffers: restore them afterwards
        # (the oracle leg below marches the workload's original bitfields)
        saved_buf = {n: b.clone() for n, b in model.named_buffers() if "density" in n}
        for name, warm in (("warmup_all_cells", True), ("sampled_cells", False)):
            rdist.update_density_grid(model, thr, 0, warmup=warm)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(3):
                rdist.update_density_grid(model, thr, i + 1, warmup=warm)
            torch.cuda.synchronize()
            dms[name] = round((time.perf_counter() - t0) / 3 * 1e3, 3)
        with torch.no_grad():
            for n_, b_ in model.named_buffers():
                if n_ in saved_buf:
                    b_.copy_(saved_buf[n_])
        cells = model.cascades * 128 ** 3
        density = {"ms": dms, "cells_per_model_warmup": cells, "models": K,
                   "kernel": "rn_field_density (hash grid + geo MLP) + morton / packbits"}
    # test-time render (row a10, ml_rendering.py:81-155): one image of
    # --test-time-rays rays through ml_render(test_time=True); not part of `value`
    test_time = None
    if args.test_time_rays and world == 1:
        log("test-time render leg")
        from radnerf_amd.rendering import ml_render
        nt = args.test_time_rays
        ot, dt_ = (torch.from_numpy(a).to(dev) for a in S.rays(nt, scale, seed=99))
        with torch.no_grad():
            res_t = ml_render(model, gate, ot, dt_, dt_, test_time=True, exp_step_factor=esf)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                res_t = ml_render(model, gate, ot, dt_, dt_, test_time=True, exp_step_factor=esf)
            torch.cuda.synchronize()
            t_el = (time.perf_counter() - t0) / reps
            # the reference's host-driven compaction loop on the same kernels
            # (fused=False), once, for comparison
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res_l = ml_render(model, gate, ot, dt_, dt_, test_time=True, exp_step_factor=esf,
                              fused=False)
            torch.cuda.synchronize()
            t_loop = time.perf_counter() - t0
        test_time = {"rays": nt, "ms_per_image": round(t_el * 1e3, 3),
                     "Mrays_per_s": round(nt / t_el / 1e6, 3),
                     "Msamples_per_s": round(float(res_t["total_samples"]) / t_el / 1e6, 1)
                     if "total_samples" in res_t else None,
                     "opacity_mean": round(float(res_t["opacity"].mean()), 4),
                     "loop_ms_per_image": round(t_loop * 1e3, 3),
                     "loop_vs_fused_rgb_linf": float((res_t["rgb"] - res_l["rgb"]).abs().max()),
                     "path": "rendering.ml_render(test_time=True): rn_render_test (wave per ray); "
                             "loop = the host compaction loop (fused=False)"}
    n_samples = samples_acc.clone()
    t_max = torch.tensor(elapsed, device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(n_samples)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max)
    total_samples = int(n_samples)
    value = total_samples / elapsed / 1e6

    # per-kernel breakdown (rank 0) and the roofline of the dominant kernel
    kms = {k: float(np.mean(v)) for k, v in kt.items()}
    if "fx_bin" in kms:             # binned fold: bin + check, then the sums (redo between)
        kms["fx_fold"] = kms["fx_bin"] + kms.get("fx_sum", 0.0)
    samples_per_step_rank = int(samples_acc) / args.steps
    bwd_ms = kms.get("field_bwd", float("nan"))
    achieved = samples_per_step_rank * FIELD_BWD_BYTES_PER_SAMPLE / (bwd_ms * 1e-3) / 1e9
    # PMC figures only for a workload that has its own pass (tools/pmc_traffic.py
    # --merge keys them by K, scale, rays and occupancy); per launch, scaled by
    # this run's sample count where it differs from the profiled run's
    binned = bool(getattr(r, "grid_bin", False) and r.grid_fx and not args.split_bwd)
    traffic, atom_req, pmc_samples, pmc_key = None, None, None, workload_key(
        K, scale, B, args.occupancy, binned)
    tj = None
    if os.path.exists(args.traffic_json) and not args.split_bwd:
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f).get("workloads", {}).get(pmc_key)
            if tj:
                pmc_samples = tj.get("samples_per_launch") or samples_per_step_rank
                traffic = tj.get("field_bwd_bytes_per_launch")
                if traffic:
                    traffic = round(traffic * samples_per_step_rank / pmc_samples)
                atom_req = tj.get("field_bwd_atomic_requests")
        except (OSError, ValueError, AttributeError):
            traffic = None
    roofline = {"kernel": "field_bwd (k_field_bwd_merged)", "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": pmc_key if traffic else None,
                "algorithmic_bytes_per_sample": FIELD_BWD_BYTES_PER_SAMPLE,
                "samples_per_launch": round(samples_per_step_rank),
                "avg_launch_ms": round(bwd_ms, 4),
                # the grid-gradient scatter is bound by the memory-side float-atomic
                # request rate, not by HBM bytes (DESIGN.md "field_bwd")
                "path_achieved_GBs": round(value / world * PATH_BYTES_PER_SAMPLE / 1e3, 1)}
    if atom_req:
        # requests per launch from the PMC pass (tools/pmc_traffic.py), scaled to
        # this run's sample count; rate against the chip-wide atomic ceiling of
        # this launch's mix of f32 adds and (fixed point) u32 adds
        req = atom_req * samples_per_step_rank / pmc_samples
        rate = req / (bwd_ms * 1e-3) / 1e9
        # fixed point: every level's records go in as u32 adds from the second
        # step of a workspace on (round 3; round 2 kept the dense levels' 8 %
        # of C3's requests in fp32)
        u32_share = 1.0 if r.grid_fx and not args.split_bwd else 0.0
        peak = 1.0 / ((1 - u32_share) / ATOMIC_PEAK_GREQ + u32_share / ATOMIC_U32_PEAK_GREQ)
        roofline["atomic"] = {"requests_per_launch": round(req), "requests_per_sample":
                              round(req / samples_per_step_rank, 2),
                              "achieved": round(rate, 2), "peak": round(peak, 2), "unit": "G req/s",
                              "u32_share": u32_share,
                              "frac": round(rate / peak, 3)}
        if binned:
            # the walk issues no grid atomics in binned mode: the pass shows
            # what is left (the dense levels' first fp32 step aside, none)
            roofline["atomic"]["note"] = "binned scatter: PMC TCC_EA0_ATOMIC of the walk"
    if binned and not atom_req:
        roofline["atomic"] = None
    if binned:
        # the binned scatter's own passes (fx_fold = rn_grid_binned_fold: bin +
        # check + sum): 8 B per record stored by the walk, 16 B moved by the bin
        # pass (read + write), 8 B read by the sum pass
        pool = r.ws._bin
        npg = min(int(pool["ctl"][0]), pool["pages"])
        recs = int((pool["meta"][:npg] >> 8).sum()) if npg else 0
        fold_ms = kms.get("fx_fold", float("nan"))
        roofline["binned"] = {
            "records_per_launch": recs, "records_per_sample": round(recs / max(1, samples_per_step_rank), 2),
            "pages": npg, "fold_ms": round(fold_ms, 4),
            "fold_bytes": 24 * recs, "fold_GBs": round(24 * recs / (fold_ms * 1e-3) / 1e9, 1),
            "fold_frac": round(24 * recs / (fold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "fold_traffic": (tj or {}).get("grid_fold_bytes_per_launch"),
            "walk_store_bytes": 8 * recs}
        # the scatter finishes in the fold: the roofline covers the merged
        # backward + bin + check + sum (algorithmic bytes as for field_bwd alone,
        # 1,064 per sample; traffic = the walk's + the fold's PMC bytes); the
        # merged backward alone stays in field_bwd_only
        if fold_ms == fold_ms:
            only = {k_: roofline[k_] for k_ in ("kernel", "achieved", "frac", "traffic",
                                                "avg_launch_ms")}
            tot_ms = bwd_ms + fold_ms
            ach = samples_per_step_rank * FIELD_BWD_BYTES_PER_SAMPLE / (tot_ms * 1e-3) / 1e9
            ft = (tj or {}).get("grid_fold_bytes_per_launch")
            roofline.update({
                "kernel": "field_bwd + binned fold (k_field_bwd_merged, k_grid_bin, k_fx_check, "
                          "k_grid_sum)",
                "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "avg_launch_ms": round(tot_ms, 4),
                "traffic": (round((traffic or 0) + ft * samples_per_step_rank / pmc_samples)
                            if traffic and ft and pmc_samples else None),
                "field_bwd_only": only})

    rgb_linf = None
    cpu_base = None
    if rank == 0 and world == 1 and args.cpu_rays > 0:
        log("oracle legs (rgb check, CPU baseline)")
        rgb_linf, cpu_base = oracle_legs(args, model, gate, bits, o_np, d_np, noises[0], r,
                                         rays_o, rays_d, bg, esf, scale, seeds_np)

    label = config_label(K, scale, B if not (args.pinned or args.pinned_sim) else 8192)
    seen = ranks_seen(rank, local, world, None, torch.cuda.current_device())
    if args.pinned_sim:
        workload = (f"{label} Rad-NeRF train_ml.py K={K} gate=ray, pinned layout simulated on one "
                    f"GPU: rank 0 of {args.pinned_sim} ({K // args.pinned_sim} sub-NeRF(s) over "
                    f"all B={B} rays + gate backward; all-gather by local copies, no all-reduce), "
                    f"scale={scale}, random 128^3 occupancy p={args.occupancy:.2f}")
    elif args.pinned:
        workload = (f"{label} Rad-NeRF train_ml.py K={K} gate=ray, sub-NeRFs pinned {K // world} "
                    f"per GPU, B={B} rays on every GPU, scale={scale}, random 128^3 occupancy "
                    f"p={args.occupancy:.2f}")
    else:
        workload = (f"{label} Rad-NeRF train_ml.py K={K} gate=ray B={B}/GPU scale={scale}, "
                    f"random 128^3 occupancy p={args.occupancy:.2f}")
    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
               "scaling": "strong" if args.pinned else "weak", "vs_baseline": None,
               "dtype": "f16/f32",
               "data": "synthetic",
               "backend": dist.get_backend() if world > 1 else None,
               "comm": comm,
               "ranks_seen": seen,
               "config": {"workload": workload,
                          "rays_per_gpu": B, "model_zoo_size": K, "scale": scale,
                          "occupancy": args.occupancy,
                          "config": label,
                          "field_fwd": "levels" if getattr(r, "level_fwd", False) else "merged",
                          "grid_scatter": ("binned" if binned else "fixed-point atomics"
                                           if r.grid_fx and not args.split_bwd else "fp32 atomics"),
                          "fx_f32_levels": list(getattr(r, "fx_f32_levels", ())),
                          "bin_f32_levels": int(getattr(r, "bin_f32_levels", 0)) if binned else None,
                          "samples_per_step_per_gpu": round(samples_per_step_rank),
                          "global_batch": B if args.pinned else B * world,
                          "parallelism": (f"pinned{args.pinned_sim}-rank0-sim" if args.pinned_sim
                                          else f"pinned{world}" if args.pinned else f"dp{world}")},
               "roofline": roofline, "cpu_baseline": cpu_base,
               "rgb_linf_vs_ref": rgb_linf,
               "forward_only": fwd_only,
               "train_step": train,
               "dropin_step": dropin,
               "api_step": api_step,
               "density_update": density,
               "test_time_render": test_time,
               # MFMA use: algorithmic MLP flops (56,832 per sample
               # fwd+bwd, unpadded) at `value`, against the dense f16 peak
               "mfma": {"achieved": round(value / world * MLP_FLOP_PER_SAMPLE / 1e6, 2),
                        "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(value / world * MLP_FLOP_PER_SAMPLE / 1e6 / MFMA_F16_PEAK_TFLOPS, 5),
                        # measured: SQ_VALU_MFMA_BUSY_CYCLES per kernel of this
                        # workload's rocprofv3 pass (tools/mfma_reduce.py,
                        # profiles/mfma.json), None when it has no pass
                        "measured": mfma_measured(pmc_key)},
               "kernel_ms": {k: round(v, 4) for k, v in sorted(kms.items())}}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def log(msg):
    """progress on stderr (a long leg must not look hung to the GPU-box watchdog)"""
    sys.stderr.write(f"[bench {time.strftime('%H:%M:%S')}] {msg}\n")
    sys.stderr.flush()


def _cgroup_cpus():
    """CPUs the cgroup quota allows (cpu.max), or None when unlimited/unknown."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def _cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _time_oracle(args_fn, reps, warm, limit=None):
    """median wall time of `reps` oracle steps after `warm` untimed ones; a
    first step slower than `limit` s ends the timing there (an oversubscribed
    thread count in the sweep: its one step is the figure)"""
    from oracle import ml_oracle
    ts, res = [], None
    for i in range(warm + reps):
        t0 = time.perf_counter()
        res = ml_oracle.ml_train_step(*args_fn())
        dt = time.perf_counter() - t0
        log(f"  oracle step {i + 1}/{warm + reps}: {dt:.2f} s")
        if i == 0 and limit is not None and dt > limit:
            return dt, res
        if i >= warm:
            ts.append(dt)
    return float(np.median(ts)), res


def oracle_legs(args, model, gate, bits, o_np, d_np, noise, r, rays_o, rays_d, bg, esf, scale,
                seeds_np):
    """rgb L_inf of the GPU path vs the CPU oracle on the first rays of the
    workload, and the CPU baseline: the oracle (C march /
    composite with OpenMP over rays + torch-CPU fp32 field) timed as 3 untimed
    + 10 timed fwd+bwd steps, median, on (a) a bounded sample of this
    workload and (b) config C1 (single NGP, 1024 rays, scale 0.5)."""
    from oracle import ml_oracle
    from radnerf_amd import layout as LY
    from radnerf_amd import synthetic as S
    n = args.cpu_rays
    rgb, _, _, _, _ = r.forward(rays_o, rays_d, rays_d, noise, bg, 1e-4, esf)
    rgb = rgb.cpu().numpy()
    gp = model.xyz_encoder.params.detach().cpu().view(-1, 2).numpy()
    mp = model.mlp_params.detach().cpu().numpy()
    ap = gate.params.detach().cpu().numpy()
    nz = noise.cpu().numpy()
    from oracle import set_threads
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    env_share = int(os.environ.get("OMP_NUM_THREADS", 0) or 0)
    quota = _cgroup_cpus()

    def use_threads(n):
        torch.set_num_threads(n)
        set_threads(n)

    # correctness leg: the GPU's rgb on the first n rays against the oracle's
    use_threads(env_share or min(16, usable))
    res = ml_oracle.ml_train_step(o_np[:n], d_np[:n], bits, np.ascontiguousarray(nz[:, :n]),
                                  gp, mp, ap, scale, seeds=tuple(np.ascontiguousarray(x[:n])
                                                                 for x in seeds_np))
    rgb_linf = float(np.abs(res["rgb"] - rgb[:n]).max())
    # (a) bounded sample of this workload, timed at each thread count: the
    # box's CPU share (OMP_NUM_THREADS), the per-GPU share of the node
    # (nproc / 8 GPUs) and every usable core (nproc); the
    # baseline is the fastest
    c = args.cpu_sample_rays
    sd = tuple(np.ascontiguousarray(x[:c]) for x in seeds_np)
    nzc = np.ascontiguousarray(nz[:, :c])
    counts = sorted({t for t in (env_share, max(1, nproc // 8), nproc, usable) if t > 0})
    sweep, best = [], None
    for t in counts:
        if quota is not None and t > quota and best is not None:
            # more threads than the cgroup's CPU quota lets run: not a
            # measurement of t cores (recorded as skipped)
            sweep.append({"threads": t, "skipped": f"cgroup CPU quota {quota} CPUs"})
            continue
        log(f"cpu baseline: {t} threads")
        use_threads(t)
        first = best is None
        t_a, res_a = _time_oracle(lambda: (o_np[:c], d_np[:c], bits, nzc, gp, mp, ap, scale, sd),
                                  args.cpu_reps if first else max(3, args.cpu_reps // 2),
                                  3 if first else 1, None if first else 3 * best[2])
        v = res_a["total"] / t_a / 1e6
        sweep.append({"threads": t, "value": round(v, 5), "s_per_step": round(t_a, 3)})
        if best is None or v > best[0]:
            best = (v, t, t_a, res_a)
    v_a, threads, t_a, res_a = best
    use_threads(threads)
    # (b) C1: single NGP (K = 1), 1024 rays, scale 0.5, the same synthetic recipe
    lv = LY.grid_levels(0.5)
    g1 = S.grid_params(lv["n_entries"], seed=3).reshape(-1, 2)
    m1 = S.mlp_params(1, LY.FIELD_PARAMS, seed=3)
    b1 = S.bitfields(1, 1, p=args.occupancy, seed=1)
    o1, d1 = S.rays(1024, 0.5, seed=11)
    n1 = S.noise(1, 1024, seed=12)
    s1 = S.loss_seeds(1024, 1, seed=13)
    gate1 = np.zeros(LY.gate_params(1), np.float32)        # softmax over one model = 1
    t_b, res_b = _time_oracle(lambda: (o1, d1, b1, n1, g1, m1, gate1, 0.5, s1), args.cpu_reps, 3)
    cpu = {"value": round(v_a, 5), "unit": "Msamples/s",
           "cores": threads, "kind": "port",
           "sample": f"{c} rays x K={args.models} ({res_a['total']} samples) of the same workload, "
                     f"fwd+bwd step of oracle/ml_oracle.py (C march/composite, OpenMP over rays; "
                     f"torch-CPU fp32 field), median of {args.cpu_reps} after 3 warm-up, "
                     f"{t_a:.2f} s/step at {threads} threads (fastest of the sweep)",
           "thread_sweep": sweep,
           "c1": {"value": round(res_b["total"] / t_b / 1e6, 5), "unit": "Msamples/s",
                  "threads": threads,
                  "sample": f"C1: single NGP, 1024 rays, scale 0.5 ({res_b['total']} samples), "
                            f"median of {args.cpu_reps} after 3 warm-up, {t_b:.2f} s/step"},
           "nproc": nproc, "usable_cpus": usable, "cgroup_cpu_quota": quota,
           "omp_num_threads_env": env_share or None,
           "cpu_model": _cpu_model_name()}
    return rgb_linf, cpu


if __name__ == "__main__":
    main()
