"""CPU: ray-batch data parallelism over torch.distributed (gloo, world size 2).
Same code path as the RCCL run of bench.py --gpus N (radnerf_amd/dist.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from radnerf_amd import dist as rdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _RecordingOpt:
    """Stands in for FusedAdam (a GPU kernel) in the epilogue test: records
    the ranges it is asked to update and the gradient they held then."""
    def __init__(self):
        self.calls, self.snap, self.began, self.ended = [], {}, False, False

    def begin_step(self):
        self.began = True

    def update_range(self, p, lo, hi, grad_scale=1.0):
        self.calls.append((p, lo, hi, grad_scale))
        self.snap[(id(p), lo)] = p.grad.view(-1)[lo:hi].clone()

    def end_step(self):
        self.ended = True

    def step(self):
        raise AssertionError("world > 1 goes through the epilogue")


def _step_schedule(rank, world, scale, K, buckets, split):
    """bench.py's N > 1 headline schedule on CPU tensors of the config's
    gradient shapes (grid, K MLPs, gate): the MLP + gate bucket, the fine grid
    levels in `buckets` pieces, the coarse levels -- every element reduced
    exactly once, the mean within rounding of one plain all-reduce (with more
    than two ranks the ring's summation order follows the bucket bounds, so
    bit-identity holds only at world 2, test_bench_self_launch_gloo) and
    bit-identical on every rank (the ranks stay consistent)."""
    from radnerf_amd import layout as LY
    lv = LY.grid_levels(scale)
    ar = rdist.GradAllReduce([torch.zeros(2 * int(lv["n_entries"])),
                              torch.zeros(K, LY.FIELD_PARAMS), torch.zeros(LY.gate_params(K))],
                             "cpu")
    gen = torch.Generator().manual_seed(1000 + rank)
    ar.flat.copy_(torch.randn(ar.flat.numel(), generator=gen))
    local = ar.flat.clone()
    rg = rdist.step_ranges(ar, lv["offset"], split)
    hs = [ar.launch_range(*rg["rest"], 1), ar.launch_range(*rg["fine"], buckets),
          ar.launch_range(*rg["coarse"], 1)]
    for h in hs:
        ar.finish(h)
    seen = torch.zeros(ar.flat.numel(), dtype=torch.int32)
    for h in hs:
        for (lo, hi), _, _ in h["parts"]:
            seen[lo:hi] += 1
    ref = local.clone()
    dist.all_reduce(ref)
    ref.div_(world)
    n_parts = sum(len(h["parts"]) for h in hs)
    r0 = ar.flat.clone()
    dist.broadcast(r0, 0)
    return (bool((seen == 1).all()) and torch.allclose(ar.flat, ref, rtol=1e-6, atol=1e-6)
            and torch.equal(ar.flat, r0) and n_parts == buckets + 2)


def _worker(rank, world, port, q, sched=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        r, local, w = rdist.init(backend="gloo")
        assert (r, w) == (rank, world)
        # disjoint contiguous ray shards covering the global batch
        lo, hi = rdist.shard_rays(1000, r, w)
        # flat-buffer gradient all-reduce (mean)
        params = [torch.zeros(5, 2), torch.zeros(3), torch.zeros(4, 4)]
        ar = rdist.GradAllReduce(params, "cpu")
        for i, v in enumerate(ar.views):
            v.fill_(float(rank + 1) * (i + 1))
        views = ar.reduce()
        mf = (world + 1) / 2          # mean of rank + 1 over the ranks
        ok_mean = all(torch.allclose(v, torch.full_like(v, mf * (i + 1)))
                      for i, v in enumerate(views))
        # the same as 3 asynchronous buckets (bench.py's headline N>1 step)
        for i, v in enumerate(ar.views):
            v.copy_(torch.arange(v.numel(), dtype=torch.float32).view_as(v) * (rank + 1) + i)
        views = ar.reduce(n_buckets=3)
        ok_mean = ok_mean and all(
            torch.allclose(v, (torch.arange(v.numel(), dtype=torch.float32).view_as(v) * mf + i))
            for i, v in enumerate(views))
        # density buffers synchronised from rank 0
        m = torch.nn.Module()
        m.register_buffer("density_bitfield_0", torch.full((8,), rank, dtype=torch.uint8))
        m.register_buffer("other", torch.full((2,), rank))
        rdist.broadcast_buffers(m)
        ok_bcast = bool((m.density_bitfield_0 == 0).all()) and int(m.other[0]) == rank
        # the density update's stream: identical draws on every rank for a step,
        # different draws for different steps
        g5 = rdist.step_generator("cpu", 7, 5)
        draw = torch.randint(128, (64, 3), generator=g5)
        other = torch.randint(128, (64, 3), generator=rdist.step_generator("cpu", 7, 6))
        got = [torch.zeros_like(draw) for _ in range(world)]
        dist.all_gather(got, draw)
        ok_stream = all(torch.equal(x, draw) for x in got) and not torch.equal(draw, other)
        # bucketed all-reduce with the optimizer as its epilogue: every element
        # updated exactly once, from its bucket's averaged gradient (scale 1)
        params2 = [torch.zeros(1000), torch.zeros(37), torch.zeros(5)]
        ar2 = rdist.GradAllReduce(params2, "cpu")
        for p_, v in zip(params2, ar2.views):
            p_.grad = v
        for i, v in enumerate(ar2.views):
            v.copy_(torch.arange(v.numel(), dtype=torch.float32) * (rank + 1) + i)
        opt = _RecordingOpt()
        ar2.reduce_and_step(opt, n_buckets=4)
        ok_epi = opt.began and opt.ended and len(opt.calls) > 3
        for p_, v in zip(params2, ar2.views):
            seen = torch.zeros(p_.numel())
            for q_, lo_, hi_, sc in opt.calls:
                if q_ is p_:
                    seen[lo_:hi_] += 1
                    ok_epi = ok_epi and sc == 1.0
                    # the bucket's mean had landed when its update was queued
                    ok_epi = ok_epi and torch.equal(opt.snap[(id(q_), lo_)], v[lo_:hi_])
            ok_epi = ok_epi and bool((seen == 1).all())
        # the views hold the mean, as after reduce()
        for i, v in enumerate(ar2.views):
            ok_epi = ok_epi and torch.equal(v, torch.arange(v.numel(), dtype=torch.float32) * mf + i)
        # a .grad rebound away from the flat buffer is refused
        params2[1].grad = torch.zeros(37)
        try:
            ar2.reduce_and_step(opt)
            ok_epi = False
        except RuntimeError:
            pass
        ok_sched = True
        if sched is not None:
            ok_sched = _step_schedule(rank, world, *sched)
        q.put((rank, lo, hi, ok_mean, ok_bcast and ok_stream and ok_epi and ok_sched,
               (ok_bcast, ok_stream, ok_epi, ok_sched)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e), False, False))


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0][1:3] == (0, 500) and res[1][1:3] == (500, 1000), res
    assert all(r[3] for r in res), res
    assert all(r[4] for r in res), res


def test_gloo_world4_c4():
    """C4's rank count (bicycle, K = 4, scale 16, 4 GPUs): 4 gloo ranks run the
    same flat reduction, broadcast, seeded stream and Adam epilogue as the
    world-2 test, plus the headline step's bucket schedule at C4's gradient
    shapes (54.5 MB grid): buckets tile the buffer, mean bit-identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 4, port, q, (16.0, 4, 4, 8))) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1:3] for r in res] == [(0, 250), (250, 500), (500, 750), (750, 1000)], res
    assert all(r[3] for r in res), res
    assert all(r[4] for r in res), res


def _timeout_worker(rank, world, port, q):
    """rank 1 never joins the second collective: rank 0's bucket wait must fail
    within the bounded timeout, naming its rank and bucket."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        rdist.init(backend="gloo", timeout_s=3)
        ar = rdist.GradAllReduce([torch.ones(256)], "cpu")
        ar.reduce(n_buckets=2)                 # both ranks: fine
        if rank == 1:
            time.sleep(12)                     # misses the next collective
            q.put((rank, "slept", ""))
            return
        t0 = time.time()
        try:
            ar.reduce(n_buckets=2)
            q.put((rank, "no error", ""))
        except rdist.CollectiveTimeout as e:
            q.put((rank, f"{time.time() - t0:.1f}", str(e)))
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_collective_timeout_names_rank_and_bucket():
    """init_process_group gets a bounded timeout, and a
    hung bucket exits with the rank and bucket in the message instead of
    running to the driver's limit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    took, msg = res[0]
    assert took not in ("no error", "error"), res
    assert float(took) < 11, res
    assert msg.startswith("rank 0: all-reduce bucket 0 [0, ") and "of 256" in msg, msg


def test_collective_timeout_default(monkeypatch):
    monkeypatch.delenv("RADNERF_DIST_TIMEOUT", raising=False)
    assert rdist.collective_timeout().total_seconds() == rdist.DEFAULT_TIMEOUT_S
    monkeypatch.setenv("RADNERF_DIST_TIMEOUT", "42")
    assert rdist.collective_timeout().total_seconds() == 42
    assert rdist.collective_timeout(7).total_seconds() == 7


def test_single_process_noop():
    ar = rdist.GradAllReduce([torch.ones(3)], "cpu")
    ar.views[0].fill_(2.0)
    assert torch.equal(ar.reduce()[0], torch.full((3,), 2.0))
    assert rdist.shard_rays(10, 0, 1) == (0, 10)
    assert rdist.shard_rays(10, 2, 3) == (8, 10)


def test_bench_self_launch_gloo():
    """bench.py --gpus 2 with no torchrun environment starts 2 ranks itself
    (torch.distributed.run child process), checks the world size and reports
    the ranks it saw (--launch-check: no GPU work, gloo on CPU)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--backend", "gloo", "--launch-check"], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["backend"] == "gloo"
    assert sorted(r["rank"] for r in rec["ranks_seen"]) == [0, 1]
    # the N > 1 collective fields: the early MLP + gate
    # bucket and 4 grid buckets, timed, with the bytes each rank moves
    c = rec["comm"]
    # MLP + gate, the fine grid levels in 4 buckets, the coarse levels (VERDICT
    # r04 item 6): the same mean as one plain all-reduce, bit for bit
    assert c["mean_ok"] and c["buckets_per_step"] == 6 and c["allreduce_ms"] > 0
    assert c["mean_bit_identical"] and c["rank_consistent"]
    rg = c["ranges"]
    from radnerf_amd import layout as LY
    n = (2 * int(LY.grid_levels(0.5)["n_entries"]) + 2 * LY.FIELD_PARAMS + LY.gate_params(2)) * 4
    assert c["bytes_per_rank"] == n and c["ring_bytes_per_rank"] == n
    # the ranges tile the flat buffer; fine / coarse meet at level 8's start
    cut = 2 * int(LY.grid_levels(0.5)["offset"][8])
    assert rg["coarse"] == [0, cut] and rg["fine"][0] == cut
    assert rg["fine"][1] == rg["rest"][0] and rg["rest"][1] * 4 == n


def test_bench_self_launch_gloo_world8():
    """bench.py --gpus 8 --launch-check (the driver's 8-GPU launch, rehearsed
    with 8 gloo ranks on CPU): 8 ranks seen, the step's six buckets tile the
    C3 gradient, the mean agrees with one plain all-reduce and every rank
    holds the same bits; ring bytes = 2 (P-1)/P of the payload."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8",
                          "--backend", "gloo", "--launch-check"], env=env, capture_output=True,
                         text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 8 and rec["backend"] == "gloo"
    assert sorted(r["rank"] for r in rec["ranks_seen"]) == list(range(8))
    assert sorted(r["local_rank"] for r in rec["ranks_seen"]) == list(range(8))
    c = rec["comm"]
    assert c["mean_ok"] and c["rank_consistent"] and c["buckets_per_step"] == 6
    assert c["ring_bytes_per_rank"] == c["bytes_per_rank"] * 2 * 7 // 8


def test_bench_world_mismatch_fails():
    """A torchrun world that differs from --gpus exits non-zero."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node=2", "--master-addr=127.0.0.1",
                          f"--master-port={_free_port()}", os.path.join(root, "bench.py"),
                          "--gpus", "4", "--backend", "gloo", "--launch-check"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode != 0
    assert "--gpus 4 but the process group has 2" in out.stderr


def test_step_ranges_tile_the_buffer():
    """dist.step_ranges: MLP + gate, fine grid levels, coarse grid levels --
    disjoint, covering the flat buffer exactly, the cut on a level boundary
    (split 0: the whole grid in "fine")."""
    from radnerf_amd import layout as LY
    for scale in (0.5, 16.0):
        lv = LY.grid_levels(scale)
        n_grid = 2 * int(lv["n_entries"])
        ar = rdist.GradAllReduce([torch.zeros(n_grid), torch.zeros(3, LY.FIELD_PARAMS),
                                  torch.zeros(LY.gate_params(3))], "cpu")
        for split in (0, 1, 8, 15, 16, 99):
            rg = rdist.step_ranges(ar, lv["offset"], split)
            seen = torch.zeros(ar.flat.numel(), dtype=torch.int32)
            for a, b in rg.values():
                seen[a:b] += 1
            assert bool((seen == 1).all()), (scale, split)
            cut = min(split, 15)      # fused.clamp_split (16 released the grid early)
            assert rg["coarse"][1] == (2 * int(lv["offset"][cut]) if cut else 0)
            assert rg["fine"][1] > rg["fine"][0], (scale, split)


def test_clamp_split_matches_renderer():
    """The renderer's fold cut and dist.step_ranges use one clamp: a split of
    16 or more sums levels [15, 16) first, never an empty first range."""
    from radnerf_amd.fused import clamp_split
    assert [clamp_split(s) for s in (-3, 0, 1, 15, 16, 40)] == [0, 0, 1, 15, 15, 15]
