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


def _worker(rank, world, port, q):
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
        ok_mean = all(torch.allclose(v, torch.full_like(v, 1.5 * (i + 1)))
                      for i, v in enumerate(views))
        # the same as 3 asynchronous buckets (bench.py's headline N>1 step)
        for i, v in enumerate(ar.views):
            v.copy_(torch.arange(v.numel(), dtype=torch.float32).view_as(v) * (rank + 1) + i)
        views = ar.reduce(n_buckets=3)
        ok_mean = ok_mean and all(
            torch.allclose(v, (torch.arange(v.numel(), dtype=torch.float32).view_as(v) * 1.5 + i))
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
            ok_epi = ok_epi and torch.equal(v, torch.arange(v.numel(), dtype=torch.float32) * 1.5 + i)
        # a .grad rebound away from the flat buffer is refused
        params2[1].grad = torch.zeros(37)
        try:
            ar2.reduce_and_step(opt)
            ok_epi = False
        except RuntimeError:
            pass
        q.put((rank, lo, hi, ok_mean, ok_bcast and ok_stream and ok_epi))
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
    rg = c["ranges"]
    from radnerf_amd import layout as LY
    n = (2 * int(LY.grid_levels(0.5)["n_entries"]) + 2 * LY.FIELD_PARAMS + LY.gate_params(2)) * 4
    assert c["bytes_per_rank"] == n and c["ring_bytes_per_rank"] == n
    # the ranges tile the flat buffer; fine / coarse meet at level 8's start
    cut = 2 * int(LY.grid_levels(0.5)["offset"][8])
    assert rg["coarse"] == [0, cut] and rg["fine"][0] == cut
    assert rg["fine"][1] == rg["rest"][0] and rg["rest"][1] * 4 == n


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
        for split in (0, 1, 8, 15):
            rg = rdist.step_ranges(ar, lv["offset"], split)
            seen = torch.zeros(ar.flat.numel(), dtype=torch.int32)
            for a, b in rg.values():
                seen[a:b] += 1
            assert bool((seen == 1).all()), (scale, split)
            assert rg["coarse"][1] == (2 * int(lv["offset"][split]) if split else 0)
