"""Ray-batch data parallelism: one process per GPU, each rank
renders its own ray batch with full replicas of the hash grid, the K sub-NeRF
MLPs, the gate and all K occupancy bitfields; gradients are summed with one
RCCL all-reduce over xGMI per step (torch.distributed backend "nccl" = RCCL
on ROCm; "gloo" for the CPU tests).

The reference is single-GPU (train_ml.py:295-304); this is the build's
addition.  Bitfields must stay identical across ranks.  `update_density_grid`
keeps them so without a collective: every rank draws the update's cells and
jitter from a generator seeded by (seed, step), and the parameters are
identical after each step's all-reduce + Adam, so the deterministic density
kernel produces the same grids.  `broadcast_buffers` (rank 0's copy, C x 256
KiB per sub-NeRF) remains for callers that update with torch's default
stream.
"""
import datetime
import os

import torch
import torch.distributed as dist

# a collective that has not completed after this many seconds fails the rank
# (VERDICT r05 item 4): torch's default is 10 min for RCCL / 30 min for gloo,
# longer than the driver gives a bench run, so a hung all-reduce would run to
# the driver's limit instead of exiting non-zero.  RADNERF_DIST_TIMEOUT
# overrides it (seconds).
DEFAULT_TIMEOUT_S = 300


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def device_index(local):
    """GPU of this rank: LOCAL_RANK, unless RADNERF_DEVICE pins every rank to one
    GPU (rehearsing the multi-rank path on a one-GPU box with gloo)."""
    pinned = os.environ.get("RADNERF_DEVICE")
    return int(pinned) if pinned is not None else local


def collective_timeout(timeout_s=None):
    """The process group's collective timeout: timeout_s, else
    $RADNERF_DIST_TIMEOUT, else DEFAULT_TIMEOUT_S seconds."""
    if timeout_s is None:
        timeout_s = float(os.environ.get("RADNERF_DIST_TIMEOUT", DEFAULT_TIMEOUT_S))
    return datetime.timedelta(seconds=float(timeout_s))


def init(backend=None, timeout_s=None):
    """Initialise the default process group from the torchrun env (no-op for 1
    rank), with a bounded collective timeout (collective_timeout).  Under RCCL
    a collective past it is caught by torch's watchdog, which aborts the
    communicator and ends the rank non-zero with the operation's sequence
    number and size in its message (TORCH_NCCL_ASYNC_ERROR_HANDLING's default
    teardown); under gloo the wait raises, and GradAllReduce re-raises it with
    the rank and bucket (CollectiveTimeout)."""
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        timeout = collective_timeout(timeout_s)
        if backend == "nccl":
            dev = device_index(local)
            torch.cuda.set_device(dev)
            dist.init_process_group(backend, device_id=torch.device("cuda", dev), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
    return rank, local, world


class CollectiveTimeout(RuntimeError):
    """A bucket's collective failed or did not complete in time; the message
    names the rank, the bucket and its range of the flat buffer."""


def _wait(work, what):
    """work.wait(), re-raising a failure with the rank and bucket `what`."""
    try:
        work.wait()
    except Exception as e:
        rank = dist.get_rank() if dist.is_initialized() else 0
        raise CollectiveTimeout(f"rank {rank}: {what} did not complete "
                                f"({type(e).__name__}: {str(e)[:300]})") from e


def shard_rays(n_total, rank, world):
    """Contiguous ray range of this rank for a global batch of n_total rays."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return lo, min(lo + per, n_total)


class GradAllReduce:
    """Flat-buffer gradient all-reduce (mean over ranks).

    All gradient tensors are views of one contiguous fp32 buffer (45.7 MB
    hash-grid gradient + MLP/gate gradients at scale 0.5), reduced as a few
    large asynchronous bucket collectives instead of one per parameter: a
    few buckets keep every RCCL ring transfer large (xGMI is point-to-point,
    ~153 GB/s per link) while the averaging / Adam of the first buckets runs
    behind the last ones."""

    def __init__(self, params, device):
        self.params = list(params)
        self.timed = []                 # finished launch_range handles (comm_stats)
        sizes = [p.numel() for p in self.params]
        self.flat = torch.zeros(sum(sizes), device=device)
        self.views = []
        off = 0
        for p, n in zip(self.params, sizes):
            self.views.append(self.flat[off:off + n].view_as(p))
            off += n

    def zero(self):
        self.flat.zero_()

    def _ranges(self, n_buckets):
        """n_buckets contiguous [a, b) ranges of the flat buffer, 64-aligned."""
        n = self.flat.numel()
        n_buckets = max(1, int(n_buckets))
        bounds = sorted({min(n, (n * i // n_buckets + 63) // 64 * 64) for i in range(n_buckets)}
                        | {n})
        if bounds[0] != 0:
            bounds = [0] + bounds
        return list(zip(bounds[:-1], bounds[1:]))

    def _check_views(self):
        """Adam reads p.grad: it must still be this buffer's view, or the step
        would use the unreduced local gradient (ranks would diverge)."""
        for p, v in zip(self.params, self.views):
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                raise RuntimeError("GradAllReduce: a parameter's .grad was rebound away from "
                                   "the flat gradient buffer; assign p.grad = view again")

    def _launch(self, n_buckets):
        """Asynchronous SUM all-reduce of every bucket; [(range, work)]."""
        return [((a, b), dist.all_reduce(self.flat[a:b], async_op=True))
                for a, b in self._ranges(n_buckets)]

    # ---- staged launches with per-bucket timing (bench.py's comm fields) ----
    def param_range(self, first, last=None):
        """[a, b) of the flat buffer spanning params[first:last]."""
        sizes = [p.numel() for p in self.params]
        last = len(sizes) if last is None else last
        return sum(sizes[:first]), sum(sizes[:last])

    def launch_range(self, a, b, n_buckets=1, stream_ordered=None, force=False):
        """Start SUM all-reduces of flat[a:b] in n_buckets pieces as soon as the
        compute stream has produced them: on a comm stream that waits for the
        compute stream, bracketed by events there (CUDA), so the collectives
        overlap whatever the compute stream does next.  Returns a handle for
        finish(); a no-op with one rank unless `force` (a one-rank RCCL group:
        the only RCCL group a one-GPU box can build, tests/rccl_worker.py)."""
        if not (dist.is_initialized() and (dist.get_world_size() > 1 or force)):
            return None
        n = b - a
        n_buckets = max(1, min(int(n_buckets), max(1, n // 64)))
        bounds = [a + (n * i // n_buckets) // 64 * 64 for i in range(n_buckets)] + [b]
        # comm-stream events need a backend whose collectives are stream-ordered
        # (nccl = RCCL); gloo blocks the host in wait(), so its buckets are all
        # launched first and timed on the host (waiting per bucket serialised
        # them: the 2-rank gloo rehearsal ran 305 instead of ~21 ms per step)
        # (stream_ordered=True forces the comm-stream form on any backend: the
        # GPU test runs it over gloo, the only multi-rank backend of a 1-GPU box)
        if stream_ordered is None:
            stream_ordered = dist.get_backend() == "nccl"
        cuda = self.flat.is_cuda and bool(stream_ordered)
        handle = {"parts": [], "cuda": cuda}
        if cuda:
            main = torch.cuda.current_stream(self.flat.device)
            if getattr(self, "_comm", None) is None:
                self._comm = torch.cuda.Stream(self.flat.device)
            comm = self._comm
            comm.wait_stream(main)
            handle["stream"] = comm
            with torch.cuda.stream(comm):
                for lo, hi in zip(bounds[:-1], bounds[1:]):
                    if hi <= lo:
                        continue
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(comm)
                    w = dist.all_reduce(self.flat[lo:hi], async_op=True)
                    w.wait()                  # the comm stream waits for the collective
                    e1.record(comm)
                    handle["parts"].append(((lo, hi), e0, e1))
        else:
            import time
            for lo, hi in zip(bounds[:-1], bounds[1:]):
                if hi <= lo:
                    continue
                t0 = time.perf_counter()
                w = dist.all_reduce(self.flat[lo:hi], async_op=True)
                handle["parts"].append(((lo, hi), w, t0))
        return handle

    def finish(self, handle, average=True):
        """Join a launch_range handle into the compute stream and average."""
        if handle is None:
            return
        world = dist.get_world_size()
        if handle["cuda"]:
            torch.cuda.current_stream(self.flat.device).wait_stream(handle["stream"])
            parts = handle["parts"]
        else:
            import time
            parts = []
            for i, (rng, w, t0) in enumerate(handle["parts"]):
                _wait(w, f"all-reduce bucket {i} [{rng[0]}, {rng[1]}) of {self.flat.numel()}")
                parts.append((rng, t0, time.perf_counter()))
            handle["parts"] = parts
        if average:
            for (lo, hi), _, _ in parts:
                self.flat[lo:hi].div_(world)
        self.timed.append(handle)

    def comm_stats(self, steps):
        """Per-step collective figures of the handles finished since
        reset_timing(): allreduce_ms (sum of the buckets' durations on the
        comm stream; host-timed backends: first launch to last completion of
        each launch_range), buckets per step, bytes per rank (payload and a ring
        all-reduce's 2 (P-1)/P of it).  Synchronises."""
        world = dist.get_world_size() if dist.is_initialized() else 1
        tot, n_parts, payload = 0.0, 0, 0
        for h in self.timed:
            for (lo, hi), a, b in h["parts"]:
                if h["cuda"]:
                    a.synchronize(); b.synchronize()
                    tot += a.elapsed_time(b)
                n_parts += 1
                payload += (hi - lo) * self.flat.element_size()
            if not h["cuda"] and h["parts"]:
                # host-timed buckets are all in flight together: the span from
                # the first launch to the last completion
                tot += (max(b for _, _, b in h["parts"]) - min(a for _, a, _ in h["parts"])) * 1e3
        steps = max(1, int(steps))
        return {"allreduce_ms": round(tot / steps, 4), "buckets_per_step": n_parts / steps,
                "bytes_per_rank": int(payload / steps),
                "ring_bytes_per_rank": int(payload / steps * 2 * (world - 1) / max(world, 1))}

    def reset_timing(self):
        self.timed = []

    def reduce(self, average=True, n_buckets=1):
        """All-reduce the flat gradient as n_buckets asynchronous collectives;
        each bucket's division by the world size is queued behind its own
        work.wait() (it orders the compute stream after the collective
        without blocking the host).  After the call the views hold the mean
        over ranks (average) or the sum."""
        if dist.is_initialized() and dist.get_world_size() > 1:
            world = dist.get_world_size()
            for i, ((a, b), w) in enumerate(self._launch(n_buckets)):
                _wait(w, f"all-reduce bucket {i} [{a}, {b}) of {self.flat.numel()}")
                if average:
                    self.flat[a:b].div_(world)
        return self.views

    def reduce_and_step(self, opt, n_buckets=4, average=True):
        """All-reduce + FusedAdam with the optimizer as the collective's
        epilogue: the flat gradient goes out as
        n_buckets asynchronous all-reduces, and each bucket's averaging and
        Adam update are queued behind its own collective, so the updates of
        the first buckets run while the last ones are still on the wire.  The
        views are left holding what reduce() leaves (the mean over ranks with
        average, else the sum), so code reading the gradients afterwards
        (clipping, logging) sees the same values on either path.  One rank:
        opt.step()."""
        self._check_views()
        world = dist.get_world_size() if dist.is_initialized() else 1
        if world == 1:
            opt.step()
            return self.views
        works = self._launch(n_buckets)
        opt.begin_step()
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += p.numel()
        for i, ((a, b), w) in enumerate(works):
            _wait(w, f"all-reduce bucket {i} [{a}, {b}) of {self.flat.numel()} (Adam epilogue)")
            if average:
                self.flat[a:b].div_(world)
            for p, o in zip(self.params, offs):
                lo, hi = max(a, o), min(b, o + p.numel())
                if lo < hi:
                    opt.update_range(p, lo - o, hi - o, 1.0)
        opt.end_step()
        return self.views


def step_ranges(ar, level_offset, split_level):
    """The data-parallel step's collective schedule over a GradAllReduce of
    [grid, MLP, gate] (bench.py's headline step, N > 1), as [a, b) ranges of
    the flat buffer in launch order:
      "rest"   MLP + gate gradients, once field_bwd has written them;
      "fine"   the hash grid's levels [split_level, 16) -- the tail of the
               level-major table, the fine hashed levels -- once the fold has
               summed them (FusedMLRenderer.after_grid_levels), so their
               collective overlaps the coarse levels' sum pass;
      "coarse" levels [0, split_level) after the fold.
    split_level 0: "fine" is the whole grid and "coarse" empty.  The level
    is clamped to [0, 15] as the renderer clamps it (fused.clamp_split): a
    cut at 16 would release the grid before any level is summed.  The three
    ranges tile the flat buffer (tests/test_dist.py)."""
    from .fused import clamp_split
    split_level = clamp_split(split_level)
    g0, g1 = ar.param_range(0, 1)
    cut = g0 + 2 * int(level_offset[split_level]) if split_level > 0 else g0
    return {"rest": ar.param_range(1), "fine": (cut, g1), "coarse": (g0, cut)}


def broadcast_buffers(module, src=0):
    """Keep density grids / bitfields identical across ranks."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        for name, b in module.named_buffers():
            if "density" in name:
                dist.broadcast(b, src)


def step_generator(device, seed, step):
    """A generator on `device` seeded identically on every rank for `step`."""
    g = torch.Generator(device=device)
    g.manual_seed((int(seed) * 1000003 + int(step)) & 0x7FFFFFFFFFFFFFFF)
    return g


def update_density_grid(model, density_threshold, step, warmup=False, seed=0, decay=0.95):
    """train_ml.py:174-177 (model.update_density_grid every update_interval
    steps) made rank-consistent: the warm-up's jitter comes from
    step_generator(seed, step), the sampled update's cells and jitter from the
    device-side hash of the same (seed, step) -- identical on every rank."""
    if warmup:
        g = step_generator(model.mlp_params.device, seed, step)
        model.update_density_grid(density_threshold, warmup=True, decay=decay, generator=g)
    else:
        # device-side draws from a hash of (seed, step): the same on every rank
        model.update_density_grid(density_threshold, warmup=False, decay=decay,
                                  seed=(int(seed) * 1000003 + int(step)) & 0x7FFFFFFFFFFFFFFF)
