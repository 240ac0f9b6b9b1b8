"""GPU worker of tests/test_gpu_dist.py::test_rccl_calls_world1 (not a test
module): RCCL (backend "nccl") initialised with ONE rank on GPU 0 -- two RCCL
ranks cannot share a device, so this is the only RCCL process group a one-GPU
box can build.  It issues every collective the multi-GPU paths use, exactly
as they issue them: the bucketed asynchronous all-reduce of
dist.GradAllReduce (slices of the flat buffer, work.wait() then the division
on the compute stream), the pinned layout's all_gather_into_tensor
(pinned.all_gather_rows), bench.py's all_gather_object (ranks_seen), its
float64 MAX all-reduce of the elapsed time, and barrier; then bench.py's
N > 1 schedule through the renderer's hooks (dp_worker.hooked_split_schedule
at scale 16: the MLP + gate bucket after field_bwd, the fine levels after
their sum pass, the coarse ones after the backward), in the comm-stream form
RCCL takes, forced with one rank; rank 0 writes what it saw."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radnerf_amd import dist as rdist  # noqa: E402
from radnerf_amd.pinned import all_gather_rows  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))
from dp_worker import hooked_split_schedule  # noqa: E402


def main(out_path):
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    params = [torch.zeros(1_000_003, device=dev), torch.zeros(18_944, device=dev)]
    ar = rdist.GradAllReduce(params, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    ar.flat.copy_(torch.randn(ar.flat.numel(), device=dev, generator=g))
    ref = ar.flat.clone()
    for (a, b), w in ar._launch(4):          # the bucketed path of reduce()
        w.wait()
        ar.flat[a:b].div_(dist.get_world_size())
    torch.cuda.synchronize()
    res["bucketed_allreduce_equal"] = bool(torch.equal(ar.flat, ref))
    res["buckets"] = len(ar._ranges(4))
    rows = torch.arange(40, dtype=torch.float32, device=dev).view(4, 10)
    out = torch.empty(4, 10, device=dev)
    all_gather_rows(out, rows)
    res["all_gather_rows_equal"] = bool(torch.equal(out, rows))
    seen = [None]
    dist.all_gather_object(seen, {"rank": 0, "device": 0})
    res["all_gather_object"] = seen
    t = torch.tensor(1.25, device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res["max_f64"] = float(t)
    res["hooked"] = hooked_split_schedule(0, dev, stream_ordered=None, force=True)
    dist.barrier()
    torch.cuda.synchronize()
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
