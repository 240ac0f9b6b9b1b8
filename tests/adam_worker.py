"""GPU worker of tests/test_gpu_dist.py::test_bucketed_adam_epilogue_matches_plain
(not a test module): 2 ranks on ONE GPU over gloo.  Two copies of the same
parameters get the same per-rank gradients; one copy steps through
GradAllReduce.reduce_and_step (bucketed all-reduce, Adam as its epilogue), the
other through reduce() + FusedAdam.step(); rank 0 writes whether they agree."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radnerf_amd import dist as rdist  # noqa: E402
from radnerf_amd.optim import FusedAdam  # noqa: E402


def main(out_path):
    rank, _, world = rdist.init(backend="gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    sizes = (1_000_003, 18_944, 1_234)            # bucket bounds fall inside the first
    g0 = torch.Generator().manual_seed(11)
    init = [torch.randn(n, generator=g0) for n in sizes]
    sets = []
    for _ in range(2):
        ps = [x.clone().to(dev) for x in init]
        ar = rdist.GradAllReduce(ps, dev)
        for p, v in zip(ps, ar.views):
            p.grad = v
        sets.append((ps, ar, FusedAdam(ps, lr=1e-2, eps=1e-15)))
    gr = torch.Generator().manual_seed(100 + rank)
    for step in range(3):
        grads = [torch.randn(n, generator=gr).to(dev) * 1e-3 for n in sizes]
        for ps, ar, _ in sets:
            for v, g in zip(ar.views, grads):
                v.copy_(g)
        (ps_a, ar_a, opt_a), (ps_b, ar_b, opt_b) = sets
        ar_a.reduce_and_step(opt_a, n_buckets=4)
        ar_b.reduce()
        opt_b.step()
    torch.cuda.synchronize()
    (ps_a, _, opt_a), (ps_b, _, opt_b) = sets
    same_p = all(torch.equal(a, b) for a, b in zip(ps_a, ps_b))
    same_m = all(torch.equal(opt_a.state[a]["exp_avg"], opt_b.state[b]["exp_avg"]) and
                 torch.equal(opt_a.state[a]["exp_avg_sq"], opt_b.state[b]["exp_avg_sq"])
                 for a, b in zip(ps_a, ps_b))
    mine = hashlib.sha256(b"".join(p.cpu().numpy().tobytes() for p in ps_a)).hexdigest()
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"world": world, "same_params": same_p, "same_moments": same_m,
                       "ranks_agree": all(a == mine for a in allr)}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
