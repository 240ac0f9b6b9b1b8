"""GPU worker of tests/test_gpu_pinned.py (not a test module): one rank of a
sub-NeRF-per-GPU step (radnerf_amd/pinned.py) rehearsed on ONE GPU over a
gloo group; rank 0 also runs the single-process FusedMLRenderer on the same
inputs and writes the comparison to the JSON path in argv[1]."""
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
from radnerf_amd.pinned import PinnedMLRenderer  # noqa: E402


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def main(out_path):
    rank, _, world = rdist.init(backend="gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    B, K = int(os.environ.get("PIN_RAYS", 2048)), int(os.environ.get("PIN_K", 2))
    scale = float(os.environ.get("PIN_SCALE", 0.5))
    esf = 1 / 256 if scale > 0.5 else 0.0
    model = MNGP(scale, size=K, seed=3).to(dev)
    gate = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, model.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(model, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=0))
    noise = torch.from_numpy(S.noise(K, B, seed=2)).to(dev)
    g_rgb, g_op, g_depth = (torch.from_numpy(s).to(dev) for s in S.loss_seeds(B, K, seed=4))
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)

    r = PinnedMLRenderer(model, gate, B)
    ar = rdist.GradAllReduce([model.xyz_encoder.params, model.mlp_params, gate.params], dev)
    ar.zero()
    rgb, op, depth, g_out, imp = r.forward(o, d, d, noise, bg, 1e-4, esf)
    n = r.ws.meta[1].to(torch.int64).clone()
    r.backward(o, d, d, g_out, bg, g_rgb, g_op, g_depth, None, 1e-4,
               grid_grad=ar.views[0], mlp_grad=ar.views[1], gate_grad=ar.views[2])
    ar.reduce(average=False)
    dist.all_reduce(n)
    torch.cuda.synchronize()
    if rank == 0:
        ref = FusedMLRenderer(model, gate, B)
        rgb_r, op_r, depth_r, g_r, _ = ref.forward(o, d, d, noise, bg, 1e-4, esf)
        gg, mg, ag = ref.backward(o, d, d, g_r, bg, g_rgb, g_op, g_depth, None, 1e-4)
        torch.cuda.synchronize()
        res = {"world": world, "samples": int(n), "samples_ref": int(ref.ws.meta[1]),
               "rgb_equal": bool(torch.equal(rgb, rgb_r)),
               "opacity_equal": bool(torch.equal(op, op_r)),
               "depth_equal": bool(torch.equal(depth, depth_r)),
               "gate_equal": bool(torch.equal(g_out, g_r)),
               "grid_rel": rel(ar.views[0], gg), "mlp_rel": rel(ar.views[1], mg),
               "gate_rel": rel(ar.views[2], ag)}
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
