"""GPU: the sub-NeRF-per-GPU layout (radnerf_amd/pinned.py, SURVEY.md §8(e)
variant C5) against the single-process fused renderer on the same inputs.

Bars: the forward outputs (rgb, opacity, depth, gate) are bit-identical (each
sub-NeRF's samples are marched, evaluated and composited by the same
per-sample arithmetic, and the gated combine sees the same K rows); the
summed gradients match within 1e-4 of the largest entry (float-atomic
accumulation order differs); the sample totals are equal."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from radnerf_amd import synthetic as S
from radnerf_amd.fused import FusedMLRenderer
from radnerf_amd.networks import MNGP, Ray_Gate
from radnerf_amd.pinned import PinnedMLRenderer

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_pinned_single_rank_matches_fused(cuda):
    B, K = 1024, 2
    m = MNGP(0.5, size=K, seed=3).to(cuda)
    g = Ray_Gate(K, seed=4).to(cuda)
    bits = S.bitfields(K, m.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(cuda) for a in S.rays(B, 0.5, seed=0))
    nz = torch.from_numpy(S.noise(K, B, seed=2)).to(cuda)
    sd = [torch.from_numpy(s).to(cuda) for s in S.loss_seeds(B, K, seed=4)]
    bg = torch.ones(3, device=cuda)
    outs, grads = [], []
    for cls in (FusedMLRenderer, PinnedMLRenderer):
        r = cls(m, g, B)
        out = r.forward(o, d, d, nz, bg)
        outs.append([t.clone() for t in out[:4]])
        grads.append(r.backward(o, d, d, out[3], bg, *sd, None, 1e-4))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for a, b in zip(*grads):
        assert _rel(a, b) <= 1e-4


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("K,rays,scale", [(2, 2048, 0.5), (8, 1024, 16.0)])
def test_pinned_two_ranks_one_gpu(tmp_path, K, rays, scale):
    """2 ranks on one GPU over gloo (K/2 sub-NeRFs each; (8, 1024, 16) is config
    C5's layout: K = 8, scale 16, exp step): the all-gather of the per-ray
    outputs and the summed all-reduce reproduce the single-process result."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path / "pinned.json"
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   LOCAL_RANK=str(rank), WORLD_SIZE="2", PIN_K=str(K), PIN_RAYS=str(rays),
                   PIN_SCALE=str(scale))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "pinned_worker.py"),
                                       str(out)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), logs
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["samples"] == res["samples_ref"], res
    assert res["rgb_equal"] and res["opacity_equal"] and res["depth_equal"] and res["gate_equal"], res
    assert res["grid_rel"] <= 1e-4 and res["mlp_rel"] <= 1e-4 and res["gate_rel"] <= 1e-4, res
