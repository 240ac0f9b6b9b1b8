"""GPU: the ray-batch data-parallel step (radnerf_amd/dist.py, the path
bench.py --gpus N runs over RCCL) rehearsed with 2 ranks on one GPU over gloo:
the averaged flat gradient equals the average of the per-rank gradients
computed in one process (within 1e-4 of the largest entry: float-atomic
accumulation order differs)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_data_parallel_two_ranks_one_gpu(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path / "dp.json"
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   LOCAL_RANK=str(rank), WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dp_worker.py"),
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
    assert res["world"] == 2, res
    assert res["grid_rel"] <= 1e-4 and res["mlp_rel"] <= 1e-4 and res["gate_rel"] <= 1e-4, res
