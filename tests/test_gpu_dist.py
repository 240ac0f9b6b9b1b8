"""GPU: the ray-batch data-parallel step (radnerf_amd/dist.py, the path
bench.py --gpus N runs over RCCL) rehearsed with 2 ranks on one GPU over gloo:
the averaged flat gradient equals the average of the per-rank gradients
computed in one process (within 1e-4 of the largest entry: float-atomic
accumulation order differs); and multi-step training (radnerf_amd.trainer)
keeps every rank's parameters, density grids and bitfields bit-identical."""
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


def _run_ranks(worker, out, timeout=100, extra=()):
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   LOCAL_RANK=str(rank), WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", worker),
                                       str(out), *extra], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), logs
    return json.loads(out.read_text())


def test_data_parallel_two_ranks_one_gpu(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks("dp_worker.py", tmp_path / "dp.json")
    assert res["world"] == 2, res
    assert res["grid_rel"] <= 1e-4 and res["mlp_rel"] <= 1e-4 and res["gate_rel"] <= 1e-4, res
    # the comm-stream staged all-reduce (bench.py's N > 1 form over RCCL), forced over gloo
    assert res["staged_cuda"] and res["staged_equal"], res
    # the renderer's hooks at scale 16: MLP + gate, fine levels after their
    # sum pass, coarse levels after the backward -- the plain mean, bit for bit
    hk = res["hooked"]
    assert hk["equal"] and hk["finite"] and hk["nonzero"], hk
    assert hk["covered_once"] and hk["n_ranges"] == 3, hk
    assert hk["splits"] == [8, 8, 8] and hk["redo"] == 0 and hk["pages"] > 0, hk
    st = res["staged_stats"]
    assert st["buckets_per_step"] == 5 and st["allreduce_ms"] > 0, st
    assert st["bytes_per_rank"] == 4 * res["n_flat"], st


def test_data_parallel_training_stays_identical(tmp_path):
    """radnerf_amd.trainer.Trainer on 2 ranks (one GPU, gloo): 14 steps with
    density-grid updates every 4 steps (warm-up over every cell, then sampled
    cells), the fused loss, the flat all-reduce and Adam.  Each rank trains on
    its own rays; parameters, density grids and bitfields stay bit-identical
    across the ranks (rank-consistent update stream, no broadcast), and the
    updates do change the bitfields."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks("train_worker.py", tmp_path / "train.json", timeout=110)
    print(res)
    assert res["world"] == 2
    assert all(res["identical"].values()), res["identical"]
    assert all(res["bitfields_changed"]), res
    assert res["finite"]


def test_data_parallel_training_stays_identical_binned(tmp_path):
    """The same at scale 16, where the grid gradient goes through the binned
    scatter (page stores, bin + exact int64 sums): the ranks' parameters,
    grids and bitfields stay bit-identical over 14 Adam steps."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks("train_worker.py", tmp_path / "train16.json", timeout=110, extra=("16",))
    print({k: v for k, v in res.items() if k != "losses"})
    assert res["world"] == 2 and res["grid_bin"] and res["bin_pages"] > 0, res
    assert all(res["identical"].values()), res["identical"]
    assert res["finite"]


def test_bucketed_adam_epilogue_matches_plain(tmp_path):
    """GradAllReduce.reduce_and_step (4 asynchronous all-reduce buckets, each
    bucket's division by the world size and FusedAdam update queued behind its
    collective) vs reduce() (one collective + division) + FusedAdam.step(),
    on identical per-rank gradients, 3 steps, buckets cutting across
    parameters: bit-identical parameters and moments on both ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks("adam_worker.py", tmp_path / "adam.json", timeout=100)
    assert res["world"] == 2
    assert res["same_params"] and res["same_moments"] and res["ranks_agree"], res


def test_rccl_calls_world1(tmp_path):
    """Every collective of the multi-GPU paths, issued through RCCL as they
    issue it, in a one-rank RCCL group on GPU 0 (tests/rccl_worker.py): the
    calls are legal for the backend (async bucket slices, tensor and object
    all-gathers, f64 MAX, barrier) and leave the data as expected; and the
    renderer's hook schedule (bench.py's early MLP + gate bucket and the split
    grid ranges) runs on RCCL's comm-stream path."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path / "rccl.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), str(out)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "nccl"
    assert res["bucketed_allreduce_equal"] and res["buckets"] == 4
    assert res["all_gather_rows_equal"]
    assert res["all_gather_object"] == [{"rank": 0, "device": 0}]
    assert res["max_f64"] == 1.25
    # the renderer's hook schedule over RCCL (comm stream, events): every range
    # once, the sum over one rank = the local values, bit for bit
    hk = res["hooked"]
    assert hk["equal"] and hk["finite"] and hk["nonzero"], hk
    assert hk["covered_once"] and hk["n_ranges"] == 3 and all(hk["cuda"]), hk
    assert hk["splits"] == [8, 8, 8] and hk["redo"] == 0 and hk["pages"] > 0, hk
