"""CPU: the sub-NeRF-per-GPU layout (radnerf_amd/pinned.py, SURVEY.md §8(e)
variant C5) -- model ranges, the ModelSlice view, and the per-ray output
exchange + gradient-sum semantics on a 2-rank gloo group (the same
collective code the RCCL run uses; no kernel is launched)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from radnerf_amd import dist as rdist
from radnerf_amd.networks import MNGP, Ray_Gate
from radnerf_amd.pinned import ModelSlice, PinnedMLRenderer, owned_range


def test_owned_range():
    assert [owned_range(8, r, 8) for r in range(8)] == [(r, r + 1) for r in range(8)]
    assert [owned_range(4, r, 2) for r in range(2)] == [(0, 2), (2, 4)]
    assert owned_range(2, 0, 1) == (0, 2)
    with pytest.raises(ValueError, match="multiple"):
        owned_range(6, 0, 4)


def test_model_slice_views():
    m = MNGP(0.5, size=4, seed=3)
    s = ModelSlice(m, 1, 3)
    assert s.size == 2
    assert s.density_bitfield_0 is m.density_bitfield_1
    assert s.density_bitfield_1 is m.density_bitfield_2
    assert s.density_grid_1 is m.density_grid_2
    assert s.mlp_params.data_ptr() == m.mlp_params[1].data_ptr()
    assert s.mlp_params.shape == (2, m.mlp_params.shape[1])
    assert s.xyz_encoder is m.xyz_encoder and s.center is m.center
    assert s.cascades == m.cascades and s.scale == m.scale
    with pytest.raises(ValueError):
        ModelSlice(m, 3, 5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, K=4, scale=0.5):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        torch.set_num_threads(1)
        rdist.init(backend="gloo")
        B = 16
        m = MNGP(scale, size=K, seed=3)
        g = Ray_Gate(K, seed=4)
        r = PinnedMLRenderer(m, g, B, device=torch.device("cpu"))
        k0, k1 = r.k0, r.k1
        # what this rank rendered: sub-NeRF k, ray b -> recognisable values
        kk = torch.arange(k0, k1, dtype=torch.float32)[:, None]
        bb = torch.arange(B, dtype=torch.float32)[None, :]
        r.ws.opacity_k.copy_(kk * 100 + bb)
        r.ws.depth_k.copy_(-(kk * 100 + bb))
        r.ws.rgb_k.copy_((kk * 100 + bb)[..., None] + torch.tensor([0.1, 0.2, 0.3]))
        op, dp, rgb = r._gather_model_outputs()
        ok_cached = all(a is b for a, b in zip((op, dp, rgb), r._model_outputs()))
        KA = torch.arange(K, dtype=torch.float32)[:, None]
        ok_gather = (torch.equal(op, KA * 100 + bb) and torch.equal(dp, -(KA * 100 + bb))
                     and torch.allclose(rgb, (KA * 100 + bb)[..., None]
                                        + torch.tensor([0.1, 0.2, 0.3])))
        # (B, K) per-ray tensors: this rank's columns
        gate = torch.arange(B * K, dtype=torch.float32).view(B, K)
        ok_cols = torch.equal(r._local_cols(gate), gate[:, k0:k1]) and ok_cached
        # gradient sum: grid partials add, MLP rows only on their owner, gate on rank 0
        ar = rdist.GradAllReduce([m.xyz_encoder.params, m.mlp_params, g.params], "cpu")
        ar.views[0].fill_(1.0)
        ar.views[1][k0:k1].fill_(float(rank + 1))
        if r.gate_grad_here:
            ar.views[2].fill_(7.0)
        grid, mlp, gp = ar.reduce(average=False)
        ok_sum = (bool((grid == world).all()) and bool((gp == 7.0).all())
                  and all(bool((mlp[k] == k // (K // world) + 1).all()) for k in range(K)))
        q.put((rank, (k0, k1), ok_gather, ok_cols, ok_sum, r.gate_grad_here))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e), False, False, False))


def test_pinned_exchange_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res[0][1] == (0, 2) and res[1][1] == (2, 4), res
    assert all(r[2] and r[3] and r[4] for r in res), res
    assert [r[5] for r in res] == [True, False], res


def test_pinned_exchange_gloo_world8_c5():
    """C5's layout (Free / road, K = 8 on 8 GPUs, scale 16): 8 gloo ranks, one
    sub-NeRF each -- every rank gathers all 8 sub-NeRFs' per-ray outputs in
    model order, takes its own (B, 1) gate column, the grid partials sum over
    the 8 ranks, each MLP row comes from its owner only and the gate gradient
    from rank 0 only."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 8, port, q, 8, 16.0)) for r in range(8)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [(k, k + 1) for k in range(8)], res
    assert all(r[2] and r[3] and r[4] for r in res), res
    assert [r[5] for r in res] == [True] + [False] * 7, res
