"""CPU: checkpoint interchange with the reference's key names and tcnn flat
layouts (radnerf_amd/checkpoint.py).  The tcnn layout itself is "parity
unpinned" (tiny-cuda-nn is absent); these tests pin what can be pinned here:
sizes (11,264 field + 14,336 gate tcnn parameters), key names
(networks.py:214-289, 17-126, 1070-1085; utils/util.py:8-31), the round trip,
and that padded rows/columns are dropped."""
import numpy as np
import pytest
import torch

from radnerf_amd import checkpoint as C
from radnerf_amd import layout as LY
from radnerf_amd.networks import MNGP, NGP, Ray_Gate


def _rand_models(K=2, seed=0):
    m, g = MNGP(0.5, size=K, seed=seed), Ray_Gate(K, seed=seed + 1)
    with torch.no_grad():
        m.mlp_params.copy_(torch.randn_like(m.mlp_params).half().float())
        g.params.copy_(torch.randn_like(g.params).half().float())
        m.xyz_encoder.params.copy_(torch.randn_like(m.xyz_encoder.params).half().float())
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").random_(0, 256)
            getattr(m, f"density_grid_{i}").uniform_()
    return m, g


def test_tcnn_sizes_and_keys():
    m, g = _rand_models()
    sd = C.reference_state_dict(m, g)["state_dict"]
    assert sd["model.geo_net_0.params"].numel() + sd["model.rgb_net_0.params"].numel() == 11264
    assert sd["gating_net.encoder.params"].numel() == 14336
    for k in ("center", "xyz_min", "xyz_max", "half_size", "grid_coords", "density_bitfield_1",
              "density_grid_1", "xyz_encoder.params", "rgb_net_1.params"):
        assert "model." + k in sd
    assert sd["model.xyz_encoder.params"].dtype == torch.float16


def test_round_trip_exact():
    m, g = _rand_models(K=2, seed=3)
    ck = C.reference_state_dict(m, g)
    m2, g2 = MNGP(0.5, size=2, seed=9), Ray_Gate(2, seed=9)
    C.load_reference_state(m2, g2, state=ck)
    assert torch.equal(m2.mlp_params, m.mlp_params)
    assert torch.equal(g2.params, g.params)
    assert torch.equal(m2.xyz_encoder.params, m.xyz_encoder.params)
    for i in range(2):
        assert torch.equal(getattr(m2, f"density_bitfield_{i}"), getattr(m, f"density_bitfield_{i}"))
        assert torch.equal(getattr(m2, f"density_grid_{i}"), getattr(m, f"density_grid_{i}"))


def test_padding_dropped_and_rm_order():
    K = 2
    geo = torch.arange(4096, dtype=torch.float32)
    rgb = torch.arange(7168, dtype=torch.float32) + 10000
    flat = C._field_from_tcnn(geo, rgb)
    w = LY.split_field_params(flat)
    # first geo layer: row-major [64, 32]; W[o, i] = o*32 + i
    assert w["g1"][5, 7] == 5 * 32 + 7
    # second geo layer [32 (17 used), 64] starts at 2048
    assert w["g2"][16, 63] == 2048 + 16 * 64 + 63
    # rgb output layer [16 (3 used), 64] after 2048 + 4096
    assert w["r3"][2, 1] == 10000 + 6144 + 2 * 64 + 1
    gate = torch.arange(14336, dtype=torch.float32)
    gf = LY.split_gate_params(C._gate_from_tcnn(gate, K), K)
    assert gf["w0"][3, 5] == 3 * 16 + 5          # input padded 6 -> 16
    assert gf["w4"][1, 2] == 1024 + 3 * 4096 + 64 + 2


def test_ngp_names_and_lightning_wrapping():
    m = NGP(0.5, seed=1)
    with torch.no_grad():
        m.mlp_params.copy_(torch.randn_like(m.mlp_params).half().float())
    ck = C.reference_state_dict(m)
    sd = ck["state_dict"]
    assert "model.geo_net.params" in sd and "model.density_bitfield" in sd
    sd["model.val_lpips.x"] = torch.zeros(1)     # other Lightning keys are ignored
    sd["directions"] = torch.zeros(4, 3)
    m2 = NGP(0.5, seed=2)
    C.load_reference_state(m2, state=ck)
    assert torch.equal(m2.mlp_params, m.mlp_params)


def test_wrong_sizes_raise():
    m, g = _rand_models()
    ck = C.reference_state_dict(m, g)
    ck["state_dict"]["model.geo_net_0.params"] = torch.zeros(4000)
    with pytest.raises(ValueError, match="geo_net"):
        C.load_reference_state(MNGP(0.5, size=2), Ray_Gate(2), state=ck)
    ck = C.reference_state_dict(m, g)
    ck["state_dict"]["model.xyz_encoder.params"] = torch.zeros(10)
    with pytest.raises(ValueError, match="xyz_encoder"):
        C.load_reference_state(MNGP(0.5, size=2), state=ck)


def test_file_round_trip_weights_only(tmp_path):
    m, g = _rand_models(K=2, seed=5)
    f = tmp_path / "ck.ckpt"
    torch.save(C.reference_state_dict(m, g), f)
    m2, g2 = MNGP(0.5, size=2), Ray_Gate(2)
    C.load_reference_state(m2, g2, path=str(f))
    assert torch.equal(m2.mlp_params, m.mlp_params) and torch.equal(g2.params, g.params)
