"""Shared GPU-test setup (not a test module): the synthetic model, gate and
workload of tests/test_gpu_ml.py, with an optional gate type."""
import torch

from radnerf_amd import layout as LY
from radnerf_amd import synthetic as S
from radnerf_amd.networks import MNGP, Ray_Gate


def setup_ml(cuda, B=384, K=2, scale=0.5, p=0.5, gate_type="ray"):
    m = MNGP(scale, size=K, seed=3)
    g = Ray_Gate(K, type=gate_type, seed=2)
    with torch.no_grad():
        m.xyz_encoder.params.copy_(torch.from_numpy(S.grid_params(m.xyz_encoder.n_entries)).view(-1))
        m.mlp_params.copy_(torch.from_numpy(S.mlp_params(K, LY.FIELD_PARAMS)))
        g.params.copy_(torch.from_numpy(S.mlp_params(1, LY.gate_params(K), seed=6)[0]))
        bits = S.bitfields(K, m.cascades, p=p)
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    m, g = m.to(cuda), g.to(cuda)
    o, d = S.rays(B, scale)
    noise = S.noise(K, B)
    seeds = S.loss_seeds(B, K)
    return m, g, o, d, noise, seeds, bits
