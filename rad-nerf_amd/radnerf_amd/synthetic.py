"""Seeded synthetic inputs of SURVEY.md §8(d) (numpy, so the CPU oracle and the
GPU path see bit-identical data):  rays seed 0, occupancy seed 1, jitter seed 2,
parameters seed 3 (module init), loss seeds seed 4."""
import numpy as np


def rays(n, scale=0.5, seed=0):
    """rays_o = R*u (u uniform on S^2, R = 3*scale), rays_d = normalize(p - rays_o),
    p ~ U([-0.8*scale, 0.8*scale]^3)."""
    rng = np.random.default_rng(seed)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = (3.0 * scale * u).astype(np.float32)
    p = rng.uniform(-0.8 * scale, 0.8 * scale, size=(n, 3))
    d = p - o
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    return np.ascontiguousarray(o), np.ascontiguousarray(d)


def bitfields(n_models, cascades, p=0.5, seed=1, grid_size=128):
    """Independent Bernoulli(p) occupancy per cell, per model and cascade."""
    rng = np.random.default_rng(seed)
    n_cells = cascades * grid_size ** 3
    occ = rng.random((n_models, n_cells)) < p
    return np.packbits(occ.reshape(n_models, -1, 8), axis=-1, bitorder="little").reshape(
        n_models, n_cells // 8)


def noise(n_models, n_rays, seed=2):
    return np.random.default_rng(seed).random((n_models, n_rays), dtype=np.float32)


def loss_seeds(n_rays, n_models, seed=4, std=1e-3):
    rng = np.random.default_rng(seed)
    return (rng.normal(0, std, (n_rays, 3)).astype(np.float32),
            rng.normal(0, std, n_rays).astype(np.float32),
            rng.normal(0, std, (n_rays, n_models)).astype(np.float32))


def grid_params(n_entries, seed=3, amp=1e-1):
    """Hash-table values.  tcnn initialises U(-1e-4, 1e-4); parity tests use a
    larger amplitude so the field is far from trivial."""
    return np.random.default_rng(seed).uniform(-amp, amp, (n_entries, 2)).astype(np.float32)


def mlp_params(n_models, n_params, seed=5, scale=0.3):
    return np.random.default_rng(seed).uniform(-scale, scale, (n_models, n_params)).astype(
        np.float32)
