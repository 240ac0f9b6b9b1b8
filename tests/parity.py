"""Gradient-parity bars shared by the GPU tests: relative L2 error per
hash-grid level (16) and per MLP layer of every sub-NeRF (g1 g2 r1 r2 r3),
each against the fp32 oracle.  The bounds are about 2x the largest value
measured on the test workloads (printed by every test that uses them; see
DESIGN.md §2).  Whole-tensor norms could hide a dropped corner or a wrong fine
level; these cannot."""
import numpy as np

from radnerf_amd import layout as LY

GRID_LEVEL_TOL = 3e-3      # measured <= 1.5e-3 (scale 16, K = 4)
MLP_LAYER_TOL = 4e-3       # measured <= 1.7e-3
GATE_TOL = 2e-3            # measured <= 9e-4
LAYERS = {"g1": (0, 2048), "g2": (2048, 3136), "r1": (3136, 5184), "r2": (5184, 9280),
          "r3": (9280, 9472)}


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def check_grads(scale, grid, grid_ref, mlp, mlp_ref, gate=None, gate_ref=None, tag="",
                grid_tol=GRID_LEVEL_TOL, mlp_tol=MLP_LAYER_TOL, gate_tol=GATE_TOL):
    """grid (entries, 2), mlp (K, 9472) numpy; returns (levels, layers, gate)."""
    lv = LY.grid_levels(scale)
    grid, grid_ref = np.asarray(grid).reshape(-1, 2), np.asarray(grid_ref).reshape(-1, 2)
    lvl = []
    for l in range(16):
        a, n = int(lv["offset"][l]), int(lv["hsize"][l])
        lvl.append(rel(grid[a:a + n], grid_ref[a:a + n]))
    mlp, mlp_ref = np.atleast_2d(mlp), np.atleast_2d(mlp_ref)
    lay = {(k, name): rel(mlp[k, a:b], mlp_ref[k, a:b]) for k in range(mlp.shape[0])
           for name, (a, b) in LAYERS.items() if np.abs(mlp_ref[k, a:b]).max() > 0}
    ga = None if gate is None else rel(gate, gate_ref)
    print(f"{tag}: grid per level max {max(lvl):.2e} {['%.1e' % v for v in lvl]}")
    print(f"{tag}: mlp per layer max {max(lay.values()):.2e}"
          + ("" if ga is None else f" gate {ga:.2e}"))
    assert max(lvl) <= grid_tol, lvl
    assert max(lay.values()) <= mlp_tol, lay
    if ga is not None:
        assert ga <= gate_tol, ga
    return lvl, lay, ga
