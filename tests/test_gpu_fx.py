"""Fixed-point accumulation of the grid gradient in the merged backward
(rn_field_bwd_merged fx_mode 2 + rn_grid_fx_fold + the fx_mode 3 redo).

* the hashed levels' gradients match the fp32-atomic backward of the same step
  per level (<= 1e-4 relative; the oracle bars are in test_gpu_ml.py);
* they are bitwise reproducible from step to step (exact integer sums);
* a scale too large for the step's records (forced here) sets the redo flag,
  and the fp32 redo yields the fp32 result; the next step is fixed point again;
* a non-finite seed propagates as in fp32 (redo).
"""
import numpy as np
import pytest
import torch

from radnerf_amd import layout as LY
from radnerf_amd.fused import get_renderer, ml_render_fused
from test_gpu_ml import _run, _setup, check_fx_vs_fp32

pytestmark = pytest.mark.gpu


def _hashed(scale):
    lv = LY.grid_levels(scale)
    return [l for l in range(16) if int(lv["res"][l]) ** 3 > int(lv["hsize"][l])], lv


def _level(g, lv, l):
    a, n = int(lv["offset"][l]), int(lv["hsize"][l])
    return g.view(-1, 2)[a:a + n]


@pytest.mark.parametrize("B,K,scale", [(2048, 2, 0.5), (1024, 4, 16.0)])
def test_fx_matches_fp32_and_is_reproducible(cuda, B, K, scale):
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_fx
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    _, gfx1 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    n_fx = check_fx_vs_fp32(m, gfx1, g32, r, f"B{B} K{K} s{scale}")
    hashed, lv = _hashed(scale)
    assert n_fx == len(hashed) > 0
    _, gfx2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    for l in hashed:        # exact integer sums: identical bits step to step
        assert torch.equal(_level(gfx1[0], lv, l), _level(gfx2[0], lv, l)), l
    acc = r.ws._fx[0]
    assert int(acc.abs().max()) == 0       # folded and re-zeroed


def test_fx_overflow_redo(cuda):
    B, K, scale = 1024, 2, 0.5
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    acc, scales, vmax, redo = r.ws._fx
    hashed, lv = _hashed(scale)
    # a scale 2^30 times too large: every level's records saturate the int32 range
    with torch.no_grad():
        cur = scales[r.ws.fx_i]
        cur[hashed] = cur[hashed] * 2.0 ** 30
    _, g_redo = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    assert int(redo[0]) == 1
    for l in range(16):
        a, b = _level(g_redo[0], lv, l), _level(g32[0], lv, l)
        assert float((a - b).norm() / b.norm().clamp_min(1e-30)) <= 1e-5, l   # fp32 order only
    for x, y in zip(g_redo[1:], g32[1:]):           # dW not added twice
        assert float((x - y).norm() / y.norm().clamp_min(1e-30)) <= 1e-5
    assert int(acc.abs().max()) == 0
    # the redo step measured the records again: the next step is fixed point
    _, gfx = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    assert int(redo[0]) == 0
    check_fx_vs_fp32(m, gfx, g32, r, "after redo")


def test_fx_nonfinite_seed_propagates(cuda):
    B, K = 512, 2
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K)
    r = get_renderer(m, g, B)
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)      # fp32 step: scales
    bad = [s.copy() for s in seeds]
    bad[0][7] = np.inf
    r.grid_fx = False                                                # fp32 reference
    _, gref = _run(ml_render_fused, m, g, o, d, noise, bad, cuda, 0.0)
    r.grid_fx = True
    _, gb = _run(ml_render_fused, m, g, o, d, noise, bad, cuda, 0.0)
    fin_ref, fin = torch.isfinite(gref[0]), torch.isfinite(gb[0])
    assert torch.equal(fin_ref, fin)
    if not bool(fin_ref.all()):
        assert int(r.ws._fx[3][0]) == 1                              # redone in fp32
