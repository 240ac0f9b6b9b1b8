"""Fixed-point accumulation of the grid gradient in the merged backward
(rn_field_bwd_merged fx_mode 2 + rn_grid_fx_fold + the fx_mode 3 redo).

* every level's gradient (hashed and, from their second step, dense) matches
  the fp32-atomic backward of the same step per level (<= 3e-4 relative; the
  oracle bars are in test_gpu_ml.py);
* they are bitwise reproducible from step to step (exact integer sums);
* a scale too large for the step's records (forced here) sets the redo flag,
  and the fp32 redo yields the fp32 result; the next step is fixed point again;
* a non-finite seed propagates as in fp32 (redo);
* an int32 entry that wraps (many same-sign records, no growth of the
  largest record) is caught by the per-level record-sum / entry-sum check.
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
    r.bin_f32_levels = 0          # (scale 16: every level fixed point, binned)
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    _, gfx1 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    n_fx = check_fx_vs_fp32(m, gfx1, g32, r, f"B{B} K{K} s{scale}")
    hashed, lv = _hashed(scale)
    # every level: the hashed ones at the record scale, the dense ones capped
    # by their largest entry (read from the first step's fp32 gradient)
    assert n_fx == 16 and len(hashed) > 0
    # from the next step on the entry cap comes from the fixed-point entries:
    # steps 3 and 4 (identical inputs) use identical scales everywhere
    _, gfx2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    check_fx_vs_fp32(m, gfx2, g32, r, f"B{B} K{K} s{scale} step 3")
    _, gfx3 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    for l in range(16):     # exact integer sums: identical bits step to step
        assert torch.equal(_level(gfx2[0], lv, l), _level(gfx3[0], lv, l)), l
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
    r.grid_fx = True                 # (512 rays x 2: fp32 by the renderer's own choice)
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


def test_fx_entry_wrap_sets_redo(cuda):
    """an int32 entry can wrap with every record under the 2^28-
    unit growth bound when many same-sign records land on it.  Here all 8192
    rays are the same ray (K = 2) with positive seeds: the coarse hashed
    levels' entries take ~16k records each.  The measured scale keeps the
    largest entry under 2^28 units; the step runs at 16x that scale, so the
    entries pass 2^31 while every record (~2^-14 of its entry) stays far
    below the 2^28-unit growth bound (the vmax check does not fire).  The
    level's exact entry sum then differs from its record sum by a multiple of
    2^32, the redo flag is set, and the result is the fp32 one."""
    B, K = 8192, 2
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K)
    o = np.repeat(o[:1], B, 0)
    d = np.repeat(d[:1], B, 0)
    seeds = tuple(np.abs(s).astype(np.float32) for s in seeds)
    r = get_renderer(m, g, B)
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)       # fp32: scales
    acc, scales, stats, redo = r.ws._fx
    cur = scales[r.ws.fx_i]
    hashed, lv = _hashed(0.5)
    # the measured scale maps the largest entry below 2^28 units; 16x pushes
    # the entries past 2^31 while the records (each a small part of its
    # entry) stay far below the 2^28-unit growth bound
    f = 16.0
    g_e = g32[0].view(-1, 2)
    units = {l: float(_level(g_e, lv, l).abs().max()) * float(cur[l]) * f for l in hashed}
    # the test's premise: some entry's exact integer sum exceeds the int32 range
    over = [l for l in hashed if units[l] > 2.0 ** 31]
    assert over, {l: f"{u:.3g}" for l, u in units.items()}
    with torch.no_grad():
        cur[hashed] = cur[hashed] * f
    _, gfx = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    assert int(redo[0]) == 1
    for l in range(16):
        a, b = _level(gfx[0], lv, l), _level(g32[0], lv, l)
        assert float((a - b).norm() / b.norm().clamp_min(1e-30)) <= 1e-5, l
    assert int(acc.abs().max()) == 0
    # statistics cleared for the next step
    assert int(stats.abs().max()) == 0


# (B, K, scale): C3's shape (int32 fixed point, atomics), C4's branch (K = 4,
# scale 16, exponential steps) and a C5-shaped one (K = 8, scale 16), both on
# the binned scatter (the default at scale 16)
# (B, K, scale, fp32 levels, bar on the 3-step Adam difference per level):
# the int32 form at C3 measured 1.14 % with round 6's units (2.66 % before),
# 0.3 % with levels 3-8 on fp32 atomics (fx_f32_levels); e5m17 0.25 %
PER_ENTRY_SHAPES = [(2048, 2, 0.5, (), 0.02), (2048, 2, 0.5, (3, 4, 5, 6, 7, 8), 0.005),
                    (4096, 4, 16.0, (), 0.01), (2048, 8, 16.0, (), 0.01)]


@pytest.mark.parametrize("B,K,scale,f32_levels,bar", PER_ENTRY_SHAPES)
def test_fx_per_entry_agreement(cuda, capsys, B, K, scale, f32_levels, bar):
    """fixed point per ENTRY, not only per-level norms.  One
    step fixed point vs fp32 over every level: the share of entries non-zero
    in fp32 but zero in fixed point, and the sign agreement of the entries
    whose fp32 gradient is above the level's fixed-point unit (1 / 2^e_l);
    then 3 FusedAdam steps (eps 1e-15, as train_ml.py) from the same start
    with either gradient: the parameter updates per level.  The measured
    values are printed (DESIGN.md §2 quotes them); the bars hold what a
    per-entry deviation may not exceed."""
    from radnerf_amd.optim import FusedAdam
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_fx and r.grid_bin == (scale > 0.5)
    r.fx_f32_levels = f32_levels
    lv = LY.grid_levels(scale)
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)              # scales
    unit = (1.0 / r.ws._fx[1][r.ws.fx_i].abs().clamp_min(1e-30)).cpu()
    _, gfx = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    assert int(r.ws._fx[3][0]) == 0                                         # no redo
    r.grid_fx = False
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.grid_fx = True
    a_all, b_all = gfx[0].view(-1, 2), g32[0].view(-1, 2)
    lost, n_nz, agree, n_big = 0, 0, 0, 0
    for l in range(16):
        a, b = _level(a_all, lv, l), _level(b_all, lv, l)
        nz = b != 0
        n_nz += int(nz.sum())
        lost += int((nz & (a == 0)).sum())
        big = b.abs() > float(unit[l])
        n_big += int(big.sum())
        agree += int((torch.sign(a[big]) == torch.sign(b[big])).sum())
    f_lost, f_agree = lost / max(n_nz, 1), agree / max(n_big, 1)
    # Adam: 3 steps from the same parameters with each gradient mode, and fp32
    # again with the rays in reverse order (the same gradient, summed in
    # another order): with eps = 1e-15 an entry whose records cancel to
    # rounding noise still takes an lr-sized step, so fp32 differs from itself
    # under reordering -- the floor any summation of these records meets
    p0 = m.xyz_encoder.params.detach().clone()
    rev = (o[::-1].copy(), d[::-1].copy(), noise[:, ::-1].copy(),
           tuple(x[::-1].copy() for x in seeds))
    deltas = {}
    for mode in ("fx", "fp32", "fp32_reordered"):
        with torch.no_grad():
            m.xyz_encoder.params.copy_(p0)
        opt = FusedAdam([m.xyz_encoder.params], lr=1e-2, eps=1e-15)
        r.grid_fx = mode == "fx"
        oo, dd, nn, ss = rev if mode == "fp32_reordered" else (o, d, noise, seeds)
        for _ in range(3):
            _run(ml_render_fused, m, g, oo, dd, nn, ss, cuda, esf)
            opt.step()
        deltas[mode] = (m.xyz_encoder.params.detach() - p0).view(-1, 2)
    r.grid_fx = True

    def upd(x, y):
        return [float((_level(deltas[x], lv, l) - _level(deltas[y], lv, l)).norm() /
                      _level(deltas[y], lv, l).norm().clamp_min(1e-30)) for l in range(16)]
    rels, floor = upd("fx", "fp32"), upd("fp32_reordered", "fp32")
    rel = max(rels)
    with capsys.disabled():
        print(f"\nfx per entry B{B} K{K} s{scale} ({'binned' if r.grid_bin else 'int32'}"
              f"{', fp32 levels ' + str(f32_levels) if f32_levels else ''}): "
              f"{f_lost:.4%} of the non-zero fp32 entries are 0 in fixed point; "
              f"sign agreement above one unit {f_agree:.5%} ({n_big} entries); "
              f"3 Adam steps: per-level update difference max {rel:.3e} "
              f"(level {int(np.argmax(rels))}); fp32 vs fp32 of the reversed rays max "
              f"{max(floor):.3e}")
        print("  per level fx-fp32 " + " ".join(f"{x:.3f}" for x in rels))
        print("  per level fp32-fp32 reordered " + " ".join(f"{x:.3f}" for x in floor))
    r.fx_f32_levels = ()
    assert f_agree >= 0.999
    assert f_lost <= 0.05
    assert rel <= bar


def _fx_weight(i):
    return (4 * int(i)) & 0xFFFFFFFF                       # fx_weight (field.hip): byte offset


@pytest.mark.parametrize("wrapped", [True, False])
def test_fx_opposite_wraps_set_redo(cuda, wrapped):
    """ADVICE r03 / VERDICT r03 item 5: two int32 entries of one level that wrap
    in opposite directions in one step (+2^32 and -2^32) leave the level's
    plain entry sum equal to its record sum; the position-weighted sums
    (element i weighted by its byte offset 4 i, mod 2^64) still differ,
    so rn_grid_fx_fold sets the redo flag.  Control: the same records without
    a wrap pass."""
    from radnerf_amd._lib import lib
    L = lib()
    scale = 0.5
    lv = LY.grid_levels(scale)
    n_el = 2 * int(lv["n_entries"])
    l = 15
    a = 2 * int(lv["offset"][l]) + 10
    b = 2 * int(lv["offset"][l]) + 1001
    rec_a, rec_b = (2 ** 31 + 100, -(2 ** 31 + 100)) if wrapped else (100, -100)
    ent_a = rec_a - 2 ** 32 if wrapped else rec_a          # the int32 entries as stored
    ent_b = rec_b + 2 ** 32 if wrapped else rec_b
    acc = torch.zeros(n_el, dtype=torch.int32, device=cuda)
    acc[a], acc[b] = ent_a, ent_b
    stats = np.zeros(160, np.int32)
    st64 = stats.view(np.int64)                             # qsum @16, esum @32, wq @48, we @64 (i64 slots)
    stats.view(np.uint32)[l] = np.float32(1.0).view(np.uint32)   # vmax: a small record
    st64[16 + l] = rec_a + rec_b                            # qsum: exact record sum (0)
    wq = (rec_a * _fx_weight(a) + rec_b * _fx_weight(b)) % (1 << 64)
    st64[48 + l] = wq if wq < (1 << 63) else wq - (1 << 64)
    stats_t = torch.from_numpy(stats).to(cuda)
    scales = torch.full((2, 16), 2.0 ** 10, device=cuda)
    redo = torch.zeros(1, dtype=torch.int32, device=cuda)
    grad = torch.zeros(n_el, device=cuda)
    assert ent_a + ent_b == rec_a + rec_b                  # the plain sums agree either way
    L.grid_fx_fold(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, lv["res"].ctypes.data,
                   acc.data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(), stats_t.data_ptr(),
                   redo.data_ptr(), grad.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(redo[0]) == (1 if wrapped else 0)
    if not wrapped:                                         # folded: entry * 2^-10
        assert float(grad[a]) == 100 / 1024 and float(grad[b]) == -100 / 1024
    assert int(acc.abs().max()) == 0                        # re-zeroed either way
