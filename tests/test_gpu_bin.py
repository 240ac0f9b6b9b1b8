"""Binned ("store and sum") grid-gradient scatter (fx_mode 4: the walk appends
fixed-point records to pages, rn_grid_bin sorts each page by slice, rn_grid_sum
adds each slice in LDS; csrc/rn_bin.h, scatter.hip).

* the bin + sum passes alone, on synthetic pages: every entry equals the
  exact integer sum of its records times 2^-e_l (bit-exact), in place and
  out of place, with pages of mixed levels, partial pages and empty slices;
* the renderer at scale 16 (where it is the default) and, forced, at scale
  0.5: every level's gradient matches the fp32-atomic backward of the same
  step within FX_LEVEL_TOL (the oracle bars are in test_gpu_ml.py, which runs
  the default path), the MLP / gate gradients are unchanged, and the grid
  gradient is bitwise identical from step to step (exact int64 sums);
* a record past the int22 range (a scale forced 2^10 too large) and a pool
  too small for the step both set the redo flag, and the step's result is the
  fp32 one; the pool then grows, and the next steps are binned again.
"""
import numpy as np
import pytest
import torch

from radnerf_amd import layout as LY
from radnerf_amd._lib import lib
from radnerf_amd.fused import get_renderer, ml_render_fused, release_renderers
from test_gpu_ml import FX_LEVEL_TOL, _run, _setup, check_fx_vs_fp32

pytestmark = pytest.mark.gpu


def _field(q):
    """the e5m17 field of record values q (rn_grid_record_encode) and the exact
    value the sum pass adds for it"""
    q = np.ascontiguousarray(q, np.float32)
    f = np.zeros(len(q), np.uint32)
    v = np.zeros(len(q), np.int64)
    lib().grid_record_encode(q.ctypes.data, len(q), f.ctypes.data)
    lib().grid_record_decode(f.ctypes.data, len(q), v.ctypes.data)
    return f, v


def _pack(idx, f0, f1, lay):
    ib, vb = lay["idx_bits"], lay["v_bits"]
    return (idx.astype(np.uint64) | (f0.astype(np.uint64) << np.uint64(ib))
            | (f1.astype(np.uint64) << np.uint64(ib + vb))).view(np.int64)


@pytest.mark.parametrize("in_place", [True, False])
def test_bin_sum_exact_on_synthetic_pages(cuda, in_place):
    L = lib()
    lay = L.bin_layout()
    PAGE = lay["page"]
    scale = 16.0
    lv = LY.grid_levels(scale)
    rng = np.random.default_rng(7)
    vmax = 2.0 ** 40          # record values over most of the e5m17 range
    pages, metas, per = [], [], []
    for l in range(16):
        hs = int(lv["hsize"][l])
        n = int(rng.integers(0, 3 * PAGE)) if l != 5 else 0          # level 5: no records
        idx = rng.integers(0, hs, n)
        if l == 15:                         # one hot entry and the range ends
            idx[: n // 4] = hs - 1
            idx[n // 4: n // 4 + 10] = 0
        # log-uniform magnitudes (1 unit .. 2^30), random signs; a few zeros
        mag = np.exp2(rng.uniform(0, np.log2(vmax), (2, n))) * (rng.random((2, n)) > 0.01)
        sg = np.where(rng.random((2, n)) < 0.5, -1.0, 1.0)
        (f0, q0), (f1, q1) = _field(mag[0] * sg[0]), _field(mag[1] * sg[1])
        per.append((idx, q0, q1))
        rec = _pack(idx, f0, f1, lay)
        fill = int(rng.integers(PAGE // 2, PAGE + 1))                # partial pages
        for a in range(0, n, fill):
            c = rec[a:a + fill]
            pg = np.zeros(PAGE, np.int64)
            pg[:len(c)] = c
            pages.append(pg)
            metas.append(l | (len(c) << 8))
    order = rng.permutation(len(pages))
    pool = len(pages) + 3
    i32 = dict(device=cuda, dtype=torch.int32)
    ctl = torch.zeros(lay["ctl_bytes"] // 4, **i32)
    ctl[0] = len(pages)
    meta = torch.zeros(pool, **i32)
    meta[:len(pages)] = torch.from_numpy(np.array([metas[i] for i in order], np.int32))
    pin = torch.zeros(pool * PAGE, device=cuda, dtype=torch.int64)
    pin[:len(pages) * PAGE] = torch.from_numpy(np.stack([pages[i] for i in order]).ravel())
    pout = pin if in_place else torch.zeros_like(pin)
    desc = torch.zeros(pool * lay["bins"], **i32)
    lpages = torch.zeros(16 * pool, **i32)
    sc = (2.0 ** rng.integers(-3, 12, 16)).astype(np.float32)
    sc_t = torch.from_numpy(sc).to(cuda)
    grad0 = rng.standard_normal(int(lv["n_entries"]) * 2).astype(np.float32)
    grad = torch.from_numpy(grad0).to(cuda)
    st = torch.cuda.current_stream().cuda_stream
    L.grid_bin(lv["hsize"].ctypes.data, ctl.data_ptr(), meta.data_ptr(), pin.data_ptr(), pout.data_ptr(), desc.data_ptr(),
               lpages.data_ptr(), pool, 64, st)
    # in two launches (fine levels first, as the data-parallel step runs it
    # to start their all-reduce early): the same sums
    for lo, hi in ((7, 16), (0, 7)):
        L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, ctl.data_ptr(),
                   desc.data_ptr(), lpages.data_ptr(), pout.data_ptr(), pool, sc_t.data_ptr(), None,
                   grad.data_ptr(), lo, hi, st)
    got = grad.cpu().numpy().reshape(-1, 2)
    want = grad0.copy().reshape(-1, 2)
    for l, (idx, q0, q1) in enumerate(per):
        off, hs = int(lv["offset"][l]), int(lv["hsize"][l])
        a0 = np.zeros(hs, np.int64)
        a1 = np.zeros(hs, np.int64)
        np.add.at(a0, idx, q0)
        np.add.at(a1, idx, q1)
        inv = np.float32(1.0) / sc[l]
        nz = (a0 != 0) | (a1 != 0)
        blk = want[off:off + hs]
        blk[nz, 0] = blk[nz, 0] + a0[nz].astype(np.float32) * inv
        blk[nz, 1] = blk[nz, 1] + a1[nz].astype(np.float32) * inv
    assert np.array_equal(got, want)
    # each level's page list holds its pages
    npg = ctl[1:17].cpu().numpy()
    assert npg.tolist() == [sum(1 for m_ in metas if (m_ & 31) == l) for l in range(16)]


def _levels(g, lv):
    return [g.view(-1, 2)[int(lv["offset"][l]):int(lv["offset"][l]) + int(lv["hsize"][l])]
            for l in range(16)]


@pytest.mark.parametrize("B,K,scale", [(1024, 4, 16.0), (2048, 2, 0.5)])
def test_binned_matches_fp32_and_is_reproducible(cuda, B, K, scale):
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_fx
    assert r.grid_bin == (scale > 0.5)
    r.grid_bin, r.bin_f32_levels = True, 0          # every level binned
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)      # fp32: scales
    _, gb1 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    assert check_fx_vs_fp32(m, gb1, g32, r, f"binned B{B} K{K} s{scale}") == 16
    pool = r.ws._bin
    assert int(pool["ctl"][0]) > 0                       # the walk took pages
    assert int(pool["ctl"][0]) <= pool["pages"]
    _, gb2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    lv = LY.grid_levels(scale)
    for l, (a, b) in enumerate(zip(_levels(gb1[0], lv), _levels(gb2[0], lv))):
        assert torch.equal(a, b), l                      # exact integer sums
    assert int(r.ws._fx[0].abs().max()) == 0             # the int32 table is unused


def test_binned_record_overflow_redo(cuda):
    B, K, scale = 1024, 4, 16.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_bin
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    acc, scales, stats, redo = r.ws._fx
    with torch.no_grad():
        cur = scales[r.ws.fx_i]
        cur.mul_(2.0 ** 10)          # the largest records map to ~2^28 units: past int22
    _, g_redo = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    assert int(redo[0]) == 1
    for x, y in zip(g_redo, g32):
        assert float((x - y).norm() / y.norm().clamp_min(1e-30)) <= 1e-5     # fp32 order only
    _, gb = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    assert int(redo[0]) == 0
    check_fx_vs_fp32(m, gb, g32, r, "binned after redo")


def test_binned_pool_overflow_redo_then_grows(cuda):
    B, K, scale = 1024, 4, 16.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    r.bin_records_per_pair = 8           # a pool far too small for the step
    r.bin_f32_levels = 0                 # (every level takes pages: each wave opens two)
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    _, g_redo = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    pool = r.ws._bin
    redo = r.ws._fx[3]
    assert int(pool["ctl"][0]) > pool["pages"]           # the walk ran out of pages
    assert int(redo[0]) == 1
    for x, y in zip(g_redo, g32):
        assert float((x - y).norm() / y.norm().clamp_min(1e-30)) <= 1e-5
    # the pool grows from the page count of the backward BIN_LAG (2) back,
    # whatever the host's lead: the next step still overflows (redone in
    # fp32, deterministically), the one after runs binned on the grown pool
    _, g_redo2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    assert int(redo[0]) == 1 and r.ws._bin["pages"] == pool["pages"]
    _, gb = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)   # grown
    assert r.ws._bin["pages"] > pool["pages"]
    assert int(redo[0]) == 0
    check_fx_vs_fp32(m, gb, g32, r, "binned after pool growth")
    assert FX_LEVEL_TOL > 0


def _pool(cuda, lay, pool, pages, metas, canary=64):
    """the pass buffers with `canary` guard elements past each one's end"""
    PAGE = lay["page"]
    i32 = dict(device=cuda, dtype=torch.int32)
    C = canary
    buf = dict(
        ctl=torch.zeros(lay["ctl_bytes"] // 4 + C, **i32),
        meta=torch.full((pool + C,), 0x5a5a5a5a, **i32),
        pin=torch.full((pool * PAGE + C,), 0x3c3c3c3c3c3c3c3c, device=cuda, dtype=torch.int64),
        pout=torch.full((pool * PAGE + C,), 0x3c3c3c3c3c3c3c3c, device=cuda, dtype=torch.int64),
        desc=torch.full((pool * lay["bins"] + C,), 0x5a5a5a5a, **i32),
        lpages=torch.full((16 * pool + C,), 0x5a5a5a5a, **i32))
    buf["ctl"][lay["ctl_bytes"] // 4:] = 0x5a5a5a5a
    buf["ctl"][0] = len(pages)
    buf["meta"][:len(metas)] = torch.tensor(metas, **i32)
    if pages:
        buf["pin"][:len(pages) * PAGE] = torch.from_numpy(np.stack(pages).ravel())
    return buf


def _canaries_intact(buf, lay, pool):
    PAGE = lay["page"]
    ends = dict(ctl=lay["ctl_bytes"] // 4, meta=pool, pin=pool * PAGE, pout=pool * PAGE,
                desc=pool * lay["bins"], lpages=16 * pool)
    for k, e in ends.items():
        t = buf[k][e:]
        want = 0x3c3c3c3c3c3c3c3c if t.dtype == torch.int64 else 0x5a5a5a5a
        assert bool((t == want).all()), k


@pytest.mark.parametrize("case", ["clean", "meta_count", "meta_level", "index"])
def test_bin_pass_refuses_corrupt_inputs(cuda, case):
    """the bin pass trusted page_meta (count and level) and
    every record's entry index; a corrupt one indexed LDS and HBM out of
    bounds.  Now a page whose meta names a level >= 16 or more than 8192
    records, or a record whose index lies outside its level, is refused: the
    GbCtl fault word is set, rn_grid_binned_fold raises the redo flag, the sum
    pass adds nothing, and no byte past any buffer changes.  Control: the same
    pages without the corruption fold exactly."""
    L = lib()
    lay = L.bin_layout()
    PAGE = lay["page"]
    scale = 16.0
    lv = LY.grid_levels(scale)
    hs = lv["hsize"]
    rng = np.random.default_rng(11)
    pages, metas, per = [], [], []
    for l in (2, 9, 15):
        n = 3000
        idx = rng.integers(0, int(hs[l]), n)
        (f0, q0), (f1, q1) = _field(rng.integers(-500, 500, n)), _field(rng.integers(-500, 500, n))
        pg = np.zeros(PAGE, np.int64)
        pg[:n] = _pack(idx, f0, f1, lay)
        pages.append(pg); metas.append(l | (n << 8)); per.append((l, idx, q0, q1))
    if case == "meta_count":
        metas[1] = 9 | ((PAGE + 1000) << 8)
    elif case == "meta_level":
        metas[1] = 20 | (3000 << 8)
    elif case == "index":
        pages[0][17] = _pack(np.array([int(hs[2]) + 5]), *_field(np.array([7]))[:1],
                             *_field(np.array([7]))[:1], lay)[0]
    pool = 4
    buf = _pool(cuda, lay, pool, pages, metas)
    sc = torch.full((2, 16), 1.0, device=cuda)
    stats = torch.zeros(160, device=cuda, dtype=torch.int32)
    redo = torch.zeros(1, device=cuda, dtype=torch.int32)
    n_el = 2 * int(lv["n_entries"])
    grad = torch.zeros(n_el + 64, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    L.grid_binned_fold(lv["offset"].ctypes.data, hs.ctypes.data, buf["ctl"].data_ptr(),
                       buf["meta"].data_ptr(), buf["pin"].data_ptr(), buf["pout"].data_ptr(),
                       buf["desc"].data_ptr(), buf["lpages"].data_ptr(), pool, sc[0].data_ptr(),
                       sc[1].data_ptr(), stats.data_ptr(), redo.data_ptr(), grad.data_ptr(), st)
    torch.cuda.synchronize()
    _canaries_intact(buf, lay, pool)
    assert bool((grad[n_el:] == 0).all())
    fault = int(buf["ctl"][17])
    if case == "clean":
        assert fault == 0 and int(redo[0]) == 0
        g = grad[:n_el].view(-1, 2).cpu().numpy()
        for l, idx, q0, q1 in per:
            off = int(lv["offset"][l])
            a0 = np.zeros(int(hs[l]), np.int64)
            np.add.at(a0, idx, q0)
            assert np.array_equal(g[off:off + int(hs[l]), 0], a0.astype(np.float32))
    else:
        assert fault == (2 if case == "index" else 1), fault
        assert int(redo[0]) == 1
        assert float(grad[:n_el].abs().max()) == 0.0          # the sum pass added nothing


def test_bin_pass_without_ctl_reset_stays_in_bounds(cuda):
    """The round-4 fault (tools/bin_probe.py, an ablation loop that re-ran the
    bin pass without zeroing GbCtl): the level page counters kept counting,
    so the second pass wrote level_pages slots past its level's row -- for
    level 15 past the end of the buffer.  Now a slot >= pool_pages is refused
    (fault bit 4) and nothing is written past the list."""
    L = lib()
    lay = L.bin_layout()
    PAGE = lay["page"]
    lv = LY.grid_levels(16.0)
    hs = lv["hsize"]
    rng = np.random.default_rng(5)
    pages, metas = [], []
    for _ in range(4):                                   # every page: level 15
        n = 1000
        f = _field(rng.integers(-9, 9, n))[0]
        pg = np.zeros(PAGE, np.int64)
        pg[:n] = _pack(rng.integers(0, int(hs[15]), n), f, f, lay)
        pages.append(pg); metas.append(15 | (n << 8))
    pool = 4
    buf = _pool(cuda, lay, pool, pages, metas)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(2):                                   # the second run: no reset
        L.grid_bin(hs.ctypes.data, buf["ctl"].data_ptr(), buf["meta"].data_ptr(),
                   buf["pin"].data_ptr(), buf["pout"].data_ptr(), buf["desc"].data_ptr(),
                   buf["lpages"].data_ptr(), pool, 64, st)
    torch.cuda.synchronize()
    _canaries_intact(buf, lay, pool)
    assert int(buf["ctl"][1 + 15]) == 8                  # counted on ...
    assert int(buf["ctl"][17]) & 4                       # ... but refused


def test_sum_pass_run_fault_is_sticky_and_raised(cuda):
    """the sum pass skipped a page run past its page and set the
    fault word, but the step's check had already run, so nothing read it.
    Now the run is also recorded in GbCtl's sticky sum_fault word (not cleared
    by the per-step reset), and the renderer raises when it reads it back."""
    L = lib()
    lay = L.bin_layout()
    PAGE = lay["page"]
    lv = LY.grid_levels(16.0)
    hs = lv["hsize"]
    rng = np.random.default_rng(3)
    n = 2000
    f = _field(rng.integers(-9, 9, n))[0]
    pg = np.zeros(PAGE, np.int64)
    pg[:n] = _pack(rng.integers(0, int(hs[12]), n), f, f, lay)
    pool = 2
    buf = _pool(cuda, lay, pool, [pg], [12 | (n << 8)])
    st = torch.cuda.current_stream().cuda_stream
    L.grid_bin(hs.ctypes.data, buf["ctl"].data_ptr(), buf["meta"].data_ptr(),
               buf["pin"].data_ptr(), buf["pout"].data_ptr(), buf["desc"].data_ptr(),
               buf["lpages"].data_ptr(), pool, 64, st)
    torch.cuda.synchronize()
    assert int(buf["ctl"][17]) == 0 and int(buf["ctl"][18]) == 0
    # one slice's run pushed past the page end
    desc = buf["desc"][:lay["bins"]]
    b = int(torch.nonzero(desc >> 16).view(-1)[0])
    buf["desc"][b] = (int(desc[b]) & 0xffff0000) | (PAGE - 3)
    sc = torch.full((16,), 1.0, device=cuda)
    redo = torch.zeros(1, device=cuda, dtype=torch.int32)
    grad = torch.zeros(2 * int(lv["n_entries"]) + 64, device=cuda)
    L.grid_sum(lv["offset"].ctypes.data, hs.ctypes.data, buf["ctl"].data_ptr(),
               buf["desc"].data_ptr(), buf["lpages"].data_ptr(), buf["pout"].data_ptr(), pool,
               sc.data_ptr(), redo.data_ptr(), grad.data_ptr(), 0, 16, st)
    torch.cuda.synchronize()
    _canaries_intact(buf, lay, pool)
    assert int(buf["ctl"][17]) & 8 and int(buf["ctl"][18]) & 8
    # the renderer: a sticky word read back raises at the next pool sizing
    from radnerf_amd.fused import GB_SUM_FAULT
    assert GB_SUM_FAULT == 18


def test_renderer_raises_on_sum_fault(cuda):
    """End to end at scale 16: the binned renderer reads GbCtl back with the
    page count; a sticky sum_fault makes the pool sizing BIN_LAG backwards
    later raise RuntimeError instead of stepping on a partial gradient.  A clean
    run leaves the word 0."""
    B, K, scale = 1024, 2, 16.0               # (rays x sub-NeRFs > 1024: fixed point)
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_bin
    for _ in range(4):
        _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    torch.cuda.synchronize()
    assert int(r.ws._bin["ctl"][18]) == 0 and int(r.ws._bin["ctl"][17]) == 0
    r.ws._bin["ctl"][18] = 8                        # as a refused run leaves it
    with pytest.raises(RuntimeError, match="sum pass refused a page run"):
        for _ in range(r.BIN_LAG + 2):
            _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    r.ws._bin["ctl"][18] = 0
    release_renderers()


@pytest.mark.parametrize("B,K", [(1024, 4), (1024, 8)])
def test_binned_default_coarse_levels_fp32(cuda, B, K):
    """Round 6 default at scale 16: the coarse levels [0, n) go in by fp32
    atomics (no page records), the rest binned.  Every level matches the fp32
    gradient of the same step (FX_LEVEL_TOL), the binned levels are bitwise
    identical step to step, the coarse levels took no pages."""
    scale = 16.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    n = r.bin_f32_levels
    assert r.grid_bin and n == (9 if K >= 8 else 8)
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    _, gb1 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    assert check_fx_vs_fp32(m, gb1, g32, r, f"binned, levels [0, {n}) fp32, B{B} K{K}") == 16 - n
    npg = r.ws._bin["ctl"][1:17].cpu()
    assert int(npg[:n].sum()) == 0 and bool((npg[n:] > 0).all()), npg
    _, gb2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 1 / 256)
    lv = LY.grid_levels(scale)
    for l, (a, b) in enumerate(zip(_levels(gb1[0], lv), _levels(gb2[0], lv))):
        if l >= n:
            assert torch.equal(a, b), l                  # exact integer sums
        else:                                            # fp32 in arrival order
            assert float((a - b).norm() / b.norm().clamp_min(1e-30)) <= 1e-5, l
