"""Pricing probe for the binned grid-gradient scatter.

Fills the page pool with synthetic walk records of a given shape (records per
sample per level from tools/records_sim.py's replay of the bench workload,
entry indices uniform over each level), then times rn_grid_bin and
rn_grid_sum on the GPU with HIP events on the launch stream and checks the
sums against an exact float64 bincount.

The question: is bin + sum (both memory-bound, 8 B per record each way)
cheaper than the 3.7 ms that the atomic form's requests cost C5's field_bwd
(8.40 ms with, 4.66 ms without atomics; profiles/r03/ablate_phases_c5_r03b.json)?

usage: python tools/bin_probe.py [shape=c5|c4|c3] [reps]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rad-nerf_amd")]
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd._lib import lib, use_ablation_build  # noqa: E402

use_ablation_build()        # rn_set_debug_flags switches live only in librn_abl.so


def _layout():
    import ctypes
    out = (ctypes.c_int32 * 8)()
    lib().grid_bin_layout(out)
    return list(out)


PAGE, MAX_BINS, SLICE, CTL_BYTES, IDX_BITS, V_BITS = _layout()[:6]

# records / sample per level (tools/records_sim.py: K 8 scale 16 B 1024, chunk 2048)
REC_C5 = [0.16, 0.25, 0.39, 0.61, 0.96, 1.51, 2.31, 3.36, 4.51, 5.56, 6.38, 6.96, 7.35, 7.60,
          7.76, 7.85]
SHAPES = {"c5": (16.0, 6227661, REC_C5)}


def _field(q):
    """e4m18 fields of integer record values (exact below 2^16 units)"""
    q = np.ascontiguousarray(q, np.float32)
    f = np.zeros(len(q), np.uint32)
    lib().grid_record_encode(q.ctypes.data, len(q), f.ctypes.data)
    return f.astype(np.uint64)


def pack(idx, q0, q1):
    return (idx.astype(np.uint64) | (_field(q0) << np.uint64(IDX_BITS))
            | (_field(q1) << np.uint64(IDX_BITS + V_BITS)))


class Pool:
    """The binned scatter's device buffers (rn_bin.h)."""

    def __init__(self, pool_pages, dev):
        self.pool_pages = pool_pages
        self.ctl = torch.zeros(CTL_BYTES // 4, dtype=torch.int32, device=dev)
        self.meta = torch.zeros(pool_pages, dtype=torch.int32, device=dev)
        self.pin = torch.zeros(pool_pages * PAGE, dtype=torch.int64, device=dev)
        self.pout = torch.zeros(pool_pages * PAGE, dtype=torch.int64, device=dev)
        self.desc = torch.zeros(pool_pages * MAX_BINS, dtype=torch.int32, device=dev)
        self.lpages = torch.zeros(16 * pool_pages, dtype=torch.int32, device=dev)


def synthetic(scale, n_samples, rec_per_level, rng, vmax=1 << 12, page_fill=1.0):
    """per-level record arrays (idx, q0, q1) and the pages holding them"""
    lv = LY.grid_levels(scale)
    per = []
    for l in range(16):
        n = int(round(rec_per_level[l] * n_samples))
        hs = int(lv["hsize"][l])
        idx = rng.integers(0, hs, n, dtype=np.int64)
        q0 = rng.integers(-vmax, vmax, n, dtype=np.int64)
        q1 = rng.integers(-vmax, vmax, n, dtype=np.int64)
        per.append((idx, q0, q1))
    return lv, per


def fill(pool, per, page_fill=1.0, rng=None):
    """lay the records out as the walk would: pages of one level each (filled
    to page_fill of 8192, pages of the levels interleaved)"""
    cap = max(1, int(PAGE * page_fill))
    pages, metas = [], []
    for l, (idx, q0, q1) in enumerate(per):
        rec = pack(idx, q0, q1).view(np.int64)
        for a in range(0, len(rec), cap):
            chunk = rec[a:a + cap]
            pg = np.zeros(PAGE, np.int64)
            pg[:len(chunk)] = chunk
            pages.append(pg)
            metas.append(l | (len(chunk) << 8))
    order = rng.permutation(len(pages)) if rng is not None else np.arange(len(pages))
    assert len(pages) <= pool.pool_pages, (len(pages), pool.pool_pages)
    buf = np.stack([pages[i] for i in order]) if pages else np.zeros((0, PAGE), np.int64)
    pool.pin[:buf.size].copy_(torch.from_numpy(buf.ravel()))
    pool.meta[:len(pages)].copy_(torch.from_numpy(np.array([metas[i] for i in order], np.int32)))
    return len(pages)


def expected(lv, per, scale_l):
    n = int(lv["n_entries"])
    g = np.zeros((n, 2), np.float64)
    for l, (idx, q0, q1) in enumerate(per):
        off = int(lv["offset"][l])
        g[:, 0] += np.bincount(idx + off, weights=q0.astype(np.float64), minlength=n)
        g[:, 1] += np.bincount(idx + off, weights=q1.astype(np.float64), minlength=n)
        g[off:off + int(lv["hsize"][l])] /= scale_l[l]
    return g


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c5"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    layout = sys.argv[3] if len(sys.argv) > 3 else "shuffled"     # or "level": pages level-major
    frac = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0       # of the shape's samples
    scale, n_samples, rec = SHAPES[shape]
    n_samples = int(n_samples * frac)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    lv, per = synthetic(scale, n_samples, rec, rng)
    n_rec = sum(len(p[0]) for p in per)
    pool = Pool(n_rec // PAGE + 32, dev)
    n_pages = fill(pool, per, rng=rng if layout == "shuffled" else None)
    scale_l = np.full(16, 2.0 ** 10, np.float32)
    scale_t = torch.from_numpy(scale_l).to(dev)
    grad = torch.zeros(int(lv["n_entries"]) * 2, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    L = lib()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tb, ts = [], []
    for it in range(reps + 1):
        grad.zero_()
        pool.ctl.zero_()
        pool.ctl[0] = n_pages
        ev[0].record(st)
        L.grid_bin(lv["hsize"].ctypes.data, pool.ctl.data_ptr(), pool.meta.data_ptr(), pool.pin.data_ptr(),
                   pool.pout.data_ptr(), pool.desc.data_ptr(), pool.lpages.data_ptr(),
                   pool.pool_pages, 2048, sp)
        ev[1].record(st)
        L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, pool.ctl.data_ptr(),
                   pool.desc.data_ptr(), pool.lpages.data_ptr(), pool.pout.data_ptr(),
                   pool.pool_pages, scale_t.data_ptr(), None, grad.data_ptr(), 0, 16, sp)
        ev[2].record(st)
        torch.cuda.synchronize()
        if it == 0:
            ref = expected(lv, per, scale_l)
            got = grad.view(-1, 2).cpu().numpy().astype(np.float64)
            err = np.abs(got - ref).max() / max(1e-30, np.abs(ref).max())
            continue
        tb.append(ev[0].elapsed_time(ev[1]))
        ts.append(ev[1].elapsed_time(ev[2]))
    # ablations of the sum pass (timing only): no LDS adds; int32 LDS adds
    abl = {}
    for name, flag in (("sum_no_lds_adds", 1 << 16), ("bis1_load_every_run", (1 << 16) | (1 << 18)),
                       ("bis2_fold_every_lane", (1 << 16) | (2 << 18)),
                       ("bis3_runs_of_64", (1 << 16) | (3 << 18)),
                       ("bis4_full_lane_loads", (1 << 16) | (4 << 18))):
        L.set_debug_flags(flag)
        t = []
        for it in range(reps):
            ev[1].record(st)
            L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, pool.ctl.data_ptr(),
                       pool.desc.data_ptr(), pool.lpages.data_ptr(), pool.pout.data_ptr(),
                       pool.pool_pages, scale_t.data_ptr(), None, grad.data_ptr(), 0, 16, sp)
            ev[2].record(st)
            torch.cuda.synchronize()
            t.append(ev[1].elapsed_time(ev[2]))
        abl[name] = round(float(np.median(t)), 4)
    L.set_debug_flags(0)
    # per-phase cycles of the sum pass (debug bit 21)
    import ctypes
    cy = (ctypes.c_ulonglong * 8)()
    L.debug_gb_cycles(cy)                  # reset
    L.set_debug_flags(1 << 21)
    ev[1].record(st)
    L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, pool.ctl.data_ptr(),
               pool.desc.data_ptr(), pool.lpages.data_ptr(), pool.pout.data_ptr(),
               pool.pool_pages, scale_t.data_ptr(), None, grad.data_ptr(), 0, 16, sp)
    ev[2].record(st)
    torch.cuda.synchronize()
    L.set_debug_flags(0)
    L.debug_gb_cycles(cy)
    waves = max(1, cy[4])
    abl["sum_prof"] = {"ms": round(ev[1].elapsed_time(ev[2]), 4), "waves": cy[4],
                       "groups_per_wave": round(cy[5] / waves, 2),
                       "cycles_per_wave": {n: round(cy[i] / waves) for i, n in
                                           enumerate(("zero", "first_fetch", "runs", "writeback"))},
                       "span_ms_inside": round((cy[7] - cy[6]) / 1e5, 4)}
    # the bin pass without the per-page rotation of the run layout
    L.set_debug_flags(1 << 20)
    t = []
    for it in range(reps):
        pool.ctl.zero_()
        pool.ctl[0] = n_pages
        L.grid_bin(lv["hsize"].ctypes.data, pool.ctl.data_ptr(), pool.meta.data_ptr(), pool.pin.data_ptr(),
                   pool.pout.data_ptr(), pool.desc.data_ptr(), pool.lpages.data_ptr(),
                   pool.pool_pages, 2048, sp)
        ev[1].record(st)
        L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, pool.ctl.data_ptr(),
                   pool.desc.data_ptr(), pool.lpages.data_ptr(), pool.pout.data_ptr(),
                   pool.pool_pages, scale_t.data_ptr(), None, grad.data_ptr(), 0, 16, sp)
        ev[2].record(st)
        torch.cuda.synchronize()
        t.append(ev[1].elapsed_time(ev[2]))
    abl["sum_unrotated_runs"] = round(float(np.median(t)), 4)
    # bin pass variants (timing only): 512 threads + next page prefetched; 256 threads
    for name, flag in (("bin_512_prefetch", 1 << 22), ("bin_256", 2 << 22)):
        L.set_debug_flags(flag)
        t = []
        for it in range(reps):
            pool.ctl.zero_()
            pool.ctl[0] = n_pages
            ev[0].record(st)
            L.grid_bin(lv["hsize"].ctypes.data, pool.ctl.data_ptr(), pool.meta.data_ptr(),
                       pool.pin.data_ptr(), pool.pout.data_ptr(), pool.desc.data_ptr(),
                       pool.lpages.data_ptr(), pool.pool_pages, 2048, sp)
            ev[1].record(st)
            torch.cuda.synchronize()
            t.append(ev[0].elapsed_time(ev[1]))
        abl[name] = round(float(np.median(t)), 4)
    L.set_debug_flags(0)
    pool.ctl.zero_()
    pool.ctl[0] = n_pages
    L.grid_bin(lv["hsize"].ctypes.data, pool.ctl.data_ptr(), pool.meta.data_ptr(), pool.pin.data_ptr(),
               pool.pout.data_ptr(), pool.desc.data_ptr(), pool.lpages.data_ptr(),
               pool.pool_pages, 2048, sp)
    # footprint test: the same runs, but every level's page list pointing at
    # 16 of its pages only (tiny footprint: TLB- and cache-resident)
    lp = pool.lpages.view(16, -1)
    npg = pool.ctl[1:17].clone()
    for l in range(16):
        n = int(npg[l])
        if n > 16:
            lp[l, :n] = lp[l, torch.arange(n, device=dev) % 16]
    t = []
    for it in range(reps):
        ev[1].record(st)
        L.grid_sum(lv["offset"].ctypes.data, lv["hsize"].ctypes.data, pool.ctl.data_ptr(),
                   pool.desc.data_ptr(), pool.lpages.data_ptr(), pool.pout.data_ptr(),
                   pool.pool_pages, scale_t.data_ptr(), None, grad.data_ptr(), 0, 16, sp)
        ev[2].record(st)
        torch.cuda.synchronize()
        t.append(ev[1].elapsed_time(ev[2]))
    abl["sum_16_pages_per_level"] = round(float(np.median(t)), 4)
    tb, ts = float(np.median(tb)), float(np.median(ts))
    out = {"shape": shape, "layout": layout, "frac": frac, "records": n_rec, "pages": n_pages, "rel_err": float(err),
           "bin_ms": round(tb, 4), "sum_ms": round(ts, 4), "bin_sum_ms": round(tb + ts, 4),
           "bin_GBs": round(16 * n_rec / tb / 1e6, 1), "sum_GBs": round(8 * n_rec / ts / 1e6, 1),
           "atomic_cost_ms_c5": 8.40 - 4.66, "ablations_ms": abl}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
