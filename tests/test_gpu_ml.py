"""End-to-end Rad-NeRF training render on the GPU: fused chain vs the drop-in
(reference-structured) chain vs the CPU oracle (oracle/ml_oracle.py).

Bars:
  * fused march: per-(model, ray) sample counts and t / dt bit-exact vs oracle;
  * fused vs drop-in GPU paths: outputs within 1e-5, gradients within 1e-3 rel
    (same kernels; only float-atomic accumulation order differs);
  * vs oracle: rgb / opacity / depth L_inf reported; rgb <= 1e-3 (the f16
    field can flip one f16 ulp of an activation vs the fp32-ordered oracle;
    the composite alone is held to 1e-4 in test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from oracle import ml_oracle
from radnerf_amd import layout as LY
from radnerf_amd import synthetic as S
from radnerf_amd.fused import ml_render_fused, get_renderer
from radnerf_amd.networks import MNGP, Ray_Gate
from radnerf_amd.rendering import ml_render as _ml_render
from parity import LAYERS, check_grads, rel as _rel  # noqa: F401


def ml_render(*a, **kw):
    """the drop-in chain: rendering.ml_render with the reference's op-by-op autograd"""
    return _ml_render(*a, fused=False, **kw)

pytestmark = pytest.mark.gpu


def _setup(cuda, B=384, K=2, scale=0.5, p=0.5):
    m = MNGP(scale, size=K, seed=3)
    g = Ray_Gate(K, seed=2)
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


def _run(fn, m, g, o, d, noise, seeds, cuda, esf):
    m.zero_grad(); g.zero_grad()
    to = lambda a: torch.from_numpy(a).to(cuda)
    res = fn(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=esf)
    torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]], [to(s) for s in seeds])
    grads = [m.xyz_encoder.params.grad.clone(), m.mlp_params.grad.clone(), g.params.grad.clone()]
    return res, grads


def check_grads_vs_oracle(m, gf, ores, tag):
    return check_grads(m.scale, gf[0].cpu().view(-1, 2).numpy(), ores["grid_grad"],
                       gf[1].cpu().numpy(), ores["mlp_grad"], gf[2].cpu().numpy(),
                       ores["gate_grad"], tag)


# fixed point vs fp32 atomics, per hash level: the largest record of a level
# maps to < 2^23 units (2^19 until round 2: measured max 3.7e-5 at scale 0.5,
# 1.2e-4 at scale 16; tcnn's own half2 atomics round each add to 2^-11 ~
# 4.9e-4)
FX_LEVEL_TOL = 3e-4


def check_fx_vs_fp32(m, g_fx, g_f32, r, tag):
    """Grid gradient of a fixed-point backward against the fp32 one of the
    same step, per hash level; MLP and gate gradients unchanged.  Returns the
    number of levels that ran in fixed point (scale != 0)."""
    acc, scales, vmax, redo = r.ws._fx
    used = scales[1 - r.ws.fx_i]          # the step just run (fx_i was swapped after it)
    assert int(redo[0]) == 0
    lv = LY.grid_levels(m.scale)
    a, b = g_fx[0].cpu().view(-1, 2).numpy(), g_f32[0].cpu().view(-1, 2).numpy()
    errs = []
    for l in range(16):
        o_, n_ = int(lv["offset"][l]), int(lv["hsize"][l])
        errs.append(_rel(a[o_:o_ + n_], b[o_:o_ + n_]))
    print(f"{tag}: fixed point vs fp32 per level max {max(errs):.2e}; "
          f"{int((used != 0).sum())} levels in fixed point")
    assert max(errs) <= FX_LEVEL_TOL, errs
    for x, y in zip(g_fx[1:], g_f32[1:]):
        assert float((x - y).norm() / y.norm().clamp_min(1e-30)) <= 1e-5
    return int((used != 0).sum())


def check_used_vs_oracle(w, ores, thr=1e-4):
    """Early-termination counts of the fused composite vs the oracle's, per
    (sub-NeRF, ray).  Both fold T serially with the same exponent; only the
    field's sigma differs (MFMA vs fp32 order, ~1e-6 relative), so a count may
    differ only where the oracle's transmittance at the break sits within
    1e-3 (relative) of T_threshold.  Returns the number of such rays."""
    used = w.used.cpu().numpy()
    cnt = w.counts.cpu().numpy()
    bad = 0
    for k in range(used.shape[0]):
        ou = ores["used"][k]
        diff = np.nonzero(ou != used[k])[0]
        for r in diff:
            n0 = int(ores["starts"][k, r]) - int(ores["starts"][k, 0])
            sig = ores["sigmas"][k][n0:n0 + cnt[k, r]].astype(np.float64)
            dl = ores["deltas"][int(ores["starts"][k, r]):int(ores["starts"][k, r]) + cnt[k, r]]
            T = np.cumprod(np.exp(-sig * dl))
            i = min(int(ou[r]), int(used[k, r]))
            assert abs(T[i] / thr - 1) < 1e-3, (k, r, ou[r], used[k, r], T[i])
            bad += 1
    return bad


# (scale, K, B): C3's shape (K = 2, scale 0.5); the scale-16 branches of C4
# (K = 4, exp step 1/256, 6 cascades, scripts/rad_360v2.sh:6-7) and C5 (K = 8,
# scripts/rad_free.sh:27-31) at batch sizes the CPU oracle finishes in seconds
@pytest.mark.parametrize("scale,K,B", [(0.5, 2, 384), (16.0, 2, 384), (0.5, 4, 384),
                                       (16.0, 4, 384), (16.0, 8, 256)])
def test_fused_vs_dropin_vs_oracle(cuda, scale, K, B):
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, scale=scale, K=K)
    # fixed point is the renderer's choice above 1024 rays x sub-NeRFs; these
    # oracle-sized batches check it too
    get_renderer(m, g, len(o)).grid_fx = True
    # the first fused backward accumulates the grid gradient in fp32 and
    # measures the records; the second runs the hashed levels in fixed point
    # (rn_grid_fx_fold): the one checked against the oracle below
    _, gf0 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    rf, gf = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    fx_used = check_fx_vs_fp32(m, gf, gf0, get_renderer(m, g, len(o)), f"s{scale} K{K}")
    rd, gd = _run(ml_render, m, g, o, d, noise, seeds, cuda, esf)
    for k in ("rgb", "opacity", "depth", "gating_code"):
        assert torch.allclose(rf[k], rd[k], atol=1e-5, rtol=0), k
    for a, b in zip(gf, gd):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel <= 1e-3, rel
    assert fx_used > 0
    ores = ml_oracle.ml_train_step(o, d, bits, noise, m.xyz_encoder.params.detach().cpu().view(-1, 2),
                                   m.mlp_params.detach().cpu(), g.params.detach().cpu(), scale,
                                   seeds=seeds)
    # fused march bit-exact vs oracle, per (model, ray) segment
    w = get_renderer(m, g, len(o)).ws
    cnt = w.counts.cpu().numpy()
    assert np.array_equal(cnt, ores["counts"])
    off = w.offsets.cpu().numpy()
    ts, dl = w.ts.cpu().numpy(), w.deltas.cpu().numpy()
    K, B = cnt.shape
    for k in range(K):
        for r in range(B):
            a, c = off[k, r], ores["starts"][k, r]
            n = cnt[k, r]
            assert np.array_equal(ts[a:a + n].view(np.uint32), ores["ts"][c:c + n].view(np.uint32))
            assert np.array_equal(dl[a:a + n].view(np.uint32), ores["deltas"][c:c + n].view(np.uint32))
    e_rgb = np.abs(rf["rgb"].detach().cpu().numpy() - ores["rgb"]).max()
    e_op = np.abs(rf["opacity"].detach().cpu().numpy() - ores["opacity"]).max()
    e_de = np.abs(rf["depth"].detach().cpu().numpy() - ores["depth"]).max()
    n_used = check_used_vs_oracle(w, ores)
    print(f"scale {scale} K {K} B {B}: {int(cnt.sum())} samples; rgb Linf {e_rgb:.2e} "
          f"opacity {e_op:.2e} depth {e_de:.2e}; termination counts off at {n_used} rays")
    # north_star bar: rgb / opacity / depth within 1e-4 of the reference path
    # (sigma and rgb leave the field in fp32, so no f16 output rounding reaches
    # the ray colour)
    assert e_rgb <= 1e-4 and e_op <= 1e-4 and e_de <= 1e-4
    check_grads_vs_oracle(m, gf, ores, f"s{scale} K{K}")


def test_workspace_reuse_is_caught(cuda):
    """A second autograd forward through the same renderer before the first
    one's backward raises; a no_grad render in between uses its own workspace
    and leaves the gradients unchanged."""
    B, K = 256, 2
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K)
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)    # fp32 step (fx scales)
    _, ref = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    to = lambda a: torch.from_numpy(a).to(cuda)
    m.zero_grad(); g.zero_grad()
    res = ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise))
    with torch.no_grad():
        ml_render_fused(m, g, to(o[::-1].copy()), to(d[::-1].copy()), to(d), noise=to(noise))
    torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]], [to(s) for s in seeds])
    for a, b in zip((m.xyz_encoder.params.grad, m.mlp_params.grad, g.params.grad), ref):
        assert float((a - b).norm() / b.norm()) <= 1e-5     # float-atomic order only
    res = ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise))
    ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise))
    with pytest.raises(RuntimeError, match="workspace was reused"):
        torch.autograd.backward([res["rgb"]], [to(seeds[0])])


@pytest.mark.parametrize("B,K,scale", [(1001, 2, 0.5), (777, 5, 0.5), (333, 8, 16.0)])
def test_fused_vs_dropin_ragged(cuda, B, K, scale):
    """Ragged batch sizes and K = 5 / 8 (merged forward with the MLP
    fragments in global memory, generic plan): the fused chain against the
    reference-structured drop-in chain, outputs and gradients."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    rf, gf = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    rd, gd = _run(ml_render, m, g, o, d, noise, seeds, cuda, esf)
    for k in ("rgb", "opacity", "depth", "gating_code"):
        assert torch.allclose(rf[k], rd[k], atol=1e-5, rtol=0), k
    for a, b in zip(gf, gd):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel <= 1e-3, rel


@pytest.mark.parametrize("B,K,scale", [(8192, 2, 0.5), (4096, 4, 16.0), (8192, 8, 16.0)])
def test_fused_full_size_properties(cuda, B, K, scale):
    """BASELINE configs at their full per-GPU sizes -- C3 (8192 rays, K = 2),
    C4 (16384 rays over 4 GPUs: 4096 x K = 4, scale 16) and C5 (65536 over 8:
    8192 x K = 8, scale 16): size-independent properties, and the backward's
    gradients finite with the merged order a permutation."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    to = lambda a: torch.from_numpy(a).to(cuda)
    res = ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=esf)
    r = get_renderer(m, g, B)
    w = r.ws
    cnt = w.counts.cpu().numpy().astype(np.int64)
    total = int(w.meta[1])
    assert total == cnt.sum() and total > 1_000_000
    assert cnt.max() <= 1024
    used = w.used.cpu().numpy()
    assert np.all((used >= 0) & (used <= cnt))
    # offsets: exclusive prefix per model, model bases aligned to 128
    off = w.offsets.cpu().numpy().astype(np.int64)
    base = w.seg_base.cpu().numpy()
    for k in range(K):
        assert base[k] % 128 == 0
        assert np.array_equal(off[k], base[k] + np.concatenate([[0], np.cumsum(cnt[k])[:-1]]))
    # t strictly increasing inside every segment (sampled rays)
    ts = w.ts.cpu().numpy()
    for k in range(K):
        for rr in range(0, B, 97):
            seg = ts[off[k, rr]:off[k, rr] + cnt[k, rr]]
            assert np.all(np.diff(seg) > 0)
    op = res["opacity"].detach().cpu().numpy()
    assert np.all(op >= -1e-6) and np.all(op <= 1 + 1e-5)
    gate = res["gating_code"].detach().cpu().numpy()
    assert np.allclose(gate.sum(1), 1, atol=1e-5)
    rgb = res["rgb"].detach().cpu().numpy()
    assert np.all(np.isfinite(rgb)) and rgb.min() >= -1e-5 and rgb.max() <= 1 + 1e-4
    # determinism of the forward (no atomics on the forward path)
    res2 = ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=esf)
    assert torch.equal(res["rgb"], res2["rgb"])
    torch.autograd.backward([res2["rgb"], res2["opacity"], res2["depth"]], [to(x) for x in seeds])
    for p in (m.xyz_encoder.params, m.mlp_params, g.params):
        assert torch.isfinite(p.grad).all() and p.grad.abs().max() > 0
    perm = w.perm[:total].cpu().numpy()
    assert int(w.mstart[B]) == total
    valid = np.zeros(w.capacity, bool)
    for k in range(K):
        valid[base[k]:base[k] + cnt[k].sum()] = True
    assert np.all(valid[perm]) and len(np.unique(perm)) == total


@pytest.mark.parametrize("B,K,scale", [(8192, 2, 0.5), (4096, 4, 16.0), (8192, 8, 16.0)])
def test_full_size_fx_vs_fp32(cuda, B, K, scale):
    """the default grid gradient at the full per-GPU sizes
    -- C3 (int32 fixed point), C4 and C5 (binned; C5 with 2048-sample chunks,
    hundreds of pages per level and the pool sized from the first step) --
    against the same step's fp32-atomic gradient, per level (FX_LEVEL_TOL),
    MLP and gate gradients unchanged; then two more default steps with
    identical inputs give identical bits (exact integer sums)."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    assert r.grid_fx and r.grid_bin == (scale > 0.5)
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)        # fp32: measures the scales
    _, gfx = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.grid_fx = False
    _, g32 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.grid_fx = True
    n_fx = check_fx_vs_fp32(m, gfx, g32, r, f"full size B{B} K{K} s{scale}")
    n32 = r.bin_f32_levels if r.grid_bin else 0      # binned: coarse levels by fp32 atomics
    assert n_fx == 16 - n32
    if r.grid_bin:
        pool = r.ws._bin
        assert 0 < int(pool["ctl"][0]) <= pool["pages"]
        assert 0 < int(pool["ctl"][1:17].sum()) <= int(pool["ctl"][0])   # pages with records listed
    _, gb = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    _, gc = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    assert int(r.ws._fx[3][0]) == 0
    lv = LY.grid_levels(scale)
    e = 2 * int(lv["offset"][n32])          # the fixed-point levels: identical bits
    assert torch.equal(gb[0][e:], gc[0][e:])
    if n32:
        a, b = gb[0][:e], gc[0][:e]
        assert float((a - b).norm() / b.norm().clamp_min(1e-30)) <= 1e-5


def _merged_vs_split(cuda, B, K, scale, p=0.5):
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale, p=p)
    r = get_renderer(m, g, B)
    out = []
    for merged in (True, False):
        r.merged_bwd = merged
        _, gr = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
        out.append(gr)
    r.merged_bwd = 1 <= K <= 8
    return r, out


@pytest.mark.parametrize("B,K,scale", [(8192, 2, 0.5), (2048, 4, 16.0), (1024, 1, 0.5),
                                       (512, 8, 0.5)])
def test_merged_backward_matches_per_model(cuda, B, K, scale):
    """rn_field_bwd_merged (K models' grid gradients scattered merged per ray)
    vs rn_field_bwd (one model per block): the same sums in another order; the
    merged kernel stages dL/dencoding as f16 in the block's gradient scale
    (as tcnn's f16 dL/dencoding), so its grid gradient is within f16 rounding
    (measured 9.4e-5) and the MLP / gate gradients agree to summation order."""
    r, (gm, gs) = _merged_vs_split(cuda, B, K, scale)
    for i, (a, b) in enumerate(zip(gm, gs)):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel <= (3e-4 if i == 0 else 1e-5), (i, rel)
    # merged order: ray-major, then t, ties by model (bit-exact)
    w = r.ws
    cnt = w.counts.cpu().numpy().astype(np.int64)
    off = w.offsets.cpu().numpy().astype(np.int64)
    ts = w.ts.cpu().numpy()
    smp, ray, mod = [], [], []
    for k in range(K):
        for rr in range(B):
            n = cnt[k, rr]
            smp.append(np.arange(off[k, rr], off[k, rr] + n)); ray.append(np.full(n, rr))
            mod.append(np.full(n, k))
    smp, ray, mod = map(np.concatenate, (smp, ray, mod))
    order = np.lexsort((mod, ts[smp], ray))
    total = len(smp)
    assert int(w.mstart[B]) == total
    assert np.array_equal(w.perm[:total].cpu().numpy(), smp[order])
    ms = w.mstart[:B].cpu().numpy()
    assert np.array_equal(ms, np.concatenate([[0], np.cumsum(cnt.sum(0))[:-1]]))


def test_merged_backward_chunking(cuda):
    """Small chunks (many queue grabs, single-ray chunks above max_chunk) and
    ramps of head chunks give the same gradients."""
    B, K = 2048, 2
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K)
    r = get_renderer(m, g, B)
    res = []
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)    # fp32 step (fx scales)
    head0 = r.head_chunk
    for mc, blocks, head in ((1024, 256, 0), (4096, 256, 0), (64, 37, 0), (300, 3, 0),
                             (1024, 256, 1024), (1536, 37, 900)):
        r.max_chunk, r.merged_blocks, r.head_chunk = mc, blocks, head
        _, gr = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
        res.append(gr)
    r.max_chunk, r.merged_blocks, r.head_chunk = 1024, 256, head0
    # other chunkings cut the walks' records elsewhere, so the fixed-point
    # rounding of the hashed levels differs (FX_LEVEL_TOL); MLP / gate: order only
    for other in res[1:]:
        for i, (a, b) in enumerate(zip(other, res[0])):
            rel = (a - b).norm() / b.norm().clamp_min(1e-30)
            assert rel <= (FX_LEVEL_TOL if i == 0 else 1e-5), rel


def _chunk_bounds(total, head_n, head, max_chunk, min_chunk, blocks):
    """host restatement of field.hip chunk_plan: the merged-position bound of
    every chunk (head chunks ramping from ~0 to head, big chunks over 15/16 of
    the work -- with blocks > 0 a multiple of blocks in number, each <=
    max_chunk -- then min_chunk)"""
    main_end = total - total // 16
    head_n = head_n if head > 0 and head * (head_n + 1) // 2 <= main_end else 0

    def hbound(c):
        return (head * c * (c + 1)) // (2 * head_n) if head_n else 0
    H = hbound(head_n)
    big, mm = max_chunk, 0
    if blocks > 0 and main_end > H:
        per = blocks * max_chunk
        mm = -(-(main_end - H) // per)
        big = min(max(-(-(main_end - H) // (blocks * mm)), min_chunk), max_chunk)
    c1 = head_n + ((main_end - H) // big if main_end > H else 0)

    def bound(c):
        if c < head_n:
            return hbound(c)
        if c <= c1:
            return H + (c - head_n) * big
        return H + (c1 - head_n) * big + (c - c1) * min_chunk
    rest = total - bound(c1)
    n = c1 + (-(-rest // min_chunk) if rest > 0 else 0)
    return [bound(c) for c in range(n)], c1 - head_n, big, mm


@pytest.mark.parametrize("B,K,scale,mc,bal,head", [(2048, 2, 0.5, 1536, 256, None),
                                                   (1024, 4, 16.0, 4096, 256, None),
                                                   (1024, 8, 16.0, 8192, 256, None),
                                                   (2048, 2, 0.5, 1536, 0, 0),
                                                   (512, 4, 16.0, 2560, 37, 2560),
                                                   (4096, 2, 0.5, 1024, 256, 700)])
def test_chunk_schedule(cuda, B, K, scale, mc, bal, head):
    """rn_bwd_plan's chunk list against the host restatement of its schedule:
    every chunk starts at the first ray whose merged start reaches its bound,
    the count is the plan's; balanced (balance_blocks > 0), no block has more
    big chunks to take than the others (C4 at 2560 left a few blocks one big
    chunk behind the rest).  head: the ramp of head chunks (None: the
    renderer's default, a ramp to max_chunk at scale 0.5)."""
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    r = get_renderer(m, g, B)
    head0 = r.head_chunk
    r.max_chunk, r.balance_chunks = mc, bal > 0
    if head is not None:
        r.head_chunk = head
    if bal:
        r.merged_blocks = bal
    _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    _, gr = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    w = r.ws
    torch.cuda.synchronize()
    ms = w.mstart[:B + 1].cpu().numpy().astype(np.int64)
    total = int(ms[B])
    head_n = r.merged_blocks if r.head_chunk else 0
    bounds, n_big, big, per_block = _chunk_bounds(total, head_n, min(r.head_chunk, mc), mc,
                                                  min(r.min_chunk, mc), bal)
    n = int(w.queue[1])
    assert n == len(bounds)
    first = r._chunks[:n + 1].cpu().numpy()
    assert np.array_equal(first[:n], np.searchsorted(ms[:B], np.array(bounds), side="left"))
    assert first[n] == B
    if bal and n_big and big > r.min_chunk:
        # at most per_block big chunks for every block, and nearly all take
        # that many (floor division leaves at most a few a chunk short)
        assert bal * (per_block - 1) < n_big <= bal * per_block and big <= mc, (n_big, big)
    r.max_chunk, r.merged_blocks, r.balance_chunks, r.head_chunk = mc, 256, True, head0
    assert all(torch.isfinite(x).all() for x in gr)


@pytest.mark.parametrize("B,K,scale", [(4096, 2, 0.5), (1024, 4, 16.0), (512, 1, 0.5),
                                     (768, 8, 16.0), (512, 5, 0.5)])
def test_merged_forward_matches_per_model(cuda, B, K, scale):
    """rn_field_fwd_merged (chunks of rays, models' tiles interleaved; encoded
    in merged order or per tile) vs rn_field_fwd: identical per-sample
    arithmetic, so sigma / rgb and the encoding cache are bit-exact."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    to = lambda a: torch.from_numpy(a).to(cuda)
    outs = []
    # merged kernel with merged-order encoding, with per-tile encoding, per-model
    # kernel, level-partitioned forward (rn_field_fwd_levels)
    for merged, enc, lv in ((True, True, False), (True, False, False), (False, False, False),
                            (True, True, True)):
        r.merged_fwd, r.merged_encode, r.level_fwd = merged, enc, lv
        ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=esf)
        w = r.ws
        off, cnt = w.offsets.cpu().numpy(), w.counts.cpu().numpy()
        idx = np.concatenate([np.arange(off[k, rr], off[k, rr] + cnt[k, rr])
                              for k in range(K) for rr in range(B)]).astype(np.int64)
        ii = torch.from_numpy(idx).to(cuda)
        feat = w.feat.view(-1, 64, 2, 8)       # [tile][lane][k-step][8]
        t, c = ii // 32, ii % 32
        cache = torch.stack([feat[t, c], feat[t, c + 32]], 1)
        outs.append((w.sigma[ii].clone(), w.rgb[ii].clone(), cache.clone()))
    r.merged_fwd, r.merged_encode, r.level_fwd = 1 < K <= 8, K > 1, True
    for o2 in outs[1:]:
        for a, b in zip(outs[0], o2):
            assert torch.equal(a, b)


@pytest.mark.parametrize("enc_blocks,mlp_blocks", [(8, 1), (24, 3), (8192, 512)])
def test_level_forward_launch_shapes(cuda, enc_blocks, mlp_blocks):
    """rn_field_fwd_levels with one block per level group (each block encodes
    every tile of its two levels), ragged splits and more blocks than tiles:
    bit-exact with the merged forward."""
    B, K = 2048, 3
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=16.0)
    r = get_renderer(m, g, B)
    to = lambda a: torch.from_numpy(a).to(cuda)
    outs = []
    for lv in (False, True):
        r.level_fwd = lv
        r.level_enc_blocks, r.level_mlp_blocks = enc_blocks, mlp_blocks
        ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=1 / 256)
        w = r.ws
        n = int(w.meta[0])
        outs.append((w.sigma[:n].clone(), w.rgb[:n].clone(), w.feat.clone()))
        w.feat.zero_()
    r.level_fwd, r.level_enc_blocks, r.level_mlp_blocks = True, 4096, 256
    w = r.ws
    off, cnt = w.offsets.cpu().numpy(), w.counts.cpu().numpy()
    idx = np.concatenate([np.arange(off[k, rr], off[k, rr] + cnt[k, rr])
                          for k in range(K) for rr in range(B)]).astype(np.int64)
    ii = torch.from_numpy(idx).to(cuda)
    for a, b in zip(outs[0][:2], outs[1][:2]):
        assert torch.equal(a[ii], b[ii])
    feat = [f.view(-1, 64, 16) for f in (outs[0][2], outs[1][2])]
    t, c = ii // 32, ii % 32
    for h in (0, 32):
        assert torch.equal(feat[0][t, c + h], feat[1][t, c + h])


@pytest.mark.parametrize("mc,blocks,threads", [(64, 3, 256), (300, 37, 1024), (4096, 256, 512)])
def test_merged_forward_chunking(cuda, mc, blocks, threads):
    """The merged forward's pipeline (merged-order encode of chunk i beside the
    MLP tiles of chunk i - 1) over many small chunks per block, ragged chunks
    and few blocks: still bit-exact with the per-model kernel."""
    B, K = 2048, 3
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K)
    r = get_renderer(m, g, B)
    to = lambda a: torch.from_numpy(a).to(cuda)
    outs = []
    for merged in (True, False):
        r.merged_fwd, r.merged_encode, r.level_fwd = merged, merged, False
        r.max_chunk, r.merged_fwd_blocks, r.merged_fwd_threads = mc, blocks, threads
        ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise))
        w = r.ws
        n = int(w.meta[0])
        outs.append((w.sigma[:n].clone(), w.rgb[:n].clone()))
    r.merged_fwd, r.merged_encode, r.max_chunk, r.level_fwd = True, True, 1024, True
    r.merged_fwd_blocks, r.merged_fwd_threads = 256, 1024
    # padding slots between segments are never written: compare the samples
    w = r.ws
    off, cnt = w.offsets.cpu().numpy(), w.counts.cpu().numpy()
    idx = np.concatenate([np.arange(off[k, rr], off[k, rr] + cnt[k, rr])
                          for k in range(K) for rr in range(B)]).astype(np.int64)
    ii = torch.from_numpy(idx).to(cuda)
    for a, b in zip(*outs):
        assert torch.equal(a[ii], b[ii])


@pytest.mark.parametrize("p,K", [(0.0, 2), (1.0, 3)])
def test_merged_backward_edge_occupancy(cuda, p, K):
    """Empty grid (no samples at all: zero chunks) and a full grid with K = 3
    (odd model count, many 1024-capped rays): merged = per-model backward."""
    B = 256
    r, (gm, gs) = _merged_vs_split(cuda, B, K, 0.5, p=p)
    for i, (a, b) in enumerate(zip(gm, gs)):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel <= (3e-4 if i == 0 else 1e-5), (i, rel)     # f16-staged dE (merged)
    if p == 0.0:
        assert int(r.ws.meta[1]) == 0
        assert float(gm[0].abs().max()) == 0.0


@pytest.mark.parametrize("B,K,scale", [(4096, 2, 0.5), (1024, 4, 16.0)])
def test_int_grad_matches_fp32(cuda, B, K, scale):
    """Exact integer accumulation of the grid gradient (returning u32 atomics +
    carries) vs fp32 atomics: equal up to the 2^-26-of-max-seed quantisation;
    bitwise reproducible across runs."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    r.int_grad = False
    _, gf = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.int_grad = True
    _, gi = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    _, gi2 = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, esf)
    r.int_grad = False
    rel = (gi[0] - gf[0]).norm() / gf[0].norm()
    assert rel <= 1e-5, rel
    assert torch.equal(gi[0], gi2[0])
    for a, b in zip(gi[1:], gf[1:]):
        assert ((a - b).norm() / b.norm()) <= 1e-5


@pytest.mark.parametrize("scale,K,B", [(0.5, 2, 256), (16.0, 4, 256)])
def test_input_grads_vs_oracle(cuda, scale, K, B):
    """--optimize_ext (train_ml.py:90-93): rays_o / rays_d require grad.  The
    gradients reach them through the gate input, the field's positions and
    directions (rn_field_dinput) and RayMarcher.backward (rn_ml_march_bw /
    rn_raymarching_train_bw): fused chain and drop-in chain vs the oracle's
    autograd + segment sums (custom_functions.py:102-112)."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    to = lambda a: torch.from_numpy(a).to(cuda)
    out = {}
    for name, fn in (("fused", ml_render_fused), ("dropin", ml_render)):
        m.zero_grad(); g.zero_grad()
        ot, dt = to(o).requires_grad_(True), to(d).requires_grad_(True)
        res = fn(m, g, ot, dt, dt, noise=to(noise), exp_step_factor=esf)
        torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]], [to(s) for s in seeds])
        out[name] = (ot.grad.cpu().numpy(), dt.grad.cpu().numpy(), m.mlp_params.grad.clone())
    ores = ml_oracle.ml_train_step(o, d, bits, noise, m.xyz_encoder.params.detach().cpu().view(-1, 2),
                                   m.mlp_params.detach().cpu(), g.params.detach().cpu(), scale,
                                   seeds=seeds, input_grads=True)
    rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    for name, (go, gd, mg) in out.items():
        eo, ed = rel(go, ores["drays_o"]), rel(gd, ores["drays_d"])
        print(f"input grads {name} scale {scale} K {K}: drays_o rel {eo:.2e}, drays_d rel {ed:.2e}")
        assert eo <= 3e-3 and ed <= 3e-3          # measured <= 1.0e-3
        # asking for input gradients leaves the parameter gradients as they were
        assert _rel(mg.cpu().numpy(), ores["mlp_grad"]) <= 4e-3
    assert rel(out["fused"][0], out["dropin"][0]) <= 1e-3
    assert rel(out["fused"][1], out["dropin"][1]) <= 1e-3


@pytest.mark.parametrize("K", [2, 4])
def test_fused_mostly_empty_rays(cuda, K):
    """Chunks are cut by merged sample positions, so a chunk spans every ray
    without samples between its first and last sample.  With 7 in 8 rays
    pointed away from the box, chunks hold thousands of empty rays: more than
    the merged backward stages in LDS (1,536), which then looks rays up in
    global memory.  Fused chain vs the drop-in chain: outputs and gradients."""
    B, scale = 8192, 0.5
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    o = o.copy()
    d = d.copy()
    away = np.arange(B) % 8 != 0
    d[away] = -d[away]                    # origins sit outside the box, aimed at it
    rf, gf = _run(ml_render_fused, m, g, o, d, noise, seeds, cuda, 0.0)
    w = get_renderer(m, g, B).ws
    cnt = w.counts.cpu().numpy().sum(0)
    assert (cnt[away] == 0).mean() > 0.99 and (cnt[~away] > 0).mean() > 0.9
    rd, gd = _run(ml_render, m, g, o, d, noise, seeds, cuda, 0.0)
    for k in ("rgb", "opacity", "depth", "gating_code"):
        assert torch.allclose(rf[k], rd[k], atol=1e-5, rtol=0), k
    for a, b in zip(gf, gd):
        rel = (a - b).norm() / b.norm().clamp_min(1e-30)
        assert rel <= 1e-3, rel


@pytest.mark.parametrize("B,K,scale", [(2048, 2, 0.5), (1024, 8, 16.0), (512, 1, 0.5)])
def test_plan_writes_level_forward_input(cuda, B, K, scale):
    """rn_bwd_plan with `prep` writes the level forward's per-position input
    (unit coordinates, sample id) as it places each sample; bit-identical to
    the separate prep pass of rn_field_fwd_levels (K = 2: the two-run merge;
    K = 8: the merge tree; K = 1: the rank path)."""
    esf = 1 / 256 if scale > 0.5 else 0.0
    m, g, o, d, noise, seeds, bits = _setup(cuda, B=B, K=K, scale=scale)
    r = get_renderer(m, g, B)
    to = lambda a: torch.from_numpy(a).to(cuda)
    preps = []
    for pp in (False, True):
        r.plan_prep, r.level_fwd = pp, True
        ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=esf)
        torch.cuda.synchronize()
        w = r.ws
        total = int(w.mstart[B])
        prep = w.level_buffers(torch.cuda.current_stream().cuda_stream)[1]
        preps.append(prep[:total].clone())
        prep.fill_(float("nan"))
    r.plan_prep = True
    assert preps[0].shape[0] > 0
    assert torch.equal(preps[0].view(torch.int32), preps[1].view(torch.int32))
