"""Per-level scatter form at C3 (dev tool, GPU): the
merged backward's grid gradient with levels [Lb, 16) binned (fx_mode 4: page
stores, k_grid_bin + k_grid_sum) and levels [0, Lb) scattered by atomics,
against today's all-atomic int32 form, on the bench workload (C3: 8192 rays,
K = 2, scale 0.5).  The non-binned levels of a binned launch go in by the
kernel's per-level fp32-atomic path (their scales zeroed before each
backward; fx_mode 4 has no int32 atomic form), a pessimistic stand-in for
int32 atomics on the coarse levels, which carry few requests.  Variants are
interleaved round by round; per variant: median step ms, field_bwd ms, the
fold's ms (int32: k_fx_fold span; binned: bin + check + sum) and, from the
all-binned run, each level's records per sample (the page fills).

    python tools/level_bin_probe.py [Lb ...]      (default 0 6 8 10 12 14)
    python tools/level_bin_probe.py atomic bin0 bin8 ...   (explicit variants)
(the renderer's own default of fp32 coarse levels, bin_f32_levels, is switched
off: every variant sets its cut here)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def main():
    toks = sys.argv[1:] or ["0", "6", "8", "10", "12", "14"]
    if all(t.isdigit() for t in toks):
        variants = ["atomic"] + [f"bin{t}" for t in toks]
    else:
        variants = toks
    dev = torch.device("cuda")
    B = int(os.environ.get("STEP_B", 8192))
    K = int(os.environ.get("STEP_K", 2))
    scale = float(os.environ.get("STEP_SCALE", 0.5))
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, m.cascades, p=0.5, seed=1)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale, seed=0))
    nz = [torch.from_numpy(S.noise(K, B, seed=2 + j)).to(dev) for j in range(4)]
    sd = [torch.from_numpy(a).to(dev) for a in S.loss_seeds(B, K, seed=4)]
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    gg = torch.zeros_like(m.xyz_encoder.params)
    mg = torch.zeros_like(m.mlp_params)
    ag = torch.zeros_like(g.params)
    state = {"cut": None}
    orig = r._field

    def patched(fwd, *a, **k):
        c = state["cut"]
        if not fwd and c and getattr(r.ws, "_fx", None) is not None:
            r.ws._fx[1][r.ws.fx_i][:c] = 0.0            # levels [0, c): fp32 atomics
        return orig(fwd, *a, **k)
    r._field = patched
    n_samples = []

    def step(i):
        gg.zero_()
        _, _, _, gt, _ = r.forward(o, d, d, nz[i % 4], bg, 1e-4, esf)
        n_samples.append(r.ws.meta[1].clone())
        r.backward(o, d, d, gt, bg, *sd, None, 1e-4, gg, mg, ag)

    def select(v):
        r.grid_bin = v != "atomic"
        r.bin_f32_levels = 0
        state["cut"] = int(v[3:]) if v.startswith("bin") else None

    times = {v: [] for v in variants}
    kern = {v: {"field_bwd": [], "fold": []} for v in variants}
    redo = {v: 0 for v in variants}
    per_level = None
    for rnd in range(6):
        for v in variants:
            select(v)
            for i in range(3):                          # scales follow the form
                step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(10):
                step(i)
            torch.cuda.synchronize()
            if rnd:
                times[v].append((time.perf_counter() - t0) / 10 * 1e3)
            # traced steps: field_bwd and the fold spans
            r.trace = {"field_bwd", "fx_bin", "fx_sum", "fx_fold"}
            r.events = {}
            for i in range(4):
                step(i)
                redo[v] += int(r.ws._fx[3][0])
            kt = r.kernel_times_ms()
            r.trace = False
            if rnd:
                kern[v]["field_bwd"] += kt.get("field_bwd", [])
                fold = [a + b for a, b in zip(kt.get("fx_bin", []), kt.get("fx_sum", []))] \
                    if v != "atomic" else kt.get("fx_fold", [])
                kern[v]["fold"] += fold
            if v == "bin0" and per_level is None:
                pool = r.ws._bin
                used = min(int(pool["ctl"][0]), int(pool["pages"]))
                meta = pool["meta"][:used].cpu().numpy().astype(np.int64)
                recs = np.bincount(meta & 0xff, weights=meta >> 8, minlength=16)
                per_level = (recs / float(n_samples[-1])).round(3).tolist()
    samples = float(torch.stack(n_samples[-10:]).float().mean())
    out = {"rays": B, "models": K, "scale": scale, "samples_per_step": samples,
           "records_per_sample_by_level": per_level,
           "variants": {v: {"step_ms": round(float(np.median(times[v])), 4),
                            "msamples_per_s": round(samples / float(np.median(times[v])) / 1e3, 1),
                            "field_bwd_ms": round(float(np.median(kern[v]["field_bwd"])), 4),
                            "fold_ms": round(float(np.median(kern[v]["fold"])), 4)
                            if kern[v]["fold"] else None,
                            "redo_steps": redo[v]} for v in variants}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
