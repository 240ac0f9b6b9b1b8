"""C3's int32 fixed-point grid gradient per entry, under variant units (dev
tool, GPU).  For the library in $RADNERF_LIB (variants
built with `make EXTRA="-DFX_TARGET_BITS=.. -DFX_ENTRY_BITS=.. -DFX_GROWTH_BITS=.."`)
and optionally levels forced to fp32 atomics ($FX_F32_LEVELS="4,5,6"; their
scales zeroed before every backward, the kernel's per-level fp32 path):

* one step fixed point vs fp32 atomics: non-zero fp32 entries that are 0 in
  fixed point, sign agreement above one unit, per level;
* 3 FusedAdam steps (eps 1e-15, train_ml.py:143) from one start with either
  gradient, and fp32 with the rays reversed (the floor): per-level update
  difference (what test_fx_per_entry_agreement prints);
* N steps with fresh rays and Adam: how many were flagged for the fp32 redo
  (a finer unit leaves less int32 headroom), and the median step time.

    RADNERF_LIB=.../librn_fx26.so python tools/fx_units_probe.py [B] [K] [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd._lib import LIB_PATH  # noqa: E402
from radnerf_amd.fused import get_renderer, ml_render_fused  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402
from radnerf_amd.optim import FusedAdam  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    scale = 0.5
    f32_levels = [int(x) for x in os.environ.get("FX_F32_LEVELS", "").split(",") if x]
    cuda = torch.device("cuda")
    m = MNGP(scale, size=K, seed=3)
    g = Ray_Gate(K, seed=2)
    with torch.no_grad():
        m.xyz_encoder.params.copy_(torch.from_numpy(S.grid_params(m.xyz_encoder.n_entries)).view(-1))
        m.mlp_params.copy_(torch.from_numpy(S.mlp_params(K, LY.FIELD_PARAMS)))
        g.params.copy_(torch.from_numpy(S.mlp_params(1, LY.gate_params(K), seed=6)[0]))
        bits = S.bitfields(K, m.cascades, p=0.5)
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    m, g = m.to(cuda), g.to(cuda)
    r = get_renderer(m, g, B)
    lv = LY.grid_levels(scale)

    orig = r._field

    def patched(fwd, *a, **k):
        if not fwd and f32_levels and r.grid_fx and getattr(r.ws, "_fx", None) is not None:
            r.ws._fx[1][r.ws.fx_i][f32_levels] = 0.0      # these levels: fp32 atomics
        return orig(fwd, *a, **k)
    r._field = patched

    def run(o, d, noise, seeds):
        m.zero_grad(); g.zero_grad()
        to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(cuda)
        res = ml_render_fused(m, g, to(o), to(d), to(d), noise=to(noise), exp_step_factor=0.0)
        torch.autograd.backward([res["rgb"], res["opacity"], res["depth"]], [to(s) for s in seeds])
        return m.xyz_encoder.params.grad.clone()

    def level(x, l):
        a, n = int(lv["offset"][l]), int(lv["hsize"][l])
        return x.view(-1, 2)[a:a + n]

    o, d = S.rays(B, scale)
    noise, seeds = S.noise(K, B), S.loss_seeds(B, K)
    run(o, d, noise, seeds)                      # the first (fp32) step measures the records
    run(o, d, noise, seeds)
    unit = (1.0 / r.ws._fx[1][r.ws.fx_i].abs().clamp_min(1e-30)).cpu()
    gfx = run(o, d, noise, seeds)
    redo_first = int(r.ws._fx[3][0])
    r.grid_fx = False
    g32 = run(o, d, noise, seeds)
    r.grid_fx = True
    per = []
    for l in range(16):
        a, b = level(gfx, l), level(g32, l)
        nz = b != 0
        big = b.abs() > float(unit[l])
        per.append(dict(level=l, nonzero=int(nz.sum()), flushed=int((nz & (a == 0)).sum()),
                        big=int(big.sum()),
                        sign_agree=int((torch.sign(a[big]) == torch.sign(b[big])).sum()),
                        unit=float(unit[l]), fp32_level=l in f32_levels))
    p0 = m.xyz_encoder.params.detach().clone()
    rev = (o[::-1].copy(), d[::-1].copy(), noise[:, ::-1].copy(), tuple(x[::-1].copy() for x in seeds))
    deltas = {}
    for mode in ("fx", "fp32", "fp32_reordered"):
        with torch.no_grad():
            m.xyz_encoder.params.copy_(p0)
        opt = FusedAdam([m.xyz_encoder.params], lr=1e-2, eps=1e-15)
        r.grid_fx = mode == "fx"
        args = rev if mode == "fp32_reordered" else (o, d, noise, seeds)
        for _ in range(3):
            run(*args)
            opt.step()
        deltas[mode] = (m.xyz_encoder.params.detach() - p0).view(-1, 2)
    r.grid_fx = True

    def upd(x, y):
        return [float((level(deltas[x], l) - level(deltas[y], l)).norm() /
                      level(deltas[y], l).norm().clamp_min(1e-30)) for l in range(16)]
    adam, floor = upd("fx", "fp32"), upd("fp32_reordered", "fp32")
    # training-like run: fresh rays every step, Adam on every parameter
    with torch.no_grad():
        m.xyz_encoder.params.copy_(p0)
    opt = FusedAdam([m.xyz_encoder.params, m.mlp_params, g.params], lr=1e-2, eps=1e-15)
    redo, ms = 0, []
    for i in range(n_steps):
        oo, dd = S.rays(B, scale, seed=100 + i)
        nn = S.noise(K, B, seed=200 + i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(oo, dd, nn, seeds)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        redo += int(r.ws._fx[3][0])
        opt.step()
    nz = sum(p["nonzero"] for p in per)
    out = dict(lib=os.path.basename(LIB_PATH), rays=B, models=K, f32_levels=f32_levels,
               flushed_frac=sum(p["flushed"] for p in per) / max(nz, 1),
               sign_agree=sum(p["sign_agree"] for p in per) / max(sum(p["big"] for p in per), 1),
               adam3_max=max(adam), adam3_level=int(np.argmax(adam)),
               adam3=[round(x, 5) for x in adam], floor=[round(x, 5) for x in floor],
               redo_first=redo_first, steps=n_steps, redo_steps=redo,
               step_ms_median=round(float(np.median(ms)), 3), levels=per)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
