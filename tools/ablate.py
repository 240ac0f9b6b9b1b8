"""Kernel ablation on the bench workload (dev tool): times field_bwd with parts
switched off (rn_set_debug_flags) interleaved in one process (rule 24 of
cdna_hip_programming.md §5.4).  bit0: no grid atomics, bit1: no dW, bit2: no
grid scatter at all, bit5 (32): rows staged but no walk (merged kernel).
Token prefixes: none = merged backward (fixed-point hashed levels: the
_field call includes rn_grid_fx_fold and the redo launch), "x" = merged
backward with fp32 grid atomics, "s" = per-model backward, "i" = merged
backward with integer accumulation, "a" = merged backward with the int32
atomic scatter where the binned one is the default (scale 16), "f" = field_fwd.
Workload from ABL_K / ABL_SCALE / ABL_RAYS (default C3)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd._lib import lib, use_ablation_build  # noqa: E402

use_ablation_build()        # rn_set_debug_flags switches live only in librn_abl.so
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def main():
    flags = sys.argv[1:] or ["0", "1", "2", "4", "6"]
    dev = torch.device("cuda")
    # workload from the environment (default: the C3 headline)
    B = int(os.environ.get("ABL_RAYS", 8192))
    K = int(os.environ.get("ABL_K", 2))
    scale = float(os.environ.get("ABL_SCALE", 0.5))
    esf = 1.0 / 256 if scale > 0.5 else 0.0
    m = MNGP(scale, size=K, seed=3).to(dev)
    g = Ray_Gate(K, seed=4).to(dev)
    bits = S.bitfields(K, m.cascades, p=0.5)
    with torch.no_grad():
        for i in range(K):
            getattr(m, f"density_bitfield_{i}").copy_(torch.from_numpy(bits[i]))
    o, d = (torch.from_numpy(a).to(dev) for a in S.rays(B, scale))
    nz = torch.from_numpy(S.noise(K, B)).to(dev)
    sd = [torch.from_numpy(a).to(dev) for a in S.loss_seeds(B, K)]
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    gg = torch.zeros_like(m.xyz_encoder.params)
    mg = torch.zeros_like(m.mlp_params)
    ag = torch.zeros_like(g.params)
    rens = {}
    for key in ("", "a"):          # "a": the int32 atomic scatter (own workspace and scales)
        rr = FusedMLRenderer(m, g, B)
        if key == "a":
            rr.grid_bin = False
        for _ in range(2):         # the first backward is fp32 and sets the scales
            _, _, _, gt, _ = rr.forward(o, d, d, nz, bg, 1e-4, esf)
            rr.backward(o, d, d, gt, bg, *sd, None, 1e-4, gg, mg, ag)
        rr.trace = {"field_bwd", "fx_fold", "fx_bin", "fx_sum", "fx_redo"}
        rens[key] = rr
    kern = {}
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    # tokens: "<flags>" = field_bwd (merged) with debug flags, "s<flags>" = the
    # per-model field_bwd, "f<flags>" = field_fwd
    times = {f: [] for f in flags}
    phases = {}
    fwd = []
    for rnd in range(5):
        for f in flags:
            L.set_debug_flags(int(f.lstrip("fsixa")))
            r = rens["a" if f.startswith("a") else ""]
            r.events = {}
            # the fixed-point scales as the primed steps left them: a timing
            # flag (no records, no vmax) must not steer the next token's scales
            fx = getattr(r.ws, "_fx", None)
            if fx is not None:
                if not hasattr(r, "_abl_fx"):
                    r._abl_fx = (fx[1].clone(), r.ws.fx_i)
                fx[1].copy_(r._abl_fx[0])
                r.ws.fx_i = r._abl_fx[1]
                fx[3].zero_()
            r.merged_bwd = not f.startswith("s")
            r.int_grad = f.startswith("i")
            r.grid_fx = not f.startswith("x")      # "x": fp32 grid atomics
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            if f.startswith("f"):
                r._field(True, o, d, st)
            else:
                r._field(False, o, d, st, gg, mg)
            b.record()
            torch.cuda.synchronize()
            times[f].append(a.elapsed_time(b))
            for kname, v in r.kernel_times_ms().items():
                kern.setdefault(f, {}).setdefault(kname, []).extend(v)
            if int(f.lstrip("fsixa")) & 4096:
                cyc = (ctypes.c_ulonglong * 8)()
                L.debug_cycles(ctypes.cast(cyc, ctypes.c_void_p).value)
                phases.setdefault(f, []).append([int(c) for c in cyc[:8]])
        L.set_debug_flags(0)
        r = rens[""]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        r._field(True, o, d, st)
        b.record()
        torch.cuda.synchronize()
        fwd.append(a.elapsed_time(b))
    out = {"samples": r.ws.n_samples(), "field_fwd_ms": float(np.median(fwd)),
           "field_bwd_ms": {str(f): float(np.median(v)) for f, v in times.items()
                            if not f.startswith("f")},
           "field_fwd_flags_ms": {str(f): float(np.median(v)) for f, v in times.items()
                                  if f.startswith("f")},
           # the launches alone (HIP events on the launch stream): the merged
           # backward and, fixed point, its fold (bin + check + sum when binned)
           "kernel_ms": {f: {k: round(float(np.median(v)), 4) for k, v in kv.items()}
                         for f, kv in kern.items()},
           # flag 4096: summed wave cycles per phase (MLP, staging, walk, chunk
           # tails), median over rounds, as fractions of their sum; inside the
           # MLP phase: model switches, forward recompute (its loads waited
           # for), bwd_window, row stores (fractions of the MLP phase)
           "phases": {f: dict(zip(("mlp", "staging", "walk", "tail"),
                                  [round(float(x), 4) for x in
                                   (np.median(np.array(v)[:, :4], 0) /
                                    np.median(np.array(v)[:, :4], 0).sum())]))
                      for f, v in phases.items()},
           "mlp_phases": {f: dict(zip(("switch", "forward", "bwd_window", "rows"),
                                      [round(float(x), 4) for x in
                                       (np.median(np.array(v)[:, 4:], 0) /
                                        max(1.0, float(np.median(np.array(v)[:, 0]))))]))
                          for f, v in phases.items()},
           # the same summed wave cycles, absolute (medians over rounds)
           "phase_cycles": {f: [float(x) for x in np.median(np.array(v), 0)]
                            for f, v in phases.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
