"""Per-level encode cost of the level-partitioned forward (dev tool): the
group spans of rn_field_fwd_levels (xq probe) under several level pairings
(rn_set_level_pairing), solved by least squares for each level's time, then
the pairing that minimises the largest pair (heaviest level with lightest)
timed against the default (g, 15 - g).  Workload from ABL_K / ABL_SCALE /
ABL_RAYS (default C3)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from radnerf_amd import synthetic as S  # noqa: E402
from radnerf_amd._lib import lib  # noqa: E402
from radnerf_amd.fused import FusedMLRenderer  # noqa: E402
from radnerf_amd.networks import MNGP, Ray_Gate  # noqa: E402


def pack(pairs):
    v = 0
    for g, (a, b) in enumerate(pairs):
        v |= (a | (b << 4)) << (8 * g)
    return v


def main():
    dev = torch.device("cuda")
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
    bg = torch.ones(3, device=dev) if esf == 0 else torch.zeros(3, device=dev)
    r = FusedMLRenderer(m, g, B)
    r.forward(o, d, d, nz, bg, 1e-4, esf)
    torch.cuda.synchronize()
    L = lib()
    w = r.ws
    st = torch.cuda.current_stream().cuda_stream
    planes, prep = w.level_buffers(st)
    xq = torch.zeros(96, device=dev, dtype=torch.int32)
    lo, lh, lr, ls = m.xyz_encoder.level_ptrs()

    def run(probe):
        L.field_fwd_levels(w.ts.data_ptr(), w.ray_of.data_ptr(), o.data_ptr(), d.data_ptr(),
                           w.seg_base.data_ptr(), w.seg_count.data_ptr(), w.B, m.size,
                           m.xyz_encoder.params_f16().data_ptr(), lo, lh, lr, ls,
                           m._h_min.ctypes.data, m._h_ext.ctypes.data,
                           m.packed_frags().data_ptr(), w.sigma.data_ptr(), w.rgb.data_ptr(),
                           w.feat.data_ptr(), w.mstart.data_ptr(), w.perm.data_ptr(),
                           planes.data_ptr(), planes.shape[1], prep.data_ptr(), 0,
                           r.level_enc_blocks, r.level_mlp_blocks,
                           xq.data_ptr() if probe else None, st)

    def spans(pairs, reps=5):
        L.set_level_pairing(pack(pairs))
        out = []
        for _ in range(reps):
            run(True)
            torch.cuda.synchronize()
            tt = xq[64:].view(torch.int64).cpu().numpy()
            out.append([float(tt[8 + i] - tt[i]) / 100.0 for i in range(8)])
        return np.median(np.array(out), 0)

    def timed(pairs, reps=9):
        L.set_level_pairing(pack(pairs))
        t = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(False)
            b.record()
            torch.cuda.synchronize()
            t.append(a.elapsed_time(b))
        return float(np.median(t))

    P = [[(q, 15 - q) for q in range(8)], [(2 * q, 2 * q + 1) for q in range(8)],
         [(q, q + 8) for q in range(8)], [(q, 7 - q) if q < 4 else (q + 4, 15 - (q - 4)) for q in range(8)]]
    rows, rhs, meas = [], [], {}
    for pairs in P:
        s = spans(pairs)
        meas[str(pairs)] = [round(x, 1) for x in s]
        for (a, b), t in zip(pairs, s):
            row = np.zeros(16)
            row[a] += 1
            row[b] += 1
            rows.append(row)
            rhs.append(t)
    c, *_ = np.linalg.lstsq(np.array(rows), np.array(rhs), rcond=None)
    order = np.argsort(-c)
    best = [(int(order[q]), int(order[15 - q])) for q in range(8)]
    res = {"K": K, "scale": scale, "rays": B, "level_cost_us": [round(float(x), 1) for x in c],
           "spans": meas, "best_pairs": best,
           "best_pairing": hex(pack(best)),
           "fwd_ms_default": timed(P[0]), "fwd_ms_best": timed(best),
           "spans_best": [round(x, 1) for x in spans(best)]}
    L.set_level_pairing(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
