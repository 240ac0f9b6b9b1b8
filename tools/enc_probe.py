"""Level-partitioned forward probe (dev tool): times rn_field_fwd_levels
(each XCD encodes two levels of every sample into per-level planes, then the
MLP tiles read them) against the merged forward on the bench workload from
ABL_K / ABL_SCALE / ABL_RAYS, over ENC_BLOCKS x MLP_BLOCKS launch sizes, and
checks sigma, rgb and the encoding cache bitwise against it."""
import ctypes
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


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("ABL_RAYS", 8192))
    K = int(os.environ.get("ABL_K", 2))
    scale = float(os.environ.get("ABL_SCALE", 0.5))
    blocks = [int(x) for x in (os.environ.get("ENC_BLOCKS", "4096").split(","))]
    mblocks = [int(x) for x in (os.environ.get("MLP_BLOCKS", "1024").split(","))]
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
    L = lib()
    w = r.ws
    st = torch.cuda.current_stream().cuda_stream
    stride = w.feat.shape[0]
    planes = torch.zeros(16, stride, device=dev, dtype=torch.int32)
    prep = torch.zeros(stride, 4, device=dev, dtype=torch.float32)
    xq = torch.zeros(96, device=dev, dtype=torch.int32)
    lo, lh, lr, ls = m.xyz_encoder.level_ptrs()

    def levels(eb, mb, probe=False, feat=True):
        L.field_fwd_levels(w.ts.data_ptr(), w.ray_of.data_ptr(), o.data_ptr(), d.data_ptr(),
                           w.seg_base.data_ptr(), w.seg_count.data_ptr(), w.B, m.size,
                           m.xyz_encoder.params_f16().data_ptr(), lo, lh, lr, ls,
                           m._h_min.ctypes.data, m._h_ext.ctypes.data,
                           m.packed_frags().data_ptr(), w.sigma.data_ptr(), w.rgb.data_ptr(),
                           w.feat.data_ptr() if feat else None, w.mstart.data_ptr(),
                           w.perm.data_ptr(),
                           planes.data_ptr(), stride, prep.data_ptr(), 0, eb, mb,
                           xq.data_ptr() if probe else None, st)

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    # correctness: the level-partitioned forward vs the merged forward:
    # sigma, rgb and the encoding cache of every sample, bitwise
    r._field(True, o, d, st)
    torch.cuda.synchronize()
    P = int(w.mstart[w.B].item())
    s = w.perm[:P].long()
    F = w.feat.view(-1, 64, 16).view(torch.int32).view(-1, 64, 8)     # f16x2 words
    ref_sig, ref_rgb = w.sigma[s].clone(), w.rgb.view(-1, 3)[s].clone()
    ref_F = [F[s >> 5, (s & 31) + 32 * h].clone() for h in (0, 1)]
    w.sigma.zero_(); w.rgb.zero_(); w.feat.zero_()
    levels(blocks[0], mblocks[0], probe=True)
    torch.cuda.synchronize()
    res = {"samples": P,
           "sigma_mismatch": int((w.sigma[s] != ref_sig).sum().item()),
           "rgb_mismatch": int((w.rgb.view(-1, 3)[s] != ref_rgb).sum().item()),
           "cache_mismatch": sum(int((F[s >> 5, (s & 31) + 32 * h] != ref_F[h]).sum().item())
                                 for h in (0, 1)),
           "group_xcd_blocks": xq[:64].view(8, 8).tolist()}
    tt = xq[64:].view(torch.int64).cpu().numpy()
    res["group_span_us"] = [round(float(tt[8 + i] - tt[i]) / 100.0, 1) for i in range(8)]
    res["group_start_us"] = [round(float(tt[i] - tt[:8].min()) / 100.0, 1) for i in range(8)]
    t = {"fwd": [], "lv_nofeat": []}
    for eb in blocks:
        for mb in mblocks:
            t[f"lv_{eb}_{mb}"] = []
    for _ in range(7):
        t["fwd"].append(timed(lambda: r._field(True, o, d, st)))
        t["lv_nofeat"].append(timed(lambda: levels(blocks[0], mblocks[0], feat=False)))
        for eb in blocks:
            for mb in mblocks:
                t[f"lv_{eb}_{mb}"].append(timed(lambda: levels(eb, mb)))
    res.update({k: round(float(np.median(v)), 4) for k, v in t.items()})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
