"""Record count of the merged backward's grid walk (dev tool, CPU only;
VERDICT r03 item 1: pricing a store-and-sum grid-gradient scatter).

For the bench workload (K sub-NeRFs, scale, B rays) this replays the walk of
k_field_bwd_merged (tools/atomic_sim2.py: chunks of whole rays, 8 eighths,
row lanes holding the even-X and odd-X corners) and counts, per level:
  records   emitted entries (one entry = both features, 8 B of gradient)
  requests  64-B segments per 32-record issue (the atomic form's cost)
and the per-slice histogram of the records for a slice of S entries (the
store-and-sum form sums one slice per workgroup in LDS).  With --dup it also
prints, per level, the distinct entries of a chunk over its records: the most
a pass that combined a page's records of one entry could save (a page holds
part of one chunk's records of its level; round 6).

usage: python tools/records_sim.py K scale B [max_chunk] [slice_entries] [--dup]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tools")]
from atomic_sim2 import merged_samples, requests, streams  # noqa: E402


def records(u, lv, sid, dup=None):
    n = len(u)
    last = np.r_[sid[1:] != sid[:-1], True]
    per_level, offs = [], []
    chunk = sid // 8
    for l in range(16):
        sc, res, hs, off = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l]), int(lv["offset"][l])
        g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
        cnt = 0
        keys = []
        for slot in (0, 1):
            for lane in range(4):
                py, pz = lane & 1, lane >> 1
                c0 = g[:, 0] & 1
                X = g[:, 0] + (c0 if slot == 0 else 1 - c0)
                Y = g[:, 1] + ((py ^ g[:, 1]) & 1)
                Z = g[:, 2] + ((pz ^ g[:, 2]) & 1)
                if res ** 3 <= hs:
                    idx = (X + Y * res + Z * res * res) % hs
                else:
                    idx = (X ^ ((Y * 2654435761) & 0xFFFFFFFF) ^ ((Z * 805459861) & 0xFFFFFFFF)) % hs
                ent = (X * 4096 + Y) * 4096 + Z
                pos = np.flatnonzero(np.r_[ent[1:] != ent[:-1], True] | last)
                cnt += len(pos)
                offs.append(idx[pos] + off)
                keys.append(chunk[pos].astype(np.int64) * (1 << 21) + idx[pos])
        per_level.append(cnt / n)
        if dup is not None:
            k = np.concatenate(keys)
            dup.append(len(np.unique(k)) / max(1, len(k)))
    return np.array(per_level), np.concatenate(offs)


def main():
    show_dup = "--dup" in sys.argv
    sys.argv = [a for a in sys.argv if a != "--dup"]
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 16.0
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    mc = int(sys.argv[4]) if len(sys.argv) > 4 else 1536
    S = int(sys.argv[5]) if len(sys.argv) > 5 else 8192
    u, ray, lv = merged_samples(B, K=K, scale=scale)
    sid = streams(ray, mc)
    dup = [] if show_dup else None
    rec, offs = records(u, lv, sid, dup)
    req = requests(u, lv, sid, lane_major=True)
    n_ent = int(lv["n_entries"])
    hist = np.bincount(offs // S, minlength=(n_ent + S - 1) // S)
    print(f"K {K} scale {scale} B {B}: {len(u)} samples, chunk {mc}")
    print("  records/sample per level: " + " ".join(f"{r:.2f}" for r in rec))
    print(f"  records/sample {rec.sum():.2f}  requests/sample {req:.2f}  "
          f"records/request {rec.sum() / req:.2f}")
    if show_dup:
        print("  distinct entries / records per chunk, per level: " + " ".join(f"{d:.3f}" for d in dup))
    print(f"  slices of {S} entries: {len(hist)}; records/slice mean {hist.mean():.0f} "
          f"max {hist.max()} min {hist.min()} (max/mean {hist.max() / hist.mean():.2f})")


if __name__ == "__main__":
    main()
