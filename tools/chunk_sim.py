"""Scale-16 replay (dev tool, CPU only): how far can
cross-ray sharing cut the merged backward's atomic requests and the forward's
gathered lines at C4 / C5?

For the oracle march of the bench workload (K sub-NeRFs, scale, B rays):
  walk       requests/sample of k_field_bwd_merged's walk (tools/atomic_sim2.py)
  ray floor  distinct (ray, level, 64-B segment) per sample: the per-ray merge
  chunk floor distinct (chunk, level, segment) per sample: every record of a
             chunk of whole rays aggregated before issue (an ideal LDS
             pre-aggregation of the chunk)
  fwd lines  distinct 128-B lines per sample of the forward's 32-sample tiles
             (x-pair rows per (level, row), tools/fwd_lines_sim.py)
each for the bench's ray order and for rays pre-sorted spatially (Morton key of
the quantised box entry and exit points: nearly coincident segments adjacent).

usage: python tools/chunk_sim.py K scale B [max_chunk]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tools")]
import oracle  # noqa: E402
from atomic_sim2 import requests, streams  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402


def march(B, K, scale, p=0.5):
    o, d = S.rays(B, scale, seed=0)
    C = LY.cascades_for_scale(scale)
    bits = S.bitfields(K, C, p=p, seed=1)
    nz = S.noise(K, B, seed=2)
    esf = 1 / 256 if scale > 0.5 else 0.0
    cnt, st, xyz, ts, dl, tot = oracle.ml_march(o, d, np.zeros(3, np.float32),
                                                np.full(3, scale, np.float32), nz, bits, C,
                                                scale, esf)
    ray = np.concatenate([np.repeat(np.arange(B), cnt[k]) for k in range(K)])
    mod = np.concatenate([np.full(cnt[k].sum(), k) for k in range(K)])
    u = np.clip((xyz + scale) / (2 * scale), 0, 1).astype(np.float32)
    return o, d, u, ray, mod, ts


def spatial_rank(o, d, scale, bits=5):
    """rank of each ray by the Morton key of its quantised box entry and exit
    points (6 coordinates x `bits` bits)"""
    inv = 1.0 / np.where(np.abs(d) < 1e-12, 1e-12, d)
    t0 = (-scale - o) * inv
    t1 = (scale - o) * inv
    tn = np.minimum(t0, t1).max(1)
    tf = np.maximum(t0, t1).min(1)
    pe = np.clip((o + tn[:, None] * d + scale) / (2 * scale), 0, 1)
    px = np.clip((o + tf[:, None] * d + scale) / (2 * scale), 0, 1)
    q = np.concatenate([pe, px], 1)
    qi = np.minimum((q * (1 << bits)).astype(np.int64), (1 << bits) - 1)
    key = np.zeros(len(o), np.int64)
    for b in range(bits - 1, -1, -1):
        for c in range(6):
            key = (key << 1) | ((qi[:, c] >> b) & 1)
    rank = np.empty(len(o), np.int64)
    rank[np.argsort(key, kind="stable")] = np.arange(len(o))
    return rank


def seg_ids(u, lv, l, c, per=8):
    sc, res, hs, off = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l]), int(lv["offset"][l])
    g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
    X, Y, Z = g[:, 0] + (c & 1), g[:, 1] + ((c >> 1) & 1), g[:, 2] + (c >> 2)
    if res ** 3 <= hs:
        idx = (X + Y * res + Z * res * res) % hs
    else:
        idx = (X ^ ((Y * 2654435761) & 0xFFFFFFFF) ^ ((Z * 805459861) & 0xFFFFFFFF)) % hs
    return (idx + off) // per


def distinct_per(u, group, lv, per=8):
    """distinct (group, level, segment) per sample"""
    total = 0
    for l in range(16):
        s = np.concatenate([seg_ids(u, lv, l, c, per) for c in range(8)])
        gg = np.tile(group, 8)
        total += len(np.unique(gg * (1 << 32) + s))
    return total / len(u)


def fwd_lines(u, lv, order):
    """distinct 128-B lines per sample, 32-sample tiles of `order`, x-pair rows"""
    n = len(order)
    tiles = np.arange(n) // 32
    total = 0
    for l in range(16):
        for r in range(4):
            c0 = (r & 1) * 2 + (r >> 1) * 4
            ids = np.stack([seg_ids(u, lv, l, c0, 32), seg_ids(u, lv, l, c0 + 1, 32)], 1)[order]
            key = np.repeat(tiles, 2) * (1 << 32) + ids.ravel()
            total += len(np.unique(key))
    return total / n


def merged_order(ray, mod, ts):
    return np.lexsort((mod, ts, ray))


def report(tag, u, ray, mod, ts, lv, mc):
    o = merged_order(ray, mod, ts)
    um, rm = u[o], ray[o]
    sid = streams(rm, mc)
    chunk = sid // 8
    walk = requests(um, lv, sid, 32, lane_major=True)
    rf = distinct_per(um, rm, lv)
    cf = distinct_per(um, chunk, lv)
    fl = fwd_lines(u, lv, o)
    print(f"  {tag:14s} walk {walk:6.2f}  ray floor {rf:6.2f}  chunk floor {cf:6.2f}  "
          f"fwd lines/sample {fl:6.2f}", flush=True)
    return walk, rf, cf, fl


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 16.0
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    mc = int(sys.argv[4]) if len(sys.argv) > 4 else (2048 if K >= 8 else 1024)
    o, d, u, ray, mod, ts = march(B, K, scale)
    lv = LY.grid_levels(scale)
    print(f"K {K} scale {scale} B {B}: {len(u)} samples, chunk {mc} merged samples; "
          f"requests (64-B segments) / sample, forward lines (128 B) / sample", flush=True)
    base = report("bench order", u, ray, mod, ts, lv, mc)
    rk = spatial_rank(o, d, scale)
    srt = report("rays sorted", u, rk[ray], mod, ts, lv, mc)
    print(f"  sorted vs bench: walk {srt[0] / base[0] - 1:+.1%}, chunk floor "
          f"{srt[2] / base[0] - 1:+.1%} of the walk, fwd lines {srt[3] / base[3] - 1:+.1%}")


if __name__ == "__main__":
    main()
