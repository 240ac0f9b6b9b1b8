"""Replay of k_field_bwd_merged's grid scatter on the bench workload (dev
tool, CPU only): counts the 64-B atomic requests (distinct segments per wave
instruction) of the row-lane walk with per-stream rings, and of variants.

Scheme (field.hip walk2_*): the merged (ray, t, model) order is cut into
chunks of whole rays (max_chunk, tail min_chunk), each chunk into 8 eighths;
a stream = (eighth, level) walks its samples in order; lane (py, pz) holds the
even-X and odd-X corners of its row; an entry is emitted when it leaves; a
stream's records are issued 32 at a time in emission order (slot 0 lanes
0-3, then slot 1 lanes 0-3 within a step); every chunk ends with a flush.

usage: python tools/atomic_sim2.py [B] [max_chunk] [issue]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import oracle  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402


def merged_samples(B, K=2, scale=0.5, p=0.5):
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
    order = np.lexsort((mod, ts, ray))
    u = np.clip((xyz + scale) / (2 * scale), 0, 1).astype(np.float32)[order]
    return u, ray[order], LY.grid_levels(scale)


def streams(ray, max_chunk, min_chunk=512, parts=8):
    """stream id (chunk * parts + part) per merged position, positions in order."""
    n = len(ray)
    first = np.r_[0, np.flatnonzero(np.diff(ray)) + 1]          # ray starts
    c1 = (n - n // 8) // max_chunk
    bounds = []
    c = 0
    while True:
        b = c * max_chunk if c <= c1 else c1 * max_chunk + (c - c1) * min_chunk
        if b >= n:
            break
        bounds.append(b)
        c += 1
    ix = np.searchsorted(first, bounds)                         # first ray start >= bound
    starts = np.unique(first[ix[ix < len(first)]])
    chunk = np.searchsorted(starts, np.arange(n), side="right") - 1
    cstart = starts[chunk]
    cend = np.r_[starts[1:], n][chunk]
    clen = cend - cstart
    E = (clen + parts - 1) // parts
    part = (np.arange(n) - cstart) // E
    return chunk * parts + part


def requests(u, lv, sid, issue=32, levels=range(16), lane_major=False, cut_min=0, ent_per_seg=8,
             sort_window=0):
    n = len(u)
    total = 0
    last = np.r_[sid[1:] != sid[:-1], True]                      # last sample of a stream
    for l in levels:
        sc, res, hs, off = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l]), int(lv["offset"][l])
        g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
        keys, segs = [], []
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
                seg = (idx + off) // ent_per_seg
                ent = (X * 4096 + Y) * 4096 + Z
                # entry at position i leaves at i+1 if the next entry differs (same stream),
                # or at the stream end (flush after the last step)
                nxt_diff = np.r_[ent[1:] != ent[:-1], True] | last
                pos = np.flatnonzero(nxt_diff)
                step = pos + 1                                     # emitted at the next step
                # order within a stream: (step, slot, lane); flush records after all steps
                keys.append(np.stack([sid[pos], step, np.full(len(pos), slot), np.full(len(pos), lane)], 1))
                segs.append(seg[pos])
        k = np.concatenate(keys)
        s = np.concatenate(segs)
        o = (np.lexsort((k[:, 2], k[:, 3], k[:, 1], k[:, 0])) if lane_major
             else np.lexsort((k[:, 3], k[:, 2], k[:, 1], k[:, 0])))
        k, s = k[o], s[o]
        st = k[:, 0]
        if sort_window:
            # rings of sort_window records: when full, issue the 32 smallest segments
            bnd = np.r_[np.flatnonzero(np.r_[True, st[1:] != st[:-1]]), len(st)]
            req = 0
            for a, b in zip(bnd[:-1], bnd[1:]):
                pend = []
                for x in s[a:b]:
                    pend.append(x)
                    if len(pend) >= sort_window:
                        pend.sort()
                        req += len(set(pend[:issue]))
                        pend = pend[issue:]
                while pend:
                    pend.sort()
                    req += len(set(pend[:issue]))
                    pend = pend[issue:]
            total += req
            continue
        if cut_min:
            # cut each instruction at a segment boundary (largest k in [cut_min, issue])
            grp = np.empty(len(st), np.int64)
            bnd = np.r_[np.flatnonzero(np.r_[True, st[1:] != st[:-1]]), len(st)]
            g = 0
            for a, b in zip(bnd[:-1], bnd[1:]):
                r = a
                while r < b:
                    e = min(r + issue, b)
                    if e < b and s[e - 1] == s[e]:
                        for e2 in range(e - 1, r + cut_min - 1, -1):
                            if s[e2 - 1] != s[e2]:
                                e = e2
                                break
                    grp[r:e] = g
                    g += 1
                    r = e
            total += len(np.unique(grp * (1 << 30) + s))
            continue
        # rank within stream -> instruction group
        newst = np.r_[True, st[1:] != st[:-1]]
        first_idx = np.maximum.accumulate(np.where(newst, np.arange(len(st)), 0))
        rank = np.arange(len(st)) - first_idx
        grp = st * 100000 + rank // issue
        total += len(np.unique(grp * (1 << 30) + s))
    return total / n


def floor(u, ray, lv, ent_per_seg=8):
    """distinct (ray, level, segment) triples per sample: every corner entry of
    a ray's samples, all K models merged, one request per distinct segment"""
    n = len(u)
    total = 0
    for l in range(16):
        sc, res, hs, off = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l]), int(lv["offset"][l])
        g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
        segs = []
        for c in range(8):
            X, Y, Z = g[:, 0] + (c & 1), g[:, 1] + ((c >> 1) & 1), g[:, 2] + (c >> 2)
            if res ** 3 <= hs:
                idx = (X + Y * res + Z * res * res) % hs
            else:
                idx = (X ^ ((Y * 2654435761) & 0xFFFFFFFF) ^ ((Z * 805459861) & 0xFFFFFFFF)) % hs
            segs.append((idx + off) // ent_per_seg)
        key = np.stack([np.repeat(ray[None], 8, 0).ravel(), np.concatenate(segs)], 1)
        total += len(np.unique(key, axis=0))
    return total / n


def eps_floor(argv):
    return int(argv[7]) if len(argv) > 7 else 8


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    mc = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    issue = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    parts = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    lane_major = len(sys.argv) > 5 and sys.argv[5] == "lane"
    cut_min = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    eps = int(sys.argv[7]) if len(sys.argv) > 7 else 8
    sw = int(sys.argv[8]) if len(sys.argv) > 8 else 0
    scale = float(os.environ.get("SIM_SCALE", 0.5))
    K = int(os.environ.get("SIM_K", 2))
    u, ray, lv = merged_samples(B, K=K, scale=scale)
    if os.environ.get("SIM_FLOOR"):
        print(f"scale {scale} K {K} B {B}: floor {floor(u, ray, lv, eps_floor(sys.argv)):.2f} "
              f"requests/sample")
    sid = streams(ray, mc, parts=parts)
    print(f"B {B} samples {len(u)} max_chunk {mc} issue {issue} parts {parts} "
          f"{'lane' if lane_major else 'slot'}-major: "
          f"requests/sample {requests(u, lv, sid, issue, lane_major=lane_major, cut_min=cut_min, ent_per_seg=eps, sort_window=sw):.2f} (cut_min {cut_min}, entries/segment {eps}, sort window {sw})")


if __name__ == "__main__":
    main()
