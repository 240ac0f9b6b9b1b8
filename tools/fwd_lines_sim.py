"""Replay of the forward gather (dev tool, CPU only): distinct 128-B lines per
gather instruction of the x-pair encoder (lanes = 32 samples x the two
x-corners of one (level, row)), for 32-sample tiles cut from the per-model
compact order (k_field_fwd_merged today) vs from the merged (ray, t, model)
order (one tile mixing the sub-NeRFs of a ray stretch).

usage: python tools/fwd_lines_sim.py [B]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd"), os.path.join(ROOT, "tools")]
import oracle  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402


def samples(B, K=2, scale=0.5, p=0.5):
    o, d = S.rays(B, scale, seed=0)
    bits = S.bitfields(K, 1, p=p, seed=1)
    nz = S.noise(K, B, seed=2)
    cnt, st, xyz, ts, dl, tot = oracle.ml_march(o, d, np.zeros(3, np.float32),
                                                np.full(3, scale, np.float32), nz, bits, 1,
                                                scale, 0.0)
    ray = np.concatenate([np.repeat(np.arange(B), cnt[k]) for k in range(K)])
    mod = np.concatenate([np.full(cnt[k].sum(), k) for k in range(K)])
    u = np.clip((xyz + scale) / (2 * scale), 0, 1).astype(np.float32)
    return u, ray, mod, ts, LY.grid_levels(scale)


def lines(u, tiles, lv):
    """sum over tiles, levels, rows of the distinct lines of one instruction"""
    total = 0
    n_instr = 0
    for l in range(16):
        sc, res, hs, off = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l]), int(lv["offset"][l])
        g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
        for r in range(4):
            Y = g[:, 1] + (r & 1)
            Z = g[:, 2] + (r >> 1)
            ids = []
            for xb in (0, 1):
                X = g[:, 0] + xb
                if res ** 3 <= hs:
                    idx = (X + Y * res + Z * res * res) % hs
                else:
                    idx = (X ^ ((Y * 2654435761) & 0xFFFFFFFF) ^ ((Z * 805459861) & 0xFFFFFFFF)) % hs
                ids.append((idx + off) // 32)
            line = np.stack(ids, 1)                      # (n, 2)
            lt = line[tiles]                             # (n_tiles, 32, 2), -1 = empty lane
            lt = np.where((tiles >= 0)[..., None], lt, -1).reshape(len(tiles), 64)
            s = np.sort(lt, 1)
            d = (s[:, 1:] != s[:, :-1]) & (s[:, 1:] >= 0)
            total += int(d.sum() + (s[:, 0] >= 0).sum())
            n_instr += len(tiles)
    return total, n_instr


def cut(order, groups):
    """32-sample tiles of `order`, never crossing a group boundary"""
    tiles = []
    g = groups[order]
    bnd = np.r_[0, np.flatnonzero(g[1:] != g[:-1]) + 1, len(order)]
    for a, b in zip(bnd[:-1], bnd[1:]):
        for t in range(a, b, 32):
            row = order[t:min(t + 32, b)]
            tiles.append(np.r_[row, np.full(32 - len(row), -1)])
    return np.array(tiles)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    u, ray, mod, ts, lv = samples(B)
    n = len(u)
    per_model = cut(np.lexsort((ts, ray, mod)), mod)          # compact: model, ray, t
    merged = cut(np.lexsort((mod, ts, ray)), np.zeros(n, np.int64))
    for name, tiles in (("per-model tiles", per_model), ("merged-order tiles", merged)):
        tot, ni = lines(u, tiles, lv)
        print(f"{name}: {len(tiles)} tiles, {tot / n:.2f} lines/sample, {tot / ni:.2f} lines/instruction")


if __name__ == "__main__":
    main()
