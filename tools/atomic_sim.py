"""Count the 64-B atomic requests the hash-grid gradient scatter issues on the
bench workload (dev tool, CPU only).

gfx950 float atomics run at the memory side at a fixed rate of 64-B requests
(MI355X_MICROARCH.md "Global float atomics"): the cost of field_bwd's scatter is
the number of distinct (wave instruction, 64-B segment) pairs.  This replays
the scatter's lane schedule on the oracle's samples (one sub-NeRF, 8192 rays,
occupancy p=0.5, scale 0.5) and prints requests/sample for:
  run    per-corner run merging (one emit per run of equal index)
  carry  corner hand-over between consecutive cells (field.hip grid_scatter_block)
  uniq   distinct segments per 256-sample block (lower bound for block-local dedupe)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rad-nerf_amd")]
import oracle  # noqa: E402
from radnerf_amd import layout as LY  # noqa: E402
from radnerf_amd import synthetic as S  # noqa: E402


def main(B=8192, scale=0.5):
    o, d = S.rays(B, scale, seed=0)
    bits = S.bitfields(1, 1, p=0.5, seed=1)
    nz = S.noise(1, B, seed=2)
    _, _, xyz, _, _, tot = oracle.ml_march(o, d, np.zeros(3, np.float32),
                                           np.full(3, scale, np.float32), nz, bits, 1, scale, 0.0)
    u = np.clip((xyz + scale) / (2 * scale), 0, 1).astype(np.float32)
    lv = LY.grid_levels(scale)
    N = (tot // 256) * 256
    u, nb = u[:N], N // 256
    cells, seg = [], np.zeros((16, 8, N), np.int64)
    for l in range(16):
        sc, res, hs = lv["scale"][l], int(lv["res"][l]), int(lv["hsize"][l])
        g = np.floor(sc * u + np.float32(0.5)).astype(np.int64)
        cells.append(g)
        for c in range(8):
            gx, gy, gz = g[:, 0] + (c & 1), g[:, 1] + ((c >> 1) & 1), g[:, 2] + (c >> 2)
            if res ** 3 <= hs:
                i = gx + gy * res + gz * res * res
            else:
                i = gx ^ ((gy * 2654435761) & 0xFFFFFFFF) ^ ((gz * 805459861) & 0xFFFFFFFF)
            seg[l, c] = ((i & 0xFFFFFFFF) % hs + int(lv["offset"][l])) // 8

    def requests(emit_fn):
        tot = 0
        for w in range(8):
            keys = []
            for l in (w, 15 - w):
                for c in range(8):
                    b_, h_, j_ = np.nonzero(emit_fn(l, c))
                    keys.append((b_ * 128 + j_) * (1 << 26) + seg[l, c].reshape(nb, 2, 128)[b_, h_, j_])
            tot += len(np.unique(np.concatenate(keys)))
        return tot / N

    def run_emit(l, c):
        ix = seg[l, c].reshape(nb, 2, 128) * 0 + cells_idx(l, c)
        nxt = np.concatenate([ix[:, :, 1:], np.full((nb, 2, 1), -1)], axis=2)
        return ix != nxt

    def cells_idx(l, c):
        g = cells[l].reshape(nb, 2, 128, 3)
        return ((g[..., 0] + (c & 1)) * 1_000_003 + (g[..., 1] + ((c >> 1) & 1))) * 1_000_003 \
            + g[..., 2] + (c >> 2)

    def carry_emit(l, c):
        g = cells[l].reshape(nb, 2, 128, 3)
        dlt = np.zeros_like(g)
        dlt[:, :, :-1] = g[:, :, 1:] - g[:, :, :-1]
        last = np.zeros((nb, 2, 128), bool)
        last[:, :, -1] = True
        m = [(c >> k) & 1 for k in range(3)]
        keep = np.ones((nb, 2, 128), bool)
        for k in range(3):
            keep &= (m[k] - dlt[..., k] >= 0) & (m[k] - dlt[..., k] <= 1)
        return ~keep | last

    uniq = 0
    for l in range(16):
        b = np.sort(seg[l].transpose(1, 0).reshape(nb, 256 * 8), axis=1)
        uniq += (np.diff(b, axis=1) != 0).sum() + nb
    print(f"samples {N}: requests/sample run {requests(run_emit):.1f}  "
          f"carry {requests(carry_emit):.1f}  uniq {uniq / N:.1f}")


if __name__ == "__main__":
    main()
