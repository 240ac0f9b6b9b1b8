"""Host-side layout tables for the HIP kernels.

* hash-grid level tables following tinycudann's GridEncoding (the absent
  third-party dependency behind models/networks.py:229-247): per-level scale,
  resolution, entry count (params_in_level) and offset;
* MFMA fragment permutations: which fp32 master weight each (fragment, lane,
  element) slot of the packed f16 weights holds (see csrc/rn_mlp.h for the
  lane maps and the k-permutation  16s + 8(j>>2) + 4h + (j&3));
* weight-gradient maps: which master parameter each (tile, acc reg, lane)
  element of the dW MFMA output accumulates into.

Master parameter layouts (fp32, row-major [out][in], no padding):
  field (per sub-NeRF, 9472):  Wg1[64,32] | Wg2[17,64] | Wr1[64,32] | Wr2[64,64] | Wr3[3,64]
  gate  (12672 + 64K):         W0[64,6] | W1[64,64] | W2[64,64] | W3[64,64] | W4[K,64]
These mirror tcnn's FullyFusedMLP (no bias, ReLU, geo 32->64->17, rgb
32->64->64->3, gate 6->64x4->K) of models/networks.py:269-289,1075-1085.
"""
import math

import numpy as np

N_LEVELS = 16
N_FEATURES = 2
N_MIN = 16

# ---------------------------------------------------------------------------
# hash grid
# ---------------------------------------------------------------------------


def per_level_scale(scale):
    """networks.py:230  b = exp(log(2048*scale/N_min)/(L-1)), as tcnn's float."""
    return np.float32(np.exp(np.log(2048 * scale / N_MIN) / (N_LEVELS - 1)))


def grid_levels(scale, log2_hashmap_size=19):
    """tcnn GridEncodingTemplated level table.

    Returns dict of numpy arrays (offset u32, hsize u32, res u32, scale f32),
    total entry count and the per-level scale b.
    """
    b = per_level_scale(scale)
    # std::log2(float) and exp2f, both correctly rounded to f32
    log2b = np.float32(math.log2(float(b)))
    T = 1 << log2_hashmap_size
    max_params = np.iinfo(np.uint32).max // 2
    offs, hs, res, sc = [], [], [], []
    offset = 0
    for l in range(N_LEVELS):
        e = np.float32(2.0 ** float(np.float32(l) * log2b))
        s = np.float32(e * np.float32(N_MIN) - np.float32(1.0))
        r = int(math.ceil(float(s))) + 1
        p = min(r ** 3, max_params) if float(r) ** 3 <= max_params else max_params
        p = (p + 7) // 8 * 8
        p = min(p, T)
        offs.append(offset)
        hs.append(p)
        res.append(r)
        sc.append(s)
        offset += p
    return {
        "offset": np.array(offs, dtype=np.uint32),
        "hsize": np.array(hs, dtype=np.uint32),
        "res": np.array(res, dtype=np.uint32),
        "scale": np.array(sc, dtype=np.float32),
        "n_entries": offset,
        "per_level_scale": b,
    }


def cascades_for_scale(scale):
    """networks.py:259  max(1 + ceil(log2(2*scale)), 1)."""
    return max(1 + int(np.ceil(np.log2(2 * scale))), 1)


# ---------------------------------------------------------------------------
# MLP fragments
# ---------------------------------------------------------------------------
FIELD_SIZES = {"g1": (64, 32), "g2": (17, 64), "r1": (64, 32), "r2": (64, 64), "r3": (3, 64)}
FIELD_OFF = {"g1": 0, "g2": 2048, "r1": 3136, "r2": 5184, "r3": 9280}
FIELD_PARAMS = 9472
FIELD_FWD_FRAGS = 24
FIELD_FRAGS = 46
FIELD_DW_TILES = 12

GATE_FWD_FRAGS = 30
GATE_FRAGS = 56
GATE_DW_TILES = 16
GATE_HIDDEN = 64


def gate_offsets(K):
    return {"w0": 0, "w1": 384, "w2": 384 + 4096, "w3": 384 + 8192, "w4": 384 + 12288}


def gate_params(K):
    return 12672 + 64 * K


def _perm(s, h, j):
    return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)


def _kin(q, h, j):
    """input index of element j, lane half h, k-step q of a multi-tile acc input."""
    return 32 * (q >> 1) + _perm(q & 1, h, j)


def _geo_out(row):
    """geo acc row -> geo output index (rows 0..15 = outputs 1..16, row 16 = output 0)."""
    if row < 16:
        return row + 1
    if row == 16:
        return 0
    return -1


def _w(name, o, i, sizes=FIELD_SIZES, offs=FIELD_OFF):
    rows, cols = sizes[name]
    if o < 0 or i < 0 or o >= rows or i >= cols:
        return -1
    return offs[name] + o * cols + i


def _frag(fn):
    """Build one fragment's 512 index slots from fn(r, h, j) -> param or -1."""
    out = np.empty(512, dtype=np.int32)
    for l in range(64):
        r, h = l & 31, l >> 5
        for j in range(8):
            out[l * 8 + j] = fn(r, h, j)
    return out


def field_frag_index():
    """(FIELD_FRAGS*512,) int32: master index per packed f16 slot."""
    F = []
    for m in range(2):
        for s in range(2):
            F.append(_frag(lambda r, h, j, m=m, s=s: _w("g1", 32 * m + r, _perm(s, h, j))))
    for q in range(4):
        F.append(_frag(lambda r, h, j, q=q: _w("g2", _geo_out(r), _kin(q, h, j))))
    for m in range(2):
        for s in range(2):
            F.append(_frag(lambda r, h, j, m=m, s=s: _w("r1", 32 * m + r, _perm(s, h, j))))
    for m in range(2):
        for q in range(4):
            F.append(_frag(lambda r, h, j, m=m, q=q: _w("r2", 32 * m + r, _kin(q, h, j))))
    for q in range(4):
        F.append(_frag(lambda r, h, j, q=q: _w("r3", r, _kin(q, h, j))))
    assert len(F) == FIELD_FWD_FRAGS
    # backward (transposed) fragments
    for m in range(2):
        F.append(_frag(lambda r, h, j, m=m: _w("r3", _perm(0, h, j), 32 * m + r)))
    for m in range(2):
        for q in range(4):
            F.append(_frag(lambda r, h, j, m=m, q=q: _w("r2", _kin(q, h, j), 32 * m + r)))
    for q in range(4):
        F.append(_frag(lambda r, h, j, q=q: _w("r1", _kin(q, h, j), 16 + r) if r < 16 else -1))
    for m in range(2):
        for s in range(2):
            F.append(_frag(lambda r, h, j, m=m, s=s: _w("g2", _geo_out(_perm(s, h, j)),
                                                        32 * m + r)))
    for q in range(4):
        F.append(_frag(lambda r, h, j, q=q: _w("g1", _kin(q, h, j), r)))
    assert len(F) == FIELD_FRAGS
    return np.concatenate(F)


def field_dinput_frag_index():
    """(4*512,) int32: the rgb net's SH columns transposed, Wr1[:, 0:16]^T as A
    fragments (rows = SH inputs 0..15, k = the 64 rgb hidden units in 4
    steps): dL/dSH = Wr1_sh^T dL/dR1 for the input gradient (rn_field_dinput)."""
    F = [_frag(lambda r, h, j, q=q: _w("r1", _kin(q, h, j), r) if r < 16 else -1)
         for q in range(4)]
    return np.concatenate(F)


def gate_dinput_frag_index(K):
    """(4*512,) int32: W0^T of the gate (rows = the 6 inputs, k = 64 hidden):
    dL/dinput = W0^T dL/dH0 (rn_gate_bwd's input gradient)."""
    sizes, offs = _gate_tables(K)
    F = [_frag(lambda r, h, j, q=q: _w("w0", _kin(q, h, j), r, sizes, offs)) for q in range(4)]
    return np.concatenate(F)


def _dw_tile(fn):
    out = np.empty(1024, dtype=np.int16)
    for i in range(16):
        for l in range(64):
            row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5)
            col = l & 31
            out[i * 64 + l] = fn(row, col)
    return out


def field_dw_map():
    T = []
    for nn in range(2):
        T.append(_dw_tile(lambda row, col, nn=nn: _w("r3", row, 32 * nn + col)))
    for m in range(2):
        for nn in range(2):
            T.append(_dw_tile(lambda row, col, m=m, nn=nn: _w("r2", 32 * m + row, 32 * nn + col)))
    for m in range(2):
        T.append(_dw_tile(lambda row, col, m=m: _w("r1", 32 * m + row, col)))
    for nn in range(2):
        T.append(_dw_tile(lambda row, col, nn=nn: _w("g2", _geo_out(row), 32 * nn + col)))
    for m in range(2):
        T.append(_dw_tile(lambda row, col, m=m: _w("g1", 32 * m + row, col)))
    assert len(T) == FIELD_DW_TILES
    return np.concatenate(T)


def _gate_tables(K):
    sizes = {"w0": (64, 6), "w1": (64, 64), "w2": (64, 64), "w3": (64, 64), "w4": (K, 64)}
    return sizes, gate_offsets(K)


def gate_frag_index(K):
    sizes, offs = _gate_tables(K)
    w = lambda n, o, i: _w(n, o, i, sizes, offs)
    F = []
    for m in range(2):
        F.append(_frag(lambda r, h, j, m=m: w("w0", 32 * m + r, _perm(0, h, j))))
    for L in range(1, 4):
        for m in range(2):
            for q in range(4):
                F.append(_frag(lambda r, h, j, L=L, m=m, q=q: w(f"w{L}", 32 * m + r,
                                                                _kin(q, h, j))))
    for q in range(4):
        F.append(_frag(lambda r, h, j, q=q: w("w4", r, _kin(q, h, j))))
    assert len(F) == GATE_FWD_FRAGS
    for m in range(2):
        F.append(_frag(lambda r, h, j, m=m: w("w4", _perm(0, h, j), 32 * m + r)))
    for L in (3, 2, 1):
        for m in range(2):
            for q in range(4):
                F.append(_frag(lambda r, h, j, L=L, m=m, q=q: w(f"w{L}", _kin(q, h, j),
                                                                32 * m + r)))
    assert len(F) == GATE_FRAGS
    return np.concatenate(F)


def gate_dw_map(K):
    sizes, offs = _gate_tables(K)
    w = lambda n, o, i: _w(n, o, i, sizes, offs)
    T = []
    for m in range(2):
        T.append(_dw_tile(lambda row, col, m=m: w("w0", 32 * m + row, col)))
    for L in range(1, 4):
        for m in range(2):
            for nn in range(2):
                T.append(_dw_tile(lambda row, col, L=L, m=m, nn=nn: w(f"w{L}", 32 * m + row,
                                                                       32 * nn + col)))
    for nn in range(2):
        T.append(_dw_tile(lambda row, col, nn=nn: w("w4", row, 32 * nn + col)))
    assert len(T) == GATE_DW_TILES
    return np.concatenate(T)


def split_field_params(flat):
    """Views of one sub-NeRF's master vector as the five [out,in] matrices."""
    out = {}
    for n, (r, c) in FIELD_SIZES.items():
        o = FIELD_OFF[n]
        out[n] = flat[o:o + r * c].reshape(r, c)
    return out


def split_gate_params(flat, K):
    sizes, offs = _gate_tables(K)
    return {n: flat[offs[n]:offs[n] + r * c].reshape(r, c) for n, (r, c) in sizes.items()}
