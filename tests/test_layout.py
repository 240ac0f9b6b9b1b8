"""CPU: host-side layout logic of the product (radnerf_amd/layout.py) — hash
grid level tables vs the oracle's independent restatement, and the MFMA
fragment / weight-gradient index tables (every master weight appears exactly
once in each table; padding slots are -1)."""
import numpy as np
import pytest

from oracle import field_oracle as fo
from radnerf_amd import layout as LY


@pytest.mark.parametrize("scale,log2T", [(0.5, 19), (16.0, 19), (1.0, 17), (4.0, 21)])
def test_level_table_matches_oracle(scale, log2T):
    a, b = LY.grid_levels(scale, log2T), fo.grid_levels(scale, log2T)
    assert a["n_entries"] == b["n_entries"]
    for k in ("offset", "hsize", "res"):
        assert np.array_equal(a[k].astype(np.int64), b[k])
    assert np.array_equal(a["scale"], b["scale"])


def test_level_table_properties():
    lv = LY.grid_levels(0.5)
    assert lv["res"][0] == 16 and lv["scale"][0] == 15.0
    assert np.all(np.diff(lv["res"]) > 0)
    assert np.all(lv["hsize"] % 8 == 0) and np.all(lv["hsize"] <= 2 ** 19)
    dense = lv["res"].astype(np.int64) ** 3 <= lv["hsize"]
    assert dense[:6].all() and not dense[6:].any()   # 6 dense levels at scale 0.5
    # f32 tcnn semantics: 2^(5*log2 b)*16-1 lands just above 63 -> resolution 65
    assert lv["res"][5] == 65 and lv["res"][15] == 1025
    assert lv["n_entries"] == 5722520
    assert LY.cascades_for_scale(0.5) == 1 and LY.cascades_for_scale(16) == 6


def _coverage(idx, n):
    v = idx[idx >= 0]
    u, c = np.unique(v, return_counts=True)
    return len(u) == n and c.min() == 1 and c.max() == 1 and v.max() < n


def test_field_fragment_tables():
    fi = LY.field_frag_index()
    assert fi.shape == (LY.FIELD_FRAGS * 512,)
    fwd, bwd = fi[:LY.FIELD_FWD_FRAGS * 512], fi[LY.FIELD_FWD_FRAGS * 512:]
    assert _coverage(fwd, LY.FIELD_PARAMS)
    # backward transposes omit nothing but the never-needed rgb input rows 0..15 of Wr1
    sl = LY.split_field_params(np.arange(LY.FIELD_PARAMS))
    excl = set(sl["r1"][:, :16].reshape(-1).tolist())
    v = bwd[bwd >= 0]
    assert len(set(v.tolist())) == len(v) == LY.FIELD_PARAMS - len(excl)
    assert not (set(v.tolist()) & excl)
    dm = LY.field_dw_map()
    assert _coverage(dm.astype(np.int64), LY.FIELD_PARAMS)


@pytest.mark.parametrize("K", [1, 2, 4, 8, 16])
def test_gate_tables(K):
    n = LY.gate_params(K)
    gi = LY.gate_frag_index(K)
    assert _coverage(gi[:LY.GATE_FWD_FRAGS * 512], n)
    assert _coverage(LY.gate_dw_map(K).astype(np.int64), n)
    sl = LY.split_gate_params(np.arange(n), K)
    assert sl["w4"].shape == (K, 64) and sl["w0"].shape == (64, 6)


def test_kperm_accumulator_identity():
    """The k-permutation of a fragment built from an accumulator tile equals
    the MFMA C-map row of the register (rn_mlp.h): reg 8s+j of lane half h
    holds row (i&3)+8(i>>2)+4h."""
    for s in range(2):
        for h in range(2):
            for j in range(8):
                i = 8 * s + j
                assert LY._perm(s, h, j) == (i & 3) + 8 * (i >> 2) + 4 * h


def test_dinput_fragment_tables():
    """Input-gradient fragments: the rgb net's SH columns Wr1[:, 0:16]^T (rows =
    SH inputs, k = 64 hidden) -- exactly the entries the backward transposes
    omit -- and the gate's W0^T (rows = the 6 inputs)."""
    fi = LY.field_dinput_frag_index()
    assert fi.shape == (4 * 512,)
    sl = LY.split_field_params(np.arange(LY.FIELD_PARAMS))
    v = fi[fi >= 0]
    assert sorted(v.tolist()) == sorted(sl["r1"][:, :16].reshape(-1).tolist())
    # slot (frag q, lane l, elem j): row r = l & 31 (SH input), k = _kin(q, h, j) (hidden)
    for q in range(4):
        for l in (0, 5, 37, 63):
            r, h = l & 31, l >> 5
            for j in range(8):
                want = sl["r1"][LY._kin(q, h, j), r] if r < 16 else -1
                assert fi[q * 512 + l * 8 + j] == want
    for K in (2, 8):
        gi = LY.gate_dinput_frag_index(K)
        sg = LY.split_gate_params(np.arange(LY.gate_params(K)), K)
        v = gi[gi >= 0]
        assert sorted(v.tolist()) == sorted(sg["w0"].reshape(-1).tolist())
