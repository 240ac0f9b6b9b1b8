"""CPU: the merged-pass entry points (rn_bwd_plan, rn_field_fwd_merged,
rn_field_bwd_merged, rn_grid_fx_fold, rn_grid_bin, rn_grid_sum, rn_grid_binned_fold,
rn_seed_scale, rn_igrad_to_f32) reject bad arguments
before any HIP call, with the messages include/radnerf.h documents."""
import ctypes

import pytest

from radnerf_amd import _lib


def test_merged_entry_points_validate_without_gpu():
    L = _lib.lib()
    P = [None] * 32
    with pytest.raises(RuntimeError, match="bad chunk sizes"):
        L.bwd_plan(*P[:5], 8, 2, 0, 0, 256, 512, 0, 10, *P[:11])
    with pytest.raises(RuntimeError, match="bad chunk sizes"):
        L.bwd_plan(*P[:5], 8, 2, 0, 0, 1024, 512, -1, 10, *P[:11])
    with pytest.raises(RuntimeError, match="rn_bwd_plan: bad sizes"):
        L.bwd_plan(*P[:5], 8, 9, 0, 0, 1024, 512, 0, 10, *P[:11])
    with pytest.raises(RuntimeError, match="n_models <= 8"):
        L.field_fwd_merged(*P[:8], 8, 9, *P[:13], 256, 512, None)
    with pytest.raises(RuntimeError, match="threads"):
        L.field_fwd_merged(*P[:8], 8, 2, *P[:13], 256, 100, None)
    V = ctypes.c_void_p(8)      # never dereferenced: the check fails first
    with pytest.raises(RuntimeError, match="merged-order encoding needs"):
        L.field_fwd_merged(*[V] * 8, 8, 2, *[V] * 10, None, V, V, 256, 512, None)
    # scratch must hold a chunk plus one ray of every model
    with pytest.raises(RuntimeError, match="scratch_rows must be"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 2047, None, 1024, 256, *P[:7], 0, *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="integer mode needs"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 4096, None, 1024, 256,
                           ctypes.c_void_p(8), None, None, *P[:4], 0, *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="fx_mode"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 4096, None, 1024, 256, *P[:7], 1, *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="fixed-point mode needs"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 4096, None, 1024, 256, *P[:7], 2, *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="redo needs"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 4096, None, 1024, 256, *P[:7], 3, *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="binned mode needs"):
        L.field_bwd_merged(*P[:10], 8, 2, 1024, *P[:14], 4096, None, 1024, 256, *P[:7], 4,
                           *P[:3], 0, None)
    with pytest.raises(RuntimeError, match="null pointer"):
        L.grid_fx_fold(*P[:10])
    with pytest.raises(RuntimeError, match="null pointer"):
        L.grid_bin(*P[:7], 16, 2048, None)
    with pytest.raises(RuntimeError, match="bad sizes"):
        L.grid_bin(*[V] * 7, 0, 2048, None)
    with pytest.raises(RuntimeError, match="null pointer"):
        L.grid_sum(*P[:6], 16, None, None, None, 0, 16, None)
    with pytest.raises(RuntimeError, match="null pointer"):
        L.grid_binned_fold(*P[:8], 16, *P[:6])
    assert L.version() == _lib.ABI_VERSION
    assert L.igrad_to_f32(0, None, None, None, None, None) == 0
    with pytest.raises(RuntimeError, match="null pointer"):
        L.seed_scale(None, None, 2, None, None, None, None, None, None)


def test_abi_constants_match_the_header():
    """the binding's ABI version and buffer sizes are the header's (ADVICE r03:
    a caller allocating an older size must not pass silently)"""
    import os
    import re

    from radnerf_amd import fused
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "radnerf.h")).read()
    assert int(re.search(r"#define RN_ABI_VERSION (\d+)", hdr).group(1)) == _lib.ABI_VERSION
    assert int(re.search(r"#define RN_FX_STATS_BYTES (\d+)", hdr).group(1)) == fused.FX_STATS_BYTES
    lay = _lib.lib().bin_layout()
    assert lay == dict(page=8192, bins=256, slice=4096, ctl_bytes=128, idx_bits=20, v_bits=22,
                       m_bits=17, target_bits=38)


def test_grid_bin_and_sum_reject_oversized_levels():
    import numpy as np
    L = _lib.lib()
    V = ctypes.c_void_p(8)
    hs = np.full(16, 1 << 21, np.uint32)          # past the 20-bit entry index
    with pytest.raises(RuntimeError, match="level too large"):
        L.grid_bin(hs.ctypes.data, *[V] * 6, 16, 2048, None)
    off = np.zeros(16, np.uint32)
    with pytest.raises(RuntimeError, match="level too large"):
        L.grid_sum(off.ctypes.data, hs.ctypes.data, *[V] * 4, 16, V, None, V, 0, 16, None)


def test_grid_slice_bits_rule():
    """rn_grid_slice_bits (host): each level's slice is the smallest power of
    two >= 64 entries that cuts the level into <= 128 slices, 4096 at most
    (csrc/rn_bin.h gb_slice_bits, used by the bin and sum passes)."""
    import numpy as np

    from radnerf_amd import layout as LY
    L = _lib.lib()
    for scale in (0.5, 16.0):
        hs = np.ascontiguousarray(LY.grid_levels(scale)["hsize"], dtype=np.uint32)
        out = np.zeros(16, np.int32)
        L.grid_slice_bits(hs.ctypes.data, out.ctypes.data)
        for h, b in zip(hs.tolist(), out.tolist()):
            assert 6 <= b <= 12, (scale, h, b)
            assert -(-h // (1 << b)) <= 128 or b == 12, (scale, h, b)
            assert b == 6 or -(-h // (1 << (b - 1))) > 128, (scale, h, b)
        if scale == 16.0:
            assert out[0] == 6 and out[-1] == 12     # 4096 entries in 64s; 2^19 in 4096s
    with pytest.raises(RuntimeError, match="level too large"):
        L.grid_slice_bits(np.full(16, 1 << 21, np.uint32).ctypes.data, np.zeros(16, np.int32).ctypes.data)


def _encode(x):
    import numpy as np
    L = _lib.lib()
    x = np.ascontiguousarray(x, np.float32)
    f = np.zeros(len(x), np.uint32)
    L.grid_record_encode(x.ctypes.data, len(x), f.ctypes.data)
    v = np.zeros(len(x), np.int64)
    L.grid_record_decode(f.ctypes.data, len(x), v.ctypes.data)
    return f, v


def test_grid_record_e5m17_format():
    """The binned scatter's record value (csrc/rn_bin.h gb_encode, VERDICT r04
    item 1): exact to one unit below 2^15 units (e = 0, m = rint(x)); above,
    14 significant bits past the leading one (relative error <= 2^-15);
    every |x| < 2^46 representable, sign-symmetric, monotone; the 22-bit
    field is mantissa [0, 17) | exponent << 17."""
    import numpy as np
    rng = np.random.default_rng(3)
    small = rng.uniform(-32767.4, 32767.4, 20000).astype(np.float32)
    f, v = _encode(small)
    assert np.array_equal(v, np.rint(small).astype(np.int64))
    assert np.all(f >> 17 == 0) and np.all(f < (1 << 22))
    # the whole range, log-uniform, both signs
    mag = np.exp2(rng.uniform(-30, 45.999, 200000)).astype(np.float32)
    x = np.where(rng.random(len(mag)) < 0.5, -mag, mag).astype(np.float32)
    f, v = _encode(x)
    assert np.all(f < (1 << 22))
    xd = x.astype(np.float64)
    err = np.abs(v - xd)
    big = np.abs(xd) >= 32768.0
    assert np.all(err[~big] <= 0.5)
    assert np.all(err[big] / np.abs(xd[big]) <= 2.0 ** -15)
    f2, v2 = _encode(-x)
    assert np.array_equal(v2, -v)
    o = np.argsort(xd)
    assert np.all(np.diff(v[o]) >= 0)                  # monotone
    # just below 2^46 units: representable, rounded to 2^-15 relative
    edge = np.array([2.0 ** 46 * (1 - 2.0 ** -24), -(2.0 ** 46) * (1 - 2.0 ** -24)], np.float32)
    f, v = _encode(edge)
    assert np.array_equal(v, np.array([2 ** 46, -(2 ** 46)], np.int64))
    assert np.all(f >> 17 == 31)


def test_fx_mode_refuses_grids_past_the_checksum_weights():
    """fx_mode 2's wrap checksums weight element i by its byte offset 4 i
    (field.hip fx_weight), injective below 2^30: a grid of more than 2^28
    gradient elements is refused before any HIP call."""
    import numpy as np
    L = _lib.lib()
    V = ctypes.c_void_p(8)
    off = np.arange(16, dtype=np.uint32) * (1 << 23)
    hs = np.full(16, 1 << 23, np.uint32)
    big = hs.copy()
    big[-1] += 1
    args = lambda h: [*[V] * 10, 8, 2, 1024, V, off.ctypes.data, h.ctypes.data, *[V] * 11, 4096, V,
                      1024, 256, None, None, None, V, V, V, V, 2, None, None, None, 0, None]
    with pytest.raises(RuntimeError, match="more than 2\\^28 gradient elements"):
        L.field_bwd_merged(*args(big))


def test_fx_weight_separates_opposite_wraps():
    """opposite +-2^32 wraps on elements a != b move the weighted sum by
    2^32 (w_a - w_b) mod 2^64 with w = 4 i: non-zero for every pair of a
    2^28-element table (the weight's difference is 4 (a - b), 0 < |a - b| <
    2^28)"""
    import numpy as np
    rng = np.random.default_rng(5)
    a = rng.integers(0, 1 << 28, 100000, dtype=np.uint64)
    b = rng.integers(0, 1 << 28, 100000, dtype=np.uint64)
    keep = a != b
    d = ((a[keep] * 4) - (b[keep] * 4)) << np.uint64(32)    # mod 2^64
    assert np.all(d != 0)
