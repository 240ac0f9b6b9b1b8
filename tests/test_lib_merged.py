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
        L.bwd_plan(*P[:5], 8, 2, 0, 0, 256, 512, 10, *P[:6])
    with pytest.raises(RuntimeError, match="rn_bwd_plan: bad sizes"):
        L.bwd_plan(*P[:5], 8, 9, 0, 0, 1024, 512, 10, *P[:6])
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
        L.grid_sum(*P[:6], 16, None, None, None, None)
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
    assert lay == dict(page=8192, bins=256, slice=4096, ctl_bytes=128, idx_bits=20, v_bits=22)


def test_grid_bin_and_sum_reject_oversized_levels():
    import numpy as np
    L = _lib.lib()
    V = ctypes.c_void_p(8)
    hs = np.full(16, 1 << 21, np.uint32)          # past the 20-bit entry index
    with pytest.raises(RuntimeError, match="level too large"):
        L.grid_bin(hs.ctypes.data, *[V] * 6, 16, 2048, None)
    off = np.zeros(16, np.uint32)
    with pytest.raises(RuntimeError, match="level too large"):
        L.grid_sum(off.ctypes.data, hs.ctypes.data, *[V] * 4, 16, V, None, V, None)


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
