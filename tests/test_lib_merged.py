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
