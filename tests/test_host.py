"""CPU: host-side module logic that mirrors the reference's networks.py
(no kernel launches)."""
import numpy as np
import torch

from radnerf_amd.networks import MNGP, NGP, Ray_Gate


def test_register_bbox_matches_reference_formulas():
    """networks.py:413-422: center/half_size from the box, cascades =
    max(1 + ceil(log2(2 * max half_size)), 1), fresh grids per sub-NeRF."""
    m = MNGP(0.5, size=3)
    bbox = np.array([[-3.0, -0.5, -0.25], [1.0, 0.5, 0.75]], np.float32)
    m.register_bbox(bbox)
    assert torch.allclose(m.center, torch.tensor([[-1.0, 0.0, 0.25]]))
    assert torch.allclose(m.half_size, torch.tensor([[2.0, 0.5, 0.5]]))
    assert m.cascades == max(1 + int(np.ceil(np.log2(2 * 2.0))), 1) == 3
    for i in range(3):
        assert getattr(m, f"density_bitfield_{i}").shape == (3 * 128 ** 3 // 8,)
        assert getattr(m, f"density_grid_{i}").shape == (3, 128 ** 3)
    # the field kernels read the box from host copies refreshed with it
    assert np.allclose(m._h_min, bbox[0]) and np.allclose(m._h_ext, bbox[1] - bbox[0])
    n = NGP(0.5)
    n.register_bbox(np.array([[-1, -1, -1], [1, 1, 1]], np.float32))
    assert n.cascades == 2 and n.density_bitfield.shape == (2 * 128 ** 3 // 8,)


def test_cascades_and_buffers_like_reference():
    """networks.py:229-262: cascades = max(1 + ceil(log2(2*scale)), 1), grid 128,
    buffer names used by ml_render / update_density_grid."""
    for scale, c in ((0.5, 1), (1.0, 2), (16.0, 6)):
        m = MNGP(scale, size=2)
        assert m.cascades == c and m.grid_size == 128
        names = dict(m.named_buffers())
        for k in ("center", "xyz_min", "xyz_max", "half_size", "grid_coords",
                  "density_bitfield_0", "density_grid_1"):
            assert k in names, k
    g = Ray_Gate(4)
    assert g.type == "ray" and g.out_dim == 4
    g.freeze_dict()
    assert not any(p.requires_grad for p in g.parameters())


def test_binned_coarse_levels_default_by_shape():
    """Round 6: the binned form (scale 16) sends the coarse levels by fp32
    atomics -- 9 with K >= 8 sub-NeRFs, 8 otherwise (profiles/r06/bin_f32/);
    scale 0.5 (the int32 atomic form) bins nothing.  The level cut of the
    data-parallel fold stays in [0, 15]."""
    import torch
    from radnerf_amd.fused import FusedMLRenderer, clamp_split
    from radnerf_amd.networks import MNGP, Ray_Gate
    cpu = torch.device("cpu")
    for scale, K, B, want_bin, want_n in ((16.0, 8, 1024, True, 9), (16.0, 4, 1024, True, 8),
                                          (16.0, 2, 1024, True, 8), (0.5, 2, 8192, False, 0),
                                          (16.0, 1, 512, False, 0)):
        r = FusedMLRenderer(MNGP(scale, size=K, seed=3), Ray_Gate(K, seed=4), B, device=cpu,
                            capacity=1024)
        assert (r.grid_bin, r.bin_f32_levels) == (want_bin, want_n), (scale, K, B)
        assert r.fx_f32_levels == ()
    assert clamp_split(16) == 15


def test_chunk_defaults_by_shape():
    """Round 6's measured chunk defaults (fused.FusedMLRenderer; profiles/r06/
    headramp/, minchunk/): head chunks ramp to max_chunk at scale 0.5 above
    1024 ray x sub-NeRF pairs, none at scale 16; the tail's chunks (the last
    1/16 of the merged positions) are 1536 merged samples at K >= 8 (8192+
    rays) at scale 16, 512 otherwise."""
    import torch
    from radnerf_amd.fused import FusedMLRenderer
    from radnerf_amd.networks import MNGP, Ray_Gate
    cpu = torch.device("cpu")
    for scale, K, B, head, mn in ((0.5, 2, 8192, 1536, 512), (0.5, 1, 8192, 1024, 512),
                                  (0.5, 1, 1024, 0, 512), (16.0, 8, 8192, 0, 1536),
                                  (16.0, 4, 4096, 0, 512), (16.0, 8, 4096, 0, 512),
                                  (16.0, 1, 65536, 0, 512)):
        r = FusedMLRenderer(MNGP(scale, size=K, seed=3), Ray_Gate(K, seed=4), B, device=cpu,
                            capacity=1024)
        assert (r.head_chunk, r.min_chunk) == (head, mn), (scale, K, B, r.head_chunk, r.min_chunk)
        assert r.head_chunk <= r.max_chunk        # (the plan takes min(min_chunk, max_chunk))
