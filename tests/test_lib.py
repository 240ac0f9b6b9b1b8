"""CPU: the C-ABI library loads, exports exactly what include/radnerf.h
declares, validates arguments without touching a GPU, and the Python binding
mirrors the reference's error behaviour (utils.h:4-6 CHECK_INPUT)."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from radnerf_amd import _lib, vren

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "radnerf.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rn_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    names = _declared()
    assert len(names) >= 25
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True).stdout
    exported = set(re.findall(r"\bT (rn_[a-z0-9_]+)", nm))
    assert set(names) <= exported
    # every declared symbol has a ctypes signature in the binding
    assert set(names) == set(_lib.exported_symbols())


def test_library_is_gfx950():
    # the HIP fat binary embeds the offload target triple of every code object
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data or b"gfx950" in data


def test_arg_validation_without_gpu():
    L = _lib.lib()
    assert L.version() >= 1
    # zero-sized work returns immediately (no launch)
    assert L.morton3d(None, 0, None, None) == 0
    assert L.composite_train_fw(None, None, None, None, None, 0, 1e-4, None, None, None, None,
                                None, None) == 0
    # invalid sizes are rejected with a message, before any HIP call
    with pytest.raises(RuntimeError, match="bad size"):
        L.morton3d(None, -1, None, None)
    with pytest.raises(RuntimeError, match="rn_raymarching_train_count.*bad sizes"):
        L.raymarching_train_count(None, None, None, None, 0, 0.5, 0.0, None, 128, 1024, 10,
                                  None, None)
    with pytest.raises(RuntimeError, match="null pointer"):
        L.packbits(None, 8, 0.5, None, None)
    with pytest.raises(RuntimeError, match="n_params mismatch"):
        L.gate_bwd(None, None, 3, 10, 2, None, None, None, 5, None, None, 1, None)
    # level-partitioned forward: level groups come in eights, at most 8 sub-NeRFs
    lv = [None] * 6 + [8, 2] + [None] * 14 + [16, None]
    with pytest.raises(RuntimeError, match="rn_field_fwd_levels.*multiple of 8"):
        L.field_fwd_levels(*lv, 0, 12, 1, None, None)
    lv[7] = 9
    with pytest.raises(RuntimeError, match="rn_field_fwd_levels.*n_models <= 8"):
        L.field_fwd_levels(*lv, 0, 16, 1, None, None)
    # a level pairing must name every level exactly once
    with pytest.raises(RuntimeError, match="every level exactly once"):
        L.set_level_pairing(0x11)
    assert L.set_level_pairing(0) == 0


def test_vren_checks_like_reference():
    cpu = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="rays_o must be a CUDA tensor"):
        vren.ray_aabb_intersect(cpu, cpu, torch.zeros(1, 3), torch.zeros(1, 3), 1)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        vren.composite_train_fw(torch.zeros(4), cpu, torch.zeros(4), torch.zeros(4),
                                torch.zeros(1, 3, dtype=torch.long), 1e-4)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        vren.distortion_loss_fw(torch.zeros(4), torch.zeros(4), torch.zeros(4),
                                torch.zeros(1, 3, dtype=torch.long))
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        vren.ray_sphere_intersect(torch.zeros(1, 3), torch.zeros(1, 3), torch.zeros(1, 3),
                                  torch.ones(1), 1)


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    with pytest.raises(ImportError, match="no CPU"):
        _lib._Lib(str(tmp_path / "librn.so"))


def test_reference_dropin_module_names():
    """`import vren` from rad-nerf_amd/ exposes the reference binding's 12 names
    (binding.cpp:234-251)."""
    import importlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "rad-nerf_amd"))
    v = importlib.import_module("vren")
    for n in ("ray_aabb_intersect", "ray_sphere_intersect", "morton3D", "morton3D_invert",
              "packbits", "raymarching_train", "raymarching_test", "composite_train_fw",
              "composite_train_bw", "composite_test_fw", "distortion_loss_fw",
              "distortion_loss_bw"):
        assert callable(getattr(v, n))
    from radnerf_amd import custom_functions as cf
    for n in ("RayAABBIntersector", "RayMarcher", "VolumeRenderer", "TruncExp"):
        assert issubclass(getattr(cf, n), torch.autograd.Function)


def test_product_library_has_one_code_path():
    """timing-study variants (the merged backward's ABL
    instantiations, the sum pass's ABL / PROF / BIS and the bin pass's
    512 / 256-thread forms) live only in librn_abl.so; librn.so holds one
    instantiation of each of those kernels per production mode."""
    import os
    import re
    from radnerf_amd import _lib
    names = {}
    for key, path in (("prod", _lib.LIB_PATH), ("abl", _lib.ABLATION_LIB_PATH)):
        data = open(path, "rb").read()
        names[key] = set(re.findall(rb"_ZN12_GLOBAL__N_1\d+(k_grid_sum|k_grid_bin|k_field_bwd_merged)I([A-Za-z0-9_]*?)EEEv", data))
        assert os.path.getsize(path) > 0
    prod = {(k.decode(), t.decode()) for k, t in names["prod"]}
    assert ("k_grid_sum", "Li0ELb0ELi0") in prod and ("k_grid_bin", "Li1024ELb0") in prod
    assert not [x for x in prod if x[0] == "k_grid_sum" and x[1] != "Li0ELb0ELi0"], prod
    assert not [x for x in prod if x[0] == "k_grid_bin" and x[1] != "Li1024ELb0"], prod
    assert not [x for x in prod if x[0] == "k_field_bwd_merged" and "Lb1E" in x[1] + "E"], prod
    abl = {(k.decode(), t.decode()) for k, t in names["abl"]}
    assert len(abl) > len(prod)
