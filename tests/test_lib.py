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


def _fake_library(tmp_path, table, version=_lib.ABI_VERSION, name="librn_fake.so"):
    """A stand-in library exporting only the load-time ABI entries (no kernel:
    the checks must refuse it before any entry is bound)."""
    src = tmp_path / "fake.c"
    sig = "" if table is None else (
        'const char* rn_abi_signatures(void) { return "%s"; }\n' % table)
    src.write_text(f"int rn_version(void) {{ return {version}; }}\n"
                   'const char* rn_last_error(void) { return ""; }\n'
                   "void rn_set_debug_flags(int f) { (void)f; }\n" + sig)
    out = tmp_path / name
    subprocess.check_call(["gcc", "-shared", "-fPIC", str(src), "-o", str(out)])
    return str(out)


def test_library_signature_table_matches_binding():
    """librn.so's rn_abi_signatures() (generated from the header at build time)
    equals the binding's argument lists entry by entry, and the generator reads
    the header the same way."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "rad-nerf_amd", "csrc"))
    import gen_sig
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.rn_abi_signatures.restype = ctypes.c_char_p
    have = _lib.parse_signature_table(lib.rn_abi_signatures().decode())
    want = _lib.binding_signatures()
    assert {n: have[n] for n in want} == want
    assert _lib.parse_signature_table(gen_sig.table(open(HEADER).read())) == have
    assert set(have) == set(_declared())


def test_mismatched_signature_table_is_refused(tmp_path):
    """a library built from another revision of the header
    (one entry's arguments changed under the same RN_ABI_VERSION, as the A/B
    leg that called rn_gate_bwd with shifted arguments) fails at load with an
    ImportError naming the entry -- before any entry is bound or called."""
    good = dict(_lib.binding_signatures())
    bad = dict(good)
    bad["rn_gate_bwd"] = good["rn_gate_bwd"] + "p"        # one more pointer argument
    table = ";".join(f"{k}:{v}" for k, v in bad.items())
    with pytest.raises(ImportError, match=r"another revision.*rn_gate_bwd: library "):
        _lib._Lib(_fake_library(tmp_path, table))
    # a missing entry is named too
    del bad["rn_gate_bwd"]
    table = ";".join(f"{k}:{v}" for k, v in bad.items())
    with pytest.raises(ImportError, match="rn_gate_bwd: library missing"):
        _lib._Lib(_fake_library(tmp_path, table, name="librn_fake2.so"))
    # a library without the table (built before ABI 9), or of another ABI version
    with pytest.raises(ImportError, match="no rn_abi_signatures"):
        _lib._Lib(_fake_library(tmp_path, None, name="librn_fake3.so"))
    with pytest.raises(ImportError, match="ABI 8, binding expects"):
        _lib._Lib(_fake_library(tmp_path, None, version=8, name="librn_fake4.so"))
    # the same table as the binding's passes the checks (then binding the
    # entries fails: the stand-in exports none of them)
    table = ";".join(f"{k}:{v}" for k, v in good.items())
    with pytest.raises(AttributeError, match="rn_ray_aabb_intersect"):
        _lib._Lib(_fake_library(tmp_path, table, name="librn_fake5.so"))


def _doc_argtypes():
    """every `L.rn_x.argtypes = ...` assignment of INTEGRATION.md's ctypes
    binding, evaluated: {name: codes} (p pointer, i int32, l int64, ...)"""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    env = dict(P=ctypes.c_void_p, I32=ctypes.c_int32, I64=ctypes.c_int64, F32=ctypes.c_float,
               F64=ctypes.c_double, U64=ctypes.c_uint64, ctypes=ctypes)
    code = {ctypes.c_void_p: "p", ctypes.c_int32: "i", ctypes.c_int64: "l",
            ctypes.c_float: "f", ctypes.c_double: "d", ctypes.c_uint64: "u"}
    out = {}
    for m in re.finditer(r"L\.(rn_\w+)\.argtypes\s*=\s*", text):
        expr, depth = "", 0
        for line in text[m.end():].split("\n"):
            line = line.split("#")[0]
            expr += line.rstrip().rstrip("\\") + " "
            depth += line.count("(") + line.count("[") - line.count(")") - line.count("]")
            if depth == 0 and not line.rstrip().endswith("\\"):
                break
        out[m.group(1)] = "".join(code[t] for t in eval(expr, env))
    return out


def test_integration_doc_argtypes_match_library():
    """INTEGRATION.md's ctypes binding (what a maintainer copies into the
    reference) declares each entry exactly as the library was built (its
    signature table) -- the round-6 check found two stale lines there."""
    doc = _doc_argtypes()
    assert len(doc) >= 15
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.rn_abi_signatures.restype = ctypes.c_char_p
    have = _lib.parse_signature_table(lib.rn_abi_signatures().decode())
    assert {n: have.get(n) for n in doc} == doc


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
