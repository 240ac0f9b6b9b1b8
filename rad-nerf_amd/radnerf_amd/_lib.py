"""ctypes binding of librn.so (include/radnerf.h).

The library is the product: there is no CPU fallback.  Loading fails loudly
when librn.so is missing, and every call checks the returned status and raises
RuntimeError with the library's message (mirroring the TORCH_CHECK errors of
models/csrc/include/utils.h:4-6 in the reference).  ctypes releases the GIL
for the duration of each call.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RADNERF_LIB", os.path.join(_HERE, "librn.so"))
# timing studies only (tools/ablate.py, bin_probe.py, march_probe.py): the same
# sources built with -DRN_ABLATION, where rn_set_debug_flags switches kernel
# parts off and selects variant kernels (csrc/rn_common.h RN_ABL).  librn.so
# ignores the switches and holds one code path per kernel.
ABLATION_LIB_PATH = os.environ.get("RADNERF_ABL_LIB", os.path.join(_HERE, "librn_abl.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F32 = ctypes.c_float
F64 = ctypes.c_double
U64 = ctypes.c_uint64

# name -> argtypes (all return int status).  Keep in sync with include/radnerf.h
SIGNATURES = {
    "rn_ray_aabb_intersect": [P, P, P, P, I64, I64, I32, P, P, P, P],
    "rn_ray_sphere_intersect": [P, P, P, P, I64, I64, I32, P, P, P, P],
    "rn_raymarching_train_bw": [P, P, P, P, I64, P, P, P],
    "rn_ml_march_bw": [P, P, I64, I32, P, P, P, P, P, P],
    "rn_field_dinput": [P, P, I64, P, P, P, P, P, P, I32, P, P, P, P, P, P, P, P, P, P, P, P, P,
                        P, I32, P],
    "rn_field_density": [P, I64, P, P, P, P, P, P, P, P, P, P, P],
    "rn_debug_cycles": [P],
    "rn_set_level_pairing": [ctypes.c_uint64],
    "rn_density_update_sampled": [P, P, I32, I32, I32, F32, F32, F32, U64, P, P, P, P, P, P, P,
                                  P, P, P, P, P, P, I32, P],
    "rn_distortion_loss_fw": [P, P, P, P, I64, P, P, P, P],
    "rn_distortion_loss_bw": [P, P, P, P, P, P, P, I64, P, P],
    "rn_raymarching_train_count": [P, P, P, P, I32, F32, F32, P, I32, I32, I64, P, P],
    "rn_raymarching_train_write": [P, P, P, P, I32, F32, F32, P, I32, I32, I64, P, P, P, P, P,
                                   P, P, P],
    "rn_scan_segments": [P, I32, I64, I32, P, P, P, P, P],
    "rn_raymarching_test": [P, P, P, P, I64, P, I32, F32, F32, I32, I32, I32, P, P, P, P, P, P],
    "rn_ml_march_count": [P, P, P, P, F32, P, P, I64, I32, I32, F32, F32, I32, I32, I64, P, P, P,
                          P],
    "rn_ml_compact": [P, P, I64, I32, I32, P, P, P, P, P, P],
    "rn_ml_march_write": [P, P, P, P, F32, P, P, I64, I32, I32, F32, F32, I32, I32, I64, P, P,
                          P, P, P, P],
    "rn_composite_train_fw": [P, P, P, P, P, I64, F32, P, P, P, P, P, P],
    "rn_composite_train_bw": [P, P, P, P, P, P, P, P, P, P, I64, P, P, P, F32, P, P, P],
    "rn_composite_test_fw": [P, P, P, P, I64, I32, P, F32, P, P, P, P, P],
    "rn_ml_composite_fw": [P, P, P, P, P, P, I64, I32, F32, P, P, P, P, P, P],
    "rn_ml_combine_fw": [P, P, P, P, P, I64, I32, P, P, P, P],
    "rn_ml_combine_bw": [P, P, P, P, P, I64, I32, P, P],
    "rn_ml_composite_bw": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I64, I32, F32, P, P, P],
    "rn_field_fwd": [P, P, I64, P, P, P, P, P, P, I32, P, P, P, P, P, P, P, P, P, P, P, I32, P],
    "rn_field_bwd": [P, P, I64, P, P, P, P, P, P, I32, P, P, P, P, P, P, P, P, P, P, P, P, P,
                     I32, P],
    "rn_bwd_plan": [P, P, P, P, P, I64, I32, I32, I32, I32, I32, I32, I32, P, P, P, P, P,
                    P, P, P, P, P, P],
    "rn_field_bwd_merged": [P, P, P, P, P, P, P, P, P, P, I64, I32, I32, P, P, P, P, P, P,
                            P, P, P, P, P, P, P, P, I64, P, I32, I32, P, P, P, P, P, P,
                            P, I32, P, P, P, I32, P],
    "rn_grid_fx_fold": [P, P, P, P, P, P, P, P, P, P],
    "rn_grid_bin_layout": [P],
    "rn_debug_gb_cycles": [P],
    "rn_grid_slice_bits": [P, P],
    "rn_grid_record_encode": [P, I64, P],
    "rn_grid_record_decode": [P, I64, P],
    "rn_grid_bin": [P, P, P, P, P, P, P, I32, I32, P],
    "rn_grid_sum": [P, P, P, P, P, P, I32, P, P, P, I32, I32, P],
    "rn_grid_bin_check": [P, P, P, P, P, P, P, I32, P, P, P, P, P],
    "rn_grid_binned_fold": [P, P, P, P, P, P, P, P, I32, P, P, P, P, P, P],
    "rn_render_test": [P, P, P, I64, I32, P, I64, I32, F32, F32, I32, I32, P, P, P, P, P, P, P,
                       P, F32, P, P, P, P, I32, P],
    "rn_seed_scale": [P, P, I32, P, P, P, P, P, P],
    "rn_igrad_to_f32": [I64, P, P, P, P, P],
    "rn_field_fwd_merged": [P, P, P, P, P, P, P, P, I64, I32, P, P, P, P, P, P, P, P, P, P, P,
                            P, P, I32, I32, P],
    "rn_field_fwd_levels": [P, P, P, P, P, P, I64, I32, P, P, P, P, P, P, P, P, P, P, P, P, P,
                            P, I64, P, I32, I32, I32, P, P],
    "rn_gate_fwd": [P, P, I32, I64, I32, P, P, P, I32, P],
    "rn_gate_bwd": [P, P, I32, I64, I32, P, P, P, I32, P, P, I32, P],
    "rn_nerf_loss": [P, P, P, P, P, P, I64, I32, F32, F32, F32, P, P, P, P, P, P],
    "rn_adam": [P, P, P, P, I64, F64, F64, F64, F64, I32, F32, P, I64, P],
    "rn_get_rays": [P, P, P, P, I64, P, P, P, P, P],
    "rn_pack_f16": [P, I64, P, I64, I32, I64, P, P],
    "rn_to_f16": [P, I64, P, P],
    "rn_morton3d": [P, I64, P, P],
    "rn_morton3d_invert": [P, I64, P, P],
    "rn_packbits": [P, I64, F32, P, P],
    "rn_scatter_max": [P, P, I64, P, P],
}

ABI_VERSION = 9
_lib = None

_CODE = {P: "p", I32: "i", I64: "l", F32: "f", F64: "d", U64: "u"}


def binding_signatures():
    """SIGNATURES in the library's table format (csrc/gen_sig.py): name ->
    one code per parameter."""
    return {n: "".join(_CODE[t] for t in a) for n, a in SIGNATURES.items()}


def parse_signature_table(text):
    """rn_abi_signatures()'s "name:codes;..." -> {name: codes}."""
    return dict(e.split(":", 1) for e in text.split(";") if e)


class _Checked:
    def __init__(self, lib, name):
        self._fn = getattr(lib, name)
        self._fn.argtypes = SIGNATURES[name]
        self._fn.restype = ctypes.c_int
        self._name = name
        self._err = lib.rn_last_error

    def __call__(self, *args):
        st = self._fn(*args)
        if st != 0:
            msg = self._err().decode("utf-8", "replace")
            raise RuntimeError(f"{self._name} failed (status {st}): {msg}")
        return st


class _Lib:
    def __init__(self, path):
        if not os.path.exists(path):
            raise ImportError(
                f"radnerf_amd: HIP library not found at {path}; build it with "
                f"`make -C rad-nerf_amd/csrc` (hipcc --offload-arch=gfx950). There is no CPU "
                f"fallback.")
        self.handle = ctypes.CDLL(path)
        self.handle.rn_last_error.restype = ctypes.c_char_p
        self.handle.rn_last_error.argtypes = []
        self.handle.rn_version.restype = ctypes.c_int
        self.handle.rn_set_debug_flags.argtypes = [ctypes.c_int]
        self.handle.rn_set_debug_flags.restype = None
        self.set_debug_flags = self.handle.rn_set_debug_flags
        self.path = path
        # the ABI checks come before any entry is bound: a library of another
        # revision is refused here, never called with shifted arguments
        self.check_version()
        self.check_signatures()
        for name in SIGNATURES:
            setattr(self, name[3:], _Checked(self.handle, name))

    def check_signatures(self):
        """Compare the library's own signature table (rn_abi_signatures,
        generated from the header it was built with) with SIGNATURES, entry by
        entry; ImportError naming every entry that differs or is missing."""
        try:
            fn = self.handle.rn_abi_signatures
        except AttributeError:
            raise ImportError(f"radnerf_amd: {self.path} exports no rn_abi_signatures "
                              f"(built before ABI 9); rebuild with `make -C rad-nerf_amd/csrc`")
        fn.restype, fn.argtypes = ctypes.c_char_p, []
        have = parse_signature_table(fn().decode())
        bad = []
        for name, codes in binding_signatures().items():
            if have.get(name) != codes:
                bad.append(f"{name}: library {have.get(name, 'missing')!s} vs binding {codes}")
        if bad:
            raise ImportError(f"radnerf_amd: {self.path} was built from another revision of "
                              f"include/radnerf.h ({len(bad)} entr{'y' if len(bad) == 1 else 'ies'}"
                              f" differ): " + "; ".join(bad[:8]))

    def version(self):
        return self.handle.rn_version()

    def bin_layout(self):
        """the binned scatter's page layout (csrc/rn_bin.h, rn_grid_bin_layout)"""
        if getattr(self, "_bin_layout", None) is None:
            out = (ctypes.c_int32 * 8)()
            self.grid_bin_layout(out)
            self._bin_layout = dict(page=out[0], bins=out[1], slice=out[2], ctl_bytes=out[3],
                                    idx_bits=out[4], v_bits=out[5], m_bits=out[6],
                                    target_bits=out[7])
        return self._bin_layout

    def check_version(self):
        """the ABI this binding was written against (include/radnerf.h RN_ABI_VERSION)"""
        v = self.version()
        if v != ABI_VERSION:
            raise ImportError(f"radnerf_amd: librn.so ABI {v}, binding expects {ABI_VERSION}; "
                              f"rebuild with `make -C rad-nerf_amd/csrc`")


def lib():
    """The loaded librn.so (raises ImportError when it is missing)."""
    global _lib
    if _lib is None:
        _lib = _Lib(LIB_PATH)
    return _lib


def use_ablation_build():
    """Timing-study tools: load librn_abl.so instead of librn.so.  Call before
    the first lib() of the process (the product path never calls it)."""
    global LIB_PATH
    if _lib is not None and _lib.path != ABLATION_LIB_PATH:
        raise RuntimeError("librn.so is already loaded in this process")
    LIB_PATH = ABLATION_LIB_PATH
    return lib()


def exported_symbols():
    return ["rn_version", "rn_last_error", "rn_set_debug_flags",
            "rn_abi_signatures"] + list(SIGNATURES)
