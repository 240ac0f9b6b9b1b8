"""GPU: the C-ABI driven from C++ with no Python or torch in the process
(tests/capi/capi_smoke.cpp, built by __graft_entry__.build()): ray-AABB ->
near clamp -> march (count, scan, write) -> composite fw / bw on device
buffers the program owns, checked against the CPU oracle -- march and
termination bit-exact, colours and gradients within 1e-4."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from radnerf_amd import synthetic as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "capi", "build", "capi_smoke")


@pytest.mark.parametrize("scale", [0.5, 16.0])
def test_capi_consumer_matches_oracle(tmp_path, scale):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build() (make -C tests/capi)")
    B = 700
    esf = 1 / 256 if scale > 0.5 else 0.0
    cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
    o, d = S.rays(B, scale, seed=31)
    nz = S.noise(1, B, seed=32)[0]
    bits = S.bitfields(1, cascades, p=0.4, seed=33)[0]
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(src, "wb") as f:
        np.array([B, bits.size], np.int64).tofile(f)
        np.array([scale, esf], np.float32).tofile(f)
        np.array([cascades], np.int32).tofile(f)
        for a in (o, d, nz):
            np.ascontiguousarray(a, np.float32).tofile(f)
        np.ascontiguousarray(bits, np.uint8).tofile(f)
    run = subprocess.run([EXE, str(src), str(dst)], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stderr
    raw = open(dst, "rb").read()
    pos = 0

    def take(dtype, n):
        nonlocal pos
        a = np.frombuffer(raw, dtype, n, pos)
        pos += a.nbytes
        return a
    total = int(take(np.int64, 1)[0])
    ra = take(np.int64, B * 3).reshape(B, 3)
    ts, dl = take(np.float32, total), take(np.float32, total)
    sig, rgbs = take(np.float32, total), take(np.float32, total * 3).reshape(-1, 3)
    tot, op, de = take(np.int64, B), take(np.float32, B), take(np.float32, B)
    rgb = take(np.float32, B * 3).reshape(B, 3)
    dsig, drgb = take(np.float32, total), take(np.float32, total * 3).reshape(-1, 3)
    # oracle: the same chain
    c, h = np.zeros((1, 3), np.float32), np.full((1, 3), scale, np.float32)
    _, ht, _ = oracle.ray_aabb_intersect(o, d, c, h, 1)
    ht = np.ascontiguousarray(ht[:, 0])
    m = (ht[:, 0] >= 0) & (ht[:, 0] < 0.01)
    ht[m, 0] = 0.01
    ora, _, _, odl, ots, otot = oracle.raymarching_train(o, d, ht, bits, cascades, scale, esf, nz)
    assert otot == total > 1000
    assert np.array_equal(ra, ora) and np.array_equal(ts, ots) and np.array_equal(dl, odl)
    ct, cop, cde, crgb, cws = oracle.composite_train_fw(sig, rgbs, dl, ts, ra)
    assert np.array_equal(tot, ct)
    assert (ct < ra[:, 2]).sum() > 10                      # some rays terminate early
    # north_star: opacity / rgb within 1e-4 absolute; depth (a distance up to
    # the box size, ~scale) within 1e-4 relative to it
    for a, b in ((op, cop), (rgb, crgb)):
        assert np.abs(a - b).max() <= 1e-4
    assert np.abs(de - cde).max() <= 1e-4 * max(1.0, float(np.abs(cde).max()))
    gO = (0.1 * np.sin(np.arange(B))).astype(np.float32)
    gD = (0.05 * np.cos(np.arange(B))).astype(np.float32)
    gR = (0.2 * np.sin(3 * np.arange(B)[:, None] + np.arange(3)[None])).astype(np.float32)
    odsig, odrgb = oracle.composite_train_bw(gO, gD, gR, np.zeros(total, np.float32), sig, rgbs,
                                             cws, dl, ts, ra, cop, cde, crgb)
    assert np.abs(drgb - odrgb).max() <= 1e-4
    assert np.abs(dsig - odsig).max() <= 1e-4 * max(1.0, np.abs(odsig).max())
