"""Mutation fuzz of the GPU lossy path against the CPU oracle.

Bit-flipped copies of lossy fixtures that still parse decode to arbitrary (often extreme)
coefficients, modes and filter parameters -- the int16 / 32-bit wrapping corners of
TransformOne, the clamps of every predictor and filter tap.  Each parseable mutant goes
through one GPU batch (K1 with its RGBA tail, and K2 separately) and must match the
oracle's Y/U/V and RGBA bit for bit.  The oracle itself is pinned to libwebp 1.6.0 by
tests/test_oracle.py; for the mutants no libwebp decode is committed, so parity here is
GPU == oracle (the reference's own tests have no corrupted-stream vectors for this path).
"""
import numpy as np
import pytest

import webp_amd
from oracle_lib import load_lossy, lossy_cases, oracle_decode

pytestmark = pytest.mark.gpu


def _mutants(seed=7, per_source=24):
    rng = np.random.default_rng(seed)
    out = []
    srcs = [n for n in lossy_cases() if n != "alpha_64x48"]
    srcs = sorted(srcs, key=lambda n: len(load_lossy(n)[0]))[:8]
    for n in srcs:
        d = bytearray(load_lossy(n)[0])
        for _ in range(per_source):
            m = bytearray(d)
            for _ in range(int(rng.integers(1, 4))):
                pos = int(rng.integers(40, len(m)))  # past the RIFF + VP8 frame headers
                m[pos] ^= 1 << int(rng.integers(0, 8))
            try:
                info, mbs = webp_amd.vp8_parse(bytes(m))
            except webp_amd.WebPError:
                continue
            out.append((bytes(m), info, mbs))
    return out


@pytest.mark.parametrize("emit", ["fused", "separate"])
def test_mutated_streams_gpu_equals_oracle(emit):
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    cases = _mutants()
    assert len(cases) >= 40, len(cases)
    ctx = webp_amd.Context(0)
    b = ctx.batch([c[0] for c in cases])
    b.set_emit(emit == "separate")
    b.run()
    checked = 0
    for i, (_, info, mbs) in enumerate(cases):
        if b.status[i] != 0:
            continue
        o = oracle_decode(info, mbs)
        y, u, v = b.yuv(i)
        np.testing.assert_array_equal(y, o["y"], err_msg=f"mutant {i} Y")
        np.testing.assert_array_equal(u, o["u"], err_msg=f"mutant {i} U")
        np.testing.assert_array_equal(v, o["v"], err_msg=f"mutant {i} V")
        np.testing.assert_array_equal(b.rgba(i), o["rgba"], err_msg=f"mutant {i} RGBA")
        checked += 1
    assert checked >= 40, checked
    b.close()
    ctx.close()


def test_mutated_lossless_streams_gpu_equals_oracle():
    """The same for VP8L: bit-flipped lossless fixtures that still parse (other prefix codes,
    transform data, palettes, cache bits) -> K3 (every kernel variant the mutants select)
    == the oracle's inverse transforms, bit for bit."""
    from oracle_lib import load_lossless, lossless_names, oracle_vp8l_decode
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    rng = np.random.default_rng(11)
    cases = []
    for n in sorted(lossless_names(), key=lambda n: len(load_lossless(n)[0]))[:10]:
        d = bytearray(load_lossless(n)[0])
        for _ in range(24):
            m = bytearray(d)
            for _ in range(int(rng.integers(1, 3))):
                pos = int(rng.integers(25, len(m)))  # past the RIFF header and VP8L size fields
                m[pos] ^= 1 << int(rng.integers(0, 8))
            try:
                info, argb, tdata = webp_amd.vp8l_parse(bytes(m))
            except webp_amd.WebPError:
                continue
            cases.append((bytes(m), info, argb, tdata))
    assert len(cases) >= 30, len(cases)
    ctx = webp_amd.Context(0)
    b = ctx.batch([c[0] for c in cases])
    b.run()
    checked = 0
    for i, (_, info, argb, tdata) in enumerate(cases):
        if b.status[i] != 0:
            continue
        np.testing.assert_array_equal(b.rgba(i), oracle_vp8l_decode(info, argb, tdata), err_msg=f"mutant {i}")
        checked += 1
    assert checked >= 30, checked
    b.close()
    ctx.close()
