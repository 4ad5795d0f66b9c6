"""Mutation fuzz of the GPU paths against libwebp 1.6.0 and the CPU oracle.

Bit-flipped copies of the smallest lossy and lossless fixtures (oracle_lib.fuzz_mutants, a
fixed seeded corpus) decode to arbitrary, often extreme, coefficients, modes and filter
parameters -- the int16 / 32-bit wrapping corners of TransformOne, the clamps of every
predictor and filter tap -- or, for VP8L, to other prefix codes, cache sizes, transform data
and palettes.  The whole corpus goes through one GPU batch, and every mutant must match
libwebp 1.6.0's WebPDecode (tests/golden/manifest.json "fuzz": status and RGBA SHA-256,
committed by make_golden.py) -- failing ones with libwebp's status -- and, where it decodes,
the oracle bit for bit (Y/U/V and RGBA for lossy: K1's tail and a separate K2; RGBA through
K7 + K3 for lossless).
"""
import hashlib

import numpy as np
import pytest

import webp_amd
from oracle_lib import (FUZZ_LOSSLESS, FUZZ_LOSSY, fuzz_mutants, manifest, oracle_decode, oracle_vp8l_decode)

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("emit", ["fused", "separate"])
def test_mutated_lossy_streams_vs_libwebp_and_oracle(emit):
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    cases = fuzz_mutants("lossy", *FUZZ_LOSSY)
    want = manifest()["fuzz"]["lossy"]
    ctx = webp_amd.Context(0)
    b = ctx.batch([d for _, d in cases])
    b.set_emit(emit == "separate")
    b.run()
    decoded = 0
    for i, (key, data) in enumerate(cases):
        w = want[key]
        assert int(b.status[i]) == w["status"], (key, int(b.status[i]), w["status"])
        if w["status"] != 0:
            continue
        rgba = b.rgba(i)
        assert _sha(rgba) == w["rgba"], f"mutant {key}: GPU != libwebp"
        info, mbs = webp_amd.vp8_parse(data)
        o = oracle_decode(info, mbs)
        y, u, v = b.yuv(i)
        np.testing.assert_array_equal(y, o["y"], err_msg=f"mutant {key} Y")
        np.testing.assert_array_equal(u, o["u"], err_msg=f"mutant {key} U")
        np.testing.assert_array_equal(v, o["v"], err_msg=f"mutant {key} V")
        np.testing.assert_array_equal(rgba, o["rgba"], err_msg=f"mutant {key} RGBA")
        decoded += 1
    assert decoded >= 100, decoded
    b.close()
    ctx.close()


def test_mutated_lossless_streams_vs_libwebp_and_oracle():
    """The same for VP8L: other prefix codes, cache sizes, transform data and palettes ->
    K7 (color cache + back-references) and K3 (every kernel variant the mutants select)."""
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    cases = fuzz_mutants("lossless", *FUZZ_LOSSLESS)
    want = manifest()["fuzz"]["lossless"]
    ctx = webp_amd.Context(0)
    b = ctx.batch([d for _, d in cases])
    b.run()
    decoded = 0
    for i, (key, data) in enumerate(cases):
        w = want[key]
        assert int(b.status[i]) == w["status"], (key, int(b.status[i]), w["status"])
        if w["status"] != 0:
            continue
        rgba = b.rgba(i)
        assert _sha(rgba) == w["rgba"], f"mutant {key}: GPU != libwebp"
        info, coded, tdata = webp_amd.vp8l_parse(data)
        np.testing.assert_array_equal(rgba, oracle_vp8l_decode(info, coded, tdata), err_msg=f"mutant {key}")
        decoded += 1
    assert decoded >= 150, decoded
    b.close()
    ctx.close()
