"""Status parity with WebPDecode on corrupted, truncated and hand-built inputs.

tests/golden/status/sweep.json holds what libwebp 1.6.0 (Pillow's bundled build, plain C and
SIMD cross-checked; generator tests/golden/make_status_sweep.py) returns for ~2900 mutants
of the committed fixtures -- consistent-RIFF truncations that reach the VP8 / VP8L / ALPH
data, raw truncations, bit flips -- each without a crop window and with two crop windows
(libwebp decodes, and so fails on, only the rows a crop window needs).  The host stages
here must return the same status for every one (wg_decode_status; the batch API reports
the same per-frame status, tests/test_gpu_status.py).
"""
import collections

import numpy as np
import pytest

import webp_amd
from oracle_lib import load_fixture, mutate, oracle_still_rgba, oracle_vp8l_resolve, status_sweep

SWEEP = status_sweep()
BY_SRC = collections.defaultdict(list)
for c in SWEEP["cases"]:
    BY_SRC[c["src"]].append(c)


def opts_of(crop):
    return webp_amd.options(crop=tuple(crop)) if crop else None


@pytest.mark.parametrize("src", sorted(BY_SRC))
def test_status_matches_libwebp(src):
    data = load_fixture(src)
    bad = []
    for c in BY_SRC[src]:
        m = mutate(data, c["op"], c["arg"])
        got = webp_amd.decode_status(m, opts_of(c["crop"]))
        if got != c["status"]:
            bad.append((c["op"], c["arg"], c["crop"], c["status"], got))
    assert not bad, f"{len(bad)}/{len(BY_SRC[src])} differ (op, arg, crop, libwebp, ours): {bad[:8]}"


def test_sweep_covers_every_status_path():
    seen = collections.Counter(c["status"] for c in SWEEP["cases"])
    # OK, OUT_OF_MEMORY (alpha init), INVALID_PARAM (crop), BITSTREAM_ERROR, NOT_ENOUGH_DATA
    assert all(seen[s] > 0 for s in (0, 1, 2, 3, 7)), seen
    cropped_fail = [c for c in SWEEP["cases"] if c["crop"] and c["status"] == 0 and
                    any(d["status"] != 0 for d in BY_SRC[c["src"]]
                        if d["op"] == c["op"] and d["arg"] == c["arg"] and d["crop"] is None)]
    assert len(cropped_fail) >= 20, "the sweep must hold failures a crop window hides"


@pytest.mark.parametrize("name", sorted(SWEEP["crafted"]))
def test_crafted_vp8l_status(name):
    data = load_fixture("status/" + name)
    assert webp_amd.decode_status(data) == SWEEP["crafted"][name]


def test_crafted_out_of_alphabet_symbol_decodes():
    """Simple code (0, 200) for distances: 200 is ignored (ReadHuffmanCode builds the table
    over the alphabet only); the pixel is the literal the other codes give."""
    data = load_fixture("status/crafted_dist_oob_symbol")
    info, coded, _ = webp_amd.vp8l_parse(data)
    assert oracle_vp8l_resolve(info, coded).ravel().tolist() == [0xff104020]
    np.testing.assert_array_equal(oracle_still_rgba(data).ravel(), [0x10, 0x40, 0x20, 0xff])


def test_crafted_65536_groups_is_cheap():
    """A meta image selecting group 0xffff: only that group's tables are built (the other
    65535 groups' codes are read and validated), as libwebp's mapping does."""
    import resource
    data = load_fixture("status/crafted_65536_groups")
    before = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    info, coded, _ = webp_amd.vp8l_parse(data)
    grew_kb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - before
    assert oracle_vp8l_resolve(info, coded).ravel().tolist() == [0x00004000]
    assert grew_kb < 64 * 1024, grew_kb
