"""Output colorspaces, cropping and flip on the oracle side (no GPU): for every
source x mode x crop window x flip x fancy/point case, the oracles' restatement of the output stage
reproduces libwebp 1.6.0's WebPDecode bytes, and windows libwebp rejects are rejected."""
import numpy as np
import pytest

import webp_amd
from oracle_lib import MODE_BPP, load_modes, mode_sources, oracle_output, parse_mode_key

SOURCES = mode_sources()


def test_output_bpp():
    for mode, bpp in MODE_BPP.items():
        assert webp_amd.output_bpp(mode) == bpp
    for mode in (11, 12, 13, -1):
        assert webp_amd.output_bpp(mode) == 0


@pytest.mark.parametrize("src", SOURCES)
def test_modes_oracle_vs_libwebp(src):
    data, gold, ent = load_modes(src)
    n = 0
    for key, st in ent["status"].items():
        mode, cname, flip, nf = parse_mode_key(key)
        crop = ent["crops"][cname]
        out = oracle_output(data, mode, crop, flip, nf)
        if st != 0:
            assert st == webp_amd.Status.INVALID_PARAM and out is None, key
            continue
        if key in gold:
            np.testing.assert_array_equal(out, gold[key], err_msg=key)
            n += 1
    assert n > 0
