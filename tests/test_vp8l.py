"""VP8L (lossless): host entropy stage + CPU oracle of the
inverse transforms against libwebp 1.6.0 (committed fixtures and the C5 bench frame's
SHA-256).  Pins the oracle that the device kernel is checked against."""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import GOLDEN, lossless_names, load_lossless, manifest, oracle_vp8l_decode


@pytest.mark.parametrize("name", lossless_names())
def test_vp8l_oracle_matches_libwebp(name):
    data, gold = load_lossless(name)
    info, coded, tdata = webp_amd.vp8l_parse(data)
    assert (info.width, info.height) == gold["rgba"].shape[1::-1]
    rgba = oracle_vp8l_decode(info, coded, tdata)
    np.testing.assert_array_equal(rgba, gold["rgba"], err_msg=name)


def test_vp8l_fixtures_cover_every_transform():
    seen = set()
    packing = set()
    for name in lossless_names():
        info, _, _ = webp_amd.vp8l_parse(load_lossless(name)[0])
        for i in range(info.num_transforms):
            seen.add(info.transform_type[i])
            if info.transform_type[i] == 3:
                packing.add(info.transform_bits[i])
    assert seen == {0, 1, 2, 3}, seen
    assert len(packing) >= 3, packing  # palette sizes exercising several pixel-packing widths


def test_vp8l_c5_bench_frames_sha256():
    """The oracle (color cache + copies + transforms) on all 8 committed C5 bitstreams vs
    libwebp's SHA-256; the tokens hold no resolved pixel (the host leaves the cache to the
    device)."""
    m = manifest()["bench"]
    for s in range(8):
        data = open(os.path.join(GOLDEN, "bench", f"c5_ll2048_s{s}.webp"), "rb").read()
        info, coded, tdata = webp_amd.vp8l_parse(data)
        assert (info.width, info.height) == (2048, 2048) and coded.cache_bits == info.cache_bits > 0
        kinds = np.bincount((coded.tokens.ravel() >> 30).astype(np.int64), minlength=4)
        assert kinds[0] == len(coded.lits) and kinds[1] > kinds[0] and kinds[3] == 0
        rgba = oracle_vp8l_decode(info, coded, tdata)
        assert hashlib.sha256(rgba.tobytes()).hexdigest() == m[f"c5_ll2048_s{s}.webp"]["sha256"]["rgba"], s


def test_vp8l_truncated_and_corrupt():
    data, _ = load_lossless("ll_corr_64x64")
    # raw cut: the VP8L chunk runs past the end of the file (DecodeInto's header pass)
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.vp8l_parse(data[: len(data) // 2])
    assert e.value.status == webp_amd.Status.NOT_ENOUGH_DATA
    # consistent RIFF, bitstream cut: any end of stream is a bitstream error in WebPDecode
    from oracle_lib import riff_truncate
    for frac in (0.3, 0.5, 0.9, 0.99):
        cut = riff_truncate(data, int(len(data) * frac))
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.vp8l_parse(cut)
        assert e.value.status == webp_amd.Status.BITSTREAM_ERROR
        assert webp_amd.decode_status(cut) == webp_amd.Status.BITSTREAM_ERROR
    with pytest.raises(webp_amd.WebPError):
        webp_amd.vp8l_parse(data[:30])
    lossy = open(os.path.join(GOLDEN, "bench", "c1_512_s0.webp"), "rb").read()
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.vp8l_parse(lossy)
    assert e.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
