"""MODE_YUV / MODE_YUVA (WebPDecodeYUV / WebPDecodeYUVInto, pkg/libwebp/decoder/webp.go:615-725):
the CPU oracle against libwebp 1.6.0's outputs (tests/golden/yuv, tests/golden/make_golden.py
section "yuv") for every source x crop x flip -- lossy planes (EmitYUV, io_dec.c.go:36-50), the
alpha plane or 0xff (EmitAlphaYUV :128-150), lossless through WebPImportYUVAFromRGBA
(vp8l_dec.c.go:606-650, dsp/yuv.go:304-385: gamma-corrected 2x2 averages, alpha-weighted in
MODE_YUVA).  CPU only; the device path is tests/test_gpu_yuv.py."""
import numpy as np
import pytest

from oracle_lib import load_yuv, oracle_yuva, parse_yuv_key, yuv_sources


def _cases():
    out = []
    for src in yuv_sources():
        _, _, ent = load_yuv(src)
        out += [(src, k) for k in sorted(ent["status"])]
    return out


@pytest.mark.parametrize("src,key", _cases())
def test_oracle_yuva_matches_libwebp(src, key):
    data, g, ent = load_yuv(src)
    mode, cname, flip = parse_yuv_key(key)
    crop = ent["crops"][cname]
    got = oracle_yuva(data, mode, crop, flip)
    if ent["status"][key] != 0:
        assert got is None, key
        return
    planes = ("y", "u", "v", "a") if mode == 12 else ("y", "u", "v")
    assert sorted(got) == sorted(planes)
    for p in planes:
        np.testing.assert_array_equal(got[p], g[f"{key}_{p}"], err_msg=f"{src} {key} {p}")


def test_sources_cover_the_yuva_paths():
    """Lossless frames with odd width and height (the odd last column / row), semi-transparent
    ones (A plane), lossy frames with and without ALPH."""
    import webp_amd
    kinds = set()
    for src in yuv_sources():
        data, _, ent = load_yuv(src)
        f = webp_amd.features(data)
        kinds.add(("ll" if f.format == 2 else "lossy", bool(f.has_alpha), ent["width"] % 2, ent["height"] % 2))
    assert ("ll", True, 1, 1) in kinds and ("lossy", True, 0, 0) in kinds and ("lossy", False, 1, 1) in kinds
