"""GPU parity of the YUV output modes (MODE_YUV / MODE_YUVA; WebPDecodeYUV / WebPDecodeYUVInto,
pkg/libwebp/decoder/webp.go:615-725): wg_decode_yuv_batch / wg_decode_yuv_into / resident batches
through K8 (device/emit_yuva.hip) against libwebp 1.6.0's planes (tests/golden/yuv: every source x
crop x flip, statuses included) and the c3 / c3a 4K frames' plane SHA-256s.  Bit-exact."""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import bench_files, load_modes, load_yuv, manifest, parse_yuv_key, yuv_sources

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_yuv_modes_crops_flip_batches_vs_libwebp(ctx):
    """Every source (lossy with and without ALPH, lossless opaque / semi-transparent / odd-sized)
    x crop (odd origins: lossy snapped, lossless exact) x flip x MODE_YUV / MODE_YUVA, one batch per
    (key, crop window): statuses and planes = WebPDecode's."""
    srcs = [load_yuv(s) for s in yuv_sources()]
    keys = sorted({k for _, _, ent in srcs for k in ent["status"]})
    checked = 0
    for key in keys:
        mode, cname, flip = parse_yuv_key(key)
        group = [(d, g, e) for d, g, e in srcs if key in e["status"]]
        crops = {tuple(e["crops"][cname]) if e["crops"][cname] else None for _, _, e in group}
        for crop in crops:
            sub = [(d, g, e) for d, g, e in group if (tuple(e["crops"][cname]) if e["crops"][cname] else None) == crop]
            outs, status = ctx.decode_yuv_batch([d for d, _, _ in sub], webp_amd.options(mode, crop, flip))
            for (d, g, e), out, st in zip(sub, outs, status):
                assert st == e["status"][key], (key, e["source"], st)
                if st == 0:
                    planes = ("y", "u", "v", "a") if mode == 12 else ("y", "u", "v")
                    assert sorted(out) == sorted(planes)
                    for p in planes:
                        np.testing.assert_array_equal(out[p], g[f"{key}_{p}"], err_msg=f"{key} {e['source']} {p}")
                    checked += 1
    assert checked > 100, checked


def test_single_frame_decode_yuv_into():
    """wg_decode_yuv_into (WebPDecodeYUVInto's path): lossy + ALPH and lossless, crops, flip."""
    for src, key in (("alpha_64x48", "m12_c1_f1"), ("alpha_64x48", "m11_none_f0"), ("ll_alpha_odd_37x23", "m12_c5_f0"),
                     ("ll_corr_123x77", "m11_c4_f0")):
        data, g, ent = load_yuv(src)
        mode, cname, flip = parse_yuv_key(key)
        out = webp_amd.decode_yuv(data, webp_amd.options(mode, ent["crops"][cname], flip))
        for p in out:
            np.testing.assert_array_equal(out[p], g[f"{key}_{p}"], err_msg=f"{src} {key} {p}")


def test_yuv_buffer_checks_and_refusals(ctx):
    """External-memory checks as CheckDecBuffer's: a short plane or stride, or MODE_YUVA without an
    A plane, is INVALID_PARAM for that frame; the single-buffer entry points refuse YUV modes."""
    import ctypes as C
    data, _, _ = load_yuv("synth_80x96")
    L = webp_amd.lib()
    for mode, bad in ((11, "y_stride"), (11, "u_size"), (12, "a")):
        out, buf = webp_amd._yuva_arrays(80, 96, mode == 12)
        setattr(buf, bad, getattr(buf, bad) - 1 if bad != "a" else None)
        b = bytes(data)
        assert L.wg_decode_yuv_into(b, len(b), C.byref(webp_amd.options(mode)), C.byref(buf)) == \
            webp_amd.Status.INVALID_PARAM, (mode, bad)
    with pytest.raises(webp_amd.WebPError) as ei:
        ctx.decode_batch_opts([data], webp_amd.options(11))
    assert ei.value.status == webp_amd.Status.INVALID_PARAM
    with pytest.raises(webp_amd.WebPError) as ei:
        webp_amd.decode_into(data, webp_amd.options(12))
    assert ei.value.status == webp_amd.Status.INVALID_PARAM


def test_resident_yuv_batch_runs_k8(ctx):
    """A batch created in MODE_YUVA with a crop window: every run is K1 (planes, no RGBA tail, no
    K2), K7 / K3 / K4 and K8 in the K6 stage (kernel_ms[5]); the planes after repeated runs are
    libwebp's.  Lossy frames of such a batch have no RGBA (UNSUPPORTED_FEATURE); lossless ones keep
    K3's; wg_batch_download refuses the batch (its output is planes)."""
    key = "m12_c4_f0"
    srcs = [load_yuv(s) for s in yuv_sources()]
    sub = [(d, g, e) for d, g, e in srcs if e["status"].get(key) == 0]
    crop = tuple(sub[0][2]["crops"]["c4"])
    b = ctx.batch([d for d, _, _ in sub], opts=webp_amd.options(12, crop, 0))
    try:
        for _ in range(2):
            b.run()
        ms = b.kernel_ms()
        assert ms[5] > 0 and ms[1] == 0, ms
        assert b.kernel_bytes()[5] > 0
        for i, (d, g, e) in enumerate(sub):
            out = b.yuva(i)
            for p in "yuva":
                np.testing.assert_array_equal(out[p], g[f"{key}_{p}"], err_msg=f"{e['source']} {p}")
            lossless = webp_amd.features(d).format == 2
            if not lossless:
                with pytest.raises(webp_amd.WebPError) as ei:
                    b.rgba(i)
                assert ei.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
            with pytest.raises(webp_amd.WebPError) as ei:
                b.download(i)
            assert ei.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
    finally:
        b.close()
    rgb = ctx.batch([sub[0][0]], opts=webp_amd.options(1))
    try:
        rgb.run()
        with pytest.raises(webp_amd.WebPError) as ei:
            rgb.yuva(0)
        assert ei.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
    finally:
        rgb.close()


@pytest.mark.parametrize("prefix,mode", [("c3_4k", 11), ("c3a_4k", 12)])
def test_yuv_bench_frames(ctx, prefix, mode):
    """4K frames in MODE_YUV (c3) and MODE_YUVA (c3a: lossless ALPH, A from K4's unfiltered plane):
    every plane's SHA-256 = libwebp's."""
    m = manifest()["bench"]
    paths = bench_files(prefix)[:4]
    outs, status = ctx.decode_yuv_batch([open(p, "rb").read() for p in paths], webp_amd.options(mode))
    assert (status == 0).all(), status
    for p, out in zip(paths, outs):
        ent = m[os.path.basename(p)]["sha256"]
        for k in out:
            assert _sha(out[k]) == ent[k], (p, k)


def test_rgb_modes_unchanged_next_to_yuv(ctx):
    """(The RGB-family path after YUV batches on the same context: a mode fixture still matches.)"""
    data, g, e = load_modes("alpha_64x48")
    outs, status = ctx.decode_batch_opts([data], webp_amd.options(7, None, 1, 0))
    np.testing.assert_array_equal(outs[0], g["m7_none_f1_nf0"])
