"""GPU parity of the ALPH path (K3 for lossless alpha streams + K4 unfilter / A channel) through
the C ABI, against libwebp 1.6.0 fixtures and the CPU oracle.  Bit-exact."""
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import (GOLDEN, alpha_names, load_alpha, load_lossless, load_lossy, manifest,
                        oracle_alpha_plane, oracle_decode)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


def _oracle_rgba(data):
    info, mbs = webp_amd.vp8_parse(data)
    rgba = oracle_decode(info, mbs)["rgba"]
    rgba[..., 3] = oracle_alpha_plane(data)[1]
    return rgba


def test_alpha_fixtures_batch_vs_golden_and_oracle(ctx):
    names = alpha_names()
    datas = [load_alpha(n)[0] for n in names]
    imgs, status = ctx.decode_batch(datas)
    assert (status == 0).all(), dict(zip(names, status))
    for n, d, img in zip(names, datas, imgs):
        np.testing.assert_array_equal(img, load_alpha(n)[1]["rgba"], err_msg=n)
        np.testing.assert_array_equal(img, _oracle_rgba(d), err_msg=n)


def test_corrupt_alph_statuses_in_a_mixed_batch(ctx):
    errs = manifest()["alpha_errors"]
    bad = sorted(errs)
    good, good_gold = load_alpha("a_ll_g_120x1100")
    datas = [open(os.path.join(GOLDEN, "alpha", n + ".webp"), "rb").read() for n in bad] + [good]
    imgs, status = ctx.decode_batch(datas)
    for n, st in zip(bad, status):
        assert st == errs[n]["status"], n
    assert status[-1] == 0
    np.testing.assert_array_equal(imgs[-1], good_gold["rgba"])


@pytest.mark.parametrize("k1", ["fused", "auto"])
def test_mixed_alpha_lossy_lossless_batch_and_timing(ctx, k1):
    a, a_gold = load_alpha("a_ll_v_97x81")
    r, r_gold = load_alpha("a_raw_g_40x1030")
    ly, _ = load_lossy("synth_80x96")
    ll, ll_gold = load_lossless("ll_corr_123x77")
    b = ctx.batch([a, ly, ll, r, a])
    if k1 == "fused":
        b.set_emit(False)  # K1's RGBA tail (the one-workgroup kernel)
    b.run()
    ms = b.kernel_ms()
    # K1, K3, K4 ran; the lossy RGBA from K1's tail (no K2), or -- the automatic choice for this
    # small batch, whose 1030-row frame has 17 quads -- the split K1 and K2
    assert ms[0] > 0 and ms[2] > 0 and ms[3] > 0, ms
    assert (ms[1] == 0) == (k1 == "fused"), ms
    np.testing.assert_array_equal(b.rgba(0), a_gold["rgba"])
    np.testing.assert_array_equal(b.rgba(2), ll_gold["rgba"])
    np.testing.assert_array_equal(b.rgba(3), r_gold["rgba"])
    np.testing.assert_array_equal(b.rgba(4), a_gold["rgba"])
    info, mbs = webp_amd.vp8_parse(ly)
    np.testing.assert_array_equal(b.rgba(1), oracle_decode(info, mbs)["rgba"])
    b.run()  # idempotent re-run (K2 rewrites A = 255, K4 the plane)
    np.testing.assert_array_equal(b.rgba(3), r_gold["rgba"])
    b.close()


@pytest.mark.parametrize("n", [5, 260])
def test_alpha_first_follows_k1_configuration(ctx, n):
    """Alpha-first batches (K4 before the YUV -> RGBA strips, which take A from its planes; capi.cpp
    set_alpha_first) are re-decided whenever the K1 configuration changes: the automatic choice (a
    small batch: the split K1 with K7 on the side stream and K4 -> K2; 260 frames: alpha-first with
    K1's tail), then K1's RGBA tail (set_emit(False): with K7 beside K1 no longer alpha-first), K2
    (set_emit(True)), forced split parts and back -- every frame equal to libwebp 1.6.0 after each
    run, the descriptors re-uploaded on every switch."""
    names = ["a_ll_h_130x70", "a_raw_h_71x33", "a_raw_g_64x64", "a_ll_v_97x81", "a_raw_g_40x1030"]
    datas = [load_alpha(x)[0] for x in names]
    golds = [load_alpha(x)[1]["rgba"] for x in names]
    idx = [i % len(names) for i in range(n)]
    b = ctx.batch([datas[i] for i in idx])
    try:
        assert (b.status == 0).all()
        steps = [("auto", None), ("tail", lambda: b.set_emit(False)), ("k2", lambda: b.set_emit(True))]
        if n < 256:  # (the split kernel is for batches of fewer frames than CUs)
            steps.append(("split3", lambda: b.set_k1_parts(3)))
        steps += [("one", lambda: b.set_k1_parts(1)), ("tail2", lambda: b.set_emit(False)),
                  ("auto2", lambda: b.set_k1_parts(0))]
        for name, act in steps:
            if act is not None:
                act()
            b.run()
            ms = b.kernel_ms()
            assert ms[0] > 0 and ms[3] > 0, (name, ms)
            for i in sorted({0, 1, 2, 3, 4, n - 1}):
                np.testing.assert_array_equal(b.rgba(i), golds[idx[i]], err_msg=f"{name} frame {i}")
    finally:
        b.close()


def test_alpha_single_decode_dropin():
    data, gold = load_alpha("a_ll_q50_80x80")
    np.testing.assert_array_equal(webp_amd.decode(data), gold["rgba"])
    data, gold = load_lossy("alpha_64x48")
    np.testing.assert_array_equal(webp_amd.decode(data), gold["rgba"])


@pytest.mark.parametrize("name", ["a_ll_h_130x70", "a_raw_h_71x33", "a_ll_none_33x65", "a_raw_none_40x30",
                                  "a_ll_v_97x81", "a_raw_g_64x64", "a_ll_best_g_96x64", "a_ll_levels_90x60",
                                  "a_ll_bin_h_133x40", "a_ll_bin_none_70x45", "a_ll_rl_h_64x33", "a_ll_many_h_66x90"])
def test_alpha_crop_windows_every_filter(ctx, name):
    """K4 writes the A bytes of a crop window: the direct row path (filters none / horizontal:
    rows from the column-0 prefix, window columns at any offset, 16-byte and dword stores; from
    raw bytes, from K3's RGBA, or -- 8-bit alpha streams: a palette of 1 / 2 / 8 pixels per
    coded pixel, or no transform -- from K7's coded image with K3 skipped) and the plane path
    (vertical / gradient), in batches large enough and small enough to change the
    rows-per-workgroup split.  Against the CPU oracle's WebPDecode with the same options."""
    from oracle_lib import oracle_output
    data = load_alpha(name)[0]
    f = webp_amd.features(data)
    W, H = f.width, f.height
    crops = [(0, 0, W, H), (2, 1, W - 2, H - 1), (4, 6, min(17, W - 4), min(9, H - 6)), (8, 0, W - 8, 3),
             (W - 5, H - 4, 5, 4)]
    for crop in crops:
        want = oracle_output(data, mode=1, crop=crop)
        opts = webp_amd.options(1, crop)
        for n in (1, 3, 70):
            b = ctx.batch([data] * n, opts=opts)
            try:
                assert (b.status == 0).all()
                b.run()
                for i in sorted({0, n - 1}):
                    got = b.download(i)
                    np.testing.assert_array_equal(got.reshape(want.shape), want, err_msg=f"{name} {crop} n={n} i={i}")
            finally:
                b.close()
