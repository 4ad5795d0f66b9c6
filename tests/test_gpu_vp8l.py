"""GPU parity of K3 (VP8L inverse transforms + RGBA) through the C ABI, against libwebp
1.6.0 fixtures, the CPU oracle and the C5 bench frame's SHA-256.  Bit-exact."""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import (GOLDEN, bench_files, load_lossless, load_lossy, lossless_names, manifest, oracle_decode,
                        oracle_vp8l_decode)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


def test_lossless_fixtures_batch_vs_golden_and_oracle(ctx):
    names = lossless_names()
    datas = [load_lossless(n)[0] for n in names]
    imgs, status = ctx.decode_batch(datas)
    assert (status == 0).all(), dict(zip(names, status))
    for n, d, img in zip(names, datas, imgs):
        gold = load_lossless(n)[1]["rgba"]
        np.testing.assert_array_equal(img, gold, err_msg=n)
        info, coded, tdata = webp_amd.vp8l_parse(d)
        np.testing.assert_array_equal(img, oracle_vp8l_decode(info, coded, tdata), err_msg=n)


def test_c5_bench_frames_sha256(ctx):
    """All 8 distinct C5 bitstreams (corr_luma seeds 0..7, the bench cycles them) through
    K7 + K3, twice in one batch (several workgroups per frame), against libwebp's SHA-256."""
    paths = bench_files("c5_ll2048")
    assert len(paths) == 8
    datas = [open(p, "rb").read() for p in paths]
    b = ctx.batch(datas + datas[:3])
    assert (b.status == 0).all(), b.status
    b.run()
    m = manifest()["bench"]
    want = [m[os.path.basename(p)]["sha256"]["rgba"] for p in paths]
    want = want + want[:3]
    for i in range(b.n):
        assert hashlib.sha256(b.rgba(i).tobytes()).hexdigest() == want[i], i
    b.run()
    assert hashlib.sha256(b.rgba(2).tobytes()).hexdigest() == want[2]  # idempotent re-run
    ms = b.kernel_ms()
    assert ms[0] == 0 and ms[1] == 0 and ms[2] > 0 and ms[3] == 0 and ms[4] > 0  # K3, K7 only
    b.close()


def test_mixed_lossy_lossless_batch(ctx):
    ll, ll_gold = load_lossless("ll_pal16_65x39")
    ll2, ll2_gold = load_lossless("ll_corr_123x77")
    ly, _ = load_lossy("synth_80x96")
    imgs, status = ctx.decode_batch([ly, ll, ly, ll2])
    assert (status == 0).all(), status
    info, mbs = webp_amd.vp8_parse(ly)
    want = oracle_decode(info, mbs)["rgba"]
    np.testing.assert_array_equal(imgs[0], want)
    np.testing.assert_array_equal(imgs[2], want)
    np.testing.assert_array_equal(imgs[1], ll_gold["rgba"])
    np.testing.assert_array_equal(imgs[3], ll2_gold["rgba"])


def test_lossless_single_decode_dropin():
    data, gold = load_lossless("ll_alpha_48x48")
    np.testing.assert_array_equal(webp_amd.decode(data), gold["rgba"])


def test_lossless_yuv_download_unsupported(ctx):
    data, _ = load_lossless("ll_corr_64x64")
    b = ctx.batch([data])
    b.run()
    with pytest.raises(webp_amd.WebPError) as e:
        b.yuv(0)
    assert e.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
    b.close()
