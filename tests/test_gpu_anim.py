"""GPU parity of the animation path: every frame's fragment through one decode batch (K1..K4),
then the device compositor (K5), against libwebp 1.6.0's WebPAnimDecoder canvases and the CPU
oracle.  Bit-exact."""
import numpy as np
import pytest

import webp_amd
from oracle_lib import anim_names, load_anim, load_lossless, load_lossy, oracle_anim

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", anim_names())
def test_anim_vs_libwebp_and_oracle(ctx, name):
    data, gold = load_anim(name)
    canv, ts = ctx.decode_anim(data)
    np.testing.assert_array_equal(ts, gold["timestamps"])
    np.testing.assert_array_equal(canv, gold["canvases"])
    ocanv, ots = oracle_anim(data)
    np.testing.assert_array_equal(canv, ocanv)


def test_still_image_as_one_frame_animation(ctx):
    for data, gold in (load_lossy("alpha_64x48"), load_lossless("ll_pal16_65x39")):
        canv, ts = ctx.decode_anim(data)
        assert canv.shape[0] == 1 and ts.tolist() == [0]
        np.testing.assert_array_equal(canv[0], gold["rgba"])


def test_animated_file_through_still_api_is_unsupported(ctx):
    data, _ = load_anim("anim_enc_mixed_96x80")
    _, status = ctx.decode_batch([data])
    assert status[0] == webp_amd.Status.UNSUPPORTED_FEATURE
    w, h, _ = webp_amd.decode_config(data)
    assert (w, h) == (96, 80)


@pytest.mark.parametrize("name", anim_names())
def test_resident_anim_batch(ctx, name):
    """wg_anim_batch_create: the animation resident in HBM, every run decoding the frames and
    compositing the canvases (K5 as the batch's last stage, its own kernel_ms entry): the
    canvases of repeated runs equal WebPAnimDecoder's."""
    data, gold = load_anim(name)
    b = ctx.anim_batch(data)
    try:
        assert (b.n, b.canvas_height, b.canvas_width) == gold["canvases"].shape[:3]
        for _ in range(2):
            b.run()
            canv, ts = b.canvases()
            np.testing.assert_array_equal(canv, gold["canvases"])
            np.testing.assert_array_equal(ts, gold["timestamps"])
        assert b.kernel_ms()[6] > 0
        assert b.kernel_bytes()[6] >= 4.0 * canv.size // 4
    finally:
        b.close()
