"""Animation (ANIM / ANMF) on the host/oracle side (no GPU): the host demux agrees with the
container's own frame headers, and host demux + oracle decodes of every fragment + the
oracle's compositing reproduce the canvases and timestamps of libwebp 1.6.0's
WebPAnimDecoder (MODE_RGBA) for every fixture."""
import numpy as np
import pytest

import webp_amd
from oracle_lib import anim_names, load_anim, load_lossless, load_lossy, manifest, oracle_anim

NAMES = anim_names()


def test_fixture_set_covers_blend_dispose_and_keyframes():
    frames = [f for v in manifest()["anim"].values() for f in v["frames"]]
    kinds = {(f["dispose_bg"], f["no_blend"], f["alpha"]) for f in frames}
    assert {(0, 0, True), (1, 0, True), (0, 1, True), (1, 1, True), (0, 1, False)} <= kinds
    assert any(v["info"]["frame_count"] == 1 for v in manifest()["anim"].values())


@pytest.mark.parametrize("name", NAMES)
def test_demux_vs_container_headers(name):
    data, _ = load_anim(name)
    info, frames = webp_amd.anim_demux(data)
    ent = manifest()["anim"][name]
    assert (info.canvas_width, info.canvas_height, info.loop_count, info.bgcolor, info.frame_count) == tuple(
        ent["info"][k] for k in ("canvas_width", "canvas_height", "loop_count", "bgcolor", "frame_count"))
    for f, m in zip(frames, ent["frames"]):
        assert (f.x_offset, f.y_offset, f.width, f.height, f.duration, f.dispose_background, f.no_blend) == (
            m["x"], m["y"], m["w"], m["h"], m["duration"], m["dispose_bg"], m["no_blend"])
        assert bool(f.has_alpha) == m["alpha"]


@pytest.mark.parametrize("name", NAMES)
def test_anim_oracle_vs_libwebp(name):
    data, gold = load_anim(name)
    canv, ts = oracle_anim(data)
    np.testing.assert_array_equal(ts, gold["timestamps"])
    np.testing.assert_array_equal(canv, gold["canvases"])


def test_still_images_demux_as_one_frame():
    for data, w, h in ((load_lossy("synth_80x96")[0], 80, 96), (load_lossless("ll_alpha_48x48")[0], 48, 48),
                       (load_lossy("alpha_64x48")[0], 64, 48)):
        info, frames = webp_amd.anim_demux(data)
        assert (info.canvas_width, info.canvas_height, info.frame_count) == (w, h, 1)
        assert (frames[0].x_offset, frames[0].y_offset, frames[0].width, frames[0].height) == (0, 0, w, h)


def test_demux_rejects_broken_containers():
    data, _ = load_anim("anim_manual_blend_dispose")
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.anim_demux(data[:len(data) - 7])  # truncated
    assert e.value.status == webp_amd.Status.NOT_ENOUGH_DATA
    b = bytearray(data)
    i = b.index(b"ANIM")
    b[i:i + 4] = b"XXXX"  # ANMF frames without a preceding ANIM
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.anim_demux(bytes(b))
    assert e.value.status == webp_amd.Status.BITSTREAM_ERROR
    b = bytearray(data)
    i = b.index(b"ANMF") + 8
    b[i:i + 3] = (30).to_bytes(3, "little")  # x offset 60 + width 64 > canvas 64
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.anim_demux(bytes(b))
    assert e.value.status == webp_amd.Status.BITSTREAM_ERROR
