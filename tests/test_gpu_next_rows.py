"""GPU parity of the bench workloads of SURVEY §8's "next" rows at full size, against libwebp
1.6.0 (manifest "bench" / "bench_anim", made by tests/golden/make_golden.py):

* c3a (f2, K4): 8 x 4K lossy + lossless-compressed ALPH frames, the bench's 256-frame layout
  (frames cycled), RGBA SHA-256 with K1's tail and with a separate K2, and point sampling; the same
  frames with the ALPH filter set to gradient (c3ag) and vertical (c3av);
* c3rgb565 (f4): C3's frames decoded to MODE_RGB_565 as a resident batch -- K1's tail emits the
  565 pixels itself (no RGBA copy, no K6) -- SHA-256 of WebPDecode's bytes;
* anim (f3, K5): the 64-frame 1920x1080 animation as a resident animation batch, every
  canvas's SHA-256 against WebPAnimDecoder and its timestamps, on repeated runs.

Plus the oracle on one frame of each (the CPU restatement the bench's cpu_baseline times)."""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import GOLDEN, bench_files, manifest, oracle_output, oracle_still_rgba

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


@pytest.mark.parametrize("mode", ["fused", "separate", "point"])
def test_c3a_alpha_frames(ctx, mode):
    paths = bench_files("c3a_4k")
    assert len(paths) == 8
    m = manifest()["bench"]
    datas = [open(p, "rb").read() for p in paths]
    n = 24  # three of each seed, interleaved as the bench cycles them
    flags = webp_amd.FLAG_NO_FANCY_UPSAMPLING if mode == "point" else 0
    b = ctx.batch([datas[i % 8] for i in range(n)], flags)
    try:
        assert (b.status == 0).all(), b.status
        b.set_emit(mode == "separate")
        for _ in range(2):
            b.run()
        ms = b.kernel_ms()
        assert ms[0] > 0 and ms[3] > 0 and ms[4] > 0, ms  # K1, K4 and the alpha streams' K7
        assert ms[2] == 0, ms  # 8-bit alpha streams (a color map only): K4 expands them from K7's output, no K3
        key = "rgba_point" if mode == "point" else "rgba"
        for i in range(n):
            want = m[os.path.basename(paths[i % 8])]["sha256"][key]
            assert _sha(b.rgba(i)) == want, (mode, i)
    finally:
        b.close()


@pytest.mark.parametrize("prefix", ["c3ag_4k", "c3av_4k"])
@pytest.mark.parametrize("mode", ["fused", "separate"])
def test_c3ag_c3av_gradient_vertical_alpha(ctx, prefix, mode):
    """c3a's frames with the ALPH filter set to gradient (c3ag) / vertical (c3av): K4 gathers the
    8-bit streams' bytes from K7's coded image through their colour map (no K3), then its wavefront /
    column-sum unfilters -- 16 frames (every seed twice), alpha-first (K4 before K1's tail) and with
    a separate K2; RGBA SHA-256 = libwebp's."""
    paths = bench_files(prefix)
    assert len(paths) == 8
    m = manifest()["bench"]
    datas = [open(p, "rb").read() for p in paths]
    n = 16
    b = ctx.batch([datas[i % 8] for i in range(n)])
    try:
        assert (b.status == 0).all(), b.status
        b.set_emit(mode == "separate")
        for _ in range(2):
            b.run()
        ms = b.kernel_ms()
        assert ms[0] > 0 and ms[3] > 0 and ms[4] > 0 and ms[2] == 0, ms  # K1, K4, K7; no K3
        for i in range(n):
            assert _sha(b.rgba(i)) == m[os.path.basename(paths[i % 8])]["sha256"]["rgba"], (prefix, mode, i)
    finally:
        b.close()


def test_c3a_oracle_one_frame():
    p = bench_files("c3a_4k")[3]
    want = manifest()["bench"][os.path.basename(p)]["sha256"]["rgba"]
    assert _sha(oracle_still_rgba(open(p, "rb").read())) == want


def test_c3_rgb565_resident_batch(ctx):
    paths = bench_files("c3_4k")
    m = manifest()["bench"]
    datas = [open(p, "rb").read() for p in paths]
    b = ctx.batch([datas[i % 8] for i in range(16)], opts=webp_amd.options(6))  # MODE_RGB_565
    try:
        for _ in range(2):
            b.run()
        ms = b.kernel_ms()
        assert ms[0] > 0 and ms[5] == 0, ms  # K1's tail writes RGB_565 itself: no RGBA copy, no K6
        for i in range(16):
            out = b.download(i)
            assert out.shape == (2160, 3840 * 2)
            assert _sha(out) == m[os.path.basename(paths[i % 8])]["sha256"]["rgb565"], i
    finally:
        b.close()


def test_c3_rgb565_oracle_one_frame():
    p = bench_files("c3_4k")[5]
    want = manifest()["bench"][os.path.basename(p)]["sha256"]["rgb565"]
    assert _sha(oracle_output(open(p, "rb").read(), mode=6)) == want


def test_anim_1080p_resident(ctx):
    ent = manifest()["bench_anim"]["anim_1080p_x64"]
    data = open(os.path.join(GOLDEN, "bench", "anim_1080p_x64.webp"), "rb").read()
    b = ctx.anim_batch(data)
    try:
        assert (b.n, b.canvas_width, b.canvas_height) == (64, 1920, 1080)
        for r in range(2):
            b.run()
            canv, ts = b.canvases()
            assert ts.tolist() == ent["timestamps"]
            got = [_sha(c) for c in canv]
            bad = [i for i, (g, w) in enumerate(zip(got, ent["canvas_sha256"])) if g != w]
            assert not bad, (r, bad[:8])
        ms = b.kernel_ms()
        assert ms[0] > 0 and ms[6] > 0, ms
    finally:
        b.close()
