"""Sharding invariance: frames decoded through 1, 2 and 4 shards give
per-frame SHA-256 identical to each other and to libwebp 1.6.0's.

On the 1-GPU box the shards are independent contexts on device 0 (each with its own stream,
worker pool, staging arena and device buffers), decoded concurrently by
wg_decode_rgba_batch_multi -- the same code path as one context per GPU.  The reference has
no multi-device code (its only parallelism is WebPWorker, frame_dec.c.go:611-667)."""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import bench_files, load_lossy, manifest

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _c2_frames(n):
    paths = bench_files("c2_1080p")
    datas = [open(p, "rb").read() for p in paths]
    m = manifest()["bench"]
    want = [m[os.path.basename(p)]["sha256"]["rgba"] for p in paths]
    return [datas[i % len(datas)] for i in range(n)], [want[i % len(want)] for i in range(n)]


@pytest.mark.parametrize("shards", [1, 2, 4])
def test_c2_shards_identical(shards):
    frames, want = _c2_frames(24)
    mc = webp_amd.MultiContext([0] * shards, host_threads=4)
    try:
        outs, status = mc.decode_batch(frames)
        assert (status == 0).all(), status
        assert [_sha(o) for o in outs] == want
        # again through the same contexts (reused pinned staging and device buffers)
        outs2, status2 = mc.decode_batch(frames[::-1])
        assert (status2 == 0).all()
        assert [_sha(o) for o in outs2] == want[::-1]
    finally:
        mc.close()


def test_shards_with_bad_frames_and_mixed_sizes():
    """Bad frames keep their own status in whichever shard they land; odd-sized fixtures and
    bench frames mixed across 3 shards decode as in one context."""
    frames, want = _c2_frames(5)
    small, gold = load_lossy("synth_481x270")
    datas = [frames[0], b"not a webp", small, frames[1][:100], frames[2], small, frames[3]]
    ctx = webp_amd.Context(0, host_threads=2)
    mc = webp_amd.MultiContext([0, 0, 0], host_threads=2)
    try:
        ref, rst = ctx.decode_batch(datas)
        got, gst = mc.decode_batch(datas)
        assert list(rst) == list(gst)
        assert rst[1] != 0 and rst[3] != 0
        for a, b in zip(ref, got):
            assert (a is None) == (b is None)
            if a is not None:
                assert np.array_equal(a, b)
        assert np.array_equal(got[2], gold["rgba"])
        assert _sha(got[0]) == want[0]
    finally:
        mc.close()
        ctx.close()


def test_default_device_selection():
    """wg_set_default_device picks the context behind webp.Decode's drop-in entry."""
    data, gold = load_lossy("synth_80x96")
    webp_amd.set_default_device(0)
    assert np.array_equal(webp_amd.decode(data), gold["rgba"])
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.set_default_device(webp_amd.device_count())
    assert e.value.status == webp_amd.Status.INVALID_PARAM
    assert np.array_equal(webp_amd.decode(data), gold["rgba"])  # still device 0


def test_dropin_repeated_calls_reuse_buffers():
    """The single-frame drop-in path (webp.Decode) reuses the default context's buffers:
    many calls in a row, every one bit-exact."""
    data, gold = load_lossy("synth_481x270")
    for _ in range(50):
        assert np.array_equal(webp_amd.decode(data), gold["rgba"])
