"""The pipelined wg_decode_rgba_batch (capi.cpp decode_pipelined): frames in chunks, chunk k + 1's
host entropy stage and upload overlapping chunk k's kernels and download, two staging arenas and
two streams.  Every frame must come out as a one-batch decode does: per-frame SHA-256 against
libwebp 1.6.0's (manifest "bench"), bad frames keeping their own status in whichever chunk they
land, into pageable or pinned (wg_host_alloc) outputs.  The reference's counterpart is the
parse / finish overlap of its threaded decode (frame_dec.c.go:505-534, 611-667)."""
import hashlib

import numpy as np
import pytest

import webp_amd
from oracle_lib import load_alpha, load_lossless, load_lossy
from test_gpu_multi import _c2_frames

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("chunk", [0, 1, 3, 7, 64])
def test_chunks_bit_exact(chunk):
    frames, want = _c2_frames(22)
    ctx = webp_amd.Context(0, host_threads=4)
    try:
        ctx.set_chunk_frames(chunk)
        outs, status = ctx.decode_batch(frames)
        assert (status == 0).all(), status
        assert [_sha(o) for o in outs] == want
        ps = ctx.pipeline_stats()
        expect_chunks = {0: None, 1: 22, 3: 8, 7: 4, 64: 1}[chunk]
        if expect_chunks is not None:
            assert ps.chunks == expect_chunks
        assert ps.frames == 22
        assert ps.d2h_bytes == sum(o.nbytes for o in outs)
        assert ps.kernel_ms > 0 and ps.wall_s > 0
    finally:
        ctx.close()


def test_pinned_outputs_and_reuse():
    """Outputs in page-locked memory (written by DMA) and the same context reused: identical
    bytes, several calls in a row with different chunkings."""
    frames, want = _c2_frames(12)
    ctx = webp_amd.Context(0, host_threads=4)
    try:
        outs = [webp_amd.pinned_empty((1080, 1920, 4)) for _ in frames]
        for chunk in (2, 5, 0):
            for o in outs:
                o.fill(0x5A)
            ctx.set_chunk_frames(chunk)
            got, status = ctx.decode_batch(frames, out=outs)
            assert (status == 0).all(), status
            assert [_sha(o) for o in outs] == want
            assert all(g is o for g, o in zip(got, outs))
    finally:
        ctx.close()


def test_bad_frames_and_mixed_content_across_chunks():
    """Broken, lossless, lossy+odd-size frames spread over chunks of 2: each frame's status and
    bytes equal a one-chunk decode's, and the goldens."""
    frames, want = _c2_frames(4)
    small, gold = load_lossy("synth_481x270")
    ll, llgold = load_lossless("ll_corr_123x77")
    datas = [frames[0], b"RIFF\x00\x00\x00\x00WEBP", small, frames[1][:500], ll, frames[2], small, b"",
             frames[3], ll]
    ctx = webp_amd.Context(0, host_threads=3)
    try:
        ctx.set_chunk_frames(len(datas))
        ref, rst = ctx.decode_batch(datas)
        ctx.set_chunk_frames(2)
        got, gst = ctx.decode_batch(datas)
        assert list(rst) == list(gst)
        assert gst[1] != 0 and gst[3] != 0 and gst[7] != 0
        for a, b in zip(ref, got):
            assert (a is None) == (b is None)
            if a is not None:
                assert np.array_equal(a, b)
        assert _sha(got[0]) == want[0] and _sha(got[5]) == want[2] and _sha(got[8]) == want[3]
        assert np.array_equal(got[2], gold["rgba"]) and np.array_equal(got[6], gold["rgba"])
        assert np.array_equal(got[4], llgold["rgba"]) and np.array_equal(got[9], llgold["rgba"])
    finally:
        ctx.close()


def test_alpha_and_wide_frames_across_chunks():
    """VP8+ALPH frames (K4 after K1 / K3 in each chunk) and frames wider than K1's LDS column
    store (its global-column instantiation) in chunks of one to three frames: every frame equals
    libwebp's RGBA."""
    names = ["a_ll_best_g_96x64", "a_raw_h_71x33", "a_ll_g_120x1100", "a_ll_q50_80x80"]
    alpha = [load_alpha(n) for n in names]
    wide = [load_lossy(n) for n in ("wide_9617x40", "wide_16383x17_simple")]
    frames_c2, want_c2 = _c2_frames(2)
    datas = [alpha[0][0], wide[0][0], frames_c2[0], alpha[1][0], alpha[2][0], wide[1][0], alpha[3][0],
             frames_c2[1]]
    golds = [alpha[0][1]["rgba"], wide[0][1]["rgba"], None, alpha[1][1]["rgba"], alpha[2][1]["rgba"],
             wide[1][1]["rgba"], alpha[3][1]["rgba"], None]
    ctx = webp_amd.Context(0, host_threads=3)
    try:
        for chunk in (1, 2, 3):
            ctx.set_chunk_frames(chunk)
            got, st = ctx.decode_batch(datas)
            assert (st == 0).all(), (chunk, st)
            for i, (g, want) in enumerate(zip(got, golds)):
                if want is not None:
                    assert np.array_equal(g, want), (chunk, i)
            assert _sha(got[2]) == want_c2[0] and _sha(got[7]) == want_c2[1]
    finally:
        ctx.close()


def test_undersized_outputs_rejected_not_overrun():
    """A reused output buffer smaller than the frame (fewer rows, or a narrower stride) is the
    frame's INVALID_PARAM and nothing is written past it (WebPDecodeRGBAInto's size check,
    webp.go:592-594): the capacity array of wg_decode_rgba_batch / wg_decode_batch is checked
    per frame.  The other frames of the batch decode normally."""
    frames, want = _c2_frames(3)
    ctx = webp_amd.Context(0, host_threads=2)
    try:
        for chunk in (0, 1):
            ctx.set_chunk_frames(chunk)
            backing = np.full((1080 + 16, 1920, 4), 0xA5, np.uint8)
            short = backing[:1000]  # 80 rows short of the frame; the sentinel rows follow it
            narrow = np.zeros((1080, 1900, 4), np.uint8)  # stride 4 * 1900 < 4 * 1920
            good = np.zeros((1080, 1920, 4), np.uint8)
            got, st = ctx.decode_batch(frames, out=[short, good, narrow])
            assert list(st) == [webp_amd.Status.INVALID_PARAM, 0, webp_amd.Status.INVALID_PARAM], st
            assert got[0] is None and got[2] is None
            assert _sha(got[1]) == want[1]
            assert (backing[1000:] == 0xA5).all(), "rows past the short buffer were written"
        # the options path (wg_decode_batch) checks the same against bpp * width
        opts = webp_amd.DecoderOptions()
        opts.colorspace = 0  # MODE_RGB, 3 bytes per pixel
        outs, st = ctx.decode_batch_opts(frames[:1], opts)
        assert st[0] == 0 and outs[0].shape == (1080, 1920 * 3)
    finally:
        ctx.close()
