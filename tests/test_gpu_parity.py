"""GPU parity tests: HIP kernels (through the C ABI) vs the CPU oracle vs libwebp 1.6.0 goldens.

Bit-exact is the bar everywhere (all arithmetic on this path is integer).
"""
import hashlib
import os

import numpy as np
import pytest

import webp_amd
from oracle_lib import (bench_files, load_lossy, lossy_cases, manifest, oracle_decode, oracle_yuv_to_rgba)

pytestmark = pytest.mark.gpu

ALPHA = {"alpha_64x48"}
OPAQUE = [n for n in lossy_cases() if n not in ALPHA]


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("emit", ["fused", "separate"])
@pytest.mark.parametrize("flags", [0, webp_amd.FLAG_BYPASS_FILTERING, webp_amd.FLAG_NO_FANCY_UPSAMPLING])
def test_batch_all_fixtures_vs_golden_and_oracle(ctx, flags, emit):
    """All opaque lossy fixtures (odd sizes 1x1..481x270, every filter type/sharpness,
    1/4 segments, 1/4/8 partitions) in ONE batch: per-frame YUV and RGBA identical to
    libwebp's and to the CPU oracle's -- with the RGBA emitted by K1's tail (default) and
    by a separate K2 launch."""
    datas, golds = [], []
    for n in OPAQUE:
        d, g = load_lossy(n)
        datas.append(d)
        golds.append(g)
    b = ctx.batch(datas, flags)
    assert (b.status == 0).all(), b.status
    b.set_emit(emit == "separate")
    b.run()
    ms = b.kernel_ms()
    assert (ms[1] > 0) == (emit == "separate"), ms
    for i, (name, d, g) in enumerate(zip(OPAQUE, datas, golds)):
        y, u, v = b.yuv(i)
        rgba = b.rgba(i)
        bypass = flags & webp_amd.FLAG_BYPASS_FILTERING
        sfx = "_nofilter" if bypass else ""
        np.testing.assert_array_equal(y, g["y" + sfx], err_msg=name)
        np.testing.assert_array_equal(u, g["u" + sfx], err_msg=name)
        np.testing.assert_array_equal(v, g["v" + sfx], err_msg=name)
        if flags & webp_amd.FLAG_NO_FANCY_UPSAMPLING:
            np.testing.assert_array_equal(rgba, g["rgba_point"], err_msg=name)
        else:
            np.testing.assert_array_equal(rgba, g["rgba" + sfx], err_msg=name)
        info, mbs = webp_amd.vp8_parse(d, flags)
        o = oracle_decode(info, mbs, fancy=not (flags & webp_amd.FLAG_NO_FANCY_UPSAMPLING))
        np.testing.assert_array_equal(rgba, o["rgba"], err_msg=name)
    b.close()


@pytest.mark.parametrize("emit", ["fused", "separate", "stage"])
@pytest.mark.parametrize("prefix", ["c1_512", "c2_1080p", "c3_4k", "c3s_4k"])
def test_bench_frames_sha256(ctx, prefix, emit):
    """Full-size bench configs (C1 512^2, C2 1080p, C3 4K deblocked, and c3s: C3's entropy-stress
    variant at sigma 18, ~2 bpp, dense coefficients and mostly i4 MBs): every frame's
    Y/U/V and RGBA SHA-256 equals libwebp's, whichever kernel emits the RGBA (K1's tail,
    K2 in the batch run, or the stage entry wg_batch_run_emit after a planes-only run)."""
    m = manifest()["bench"]
    paths = bench_files(prefix)
    datas = [open(p, "rb").read() for p in paths]
    b = ctx.batch(datas)
    assert (b.status == 0).all()
    if emit == "stage":
        b.set_emit(True)
        b.run()  # planes + RGBA
        b.set_emit(False)
        b.run()  # the tail rewrites the RGBA
        b.run_emit()  # and the stage alone once more
    else:
        b.set_emit(emit == "separate")
        b.run()
    for i, p in enumerate(paths):
        ent = m[p.rsplit("/", 1)[1]]["sha256"]
        y, u, v = b.yuv(i)
        assert _sha(y) == ent["y"], p
        assert _sha(u) == ent["u"], p
        assert _sha(v) == ent["v"], p
        assert _sha(b.rgba(i)) == ent["rgba"], p
    b.close()


@pytest.mark.parametrize("flags", [webp_amd.FLAG_BYPASS_FILTERING, webp_amd.FLAG_NO_FANCY_UPSAMPLING])
def test_c3s_dense_frames_other_paths(ctx, flags):
    """The c3s frames (dense coefficients, i4-heavy) with the loop filter bypassed and with
    point-sampled RGBA: planes and RGBA SHA-256 equal libwebp's for all eight seeds."""
    m = manifest()["bench"]
    paths = bench_files("c3s_4k")
    assert len(paths) == 8
    b = ctx.batch([open(p, "rb").read() for p in paths], flags)
    assert (b.status == 0).all()
    b.run()
    bypass = flags & webp_amd.FLAG_BYPASS_FILTERING
    sfx = "_nofilter" if bypass else ""
    for i, p in enumerate(paths):
        ent = m[p.rsplit("/", 1)[1]]["sha256"]
        y, u, v = b.yuv(i)
        assert (_sha(y), _sha(u), _sha(v)) == (ent["y" + sfx], ent["u" + sfx], ent["v" + sfx]), p
        assert _sha(b.rgba(i)) == ent["rgba_nofilter" if bypass else "rgba_point"], p
    b.close()


def test_repeated_runs_identical(ctx):
    """Idempotence of the device path: re-running a resident batch gives the same bytes
    (no state leaks across launches through LDS/progress counters)."""
    datas = [open(p, "rb").read() for p in bench_files("c2_1080p")[:3]]
    datas += [load_lossy(n)[0] for n in OPAQUE[:5]]
    b = ctx.batch(datas)
    b.run()
    first = [_sha(b.rgba(i)) for i in range(b.n)]
    for _ in range(3):
        b.run()
    assert [_sha(b.rgba(i)) for i in range(b.n)] == first
    b.close()


def test_decode_single_dropin():
    """webp_amd.decode == webp.Decode drop-in: one frame through wg_decode_rgba_into."""
    for n in ["synth_17x9", "noise_97x63_q20", "smooth_161x113_simple"]:
        d, g = load_lossy(n)
        np.testing.assert_array_equal(webp_amd.decode(d), g["rgba"])
        np.testing.assert_array_equal(webp_amd.decode(d, webp_amd.FLAG_NO_FANCY_UPSAMPLING), g["rgba_point"])


def test_bad_frames_do_not_poison_batch(ctx):
    good, g = load_lossy("synth_80x96")
    trunc = good[: len(good) // 2]
    garbage = b"RIFF\x10\x00\x00\x00WEBPVP8 " + bytes(20)
    empty = b""
    datas = [good, trunc, garbage, empty, good]
    outs, status = ctx.decode_batch(datas)
    assert status[0] == 0 and status[4] == 0
    assert (status[1:4] != 0).all(), status
    np.testing.assert_array_equal(outs[0], g["rgba"])
    np.testing.assert_array_equal(outs[4], g["rgba"])


def test_decode_batch_hundred_frames_with_bad_ones(ctx):
    """wg_decode_rgba_batch over 100 frames (every opaque lossy fixture and the alpha frame, cycled,
    with truncated frames in between): every good frame equals libwebp's RGBA and the statuses
    land on the right frames."""
    names = OPAQUE + ["alpha_64x48"]
    good = [load_lossy(n) for n in names]
    datas, want = [], []
    for k in range(100):
        if k % 23 == 7:
            datas.append(good[0][0][: len(good[0][0]) // 3])  # truncated: fails in its chunk only
            want.append(None)
        else:
            d, g = good[k % len(good)]
            datas.append(d)
            want.append(g["rgba"])
    outs, status = ctx.decode_batch(datas)
    for k, (o, w, s) in enumerate(zip(outs, want, status)):
        if w is None:
            assert s != 0, k
        else:
            assert s == 0, (k, s)
            np.testing.assert_array_equal(o, w, err_msg=str(k))


def test_lossy_alpha_frame_in_the_lossy_set(ctx):
    """VP8+ALPH: the lossy set's alpha frame decodes to libwebp's RGBA."""
    al, g = load_lossy("alpha_64x48")
    outs, status = ctx.decode_batch([al])
    assert (status == 0).all()
    np.testing.assert_array_equal(outs[0], g["rgba"])


def test_yuv_to_rgba_device_stage_vs_oracle():
    """Stage entry point on torch device tensors, random planes incl. odd sizes."""
    import torch
    rng = np.random.default_rng(5)
    for (h, w) in [(1, 1), (3, 5), (17, 33), (64, 64), (129, 1041), (270, 481), (1080, 1920)]:
        uw, uh = (w + 1) // 2, (h + 1) // 2
        ys, uvs = (w + 15) // 16 * 16 + 16, (uw + 7) // 8 * 8 + 4
        Y = rng.integers(0, 256, (h, ys), dtype=np.uint8)
        U = rng.integers(0, 256, (uh, uvs), dtype=np.uint8)
        V = rng.integers(0, 256, (uh, uvs), dtype=np.uint8)
        dY, dU, dV = (torch.from_numpy(a).cuda() for a in (Y, U, V))
        for fancy in (True, False):
            out = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
            webp_amd.yuv420_to_rgba_device(dY.data_ptr(), dU.data_ptr(), dV.data_ptr(), ys, uvs, out.data_ptr(),
                                           4 * w, w, h, fancy, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ref = oracle_yuv_to_rgba(Y[:, :w], U[:, :uw], V[:, :uw], fancy=fancy)
            np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"{h}x{w} fancy={fancy}")


def test_yuv_to_rgba_device_every_yuv_triple():
    """The device's packed 16-bit VP8YuvToRgba over ALL 2^24 (y, u, v): a 4096 x 4096 frame
    whose 2x2 blocks hold every (u, v) pair 64 times and, across those 64 blocks, every y.
    Point sampling gives each pixel exactly its block's (u, v), so the RGBA must equal
    conversion.go:28-49 (MultHi, Clip8) evaluated in numpy; the same planes fancy-upsampled
    must equal the oracle."""
    import torch
    n = 4096
    b = np.arange((n // 2) * (n // 2), dtype=np.int64).reshape(n // 2, n // 2)  # block index
    U = ((b >> 14) & 255).astype(np.uint8)
    V = ((b >> 6) & 255).astype(np.uint8)
    Y = np.empty((n, n), np.uint8)
    for dy in range(2):
        for dx in range(2):
            Y[dy::2, dx::2] = (((b & 63) << 2) + 2 * dy + dx).astype(np.uint8)
    dY, dU, dV = (torch.from_numpy(a).cuda() for a in (Y, U, V))
    out = torch.zeros((n, n, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    webp_amd.yuv420_to_rgba_device(dY.data_ptr(), dU.data_ptr(), dV.data_ptr(), n, n // 2, out.data_ptr(), 4 * n, n,
                                   n, False, stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    y = Y.astype(np.int64)
    u = np.repeat(np.repeat(U, 2, 0), 2, 1).astype(np.int64)
    v = np.repeat(np.repeat(V, 2, 0), 2, 1).astype(np.int64)
    seen = np.zeros(1 << 24, bool)
    seen[(y << 16 | u << 8 | v).ravel()] = True
    assert seen.all()  # every (y, u, v) occurs

    def clip8(x):
        return np.clip(x >> 6, 0, 255)
    y1 = (y * 19077) >> 8
    np.testing.assert_array_equal(got[..., 0], clip8(y1 + ((v * 26149) >> 8) - 14234))
    np.testing.assert_array_equal(got[..., 1], clip8(y1 - ((u * 6419) >> 8) - ((v * 13320) >> 8) + 8708))
    np.testing.assert_array_equal(got[..., 2], clip8(y1 + ((u * 33050) >> 8) - 17685))
    assert (got[..., 3] == 255).all()
    webp_amd.yuv420_to_rgba_device(dY.data_ptr(), dU.data_ptr(), dV.data_ptr(), n, n // 2, out.data_ptr(), 4 * n, n,
                                   n, True, stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle_yuv_to_rgba(Y, U, V, fancy=True))


def test_wide_frames_global_column_store(ctx):
    """Frames wider than K1's LDS column store (mb_w > 600, up to VP8's 16383 px) take the
    global-store K1 variant: alone, interleaved with narrow frames (both variants launched on
    one batch), and cropped (K2 over the compact window).  libwebp + oracle parity."""
    assert webp_amd.vp8_parse(load_lossy("wide_9617x40")[0])[0].mb_w > 600
    wide = ["wide_9617x40", "wide_16383x17_simple"]
    for names in (wide, ["wide_9617x40", "synth_80x96", "wide_16383x17_simple", "synth_17x9"]):
        imgs, status = ctx.decode_batch([load_lossy(n)[0] for n in names])
        assert (status == 0).all(), status
        for n, img in zip(names, imgs):
            np.testing.assert_array_equal(img, load_lossy(n)[1]["rgba"], err_msg=n)
    d, g = load_lossy("wide_16383x17_simple")
    for flags, key in ((webp_amd.FLAG_BYPASS_FILTERING, "rgba_nofilter"), (webp_amd.FLAG_NO_FANCY_UPSAMPLING,
                                                                            "rgba_point")):
        imgs, status = ctx.decode_batch([d], flags)
        assert status[0] == 0
        np.testing.assert_array_equal(imgs[0], g[key], err_msg=key)
    from oracle_lib import oracle_output

    crop = (9000, 3, 7001, 13)
    outs, status = ctx.decode_batch_opts([d, load_lossy("wide_9617x40")[0]], webp_amd.options(1, crop))
    assert status[0] == 0 and status[1] != 0  # the window exceeds the 9617-px frame
    np.testing.assert_array_equal(outs[0], oracle_output(d, 1, crop))


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_split_k1_bench_frames(ctx, parts):
    """K1's split kernel (wg_batch_set_k1_parts): a frame's MB-row quads spread over `parts`
    workgroups, part-boundary hand-offs through global progress flags and sc1 column-store
    traffic.  4K (34 quads: slabs of 12; with 2 parts more quads than 2 x 12 -- part 0 alone),
    the dense c3s frames and 1080p (17 quads), every frame's RGBA SHA-256 = libwebp's, on
    repeated runs (a fresh flag epoch per launch)."""
    m = manifest()["bench"]
    for prefix in ("c3_4k", "c3s_4k", "c2_1080p"):
        paths = bench_files(prefix)[:5]
        b = ctx.batch([open(p, "rb").read() for p in paths])
        try:
            b.set_k1_parts(parts)
            for r in range(3):
                b.run()
                for i, p in enumerate(paths):
                    assert _sha(b.rgba(i)) == m[os.path.basename(p)]["sha256"]["rgba"], (prefix, parts, r, i)
            ms = b.kernel_ms()
            assert ms[0] > 0 and ms[1] > 0, ms  # split K1, then K2
        finally:
            b.close()


@pytest.mark.parametrize("parts", [2, 3])
def test_split_k1_fixtures(ctx, parts):
    """Every opaque lossy fixture through the split kernel: tall narrow frames (16 quads: two
    slabs), one-column frames, partial last quads, wide frames (global column store anyway),
    both filter types -- planes and RGBA equal to libwebp's and the oracle's."""
    datas, golds = zip(*[load_lossy(n) for n in OPAQUE])
    b = ctx.batch(list(datas))
    try:
        b.set_k1_parts(parts)
        b.run()
        b.run()
        for i, (name, g) in enumerate(zip(OPAQUE, golds)):
            y, u, v = b.yuv(i)
            np.testing.assert_array_equal(y, g["y"], err_msg=name)
            np.testing.assert_array_equal(u, g["u"], err_msg=name)
            np.testing.assert_array_equal(v, g["v"], err_msg=name)
            np.testing.assert_array_equal(b.rgba(i), g["rgba"], err_msg=name)
    finally:
        b.close()


def test_split_k1_epoch_wrap(ctx):
    """The split kernel's progress-flag tags are 16 bits from a process-wide counter, so they
    repeat every 65,535 split launches.  Run 1 (3 parts: 4K slabs of 12 + 12 + 10 quads) leaves
    its boundary flags at "tag T, all columns done"; run 2 (2 parts: 34 quads > 2 x 12, the frame
    on part 0 alone) publishes no flag and leaves the frame's BOTTOM row in the column store; run
    3 (3 parts again) gets tag T once more -- as a run one tag cycle later would
    (wg_debug_set_epoch moves the counter back).  Had run 1's flags survived, parts 1 and 2 would
    start at once and read run 2's bottom-row columns: the flags are cleared before every split
    launch, so every frame's RGBA is still libwebp's (c3 and the dense c3s 4K frames)."""
    L = webp_amd.lib()
    m = manifest()["bench"]
    paths = bench_files("c3_4k")[:3] + bench_files("c3s_4k")[:2]
    b = ctx.batch([open(p, "rb").read() for p in paths])

    def check(tag):
        for i, p in enumerate(paths):
            assert _sha(b.rgba(i)) == m[os.path.basename(p)]["sha256"]["rgba"], (tag, i)
    try:
        for rep in range(2):
            b.set_k1_parts(3)
            b.run()
            check(("run1", rep))
            last = L.wg_debug_set_epoch(0)  # the counter after run 1: its low 16 bits are run 1's tag
            L.wg_debug_set_epoch(last)
            b.set_k1_parts(2)
            b.run()
            check(("run2", rep))
            L.wg_debug_set_epoch((last - 1) & 0xffffffff)  # run 3 takes tag T again
            b.set_k1_parts(3)
            b.run()
            check(("run3", rep))
    finally:
        b.close()


def test_one_part_after_split_restores_tail(ctx):
    """wg_batch_set_k1_parts(b, 1) after a split of the whole batch runs the one-workgroup kernel
    with its RGBA tail again (no K2 launch: kernel_ms[1] == 0); a batch set to K2 by set_emit(True)
    keeps K2.  RGBA = libwebp's either way."""
    m = manifest()["bench"]
    paths = bench_files("c2_1080p")[:3]
    b = ctx.batch([open(p, "rb").read() for p in paths])
    try:
        def check(k2):
            b.run()
            ms = b.kernel_ms()
            assert (ms[1] > 0) == k2, ms
            for i, p in enumerate(paths):
                assert _sha(b.rgba(i)) == m[os.path.basename(p)]["sha256"]["rgba"], (k2, i)
        b.set_k1_parts(3)
        check(True)
        b.set_k1_parts(1)
        check(False)
        b.set_emit(True)
        b.set_k1_parts(1)
        check(True)
    finally:
        b.close()


def test_single_frame_decode_uses_split_and_matches():
    """The single-frame drop-in (webp.Decode's path) on a 4K frame -- one frame, so the automatic
    choice runs the split kernel: libwebp's RGBA."""
    m = manifest()["bench"]
    for p in bench_files("c3_4k")[:2] + bench_files("c3s_4k")[:1]:
        assert _sha(webp_amd.decode(open(p, "rb").read())) == m[os.path.basename(p)]["sha256"]["rgba"]


def test_short_last_round_on_split_kernel(ctx):
    """More frames than CUs: whole rounds of 256 on the one-workgroup kernel (RGBA in its tail),
    the short remainder behind them on the split kernel and a K2 over the remainder alone.  258
    1080p frames (17 quads: two slabs): every frame's RGBA = libwebp's, the head's and the
    remainder's; then the same batch switched to separate K2 (remainder still split)."""
    paths = bench_files("c2_1080p")
    m = manifest()["bench"]
    datas = [open(p, "rb").read() for p in paths]
    n = 258
    b = ctx.batch([datas[i % len(datas)] for i in range(n)])
    try:
        for sep in (False, True):
            if sep:
                b.set_emit(True)
            b.run()
            ms = b.kernel_ms()
            assert ms[0] > 0 and ms[1] > 0, ms  # K1 (both kernels), K2 (the remainder / every frame)
            for i in (0, 1, 100, 255, 256, 257):
                want = m[os.path.basename(paths[i % len(paths)])]["sha256"]["rgba"]
                assert _sha(b.rgba(i)) == want, (sep, i)
    finally:
        b.close()
