"""CPU tests: host entropy stage + CPU oracle pinned against libwebp 1.6.0 goldens,
and the known-answer properties that justify the device decomposition."""
import ctypes as C

import numpy as np
import pytest

import webp_amd
from oracle_lib import (lossy_cases, load_lossy, oracle, oracle_decode, oracle_yuv_to_rgba, manifest,
                        bench_files)

ALPHA_CASES = {"alpha_64x48"}


@pytest.mark.parametrize("name", lossy_cases())
def test_oracle_matches_libwebp_golden(name):
    data, gold = load_lossy(name)
    info, mbs = webp_amd.vp8_parse(data)
    assert (info.width, info.height) == gold["y"].shape[::-1]
    out = oracle_decode(info, mbs, fancy=True)
    np.testing.assert_array_equal(out["y"], gold["y"])
    np.testing.assert_array_equal(out["u"], gold["u"])
    np.testing.assert_array_equal(out["v"], gold["v"])
    if name not in ALPHA_CASES:  # ALPH plane is a later §8(f) row; colour must still match
        np.testing.assert_array_equal(out["rgba"], gold["rgba"])
    else:
        np.testing.assert_array_equal(out["rgba"][..., :3], gold["rgba"][..., :3])
    pt = oracle_yuv_to_rgba(out["y"], out["u"], out["v"], fancy=False)
    if name not in ALPHA_CASES:
        np.testing.assert_array_equal(pt, gold["rgba_point"])


@pytest.mark.parametrize("name", lossy_cases())
def test_oracle_bypass_filter_matches_golden(name):
    data, gold = load_lossy(name)
    info, mbs = webp_amd.vp8_parse(data, flags=webp_amd.FLAG_BYPASS_FILTERING)
    assert info.filter_type == 0
    out = oracle_decode(info, mbs)
    np.testing.assert_array_equal(out["y"], gold["y_nofilter"])
    np.testing.assert_array_equal(out["u"], gold["u_nofilter"])
    np.testing.assert_array_equal(out["v"], gold["v_nofilter"])
    if name not in ALPHA_CASES:
        np.testing.assert_array_equal(out["rgba"], gold["rgba_nofilter"])


def test_fixture_coverage():
    """The fixture set exercises every filter type, sharpness, segments and partitions."""
    m = manifest()["lossy"]
    hdrs = [v["header"] for v in m.values()]
    assert {h["simple"] for h in hdrs if h["level"]} == {0, 1}
    assert any(h["level"] == 0 for h in hdrs)
    assert {0, 3, 7} <= {h["sharpness"] for h in hdrs}
    assert {0, 1} <= {h["segments"] for h in hdrs}
    assert {1, 4, 8} <= {h["partitions"] for h in hdrs}


def test_parse_modes_and_codes_cover_all_paths():
    seen_i4 = set()
    seen_i16 = set()
    seen_uv = set()
    codes = set()
    for name in lossy_cases():
        data, _ = load_lossy(name)
        info, mbs = webp_amd.vp8_parse(data)
        i4 = mbs["is_i4x4"] == 1
        seen_i4 |= set(np.unique(mbs["imodes"][i4]).tolist())
        seen_i16 |= set(np.unique(mbs["imodes"][~i4, 0]).tolist())
        seen_uv |= set(np.unique(mbs["uvmode"]).tolist())
        for s in range(16):
            codes |= set(np.unique((mbs["non_zero_y"] >> (30 - 2 * s)) & 3).tolist())
    assert seen_i4 == set(range(10)), seen_i4
    assert seen_i16 == {0, 1, 2, 3}
    assert seen_uv == {0, 1, 2, 3}
    assert codes == {0, 1, 2, 3}


def _transform(coeffs, code, pred):
    dst = np.zeros((4, 32), np.uint8)
    dst[:, :4] = pred
    c = np.ascontiguousarray(coeffs, np.int16)
    oracle().oracle_transform_block(c.ctypes.data, dst.ctypes.data, code)
    return dst[:, :4].copy()


def test_avg3_lerp_identity():
    """K1's i4 AVG3 (dec.c.go AVG3, (a + 2b + c + 2) >> 2) as two v_lerp_u8 byte averages:
    floor average of a and c, then the rounding-up average with b -- exact for all bytes."""
    a, b, c = np.meshgrid(np.arange(256), np.arange(256), np.arange(256), indexing="ij")
    np.testing.assert_array_equal((((a + c) >> 1) + b + 1) >> 1, (a + 2 * b + c + 2) >> 2)
    # AVG2 (a + b + 1) >> 1 is stored as AVG3(a, b, a) in pred4_table.inc
    np.testing.assert_array_equal((a[:, :, 0] + 2 * b[:, :, 0] + a[:, :, 0] + 2) >> 2,
                                  (a[:, :, 0] + b[:, :, 0] + 1) >> 1)


def test_transform_shortcuts_exact():
    """TransformAC3 / TransformDC == TransformOne on their coefficient patterns
    (dec.c.go:49-126): the device may always run TransformOne."""
    rng = np.random.default_rng(0)
    for it in range(20000):
        pred = rng.integers(0, 256, (4, 4), dtype=np.uint8)
        c = np.zeros(16, np.int16)
        c[0] = rng.integers(-2048, 2048)
        if it % 2:
            c[1] = rng.integers(-2048, 2048)
            c[4] = rng.integers(-2048, 2048)
            code = 2
        else:
            code = 1
        np.testing.assert_array_equal(_transform(c, code, pred), _transform(c, -1, pred))


def test_residual_independent_of_prediction():
    """dst = clip8(pred + (v >> 3)): the residual does not depend on pred (STORE macro)."""
    rng = np.random.default_rng(1)
    zero = np.zeros((4, 4), np.uint8)
    mid = np.full((4, 4), 128, np.uint8)
    for _ in range(2000):
        c = rng.integers(-600, 600, 16).astype(np.int16)
        pred = rng.integers(0, 256, (4, 4), dtype=np.uint8)
        r = _transform(c, -1, mid).astype(int) - 128  # exact while |res| < 128
        if np.abs(r).max() >= 127:
            continue
        np.testing.assert_array_equal(_transform(c, -1, pred), np.clip(pred.astype(int) + r, 0, 255))


def test_upsampler_closed_form():
    """The packed-u/v line-pair upsampler == (9a+3b+3c+d+8)>>4 with edge clamping."""
    rng = np.random.default_rng(2)
    for (h, w) in [(1, 1), (2, 3), (5, 7), (8, 8), (9, 17), (16, 2)]:
        y = rng.integers(0, 256, (h, w), dtype=np.uint8)
        uw, uh = (w + 1) // 2, (h + 1) // 2
        u = rng.integers(0, 256, (uh, uw), dtype=np.uint8)
        v = rng.integers(0, 256, (uh, uw), dtype=np.uint8)
        got = oracle_yuv_to_rgba(y, u, v, fancy=True)

        def up(p):
            out = np.zeros((h, w), int)
            for yy in range(h):
                nr = yy >> 1
                fr = min(max(nr + (1 if yy & 1 else -1), 0), uh - 1)
                for xx in range(w):
                    nc = xx >> 1
                    fc = min(max(nc + (1 if xx & 1 else -1), 0), uw - 1)
                    out[yy, xx] = (9 * int(p[nr, nc]) + 3 * int(p[nr, fc]) + 3 * int(p[fr, nc]) + int(p[fr, fc]) + 8) >> 4
            return out
        U, V = up(u), up(v)
        Y = y.astype(int)

        def clip8(x):
            return np.clip(x >> 6, 0, 255)
        y1 = (Y * 19077) >> 8
        R = clip8(y1 + ((V * 26149) >> 8) - 14234)
        G = clip8(y1 - ((U * 6419) >> 8) - ((V * 13320) >> 8) + 8708)
        B = clip8(y1 + ((U * 33050) >> 8) - 17685)
        np.testing.assert_array_equal(got[..., 0], R)
        np.testing.assert_array_equal(got[..., 1], G)
        np.testing.assert_array_equal(got[..., 2], B)
        assert (got[..., 3] == 255).all()


def test_packed_yuv_formulas():
    """K2's packed 16-bit VP8YuvToRgba (yuv_rgba_strip.h::yuv_to_rgba2) == conversion.go:28-49
    for every (y, u, v): MultHi split at the multiplier's high byte, saturating subtract
    before the >> 6, every intermediate within 16 bits unsigned (or wrapping by design).  And the packed vertical
    blend + horizontal taps (upsample4) stay within 16 bits."""
    y, u, v = (a.ravel().astype(np.int64) for a in np.meshgrid(*(np.arange(256),) * 3, indexing="ij"))

    def mh(a, c):
        return (a * c) >> 8

    def c8(x):
        return np.clip(x >> 6, 0, 255)
    R = c8(mh(y, 19077) + mh(v, 26149) - 14234)
    G = c8(mh(y, 19077) - mh(u, 6419) - mh(v, 13320) + 8708)
    B = c8(mh(y, 19077) + mh(u, 33050) - 17685)

    def u16(x):
        assert x.min() >= 0 and x.max() < 65536
        return x

    def sat(a, b):
        return np.maximum(a - b, 0)
    # y1g = MultHi(y, 19077) + 8708 (G's constant, folded into R's and B's subtrahends), from the
    # luma lane y + 32000 (high byte 0x7d from v_perm's constant source) by two wrapping
    # v_pk_mad_u16: (133 yl + 4864) mod 2^16 = 133 y + 1024, and 74 yl mod 2^16 = 74 y + 8704
    yl = y + 32000
    t4 = ((133 * yl + 4864) % 65536) >> 8
    assert ((133 * yl + 4864) % 65536 == 133 * y + 1024).all()
    y1g = u16((74 * yl + t4) % 65536)
    np.testing.assert_array_equal(y1g, mh(y, 19077) + 8708)
    r = np.minimum(sat(u16(y1g + u16(102 * v + (u16(37 * v) >> 8))), 14234 + 8708) >> 6, 255)
    gu = u16(25 * u + (u16(19 * u) >> 8))
    gv = u16(52 * v + (v >> 5))
    g = np.minimum(sat(sat(y1g, gu), gv) >> 6, 255)
    b = np.minimum(sat(u16(y1g + u16(129 * u + (u16(26 * u) >> 8))), 17685 + 8708) >> 6, 255)
    np.testing.assert_array_equal(r, R)
    np.testing.assert_array_equal(g, G)
    np.testing.assert_array_equal(b, B)
    # upsample4: a = 3 * near + (far + 2) per chroma column, then (3 a[near col] + a[far col]) >> 4
    # = (9a + 3b + 3c + d + 8) >> 4 (the rounding 8 = 3 * 2 + 2); every value within 16 bits
    n, f, n2, f2 = (np.random.default_rng(9).integers(0, 256, 1 << 16) for _ in range(4))
    a_near, a_far = 3 * n + (f + 2), 3 * n2 + (f2 + 2)
    np.testing.assert_array_equal((3 * a_near + a_far) >> 4, (9 * n + 3 * f + 3 * n2 + f2 + 8) >> 4)
    a = 3 * 255 + 255 + 2
    assert 3 * a + a < 65536
    # the final `>> 6` + Clip8 as the high byte of a saturating x4 (v_pk_mad_u16 ... clamp)
    x = np.arange(65536)
    np.testing.assert_array_equal(np.minimum(4 * x, 65535) >> 8, np.minimum(x >> 6, 255))


def test_bench_c1_frame_sha256():
    """Plumbing config C1 (512x512 lossy, webp.Decode on the CPU path): parse + oracle
    reproduce libwebp's RGBA bit for bit (SHA-256 from the manifest)."""
    import hashlib
    m = manifest()["bench"]
    (path,) = bench_files("c1_512")
    data = open(path, "rb").read()
    info, mbs = webp_amd.vp8_parse(data)
    out = oracle_decode(info, mbs)
    ent = m["c1_512_s0.webp"]["sha256"]
    assert hashlib.sha256(out["rgba"].tobytes()).hexdigest() == ent["rgba"]
    assert hashlib.sha256(out["y"].tobytes()).hexdigest() == ent["y"]


@pytest.mark.parametrize("prefix", ["c2_1080p", "c3_4k", "c3s_4k"])
def test_bench_frames_sha256(prefix):
    """The bench bitstreams (C2 1080p, C3 4K deblocked, c3s: C3 at sigma 18, ~2 bpp) decode
    bit-exactly on the CPU checker; the GPU parity tests compare against the same SHA-256s."""
    import hashlib
    m = manifest()["bench"]
    for path in bench_files(prefix)[:2]:
        data = open(path, "rb").read()
        info, mbs = webp_amd.vp8_parse(data)
        out = oracle_decode(info, mbs)
        ent = m[path.rsplit("/", 1)[1]]["sha256"]
        assert hashlib.sha256(out["rgba"].tobytes()).hexdigest() == ent["rgba"]
        assert hashlib.sha256(out["y"].tobytes()).hexdigest() == ent["y"]
        assert hashlib.sha256(out["u"].tobytes()).hexdigest() == ent["u"]


def _pred4_table():
    import os, re
    from oracle_lib import ROOT
    src = open(os.path.join(ROOT, "go-webp_amd", "csrc", "device", "pred4_table.inc")).read()
    body = src[src.index("{"):]
    return [int(v, 16) for v in re.findall(r"0x([0-9a-f]+)u", body)]


def test_pred4_table_matches_oracle_predictors():
    """The device's per-pixel recipe table (kind + 3 edge offsets) reproduces every
    libwebp 4x4 predictor (dec.c.go:261-410) exactly, on random edges."""
    tab = _pred4_table()
    assert len(tab) == 160
    L = oracle()
    L.oracle_pred_luma4.argtypes = [C.c_int, C.c_void_p]
    L.oracle_pred_luma4.restype = None
    rng = np.random.default_rng(3)
    BPS = 32
    for it in range(400):
        ws = rng.integers(0, 256, (8, BPS), dtype=np.uint8)
        if it % 4 == 0:
            ws[:] = rng.integers(0, 2) * 255  # saturating edges
        org = 2 * BPS + 8  # block origin (row 2, col 8)
        flat = ws.reshape(-1)
        for mode in range(10):
            ref = flat.copy()
            L.oracle_pred_luma4(mode, ref.ctypes.data + org)
            for y in range(4):
                for x in range(4):
                    w = tab[mode * 16 + y * 4 + x]
                    kind = w >> 24
                    assert kind in (0x00, 0x80, 0xC0), hex(w)
                    offs = [((w >> (8 * k)) & 0xff) for k in range(3)]
                    offs = [o - 256 if o >= 128 else o for o in offs]
                    a, b, c = (int(flat[org + o]) for o in offs)
                    if kind == 0x00:
                        v = (a + 2 * b + c + 2) >> 2
                    elif kind == 0x80:
                        v = min(max(a + b - c, 0), 255)
                    else:
                        assert w == 0xC0000000  # the kernel tests DC by the whole word
                        top = sum(int(flat[org - BPS + k]) for k in range(4))
                        left = sum(int(flat[org + k * BPS - 1]) for k in range(4))
                        v = (top + left + 4) >> 3
                    assert v == ref[org + y * BPS + x], (mode, x, y)
