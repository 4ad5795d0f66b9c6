#!/usr/bin/env python3
"""Generate the committed golden fixtures for the WebP decode path.

Test infrastructure only -- runs in the build container, never on the GPU box.

The reference (DaanV2/go-webp) is an unbuildable Go translation of libwebp 1.6.0
(``pkg/vp8/constants.go:18-20`` pins DEC_MAJ/MIN/REV_VERSION = 1/6/0; SURVEY.md
§0, §8(c)).  The upstream it translates is available offline here as Pillow's
bundled ``libwebp`` (``WebPGetDecoderVersion() == 0x010600``).  We load it with
ctypes, force its *plain-C* DSP kernels (``VP8GetCPUInfo = NULL``: exactly the
functions ``pkg/libwebp/dsp/dec.c.go``, ``upsampling.c.go`` and ``lossless.go``
translate) and write, per bitstream:

* lossy:  post-filter Y/U/V planes (``WebPDecodeYUV``), recon-only planes
  (``bypass_filtering=1``), fancy-upsampled RGBA (``WebPDecodeRGBA``, the
  default ``EmitFancyRGB`` path, ``io_dec.c.go:65-115``) and point-sampled
  RGBA (``no_fancy_upsampling=1``, ``EmitSampledRGB`` ``io_dec.c.go:53-59``);
* lossless: RGBA.

Small cases are stored as ``.webp`` + compressed ``.npz``; the large bench
frames (SURVEY.md §8(d), Appendix B generators) are stored as ``.webp`` plus
SHA-256 of their decodes in ``manifest.json``.  Every decode is also checked
against libwebp's SIMD path (must be byte-identical) before it is written.

Usage:  python tests/golden/make_golden.py [lossy|lossless|alpha|modes|yuv|anim|bench ...]
        (rewrites tests/golden/<section>/; default all sections)
"""
import ctypes as C
import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PIL_LIBS = "/usr/local/lib/python3.10/dist-packages/pillow.libs/"
ABI = 0x0210  # WEBP_{ENCODER,DECODER}_ABI_VERSION of 1.6.0 (pkg/constants/versions.go:4-5)

MODE_RGBA = 1
MODE_YUV = 11


def load_libwebp():
    C.CDLL(glob.glob(PIL_LIBS + "libsharpyuv-*.so*")[0], mode=C.RTLD_GLOBAL)
    lib = C.CDLL(glob.glob(PIL_LIBS + "libwebp-*.so*")[0])
    assert lib.WebPGetDecoderVersion() == 0x010600, hex(lib.WebPGetDecoderVersion())
    lib.WebPDecodeRGBA.restype = C.c_void_p
    lib.WebPDecodeYUV.restype = C.c_void_p
    lib.WebPFree.argtypes = [C.c_void_p]
    lib.WebPMemoryWriterClear.argtypes = [C.c_void_p]
    return lib


LIB = load_libwebp()
_CPU = C.c_void_p.in_dll(LIB, "VP8GetCPUInfo")
_SIMD = _CPU.value


def _plain_c(on):
    _CPU.value = None if on else _SIMD


# ----------------------------------------------------------------------------- encode
def encode(img, quality=75.0, lossless=0, method=4, segments=4, sns=50, filter_strength=60,
           sharpness=0, filter_type=1, autofilter=0, partitions=0, low_memory=0, exact=0,
           alpha_compression=1, alpha_filtering=1, alpha_quality=100):
    """img: HxWx3 or HxWx4 uint8.  Returns the encoded RIFF bytes."""
    h, w, ch = img.shape
    cfg = (C.c_int32 * 64)()
    assert LIB.WebPConfigInitInternal(cfg, 0, C.c_float(quality), ABI)
    cfgf = C.cast(cfg, C.POINTER(C.c_float))
    cfg[0] = lossless
    cfgf[1] = quality
    cfg[2] = method
    cfg[6] = segments
    cfg[7] = sns
    cfg[8] = filter_strength
    cfg[9] = sharpness
    cfg[10] = filter_type
    cfg[11] = autofilter
    cfg[12] = alpha_compression  # 0 raw, 1 lossless
    cfg[13] = alpha_filtering    # 0 none, 1 fast, 2 best
    cfg[14] = alpha_quality      # < 100: level pre-processing
    cfg[18] = partitions
    cfg[22] = low_memory
    cfg[24] = exact
    assert LIB.WebPValidateConfig(cfg), "bad config"
    pic = (C.c_uint8 * 512)()
    assert LIB.WebPPictureInitInternal(pic, ABI)
    pi = C.cast(pic, C.POINTER(C.c_int32))
    pi[0] = 1 if lossless else 0  # use_argb
    pi[2] = w
    pi[3] = h
    wr = (C.c_uint8 * 64)()
    LIB.WebPMemoryWriterInit(wr)
    pp = C.cast(pic, C.POINTER(C.c_void_p))
    pp[96 // 8] = C.cast(LIB.WebPMemoryWrite, C.c_void_p).value
    pp[104 // 8] = C.addressof(wr)
    buf = np.ascontiguousarray(img)
    if ch == 3:
        ok = LIB.WebPPictureImportRGB(pic, buf.ctypes.data_as(C.c_void_p), w * 3)
    else:
        ok = LIB.WebPPictureImportRGBA(pic, buf.ctypes.data_as(C.c_void_p), w * 4)
    assert ok
    ok = LIB.WebPEncode(cfg, pic)
    err = pi[136 // 4]
    assert ok, f"encode failed err={err}"
    wp = C.cast(wr, C.POINTER(C.c_void_p))
    size = C.cast(wr, C.POINTER(C.c_size_t))[1]
    out = C.string_at(wp[0], size)
    LIB.WebPMemoryWriterClear(wr)
    LIB.WebPPictureFree(pic)
    return out


# ----------------------------------------------------------------------------- decode
def _decode_cfg(data, colorspace, bypass=0, no_fancy=0):
    cfg = (C.c_uint8 * 512)()
    assert LIB.WebPInitDecoderConfigInternal(cfg, ABI)
    ci = C.cast(cfg, C.POINTER(C.c_int32))
    ci[40 // 4] = colorspace
    ci[160 // 4] = bypass
    ci[164 // 4] = no_fancy
    st = LIB.WebPDecode(data, C.c_size_t(len(data)), cfg)
    assert st == 0, f"WebPDecode status {st}"
    w, h = ci[44 // 4], ci[48 // 4]
    cp = C.cast(cfg, C.POINTER(C.c_void_p))
    if colorspace == MODE_YUV:
        ys, us, vs = ci[88 // 4], ci[92 // 4], ci[96 // 4]
        uw, uh = (w + 1) // 2, (h + 1) // 2

        def plane(ptr, stride, pw, ph):
            raw = np.frombuffer(C.string_at(ptr, stride * (ph - 1) + pw), np.uint8)
            return np.stack([raw[r * stride:r * stride + pw] for r in range(ph)])

        out = (plane(cp[56 // 8], ys, w, h), plane(cp[64 // 8], us, uw, uh),
               plane(cp[72 // 8], vs, uw, uh))
    else:
        stride = ci[64 // 4]
        raw = np.frombuffer(C.string_at(cp[56 // 8], stride * h), np.uint8)
        out = raw.reshape(h, stride)[:, :w * 4].reshape(h, w, 4).copy()
    LIB.WebPFreeDecBuffer(C.byref(cfg, 40))
    return out


def decode_all(data, lossy=True):
    """Decode with plain-C kernels; assert SIMD path is identical."""
    res = {}
    for plain in (True, False):
        _plain_c(plain)
        r = {"rgba": _decode_cfg(data, MODE_RGBA)}
        if lossy:
            r["rgba_point"] = _decode_cfg(data, MODE_RGBA, no_fancy=1)
            y, u, v = _decode_cfg(data, MODE_YUV)
            r.update(y=y, u=u, v=v)
            y, u, v = _decode_cfg(data, MODE_YUV, bypass=1)
            r.update(y_nofilter=y, u_nofilter=u, v_nofilter=v)
            r["rgba_nofilter"] = _decode_cfg(data, MODE_RGBA, bypass=1)
        if plain:
            res = r
        else:
            for k in r:
                assert np.array_equal(r[k], res[k]), f"plain-C != SIMD for {k}"
    _plain_c(True)
    return res


# ----------------------------------------------------------------------------- header probe
class _Bool:  # RFC 6386 §7 bool decoder, used to label fixtures
    def __init__(s, b):
        s.b = b; s.p = 2; s.value = (b[0] << 8) | b[1]; s.range = 255; s.bit_count = 0

    def bit(s, prob):
        split = 1 + (((s.range - 1) * prob) >> 8); big = split << 8
        if s.value >= big:
            r = 1; s.range -= split; s.value -= big
        else:
            r = 0; s.range = split
        while s.range < 128:
            s.value <<= 1; s.range <<= 1; s.bit_count += 1
            if s.bit_count == 8:
                s.bit_count = 0
                if s.p < len(s.b):
                    s.value |= s.b[s.p]
                s.p += 1
        return r

    def lit(s, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | s.bit(128)
        return v

    def sval(s, n):
        v = s.lit(n)
        return -v if s.bit(128) else v


def vp8_header(data):
    i = data.find(b"VP8 ")
    f = data[i + 8:]
    p0 = (f[0] | (f[1] << 8) | (f[2] << 16)) >> 5
    br = _Bool(f[10:10 + p0]); br.bit(128); br.bit(128)
    segs = 0
    if br.bit(128):
        segs = 1
        upd_map = br.bit(128)
        if br.bit(128):
            br.bit(128)
            [br.sval(7) if br.bit(128) else 0 for _ in range(4)]
            [br.sval(6) if br.bit(128) else 0 for _ in range(4)]
        if upd_map:
            [br.lit(8) if br.bit(128) else 255 for _ in range(3)]
    simple = br.bit(128); level = br.lit(6); sharp = br.lit(3)
    if br.bit(128) and br.bit(128):
        for _ in range(8):
            if br.bit(128):
                br.sval(6)
    parts = 1 << br.lit(2)
    return dict(segments=segs, simple=simple, level=level, sharpness=sharp, partitions=parts)


# ----------------------------------------------------------------------------- synthetic images
def synth(H, W, seed, sigma):  # SURVEY.md Appendix B (lossy C1-C4)
    rng = np.random.default_rng(seed); yy, xx = np.mgrid[0:H, 0:W]
    base = np.stack([(xx * 255) // W, (yy * 255) // H, (((xx // 64) + (yy // 64)) % 2) * 160 + 40], -1)
    return np.clip(base + rng.normal(0, sigma, (H, W, 3)), 0, 255).astype(np.uint8)


def corr_luma(H, W, seed):  # SURVEY.md Appendix B (lossless C5)
    rng = np.random.default_rng(seed); yy, xx = np.mgrid[0:H, 0:W]
    lum = 128 + 100 * np.sin(xx / 37.0) * np.cos(yy / 53.0) + rng.normal(0, 4, (H, W))
    return np.clip(np.stack([lum + 10, lum, lum - 15 + 20 * np.sin(yy / 91.0)], -1), 0, 255).astype(np.uint8)


def smooth(H, W, seed):  # i16-heavy content
    rng = np.random.default_rng(seed); yy, xx = np.mgrid[0:H, 0:W]
    r = 128 + 90 * np.sin(xx / 23.0 + seed) * np.cos(yy / 31.0)
    g = 128 + 80 * np.cos((xx + yy) / 41.0)
    b = 64 + (xx * 127) // max(W - 1, 1)
    return np.clip(np.stack([r, g, b], -1) + rng.normal(0, 1.0, (H, W, 3)), 0, 255).astype(np.uint8)


def noise(H, W, seed, sigma=60):  # i4x4-heavy content, many coefficients
    rng = np.random.default_rng(seed)
    img = synth(H, W, seed, 0).astype(np.float64)
    return np.clip(img + rng.normal(0, sigma, (H, W, 3)), 0, 255).astype(np.uint8)


def palette_img(H, W, seed, ncol):
    rng = np.random.default_rng(seed)
    pal = rng.integers(0, 256, (ncol, 4), dtype=np.uint8)
    pal[:, 3] = 255
    yy, xx = np.mgrid[0:H, 0:W]
    idx = ((xx // 3) + (yy // 5) * 7 + rng.integers(0, 2, (H, W))) % ncol
    return pal[idx]


def with_alpha(img, seed):
    rng = np.random.default_rng(seed)
    H, W, _ = img.shape
    yy, xx = np.mgrid[0:H, 0:W]
    a = np.clip(128 + 127 * np.sin(xx / 13.0) * np.cos(yy / 7.0) + rng.normal(0, 3, (H, W)), 0, 255)
    a[: H // 4, : W // 4] = 0
    return np.concatenate([img, a.astype(np.uint8)[..., None]], -1)


def cutout_alpha(H, W, seed):
    """The alpha of a cut-out (a product shot, a sticker): an off-centre ellipse with a 24-px
    feathered edge, a half-transparent band below it, transparent elsewhere."""
    rng = np.random.default_rng(1000 + seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    cy, cx = H * (0.4 + 0.1 * rng.random()), W * (0.4 + 0.2 * rng.random())
    ry, rx = H * 0.38, W * 0.33
    d = np.sqrt(((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2)
    a = np.clip((1.0 - d) * min(ry, rx) / 24.0, 0.0, 1.0) * 255.0
    band = (yy > H * 0.82) & (yy < H * 0.9)
    a[band] = np.maximum(a[band], 128.0)
    return a.astype(np.uint8)


def anim_scene(H, W, n, seed):
    """n full-canvas RGBA frames: an opaque textured background, a semi-transparent sprite a
    quarter of the canvas wide sliding across it and a small opaque box changing colour:
    WebPAnimEncoder emits blended sub-rectangles, as sticker / screen-capture animations do."""
    rng = np.random.default_rng(seed)
    base = np.concatenate([synth(H, W, seed, 4), np.full((H, W, 1), 255, np.uint8)], -1)
    sh, sw = H // 3, W // 4
    spr = np.concatenate([synth(sh, sw, seed + 1, 10), np.full((sh, sw, 1), 170, np.uint8)], -1)
    out = []
    for i in range(n):
        img = base.copy()
        y0, x0 = (H - sh) // 2 + int(40 * np.sin(i / 5.0)), (i * (W - sw)) // max(1, n - 1)
        region = img[y0:y0 + sh, x0:x0 + sw].astype(np.int32)
        a = spr[..., 3:4].astype(np.int32)
        img[y0:y0 + sh, x0:x0 + sw, :3] = ((spr[..., :3] * a + region[..., :3] * (255 - a)) // 255).astype(np.uint8)
        img[32:96, 32:160, :3] = rng.integers(0, 256, 3, dtype=np.uint8)
        out.append(img)
    return out


def alpha_pattern(H, W, seed, kind):
    """RGB content plus an alpha plane shaped so one unfilter wins: 'h' rows of ramps with
    random row offsets, 'v' the transpose, 'g' a plane plus a mild texture, 'lv' four levels."""
    rng = np.random.default_rng(seed)
    img = synth(H, W, seed, 6)
    yy, xx = np.mgrid[0:H, 0:W]
    if kind == "h":
        a = xx * 3 + rng.integers(0, 256, (H, 1))
    elif kind == "v":
        a = yy * 3 + rng.integers(0, 256, (1, W))
    elif kind == "g":
        a = xx * 5 + yy * 7 + (rng.integers(0, 3, (H, W)))
    elif kind == "lv":
        a = ((xx // 7 + yy // 5) % 4) * 85
    elif kind == "bin":  # two levels: a 2-colour palette, eight pixels per coded pixel
        a = ((xx // 9 + yy // 6) % 3 == 0) * 255
    elif kind == "rl":  # 40 random levels: a palette of more than 16 colours
        a = rng.integers(0, 40, (H, W)) * 6
    elif kind == "many":  # 61 levels: a palette of more than 16 colours, one pixel per coded pixel
        a = ((xx * 2 + yy) % 61) * 4
    elif kind == "l12":  # 12 levels: a palette of 5..16 colours, two pixels per coded pixel
        a = ((xx // 5 + yy // 3) % 12) * 20
    else:
        a = rng.integers(0, 256, (H, W))
    return np.concatenate([img, (a % 256).astype(np.uint8)[..., None]], -1)


def alpha_header(data):
    """ALPH chunk header byte of a VP8X file -> (method, filter, pre_processing)."""
    p = 12
    while p + 8 <= len(data):
        tag, size = data[p:p + 4], int.from_bytes(data[p + 4:p + 8], "little")
        if tag == b"ALPH":
            b0 = data[p + 8]
            return dict(method=b0 & 3, filter=(b0 >> 2) & 3, pre=(b0 >> 4) & 3)
        p += 8 + size + (size & 1)
    return None


def set_alpha_filter(data, filt):
    """Rewrite the ALPH header's filter bits.  libwebp never filters raw (method 0) alpha
    ("filtering will make no impact on compressed size"), but its decoder unfilters any
    method; the payload bytes are then read as filtered data and libwebp's decode of the
    edited file is the expected output."""
    b = bytearray(data)
    p = 12
    while p + 8 <= len(b):
        tag, size = bytes(b[p:p + 4]), int.from_bytes(b[p + 4:p + 8], "little")
        if tag == b"ALPH":
            b[p + 8] = (b[p + 8] & ~0x0c) | (filt << 2)
            return bytes(b)
        p += 8 + size + (size & 1)
    raise ValueError("no ALPH chunk")


def riff_chunks(data):
    """[(tag, payload)] of a RIFF/WEBP file."""
    out, p = [], 12
    while p + 8 <= len(data):
        tag, size = data[p:p + 4], int.from_bytes(data[p + 4:p + 8], "little")
        out.append((tag, data[p + 8:p + 8 + size]))
        p += 8 + size + (size & 1)
    return out


def riff_build(chunks):
    body = b"WEBP"
    for tag, payload in chunks:
        body += tag + len(payload).to_bytes(4, "little") + payload + (b"\0" if len(payload) & 1 else b"")
    return b"RIFF" + len(body).to_bytes(4, "little") + body


def edit_alph(data, fn):
    return riff_build([(t, fn(pl) if t == b"ALPH" else pl) for t, pl in riff_chunks(data)])


def decode_status(data):
    """WebPDecode's status for RGBA output (plain-C kernels)."""
    cfg = (C.c_uint8 * 512)()
    assert LIB.WebPInitDecoderConfigInternal(cfg, ABI)
    C.cast(cfg, C.POINTER(C.c_int32))[40 // 4] = MODE_RGBA
    st = LIB.WebPDecode(data, C.c_size_t(len(data)), cfg)
    LIB.WebPFreeDecBuffer(C.byref(cfg, 40))
    return st


# corrupted ALPH chunks: (name, source fixture, edit of the chunk payload)
ALPHA_ERROR_CASES = [
    ("e_reserved_bits", "a_raw_none_40x30", lambda pl: bytes([pl[0] | 0x40]) + pl[1:]),
    ("e_method2", "a_raw_none_40x30", lambda pl: bytes([(pl[0] & ~3) | 2]) + pl[1:]),
    ("e_preproc2", "a_ll_none_33x65", lambda pl: bytes([(pl[0] & ~0x30) | 0x20]) + pl[1:]),
    ("e_raw_short", "a_raw_h_71x33", lambda pl: pl[:-1]),
    ("e_header_only", "a_ll_h_130x70", lambda pl: pl[:1]),
    ("e_ll_stream_2b", "a_ll_h_130x70", lambda pl: pl[:3]),
    ("e_ll_stream_half", "a_ll_g_120x1100", lambda pl: pl[:len(pl) // 2]),
    ("e_ll_stream_zeros", "a_ll_v_97x81", lambda pl: pl[:1] + bytes(len(pl) - 1)),
]


# ----------------------------------------------------------------------------- output modes
# WEBP_CSP_MODE (pkg/libwebp/webp/decode.go enums): bytes per pixel of each RGB-family mode
MODE_BPP = {0: 3, 1: 4, 2: 3, 3: 4, 4: 4, 5: 2, 6: 2, 7: 4, 8: 4, 9: 4, 10: 2}


def decode_mode(data, mode, crop=None, flip=0, no_fancy=0, bypass=0):
    """WebPDecode with config.output.colorspace = mode (+ cropping / flip options) -> (status,
    (h, w * bpp) uint8 rows)."""
    cfg = (C.c_uint8 * 512)()
    assert LIB.WebPInitDecoderConfigInternal(cfg, ABI)
    ci = C.cast(cfg, C.POINTER(C.c_int32))
    ci[40 // 4] = mode
    ci[160 // 4] = bypass
    ci[164 // 4] = no_fancy
    if crop is not None:
        ci[168 // 4] = 1
        ci[172 // 4], ci[176 // 4], ci[180 // 4], ci[184 // 4] = crop
    ci[208 // 4] = flip
    st = LIB.WebPDecode(data, C.c_size_t(len(data)), cfg)
    if st != 0:
        return st, None
    w, h = ci[44 // 4], ci[48 // 4]
    cp = C.cast(cfg, C.POINTER(C.c_void_p))
    stride = ci[64 // 4]
    bpp = MODE_BPP[mode]
    base = cp[56 // 8]  # with flip, DecodeInto restores pointer and stride: rows are stored flipped
    rows = [np.frombuffer(C.string_at(base + r * stride, w * bpp), np.uint8) for r in range(h)]
    LIB.WebPFreeDecBuffer(C.byref(cfg, 40))
    return 0, np.stack(rows)


MODE_SOURCES = [("lossy", "synth_17x9"), ("lossy", "synth_80x96"), ("alpha", "a_raw_g_64x64"),
                ("lossy", "alpha_64x48"), ("lossless", "ll_alpha_48x48"), ("lossless", "ll_pal4_63x41")]
# (crop_left, crop_top, crop_width, crop_height); odd left/top are snapped to even by libwebp
MODE_CROPS = {"none": None, "c1": (3, 5, 20, 11), "c2": (0, 0, 9, 1), "c3": (6, 2, 1, 7), "c4": (5, 3, 12, 6)}


def mode_cases(data, w, h, lossy):
    """Outputs of every mode x crop (+ flip / no-fancy on two crops, no-fancy for lossy only);
    the 'full' crop (= no crop) and the out-of-bounds one only record a status."""
    out, statuses = {}, {}
    crops = dict(MODE_CROPS)
    crops["full"] = (0, 0, w, h)
    crops["oob"] = (w - 4, 0, 8, 2)  # past the right edge: INVALID_PARAM
    for cname, crop in crops.items():
        for mode in MODE_BPP:
            for flip in (0, 1):
                for nf in (0, 1):
                    if (flip or nf) and cname not in ("none", "c1") or (nf and not lossy):
                        continue
                    key = f"m{mode}_{cname}_f{flip}_nf{nf}"
                    st, arr = decode_mode(data, mode, crop, flip, nf)
                    _plain_c(False)
                    st2, arr2 = decode_mode(data, mode, crop, flip, nf)
                    _plain_c(True)
                    assert st == st2 and (arr is None or np.array_equal(arr, arr2)), key
                    statuses[key] = st
                    if arr is not None and cname != "full":
                        out[key] = arr
    return out, statuses


# ----------------------------------------------------------------------------- YUV output modes
# MODE_YUV = 11, MODE_YUVA = 12 (WebPDecodeYUV / WebPDecodeYUVInto, webp.go:615-725; EmitYUV /
# EmitAlphaYUV io_dec.c.go:36-60, 128-150 for lossy; libwebp 1.6.0 converts lossless rows with
# ConvertToYUVA, vp8l_dec.c.go:544-563)
def decode_yuva(data, mode, crop=None, flip=0, bypass=0):
    """WebPDecode with config.output.colorspace = MODE_YUV / MODE_YUVA (+ crop / flip) -> (status,
    {"y", "u", "v"[, "a"]} arrays)."""
    cfg = (C.c_uint8 * 512)()
    assert LIB.WebPInitDecoderConfigInternal(cfg, ABI)
    ci = C.cast(cfg, C.POINTER(C.c_int32))
    ci[40 // 4] = mode
    ci[160 // 4] = bypass
    if crop is not None:
        ci[168 // 4] = 1
        ci[172 // 4], ci[176 // 4], ci[180 // 4], ci[184 // 4] = crop
    ci[208 // 4] = flip
    st = LIB.WebPDecode(data, C.c_size_t(len(data)), cfg)
    if st != 0:
        return st, None
    w, h = ci[44 // 4], ci[48 // 4]
    cp = C.cast(cfg, C.POINTER(C.c_void_p))
    # WebPYUVABuffer: y, u, v, a pointers at 56..80, strides y/u/v/a at 88..100
    uw, uh = (w + 1) // 2, (h + 1) // 2

    def plane(ptr, stride, pw, ph):  # (flip: DecodeInto restores pointer and stride, rows stored flipped)
        return np.stack([np.frombuffer(C.string_at(ptr + r * stride, pw), np.uint8) for r in range(ph)])
    out = {"y": plane(cp[56 // 8], ci[88 // 4], w, h), "u": plane(cp[64 // 8], ci[92 // 4], uw, uh),
           "v": plane(cp[72 // 8], ci[96 // 4], uw, uh)}
    if mode == 12:
        out["a"] = plane(cp[80 // 8], ci[100 // 4], w, h)
    LIB.WebPFreeDecBuffer(C.byref(cfg, 40))
    return 0, out


# sources: the output-mode ones (lossy with and without ALPH, lossless with alpha and palette) plus
# lossless frames with odd sizes (the odd last column / row of ConvertToYUVA) and a
# semi-transparent one with fully transparent and opaque regions (the A plane), and lossy ALPH
# with level-quantized alpha
YUV_SOURCES = MODE_SOURCES + [("lossless", "ll_corr_123x77"), ("alpha", "a_ll_q50_80x80"),
                              ("yuv", "ll_alpha_odd_37x23")]
YUV_CROPS = {"none": None, "c1": (3, 5, 20, 11), "c2": (0, 0, 9, 1), "c3": (6, 2, 1, 7), "c4": (5, 3, 12, 6),
             "c5": (1, 1, 7, 5)}


def yuv_extra_sources():
    """Fixtures only the YUV section uses: written to tests/golden/yuv/."""
    img = with_alpha(corr_luma(23, 37, 21), 21)
    img[5:9, 20:30, 3] = 255  # an opaque patch among the semi-transparent and transparent ones
    return {"ll_alpha_odd_37x23": encode(img, lossless=1, exact=1)}


def yuv_cases(data, w, h):
    """MODE_YUV / MODE_YUVA outputs per crop (flip on two crops); 'oob' records a status."""
    out, statuses = {}, {}
    crops = dict(YUV_CROPS)
    crops["oob"] = (w - 4, 0, 8, 2)
    for cname, crop in crops.items():
        for mode in (11, 12):
            for flip in (0, 1):
                if flip and cname not in ("none", "c1"):
                    continue
                key = f"m{mode}_{cname}_f{flip}"
                st, arrs = decode_yuva(data, mode, crop, flip)
                _plain_c(False)
                st2, arrs2 = decode_yuva(data, mode, crop, flip)
                _plain_c(True)
                assert st == st2, key
                if arrs is not None:
                    for k in arrs:
                        assert np.array_equal(arrs[k], arrs2[k]), (key, k)
                        out[f"{key}_{k}"] = arrs[k]
                statuses[key] = st
    return out, statuses


# ----------------------------------------------------------------------------- animation
DEMUX_ABI = 0x0107  # WEBP_DEMUX_ABI_VERSION of 1.6.0
MUX_ABI = 0x0109    # WEBP_MUX_ABI_VERSION of 1.6.0


def _load_anim_libs():
    mux = C.CDLL(glob.glob(PIL_LIBS + "libwebpmux-*.so*")[0])
    dmx = C.CDLL(glob.glob(PIL_LIBS + "libwebpdemux-*.so*")[0])
    mux.WebPAnimEncoderNewInternal.restype = C.c_void_p
    mux.WebPAnimEncoderNewInternal.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int]
    mux.WebPAnimEncoderAdd.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    mux.WebPAnimEncoderAssemble.argtypes = [C.c_void_p, C.c_void_p]
    mux.WebPAnimEncoderDelete.argtypes = [C.c_void_p]
    dmx.WebPAnimDecoderNewInternal.restype = C.c_void_p
    dmx.WebPAnimDecoderNewInternal.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    dmx.WebPAnimDecoderGetInfo.argtypes = [C.c_void_p, C.c_void_p]
    dmx.WebPAnimDecoderHasMoreFrames.argtypes = [C.c_void_p]
    dmx.WebPAnimDecoderGetNext.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    dmx.WebPAnimDecoderDelete.argtypes = [C.c_void_p]
    return mux, dmx


class WebPData(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("size", C.c_size_t)]


def _picture(img):
    h, w, ch = img.shape
    pic = (C.c_uint8 * 512)()
    assert LIB.WebPPictureInitInternal(pic, ABI)
    pi = C.cast(pic, C.POINTER(C.c_int32))
    pi[0] = 1
    pi[2] = w
    pi[3] = h
    buf = np.ascontiguousarray(img)
    ok = (LIB.WebPPictureImportRGBA if ch == 4 else LIB.WebPPictureImportRGB)(pic, buf.ctypes.data_as(C.c_void_p),
                                                                             w * ch)
    assert ok
    return pic


def _config(lossless, quality=75.0):
    cfg = (C.c_int32 * 64)()
    assert LIB.WebPConfigInitInternal(cfg, 0, C.c_float(quality), ABI)
    cfg[0] = lossless
    C.cast(cfg, C.POINTER(C.c_float))[1] = quality
    assert LIB.WebPValidateConfig(cfg)
    return cfg


def anim_encode(frames, durations, lossless_flags, allow_mixed=1, kmax=0, loop=0, bgcolor=0xffffffff):
    """WebPAnimEncoder over full-canvas frames (it picks sub-rectangles, blend and dispose)."""
    mux, _ = _load_anim_libs()
    h, w = frames[0].shape[:2]
    opt = (C.c_int32 * 16)()
    assert mux.WebPAnimEncoderOptionsInitInternal(opt, MUX_ABI)
    opt[0] = C.c_int32(bgcolor - (1 << 32) if bgcolor >= 1 << 31 else bgcolor).value  # anim_params.bgcolor
    opt[1] = loop                     # anim_params.loop_count
    opt[3] = 0 if kmax == 0 else max(1, kmax - 1)  # kmin
    opt[4] = kmax                     # kmax
    opt[5] = allow_mixed
    enc = mux.WebPAnimEncoderNewInternal(w, h, opt, MUX_ABI)
    assert enc
    t = 0
    for img, d, ll in zip(frames, durations, lossless_flags):
        pic = _picture(img)
        assert mux.WebPAnimEncoderAdd(enc, pic, t, _config(ll)), "AnimEncoderAdd"
        LIB.WebPPictureFree(pic)
        t += d
    assert mux.WebPAnimEncoderAdd(enc, None, t, None)
    data = WebPData()
    assert mux.WebPAnimEncoderAssemble(enc, C.byref(data))
    out = C.string_at(data.bytes, data.size)
    LIB.WebPFree(C.c_void_p(data.bytes))
    mux.WebPAnimEncoderDelete(enc)
    return out


def image_chunks(data):
    """The ALPH / VP8 / VP8L chunks (header + padded payload) of a still image file."""
    return b"".join(t + len(pl).to_bytes(4, "little") + pl + (b"\0" if len(pl) & 1 else b"")
                    for t, pl in riff_chunks(data) if t in (b"ALPH", b"VP8 ", b"VP8L"))


def anim_build(canvas_w, canvas_h, frames, loop=0, bgcolor=0xffffffff):
    """Hand-built animation: frames = [(encoded still, x, y, duration, dispose_bg, no_blend)]."""
    has_alpha = any(b"ALPH" in f[0] or b"VP8L" in f[0] for f in frames)
    vp8x = bytes([0x02 | (0x10 if has_alpha else 0), 0, 0, 0]) + (canvas_w - 1).to_bytes(3, "little") + \
        (canvas_h - 1).to_bytes(3, "little")
    chunks = [(b"VP8X", vp8x), (b"ANIM", bgcolor.to_bytes(4, "little") + loop.to_bytes(2, "little"))]
    for data, x, y, dur, dispose_bg, no_blend in frames:
        assert x % 2 == 0 and y % 2 == 0
        fw, fh = None, None
        for t, pl in riff_chunks(data):
            if t == b"VP8X":
                fw, fh = 1 + int.from_bytes(pl[4:7], "little"), 1 + int.from_bytes(pl[7:10], "little")
        if fw is None:
            t, pl = riff_chunks(data)[0]
            if t == b"VP8 ":
                fw, fh = int.from_bytes(pl[6:8], "little") & 0x3fff, int.from_bytes(pl[8:10], "little") & 0x3fff
            else:
                v = int.from_bytes(pl[1:5], "little")
                fw, fh = (v & 0x3fff) + 1, ((v >> 14) & 0x3fff) + 1
        hdr = (x // 2).to_bytes(3, "little") + (y // 2).to_bytes(3, "little") + (fw - 1).to_bytes(3, "little") + \
            (fh - 1).to_bytes(3, "little") + dur.to_bytes(3, "little") + bytes([(1 if dispose_bg else 0) |
                                                                                 (2 if no_blend else 0)])
        chunks.append((b"ANMF", hdr + image_chunks(data)))
    return riff_build(chunks)


def anim_decode(data):
    """WebPAnimDecoder (MODE_RGBA): (info dict, canvases (F, H, W, 4), timestamps)."""
    _, dmx = _load_anim_libs()
    opt = (C.c_int32 * 9)()
    assert dmx.WebPAnimDecoderOptionsInitInternal(opt, DEMUX_ABI)
    opt[0] = MODE_RGBA
    wd = WebPData(C.cast(C.c_char_p(data), C.c_void_p).value, len(data))
    dec = dmx.WebPAnimDecoderNewInternal(C.byref(wd), opt, DEMUX_ABI)
    assert dec, "WebPAnimDecoderNew failed"
    info = (C.c_uint32 * 9)()
    assert dmx.WebPAnimDecoderGetInfo(dec, info)
    w, h = info[0], info[1]
    frames, ts = [], []
    while dmx.WebPAnimDecoderHasMoreFrames(dec):
        buf, t = C.c_void_p(), C.c_int()
        assert dmx.WebPAnimDecoderGetNext(dec, C.byref(buf), C.byref(t))
        frames.append(np.frombuffer(C.string_at(buf, w * h * 4), np.uint8).reshape(h, w, 4).copy())
        ts.append(t.value)
    dmx.WebPAnimDecoderDelete(dec)
    return (dict(canvas_width=w, canvas_height=h, loop_count=info[2], bgcolor=info[3], frame_count=info[4]),
            np.stack(frames), np.array(ts, np.int32))


def moving_scene(H, W, n, seed, alpha=False):
    """n full-canvas frames: a textured background with a square moving across it; with
    alpha, the background is partly transparent and the square semi-transparent."""
    rng = np.random.default_rng(seed)
    base = synth(H, W, seed, 4)
    out = []
    for i in range(n):
        img = base.copy()
        s = max(4, min(H, W) // 4)
        y0, x0 = (i * 5) % (H - s), (i * 9) % (W - s)
        img[y0:y0 + s, x0:x0 + s] = (40 * i % 256, 200, 90)
        if alpha:
            a = np.full((H, W, 1), 255, np.uint8)
            a[: H // 3, :] = 0
            a[y0:y0 + s, x0:x0 + s] = 128 + 20 * i % 100
            a[H // 2:, : W // 3] = rng.integers(0, 256, (H - H // 2, W // 3, 1))
            img = np.concatenate([img, a], -1)
        out.append(img)
    return out


def sprite(h, w, seed, alpha_kind):
    rng = np.random.default_rng(seed)
    img = synth(h, w, seed, 10)
    a = {"opaque": np.full((h, w), 255), "half": np.full((h, w), 128), "mixed": rng.integers(0, 256, (h, w)),
         "holes": np.where((np.arange(w)[None, :] // 3 + np.arange(h)[:, None] // 3) % 2 == 0, 255, 0)}[alpha_kind]
    return np.concatenate([img, a.astype(np.uint8)[..., None]], -1)


def _manual_anims():
    lossy_full = encode(synth(48, 64, 50, 6))
    ll_sprite = encode(sprite(20, 30, 51, "mixed"), lossless=1, exact=1)
    lossy_alpha_sprite = encode(sprite(16, 16, 52, "half"))
    ll_holes = encode(sprite(30, 40, 53, "holes"), lossless=1, exact=1)
    ll_full_alpha = encode(sprite(48, 64, 54, "mixed"), lossless=1, exact=1)
    lossy_sprite = encode(synth(12, 18, 55, 6))
    return {
        # blend over dispose-none, blend over dispose-background (blend only outside the previous
        # rectangle), an opaque sub-frame, a full no-blend frame, dispose of a full frame
        "anim_manual_blend_dispose": anim_build(64, 48, [
            (lossy_full, 0, 0, 100, False, False),
            (ll_sprite, 10, 8, 50, False, False),
            (lossy_alpha_sprite, 20, 10, 70, True, False),
            (ll_holes, 0, 0, 40, False, False),
            (lossy_sprite, 40, 30, 30, True, True),
            (ll_full_alpha, 0, 0, 60, True, True),
            (ll_sprite, 34, 28, 20, False, False),
        ], loop=3, bgcolor=0xff336699),
        # key-frame rules: a no-blend full frame with alpha, a frame after a full dispose-background
        "anim_manual_keyframes": anim_build(64, 48, [
            (ll_sprite, 4, 4, 10, True, False),
            (ll_full_alpha, 0, 0, 10, False, True),
            (lossy_alpha_sprite, 2, 2, 10, False, False),
            (ll_full_alpha, 0, 0, 10, True, False),
            (ll_holes, 12, 6, 10, False, False),
        ]),
        "anim_manual_single": anim_build(30, 20, [(ll_sprite, 0, 0, 0, False, False)], loop=1),
    }


ANIM_CASES = [
    # name, builder
    ("anim_enc_mixed_96x80", lambda: anim_encode(moving_scene(80, 96, 8, 60), [40] * 8, [0, 1, 0, 0, 1, 0, 0, 1])),
    ("anim_enc_alpha_lossless_72x56", lambda: anim_encode(moving_scene(56, 72, 6, 61, alpha=True),
                                                         [30, 60, 30, 60, 30, 60], [1] * 6)),
    ("anim_enc_alpha_lossy_80x64", lambda: anim_encode(moving_scene(64, 80, 6, 62, alpha=True), [25] * 6, [0] * 6,
                                                      allow_mixed=0)),
    ("anim_enc_keyframes_64x64", lambda: anim_encode(moving_scene(64, 64, 9, 63, alpha=True), [20] * 9,
                                                    [0, 1] * 4 + [0], kmax=3)),
]


# ----------------------------------------------------------------------------- cases
LOSSY_CASES = [
    # name, image-fn, encoder kwargs
    ("synth_17x9", lambda: synth(9, 17, 1, 6), {}),
    ("synth_1x1", lambda: synth(1, 1, 2, 6), {}),
    ("synth_2x3", lambda: synth(3, 2, 2, 6), {}),
    ("synth_80x96", lambda: synth(96, 80, 3, 6), {}),
    ("synth_128x128_q90", lambda: synth(128, 128, 4, 6), {"quality": 90}),
    ("synth_481x270", lambda: synth(270, 481, 5, 6), {}),
    ("noise_96x64_complex_s0", lambda: noise(64, 96, 6), {"sharpness": 0}),
    ("noise_96x64_complex_s3", lambda: noise(64, 96, 7), {"sharpness": 3, "filter_strength": 80}),
    ("noise_96x64_complex_s7", lambda: noise(64, 96, 8), {"sharpness": 7, "filter_strength": 100}),
    ("noise_96x64_simple", lambda: noise(64, 96, 9), {"filter_type": 0, "filter_strength": 70}),
    ("noise_96x64_simple_s5", lambda: noise(64, 96, 10), {"filter_type": 0, "sharpness": 5, "filter_strength": 50}),
    ("noise_96x64_nofilter", lambda: noise(64, 96, 11), {"filter_strength": 0}),
    ("noise_97x63_q20", lambda: noise(63, 97, 12, 40), {"quality": 20, "filter_strength": 100}),
    ("noise_64x64_q100", lambda: noise(64, 64, 13, 80), {"quality": 100}),
    ("smooth_160x112", lambda: smooth(112, 160, 14), {}),
    ("smooth_161x113_simple", lambda: smooth(113, 161, 15), {"filter_type": 0}),
    ("synth_200x150_seg1", lambda: synth(150, 200, 16, 12), {"segments": 1}),
    ("synth_200x150_part4", lambda: synth(150, 200, 17, 12), {"partitions": 2, "method": 2}),
    ("synth_200x150_part8", lambda: synth(150, 200, 18, 12), {"partitions": 3, "low_memory": 1}),
    ("noise_130x70_q5", lambda: noise(70, 130, 19, 30), {"quality": 5, "filter_strength": 100}),
    ("synth_256x256_sns100", lambda: synth(256, 256, 20, 20), {"sns": 100, "filter_strength": 40}),
    ("alpha_64x48", lambda: with_alpha(synth(48, 64, 21, 6), 21), {}),
    # wider than K1's LDS column store (mb_w > 600): the global-store variant
    ("wide_9617x40", lambda: synth(40, 9617, 22, 6), {"quality": 60}),
    ("wide_16383x17_simple", lambda: smooth(17, 16383, 23), {"filter_type": 0, "quality": 50}),
]

# Narrow and tall frames for K1's quad geometry (4 MB rows per wave, 12 waves): one MB column
# (the first MB is also the last), partial last quads (mb_h % 4 = 1..3), more quads than waves
# (the progress ring wraps), i4-heavy content under both filters.  Generated by the
# "lossy_extra" section, which adds to the lossy fixtures without re-encoding the others.
LOSSY_EXTRA_CASES = [
    ("synth_16x200", lambda: synth(200, 16, 24, 6), {}),
    ("noise_9x300_complex", lambda: noise(300, 9, 25), {"filter_strength": 80}),
    ("noise_40x336", lambda: noise(336, 40, 26), {"sharpness": 2}),
    ("smooth_24x1000_simple", lambda: smooth(1000, 24, 27), {"filter_type": 0, "filter_strength": 70}),
    ("noise_33x1000", lambda: noise(1000, 33, 28, 40), {"filter_strength": 60}),
    ("synth_600x70", lambda: synth(70, 600, 29, 10), {}),
    ("noise_250x100_q30", lambda: noise(100, 250, 30, 50), {"quality": 30, "filter_strength": 90}),
]

LOSSLESS_CASES = [
    ("ll_corr_64x64", lambda: corr_luma(64, 64, 1), {"method": 4}),
    ("ll_corr_123x77", lambda: corr_luma(77, 123, 2), {"method": 6, "quality": 100}),
    ("ll_synth_90x33_m0", lambda: synth(33, 90, 3, 10), {"method": 0}),
    ("ll_noise_50x50", lambda: noise(50, 50, 4, 30), {"method": 4}),
    ("ll_pal2_64x40", lambda: palette_img(40, 64, 5, 2), {}),
    ("ll_pal4_63x41", lambda: palette_img(41, 63, 6, 4), {}),
    ("ll_pal16_65x39", lambda: palette_img(39, 65, 7, 16), {}),
    ("ll_pal200_70x30", lambda: palette_img(30, 70, 8, 200), {}),
    ("ll_alpha_48x48", lambda: with_alpha(corr_luma(48, 48, 9), 9), {"exact": 1}),
    ("ll_smooth_100x60_q0", lambda: smooth(60, 100, 10), {"quality": 0, "method": 1}),
]

ALPHA_CASES = [
    # name, image-fn, encoder kwargs, expected (method, filter)
    ("a_raw_none_40x30", lambda: alpha_pattern(30, 40, 31, "n"),
     {"alpha_compression": 0, "alpha_filtering": 0}, (0, 0)),
    # set_filter: the ALPH filter bits rewritten after encoding (set_alpha_filter)
    ("a_raw_h_71x33", lambda: alpha_pattern(33, 71, 32, "n"), {"alpha_compression": 0, "set_filter": 1}, (0, 1)),
    ("a_raw_v_50x47", lambda: alpha_pattern(47, 50, 33, "n"), {"alpha_compression": 0, "set_filter": 2}, (0, 2)),
    ("a_raw_g_64x64", lambda: alpha_pattern(64, 64, 34, "n"), {"alpha_compression": 0, "set_filter": 3}, (0, 3)),
    ("a_raw_g_40x1030", lambda: alpha_pattern(1030, 40, 42, "n"), {"alpha_compression": 0, "set_filter": 3},
     (0, 3)),
    ("a_ll_none_33x65", lambda: alpha_pattern(65, 33, 35, "h"), {"alpha_filtering": 0}, (1, 0)),
    ("a_ll_h_130x70", lambda: alpha_pattern(70, 130, 36, "h"), {"alpha_filtering": 0, "set_filter": 1}, (1, 1)),
    ("a_ll_v_97x81", lambda: alpha_pattern(81, 97, 37, "v"), {"alpha_filtering": 0, "set_filter": 2}, (1, 2)),
    ("a_ll_g_120x1100", lambda: alpha_pattern(1100, 120, 38, "g"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_best_h_96x64", lambda: alpha_pattern(64, 96, 43, "h"), {"alpha_filtering": 2}, None),
    ("a_ll_best_g_96x64", lambda: alpha_pattern(64, 96, 44, "g"), {"alpha_filtering": 2}, None),
    ("a_ll_levels_90x60", lambda: alpha_pattern(60, 90, 39, "lv"), {"alpha_filtering": 0}, (1, 0)),
    ("a_ll_q50_80x80", lambda: alpha_pattern(80, 80, 40, "g"), {"alpha_filtering": 1, "alpha_quality": 50}, None),
    ("a_ll_1x1", lambda: alpha_pattern(1, 1, 41, "n"), {}, None),
]
# section alpha_r5 (added to "alpha"): alpha streams under filters none / horizontal -- 8-bit ones
# (a palette, 1 or 8 pixels per coded pixel), which K4 expands straight from K7's output (no K3),
# and predictor-coded ones (K3, then K4 from its RGBA)
ALPHA_CASES_R5 = [
    ("a_ll_bin_none_70x45", lambda: alpha_pattern(45, 70, 45, "bin"), {"alpha_filtering": 0}, (1, 0)),
    ("a_ll_bin_h_133x40", lambda: alpha_pattern(40, 133, 46, "bin"), {"alpha_filtering": 0, "set_filter": 1}, (1, 1)),
    ("a_ll_many_none_75x50", lambda: alpha_pattern(50, 75, 47, "many"), {"alpha_filtering": 0}, (1, 0)),
    ("a_ll_many_h_66x90", lambda: alpha_pattern(90, 66, 48, "many"), {"alpha_filtering": 0, "set_filter": 1}, (1, 1)),
    ("a_ll_rl_none_61x29", lambda: alpha_pattern(29, 61, 49, "rl"), {"alpha_filtering": 0}, (1, 0)),
    ("a_ll_rl_h_64x33", lambda: alpha_pattern(33, 64, 50, "rl"), {"alpha_filtering": 0, "set_filter": 1}, (1, 1)),
]
# section alpha_r6 (added to "alpha"): 8-bit streams under vertical / gradient, whose filtered bytes
# K7 writes itself (into the plane; gradient rows into band tiles) -- maps of 2, 4 and 12 colours
# (8, 4, 2 pixels per coded pixel) and none, widths off the 8- and 16-byte grid, several bands
ALPHA_CASES_R6 = [
    ("a_ll_bin_g_70x150", lambda: alpha_pattern(150, 70, 51, "bin"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_lv_g_90x130", lambda: alpha_pattern(130, 90, 52, "lv"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_l12_g_88x140", lambda: alpha_pattern(140, 88, 53, "l12"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_l12_g_256x70", lambda: alpha_pattern(70, 256, 54, "l12"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_rl_g_61x100", lambda: alpha_pattern(100, 61, 55, "rl"), {"alpha_filtering": 0, "set_filter": 3}, (1, 3)),
    ("a_ll_l12_v_88x50", lambda: alpha_pattern(50, 88, 56, "l12"), {"alpha_filtering": 0, "set_filter": 2}, (1, 2)),
    ("a_ll_rl_v_61x40", lambda: alpha_pattern(40, 61, 57, "rl"), {"alpha_filtering": 0, "set_filter": 2}, (1, 2)),
    ("a_ll_l12_none_72x30", lambda: alpha_pattern(30, 72, 58, "l12"), {"alpha_filtering": 0}, (1, 0)),
]

BENCH_CASES = [
    # name, H, W, seeds, kwargs, generator  
    ("c1_512", 512, 512, [0], {}, "synth6"),
    ("c2_1080p", 1080, 1920, list(range(8)), {}, "synth6"),
    ("c3_4k", 2160, 3840, list(range(8)), {"filter_type": 1, "filter_strength": 60}, "synth6"),
    ("c5_ll2048", 2048, 2048, [0], {"lossless": 1}, "corr"),
]
# section bench_c5x: the other C5 seeds (K = 8 distinct lossless frames, like C2 / C3)
BENCH_C5X = [("c5_ll2048", 2048, 2048, list(range(1, 8)), {"lossless": 1}, "corr")]
# section bench_c3s: SURVEY §8(d)'s entropy-stress variant of C3 (sigma = 18, ~2 bpp: dense
# coefficients, i4-heavy), 8 seeds, the C3 encoder settings
BENCH_C3S = [("c3s_4k", 2160, 3840, list(range(8)), {"filter_type": 1, "filter_strength": 60}, "synth18")]
# section bench_c3a: the "next" row f2 (ALPH, K4) at C3's size: C3's frames (same encoder
# settings) with a feathered cut-out alpha plane, lossless-compressed ALPH, 8 seeds
BENCH_C3A = [("c3a_4k", 2160, 3840, list(range(8)), {"filter_type": 1, "filter_strength": 60}, "synth6a")]
# section bench_anim: the "next" row f3 (animation, K5): 64 frames of a 1920x1080 canvas through
# WebPAnimEncoder (lossy, blended sub-rectangles); per-canvas SHA-256 of WebPAnimDecoder's output
BENCH_ANIM = [("anim_1080p_x64", 1080, 1920, 64, 70)]
# section bench_modes: the "next" row f4 (output colorspace, K6) on C3's frames: SHA-256 of
# WebPDecode's MODE_RGB_565 bytes (fancy upsampling) added to the C3 entries
BENCH_MODES = [("c3_4k", 6, "rgb565")]  # MODE_RGB_565 = 6 (WEBP_CSP_MODE)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main(argv):
    """argv: sections to (re)generate among lossy, lossy_extra, lossless, alpha, modes, anim, bench (default: all);
    the manifest entries of the other sections are kept."""
    sections = set(argv) or {"lossy", "lossy_extra", "lossless", "alpha", "modes", "yuv", "anim", "bench", "bench_c5x",
                             "bench_c3s", "bench_c3a", "bench_anim", "bench_modes", "fuzz", "alpha_r5", "alpha_r6", "bench_yuva",
                             "bench_c3ag"}
    os.makedirs(os.path.join(HERE, "lossy"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "lossless"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "bench"), exist_ok=True)
    mpath = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    manifest["libwebp"] = "1.6.0 (Pillow 12.2.0 bundle, plain-C DSP)"
    for sec in sections - {"bench_c5x", "bench_c3s", "bench_c3a", "bench_modes", "alpha_r5", "alpha_r6", "bench_yuva",
                           "bench_c3ag"}:  # (these add)
        manifest[sec] = {}
    manifest.setdefault("alpha", {})
    manifest.setdefault("bench", {})
    if "alpha" in sections:
        manifest["alpha_errors"] = {}
    extra = LOSSY_EXTRA_CASES if "lossy_extra" in sections else []
    manifest.pop("lossy_extra", None)
    manifest.setdefault("lossy", {})
    for name, fn, kw in (LOSSY_CASES if "lossy" in sections else []) + extra:
        img = fn()
        data = encode(img, **kw)
        r = decode_all(data, lossy=True)
        with open(os.path.join(HERE, "lossy", name + ".webp"), "wb") as f:
            f.write(data)
        np.savez_compressed(os.path.join(HERE, "lossy", name + ".npz"), **r)
        hdr = vp8_header(data)
        manifest["lossy"][name] = dict(bytes=len(data), width=img.shape[1], height=img.shape[0],
                                       header=hdr, encoder=kw)
        print(name, len(data), hdr, flush=True)
    for name, fn, kw in LOSSLESS_CASES if "lossless" in sections else []:
        img = fn()
        data = encode(img, lossless=1, **kw)
        r = decode_all(data, lossy=False)
        with open(os.path.join(HERE, "lossless", name + ".webp"), "wb") as f:
            f.write(data)
        np.savez_compressed(os.path.join(HERE, "lossless", name + ".npz"), **r)
        manifest["lossless"][name] = dict(bytes=len(data), width=img.shape[1], height=img.shape[0], encoder=kw)
        print(name, len(data), flush=True)
    os.makedirs(os.path.join(HERE, "alpha"), exist_ok=True)
    for name, fn, kw, want in (ALPHA_CASES if "alpha" in sections else []) + \
            (ALPHA_CASES_R5 if sections & {"alpha", "alpha_r5"} else []) + \
            (ALPHA_CASES_R6 if sections & {"alpha", "alpha_r6"} else []):
        img = fn()
        kw = dict(kw)
        filt = kw.pop("set_filter", None)
        data = encode(img, **kw)
        if filt is not None:
            data = set_alpha_filter(data, filt)
            kw["set_filter"] = filt
        hdr = alpha_header(data)
        assert hdr is not None, name
        if want is not None:
            assert (hdr["method"], hdr["filter"]) == want, (name, hdr)
        r = decode_all(data, lossy=False)
        with open(os.path.join(HERE, "alpha", name + ".webp"), "wb") as f:
            f.write(data)
        np.savez_compressed(os.path.join(HERE, "alpha", name + ".npz"), **r)
        manifest["alpha"][name] = dict(bytes=len(data), width=img.shape[1], height=img.shape[0], alph=hdr,
                                       encoder=kw)
        print(name, len(data), hdr, flush=True)
    for name, src, fn in ALPHA_ERROR_CASES if "alpha" in sections else []:
        data = edit_alph(open(os.path.join(HERE, "alpha", src + ".webp"), "rb").read(), fn)
        st = decode_status(data)
        _plain_c(False)
        assert decode_status(data) == st, name
        _plain_c(True)
        with open(os.path.join(HERE, "alpha", name + ".webp"), "wb") as f:
            f.write(data)
        manifest["alpha_errors"] = manifest.get("alpha_errors", {})
        manifest["alpha_errors"][name] = dict(source=src, status=st, bytes=len(data))
        print(name, "status", st, flush=True)
    if "modes" in sections:
        os.makedirs(os.path.join(HERE, "modes"), exist_ok=True)
        for kind, src in MODE_SOURCES:
            data = open(os.path.join(HERE, kind, src + ".webp"), "rb").read()
            w, h = _decode_cfg(data, MODE_RGBA).shape[1::-1]
            arrs, statuses = mode_cases(data, w, h, kind != "lossless")
            np.savez_compressed(os.path.join(HERE, "modes", src + ".npz"), **arrs)
            manifest["modes"][src] = dict(source=f"{kind}/{src}.webp", width=w, height=h,
                                          crops={k: v for k, v in MODE_CROPS.items()} | {"full": [0, 0, w, h],
                                                                                       "oob": [w - 4, 0, 8, 2]},
                                          status=statuses)
            print(src, len(arrs), "outputs", sum(1 for v in statuses.values() if v), "errors", flush=True)
    if "yuv" in sections:
        os.makedirs(os.path.join(HERE, "yuv"), exist_ok=True)
        for name, data in yuv_extra_sources().items():
            with open(os.path.join(HERE, "yuv", name + ".webp"), "wb") as f:
                f.write(data)
        for kind, src in YUV_SOURCES:
            data = open(os.path.join(HERE, kind, src + ".webp"), "rb").read()
            w, h = _decode_cfg(data, MODE_RGBA).shape[1::-1]
            arrs, statuses = yuv_cases(data, w, h)
            np.savez_compressed(os.path.join(HERE, "yuv", src + ".npz"), **arrs)
            manifest["yuv"][src] = dict(source=f"{kind}/{src}.webp", width=w, height=h,
                                        crops={k: v for k, v in YUV_CROPS.items()} | {"oob": [w - 4, 0, 8, 2]},
                                        status=statuses)
            print(src, len(arrs), "planes", sum(1 for v in statuses.values() if v), "errors", flush=True)
    if "anim" in sections:
        os.makedirs(os.path.join(HERE, "anim"), exist_ok=True)
        builders = list(ANIM_CASES) + [(k, (lambda v=v: v)) for k, v in _manual_anims().items()]
        for name, build in builders:
            data = build()
            info, canv, ts = anim_decode(data)
            _plain_c(False)
            _, canv_simd, ts_simd = anim_decode(data)
            _plain_c(True)
            assert np.array_equal(canv, canv_simd) and np.array_equal(ts, ts_simd), name
            with open(os.path.join(HERE, "anim", name + ".webp"), "wb") as f:
                f.write(data)
            np.savez_compressed(os.path.join(HERE, "anim", name + ".npz"), canvases=canv, timestamps=ts)
            flags = []
            for t, pl in riff_chunks(data):
                if t == b"ANMF":
                    flags.append(dict(x=2 * int.from_bytes(pl[0:3], "little"), y=2 * int.from_bytes(pl[3:6], "little"),
                                      w=1 + int.from_bytes(pl[6:9], "little"), h=1 + int.from_bytes(pl[9:12], "little"),
                                      duration=int.from_bytes(pl[12:15], "little"), dispose_bg=pl[15] & 1,
                                      no_blend=(pl[15] >> 1) & 1, alpha=b"ALPH" in pl or b"VP8L" in pl))
            manifest["anim"][name] = dict(bytes=len(data), info=info, frames=flags)
            print(name, len(data), info, [(f["x"], f["y"], f["w"], f["h"], f["dispose_bg"], f["no_blend"])
                                          for f in flags], flush=True)
    bench = ((BENCH_CASES if "bench" in sections else []) + (BENCH_C5X if "bench_c5x" in sections else []) +
             (BENCH_C3S if "bench_c3s" in sections else []) + (BENCH_C3A if "bench_c3a" in sections else []))
    for name, H, W, seeds, kw, gen in bench:
        for s in seeds:
            img = (synth(H, W, s, 6) if gen == "synth6" else synth(H, W, s, 18) if gen == "synth18"
                   else np.concatenate([synth(H, W, s, 6), cutout_alpha(H, W, s)[..., None]], -1) if gen == "synth6a"
                   else corr_luma(H, W, s))
            lossless = kw.get("lossless", 0)
            data = encode(img, **kw)
            r = decode_all(data, lossy=not lossless)
            fn = f"{name}_s{s}.webp"
            with open(os.path.join(HERE, "bench", fn), "wb") as f:
                f.write(data)
            ent = dict(bytes=len(data), width=W, height=H, bpp=8.0 * len(data) / (W * H),
                       sha256={k: sha(v) for k, v in r.items()})
            if not lossless:
                ent["header"] = vp8_header(data)
            if gen == "synth6a":
                ent["alph"] = alpha_header(data)
            manifest["bench"][fn] = ent
            print(fn, len(data), flush=True)
    for name, mode, key in BENCH_MODES if "bench_modes" in sections else []:
        for fn in sorted(k for k in manifest["bench"] if k.startswith(name + "_s")):
            data = open(os.path.join(HERE, "bench", fn), "rb").read()
            st, out = decode_mode(data, mode)
            _plain_c(False)
            st2, out2 = decode_mode(data, mode)
            _plain_c(True)
            assert st == 0 and st2 == 0 and np.array_equal(out, out2), fn
            manifest["bench"][fn]["sha256"][key] = sha(out)
            print(fn, key, flush=True)
    if "bench_c3ag" in sections:  # c3a's frames with the ALPH filter bits set to gradient / vertical
        # (libwebp's encoder picks none / horizontal for every alpha plane we tried at 4K, even with
        # alpha_filtering = best on linear ramps: K4's wavefront unfilters get their workload this way;
        # libwebp's decode of the edited file is the expected output, as for the a_*_g / _v fixtures)
        for fn in sorted(k for k in manifest["bench"] if k.startswith("c3a_4k_s")):
            src = open(os.path.join(HERE, "bench", fn), "rb").read()
            for tag, filt in (("c3ag", 3), ("c3av", 2)):
                data = set_alpha_filter(src, filt)
                r = decode_all(data, lossy=True)
                out = fn.replace("c3a_", tag + "_")
                with open(os.path.join(HERE, "bench", out), "wb") as f:
                    f.write(data)
                ent = dict(manifest["bench"][fn])
                ent.update(bytes=len(data), sha256={k: sha(v) for k, v in r.items()}, alph=alpha_header(data))
                manifest["bench"][out] = ent
                print(out, ent["alph"], flush=True)
    if "bench_yuva" in sections:  # MODE_YUVA's A plane of the c3a frames (the Y / U / V are the planes')
        for fn in sorted(k for k in manifest["bench"] if k.startswith("c3a_4k_s")):
            data = open(os.path.join(HERE, "bench", fn), "rb").read()
            st, out = decode_yuva(data, 12)
            assert st == 0 and all(sha(out[k]) == manifest["bench"][fn]["sha256"][k] for k in "yuv"), fn
            manifest["bench"][fn]["sha256"]["a"] = sha(out["a"])
            print(fn, "yuva a", flush=True)
    if "bench_anim" in sections:
        manifest["bench_anim"] = {}
        for name, H, W, n, seed in BENCH_ANIM:
            data = anim_encode(anim_scene(H, W, n, seed), [40] * n, [0] * n, allow_mixed=0)
            info, canv, ts = anim_decode(data)
            _plain_c(False)
            _, canv_simd, ts_simd = anim_decode(data)
            _plain_c(True)
            assert np.array_equal(canv, canv_simd) and np.array_equal(ts, ts_simd), name
            with open(os.path.join(HERE, "bench", name + ".webp"), "wb") as f:
                f.write(data)
            frames = []
            for t, pl in riff_chunks(data):
                if t == b"ANMF":
                    frames.append([2 * int.from_bytes(pl[0:3], "little"), 2 * int.from_bytes(pl[3:6], "little"),
                                   1 + int.from_bytes(pl[6:9], "little"), 1 + int.from_bytes(pl[9:12], "little"),
                                   pl[15] & 1, (pl[15] >> 1) & 1])
            manifest["bench_anim"][name] = dict(bytes=len(data), info=info, timestamps=ts.tolist(),
                                                canvas_sha256=[sha(c) for c in canv], frames=frames)
            print(name, len(data), info, "frame rects", frames[:4], flush=True)
    if "fuzz" in sections:
        # libwebp's WebPDecode status and RGBA digest of every mutant of the fuzz corpora
        # (oracle_lib.fuzz_mutants), so the GPU fuzz tests compare against libwebp too
        sys.path.insert(0, os.path.dirname(HERE))
        from oracle_lib import FUZZ_LOSSLESS, FUZZ_LOSSY, fuzz_mutants
        for kind, args in (("lossy", FUZZ_LOSSY), ("lossless", FUZZ_LOSSLESS)):
            ent = {}
            for key, data in fuzz_mutants(kind, *args):
                st, rgba = decode_mode(data, MODE_RGBA)
                _plain_c(False)
                st2, rgba2 = decode_mode(data, MODE_RGBA)
                _plain_c(True)
                assert st == st2 and (rgba is None or np.array_equal(rgba, rgba2)), key
                ent[key] = dict(status=st, rgba=sha(rgba) if rgba is not None else None)
            manifest["fuzz"][kind] = ent
            print("fuzz", kind, len(ent), "mutants,", sum(1 for e in ent.values() if e["status"] == 0), "decode",
                  flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
