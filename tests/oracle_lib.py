"""ctypes binding of the CPU oracle (oracle/build/liboracle.so) + golden-fixture loaders.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg use this module.
"""
import ctypes as C
import glob
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

_lib = None


def oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(ORACLE_SO)
        P = C.c_void_p
        L.oracle_vp8_decode.argtypes = [P, P, P, P, P, P, C.c_int]
        L.oracle_vp8_reconstruct.argtypes = [P, P, P, P, P]
        L.oracle_yuv_to_rgba_fancy.argtypes = [P, C.c_int, P, P, C.c_int, P, C.c_int, C.c_int, C.c_int]
        L.oracle_yuv_to_rgba_point.argtypes = [P, C.c_int, P, P, C.c_int, P, C.c_int, C.c_int, C.c_int]
        L.oracle_rgba_to_yuva.argtypes = [P, C.c_int, C.c_int, C.c_int, P, C.c_int, P, P, C.c_int, P, C.c_int,
                                          C.c_int]
        L.oracle_transform_block.argtypes = [P, P, C.c_int]
        L.oracle_transform_block.restype = None
        L.oracle_vp8l_decode.argtypes = [P, P, P, P]
        L.oracle_vp8l_resolve.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P]
        L.oracle_alpha_unfilter.argtypes = [C.c_int, C.c_int, C.c_int, P, P]
        L.oracle_anim_compose.argtypes = [P, C.c_int, C.c_int, C.c_int, P, P]
        L.oracle_emit.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]
        _lib = L
    return _lib


def oracle_decode(info, mbs, fancy=True):
    """CPU decode of a parsed frame -> dict(y, u, v, rgba)."""
    w, h = info.width, info.height
    uw, uh = (w + 1) // 2, (h + 1) // 2
    y = np.empty((h, w), np.uint8)
    u = np.empty((uh, uw), np.uint8)
    v = np.empty((uh, uw), np.uint8)
    rgba = np.empty((h, w, 4), np.uint8)
    st = oracle().oracle_vp8_decode(C.addressof(info), mbs.ctypes.data, y.ctypes.data, u.ctypes.data,
                                    v.ctypes.data, rgba.ctypes.data, 1 if fancy else 0)
    assert st == 0
    return dict(y=y, u=u, v=v, rgba=rgba)


def oracle_vp8l_resolve(info, coded):
    """CPU color cache + back-references (the reference's pixel loop) of the tokens from
    webp_amd.vp8l_parse: -> the coded ARGB image, (height, coded_width) uint32."""
    toks = np.ascontiguousarray(coded.tokens, np.uint32)
    lits = np.ascontiguousarray(coded.lits, np.uint32)
    argb = np.empty((info.height, info.coded_width), np.uint32)
    assert oracle().oracle_vp8l_resolve(toks.ctypes.data, lits.ctypes.data, len(lits), argb.size, coded.cache_bits,
                                        argb.ctypes.data) == 0
    return argb


def oracle_vp8l_decode(info, coded, tdata):
    """CPU decode of a lossless frame from webp_amd.vp8l_parse: the color cache and copies
    (oracle_vp8l_resolve), then the inverse transforms + BGRA->RGBA.  `coded` may also be an
    already resolved ARGB array."""
    argb = coded if isinstance(coded, np.ndarray) else oracle_vp8l_resolve(info, coded)
    rgba = np.empty((info.height, info.width, 4), np.uint8)
    ptrs = (C.c_void_p * 4)(*([t.ctypes.data for t in tdata] + [None] * (4 - len(tdata))))
    assert oracle().oracle_vp8l_decode(C.addressof(info), argb.ctypes.data, ptrs, rgba.ctypes.data) == 0
    return rgba


def load_lossless(name):
    with open(os.path.join(GOLDEN, "lossless", name + ".webp"), "rb") as f:
        data = f.read()
    return data, dict(np.load(os.path.join(GOLDEN, "lossless", name + ".npz")))


def lossless_names():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "lossless", "*.webp")))


def oracle_yuv_to_rgba(y, u, v, fancy=True):
    h, w = y.shape
    rgba = np.empty((h, w, 4), np.uint8)
    y = np.ascontiguousarray(y); u = np.ascontiguousarray(u); v = np.ascontiguousarray(v)
    fn = oracle().oracle_yuv_to_rgba_fancy if fancy else oracle().oracle_yuv_to_rgba_point
    fn(y.ctypes.data, y.strides[0], u.ctypes.data, v.ctypes.data, u.strides[0], rgba.ctypes.data, 4 * w, w, h)
    return rgba


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def lossy_cases():
    return sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "lossy", "*.webp")))


def load_lossy(name):
    with open(os.path.join(GOLDEN, "lossy", name + ".webp"), "rb") as f:
        data = f.read()
    return data, dict(np.load(os.path.join(GOLDEN, "lossy", name + ".npz")))


def fuzz_mutants(kind, seed, per_source, n_sources, lo, flips):
    """The mutation fuzz corpus (tests/test_gpu_fuzz.py; libwebp's results for it are committed
    by tests/golden/make_golden.py `fuzz`): for the n_sources smallest fixtures of `kind`
    ('lossy' without the ALPH one, or 'lossless'), per_source copies with 1..flips-1 random bit
    flips at byte positions >= lo.  -> [(key, bytes)] in generation order, key 'src:k'."""
    rng = np.random.default_rng(seed)
    if kind == "lossy":
        names = [n for n in lossy_cases() if n != "alpha_64x48"]
        load = load_lossy
    else:
        names = lossless_names()
        load = load_lossless
    out = []
    for n in sorted(names, key=lambda n: len(load(n)[0]))[:n_sources]:
        d = bytearray(load(n)[0])
        for k in range(per_source):
            m = bytearray(d)
            for _ in range(int(rng.integers(1, flips))):
                pos = int(rng.integers(lo, len(m)))
                m[pos] ^= 1 << int(rng.integers(0, 8))
            out.append((f"{n}:{k}", bytes(m)))
    return out


# (seed, per_source, n_sources, first byte, flips) of the two fuzz corpora
FUZZ_LOSSY = (7, 24, 8, 40, 4)
FUZZ_LOSSLESS = (11, 24, 10, 25, 3)


def bench_files(prefix):
    return sorted(glob.glob(os.path.join(GOLDEN, "bench", prefix + "_s*.webp")))


def oracle_alpha_plane(data):
    """CPU alpha plane of a lossy+ALPH file: host stage (webp_amd.alpha_parse), then for a
    lossless stream the oracle's inverse transforms (alpha = green), then the oracle's
    unfilter.  -> (AlphaInfo, (height, width) uint8)."""
    import webp_amd

    info, payload = webp_amd.alpha_parse(data)
    if info.method == 0:
        filtered = payload
    else:
        ll, coded, tdata = payload
        filtered = np.ascontiguousarray(oracle_vp8l_decode(ll, coded, tdata)[..., 1])
    out = np.empty((info.height, info.width), np.uint8)
    assert oracle().oracle_alpha_unfilter(info.filter, info.width, info.height, filtered.ctypes.data,
                                          out.ctypes.data) == 0
    return info, out


def alpha_names():
    return sorted(manifest().get("alpha", {}))


def load_alpha(name):
    """(bytes, golden dict with 'rgba') of an ALPH fixture."""
    d = os.path.join(GOLDEN, "alpha")
    data = open(os.path.join(d, name + ".webp"), "rb").read()
    return data, dict(np.load(os.path.join(d, name + ".npz")))


def oracle_still_rgba(data):
    """CPU RGBA of a still bitstream (whole file or an animation frame's fragment) with the
    oracles: lossless -> vp8l oracle; lossy -> lossy oracle, A from the ALPH oracle if present."""
    import webp_amd

    if webp_amd.features(data).format == 2:
        info, coded, tdata = webp_amd.vp8l_parse(data)
        return oracle_vp8l_decode(info, coded, tdata)
    info, mbs = webp_amd.vp8_parse(data)
    rgba = oracle_decode(info, mbs)["rgba"]
    try:
        rgba[..., 3] = oracle_alpha_plane(data)[1]
    except webp_amd.WebPError as e:
        if e.status != webp_amd.Status.UNSUPPORTED_FEATURE:
            raise
    return rgba


class _OFrame(C.Structure):
    _fields_ = [("rgba", C.c_void_p), ("x", C.c_int), ("y", C.c_int), ("width", C.c_int), ("height", C.c_int),
                ("duration", C.c_int), ("dispose_bg", C.c_int), ("no_blend", C.c_int), ("has_alpha", C.c_int)]


def oracle_anim(data):
    """CPU animation decode: host demux, oracle decode of every fragment, oracle compositing.
    -> (canvases (F, H, W, 4), timestamps)."""
    import webp_amd

    info, frames = webp_amd.anim_demux(data)
    stills = [np.ascontiguousarray(oracle_still_rgba(data[f.fragment_offset:f.fragment_offset + f.fragment_size]))
              for f in frames]
    of = (_OFrame * len(frames))()
    for o, f, r in zip(of, frames, stills):
        assert r.shape[:2] == (f.height, f.width)
        o.rgba, o.x, o.y, o.width, o.height = r.ctypes.data, f.x_offset, f.y_offset, f.width, f.height
        o.duration, o.dispose_bg, o.no_blend, o.has_alpha = f.duration, f.dispose_background, f.no_blend, f.has_alpha
    canv = np.empty((len(frames), info.canvas_height, info.canvas_width, 4), np.uint8)
    ts = np.empty(len(frames), np.int32)
    assert oracle().oracle_anim_compose(of, len(frames), info.canvas_width, info.canvas_height, canv.ctypes.data,
                                        ts.ctypes.data) == 0
    return canv, ts


def anim_names():
    return sorted(manifest().get("anim", {}))


def load_anim(name):
    d = os.path.join(GOLDEN, "anim")
    data = open(os.path.join(d, name + ".webp"), "rb").read()
    return data, dict(np.load(os.path.join(d, name + ".npz")))


MODE_BPP = {0: 3, 1: 4, 2: 3, 3: 4, 4: 4, 5: 2, 6: 2, 7: 4, 8: 4, 9: 4, 10: 2}


# ----------------------------------------------------------------------------- YUV output modes
def yuv_sources():
    return sorted(manifest().get("yuv", {}))


def load_yuv(src):
    ent = manifest()["yuv"][src]
    data = open(os.path.join(GOLDEN, ent["source"]), "rb").read()
    return data, dict(np.load(os.path.join(GOLDEN, "yuv", src + ".npz"))), ent


def parse_yuv_key(key):
    """'m{mode}_{crop}_f{flip}' -> (mode, crop name, flip)."""
    m, crop, fl = key.split("_")
    return int(m[1:]), crop, int(fl[1:])


def yuv_window(data, crop):
    """The output window WebPDecode uses for a crop (None = the frame): (x, y, w, h), or None when
    libwebp reports INVALID_PARAM.  Lossy origins snap to even (WebPIoInitFromOptions with a YUV
    source), lossless keep theirs; the buffer check uses the snapped origin either way."""
    import webp_amd

    f = webp_amd.features(data)
    W, H = f.width, f.height
    if crop is None:
        return 0, 0, W, H
    cw, ch = crop[2], crop[3]
    x, y = (crop[0], crop[1]) if f.format == 2 else (crop[0] & ~1, crop[1] & ~1)
    ok = lambda a, b: a >= 0 and b >= 0 and cw > 0 and ch > 0 and a + cw <= W and b + ch <= H  # noqa: E731
    return (x, y, cw, ch) if ok(crop[0] & ~1, crop[1] & ~1) and ok(x, y) else None


def oracle_yuva(data, mode, crop=None, flip=0):
    """CPU WebPDecode in MODE_YUV (11) / MODE_YUVA (12) from the oracles -> {"y", "u", "v"[, "a"]},
    or None for an invalid crop.  Lossy: the reconstructed planes' window (EmitYUV, io_dec.c.go:36-50),
    A = the ALPH oracle's plane or 0xff (EmitAlphaYUV :128-150).  Lossless: the RGBA window through
    oracle_rgba_to_yuva (WebPImportYUVAFromRGBA, dsp/yuv.go:304-385)."""
    import webp_amd

    win = yuv_window(data, crop)
    if win is None:
        return None
    x, y, w, h = win
    uw, uh = (w + 1) // 2, (h + 1) // 2
    f = webp_amd.features(data)
    if f.format == 2:
        info, coded, tdata = webp_amd.vp8l_parse(data)
        rgba = np.ascontiguousarray(oracle_vp8l_decode(info, coded, tdata)[y:y + h, x:x + w])
        out = {"y": np.empty((h, w), np.uint8), "u": np.empty((uh, uw), np.uint8), "v": np.empty((uh, uw), np.uint8)}
        a = np.empty((h, w), np.uint8) if mode == 12 else None
        assert oracle().oracle_rgba_to_yuva(rgba.ctypes.data, w, h, 4 * w, out["y"].ctypes.data, w,
                                            out["u"].ctypes.data, out["v"].ctypes.data, uw,
                                            a.ctypes.data if a is not None else None, w, flip) == 0
        if a is not None:
            out["a"] = a
        return out
    info, mbs = webp_amd.vp8_parse(data)
    planes = oracle_decode(info, mbs)
    fl = (lambda p: p[::-1]) if flip else (lambda p: p)  # noqa: E731
    out = {"y": fl(planes["y"][y:y + h, x:x + w]), "u": fl(planes["u"][y // 2:y // 2 + uh, x // 2:x // 2 + uw]),
           "v": fl(planes["v"][y // 2:y // 2 + uh, x // 2:x // 2 + uw])}
    if mode == 12:
        try:
            out["a"] = fl(oracle_alpha_plane(data)[1][y:y + h, x:x + w])
        except webp_amd.WebPError as e:
            if e.status != webp_amd.Status.UNSUPPORTED_FEATURE:
                raise
            out["a"] = np.full((h, w), 255, np.uint8)
    return {k: np.ascontiguousarray(v) for k, v in out.items()}


def oracle_output(data, mode=1, crop=None, flip=0, no_fancy=0, bypass=0):
    """CPU WebPDecode with output options, from the oracles: the RGBA of the output window
    (lossless: a window of the full decode; lossy: the cropped planes upsampled as a standalone
    image, A from the ALPH oracle's window), then the oracle's mode packing / premultiply / flip.
    -> (h, w * bpp) uint8, or None when libwebp reports INVALID_PARAM for the crop."""
    import webp_amd

    f = webp_amd.features(data)
    W, H = f.width, f.height
    x, y, cw, ch = 0, 0, W, H
    if crop is not None:
        # WebPAllocateDecBuffer checks the window with the origin snapped to even; the io window
        # (WebPIoInitFromOptions) snaps only for YUV sources (lossy), lossless keeps odd origins
        ok = lambda a, b: a >= 0 and b >= 0 and cw > 0 and ch > 0 and a + cw <= W and b + ch <= H  # noqa: E731
        cw, ch = crop[2], crop[3]
        x, y = (crop[0], crop[1]) if f.format == 2 else (crop[0] & ~1, crop[1] & ~1)
        if not (ok(crop[0] & ~1, crop[1] & ~1) and ok(x, y)):
            return None
    if f.format == 2:
        info, coded, tdata = webp_amd.vp8l_parse(data)
        rgba = oracle_vp8l_decode(info, coded, tdata)[y:y + ch, x:x + cw]
    else:
        info, mbs = webp_amd.vp8_parse(data, flags=1 if bypass else 0)
        planes = oracle_decode(info, mbs)
        uh, uw = (ch + 1) // 2, (cw + 1) // 2
        rgba = oracle_yuv_to_rgba(np.ascontiguousarray(planes["y"][y:y + ch, x:x + cw]),
                                  np.ascontiguousarray(planes["u"][y // 2:y // 2 + uh, x // 2:x // 2 + uw]),
                                  np.ascontiguousarray(planes["v"][y // 2:y // 2 + uh, x // 2:x // 2 + uw]),
                                  fancy=not no_fancy)
        try:
            rgba[..., 3] = oracle_alpha_plane(data)[1][y:y + ch, x:x + cw]
        except webp_amd.WebPError as e:
            if e.status != webp_amd.Status.UNSUPPORTED_FEATURE:
                raise
    rgba = np.ascontiguousarray(rgba)
    out = np.empty((ch, cw * MODE_BPP[mode]), np.uint8)
    assert oracle().oracle_emit(rgba.ctypes.data, cw, ch, cw * 4, mode, flip, out.ctypes.data, out.shape[1]) == 0
    return out


def mode_sources():
    return sorted(manifest().get("modes", {}))


def load_modes(src):
    ent = manifest()["modes"][src]
    data = open(os.path.join(GOLDEN, ent["source"]), "rb").read()
    return data, dict(np.load(os.path.join(GOLDEN, "modes", src + ".npz"))), ent


def parse_mode_key(key):
    """'m{mode}_{crop}_f{flip}_nf{nf}' -> (mode, crop name, flip, nf)."""
    m, rest = key.split("_", 1)
    crop, fl, nf = rest.rsplit("_", 2)
    return int(m[1:]), crop, int(fl[1:]), int(nf[2:])


# ----------------------------------------------------------------------------- status sweep
def riff_truncate(data, cut):
    """`data` cut to `cut` bytes with a consistent RIFF: the cut chunk's size field and the
    RIFF size rewritten (pad byte added for an odd chunk), so the container parses and the
    truncation reaches the bitstream.  None when the cut falls inside a chunk header."""
    if cut < 20:
        return None
    off = 12
    while off < len(data):
        size = int.from_bytes(data[off + 4:off + 8], "little")
        end = off + 8 + size + (size & 1)
        if cut == off:
            out = bytearray(data[:cut])
            break
        if cut <= off + 8:
            return None
        if cut < end:
            n = cut - off - 8
            out = bytearray(data[:cut])
            out[off + 4:off + 8] = n.to_bytes(4, "little")
            if n & 1:
                out.append(0)
            break
        off = end
    else:
        return None
    out[4:8] = (len(out) - 8).to_bytes(4, "little")
    return bytes(out)


def mutate(data, op, arg):
    """One status-sweep mutant (tests/golden/status/sweep.json): 'none', 'trunc_riff'
    (fraction, riff_truncate), 'trunc' (fraction, raw cut) or 'flip' ([[pos, bit], ...])."""
    if op == "none":
        return data
    if op == "trunc_riff":
        return riff_truncate(data, int(len(data) * arg))
    if op == "trunc":
        return data[:int(len(data) * arg)]
    if op == "flip":
        m = bytearray(data)
        for pos, bit in arg:
            m[pos] ^= 1 << bit
        return bytes(m)
    raise ValueError(op)


def status_sweep():
    with open(os.path.join(GOLDEN, "status", "sweep.json")) as f:
        return json.load(f)


def load_fixture(src):
    """Bytes of tests/golden/<section>/<name>.webp for src = '<section>/<name>'."""
    with open(os.path.join(GOLDEN, src + ".webp"), "rb") as f:
        return f.read()
