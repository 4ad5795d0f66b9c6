"""webp_amd -- Python host binding of the MI355X-native WebP decode path.

Thin ctypes layer over ``libgowebp_amd.so`` (the C ABI in ``include/gowebp_amd.h``).
It mirrors the reference's public decode surface (``decode.go:8-14``):

* :func:`decode_config`  <- ``webp.DecodeConfig(r)``  (WebPGetFeatures, host only)
* :func:`decode`         <- ``webp.Decode(r)``        (GPU decode, RGBA ndarray)

plus the batch API the GPU path is built around (:class:`Context`, :class:`Batch`).
There is deliberately no CPU fallback: if the HIP library or a GPU is missing the
decode calls raise.
"""
import ctypes as C
import os
import weakref

import numpy as np

__all__ = [
    "Status", "WebPError", "FLAG_BYPASS_FILTERING", "FLAG_NO_FANCY_UPSAMPLING", "Features",
    "lib", "features", "decode_config", "decode", "Context", "Batch", "vp8_parse", "vp8l_parse", "MB_DTYPE",
    "VP8Info", "VP8LInfo", "VP8LCoded", "device_count", "yuv420_to_rgba_device", "vp8l_resolve_device", "MultiContext", "set_default_device",
    "pinned_empty", "PipelineStats",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# WG_LIB_VARIANT=timing selects the K1 section-timing build (scripts/k1_sections.py).
LIB_PATH = os.path.join(_HERE, "libgowebp_amd%s.so" % (
    "_" + os.environ["WG_LIB_VARIANT"] if os.environ.get("WG_LIB_VARIANT") else ""))

FLAG_BYPASS_FILTERING = 1
FLAG_NO_FANCY_UPSAMPLING = 2


class Status:
    """VP8StatusCode values (pkg/vp8/enums.go:20-31)."""
    OK = 0
    OUT_OF_MEMORY = 1
    INVALID_PARAM = 2
    BITSTREAM_ERROR = 3
    UNSUPPORTED_FEATURE = 4
    SUSPENDED = 5
    USER_ABORT = 6
    NOT_ENOUGH_DATA = 7
    NAMES = {0: "OK", 1: "OUT_OF_MEMORY", 2: "INVALID_PARAM", 3: "BITSTREAM_ERROR",
             4: "UNSUPPORTED_FEATURE", 5: "SUSPENDED", 6: "USER_ABORT", 7: "NOT_ENOUGH_DATA"}


class WebPError(Exception):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__(f"{what}: {Status.NAMES.get(status, status)}")


class Features(C.Structure):
    """WebPBitstreamFeatures (pkg/libwebp/webp/decode.go:33-41)."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("has_alpha", C.c_int32),
                ("has_animation", C.c_int32), ("format", C.c_int32)]


class VP8Info(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("mb_w", C.c_int32), ("mb_h", C.c_int32),
                ("filter_type", C.c_int32), ("num_parts", C.c_int32), ("use_segment", C.c_int32),
                ("frame_offset", C.c_int32)]


class DecoderOptions(C.Structure):
    """wg_decoder_options (WebPDecoderConfig output colorspace + options subset)."""
    _fields_ = [("colorspace", C.c_int32), ("bypass_filtering", C.c_int32), ("no_fancy_upsampling", C.c_int32),
                ("use_cropping", C.c_int32), ("crop_left", C.c_int32), ("crop_top", C.c_int32),
                ("crop_width", C.c_int32), ("crop_height", C.c_int32), ("use_scaling", C.c_int32),
                ("scaled_width", C.c_int32), ("scaled_height", C.c_int32), ("flip", C.c_int32),
                ("reserved", C.c_int32 * 4)]


def options(colorspace=1, crop=None, flip=0, no_fancy=0, bypass=0, scale=None):
    """DecoderOptions from keywords; crop = (left, top, width, height), scale = (w, h)."""
    o = DecoderOptions()
    o.colorspace, o.flip, o.no_fancy_upsampling, o.bypass_filtering = colorspace, flip, no_fancy, bypass
    if crop is not None:
        o.use_cropping = 1
        o.crop_left, o.crop_top, o.crop_width, o.crop_height = crop
    if scale is not None:
        o.use_scaling = 1
        o.scaled_width, o.scaled_height = scale
    return o


class YUVABuffer(C.Structure):
    """wg_yuva_buffer = WebPYUVABuffer (pkg/libwebp/webp/buffer.go:17-25): caller memory of the
    MODE_YUV / MODE_YUVA planes."""
    _fields_ = [("y", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p), ("a", C.c_void_p),
                ("y_stride", C.c_int32), ("u_stride", C.c_int32), ("v_stride", C.c_int32), ("a_stride", C.c_int32),
                ("y_size", C.c_size_t), ("u_size", C.c_size_t), ("v_size", C.c_size_t), ("a_size", C.c_size_t)]


def _yuva_arrays(w, h, alpha):
    """Contiguous output planes of a w x h window and the YUVABuffer over them."""
    uw, uh = (w + 1) // 2, (h + 1) // 2
    out = {"y": np.empty((h, w), np.uint8), "u": np.empty((uh, uw), np.uint8), "v": np.empty((uh, uw), np.uint8)}
    if alpha:
        out["a"] = np.empty((h, w), np.uint8)
    buf = YUVABuffer()
    for k, arr in out.items():
        setattr(buf, k, arr.ctypes.data)
        setattr(buf, k + "_stride", arr.shape[1])
        setattr(buf, k + "_size", arr.nbytes)
    return out, buf


class AnimInfo(C.Structure):
    """wg_anim_info = WebPAnimInfo."""
    _fields_ = [("canvas_width", C.c_uint32), ("canvas_height", C.c_uint32), ("loop_count", C.c_uint32),
                ("bgcolor", C.c_uint32), ("frame_count", C.c_uint32), ("pad", C.c_uint32 * 4)]


class AnimFrame(C.Structure):
    """wg_anim_frame: one frame as the demux iterator describes it."""
    _fields_ = [("x_offset", C.c_int32), ("y_offset", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("duration", C.c_int32), ("dispose_background", C.c_int32), ("no_blend", C.c_int32),
                ("has_alpha", C.c_int32), ("fragment_offset", C.c_uint64), ("fragment_size", C.c_uint64)]


class AlphaInfo(C.Structure):
    """wg_alpha_info: the ALPH chunk of a lossy frame."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("method", C.c_int32), ("filter", C.c_int32),
                ("pre_processing", C.c_int32), ("reserved", C.c_int32)]


class VP8LInfo(C.Structure):
    """wg_vp8l_info: a lossless frame after the host entropy stage."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("has_alpha", C.c_int32),
                ("coded_width", C.c_int32), ("num_transforms", C.c_int32),
                ("transform_type", C.c_int32 * 4), ("transform_bits", C.c_int32 * 4),
                ("transform_xsize", C.c_int32 * 4), ("transform_size", C.c_int32 * 4),
                ("cache_bits", C.c_int32), ("num_literals", C.c_int32)]


class PipelineStats(C.Structure):
    """wg_pipeline_stats: where the last pipelined decode_batch's time went."""
    _fields_ = [("frames", C.c_int32), ("chunks", C.c_int32), ("host_threads", C.c_int32), ("reserved", C.c_int32),
                ("wall_s", C.c_double), ("parse_s", C.c_double), ("parse_wait_s", C.c_double),
                ("h2d_ms", C.c_double), ("kernel_ms", C.c_double), ("d2h_ms", C.c_double),
                ("h2d_bytes", C.c_double), ("d2h_bytes", C.c_double), ("drain_s", C.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}


class _PinnedBlock:
    """Owner of one wg_host_alloc block (freed with the last array that views it)."""

    def __init__(self, nbytes):
        self.ptr = lib().wg_host_alloc(max(1, nbytes))
        if not self.ptr:
            raise WebPError(Status.OUT_OF_MEMORY, f"wg_host_alloc({nbytes})")
        self.nbytes = nbytes

    def __del__(self):
        try:
            if self.ptr:
                lib().wg_host_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


def pinned_empty(shape, dtype=np.uint8):
    """An uninitialised ndarray in page-locked host memory (wg_host_alloc): decode outputs there
    are written by DMA instead of the HIP runtime's staged copies."""
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dtype.itemsize
    blk = _PinnedBlock(nbytes)
    buf = (C.c_uint8 * max(1, nbytes)).from_address(blk.ptr)
    buf._owner = blk  # the ctypes buffer keeps the block alive; the array keeps the buffer
    return np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)


class VP8LCoded:
    """A lossless image after the host prefix-code walk: one token per coded pixel
    (tokens: (height, coded_width) uint32; bits 31..30 = 0 literal index, 1 color-cache key,
    2 backward distance, 3 unset), the literal ARGB values and the color cache bits.  The
    device (K7) resolves it into the coded ARGB image."""

    def __init__(self, tokens, lits, cache_bits):
        self.tokens, self.lits, self.cache_bits = tokens, lits, cache_bits


# wg_vp8_mb: VP8MBData + VP8FInfo (pkg/vp8/models.go:66-107)
MB_DTYPE = np.dtype([("coeffs", "<i2", (384,)), ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"),
                     ("is_i4x4", "u1"), ("uvmode", "u1"), ("segment", "u1"), ("skip", "u1"),
                     ("imodes", "u1", (16,)), ("f_limit", "u1"), ("f_ilevel", "u1"), ("f_inner", "u1"),
                     ("hev_thresh", "u1")])
assert MB_DTYPE.itemsize == 800

_lib = None

_P = C.c_void_p
_SIGS = {
    "wg_version": (C.c_int, []),
    "wg_device_count": (C.c_int, []),
    "wg_get_features": (C.c_int, [_P, C.c_size_t, C.POINTER(Features)]),
    "wg_decode_rgba_into": (C.c_int, [_P, C.c_size_t, _P, C.c_size_t, C.c_int, C.c_int]),
    "wg_ctx_create": (_P, [C.c_int, C.c_int]),
    "wg_ctx_destroy": (None, [_P]),
    "wg_decode_rgba_batch": (C.c_int, [_P, _P, _P, C.c_int, _P, _P, _P, _P, C.c_int32]),
    "wg_batch_create": (_P, [_P, _P, _P, C.c_int, C.c_int32, _P]),
    "wg_batch_destroy": (None, [_P]),
    "wg_batch_run": (C.c_int, [_P, _P]),
    "wg_batch_set_emit": (C.c_int, [_P, C.c_int]),
    "wg_batch_run_emit": (C.c_int, [_P, _P]),
    "wg_batch_kernel_ms": (C.c_int, [_P, _P, C.c_int]),
    "wg_batch_kernel_bytes": (C.c_int, [_P, _P, C.c_int]),
    "wg_batch_size": (C.c_int, [_P]),
    "wg_batch_frame_dims": (C.c_int, [_P, C.c_int, _P, _P]),
    "wg_batch_pixels": (C.c_int64, [_P]),
    "wg_batch_download_rgba": (C.c_int, [_P, C.c_int, _P, C.c_int]),
    "wg_batch_download_yuv": (C.c_int, [_P, C.c_int, _P, _P, _P]),
    "wg_yuv420_to_rgba_device": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int,
                                           C.c_int, _P]),
    "wg_vp8_parse": (C.c_int, [_P, C.c_size_t, C.c_int, C.POINTER(VP8Info), _P]),
    "wg_vp8l_parse": (C.c_int, [_P, C.c_size_t, C.POINTER(VP8LInfo), _P, _P, _P]),
    "wg_alpha_parse": (C.c_int, [_P, C.c_size_t, _P, _P, _P, _P, _P, _P]),
    "wg_anim_demux": (C.c_int, [_P, C.c_size_t, _P, _P, C.c_int]),
    "wg_output_bpp": (C.c_int, [C.c_int]),
    "wg_decode_into": (C.c_int, [_P, C.c_size_t, _P, _P, C.c_size_t, C.c_int]),
    "wg_decode_batch": (C.c_int, [_P, _P, _P, C.c_int, _P, _P, _P, _P, _P]),
    "wg_batch_create_ex": (_P, [_P, _P, _P, C.c_int, _P, _P]),
    "wg_batch_download": (C.c_int, [_P, C.c_int, _P, C.c_int]),
    "wg_batch_frame_status": (C.c_int, [_P, C.c_int]),
    "wg_anim_decode": (C.c_int, [_P, _P, C.c_size_t, _P, _P, C.c_int32]),
    "wg_decode_status": (C.c_int, [_P, C.c_size_t, _P]),
    "wg_set_default_device": (C.c_int, [C.c_int]),
    "wg_vp8l_resolve_device": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "wg_decode_rgba_batch_multi": (C.c_int, [_P, C.c_int, _P, _P, C.c_int, _P, _P, _P, _P, C.c_int32]),
    "wg_ctx_set_chunk_frames": (C.c_int, [_P, C.c_int]),
    "wg_ctx_pipeline_stats": (C.c_int, [_P, _P]),
    "wg_host_alloc": (_P, [C.c_size_t]),
    "wg_host_free": (None, [_P]),
    "wg_batch_set_k1_parts": (C.c_int, [_P, C.c_int]),
    "wg_anim_batch_create": (_P, [_P, _P, C.c_size_t, C.c_int32, _P]),
    "wg_anim_batch_info": (C.c_int, [_P, _P, _P, _P]),
    "wg_anim_batch_download": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "wg_debug_set_epoch": (C.c_uint32, [C.c_uint32]),
    "wg_decode_yuv_into": (C.c_int, [_P, C.c_size_t, _P, _P]),
    "wg_decode_yuv_batch": (C.c_int, [_P, _P, _P, C.c_int, _P, _P, _P]),
    "wg_batch_download_yuva": (C.c_int, [_P, C.c_int, _P]),
}
EXPORTED = tuple(_SIGS)


def _bind_torch_runtime():
    """If torch (ROCm wheel) is installed, import it BEFORE loading our library.

    The wheel bundles its own libamdhip64 (SONAME libamdhip64.so.7).  Loaded first, it
    satisfies our library's DT_NEEDED, so the process has ONE HIP/HSA runtime and device
    pointers / streams can be shared with torch.  Loaded after /opt/rocm's copy, torch
    would bring up a second runtime (and fail to see the GPU)."""
    try:
        import importlib.util
        if importlib.util.find_spec("torch") is not None:
            import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libgowebp_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        _bind_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C go-webp_amd/csrc` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("WG_LIB_VARIANT") and not hasattr(L, name):
                continue  # measurement variants built from older sources (A/B runs)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _buf(data):
    if isinstance(data, np.ndarray):
        data = data.tobytes()
    return bytes(data)


def device_count():
    return lib().wg_device_count()


def set_default_device(device):
    """Device of the context behind decode() / decode_into() (wg_set_default_device)."""
    st = lib().wg_set_default_device(device)
    if st != Status.OK:
        raise WebPError(st, f"wg_set_default_device({device})")


def features(data):
    f = Features()
    b = _buf(data)
    st = lib().wg_get_features(b, len(b), C.byref(f))
    if st != Status.OK:
        raise WebPError(st, "wg_get_features")
    return f


def output_bpp(colorspace):
    return lib().wg_output_bpp(colorspace)


def decode_into(data, opts):
    """Mirror of WebPDecode with output options: one frame -> (h, w * bpp) uint8 rows in the
    options' colorspace / crop window / orientation."""
    b = _buf(data)
    f = features(b)
    bpp = output_bpp(opts.colorspace) or 4
    w, h = (opts.crop_width, opts.crop_height) if opts.use_cropping else (f.width, f.height)
    out = np.empty((max(h, 1), max(w, 1) * bpp), np.uint8)
    st = lib().wg_decode_into(b, len(b), C.byref(opts), out.ctypes.data, out.nbytes, out.shape[1])
    if st != Status.OK:
        raise WebPError(st, "wg_decode_into")
    return out


def decode_yuv(data, opts=None):
    """Mirror of WebPDecodeYUV / WebPDecode in MODE_YUV (11) or MODE_YUVA (12) (opts.colorspace;
    default MODE_YUV, no crop): one frame -> {"y", "u", "v"[, "a"]} planes of the output window."""
    if opts is None:
        opts = options(11)
    b = _buf(data)
    f = features(b)
    w, h = (opts.crop_width, opts.crop_height) if opts.use_cropping else (f.width, f.height)
    out, buf = _yuva_arrays(max(w, 1), max(h, 1), opts.colorspace == 12)
    st = lib().wg_decode_yuv_into(b, len(b), C.byref(opts), C.byref(buf))
    if st != Status.OK:
        raise WebPError(st, "wg_decode_yuv_into")
    return out


def decode_config(data):
    """Mirror of webp.DecodeConfig: returns (width, height, has_alpha)."""
    f = features(data)
    return f.width, f.height, bool(f.has_alpha)


def decode(data, flags=0):
    """Mirror of webp.Decode: GPU decode of one frame to an HxWx4 uint8 RGBA array."""
    b = _buf(data)
    f = features(b)
    out = np.empty((f.height, f.width, 4), np.uint8)
    st = lib().wg_decode_rgba_into(b, len(b), out.ctypes.data, out.nbytes, 4 * f.width, flags)
    if st != Status.OK:
        raise WebPError(st, "wg_decode_rgba_into")
    return out


def decode_status(data, opts=None):
    """WebPDecode's status for `data` under DecoderOptions `opts` (None = RGBA), host only."""
    b = bytes(data)
    return lib().wg_decode_status(b, len(b), C.byref(opts) if opts is not None else None)


def vp8_parse(data, flags=0, with_mbs=True):
    """Host entropy stage only: (VP8Info, structured ndarray of MB_DTYPE or None)."""
    b = _buf(data)
    info = VP8Info()
    L = lib()
    st = L.wg_vp8_parse(b, len(b), flags, C.byref(info), None)
    if st != Status.OK:
        raise WebPError(st, "wg_vp8_parse")
    if not with_mbs:
        return info, None
    mbs = np.zeros(info.mb_w * info.mb_h, MB_DTYPE)
    st = L.wg_vp8_parse(b, len(b), flags, C.byref(info), mbs.ctypes.data)
    if st != Status.OK:
        raise WebPError(st, "wg_vp8_parse")
    return info, mbs


def _vp8l_outputs(info):
    tokens = np.zeros((info.height, info.coded_width), np.uint32)
    lits = np.zeros(max(1, info.num_literals), np.uint32)
    tdata = [np.zeros(max(1, info.transform_size[i]), np.uint32) for i in range(info.num_transforms)]
    ptrs = (C.c_void_p * 4)(*([t.ctypes.data for t in tdata] + [None] * (4 - len(tdata))))
    return tokens, lits, tdata, ptrs


def vp8l_parse(data):
    """Host entropy stage of a lossless file: (VP8LInfo, VP8LCoded, [transform data arrays
    in read order])."""
    b = _buf(data)
    info = VP8LInfo()
    L = lib()
    st = L.wg_vp8l_parse(b, len(b), C.byref(info), None, None, None)
    if st != Status.OK:
        raise WebPError(st, "wg_vp8l_parse")
    tokens, lits, tdata, ptrs = _vp8l_outputs(info)
    st = L.wg_vp8l_parse(b, len(b), C.byref(info), tokens.ctypes.data, lits.ctypes.data, ptrs)
    if st != Status.OK:
        raise WebPError(st, "wg_vp8l_parse")
    return info, VP8LCoded(tokens, lits[:info.num_literals], info.cache_bits), tdata


def alpha_parse(data):
    """Host stage of the ALPH chunk of a lossy file: (AlphaInfo, payload) with payload the
    (height, width) filtered bytes for method 0, or (VP8LInfo, VP8LCoded, tdata) of the alpha
    stream (as vp8l_parse returns them) for method 1."""
    b = _buf(data)
    info = AlphaInfo()
    ll = VP8LInfo()
    L = lib()
    st = L.wg_alpha_parse(b, len(b), C.byref(info), None, C.byref(ll), None, None, None)
    if st != Status.OK:
        raise WebPError(st, "wg_alpha_parse")
    if info.method == 0:
        filt = np.zeros((info.height, info.width), np.uint8)
        st = L.wg_alpha_parse(b, len(b), C.byref(info), filt.ctypes.data, None, None, None, None)
        if st != Status.OK:
            raise WebPError(st, "wg_alpha_parse")
        return info, filt
    tokens, lits, tdata, ptrs = _vp8l_outputs(ll)
    st = L.wg_alpha_parse(b, len(b), C.byref(info), None, C.byref(ll), tokens.ctypes.data, lits.ctypes.data, ptrs)
    if st != Status.OK:
        raise WebPError(st, "wg_alpha_parse")
    return info, (ll, VP8LCoded(tokens, lits[:ll.num_literals], ll.cache_bits), tdata)


def anim_demux(data):
    """Host demux (WebPDemux + frame iterator): (AnimInfo, [AnimFrame]); a still image is one
    frame.  frame.fragment_offset / fragment_size delimit its standalone bitstream."""
    b = _buf(data)
    info = AnimInfo()
    L = lib()
    st = L.wg_anim_demux(b, len(b), C.byref(info), None, 0)
    if st != Status.OK:
        raise WebPError(st, "wg_anim_demux")
    frames = (AnimFrame * max(1, info.frame_count))()
    st = L.wg_anim_demux(b, len(b), C.byref(info), frames, info.frame_count)
    if st != Status.OK:
        raise WebPError(st, "wg_anim_demux")
    return info, list(frames)[:info.frame_count]


def _ptr_arrays(datas):
    bufs = [_buf(d) for d in datas]
    n = len(bufs)
    ptrs = (C.c_void_p * n)(*[C.cast(C.c_char_p(b), C.c_void_p).value for b in bufs])
    sizes = (C.c_size_t * n)(*[len(b) for b in bufs])
    return bufs, ptrs, sizes


class Batch:
    """Device-resident batch: host parse + H2D once, then run() the device path many times."""

    def __init__(self, ctx, datas, flags=0, opts=None):
        """opts: DecoderOptions (wg_batch_create_ex: colorspace, crop, flip; a non-RGBA colorspace or
        flip adds K6 to every run) instead of flags."""
        self._ctx = ctx  # keep the context alive while the batch exists
        self._h = None
        self._bufs, ptrs, sizes = _ptr_arrays(datas)
        n = len(self._bufs)
        self.status = np.zeros(n, np.int32)
        self.opts = opts
        if opts is not None:
            self._h = lib().wg_batch_create_ex(ctx._h, ptrs, sizes, n, C.byref(opts), self.status.ctypes.data)
        else:
            self._h = lib().wg_batch_create(ctx._h, ptrs, sizes, n, flags, self.status.ctypes.data)
        if not self._h:
            raise WebPError(int(self.status.max() or Status.OUT_OF_MEMORY), "wg_batch_create")
        self.n = n
        self.flags = flags
        ctx._batches.add(self)

    def run(self, stream=None):
        st = lib().wg_batch_run(self._h, stream)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_run")

    def set_emit(self, separate):
        """separate=False (default for uncropped batches): K1 emits the lossy RGBA in its
        tail; True: K1 writes the planes and a K2 launch converts them."""
        st = lib().wg_batch_set_emit(self._h, 1 if separate else 0)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_set_emit")

    def set_k1_parts(self, parts):
        """K1 workgroups per frame: 1 (the kernels with the RGBA tail), 2..4 (the split kernel;
        K2 converts), 0 (automatic: split for batches of fewer frames than CUs)."""
        st = lib().wg_batch_set_k1_parts(self._h, parts)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_set_k1_parts")

    def run_emit(self, stream=None):
        """The YUV420->RGBA stage alone (K2) over the planes of the last run."""
        st = lib().wg_batch_run_emit(self._h, stream)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_run_emit")

    def kernel_ms(self):
        """(K1, K2, K3, K4, K7, K6, K5) per-launch ms averaged over the runs since the last call."""
        ms = (C.c_float * 7)()
        st = lib().wg_batch_kernel_ms(self._h, ms, 7)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_kernel_ms")
        return tuple(float(v) for v in ms)

    def kernel_bytes(self):
        """Algorithmic HBM bytes per launch of (K1, K2, K3, K4, K7, K6, K5)."""
        b = (C.c_double * 7)()
        lib().wg_batch_kernel_bytes(self._h, b, 7)
        return tuple(float(v) for v in b)

    @property
    def pixels(self):
        return int(lib().wg_batch_pixels(self._h))

    def dims(self, i):
        w, h = C.c_int32(), C.c_int32()
        st = lib().wg_batch_frame_dims(self._h, i, C.byref(w), C.byref(h))
        if st != Status.OK:
            raise WebPError(st, "wg_batch_frame_dims")
        return w.value, h.value

    def rgba(self, i):
        w, h = self.dims(i)
        out = np.empty((h, w, 4), np.uint8)
        st = lib().wg_batch_download_rgba(self._h, i, out.ctypes.data, 4 * w)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_download_rgba")
        return out

    def download(self, i):
        """Frame i in the batch's output colorspace: (h, w * bpp) uint8 rows (wg_batch_download)."""
        w, h = self.dims(i)
        bpp = output_bpp(self.opts.colorspace) if self.opts is not None else 4
        out = np.empty((h, w * bpp), np.uint8)
        st = lib().wg_batch_download(self._h, i, out.ctypes.data, w * bpp)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_download")
        return out

    def yuv(self, i):
        w, h = self.dims(i)
        y = np.empty((h, w), np.uint8)
        u = np.empty(((h + 1) // 2, (w + 1) // 2), np.uint8)
        v = np.empty_like(u)
        st = lib().wg_batch_download_yuv(self._h, i, y.ctypes.data, u.ctypes.data, v.ctypes.data)
        if st != Status.OK:
            raise WebPError(st, "wg_batch_download_yuv")
        return y, u, v

    def yuva(self, i):
        """Frame i's MODE_YUV / MODE_YUVA planes of a batch created with colorspace 11 / 12
        (wg_batch_download_yuva): {"y", "u", "v"[, "a"]}."""
        w, h = self.dims(i)
        out, buf = _yuva_arrays(w, h, self.opts is not None and self.opts.colorspace == 12)
        st = lib().wg_batch_download_yuva(self._h, i, C.byref(buf))
        if st != Status.OK:
            raise WebPError(st, "wg_batch_download_yuva")
        return out

    def close(self):
        if self._h:
            lib().wg_batch_destroy(self._h)
            self._h = None
            self._ctx._batches.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AnimBatch(Batch):
    """An animation resident in HBM (wg_anim_batch_create): run() decodes every frame (K1..K4) and
    composites every canvas (K5); canvases() downloads them with the end timestamps."""

    def __init__(self, ctx, data, flags=0):
        self._ctx = ctx
        self._h = None
        self._bufs = [_buf(data)]
        st = C.c_int32(0)
        self._h = lib().wg_anim_batch_create(ctx._h, self._bufs[0], len(self._bufs[0]), flags, C.byref(st))
        if not self._h:
            raise WebPError(st.value or Status.OUT_OF_MEMORY, "wg_anim_batch_create")
        w, h, n = C.c_int32(), C.c_int32(), C.c_int32()
        lib().wg_anim_batch_info(self._h, C.byref(w), C.byref(h), C.byref(n))
        self.canvas_width, self.canvas_height, self.n = w.value, h.value, n.value
        self.status = np.zeros(self.n, np.int32)
        self.opts = None
        self.flags = flags
        ctx._batches.add(self)

    def canvases(self):
        """((frames, H, W, 4) uint8 canvases of the last run, (frames,) int32 end timestamps in ms)."""
        canv = np.empty((self.n, self.canvas_height, self.canvas_width, 4), np.uint8)
        ts = np.empty(self.n, np.int32)
        st = lib().wg_anim_batch_download(self._h, canv.ctypes.data, canv.nbytes, ts.ctypes.data)
        if st != Status.OK:
            raise WebPError(st, "wg_anim_batch_download")
        return canv, ts


class Context:
    """One decode context per HIP device (wg_ctx)."""

    def __init__(self, device=0, host_threads=0):
        self._batches = weakref.WeakSet()
        self._h = lib().wg_ctx_create(device, host_threads)
        if not self._h:
            raise WebPError(Status.UNSUPPORTED_FEATURE, f"wg_ctx_create(device={device}) (no GPU?)")
        self.device = device

    def batch(self, datas, flags=0, opts=None):
        return Batch(self, datas, flags, opts)

    def anim_batch(self, data, flags=0):
        return AnimBatch(self, data, flags)

    def decode_batch_opts(self, datas, opts):
        """wg_decode_batch: frames -> ([(h, w * bpp) uint8 rows or None], status)."""
        bufs, ptrs, sizes = _ptr_arrays(datas)
        n = len(bufs)
        bpp = output_bpp(opts.colorspace) or 4
        outs = []
        for b in bufs:
            try:
                f = features(b)
                w, h = (opts.crop_width, opts.crop_height) if opts.use_cropping else (f.width, f.height)
            except WebPError:
                w = h = 1
            outs.append(np.zeros((max(h, 1), max(w, 1) * bpp), np.uint8))
        optr = (C.c_void_p * n)(*[o.ctypes.data for o in outs])
        strides = (C.c_int32 * n)(*[o.shape[1] for o in outs])
        caps = (C.c_size_t * n)(*[o.nbytes for o in outs])
        status = np.zeros(n, np.int32)
        st = lib().wg_decode_batch(self._h, ptrs, sizes, n, C.byref(opts), optr, strides, caps, status.ctypes.data)
        if st != Status.OK:
            raise WebPError(st, "wg_decode_batch")
        return [o if s == 0 else None for o, s in zip(outs, status)], status

    def decode_yuv_batch(self, datas, opts):
        """wg_decode_yuv_batch (opts.colorspace 11 / 12): frames -> ([{"y", "u", "v"[, "a"]} or None],
        status)."""
        bufs, ptrs, sizes = _ptr_arrays(datas)
        n = len(bufs)
        outs, yb = [], (YUVABuffer * n)()
        for i, b in enumerate(bufs):
            try:
                f = features(b)
                w, h = (opts.crop_width, opts.crop_height) if opts.use_cropping else (f.width, f.height)
            except WebPError:
                w = h = 1
            o, yb[i] = _yuva_arrays(max(w, 1), max(h, 1), opts.colorspace == 12)
            outs.append(o)
        status = np.zeros(n, np.int32)
        st = lib().wg_decode_yuv_batch(self._h, ptrs, sizes, n, C.byref(opts), yb, status.ctypes.data)
        if st != Status.OK:
            raise WebPError(st, "wg_decode_yuv_batch")
        return [o if s == 0 else None for o, s in zip(outs, status)], status

    def decode_anim(self, data, flags=0):
        """Whole animation -> (canvases (frames, H, W, 4) uint8 RGBA, timestamps int32 ms), as
        the WebPAnimDecoderGetNext loop returns them."""
        info, _ = anim_demux(data)
        b = _buf(data)
        canv = np.empty((info.frame_count, info.canvas_height, info.canvas_width, 4), np.uint8)
        ts = np.empty(info.frame_count, np.int32)
        st = lib().wg_anim_decode(self._h, b, len(b), canv.ctypes.data, ts.ctypes.data, flags)
        if st != Status.OK:
            raise WebPError(st, "wg_anim_decode")
        return canv, ts

    def set_chunk_frames(self, frames):
        """Frames per pipeline chunk of decode_batch (0 = automatic)."""
        st = lib().wg_ctx_set_chunk_frames(self._h, frames)
        if st != Status.OK:
            raise WebPError(st, "wg_ctx_set_chunk_frames")

    def pipeline_stats(self):
        """PipelineStats of the last decode_batch (wg_ctx_pipeline_stats)."""
        ps = PipelineStats()
        st = lib().wg_ctx_pipeline_stats(self._h, C.byref(ps))
        if st != Status.OK:
            raise WebPError(st, "wg_ctx_pipeline_stats")
        return ps

    def decode_batch(self, datas, flags=0, out=None):
        """Decode a list of WebP files; returns (list of RGBA arrays or None, status array).
        `out`: optional preallocated (H, W, 4) uint8 arrays, one per input (pinned_empty()
        arrays are written by DMA).  Pipelined in chunks (wg_decode_rgba_batch)."""
        bufs, ptrs, sizes = _ptr_arrays(datas)
        n = len(bufs)
        outs, optr, strides, caps = _rgba_outs(bufs, out)
        status = np.zeros(n, np.int32)
        st = lib().wg_decode_rgba_batch(self._h, ptrs, sizes, n, optr, strides, caps, status.ctypes.data, flags)
        if st != Status.OK:
            raise WebPError(st, "wg_decode_rgba_batch")
        return [o if s == Status.OK else None for o, s in zip(outs, status)], status

    def close(self):
        for b in list(self._batches):
            b.close()
        if self._h:
            lib().wg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _rgba_outs(bufs, out):
    n = len(bufs)
    outs, optr, strides, caps = [], (C.c_void_p * n)(), (C.c_int32 * n)(), (C.c_size_t * n)()
    for i, b in enumerate(bufs):
        if out is not None:
            a = out[i]
            if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 4 or not a.flags.c_contiguous:
                raise ValueError("out arrays must be C-contiguous (H, W, 4) uint8")
        else:
            try:
                f = features(b)
                a = np.empty((f.height, f.width, 4), np.uint8)
            except WebPError:
                a = np.empty((1, 1, 4), np.uint8)
        outs.append(a)
        optr[i] = a.ctypes.data
        strides[i] = a.shape[1] * 4
        caps[i] = a.nbytes  # the C side checks every frame's window against it
    return outs, optr, strides, caps


class MultiContext:
    """Frames sharded over several decode contexts: one Context per entry of
    `devices` (a device may repeat: independent contexts on one GPU), decode_batch() splits the
    list into contiguous shards decoded concurrently (wg_decode_rgba_batch_multi)."""

    def __init__(self, devices, host_threads=0):
        self.contexts = [Context(d, host_threads) for d in devices]

    def decode_batch(self, datas, flags=0, out=None):
        """Same contract as Context.decode_batch: (list of RGBA arrays or None, status)."""
        bufs, ptrs, sizes = _ptr_arrays(datas)
        n = len(bufs)
        outs, optr, strides, caps = _rgba_outs(bufs, out)
        status = np.zeros(n, np.int32)
        hs = (C.c_void_p * len(self.contexts))(*[c._h for c in self.contexts])
        st = lib().wg_decode_rgba_batch_multi(hs, len(self.contexts), ptrs, sizes, n, optr, strides, caps,
                                              status.ctypes.data, flags)
        if st != Status.OK:
            raise WebPError(st, "wg_decode_rgba_batch_multi")
        return [o if s == Status.OK else None for o, s in zip(outs, status)], status

    def close(self):
        for c in self.contexts:
            c.close()


def yuv420_to_rgba_device(y_ptr, u_ptr, v_ptr, y_stride, uv_stride, rgba_ptr, rgba_stride, width, height,
                          fancy=True, stream=None):
    """Stage entry point on device pointers (ints), e.g. torch tensors' data_ptr()."""
    st = lib().wg_yuv420_to_rgba_device(y_ptr, u_ptr, v_ptr, y_stride, uv_stride, rgba_ptr, rgba_stride,
                                        width, height, 1 if fancy else 0, stream)
    if st != Status.OK:
        raise WebPError(st, "wg_yuv420_to_rgba_device")


def vp8l_resolve_device(tokens_ptr, lits_ptr, n_lits, n_px, cache_bits, argb_ptr, stream=None):
    """Stage entry point on device pointers (ints): the color cache + back-references of one
    VP8L token stream (the tokens of webp_amd.vp8l_parse's VP8LCoded) -> n_px coded ARGB words."""
    st = lib().wg_vp8l_resolve_device(tokens_ptr, lits_ptr, n_lits, n_px, cache_bits, argb_ptr, stream)
    if st != Status.OK:
        raise WebPError(st, "wg_vp8l_resolve_device")
