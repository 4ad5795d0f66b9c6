"""CPU tests of the C ABI boundary: the library loads, exports every declared symbol,
and its host-only entry points (features / entropy stage) behave like libwebp's."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

import webp_amd
from oracle_lib import GOLDEN, ROOT, load_lossy, lossy_cases, manifest


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "gowebp_amd.h")).read()
    declared = set(re.findall(r"^\w+\s*\*?\s+(wg_[a-z0-9_]+)\s*\(", hdr, re.M))
    L = C.CDLL(webp_amd.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert declared == set(webp_amd.EXPORTED), declared ^ set(webp_amd.EXPORTED)


def test_version():
    assert webp_amd.lib().wg_version() == 0x000100


@pytest.mark.parametrize("kind", ["lossy", "lossless", "bench"])
def test_features_match_manifest(kind):
    m = manifest()[kind]
    for fn, ent in m.items():
        name = fn if fn.endswith(".webp") else fn + ".webp"
        data = open(os.path.join(GOLDEN, kind, name), "rb").read()
        w, h, has_alpha = webp_amd.decode_config(data)
        assert (w, h) == (ent["width"], ent["height"]), fn
        f = webp_amd.features(data)
        assert f.format == (2 if kind == "lossless" or fn.startswith("c5") else 1)
        if "alpha" in fn:
            assert has_alpha


def test_features_error_statuses():
    data, _ = load_lossy("synth_80x96")
    S = webp_amd.Status
    for bad, want in [(b"", S.NOT_ENOUGH_DATA), (data[:11], S.NOT_ENOUGH_DATA),
                      (b"RIFF\x00\x00\x00\x00WEBPVP8 ", S.BITSTREAM_ERROR),
                      (b"RIFX" + data[4:], None), (data[:20], S.NOT_ENOUGH_DATA)]:
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.features(bad)
        if want is not None:
            assert e.value.status == want, (bad[:16], e.value.status)


def test_truncated_frames_fail_in_entropy_stage():
    data, _ = load_lossy("noise_96x64_complex_s0")
    for cut in (30, 200, len(data) // 2, len(data) - 10):
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.vp8_parse(data[:cut])
        assert e.value.status in (webp_amd.Status.NOT_ENOUGH_DATA, webp_amd.Status.BITSTREAM_ERROR)


def test_parse_info_fields():
    m = manifest()["lossy"]
    for name in lossy_cases():
        data, _ = load_lossy(name)
        info, mbs = webp_amd.vp8_parse(data, with_mbs=True)
        hdr = m[name]["header"]
        assert info.mb_w == (info.width + 15) // 16 and info.mb_h == (info.height + 15) // 16
        assert info.num_parts == hdr["partitions"]
        want_ft = 0 if hdr["level"] == 0 else (1 if hdr["simple"] else 2)
        assert info.filter_type == want_ft
        assert info.use_segment == hdr["segments"]
        assert mbs.shape == (info.mb_w * info.mb_h,)
        # f_limit is only set when the frame is filtered (PrecomputeFilterStrengths)
        if want_ft == 0:
            assert (mbs["f_limit"] == 0).all()


def test_no_cpu_fallback_without_gpu():
    """The product decode path fails loudly instead of falling back to a CPU path."""
    if webp_amd.device_count() > 0:
        pytest.skip("GPU present")
    data, _ = load_lossy("synth_17x9")
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.decode(data)
    assert e.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
    with pytest.raises(webp_amd.WebPError):
        webp_amd.Context(0)


def test_yuv_stage_entry_rejects_bad_geometry_before_any_device_call():
    """wg_yuv420_to_rgba_device validates its arguments on the host (no device access, so it
    runs without a GPU): strides below the row sizes, misaligned planes, and an RGBA extent
    beyond the emitter's 32-bit offsets are INVALID_PARAM."""
    p = 1 << 20  # aligned dummy addresses: never dereferenced on these paths
    bad = [
        dict(w=16, h=16, ys=8, uvs=8, rs=64),           # y_stride < width
        dict(w=16, h=16, ys=16, uvs=4, rs=64),          # uv_stride < chroma width
        dict(w=16, h=16, ys=16, uvs=8, rs=32),          # rgba_stride < 4 * width
        dict(w=16, h=16, ys=24, uvs=8, rs=64),          # y_stride not a multiple of 16
        dict(w=4096, h=16383, ys=4096, uvs=2048, rs=1 << 17),  # rgba_stride * height > INT32_MAX
        dict(w=0, h=16, ys=16, uvs=8, rs=64),
    ]
    for a in bad:
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.yuv420_to_rgba_device(p, p, p, a["ys"], a["uvs"], p, a["rs"], a["w"], a["h"], True, None)
        assert e.value.status == webp_amd.Status.INVALID_PARAM, a


def test_resolve_stage_entry_validates_before_any_device_call():
    """wg_vp8l_resolve_device (K7's stage entry) rejects bad arguments on the host, and an empty
    stream is a no-op: none of these touch the device, so they run without a GPU."""
    p = 1 << 20  # aligned dummy addresses: never dereferenced on these paths
    bad = [
        dict(t=0, l=p, nl=1, n=16, cb=4, o=p),            # null tokens
        dict(t=p, l=p, nl=1, n=16, cb=4, o=0),            # null output
        dict(t=p + 4, l=p, nl=1, n=16, cb=4, o=p),        # misaligned tokens
        dict(t=p, l=p, nl=1, n=16, cb=4, o=p + 8),        # misaligned output
        dict(t=p, l=0, nl=1, n=16, cb=4, o=p),            # literals announced, none given
        dict(t=p, l=p, nl=-1, n=16, cb=4, o=p),
        dict(t=p, l=p, nl=1, n=-1, cb=4, o=p),
        dict(t=p, l=p, nl=1, n=16, cb=12, o=p),           # cache_bits > MAX_CACHE_BITS
        dict(t=p, l=p, nl=1, n=16, cb=-1, o=p),
        dict(t=p, l=p, nl=1, n=1 << 29, cb=4, o=p),       # 32-bit byte offsets
    ]
    for a in bad:
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.vp8l_resolve_device(a["t"], a["l"], a["nl"], a["n"], a["cb"], a["o"])
        assert e.value.status == webp_amd.Status.INVALID_PARAM, a
    webp_amd.vp8l_resolve_device(p, 0, 0, 0, 4, p)  # empty: OK, nothing launched


def test_go_shim_calls_only_exported_entry_points():
    """go/webp/decode_amd.go (the cgo binding a maintainer of the reference would add; no Go
    toolchain here to compile it) calls only entry points the header declares and the
    library exports, and guards empty inputs before indexing them."""
    src = open(os.path.join(ROOT, "go", "webp", "decode_amd.go")).read()
    called = set(re.findall(r"\bC\.(wg_[a-z0-9_]+)\s*\(", src))
    assert called >= {"wg_get_features", "wg_decode_rgba_into", "wg_decode_rgba_batch", "wg_decode_rgba_batch_multi",
                      "wg_ctx_create", "wg_ctx_destroy", "wg_set_default_device", "wg_anim_decode"}
    assert called <= set(webp_amd.EXPORTED), called - set(webp_amd.EXPORTED)
    L = C.CDLL(webp_amd.LIB_PATH)
    assert all(hasattr(L, s) for s in called)
    # every `&x[0]` of a caller slice sits behind a length check
    assert "if len(f) > 0" in src and "if len(data) == 0" in src
