"""GPU parity of the output stage: colorspaces, cropping and flip through
wg_decode_batch / wg_decode_into, against libwebp 1.6.0's WebPDecode bytes.  Bit-exact."""
import numpy as np
import pytest

import webp_amd
from oracle_lib import load_modes, mode_sources, parse_mode_key

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    c = webp_amd.Context(0)
    yield c
    c.close()


def test_modes_crops_flip_batches_vs_libwebp(ctx):
    srcs = [load_modes(s) for s in mode_sources()]
    keys = sorted({k for _, _, ent in srcs for k in ent["status"]})
    checked = 0
    for key in keys:
        mode, cname, flip, nf = parse_mode_key(key)
        group = [(d, g, e) for d, g, e in srcs if key in e["status"]]
        crops = {tuple(e["crops"][cname]) if e["crops"][cname] else None for _, _, e in group}
        for crop in crops:  # sources share a crop window unless it depends on the frame size
            sub = [(d, g, e) for d, g, e in group if (tuple(e["crops"][cname]) if e["crops"][cname] else None) == crop]
            opts = webp_amd.options(mode, crop, flip, nf)
            outs, status = ctx.decode_batch_opts([d for d, _, _ in sub], opts)
            for (d, g, e), out, st in zip(sub, outs, status):
                assert st == e["status"][key], (key, e["source"], st)
                if st == 0 and key in g:
                    np.testing.assert_array_equal(out, g[key], err_msg=f"{key} {e['source']}")
                    checked += 1
    assert checked > 500


def test_single_frame_decode_into():
    data, gold, _ = load_modes("alpha_64x48")
    for key in ("m7_c1_f1_nf0", "m10_none_f0_nf0", "m6_c4_f0_nf0", "m0_none_f1_nf1"):
        mode, cname, flip, nf = parse_mode_key(key)
        out = webp_amd.decode_into(data, webp_amd.options(mode, load_modes("alpha_64x48")[2]["crops"][cname], flip, nf))
        np.testing.assert_array_equal(out, gold[key], err_msg=key)


def test_unsupported_and_invalid_options(ctx):
    data, _, _ = load_modes("synth_80x96")
    for opts, want in ((webp_amd.options(13), webp_amd.Status.INVALID_PARAM),
                       (webp_amd.options(1, scale=(40, 48)), webp_amd.Status.UNSUPPORTED_FEATURE),
                       (webp_amd.options(1, crop=(0, 0, 0, 5)), webp_amd.Status.INVALID_PARAM)):
        _, status = ctx.decode_batch_opts([data], opts)
        assert status[0] == want


def test_cropped_batch_keeps_separate_emit(ctx):
    """A batch with a crop window converts through K2 (the window is upsampled as a standalone
    image): wg_batch_set_emit refuses to switch it to K1's tail; separate stays accepted."""
    import ctypes as C
    from oracle_lib import load_lossy
    d, _ = load_lossy("synth_481x270")
    bufs, ptrs, sizes = webp_amd._ptr_arrays([d])
    st = np.zeros(1, np.int32)
    opt = webp_amd.options(crop=(10, 12, 64, 40))
    L = webp_amd.lib()
    h = L.wg_batch_create_ex(ctx._h, ptrs, sizes, 1, C.byref(opt), st.ctypes.data)
    assert h and st[0] == 0, st
    try:
        assert L.wg_batch_set_emit(h, 0) == webp_amd.Status.INVALID_PARAM
        assert L.wg_batch_set_emit(h, 1) == webp_amd.Status.OK
        assert L.wg_batch_run(h, None) == webp_amd.Status.OK
        ms = (C.c_float * 4)()
        assert L.wg_batch_kernel_ms(h, ms, 4) == webp_amd.Status.OK
        assert ms[0] > 0 and ms[1] > 0, list(ms)  # K1 planes + K2 on the crop window
    finally:
        L.wg_batch_destroy(h)
    assert L.wg_batch_set_emit(None, 0) == webp_amd.Status.INVALID_PARAM


@pytest.mark.parametrize("key", ["m0_none_f1_nf0", "m7_none_f0_nf0", "m4_none_f0_nf1", "m1_none_f1_nf0"])
def test_resident_batch_runs_k6_as_a_stage(ctx, key):
    """A batch created with an output colorspace (or flip) runs K6 as the last stage of every
    wg_batch_run (its own kernel_ms entry) over the frames the YUV -> RGB strips do not emit
    directly (lossless frames and frames with alpha); downloads copy its output: equal to
    WebPDecode's bytes after repeated runs (RGB flipped, rgbA premultiplied, ARGB point-sampled,
    RGBA flipped).  The directly emitted frames have no RGBA copy (UNSUPPORTED_FEATURE)."""
    mode, cname, flip, nf = parse_mode_key(key)
    srcs = [load_modes(s) for s in mode_sources()]
    sub = [(d, g) for d, g, e in srcs if e["status"].get(key) == 0 and key in g]
    assert len(sub) >= 3
    b = ctx.batch([d for d, _ in sub], opts=webp_amd.options(mode, None, flip, nf))
    try:
        for _ in range(2):
            b.run()
        ms = b.kernel_ms()
        assert ms[5] > 0, ms
        by = b.kernel_bytes()
        bpp = webp_amd.output_bpp(mode)
        direct = [webp_amd.features(d).format != 2 and not webp_amd.features(d).has_alpha for d, _ in sub]
        assert any(direct) and not all(direct)
        assert by[5] == sum((4 + bpp) * g[key].shape[0] * g[key].shape[1] // bpp
                            for (_, g), dr in zip(sub, direct) if not dr)
        for i, (_, g) in enumerate(sub):
            np.testing.assert_array_equal(b.download(i), g[key], err_msg=f"{key} frame {i}")
            if direct[i]:  # (written in the batch's mode only: no RGBA copy to download)
                with pytest.raises(webp_amd.WebPError) as ei:
                    b.rgba(i)
                assert ei.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
    finally:
        b.close()


def _modes_from_rgba(rgba, mode, flip):
    """WebPDecode's bytes of an opaque frame in `mode` from its RGBA (emit_px.h's packings; the
    premultiplied modes equal the plain ones at a = 255)."""
    r, g, b, a = (rgba[..., c].astype(np.uint32) for c in range(4))
    m = {7: 1, 8: 3, 9: 4, 10: 5}.get(mode, mode)
    if m == 0:
        out = np.stack([r, g, b], -1)
    elif m == 1:
        out = np.stack([r, g, b, a], -1)
    elif m == 2:
        out = np.stack([b, g, r], -1)
    elif m == 3:
        out = np.stack([b, g, r, a], -1)
    elif m == 4:
        out = np.stack([a, r, g, b], -1)
    elif m == 5:
        out = np.stack([(r & 0xf0) | (g >> 4), (b & 0xf0) | (a >> 4)], -1)
    else:
        out = np.stack([(r & 0xf8) | (g >> 5), ((g << 3) & 0xe0) | (b >> 3)], -1)
    out = out.astype(np.uint8).reshape(rgba.shape[0], -1)
    return out[::-1] if flip else out


@pytest.mark.parametrize("emit", ["auto", "tail"])
def test_direct_emission_every_mode_4k(ctx, emit):
    """Lossy 4K frames without alpha emitted straight into every output colorspace, flipped or
    not: by K2 (a 3-frame batch runs the split K1, K2 converts) or by K1's tail (set_emit(False):
    RGBA / rgbA / RGB_565; the other modes refuse the tail and keep K2).  No K6; the bytes equal
    the packing of the frames' RGBA, itself checked against libwebp's SHA-256."""
    import hashlib
    import os
    from oracle_lib import bench_files, manifest
    paths = bench_files("c3_4k")
    want = manifest()["bench"]
    n = 3
    datas = [open(paths[i], "rb").read() for i in range(n)]
    ref = ctx.batch(datas)
    try:
        ref.run()
        rgbas = [ref.rgba(i) for i in range(n)]
    finally:
        ref.close()
    for i, im in enumerate(rgbas):
        assert hashlib.sha256(im.tobytes()).hexdigest() == want[os.path.basename(paths[i])]["sha256"]["rgba"]
    for mode in range(11):
        for flip in (0, 1):
            if mode == 1 and not flip:
                continue  # (plain RGBA: no K6 batch)
            b = ctx.batch(datas, opts=webp_amd.options(mode, None, flip))
            try:
                tail = emit == "tail" and mode in (1, 6, 7)
                if emit == "tail":
                    if tail:
                        b.set_emit(False)
                    else:
                        with pytest.raises(webp_amd.WebPError):
                            b.set_emit(False)
                b.run()
                ms = b.kernel_ms()
                assert ms[5] == 0, (mode, flip, ms)  # no K6: every frame emitted directly
                assert (ms[1] > 0) == (not tail), (mode, flip, ms)  # K2, or K1's tail
                for i, im in enumerate(rgbas):
                    np.testing.assert_array_equal(b.download(i), _modes_from_rgba(im, mode, flip),
                                                  err_msg=f"mode {mode} flip {flip} frame {i}")
            finally:
                b.close()
