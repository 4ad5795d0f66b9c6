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
    for opts, want in ((webp_amd.options(11), webp_amd.Status.UNSUPPORTED_FEATURE),
                       (webp_amd.options(13), webp_amd.Status.INVALID_PARAM),
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
    wg_batch_run (its own kernel_ms entry); downloads copy its output: equal to WebPDecode's
    bytes after repeated runs (RGB flipped, rgbA premultiplied, ARGB point-sampled, RGBA
    flipped)."""
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
        assert by[5] == sum((4 + bpp) * g[key].shape[0] * g[key].shape[1] // bpp for _, g in sub)
        for i, (_, g) in enumerate(sub):
            np.testing.assert_array_equal(b.download(i), g[key], err_msg=f"{key} frame {i}")
    finally:
        b.close()
