"""WebPDecode status parity through the batch API on the GPU (tests/golden/status/).

Every mutant of the status sweep goes through wg_decode_batch with its crop window; the
per-frame statuses must equal libwebp's.  Frames that decode are checked bit for bit: where
the whole image also decodes, against the CPU oracle's output window; where only the crop
window decodes (libwebp never reads the corrupt rows below it -- the host stage bounds its
parse the same way), against libwebp's own RGBA stored by the generator.
"""
import collections

import numpy as np
import pytest

import webp_amd
from oracle_lib import GOLDEN, load_fixture, mutate, oracle_output, status_sweep

pytestmark = pytest.mark.gpu


def test_batch_statuses_and_pixels_match_libwebp():
    if webp_amd.device_count() < 1:
        pytest.fail("no HIP device visible")
    sweep = status_sweep()
    hidden = np.load(f"{GOLDEN}/status/crop_hidden.npz")
    groups = collections.defaultdict(list)  # (src, crop) -> case indices
    for i, c in enumerate(sweep["cases"]):
        groups[(c["src"], tuple(c["crop"]) if c["crop"] else None)].append(i)
    ctx = webp_amd.Context(0)
    checked = hidden_checked = 0
    bad = []
    for (src, crop), idx in sorted(groups.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
        data = load_fixture(src)
        muts = [mutate(data, sweep["cases"][i]["op"], sweep["cases"][i]["arg"]) for i in idx]
        opts = webp_amd.options(crop=crop) if crop else webp_amd.options()
        outs, status = ctx.decode_batch_opts(muts, opts)
        for k, i in enumerate(idx):
            c = sweep["cases"][i]
            if int(status[k]) != c["status"]:
                bad.append((src, c["op"], c["arg"], crop, c["status"], int(status[k])))
                continue
            if c["status"] != 0:
                continue
            if str(i) in hidden:
                np.testing.assert_array_equal(outs[k], hidden[str(i)], err_msg=f"{src} {c['op']} {c['arg']} {crop}")
                hidden_checked += 1
            else:
                np.testing.assert_array_equal(outs[k], oracle_output(muts[k], crop=crop),
                                              err_msg=f"{src} {c['op']} {c['arg']} {crop}")
                checked += 1
    ctx.close()
    assert not bad, f"{len(bad)} status mismatches: {bad[:10]}"
    assert checked > 500 and hidden_checked == len(hidden.files), (checked, hidden_checked)


def test_crafted_vp8l_streams_decode_on_gpu():
    sweep = status_sweep()
    names = sorted(sweep["crafted"])
    ctx = webp_amd.Context(0)
    outs, status = ctx.decode_batch([load_fixture("status/" + n) for n in names])
    ctx.close()
    for n, o, s in zip(names, outs, status):
        assert int(s) == sweep["crafted"][n], n
        if s == 0:
            np.testing.assert_array_equal(o.reshape(o.shape[0], -1), oracle_output(load_fixture("status/" + n)),
                                          err_msg=n)
