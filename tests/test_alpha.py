"""ALPH planes on the host/oracle side (no GPU): the host stage (wg_alpha_parse) + the CPU
oracle's inverse transforms and unfilters reproduce libwebp 1.6.0's A channel of every
alpha fixture, the lossy colour channels come from the lossy oracle, and corrupted ALPH
chunks get libwebp's own WebPDecode status (recorded in the manifest at fixture time)."""
import numpy as np
import pytest

import webp_amd
from oracle_lib import GOLDEN, alpha_names, load_alpha, manifest, oracle_alpha_plane, oracle_decode

NAMES = alpha_names()


def test_fixture_set_covers_methods_and_filters():
    hdrs = {(v["alph"]["method"], v["alph"]["filter"]) for v in manifest()["alpha"].values()}
    assert {(m, f) for m in (0, 1) for f in range(4)} <= hdrs
    assert any(v["alph"]["pre"] == 1 for v in manifest()["alpha"].values())
    assert any(v["height"] > 1024 and v["alph"]["filter"] == 3 for v in manifest()["alpha"].values())


@pytest.mark.parametrize("name", NAMES)
def test_alpha_plane_oracle_vs_libwebp(name):
    data, gold = load_alpha(name)
    info, plane = oracle_alpha_plane(data)
    ent = manifest()["alpha"][name]
    assert (info.method, info.filter, info.pre_processing) == (ent["alph"]["method"], ent["alph"]["filter"],
                                                               ent["alph"]["pre"])
    np.testing.assert_array_equal(plane, gold["rgba"][..., 3])


@pytest.mark.parametrize("name", NAMES)
def test_alpha_frame_colour_from_lossy_oracle(name):
    data, gold = load_alpha(name)
    feats = webp_amd.features(data)
    assert feats.has_alpha
    info, mbs = webp_amd.vp8_parse(data)
    np.testing.assert_array_equal(oracle_decode(info, mbs)["rgba"][..., :3], gold["rgba"][..., :3])


@pytest.mark.parametrize("name", sorted(manifest().get("alpha_errors", {})))
def test_corrupt_alph_status_matches_libwebp(name):
    import os

    data = open(os.path.join(GOLDEN, "alpha", name + ".webp"), "rb").read()
    want = manifest()["alpha_errors"][name]["status"]
    with pytest.raises(webp_amd.WebPError) as e:
        webp_amd.alpha_parse(data)
    assert e.value.status == want


def test_alpha_parse_rejects_frames_without_alph():
    from oracle_lib import load_lossless, load_lossy

    for data in (load_lossy("synth_80x96")[0], load_lossless("ll_corr_64x64")[0]):
        with pytest.raises(webp_amd.WebPError) as e:
            webp_amd.alpha_parse(data)
        assert e.value.status == webp_amd.Status.UNSUPPORTED_FEATURE
