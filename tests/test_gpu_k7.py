"""K7 (color cache + back-references, vp8l_resolve.hip) through its stage entry
wg_vp8l_resolve_device, bit-exact against the oracle's restatement of the reference's pixel
loop (oracle_vp8l_resolve: pkg/vp8/vp8l_dec.c.go:1038-1189, color_cache.go:46-63) on synthetic
token streams aimed at each of K7's paths (tests/k7_streams.py) and on the C5 bench streams'
real tokens.  (The batch path -- host entropy stage -> K7 -> K3 -- is covered against libwebp
by test_gpu_vp8l.py and test_gpu_fuzz.py.)"""
import os
import zlib

import numpy as np
import pytest

import k7_streams
from oracle_lib import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def oracle_resolve(toks, lits, bits):
    out = np.empty(toks.size, np.uint32)
    assert oracle().oracle_vp8l_resolve(toks.ctypes.data, lits.ctypes.data, lits.size, toks.size, bits,
                                        out.ctypes.data) == 0
    return out


def device_resolve(toks, lits, bits):
    import torch
    import webp_amd
    dt = torch.from_numpy(toks.view(np.int32)).cuda()
    dl = torch.from_numpy(lits.view(np.int32)).cuda()
    out = torch.full((toks.size,), -1, dtype=torch.int32, device="cuda")
    webp_amd.vp8l_resolve_device(dt.data_ptr(), dl.data_ptr(), lits.size, toks.size, bits, out.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("name,n,bits,kw", k7_streams.CASES, ids=[c[0] for c in k7_streams.CASES])
def test_k7_synthetic_streams(name, n, bits, kw):
    toks, lits = k7_streams.make_stream(n, bits, seed=zlib.crc32(name.encode()), **kw)
    want = oracle_resolve(toks, lits, bits)
    got = device_resolve(toks, lits, bits)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{name}: {bad.size} pixels differ, first at {bad[:5]}"


def test_k7_c5_streams():
    import webp_amd
    for s in range(8):
        path = os.path.join(ROOT, "tests", "golden", "bench", f"c5_ll2048_s{s}.webp")
        info, coded, _ = webp_amd.vp8l_parse(open(path, "rb").read())
        toks = np.ascontiguousarray(coded.tokens, np.uint32).ravel()
        lits = np.ascontiguousarray(coded.lits, np.uint32)
        want = oracle_resolve(toks, lits, coded.cache_bits)
        got = device_resolve(toks, lits, coded.cache_bits)
        assert np.array_equal(got, want), f"s{s}: {(got != want).sum()} pixels differ"


def test_k7_c3a_alpha_streams():
    """The alpha streams of the c3a bench frames (ALPH method 1: green-only VP8L, no cache):
    nearly every token a distance-1 or one-row copy."""
    import webp_amd
    for s in (0, 5):
        path = os.path.join(ROOT, "tests", "golden", "bench", f"c3a_4k_s{s}.webp")
        info, (ll, coded, _) = webp_amd.alpha_parse(open(path, "rb").read())
        toks = np.ascontiguousarray(coded.tokens, np.uint32).ravel()
        lits = np.ascontiguousarray(coded.lits, np.uint32)
        want = oracle_resolve(toks, lits, coded.cache_bits)
        got = device_resolve(toks, lits, coded.cache_bits)
        assert np.array_equal(got, want), f"s{s}: {(got != want).sum()} pixels differ"


_STATS_CHILD = r"""
import ctypes as C, sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import webp_amd, k7_streams
toks, lits = k7_streams.make_cross_window_stream(4, seed=5)
dt = torch.from_numpy(toks.view(np.int32)).cuda()
dl = torch.from_numpy(lits.view(np.int32)).cuda()
out = torch.empty(toks.size, dtype=torch.int32, device="cuda")
L = webp_amd.lib()
st = (C.c_ulonglong * (16 * 17))()
L.wg_debug_k7_stats(st, 1)
webp_amd.vp8l_resolve_device(dt.data_ptr(), dl.data_ptr(), lits.size, toks.size, 11, out.data_ptr())
torch.cuda.synchronize()
L.wg_debug_k7_stats(st, 1)
print("K7STATS", st[0], st[1], st[2], st[3], st[9], st[10])
"""


def test_k7_cross_window_lookup_sources():
    """Blocks that run as several windows (cache_bits 11: 256 ranks per window) where a later
    window's in-block copies take their value from lookups of an earlier window that had no
    pending copy (so its lookups resolved on the no-rounds path): bit-exact against the oracle,
    and -- through the measurement build's counters, when it has been built -- no window hits
    the round cap or falls to the serial path (the performance cliff the lookups' missing
    'known' state used to cause)."""
    import subprocess
    import sys
    toks, lits = k7_streams.make_cross_window_stream(4, seed=5)
    want = oracle_resolve(toks, lits, 11)
    got = device_resolve(toks, lits, 11)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} pixels differ, first at {bad[:5]}"
    timing = os.path.join(ROOT, "go-webp_amd", "webp_amd", "libgowebp_amd_timing.so")
    if not os.path.exists(timing):
        pytest.skip("measurement build (make VARIANT=timing) absent: counters not checked")
    env = dict(os.environ, WG_LIB_VARIANT="timing")
    r = subprocess.run([sys.executable, "-c", _STATS_CHILD, os.path.join(ROOT, "go-webp_amd"),
                        os.path.join(ROOT, "tests")], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("K7STATS")][-1]
    blocks, serial, rounds, windows, empty, caps = map(int, line.split()[1:])
    assert blocks == 4 and windows > blocks, line  # the stream really runs as several windows
    assert caps == 0 and serial == 0, f"round caps {caps}, serial windows {serial} ({line})"


def test_k7_rejects_bad_params():
    import webp_amd
    with pytest.raises(webp_amd.WebPError):
        webp_amd.vp8l_resolve_device(0, 0, 0, 16, 4, 0)


def _resolve_oob_zero(toks, lits, bits):
    """The stage entry's documented rule for tokens the host stage never emits (literal index
    >= n_lits, key >= 1 << cache_bits, distance 0 or before the start): the pixel resolves to 0
    and, like any pixel, is inserted into the cache (gowebp_amd.h).  A plain loop; small n."""
    cache = [0] * (1 << bits if bits else 1)
    out = [0] * toks.size
    for i, t in enumerate(toks.tolist()):
        kind, pl = t >> 30, t & 0x3FFFFFFF
        v = 0
        if kind == 0:
            v = int(lits[pl]) if pl < lits.size else 0
        elif kind == 1:
            v = cache[pl] if bits and pl < (1 << bits) else 0
        elif kind == 2:
            v = out[i - pl] if 1 <= pl <= i else 0
        out[i] = v
        if kind != 3 and bits:
            cache[((v * 0x1E35A7BD) & 0xFFFFFFFF) >> (32 - bits)] = v
    return np.asarray(out, np.uint32)


def test_k7_untrusted_tokens_out_of_bounds():
    """The stage entry takes caller tokens (not host-validated, unlike the batch path): literal
    indices past n_lits, keys past the cache, distance 0 and distances before the start resolve
    to 0 (the serial path), in several blocks and next to ordinary tokens."""
    toks, lits = k7_streams.make_stream(3 * 4096 + 50, 6, seed=7, p_lit=0.2, p_copy=0.2, dist=(1, "near"), run=6)
    rng = np.random.default_rng(11)
    pos = rng.choice(np.arange(10, toks.size), size=40, replace=False)
    for k, i in enumerate(pos.tolist()):
        toks[i] = [(0 << 30) | (lits.size + k), (1 << 30) | (64 + k), (2 << 30) | 0, (2 << 30) | (i + 1 + k)][k % 4]
    want = _resolve_oob_zero(toks, lits, 6)
    got = device_resolve(toks, lits, 6)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} pixels differ, first at {bad[:5]}"


def test_k7_random_streams():
    """Randomised token streams (a fixed seed per case): cache sizes 0..11 bits, literal / copy
    mixes, run lengths and distance classes drawn at random, lengths across block boundaries --
    each bit-exact against the oracle."""
    rng = np.random.default_rng(20261017)
    dist_sets = [(1,), (1, "near"), ("w", "near"), ("far", 1), (4096, 4097, "near"), (1, 2, 3, 4)]
    for case in range(24):
        bits = int(rng.integers(0, 12))
        n = int(rng.integers(1, 3 * 4096 + 200))
        kw = dict(p_lit=float(rng.uniform(0.01, 0.6)), p_copy=float(rng.uniform(0.0, 0.4)),
                  dist=dist_sets[int(rng.integers(len(dist_sets)))], run=int(rng.integers(1, 64)),
                  palette=int(rng.integers(2, 3000)), width=int(rng.integers(16, 2048)),
                  p_empty=float(rng.choice([0.0, 0.0, 0.002])))
        toks, lits = k7_streams.make_stream(n, bits, seed=1000 + case, **kw)
        want = oracle_resolve(toks, lits, bits)
        got = device_resolve(toks, lits, bits)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"case {case} (n={n}, bits={bits}, {kw}): {bad.size} pixels differ, first at {bad[:5]}"


def test_k7_random_dense_streams():
    """Randomised dense streams for the small-cache instantiation (cache_bits 0..7): nearly every
    pixel a copy (runs up to 3,000 of distance 1, one row, or short distances), few literals, a
    few lookups, and random lookup-free stretches -- each bit-exact against the oracle."""
    rng = np.random.default_rng(20261018)
    dist_sets = [(1,), (1, "w"), (1, 1, "w", 2), ("w", "near"), (1, 3, "near")]
    for case in range(16):
        bits = int(rng.integers(0, 8))
        n = int(rng.integers(4096, 5 * 4096 + 300))
        p_lit = float(rng.uniform(0.003, 0.15))
        a = int(rng.integers(0, n))
        kw = dict(p_lit=p_lit, p_copy=float(rng.uniform(0.6, 0.995 - p_lit)), dist=dist_sets[int(rng.integers(len(dist_sets)))],
                  run=int(rng.integers(2, 3000)), palette=int(rng.integers(2, 64)), width=int(rng.integers(64, 2048)),
                  quiet=((a, a + int(rng.integers(0, 2 * 4096))),))
        toks, lits = k7_streams.make_stream(n, bits, seed=2000 + case, **kw)
        want = oracle_resolve(toks, lits, bits)
        got = device_resolve(toks, lits, bits)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"case {case} (bits {bits}, {kw}): {bad.size} pixels differ, first at {bad[:5]}"
