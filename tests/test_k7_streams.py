"""CPU check of the K7 test streams (tests/k7_streams.py): every case is a valid token stream
for the oracle's restatement of the reference's pixel loop, and each reaches the K7 path it is
named for (windows: more updaters in some 4096-pixel block than the rank masks of its cache
size hold, 64 x min(32, 8192 >> bits); copy cases: in-block and older sources)."""
import zlib

import numpy as np
import pytest

import k7_streams
from oracle_lib import oracle


@pytest.mark.parametrize("name,n,bits,kw", k7_streams.CASES, ids=[c[0] for c in k7_streams.CASES])
def test_stream_valid(name, n, bits, kw):
    toks, lits = k7_streams.make_stream(n, bits, seed=zlib.crc32(name.encode()), **kw)
    out = np.empty(n, np.uint32)
    assert oracle().oracle_vp8l_resolve(toks.ctypes.data, lits.ctypes.data, lits.size, n, bits, out.ctypes.data) == 0
    kind = toks >> 30
    if name.startswith("windows"):
        cap = 64 * min(32, 8192 >> bits)
        upd = (kind == 0) | (kind == 2)
        per_block = [upd[i:i + 4096].sum() for i in range(0, n, 4096)]
        assert max(per_block) > cap
    if name.startswith("copy"):
        d = toks[kind == 2] & ((1 << 30) - 1)
        assert (d < 4096).any() and (name != "copy_far" or (d > 8192).any())
