#!/usr/bin/env python3
"""Debug aid: run one tests/k7_streams.py case through wg_vp8l_resolve_device and print the
pixels that differ from the oracle with their tokens."""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import k7_streams  # noqa: E402
from test_gpu_k7 import device_resolve, oracle_resolve  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "copy_far"
case = [c for c in k7_streams.CASES if c[0] == name][0]
_, n, bits, kw = case
toks, lits = k7_streams.make_stream(n, bits, seed=zlib.crc32(name.encode()), **kw)
want = oracle_resolve(toks, lits, bits)
got = device_resolve(toks, lits, bits)
bad = np.nonzero(got != want)[0]
print(name, "differ:", bad.size)
for i in bad[:40]:
    t = toks[i]
    k, pl = t >> 30, t & ((1 << 30) - 1)
    extra = ""
    if k == 2:
        s = i - pl
        extra = f" src {s} (block {s // 4096}) want[src] {want[s]:08x} got[src] {got[s]:08x}"
    print(f"  {i} (block {i // 4096}, off {i % 4096}) kind {k} pl {pl} got {got[i]:08x} want {want[i]:08x}{extra}")
