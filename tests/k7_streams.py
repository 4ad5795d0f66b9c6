"""Synthetic VP8L token streams for K7 (vp8l_resolve.hip) parity tests.

A token stream is what the host entropy stage hands K7 (device_format.h kTok*): one uint32 per
pixel, kind in bits 31:30 (0 literal index, 1 color-cache key, 2 backward distance, 3 unset)
and the payload in bits 29:0, plus the literal ARGB values.  The streams are generated the way
an encoder would emit them -- every lookup names a key whose slot holds a value, unless a case
asks for lookups of never-written slots -- by running the reference's pixel loop
(pkg/vp8/vp8l_dec.c.go:1038-1189, color_cache.go:46-63) alongside, so each case can aim at one
of K7's paths: windows (more updaters per block than the rank masks hold), in-block copy chains
(pointer jumping), copies reaching back more than one block, the serial fallback (empty slots,
the round cap).  The expected output is always the oracle's (oracle_vp8l_resolve), not this
generator's.
"""
import numpy as np

HASH_MUL = 0x1E35A7BD
LIT, CACHE, COPY, UNSET = 0, 1, 2, 3


def hash_px(v, bits):
    return ((v * HASH_MUL) & 0xFFFFFFFF) >> (32 - bits)


def make_stream(n, bits, seed, p_lit=0.035, p_copy=0.0, dist=(1,), palette=256, width=2048, run=1,
                p_empty=0.0, chain=False, quiet=()):
    """-> (tokens uint32[n], lits uint32[]).  p_lit / p_copy: probabilities of a literal / a copy
    run (length 1..run, distances drawn from `dist`: ints, or "w" (the row above), "near"
    (1..64), "far" (4096..20000)); the rest are cache lookups of keys whose slot holds a value
    (p_empty of them of a never-written slot instead).  quiet: (start, end) pixel ranges with no
    lookups (their lookups become copies): lookup-free blocks between blocks with lookups.  chain: alternate one-pixel copies of
    distance 1 and lookups (each copy's source is a lookup: one round per pair)."""
    rng = np.random.default_rng(seed)
    pal = rng.integers(0, 1 << 32, size=palette, dtype=np.uint64).astype(np.uint32)
    pal[0] = 0
    nk = 1 << bits if bits else 0
    cache = [0] * max(nk, 1)
    written = set()
    vals = []
    toks = np.empty(n, np.uint32)
    lits = []
    keys = []  # written keys, for lookups

    def insert(v):
        if nk:
            h = hash_px(v, bits)
            if h not in written:
                written.add(h)
                keys.append(h)
            cache[h] = v

    i = 0
    while i < n:
        r = rng.random()
        if chain and i > 0 and keys:
            if i % 2:
                toks[i] = (COPY << 30) | 1
                v = vals[i - 1]
            else:
                k = keys[int(rng.integers(len(keys)))]
                toks[i] = (CACHE << 30) | k
                v = cache[k]
            vals.append(v)
            insert(v)
            i += 1
            continue
        if i == 0 or r < p_lit or (nk and not keys and r >= p_lit + p_copy):
            v = int(pal[int(rng.integers(palette))])
            toks[i] = (LIT << 30) | len(lits)
            lits.append(v)
            vals.append(v)
            insert(v)
            i += 1
        elif r < p_lit + p_copy or not nk or any(a <= i < e for a, e in quiet):
            d = dist[int(rng.integers(len(dist)))]
            if d == "w":
                d = width
            elif d == "near":
                d = int(rng.integers(1, 65))
            elif d == "far":
                d = int(rng.integers(4096, 20001))
            d = min(int(d), i)
            ln = int(rng.integers(1, run + 1))
            for _ in range(min(ln, n - i)):
                toks[i] = (COPY << 30) | d
                v = vals[i - d]
                vals.append(v)
                insert(v)
                i += 1
        else:
            if p_empty and rng.random() < p_empty and nk > 1:
                k = int(rng.integers(1, nk))
                while k in written and len(written) < nk - 1:
                    k = int(rng.integers(1, nk))
            else:
                k = keys[int(rng.integers(len(keys)))]
            toks[i] = (CACHE << 30) | k
            v = cache[k]
            vals.append(v)
            insert(v)
            i += 1
    return toks, np.asarray(lits if lits else [0], np.uint32)


def make_cross_window_stream(blocks, seed, bits=11, p_lit=0.4, p_copy=0.12):
    """-> (tokens, lits): blocks of 4096 pixels whose first half holds only literals and cache
    lookups and whose second half adds in-block copies whose SOURCE is one of the first half's
    lookups.  At cache_bits 11 K7's rank masks hold 256 updaters per window, so with ~40 %
    literals a block runs as several windows: the early windows have no pending copy (their
    lookups resolve on the no-rounds path) and a later window's copies read those lookups'
    states -- the case that must not fall into the round cap / serial path."""
    rng = np.random.default_rng(seed)
    nk = 1 << bits
    cache = [0] * nk
    keys, written = [], set()
    vals, toks, lits = [], [], []

    def insert(v):
        h = hash_px(v, bits)
        if h not in written:
            written.add(h)
            keys.append(h)
        cache[h] = v

    for b in range(blocks):
        base = 4096 * b
        lookup_pos = []
        for li in range(4096):
            i = base + li
            r = rng.random()
            if i == 0 or not keys or r < p_lit:
                v = int(rng.integers(1, 1 << 32))
                toks.append((LIT << 30) | len(lits))
                lits.append(v)
            elif li >= 2048 and lookup_pos and r < p_lit + p_copy:
                src = lookup_pos[int(rng.integers(len(lookup_pos)))]
                toks.append((COPY << 30) | (i - src))
                v = vals[src]
            else:
                k = keys[int(rng.integers(len(keys)))]
                toks.append((CACHE << 30) | k)
                v = cache[k]
                if li < 2048:
                    lookup_pos.append(i)
            vals.append(v)
            insert(v)
    return np.asarray(toks, np.uint32), np.asarray(lits, np.uint32)


# (name, n_px, cache_bits, kwargs): each aims at one path of K7
CASES = [
    ("c5like", 3 * 4096 + 123, 10, dict(p_lit=0.035, palette=300)),
    ("windows_b11", 2 * 4096 + 7, 11, dict(p_lit=0.45, p_copy=0.15, dist=(1, "near"), palette=4000)),
    ("windows_b8", 2 * 4096, 8, dict(p_lit=0.7, palette=2000)),
    ("copy_runs", 3 * 4096 + 1, 8, dict(p_lit=0.05, p_copy=0.3, dist=(1, "w", "near"), run=300, width=1000)),
    ("copy_far", 6 * 4096 + 5, 10, dict(p_lit=0.05, p_copy=0.3, dist=("far", 4096, 4097, 8191, 8192), run=20)),
    ("no_cache", 2 * 4096 + 9, 0, dict(p_lit=0.4, p_copy=0.6, dist=(1, 3, "near", "far"), run=50)),
    ("empty_slots", 4096 + 100, 6, dict(p_lit=0.05, p_empty=0.01, palette=40)),
    ("round_cap", 4096 + 64, 9, dict(chain=True, palette=64)),
    ("one_px", 1, 10, dict()),
    ("three_px", 3, 4, dict()),
    ("block_edge", 4097, 10, dict(p_lit=0.2, p_copy=0.2, dist=(1, "near"), run=8)),
    ("b1", 4096 + 33, 1, dict(p_lit=0.3, palette=8)),
    # alpha-plane shaped (ALPH streams: almost all copies, runs of distance 1 and of one row):
    # distance-1 runs collapse to their root by the block max-scan, across blocks too
    ("alpha_runs", 5 * 4096 + 77, 0, dict(p_lit=0.01, p_copy=0.99, dist=(1, 1, "w"), run=2500, width=1920,
                                          palette=12)),
    ("alpha_runs_cached", 4 * 4096 + 3, 3, dict(p_lit=0.02, p_copy=0.9, dist=(1, "w", 2), run=900, width=700,
                                                palette=20)),
    ("long_run", 3 * 4096 + 500, 0, dict(p_lit=0.0005, p_copy=0.9995, dist=(1,), run=20000)),
    ("short_runs", 2 * 4096 + 11, 4, dict(p_lit=0.2, p_copy=0.6, dist=(1, 1, 1, "near"), run=3, palette=30)),
    # every pixel an updater (registration combined per key across a wave's lanes), with lookups
    # straddling them: few keys (b2) and many (b10), windows of 2048 updaters
    ("dense_b2", 3 * 4096 + 9, 2, dict(p_lit=0.1, p_copy=0.85, dist=(1, 2, "w", "near"), run=40, width=300,
                                       palette=6)),
    ("dense_b10", 3 * 4096 + 70, 10, dict(p_lit=0.3, p_copy=0.6, dist=(1, "near", "far"), run=12, palette=3000)),
    # the 64-mask-word instantiation (cache bits <= 7): one window of up to 4096 ranks, lookups
    # straddling updaters of their key in the words above 32
    ("w64_straddle", 4 * 4096 + 21, 6, dict(p_lit=0.55, p_copy=0.35, dist=(1, 2, "near"), run=4, palette=90)),
    ("w64_b7_lits", 3 * 4096 + 5, 7, dict(p_lit=0.9, p_copy=0.02, palette=400)),
    # lookup-free blocks (no rank masks: the slot table from one max pass) between blocks whose
    # lookups read what they left
    ("w64_quiet_blocks", 6 * 4096 + 17, 4, dict(p_lit=0.1, p_copy=0.8, dist=(1, "w", 3), run=30, width=900,
                                                palette=40, quiet=((4096, 3 * 4096), (4 * 4096 + 100, 5 * 4096 + 7)))),
    # round 6's rank-free dense blocks (cache bits <= 7): copies of lookups (a lookup's key is their
    # hash before its value is known), lookups whose last pixel of the key is such a copy or another
    # lookup, and the copy / lookup chain walked across rounds
    ("w64_lookup_dense", 3 * 4096 + 41, 3, dict(p_lit=0.01, p_copy=0.7, dist=(1, 2, "w", "near"), run=6, width=500,
                                                palette=10)),
    ("w64_chain", 2 * 4096 + 3, 4, dict(chain=True, palette=24)),
]
