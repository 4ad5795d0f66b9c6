#!/usr/bin/env python3
"""Status-parity fixtures: what WebPDecode (libwebp 1.6.0, Pillow's bundled build, plain-C
and SIMD paths cross-checked) returns for corrupted and truncated inputs.

Test infrastructure only -- runs in the build container, never on the GPU box.

For every source fixture: the file itself, consistent-RIFF truncations at many points
(the truncation reaches the VP8 / VP8L / ALPH data), raw truncations (container errors)
and seeded bit flips past the RIFF header, each decoded without a crop window and with
two crop windows (the rows libwebp decodes -- and so the errors it sees -- depend on the
crop bottom).  The mutants are regenerated from the committed sources by
oracle_lib.mutate(); only the ops and the statuses are stored (status/sweep.json), plus
libwebp's RGBA for the mutants whose crop window decodes although the whole image fails
(status/crop_hidden.npz).

Plus hand-built VP8L streams (status/crafted_*.webp) pinning prefix-code corner cases:
a simple code whose symbol lies past its alphabet, a meta image selecting group 0xffff,
an invalid code in a group the meta image never selects.

Usage:  python tests/golden/make_status_sweep.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import make_golden as mg  # noqa: E402
from oracle_lib import mutate  # noqa: E402

SOURCES = [
    "lossless/" + n for n in ("ll_alpha_48x48", "ll_corr_123x77", "ll_corr_64x64", "ll_noise_50x50", "ll_pal16_65x39",
                              "ll_pal200_70x30", "ll_pal2_64x40", "ll_pal4_63x41", "ll_smooth_100x60_q0",
                              "ll_synth_90x33_m0")
] + [
    "lossy/" + n for n in ("synth_1x1", "synth_2x3", "synth_17x9", "synth_80x96", "noise_96x64_complex_s0",
                           "noise_96x64_simple", "noise_96x64_nofilter", "smooth_161x113_simple", "noise_130x70_q5",
                           "synth_200x150_part4", "alpha_64x48")
] + [
    "alpha/" + n for n in ("a_ll_1x1", "a_ll_h_130x70", "a_ll_levels_90x60", "a_ll_none_33x65", "a_ll_q50_80x80",
                           "a_ll_v_97x81", "a_ll_best_g_96x64", "a_raw_g_64x64", "a_raw_h_71x33", "e_header_only",
                           "e_ll_stream_2b", "e_ll_stream_half", "e_ll_stream_zeros", "e_method2", "e_preproc2",
                           "e_raw_short", "e_reserved_bits")
]
TRUNC_RIFF = (0.03, 0.06, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 0.95, 0.99, 0.995)
TRUNC_RAW = (0.1, 0.5, 0.9)
N_FLIPS = 12


def size_of(data):
    st, rows = mg.decode_mode(data, mg.MODE_RGBA)
    assert st == 0
    return rows.shape[1] // 4, rows.shape[0]


def crops(w, h):
    c2t = (h // 2) | 1
    return [None, (0, 0, w, max(1, h // 3)), ((w // 4) | 1, c2t, w // 2, h - c2t - 1)]


def status(data, crop):
    out = []
    for plain in (True, False):
        mg._plain_c(plain)
        out.append(mg.decode_mode(data, mg.MODE_RGBA, crop)[0])
    mg._plain_c(True)
    assert out[0] == out[1], out
    return out[0]


# ---------------------------------------------------------------- hand-built VP8L streams
class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, value, nbits):
        self.v |= (value & ((1 << nbits) - 1)) << self.n
        self.n += nbits

    def simple(self, *syms):  # simple prefix code of one or two symbols
        self.put(1, 1)
        self.put(len(syms) - 1, 1)
        if syms[0] < 2:
            self.put(0, 1)
            self.put(syms[0], 1)
        else:
            self.put(1, 1)
            self.put(syms[0], 8)
        if len(syms) == 2:
            self.put(syms[1], 8)

    def tobytes(self, pad=4):
        return self.v.to_bytes((self.n + 7) // 8 + pad, "little")


def vp8l_file(w, h, body):
    b = Bits()
    b.put(0x2f, 8)
    b.put(w - 1, 14)
    b.put(h - 1, 14)
    b.put(1, 1)  # alpha_is_used
    b.put(0, 3)  # version
    b.v |= body.v << b.n
    b.n += body.n
    payload = b.tobytes()
    if len(payload) & 1:
        payload += b"\0"
    chunk = b"VP8L" + len(payload).to_bytes(4, "little") + payload
    return b"RIFF" + (4 + len(chunk)).to_bytes(4, "little") + b"WEBP" + chunk


def crafted():
    out = {}
    # 1x1, distance code simple(0, 200): symbol 200 is past the 40-symbol alphabet, ignored
    b = Bits()
    b.put(0, 1)  # no transform
    b.put(0, 1)  # no color cache
    b.put(0, 1)  # no meta codes
    for syms in ((0x40,), (0x10,), (0x20,), (0xff,), (0, 200)):
        b.simple(*syms)
    out["crafted_dist_oob_symbol"] = vp8l_file(1, 1, b)
    # the same with both distance symbols past the alphabet: no symbol left -> invalid code
    b = Bits()
    b.put(0, 3)  # no transform, no color cache, no meta codes
    for syms in ((0x40,), (0x10,), (0x20,), (0xff,), (200, 201)):
        b.simple(*syms)
    out["crafted_dist_no_symbol"] = vp8l_file(1, 1, b)
    # meta image of one pixel selecting group 0xffff: 65536 groups of five 1-symbol codes
    b = Bits()
    b.put(0, 1)  # no transform
    b.put(0, 1)  # no color cache
    b.put(1, 1)  # meta codes
    b.put(0, 3)  # huffman bits 2
    b.put(0, 1)  # meta image: no color cache
    for syms in ((0xff,), (0xff,), (0,), (0,), (0,)):  # green, red (group = red << 8 | green)
        b.simple(*syms)
    for g in range(65536):
        for j in range(5):
            b.simple(0x40 if (g == 0xffff and j == 0) else 0)
    out["crafted_65536_groups"] = vp8l_file(1, 1, b)
    # 4x4 image, one meta tile selecting group 5 (6 groups <= 16 pixels: libwebp keeps all); group 2's distance code is invalid
    b = Bits()
    b.put(0, 2)  # no transform, no color cache
    b.put(1, 1)  # meta codes
    b.put(0, 3)  # huffman bits 2 -> one meta pixel
    b.put(0, 1)
    for syms in ((5,), (0,), (0,), (0,), (0,)):
        b.simple(*syms)
    for g in range(6):
        for j in range(5):
            if g == 2 and j == 4:
                b.simple(200)  # no symbol inside the alphabet
            else:
                b.simple(0x33 if j < 4 else 0)
    out["crafted_invalid_unused_group"] = vp8l_file(4, 4, b)
    # the same stream with group 2 valid (decodes)
    b = Bits()
    b.put(0, 2)
    b.put(1, 1)
    b.put(0, 3)
    b.put(0, 1)
    for syms in ((5,), (0,), (0,), (0,), (0,)):
        b.simple(*syms)
    for g in range(6):
        for j in range(5):
            b.simple(0x33 if j < 4 else 0)
    out["crafted_unused_groups_ok"] = vp8l_file(4, 4, b)
    return out


def main():
    sdir = os.path.join(HERE, "status")
    os.makedirs(sdir, exist_ok=True)
    rng = np.random.default_rng(2024)
    cases = []
    hidden = {}  # case index -> RGBA rows of a crop that decodes although the full image fails
    for src in SOURCES:
        with open(os.path.join(HERE, src + ".webp"), "rb") as f:
            data = f.read()
        w, h = size_of(data) if mg.decode_mode(data, mg.MODE_RGBA)[0] == 0 else (0, 0)
        ops = [("none", None)] + [("trunc_riff", f) for f in TRUNC_RIFF] + [("trunc", f) for f in TRUNC_RAW]
        for _ in range(N_FLIPS):
            k = int(rng.integers(1, 4))
            ops.append(("flip", [[int(rng.integers(12, len(data))), int(rng.integers(0, 8))] for _ in range(k)]))
        for op, arg in ops:
            m = mutate(data, op, arg)
            if m is None:
                continue
            full = None
            for crop in (crops(w, h) if w else [None]):
                st = status(m, crop)
                if crop is None:
                    full = st
                elif st == 0 and full != 0:
                    # the crop window hides the failure: keep libwebp's output as the golden
                    hidden[str(len(cases))] = mg.decode_mode(m, mg.MODE_RGBA, crop)[1]
                cases.append({"src": src, "op": op, "arg": arg, "crop": list(crop) if crop else None, "status": st})
    statuses = {}
    for name, data in crafted().items():
        with open(os.path.join(sdir, name + ".webp"), "wb") as f:
            f.write(data)
        statuses[name] = status(data, None)
    with open(os.path.join(sdir, "sweep.json"), "w") as f:
        json.dump({"libwebp": "1.6.0 (Pillow bundled), WebPDecode MODE_RGBA", "cases": cases, "crafted": statuses},
                  f, indent=0)
    np.savez_compressed(os.path.join(sdir, "crop_hidden.npz"), **hidden)
    hist = {}
    for c in cases:
        hist[c["status"]] = hist.get(c["status"], 0) + 1
    print(f"{len(cases)} cases, statuses {hist}; {len(hidden)} crop-hidden failures; crafted {statuses}")


if __name__ == "__main__":
    main()
