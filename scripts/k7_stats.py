#!/usr/bin/env python3
"""K7 (vp8l_resolve.hip) block statistics from the measurement build (make VARIANT=timing,
WG_LIB_VARIANT=timing): blocks, blocks redone serially, rounds, and wave 0's cycles per phase
(tokens + ranks, windows, serial path, stores) for one batch of a bench workload:
k7_stats.py [frames] [workload: c5 (default) | c3a (the ALPH streams)]."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]
os.environ.setdefault("WG_LIB_VARIANT", "timing")


def main():
    import torch  # noqa: F401
    import webp_amd
    from bench import WORKLOADS, _load_frames
    wl = sys.argv[2] if len(sys.argv) > 2 else "c5"
    datas, _ = _load_frames(WORKLOADS[wl]["prefix"])
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch([datas[i % len(datas)] for i in range(n)])
    L = webp_amd.lib()
    st = (C.c_ulonglong * (16 * 17))()
    b.run()
    print("kernel ms", b.kernel_ms())
    L.wg_debug_k7_stats(st, 1)
    b.run()
    ms = b.kernel_ms()
    L.wg_debug_k7_stats(st, 1)
    blocks, serial, rounds, windows = st[0], st[1], st[2], st[3]
    # (the 64-word instantiation's dense blocks reuse the slots: 6 far copies + setup, 5 R jumping, 11 H last pixels, 12 L
    # lookups, 13 J jumping, 7 T slot table + end of block)
    phases = ((8, "classify (lit wait)"), (15, "prev-block copies+store"), (14, "issue next loads"), (4, "ranks + barrier"),
              (11, "registration | H"), (12, "lookups | L"), (5, "copies (rounds b) | R"),
              (13, "slot table | J"), (6, "serial path | setup"), (7, "store + pipeline | T"))
    tot = sum(st[i] for i, _ in phases)
    print(f"frames {n}: K7 {ms[4]:.3f} ms; blocks {blocks}, windows/block {windows / blocks:.3f}, "
          f"rounds/window {rounds / max(windows, 1):.3f}, serial windows {serial}")
    for i, name in phases:
        print(f"  {name:20s} {st[i] / blocks:10.0f} cycles/block  {st[i] / max(tot, 1):.3f}")
    wv = [[st[16 + 16 * w + i] / blocks for i in range(16)] for w in range(16)]
    print("  per wave (cycles/block):  " + " ".join(f"{name[:10]:>10s}" for _, name in phases))
    for w in range(16):
        print(f"    wave {w:2d}               " + " ".join(f"{wv[w][i]:10.0f}" for i, _ in phases))
    print(f"  serial causes (events): empty slot {st[9]}, round cap {st[10]}")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
