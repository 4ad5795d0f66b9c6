#!/usr/bin/env python3
"""K7 (vp8l_resolve.hip) block statistics from the measurement build (make VARIANT=timing,
WG_LIB_VARIANT=timing): blocks, blocks redone serially, rounds, and wave 0's cycles per phase
(1 = tokens/literals/far copies, 2 = rounds, 3 = stores, 4 = slot table) for one c5 batch."""
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
    datas, _ = _load_frames(WORKLOADS["c5"]["prefix"])
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch([datas[i % len(datas)] for i in range(n)])
    L = webp_amd.lib()
    st = (C.c_ulonglong * 12)()
    b.run()
    print("kernel ms", b.kernel_ms())
    L.wg_debug_k7_stats(st, 1)
    b.run()
    ms = b.kernel_ms()
    L.wg_debug_k7_stats(st, 1)
    blocks, slow, rounds = st[0], st[1], st[2]
    tot = sum(st[3:7])
    print(f"frames {n}: K7 {ms[4]:.3f} ms; blocks {blocks}, serial {slow} ({slow / blocks:.4f}), "
          f"rounds/block {rounds / blocks:.2f}")
    for i, name in zip(range(3, 7), ("tokens+literals+far copies", "rounds", "stores", "slot table")):
        print(f"  {name:28s} {st[i] / blocks:10.0f} cycles/block  {st[i] / tot:.3f}")
    print(f"  serial causes (events): bad token {st[7]}, empty slot {st[8]}, long walk {st[9]}, round cap {st[10]}")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
