#!/usr/bin/env python3
"""Transfer and host-stage rates that bound the end-to-end decode (design data for the
pipelined wg_decode_rgba_batch): D2H / H2D into pageable (first touch and reused) and pinned
host memory, and the host entropy stage of one c3 batch alone (wg_batch_create minus its H2D)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def rate(fn, nbytes, reps=3):
    import torch
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return nbytes / best / 1e9, best


def main():
    import numpy as np
    import torch
    n = 1 << 30
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev.fill_(7)
    pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    page = torch.from_numpy(np.empty(n, np.uint8))
    print("D2H pinned   %.1f GB/s (%.3f s)" % rate(lambda: pin.copy_(dev, non_blocking=True), n))
    fresh = lambda: torch.from_numpy(np.empty(n, np.uint8)).copy_(dev)  # noqa: E731
    print("D2H pageable first touch %.1f GB/s (%.3f s)" % rate(fresh, n, reps=2))
    print("D2H pageable reused %.1f GB/s (%.3f s)" % rate(lambda: page.copy_(dev), n))
    print("H2D pinned   %.1f GB/s (%.3f s)" % rate(lambda: dev.copy_(pin, non_blocking=True), n))
    print("H2D pageable %.1f GB/s (%.3f s)" % rate(lambda: dev.copy_(page), n))
    a = np.empty(n, np.uint8)
    a[:] = 1
    b = np.empty(n, np.uint8)
    b[:] = 2
    t0 = time.perf_counter()
    np.copyto(b, a)
    print("host memcpy 1 thread %.1f GB/s" % (n / (time.perf_counter() - t0) / 1e9))
    del dev, pin, page, a, b

    import webp_amd
    from bench import WORKLOADS, _load_frames
    datas, _ = _load_frames(WORKLOADS["c3"]["prefix"])
    frames = [datas[i % len(datas)] for i in range(256)]
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    ctx = webp_amd.Context(0, host_threads=threads)
    for rep in range(3):
        t0 = time.perf_counter()
        b = ctx.batch(frames)
        t1 = time.perf_counter()
        b.close()
        print(f"batch create (parse + H2D of 256 c3 frames, {threads} threads) rep {rep}: {t1 - t0:.3f} s")
    ctx.close()


if __name__ == "__main__":
    main()
