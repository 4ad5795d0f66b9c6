#!/usr/bin/env python3
"""Where the end-to-end (host bitstreams in, host RGBA out) time of one c3 batch goes:
batch create (host entropy stage + device allocation + H2D), run, per-frame D2H, destroy."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def main():
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime)
    import webp_amd
    from bench import WORKLOADS, _load_frames
    datas, _ = _load_frames(WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"]["prefix"])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    frames = [datas[i % len(datas)] for i in range(n)]
    ctx = webp_amd.Context(0, host_threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ctx.decode_batch(frames[:2])
    for rep in range(2):
        t0 = time.perf_counter()
        b = ctx.batch(frames)
        t1 = time.perf_counter()
        b.run()
        import ctypes
        webp_amd.lib().wg_batch_kernel_ms(b._h, (ctypes.c_float * 4)(), 4)  # syncs the batch
        t2 = time.perf_counter()
        w, h = b.dims(0)
        out = np.empty((h, w, 4), np.uint8)
        for i in range(b.n):
            st = webp_amd.lib().wg_batch_download_rgba(b._h, i, out.ctypes.data, 4 * w)
            assert st == 0
        t3 = time.perf_counter()
        b.close()
        t4 = time.perf_counter()
        print(f"rep {rep}: create {t1 - t0:.3f} s, run {t2 - t1:.3f} s, D2H {t3 - t2:.3f} s "
              f"({b.pixels * 4 / (t3 - t2) / 1e9:.1f} GB/s), destroy {t4 - t3:.3f} s")
    ctx.close()


if __name__ == "__main__":
    main()
