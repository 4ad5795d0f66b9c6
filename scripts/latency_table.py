#!/usr/bin/env python3
"""Latency / batch-size table of the lossy device path.

* webp_amd.decode() (the single-frame drop-in behind webp.Decode, decode.go:8-14): wall time
  per call for C1 (512x512) and one 4K C3 frame, host in / host out, median of N calls, next
  to the 1-core CPU restatement (entropy stage + oracle) and libwebp 1.6.0 (SIMD, 1 core) on
  the same frame;
* the resident device path (wg_batch_run) at batch sizes 1 .. 512 of C3 frames: the step time
  (HIP events around K1 + its tail) and the throughput it implies.

Prints one JSON object; `--out FILE` also writes it."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def _median_call(fn, n):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--batches", default="1,2,16,64,128,255,256,257,512")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, shared with torch)
    import bench
    import webp_amd
    from oracle_lib import bench_files, oracle_decode

    res = {"decode": {}, "batch": []}
    c1 = open(bench_files("c1_512")[0], "rb").read()
    c3 = [open(p, "rb").read() for p in bench_files("c3_4k")]
    lw = None
    try:
        lw, cpu, simd = bench._libwebp()
        cpu.value = simd
    except Exception as e:  # noqa: BLE001
        res["libwebp_unavailable"] = str(e)
    import numpy as np
    for name, data in (("c1_512", c1), ("c3_4k_one_frame", c3[0])):
        webp_amd.decode(data)  # warm: the default context, its pools and device buffers
        med, best = _median_call(lambda: webp_amd.decode(data), args.calls)
        f = webp_amd.features(data)
        px = f.width * f.height
        cpu_s, _ = _median_call(lambda: bench._cpu_decode_one(data), max(3, args.calls // 4))
        ent = {"pixels": px, "gpu_decode_ms_median": round(med * 1e3, 3), "gpu_decode_ms_best": round(best * 1e3, 3),
               "cpu_port_1_core_ms": round(cpu_s * 1e3, 3), "speedup_vs_port": round(cpu_s / med, 2)}
        if lw is not None:
            out = np.empty(px * 4, np.uint8)
            lw_s, _ = _median_call(lambda: lw.WebPDecodeRGBAInto(data, len(data), out.ctypes.data, out.nbytes,
                                                                  4 * f.width), max(3, args.calls // 4))
            ent["libwebp_simd_1_core_ms"] = round(lw_s * 1e3, 3)
            ent["speedup_vs_libwebp_1_core"] = round(lw_s / med, 2)
        res["decode"][name] = ent
        print(name, ent, file=sys.stderr, flush=True)
    ctx = webp_amd.Context(0)
    for n in [int(x) for x in args.batches.split(",")]:
        b = ctx.batch([c3[i % len(c3)] for i in range(n)])
        for _ in range(2):
            b.run()
        b.kernel_ms()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b.run()
        ms = b.kernel_ms()
        wall = (time.perf_counter() - t0) / args.steps
        ent = {"frames": n, "k1_ms": round(ms[0], 4), "step_wall_ms": round(wall * 1e3, 3),
               "mpix_s": round(b.pixels / (ms[0] * 1e-3) / 1e6, 1)}
        res["batch"].append(ent)
        print(ent, file=sys.stderr, flush=True)
        b.close()
    ctx.close()
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
