#!/usr/bin/env python3
"""Per-stage breakdown of the single-frame drop-in (webp_amd.decode = wg_decode_rgba_into, the path
behind webp.Decode, /root/reference/decode.go:8-14) for C1 (512x512) and one 4K C3 frame
("first commit a per-stage breakdown").

Per frame, medians over --calls calls:
* decode_ms      webp_amd.decode(): host in, host out (pageable numpy output), wall clock;
* parse_ms       the host stages alone (wg_decode_status: container, headers, entropy stage into
                 heap memory) -- the serial part of one frame;
* pipeline       Context.decode_batch([frame]) on an explicit context (the same decode_pipelined
                 path, one chunk) and its wg_pipeline_stats: parse_s, h2d_ms, kernel_ms, d2h_ms,
                 drain_s, wall_s; `other_ms` = wall - parse - h2d - kernels - d2h (launch and
                 synchronisation overheads, allocations from the caches);
* resident_ms    the device work alone for that frame resident in HBM (wg_batch_run: K1 and,
                 for split frames, K2), HIP-event step time;
* libwebp_ms     libwebp 1.6.0 WebPDecodeRGBAInto (SIMD, 1 core) on the same frame.

Prints one JSON object; `--out FILE` also writes it."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def _median(fn, n):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--out")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime, shared with torch)

    import bench
    import webp_amd
    from oracle_lib import bench_files

    lw = None
    try:
        lw, cpu, simd = bench._libwebp()
        cpu.value = simd
    except Exception:  # noqa: BLE001
        pass
    ctx = webp_amd.Context(0)
    res = {}
    for name, data in (("c1_512", open(bench_files("c1_512")[0], "rb").read()),
                       ("c3_4k_one_frame", open(bench_files("c3_4k")[0], "rb").read())):
        f = webp_amd.features(data)
        webp_amd.decode(data)
        ent = {"pixels": f.width * f.height}
        ent["decode_ms"] = round(_median(lambda: webp_amd.decode(data), args.calls), 3)
        ent["parse_ms"] = round(_median(lambda: webp_amd.decode_status(data), args.calls), 3)
        out = [np.empty((f.height, f.width, 4), np.uint8)]
        ctx.decode_batch([data], out=out)
        walls, parts = [], []
        for _ in range(args.calls):
            t0 = time.perf_counter()
            ctx.decode_batch([data], out=out)
            walls.append((time.perf_counter() - t0) * 1e3)
            ps = ctx.pipeline_stats()
            parts.append((ps.parse_s * 1e3, ps.h2d_ms, ps.kernel_ms, ps.d2h_ms, ps.drain_s * 1e3, ps.wall_s * 1e3))
        med = [statistics.median(p[i] for p in parts) for i in range(6)]
        ent["pipeline"] = {"call_ms": round(statistics.median(walls), 3), "parse_ms": round(med[0], 3),
                           "h2d_ms": round(med[1], 3), "kernel_ms": round(med[2], 3), "d2h_ms": round(med[3], 3),
                           "drain_ms": round(med[4], 3), "wall_ms": round(med[5], 3),
                           "other_ms": round(med[5] - med[0] - med[1] - med[2] - med[3], 3)}
        b = ctx.batch([data])
        for _ in range(3):
            b.run()
        b.kernel_ms()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            b.run()
        torch.cuda.synchronize()
        ent["resident_step_ms"] = round((time.perf_counter() - t0) / args.calls * 1e3, 3)
        ent["resident_kernel_ms"] = [round(x, 3) for x in b.kernel_ms()[:2]]
        b.close()
        if lw is not None:
            o = np.empty(f.width * f.height * 4, np.uint8)
            ent["libwebp_simd_1_core_ms"] = round(_median(
                lambda: lw.WebPDecodeRGBAInto(data, len(data), o.ctypes.data, o.nbytes, 4 * f.width), args.calls), 3)
        res[name] = ent
        print(name, json.dumps(ent), file=sys.stderr, flush=True)
    ctx.close()
    s = json.dumps(res)
    print(s)
    if args.out:
        with open(args.out, "w") as fo:
            fo.write(s + "\n")


if __name__ == "__main__":
    main()
