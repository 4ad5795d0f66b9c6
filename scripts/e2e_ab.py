#!/usr/bin/env python3
"""Same-box A/B of the pipelined end-to-end decode (wg_decode_rgba_batch) over chunk settings:
one 256-frame batch of a workload into page-locked outputs, best of `reps` calls per setting,
with the pipeline's own breakdown.  Usage: e2e_ab.py [workload] [chunk settings...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch  # noqa: F401  (one HIP runtime)
    import webp_amd
    from bench import WORKLOADS, _load_frames
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    settings = [int(x) for x in sys.argv[2:]] or [0, 32, 16, 64, 256]
    datas, _ = _load_frames(WORKLOADS[wl]["prefix"])
    frames = [datas[i % len(datas)] for i in range(256)]
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    ctx = webp_amd.Context(0, host_threads=threads)
    w, h = webp_amd.features(frames[0]).width, webp_amd.features(frames[0]).height
    outs = [webp_amd.pinned_empty((h, w, 4)) for _ in frames]
    ctx.decode_batch(frames, out=outs)  # grow staging / device buffers
    px = 256 * w * h
    for rnd in range(2):
        for chunk in settings:
            ctx.set_chunk_frames(chunk)
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                _, st = ctx.decode_batch(frames, out=outs)
                dt = time.perf_counter() - t0
                assert (st == 0).all()
                ps = ctx.pipeline_stats()
                if best is None or dt < best[0]:
                    best = (dt, ps)
            dt, ps = best
            print(f"round {rnd} chunk {chunk:3d}: {dt:.4f} s = {px / dt / 1e6:7.1f} MPix/s | chunks {ps.chunks} "
                  f"parse {ps.parse_s:.4f} wait {ps.parse_wait_s:.4f} drain {ps.drain_s:.4f} "
                  f"h2d {ps.h2d_ms:.1f} kern {ps.kernel_ms:.1f} d2h {ps.d2h_ms:.1f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
