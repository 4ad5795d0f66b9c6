#!/usr/bin/env python3
"""Per-section cycle breakdown of K3 (vp8l_transforms_kernel) on the bench workload.

Uses the timing build (make -C go-webp_amd/csrc VARIANT=timing): every wave sums
s_memtime deltas per loop section; this prints each section's share of the summed
wave-cycles.  Wave-cycles include cycles a wave spends waiting while the other waves of
its SIMD issue, so shares (not absolute values) are the useful reading.
"""
import argparse
import ctypes as C
import os
import sys

os.environ["WG_LIB_VARIANT"] = "timing"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]

NAMES = ["issue", "wait-prev", "wait-next", "ring", "steps", "slot-out", "band-start", "emit", "stage", "load"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    import torch
    import webp_amd
    from bench import WORKLOADS, _load_frames

    L = webp_amd.lib()
    L.wg_debug_k3_sections.restype = C.c_int
    L.wg_debug_k3_sections.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    datas, _ = _load_frames(WORKLOADS[args.workload]["prefix"])
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch([datas[i % len(datas)] for i in range(args.batch)])
    stream = torch.cuda.current_stream().cuda_stream
    b.run(stream)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * len(NAMES))()
    L.wg_debug_k3_sections(buf, len(NAMES), 1)  # reset after warmup
    for _ in range(args.runs):
        b.run(stream)
    torch.cuda.synchronize()
    ms = b.kernel_ms()
    L.wg_debug_k3_sections(buf, len(NAMES), 1)
    tot = sum(buf)
    print(f"workload {args.workload} batch {args.batch} runs {args.runs}: K3 {ms[2]:.3f} ms")
    for n, v in sorted(zip(NAMES, buf), key=lambda t: -t[1]):
        print(f"  {n:10s} {100.0 * v / tot:6.2f}%  {v / args.runs / 1e6:10.1f} Mcyc/run")
    # per band: start / end of its loop, % of the frame span (last run, mean over frames)
    import numpy as np
    L.wg_debug_k3_bands.restype = C.c_int
    L.wg_debug_k3_bands.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    nf = min(args.batch, 1024)
    buf2 = (C.c_ulonglong * (nf * 65 * 2))()
    L.wg_debug_k3_bands(buf2, nf)
    t = np.frombuffer(buf2, dtype=np.uint64).reshape(nf, 65, 2).astype(np.int64)
    t0 = t[:, 0, 0]
    nb = int((t[0, 1:, 1] > 0).sum())
    st, en = t[:, 1:1 + nb, 0] - t0[:, None], t[:, 1:1 + nb, 1] - t0[:, None]
    span = en.max(1)
    print(f"  frame span {span.mean() / 100:.1f} us; band start-end, % of span:")
    print("   " + " ".join(f"{k}:{100 * (st[:, k] / span).mean():.0f}-{100 * (en[:, k] / span).mean():.0f}"
                          for k in range(nb)))
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
