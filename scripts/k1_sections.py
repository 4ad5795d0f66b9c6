#!/usr/bin/env python3
"""Per-section cycle breakdown of K1 (vp8_recon_filter_kernel) on the bench workload.

Uses the timing build (make -C go-webp_amd/csrc VARIANT=timing): every wave sums
s_memtime deltas per loop section; this prints each section's share of the summed
wave-cycles.  Wave-cycles include cycles a wave spends waiting while the other waves of
its SIMD issue, so shares (not absolute values) are the useful reading.
"""
import argparse
import ctypes as C
import os
import sys

os.environ["WG_LIB_VARIANT"] = os.environ.get("K1_TIMING_VARIANT", "timing")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]

NAMES = ["prefetch", "wait", "prologue", "top", "idct", "lumapred", "i4", "chroma", "window", "filter", "deposit",
         "hbm", "rotate", "loop-tail"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    import torch
    import webp_amd
    from bench import WORKLOADS, _load_frames

    L = webp_amd.lib()
    L.wg_debug_k1_sections.restype = C.c_int
    L.wg_debug_k1_sections.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    datas, _ = _load_frames(WORKLOADS[args.workload]["prefix"])
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch([datas[i % len(datas)] for i in range(args.batch)])
    stream = torch.cuda.current_stream().cuda_stream
    b.run(stream)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * len(NAMES))()
    L.wg_debug_k1_sections(buf, len(NAMES), 1)  # reset after warmup
    for _ in range(args.runs):
        b.run(stream)
    torch.cuda.synchronize()
    ms = b.kernel_ms()
    L.wg_debug_k1_sections(buf, len(NAMES), 1)
    tot = sum(buf)
    print(f"workload {args.workload} batch {args.batch} runs {args.runs}: K1 {ms[0]:.3f} ms, K2 {ms[1]:.3f} ms")
    for n, v in sorted(zip(NAMES, buf), key=lambda t: -t[1]):
        print(f"  {n:10s} {100.0 * v / tot:6.2f}%  {v / args.runs / 1e6:10.1f} Mcyc/run")
    # timeline of the last run: per frame, how long each wave sat idle after its last pair
    L.wg_debug_k1_timeline.restype = C.c_int
    L.wg_debug_k1_timeline.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    nf = min(args.batch, 1024)
    tl = (C.c_ulonglong * (nf * 33))()
    L.wg_debug_k1_timeline(tl, nf)
    import numpy as np
    t = np.frombuffer(tl, dtype=np.uint64).reshape(nf, 33).astype(np.int64)
    start, ends, kend = t[:, :1], t[:, 1:17], t[:, 17:]
    dur = ends.max(1) - start[:, 0]
    idle = (ends.max(1, keepdims=True) - ends).sum(1) / (16.0 * dur)
    srt = np.sort(ends - start, axis=1)
    print(f"timeline (100 MHz ticks): frame span mean {dur.mean() / 100:.1f} us (min {dur.min() / 100:.1f}, "
          f"max {dur.max() / 100:.1f}); idle wave-time after exit {100 * idle.mean():.1f}%")
    print("  mean exit time of the k-th wave to finish, % of frame span:",
          " ".join(f"{100 * (srt[:, k] / dur).mean():.0f}" for k in range(16)))
    print("  mean reconstruction exit per wave index, % of span:",
          " ".join(f"{100 * ((ends[:, w] - start[:, 0]) / dur).mean():.0f}" for w in range(16)))
    fend = kend.max(1) - start[:, 0]
    print(f"  frame end (last wave leaves the kernel) {100 * (fend / dur).mean():.1f}% of the reconstruction span "
          f"({fend.mean() / 100:.1f} us)")
    L.wg_debug_k1_quads.restype = C.c_int
    L.wg_debug_k1_quads.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    qb = (C.c_ulonglong * (nf * 64 * 2))()
    L.wg_debug_k1_quads(qb, nf)
    q = np.frombuffer(qb, dtype=np.uint64).reshape(nf, 64, 2).astype(np.int64)
    nq = int((q[0, :, 1] > 0).sum())
    rel = lambda v: 100 * ((v - start) / dur[:, None]).mean(0)
    qs, qe = rel(q[:, :nq, 0]), rel(q[:, :nq, 1])
    print("  quad start/end, % of span:", " ".join(f"{k}:{a:.0f}-{b:.0f}" for k, (a, b) in enumerate(zip(qs, qe))))
    st = start[:, 0] - start.min()
    print(f"  frame start spread {st.max() / 100:.1f} us; kernel span {(ends.max() - start.min()) / 100:.1f} us")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
