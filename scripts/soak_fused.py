#!/usr/bin/env python3
"""Soak check of K1's RGBA tail (cross-wave plane hand-off): a full c3 batch (256 x 4K, the
R = 12 path; `soak_fused.py <runs> c2_1080p` for 1080p, whose last quad is full) run many times; after every run a sample of frames' RGBA is hashed against the
libwebp 1.6.0 SHA-256 in the manifest.  Any mismatch (a converter reading a plane row before
its stores landed) fails the script."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-webp_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch  # noqa: F401
    import webp_amd
    from oracle_lib import bench_files, manifest
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    paths = bench_files(sys.argv[2] if len(sys.argv) > 2 else "c3_4k")  # or c2_1080p
    m = manifest()["bench"]
    want = [m[os.path.basename(p)]["sha256"]["rgba"] for p in paths]
    datas = [open(p, "rb").read() for p in paths]
    n = 256
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch([datas[i % len(datas)] for i in range(n)])
    bad = 0
    for r in range(runs):
        b.run()
        for i in range(r % 16, n, 16):  # 16 frames per run, a different slice each time
            got = hashlib.sha256(b.rgba(i).tobytes()).hexdigest()
            if got != want[i % len(datas)]:
                bad += 1
                print(f"run {r} frame {i}: MISMATCH", flush=True)
        if r % 10 == 9:
            print(f"{r + 1} runs, {bad} mismatches", flush=True)
    b.close()
    ctx.close()
    print("SOAK", "FAIL" if bad else "OK", f"({runs} runs x 16 frames checked)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
