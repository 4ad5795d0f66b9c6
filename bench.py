#!/usr/bin/env python3
"""bench.py -- decoded MPix/s of the MI355X WebP decode path, one process per GPU.

Metric (BASELINE.json): "decoded MPixels/sec at 1/2/4/8 GPUs; % HBM roofline (YUV->RGBA)".

A step = one pass of the device decode path over one resident batch of frames: by default
config C3, 256 x 3840x2160 VP8-lossy frames with the in-loop deblocking
filter (K1: Y2 WHT + IDCT + reconstruction + deblocking + YUV420->RGBA in its tail), 8
distinct libwebp-encoded synthetic bitstreams cycled (each frame has its own HBM buffers).
The entropy stage (host) and the H2D upload happen before the timed region: `value` is
device throughput with inputs resident in HBM.

Multi-GPU: every rank decodes its own `--batch` frames on its own GPU
(weak scaling); ranks exchange nothing on the data path.  `--gpus N` without a launcher
spawns N rank processes itself (before anything touches a GPU); under torch.distributed.run
the launcher's RANK / LOCAL_RANK / WORLD_SIZE are used.  The timing barrier and the
max-time / sum-pixels reduction go over gloo (host sockets), not RCCL.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-webp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)

WORKLOADS = {
    "c2": dict(prefix="c2_1080p", name="c2_1080p_x256", desc="1920x1080 VP8-lossy (deblock on), batch 256"),
    "c3": dict(prefix="c3_4k", name="c3_4k_deblock_x256", desc="3840x2160 VP8-lossy, deblock on, batch 256"),
    "c3s": dict(prefix="c3s_4k", name="c3s_4k_deblock_x256",
                desc="3840x2160 VP8-lossy, sigma 18 (~2 bpp: SURVEY 8(d)'s entropy-stress variant of C3), deblock on, "
                     "batch 256"),
    "c5": dict(prefix="c5_ll2048", name="c5_ll2048_x256",
               desc="2048x2048 VP8L lossless (predictor + cross-color + subtract-green + color cache), batch 256"),
    # SURVEY §8's "next" rows, each measured with its kernel's roofline (`roofline_target`)
    "c3a": dict(prefix="c3a_4k", name="c3a_4k_alpha_x256", target="alpha_kernel",
                desc="3840x2160 VP8-lossy + ALPH (lossless-compressed feathered cut-out alpha), deblock on, batch 256: "
                     "K1 + the alpha streams' K7 / K3 + K4 (SURVEY 8 f2)"),
    "c3ag": dict(prefix="c3ag_4k", name="c3ag_4k_alpha_gradient_x256", target="alpha_kernel",
                 desc="C3a's frames with the ALPH filter set to gradient (libwebp's GradientUnfilter: a 2-D "
                      "wavefront), batch 256: K1 + the alpha streams' K7 / K3 + K4 (SURVEY 8 f2)"),
    "c3av": dict(prefix="c3av_4k", name="c3av_4k_alpha_vertical_x256", target="alpha_kernel",
                 desc="C3a's frames with the ALPH filter set to vertical (column running sums), batch 256: "
                      "K1 + the alpha streams' K7 / K3 + K4 (SURVEY 8 f2)"),
    "c3rgb565": dict(prefix="c3_4k", name="c3_4k_rgb565_x256", target="vp8_recon_filter_kernel", colorspace=6,
                     desc="C3's frames decoded to MODE_RGB_565 (fancy upsampling), batch 256: K1, whose tail writes "
                          "the 565 pixels directly (no RGBA copy, no K6) (SURVEY 8 f4)"),
    "anim": dict(prefix="anim_1080p_x64", name="anim_1080p_x64", target="anim_compose_kernel", kind="anim",
                 desc="one 64-frame 1920x1080 lossy animation per GPU (WebPAnimEncoder: blended sub-rectangles), "
                      "resident: frames K1..K4, 64 canvases K5; value = canvas pixels / s (SURVEY 8 f3)"),
}
# the order of Batch.kernel_ms() / kernel_bytes(): K1, K2, K3, K4, K7, K6, K5
KERNELS = ("vp8_recon_filter_kernel", "yuv_to_rgba_kernel", "vp8l_transforms_kernel", "alpha_kernel",
           "vp8l_resolve_kernel", "emit_kernel", "anim_compose_kernel")


def _load_frames(prefix):
    from oracle_lib import GOLDEN, bench_files, manifest
    ent = manifest().get("bench_anim", {}).get(prefix)
    if ent is not None:  # one animation file: bits per canvas pixel
        data = open(os.path.join(GOLDEN, "bench", prefix + ".webp"), "rb").read()
        inf = ent["info"]
        return [data], 8.0 * len(data) / (inf["canvas_width"] * inf["canvas_height"] * inf["frame_count"])
    paths = bench_files(prefix)
    datas = [open(p, "rb").read() for p in paths]
    m = manifest()["bench"]
    bpp = sum(m[os.path.basename(p)]["bpp"] for p in paths) / len(paths)
    return datas, bpp


def _traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 --pmc measurement, if present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except Exception:
        return None


def _valu_ceiling():
    """Static-mix VALU issue ceilings per kernel (scripts/valu_ceiling.py), if present."""
    p = os.path.join(ROOT, "profiles", "valu_ceiling.json")
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


CUS = 256  # MI355X compute units (4 SIMDs each)


def valu_roof(kernel, workload, ms, n_workgroups):
    """The instruction-issue ceiling of a kernel that is not HBM-bound: measured VALU
    wave-instructions per launch (committed SQ_INSTS_VALU, profiles/pmc_traffic.json) over the
    SIMDs its workgroups occupy and this run's launch time, against the probe-based ceiling for
    its instruction mix (profiles/valu_ceiling.json); plus VALUUtilization (active lanes)."""
    tr = ((_traffic(workload) or {}).get(kernel) or {}).get("valu")
    ce = _valu_ceiling().get(kernel)
    if not tr or not ce or ms <= 0:
        return None
    simds = 4 * min(CUS, max(1, n_workgroups))
    ach = tr["insts_valu"] / (simds * ms * 1e6)
    peak = ce["ceiling_valu_per_ns_per_simd"]
    return {"bound": "valu", "achieved": round(ach, 4), "peak": peak, "unit": "VALU wave-instr / ns / SIMD",
            "frac": round(ach / peak, 4), "insts_valu_per_launch": tr["insts_valu"], "simds": simds,
            "valu_utilization": tr.get("valu_utilization"),
            "note": "issue rate from the committed SQ_INSTS_VALU (rocprofv3 --pmc) over this run's launch time; "
                    "peak = probe-measured issue cost of the kernel's static instruction mix (DESIGN.md 4)"}


def shard_frames(datas, rank, batch):
    """Frames of one rank: `batch` frames cycling the distinct bitstreams, offset by rank
    (independent frames, no exchange between ranks -- SURVEY §8(e))."""
    return [datas[(rank + i) % len(datas)] for i in range(batch)]


def reduce_job(dist, device, dt, pixels):
    """Whole-job figures over all ranks: (max elapsed seconds, total pixels).  `dist` None =
    single process; otherwise an initialised torch.distributed gloo group (CPU tensors)."""
    if dist is None:
        return dt, pixels
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    p = torch.tensor([float(pixels)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(p, op=dist.ReduceOp.SUM)
    return float(t.item()), int(p.item())


# ------------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, timeout=None):
    """Run `bench.py argv` as n rank processes (RANK = LOCAL_RANK = r, WORLD_SIZE = n, gloo
    rendezvous on 127.0.0.1) and return the worst exit code.  The parent never touches a GPU:
    each rank initialises only its own device.  If a rank fails, the others are stopped (their
    exact PIDs) instead of waiting at the barrier."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    t0 = time.time()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:
                    q.kill()
        if timeout is not None and time.time() - t0 > timeout:
            for q in live:
                q.kill()
            return 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


# ------------------------------------------------------------------------------- CPU legs
def _cpu_decode_one(d, wl=None):
    """One frame (an animation: all its canvases) through the CPU path (host entropy stage +
    oracle) as the workload `wl` needs it; returns its pixels."""
    import webp_amd
    from oracle_lib import oracle_anim, oracle_decode, oracle_output, oracle_still_rgba, oracle_vp8l_decode
    wl = wl or {}
    if wl.get("kind") == "anim":
        canv, _ = oracle_anim(d)
        return canv.shape[0] * canv.shape[1] * canv.shape[2]
    if wl.get("colorspace") is not None:
        out = oracle_output(d, mode=wl["colorspace"])
        f = webp_amd.features(d)
        assert out is not None
        return f.width * f.height
    if wl.get("target") == "alpha_kernel":
        rgba = oracle_still_rgba(d)
        return rgba.shape[0] * rgba.shape[1]
    if webp_amd.features(d).format == 2:
        info, coded, tdata = webp_amd.vp8l_parse(d)
        oracle_vp8l_decode(info, coded, tdata)
    else:
        info, mbs = webp_amd.vp8_parse(d)
        oracle_decode(info, mbs)
    return info.width * info.height


def cpu_baseline(datas, seconds, wl=None):
    """CPU oracle (C restatement, 1 thread): host entropy stage + reconstruct + filter +
    fancy RGBA (+ the workload's alpha / colorspace / compositing), frames decoded serially
    until `seconds` elapse."""
    pix, n, t0 = 0, 0, time.perf_counter()
    while True:
        d = datas[n % len(datas)]
        pix += _cpu_decode_one(d, wl)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return dict(value=pix / el / 1e6, unit="MPix/s", cores=1, kind="port",
                sample=f"{n} frames of the same workload decoded serially on 1 host core "
                       f"(host entropy stage + oracle/ CPU restatement of the device path), {el:.1f}s")


def cpu_baseline_dsp(datas, seconds):
    """The same CPU restatement on pre-parsed frames (entropy stage outside the timing): the
    work the device kernels do, timed on 1 host core -- the like-for-like baseline for
    `value`."""
    import webp_amd
    from oracle_lib import oracle_decode, oracle_vp8l_decode
    parsed = []
    for d in datas:
        if webp_amd.features(d).format == 2:
            parsed.append(("ll", webp_amd.vp8l_parse(d)))
        else:
            parsed.append(("vp8", webp_amd.vp8_parse(d)))
    pix, n, t0 = 0, 0, time.perf_counter()
    while True:
        kind, p = parsed[n % len(parsed)]
        if kind == "ll":
            oracle_vp8l_decode(*p)
        else:
            oracle_decode(*p)
        pix += p[0].width * p[0].height
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return dict(value=pix / el / 1e6, unit="MPix/s", cores=1, kind="port",
                sample=f"{n} pre-parsed frames through the oracle/ CPU restatement of the device path "
                       f"(reconstruct + filter + RGBA, or the VP8L inverse transforms) on 1 host core, {el:.1f}s")


def cpu_baseline_parallel(datas, seconds, threads, wl=None):
    """The same CPU path on `threads` host threads, frames decoded concurrently (ctypes
    releases the GIL inside the entropy stage and the oracle)."""
    import threading
    import webp_amd
    from oracle_lib import oracle
    oracle()
    webp_amd.lib()
    _cpu_decode_one(datas[0], wl)
    pix = [0] * threads
    cnt = [0] * threads
    t0 = time.perf_counter()
    stop = t0 + seconds

    def work(t):
        n = t
        while time.perf_counter() < stop:
            pix[t] += _cpu_decode_one(datas[n % len(datas)], wl)
            cnt[t] += 1
            n += threads

    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    return dict(value=sum(pix) / el / 1e6, unit="MPix/s", cores=threads, kind="port",
                sample=f"{sum(cnt)} frames of the same workload on {threads} host threads "
                       f"(entropy stage + oracle/ CPU restatement), {el:.1f}s")


def _libwebp():
    """libwebp 1.6.0 as Pillow bundles it (the upstream the reference translates,
    pkg/vp8/constants.go:18-20), loaded by ctypes: a real-world CPU decoder to set beside the
    restatement.  Returns (lib, cpuinfo pointer cell, its SIMD value) or raises."""
    import ctypes as C
    import glob
    import PIL
    libs = os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs")
    C.CDLL(glob.glob(os.path.join(libs, "libsharpyuv-*.so*"))[0], mode=C.RTLD_GLOBAL)
    lib = C.CDLL(glob.glob(os.path.join(libs, "libwebp-*.so*"))[0])
    ver = lib.WebPGetDecoderVersion()
    if ver != 0x010600:
        raise RuntimeError(f"libwebp version {ver:#x}, not 1.6.0")
    lib.WebPDecodeRGBAInto.restype = C.c_void_p
    lib.WebPDecodeRGBAInto.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    cpu = C.c_void_p.in_dll(lib, "VP8GetCPUInfo")
    return lib, cpu, cpu.value


def cpu_baseline_libwebp(datas, seconds, threads=1, simd=True):
    """libwebp 1.6.0's WebPDecodeRGBAInto (the C library the reference is a translation of) on
    `threads` host threads, with its SIMD kernels or, simd=False, its plain-C ones
    (VP8GetCPUInfo = NULL, the code the reference's Go translates).  Frames decoded until
    `seconds` elapse; ctypes releases the GIL inside the call."""
    import threading
    import webp_amd
    lib, cpu, simd_ptr = _libwebp()
    cpu.value = simd_ptr if simd else None
    dims = [(webp_amd.features(d).width, webp_amd.features(d).height) for d in datas]
    outs = [np.empty(max(w * h * 4 for w, h in dims), np.uint8) for _ in range(threads)]
    # warm-up: runs libwebp's DSP init for this cpuinfo setting before the threads start
    w0, h0 = dims[0]
    if not lib.WebPDecodeRGBAInto(datas[0], len(datas[0]), outs[0].ctypes.data, outs[0].nbytes, 4 * w0):
        raise RuntimeError("WebPDecodeRGBAInto failed")
    pix, cnt = [0] * threads, [0] * threads
    t0 = time.perf_counter()
    stop = t0 + seconds

    def work(t):
        n = t
        o = outs[t]
        while time.perf_counter() < stop:
            d = datas[n % len(datas)]
            w, h = dims[n % len(datas)]
            lib.WebPDecodeRGBAInto(d, len(d), o.ctypes.data, o.nbytes, 4 * w)
            pix[t] += w * h
            cnt[t] += 1
            n += threads

    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    cpu.value = simd_ptr
    return dict(value=round(sum(pix) / el / 1e6, 2), unit="MPix/s", cores=threads, kind="libwebp-1.6.0",
                simd=simd, sample=f"{sum(cnt)} frames of the same workload through libwebp 1.6.0 WebPDecodeRGBAInto "
                                  f"({'SIMD' if simd else 'plain-C'} DSP, Pillow's bundled build) on {threads} "
                                  f"host thread(s), {el:.1f}s")


def _libwebp_frame_fn(wl, lib):
    """A callable decoding one input with libwebp 1.6.0 as the workload needs it -> pixels out:
    WebPDecode with a WebPDecoderConfig (output colorspace) for a colorspace workload, the
    WebPAnimDecoder loop (every canvas, MODE_RGBA; libwebpdemux) for the animation one, else
    WebPDecodeRGBAInto (see cpu_baseline_libwebp)."""
    import ctypes as C
    import glob
    import PIL
    abi = 0x0210  # WEBP_DECODER_ABI_VERSION of 1.6.0
    if wl.get("colorspace") is not None:
        mode = wl["colorspace"]

        def dec(d):
            cfg = (C.c_uint8 * 512)()
            assert lib.WebPInitDecoderConfigInternal(cfg, abi)
            ci = C.cast(cfg, C.POINTER(C.c_int32))
            ci[40 // 4] = mode  # config.output.colorspace
            assert lib.WebPDecode(d, C.c_size_t(len(d)), cfg) == 0
            px = ci[44 // 4] * ci[48 // 4]
            lib.WebPFreeDecBuffer(C.byref(cfg, 40))
            return px
        return dec
    if wl.get("kind") == "anim":
        libs = os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs")
        dmx = C.CDLL(glob.glob(os.path.join(libs, "libwebpdemux-*.so*"))[0])
        dmx.WebPAnimDecoderNewInternal.restype = C.c_void_p
        dmx.WebPAnimDecoderNewInternal.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        for f in ("WebPAnimDecoderGetInfo", "WebPAnimDecoderGetNext"):
            getattr(dmx, f).argtypes = [C.c_void_p] + [C.c_void_p] * (1 if f.endswith("Info") else 2)
        dmx.WebPAnimDecoderHasMoreFrames.argtypes = [C.c_void_p]
        dmx.WebPAnimDecoderDelete.argtypes = [C.c_void_p]

        class _Data(C.Structure):
            _fields_ = [("bytes", C.c_void_p), ("size", C.c_size_t)]

        def dec(d):
            opt = (C.c_int32 * 9)()
            assert dmx.WebPAnimDecoderOptionsInitInternal(opt, 0x0107)  # WEBP_DEMUX_ABI_VERSION
            opt[0] = 1  # MODE_RGBA
            buf = C.c_char_p(d)
            wd = _Data(C.cast(buf, C.c_void_p).value, len(d))
            h = dmx.WebPAnimDecoderNewInternal(C.byref(wd), opt, 0x0107)
            info = (C.c_uint32 * 9)()
            dmx.WebPAnimDecoderGetInfo(h, info)
            px = 0
            out, ts = C.c_void_p(), C.c_int()
            while dmx.WebPAnimDecoderHasMoreFrames(h):
                dmx.WebPAnimDecoderGetNext(h, C.byref(out), C.byref(ts))
                px += info[0] * info[1]
            dmx.WebPAnimDecoderDelete(h)
            return px
        return dec
    return None


def cpu_baseline_libwebp_wl(datas, seconds, threads, simd, wl):
    """cpu_baseline_libwebp for the colorspace / animation workloads (_libwebp_frame_fn)."""
    import threading
    lib, cpu, simd_ptr = _libwebp()
    dec = _libwebp_frame_fn(wl, lib)
    cpu.value = simd_ptr if simd else None
    dec(datas[0])
    pix, cnt = [0] * threads, [0] * threads
    t0 = time.perf_counter()
    stop = t0 + seconds

    def work(t):
        n = t
        while time.perf_counter() < stop:
            pix[t] += dec(datas[n % len(datas)])
            cnt[t] += 1
            n += threads

    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    cpu.value = simd_ptr
    what = "WebPAnimDecoder, every canvas" if wl.get("kind") == "anim" else f"WebPDecode to colorspace {wl['colorspace']}"
    return dict(value=round(sum(pix) / el / 1e6, 2), unit="MPix/s", cores=threads, kind="libwebp-1.6.0", simd=simd,
                sample=f"{sum(cnt)} inputs of the same workload through libwebp 1.6.0 {what} "
                       f"({'SIMD' if simd else 'plain-C'} DSP, Pillow's bundled build) on {threads} host thread(s), {el:.1f}s")


def cpu_baselines_libwebp(datas, seconds, threads, wl=None):
    """1-core SIMD, 1-core plain-C and all-cores SIMD libwebp figures, or the reason there are none."""
    wl = wl or {}
    try:
        if wl.get("kind") == "anim" or wl.get("colorspace") is not None:
            f = lambda th, simd: cpu_baseline_libwebp_wl(datas, seconds, th, simd, wl)  # noqa: E731
        else:
            f = lambda th, simd: cpu_baseline_libwebp(datas, seconds, th, simd)  # noqa: E731
        return {"simd_1_core": f(1, True), "plain_c_1_core": f(1, False), "simd_all_cores": f(threads, True)}
    except Exception as e:  # noqa: BLE001 -- recorded in the line, never fatal
        return {"unavailable": f"{type(e).__name__}: {e}"}


# ------------------------------------------------------------------------------- host cores
def host_cpus():
    """CPUs this job may use: the affinity mask, bounded by the cgroup's CPU quota (a GPU box
    grants a share of a larger machine: os.cpu_count() shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def rank_host_threads(requested, world):
    """Entropy-stage threads of one rank: --host-threads, capped at the job's CPUs / ranks."""
    return max(1, min(requested, 64, host_cpus() // max(1, world)))


def host_info(world, threads):
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        nproc = None
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": nproc, "os_cpu_count": os.cpu_count(), "job_cpus": host_cpus(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model, "ranks": world,
            "host_threads_per_rank": threads}


def end_to_end(args, ctx, b, frames, dist, barrier, px_rank, threads):
    """Host bitstreams in, host RGBA out, on EVERY rank at once (each its own shard and GPU):
    entropy stage on the rank's host threads + H2D + kernels + D2H, pipelined in chunks
    (wg_decode_rgba_batch).  Outputs allocated outside the timing: page-locked (written by
    DMA, the `end_to_end` figure) and pageable numpy memory (`end_to_end_pageable`).  Whole-job
    value = all ranks' pixels / the slowest rank's time; best of two calls (the first also grows
    the context's pinned staging and device buffers)."""
    res = {}
    for kind in ("pinned", "pageable"):
        if args.mock:
            outs = None
        elif kind == "pinned":
            import webp_amd
            outs = [webp_amd.pinned_empty((b.dims(i)[1], b.dims(i)[0], 4)) for i in range(b.n)]
        else:
            outs = [np.empty((b.dims(i)[1], b.dims(i)[0], 4), np.uint8) for i in range(b.n)]
            for o in outs:
                o.fill(0)  # fault the pages in outside the timing
        runs = []
        for _ in range(2):
            barrier()
            t_e = time.perf_counter()
            ctx.decode_batch(frames, out=outs)
            t_e = time.perf_counter() - t_e
            t_max, px = reduce_job(dist, "cpu", t_e, px_rank)
            runs.append((t_max, t_e, ctx.pipeline_stats().as_dict()))
        t_max, t_mine, ps = min(runs, key=lambda r: r[0])
        world = 1 if dist is None else dist.get_world_size()
        res[kind] = {"value": round(px / t_max / 1e6, 1), "unit": "MPix/s", "n_gpus": world,
                     "seconds": round(t_max, 4), "seconds_first_call": round(runs[0][0], 4),
                     "host_threads_per_rank": threads, "output_memory": kind,
                     "breakdown_rank0": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in ps.items()},
                     "note": "host entropy stage + H2D + kernels + D2H, pipelined in chunks on every rank; "
                             "host-bound; not the headline value"}
        del outs
    return res


class _MockContext:
    """--mock: stand-in for webp_amd.Context's end-to-end entry."""

    def decode_batch(self, frames, out=None):
        time.sleep(0.003)

    def pipeline_stats(self):
        class _PS:
            def as_dict(self):
                return {"chunks": 1, "wall_s": 0.003}
        return _PS()

    def close(self):
        pass


# ------------------------------------------------------------------------------- one rank
class _MockBatch:
    """--mock (CPU tests of the launcher): a stand-in for webp_amd.Batch that sleeps instead of
    decoding, so the rank / reduction / JSON plumbing runs without a GPU."""
    n = 4
    pixels = 4 * 1000

    def run(self, stream=None):
        time.sleep(0.002)

    def kernel_ms(self):
        return (0.0,) * len(KERNELS)

    def kernel_bytes(self):
        return (0.0,) * len(KERNELS)

    def close(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host in, host out) leg")
    ap.add_argument("--emit", choices=("fused", "separate"), default="fused",
                    help="lossy RGBA from K1's tail (default) or a separate K2 launch")
    ap.add_argument("--host-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="entropy-stage threads per rank, capped at the job's host CPUs / ranks")
    ap.add_argument("--mock", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start one rank per GPU ourselves, before anything touches a GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0 and args.gpus != 1:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    import torch
    dist = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        # Gloo reports each rank's connections on the C-level stdout: route them to stderr so that
        # stdout carries only rank 0's JSON line (the driver's contract)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    def barrier():
        if dist is not None:
            dist.barrier()

    wl = WORKLOADS[args.workload]
    oversubscribed = False
    if args.mock:
        datas, bpp = _load_frames(wl["prefix"])  # (the CPU baseline legs still run for real)
        b, ctx, t_prep, stream = _MockBatch(), _MockContext(), 0.0, None
        frames, ctx_threads = None, rank_host_threads(args.host_threads, world)
        sync = lambda: None  # noqa: E731
    else:
        import webp_amd
        # one GPU per rank; more ranks than GPUs (a rehearsal of the multi-rank path on a small box)
        # share devices round-robin and say so in the line (`oversubscribed`: not a scaling figure)
        ndev = torch.cuda.device_count()
        device = local % max(1, ndev)
        oversubscribed = world > ndev
        torch.cuda.set_device(device)
        datas, bpp = _load_frames(wl["prefix"])
        ctx_threads = rank_host_threads(args.host_threads, world)
        ctx = webp_amd.Context(device, host_threads=ctx_threads)
        t_prep = time.perf_counter()
        if wl.get("kind") == "anim":  # one animation per rank, resident (frames + canvases)
            frames = None
            b = ctx.anim_batch(datas[rank % len(datas)])
        else:
            frames = shard_frames(datas, rank, args.batch)
            opts = webp_amd.options(wl["colorspace"]) if wl.get("colorspace") is not None else None
            b = ctx.batch(frames, opts=opts)
        t_prep = time.perf_counter() - t_prep
        if not (b.status == 0).all():
            raise SystemExit(f"rank {rank}: frames failed to parse: {b.status}")
        stream = torch.cuda.current_stream().cuda_stream
        if wl.get("kind") != "anim":
            b.set_emit(args.emit == "separate")
        sync = torch.cuda.synchronize

    for _ in range(args.warmup):
        b.run(stream)
    sync()
    b.kernel_ms()  # drop warmup timings

    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.run(stream)
    sync()
    barrier()
    dt = time.perf_counter() - t0
    kms = list(b.kernel_ms())  # per-launch averages over the timed steps (HIP events): K1..K4
    kby = b.kernel_bytes()
    stage_ms = 0.0
    if kms[0] > 0 and kms[1] == 0:
        # the metric's YUV->RGBA stage, which K1's tail performs inside the timed steps, timed
        # alone (K2 over the same reconstructed planes) for its own roofline figure
        for _ in range(2):
            b.run_emit(stream)
        sync()
        b.kernel_ms()
        for _ in range(args.steps):
            b.run_emit(stream)
        stage_ms = b.kernel_ms()[1]
    # pixels per step: decoded frame pixels (an animation: every canvas it composites)
    px_rank = b.pixels if wl.get("kind") != "anim" or args.mock else b.n * b.canvas_width * b.canvas_height
    dt, total_px = reduce_job(dist, "cpu", dt, px_rank * args.steps)
    e2e = None
    # the end-to-end leg (host in, host out through wg_decode_rgba_batch) exists for RGBA stills
    if not args.no_e2e and wl.get("kind") != "anim" and wl.get("colorspace") is None:
        e2e = end_to_end(args, ctx, b, frames if not args.mock else None, dist, barrier, px_rank, ctx_threads)
    value = total_px / dt / 1e6
    ranks = [(rank, local, os.getpid())]
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, local, os.getpid()))
        ranks = gathered

    frames_per_gpu = b.n if wl.get("kind") == "anim" and not args.mock else args.batch
    if rank == 0:
        def roof(bytes_, ms, kernel):
            ach = bytes_ / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            tr = _traffic(wl["name"])
            return {"kernel": kernel, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": ((tr or {}).get(kernel) or {}).get("bytes"), "algorithmic_bytes": int(bytes_),
                    "avg_launch_ms": round(ms, 4)}
        ran = [k for k in range(len(KERNELS)) if kms[k] > 0]
        roofs = {KERNELS[k]: roof(kby[k], kms[k], KERNELS[k]) for k in ran}
        for k in ran:  # the second ceiling: instruction issue (K2 spreads over every CU)
            vr = valu_roof(KERNELS[k], wl["name"], kms[k], CUS if k == 1 else args.batch)
            if vr:
                roofs[KERNELS[k]]["valu"] = vr
                # the ceiling the kernel is closest to (the contract's `bound` names the HBM roofline)
                roofs[KERNELS[k]]["binding"] = "valu" if vr["frac"] > roofs[KERNELS[k]]["frac"] else "hbm"
        dominant = roofs[KERNELS[max(ran, key=lambda k: kms[k])]] if ran else None
        target = roofs.get(wl.get("target")) if wl.get("target") else None
        if dominant and dominant["kernel"] == "vp8_recon_filter_kernel":
            # measured limiter: instruction issue / latency on the frame's CU, not HBM
            dominant["limiter"] = "VALU instruction issue on the frame's CU (roofline.valu; DESIGN.md §4)"
        if stage_ms > 0:
            roofs["yuv_to_rgba_kernel"] = dict(roof(kby[1], stage_ms, "yuv_to_rgba_kernel"),
                                               note="stage timed alone over the same planes; in the "
                                                    "timed steps K1's tail performs it (--emit fused)")
            vr = valu_roof("yuv_to_rgba_kernel", wl["name"], stage_ms, CUS)
            if vr:
                roofs["yuv_to_rgba_kernel"]["valu"] = vr
                roofs["yuv_to_rgba_kernel"]["binding"] = ("valu" if vr["frac"] > roofs["yuv_to_rgba_kernel"]["frac"]
                                                          else "hbm")
        out = {
            "metric": "decoded MPixels/sec at 1/2/4/8 GPUs; % HBM roofline (YUV->RGBA)",
            "value": round(value, 1),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (SURVEY App. B frames encoded by libwebp 1.6.0, committed bitstreams)",
            "config": {"workload": wl["name"], "description": wl["desc"], "frames_per_gpu": frames_per_gpu,
                       "frames_total": frames_per_gpu * world,
                       "distinct_bitstreams": len(datas), "input_bpp": round(bpp, 3),
                       "parallelism": f"frame-sharded over {world} GPU(s), one process each, no collectives "
                                      f"(gloo barrier + timing reduction only)",
                       "inputs": "resident in HBM (host entropy stage + H2D outside the timed region)"},
            "roofline": dominant,
            "kernel_ms": {KERNELS[k]: round(kms[k], 4) for k in ran},
            "roofline_all": roofs,
            "lossy_emit": args.emit if kms[0] > 0 else None,
            "host_prepare_s": round(t_prep, 3),
            "ranks": [{"rank": r, "local_rank": lr, "pid": pid} for r, lr, pid in sorted(ranks)],
        }
        if args.mock:
            out["mock"] = True
        if oversubscribed:
            out["oversubscribed"] = ("more ranks than GPUs: ranks share devices round-robin; a rehearsal of the "
                                     "multi-rank path, not a scaling figure")
        if "yuv_to_rgba_kernel" in roofs:
            out["roofline_yuv_to_rgba"] = roofs["yuv_to_rgba_kernel"]
        if target is not None:  # the kernel this "next"-row workload exists for
            out["roofline_target"] = target
        if e2e is not None:
            out["end_to_end"] = e2e["pinned"]
            out["end_to_end_pageable"] = e2e["pageable"]
        out["host"] = host_info(world, ctx_threads)
        if not args.no_cpu_baseline:
            # rank 0 only, on the host cores of this job; the other ranks wait at the final barrier
            cb = cpu_baseline(datas, args.cpu_seconds, wl)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1)
            if not wl.get("target"):  # (the pre-parsed leg restates the (a) rows only)
                cbd = cpu_baseline_dsp(datas, max(2.0, args.cpu_seconds / 2))
                out["cpu_baseline_dsp"] = cbd
                out["speedup_vs_cpu_dsp"] = round(value / cbd["value"], 1)
            threads = max(1, min(64, host_cpus()))  # every CPU of the job
            cba = cpu_baseline_parallel(datas, max(2.0, args.cpu_seconds / 2), threads, wl)
            out["cpu_baseline_all_cores"] = cba
            out["speedup_vs_cpu_all_cores"] = round(value / cba["value"], 1)
            if "end_to_end" in out:
                out["end_to_end"]["vs_cpu_all_cores"] = round(out["end_to_end"]["value"] / cba["value"], 2)
                out["end_to_end"]["vs_cpu_1_core"] = round(out["end_to_end"]["value"] / cb["value"], 1)
            # a real-world CPU decoder beside the restatement (not the contract's cpu_baseline)
            lw = cpu_baselines_libwebp(datas, max(2.0, args.cpu_seconds / 4), threads, wl)
            out["cpu_baseline_libwebp"] = lw
            if "simd_1_core" in lw:
                out["speedup_vs_libwebp_simd_1_core"] = round(value / lw["simd_1_core"]["value"], 1)
                out["speedup_vs_libwebp_simd_all_cores"] = round(value / lw["simd_all_cores"]["value"], 1)
                if "end_to_end" in out:
                    out["end_to_end"]["vs_libwebp_simd_all_cores"] = round(
                        out["end_to_end"]["value"] / lw["simd_all_cores"]["value"], 2)
        print(json.dumps(out), flush=True)
    barrier()
    b.close()
    if ctx is not None:
        ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
