"""BASELINE config C4 -- 3840x2160, 2048 frames sharded over 8 GPUs (independent per frame, no
RCCL) -- in its exact layout on the one-GPU box: bench.shard_frames(datas, r, 256) for ranks
r = 0..7, each shard decoded by its own context (as each rank's process does on its own GPU in
`bench.py --gpus 8`), here one after the other on device 0 (one 256-frame 4K shard holds about
14 GB of device buffers).  Every one of the 2,048 frames is checked bit-exact on the device
(torch.equal against the eight distinct frames' decodes, themselves checked against libwebp
1.6.0's SHA-256), so 68 GB of RGBA never cross PCIe.  The reference has no multi-device code
(its only parallelism is WebPWorker, pkg/libwebp/decoder/frame_dec.c.go:611-667)."""
import hashlib
import os
import sys

import numpy as np
import pytest

import webp_amd
from oracle_lib import bench_files, manifest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c4_layout_2048_frames_over_8_shards():
    import torch
    sys.path.insert(0, ROOT)
    from bench import shard_frames
    paths = bench_files("c3_4k")
    datas = [open(p, "rb").read() for p in paths]
    want = [manifest()["bench"][os.path.basename(p)]["sha256"]["rgba"] for p in paths]
    assert len(datas) == 8
    torch.cuda.set_device(0)
    # the eight distinct frames, checked against libwebp, kept on the device
    ctx = webp_amd.Context(0, host_threads=16)
    b = ctx.batch(datas)
    assert (b.status == 0).all()
    b.run()
    ref = []
    for i in range(8):
        host = b.rgba(i)
        assert hashlib.sha256(host.tobytes()).hexdigest() == want[i], f"distinct frame {i}"
        ref.append(torch.from_numpy(host).cuda())
    b.close()
    ctx.close()
    w, h = 3840, 2160
    scratch = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    lib = webp_amd.lib()
    checked = 0
    for r in range(8):
        frames = shard_frames(datas, r, 256)
        ctx = webp_amd.Context(0, host_threads=16)
        try:
            b = ctx.batch(frames)
            assert (b.status == 0).all(), f"shard {r}: {b.status}"
            b.run()
            for i in range(b.n):
                assert b.dims(i) == (w, h)
                # device-to-device copy of frame i's RGBA (wg_batch_download_rgba into device memory)
                assert lib.wg_batch_download_rgba(b._h, i, scratch.data_ptr(), 4 * w) == 0
                torch.cuda.synchronize()  # (a device-to-device copy may return before it completes)
                assert torch.equal(scratch, ref[(r + i) % 8]), f"shard {r} frame {i} (bitstream {(r + i) % 8})"
                checked += 1
            b.close()
        finally:
            ctx.close()
    assert checked == 2048
