"""N>1 path of bench.py on CPU: world_size-2 gloo processes (frames shard
across GPUs with no data-path collective; the only cross-rank traffic is the timing
reduction).  Exercises bench.shard_frames and bench.reduce_job exactly as the 8-GPU run
uses them, with the gloo backend instead of nccl."""
import os
import socket

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        datas = [b"f0", b"f1", b"f2"]
        frames = bench.shard_frames(datas, rank, 4)
        # rank r: 4 frames of (r+1)*1000 px, elapsed 1.0 + r seconds
        dt, px = bench.reduce_job(dist, "cpu", 1.0 + rank, 4 * (rank + 1) * 1000)
        q.put((rank, frames, dt, px))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_reduction_and_sharding():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, frames, dt, px = q.get(timeout=120)
        res[rank] = (frames, dt, px)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards: rank-offset cycling, independent per rank
    assert res[0][0] == [b"f0", b"f1", b"f2", b"f0"]
    assert res[1][0] == [b"f1", b"f2", b"f0", b"f1"]
    # whole-job: max time over ranks, sum of pixels over ranks, identical on every rank
    for r in (0, 1):
        assert res[r][1] == pytest.approx(2.0)
        assert res[r][2] == 4 * 1000 + 4 * 2000


def test_single_process_reduce_is_identity():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.reduce_job(None, "cpu", 1.5, 123) == (1.5, 123)
