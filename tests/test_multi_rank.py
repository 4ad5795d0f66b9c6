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


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # only rank 0 prints, one JSON line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_one_rank_per_gpu(n):
    """`bench.py --gpus N` with no launcher starts N rank processes itself (the 1->8 GPU
    curve, C4): one JSON line from rank 0 with n_gpus == N, every rank on its own
    LOCAL_RANK (= device), whole-job pixels summed over the ranks.  --mock replaces the
    device decode by a sleep, so this runs on CPU; the barrier and reduction are the real
    gloo ones."""
    out = _run_bench(["--gpus", str(n), "--mock", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.5"])
    assert out["n_gpus"] == n and out["mock"] is True
    # the end-to-end leg runs on every rank and is reduced like `value`; the CPU baseline and
    # the host's core counts stay in N > 1 lines
    assert out["end_to_end"]["n_gpus"] == n and out["end_to_end_pageable"]["n_gpus"] == n
    assert out["cpu_baseline"]["value"] > 0 and out["cpu_baseline_all_cores"]["cores"] >= 1
    assert out["host"]["nproc"] >= 1 and out["host"]["ranks"] == n
    assert 1 <= out["host"]["host_threads_per_rank"] <= max(1, out["host"]["job_cpus"] // n)
    ranks = out["ranks"]
    assert sorted(r["rank"] for r in ranks) == list(range(n))
    assert sorted(r["local_rank"] for r in ranks) == list(range(n))
    assert len({r["pid"] for r in ranks}) == n  # separate processes
    assert out["value"] > 0 and out["scaling"] == "weak"
    # every rank decoded 4 mock frames of 1000 px per step: value = n * 4000 * steps / max time
    # (value is rounded to 0.1 MPix/s, ms_per_step to 1 us)
    assert out["value"] == pytest.approx(n * 4000 * 3 / (out["ms_per_step"] * 3 * 1e-3) / 1e6, abs=0.1)


def test_bench_under_external_launcher_env():
    """Under torch.distributed.run the launcher's WORLD_SIZE / RANK / LOCAL_RANK are used and
    nothing is spawned: a single process with WORLD_SIZE=1 reports n_gpus == 1."""
    out = _run_bench(["--mock", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                     {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1
