"""ThreadSanitizer build of the batch host stage (race detection on the host
thread pool).  tests/native/tsan_batch.cpp runs parse_all -- the worker pool and staging
arena behind wg_batch_create (go-webp_amd/csrc/host/batch_parse.cpp, staging.h) -- over the
fixtures on 9 threads, three batches in a row, and checks every frame's staged bytes against
a single-thread run.  CPU only; a data race makes TSan exit non-zero."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "go-webp_amd", "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_batch_host_stage_under_tsan(tmp_path):
    exe = str(tmp_path / "tsan_batch")
    srcs = [os.path.join(ROOT, "tests", "native", "tsan_batch.cpp")] + sorted(glob.glob(os.path.join(HOST, "*.cpp")))
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-I", HOST, "-o", exe] + srcs)
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "lossy", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "lossless", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "alpha", "*.webp")))
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe] + files, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "tsan batch OK" in r.stdout
