"""Mutation fuzz of the host entropy stages under ASan/UBSan (CPU only).

Builds tests/native/host_fuzz.cpp together with the product's host sources
(go-webp_amd/csrc/host/*.cpp) with -fsanitize=address,undefined and runs it over every
fixture: truncated and bit-flipped streams must come back as a status code, and successful
VP8 parses must satisfy the record/block invariants K1 relies on (its bounds come from
them).  The reference's own tests cover corrupted input only through its golden error
statuses (tests/test_alpha.py, tests/test_capi.py); this adds the memory-safety side.
"""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "go-webp_amd", "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_stages_fuzz_asan(tmp_path):
    exe = str(tmp_path / "host_fuzz")
    srcs = [os.path.join(ROOT, "tests", "native", "host_fuzz.cpp")] + sorted(glob.glob(os.path.join(HOST, "*.cpp")))
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-I", HOST, "-o", exe] + srcs)
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "lossy", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "lossless", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "anim", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "alpha", "*.webp")) +
                   glob.glob(os.path.join(ROOT, "tests", "golden", "status", "*.webp")))
    env = dict(os.environ, WG_FUZZ_ITERS="150", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe] + files, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "fuzz runs OK" in r.stdout


def test_allocation_failure_is_out_of_memory(tmp_path):
    """A 16384 x 16384 VP8L stream of zero-bit codes needs a 1 GiB coded image: under an
    address-space limit the allocation fails, and the C ABI reports OUT_OF_MEMORY (as
    WebPDecode does) instead of letting std::bad_alloc terminate the process."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_status_sweep import Bits, vp8l_file
    b = Bits()
    b.put(0, 3)
    for _ in range(5):
        b.simple(0)
    path = tmp_path / "huge.webp"
    path.write_bytes(vp8l_file(16384, 16384, b))
    lib = os.path.join(ROOT, "go-webp_amd", "webp_amd", "libgowebp_amd.so")
    code = f"""
import ctypes, resource, re
L = ctypes.CDLL({lib!r})
vm = int(re.search(r"VmSize:\\s+(\\d+)", open("/proc/self/status").read()).group(1)) * 1024
resource.setrlimit(resource.RLIMIT_AS, (vm + (512 << 20), vm + (512 << 20)))
d = open({str(path)!r}, "rb").read()
print("status", L.wg_decode_status(d, len(d), None))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "status 1" in r.stdout, r.stdout
