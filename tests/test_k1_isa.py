"""Static ISA guards for K1 (device/vp8_recon_filter.hip) and K2 (device/yuv_to_rgba.hip).

K1 sits at gfx950's 128-VGPR budget for four waves per SIMD, and its register state is easy to
push into spills by an innocent-looking change: a lane test hoisted out of a loop becomes a 64-bit
SGPR mask held across it, eight such masks push the quad loop's state into v_readlane /
v_writelane spills, a VGPR pushed out goes to scratch memory.  Round 5 had 2 VGPR spills (12 B of
scratch per lane) and 106 SGPR spills in K1's product instantiation.  This test compiles the
kernels for gfx950 exactly as the Makefile does (to assembly: the markers inside inline asm
survive there) and checks:

1. every K1 instantiation: no VGPR spill, no private (scratch) segment, no scratch instruction;
2. K1's MB step loop (the hot path: one iteration per wave step of four MBs): SGPR-spill
   reloads (v_readlane from a VGPR lane, no memory) only on the progress-wait timeout path (the
   one that reports the error with `global_atomic_or`) -- in the split kernel also on the
   part-boundary publish path, and at most two elsewhere;
3. every K2 instantiation (the metric's YUV->RGBA stage): no spill of any kind;
4. the split kernel's part hand-off (MI355X_MICROARCH.md's sc1 form): the publish marker's
   `s_waitcnt vmcnt(0)` is the last vector-memory wait before the flag store, which is an `sc1`
   global store with no other vector-memory instruction in between; the poll marker (a compiler
   barrier keeping the column-store loads behind the poll) follows a waited `sc1` poll load.

CPU only: hipcc cross-compiles.  The reference's loops these kernels replace:
ReconstructRow / DoFilter (pkg/libwebp/decoder/frame_dec.c.go:69-261) and EmitFancyRGB
(pkg/libwebp/decoder/io_dec.c.go:65-115)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = os.path.join(ROOT, "go-webp_amd", "csrc", "device")
HIPCC = "/opt/rocm/bin/hipcc"
K1_KERNELS = ("vp8_recon_filter_kernelILb0ELb0", "vp8_recon_filter_kernelILb1ELb0", "vp8_recon_filter_kernelILb1ELb1")


def _compile(src, out):
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-x", "hip",
                    src, "-o", out], check=True, capture_output=True)
    return open(out).read()


def _functions(asm):
    """name -> list of assembly lines of that kernel's body."""
    funcs, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None and line.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur is not None:
            cur.append(line)
    return funcs


def _metadata(asm):
    """kernel name -> {private_segment_fixed_size, sgpr_spill_count, vgpr_spill_count} from the
    code object's metadata (the amdhsa.kernels YAML at the end of the assembly)."""
    meta, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^\s+\.name:\s+(\S+)", line)
        if m:
            cur = meta.setdefault(m.group(1), {})
            continue
        m = re.match(r"^\s+\.(private_segment_fixed_size|sgpr_spill_count|vgpr_spill_count):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return meta


def _insts(lines):
    return [l.strip() for l in lines if re.match(r"^\s+[a-z_]+[a-z0-9_]*\b", l) and not l.strip().startswith(".")]


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("k1isa")
    return {"k1": _compile(os.path.join(DEV, "vp8_recon_filter.hip"), str(d / "k1.s")),
            "k2": _compile(os.path.join(DEV, "yuv_to_rgba.hip"), str(d / "k2.s"))}


def _k1(asm):
    funcs = _functions(asm["k1"])
    out = {}
    for key in K1_KERNELS:
        names = [n for n in funcs if key in n]
        assert len(names) == 1, (key, sorted(funcs))
        out[key] = (names[0], funcs[names[0]])
    return out


def test_k1_no_vgpr_spill_no_scratch(asm):
    meta = _metadata(asm["k1"])
    for key, (name, lines) in _k1(asm).items():
        md = meta[name]
        assert md["vgpr_spill_count"] == 0, (key, md)
        assert md["private_segment_fixed_size"] == 0, (key, md)
        scratch = [l for l in _insts(lines) if l.startswith("scratch_") or re.search(r"buffer_(load|store)\S* .*off,.*off", l)]
        assert not scratch, (key, scratch[:5])
        # (SGPR spills go to VGPR lanes, no memory; round 5's product kernel had 106 -- the bound
        # keeps them from creeping back up unnoticed)
        assert md["sgpr_spill_count"] <= 64, (key, md)


def _step_loop(lines):
    """Lines of the MB step loop: the blocks LLVM annotates as inside the first depth-2 loop (and
    its inner spin loops)."""
    hdr = None
    for l in lines:
        m = re.search(r"\.(LBB\d+_\d+):.*=>\s+This Loop Header: Depth=2", l)
        if m:
            hdr = m.group(1)
            break
        if "=>  This Loop Header: Depth=2" in l:
            break
    # the header label is on the line before a bare "=> This Loop Header" comment line
    if hdr is None:
        for i, l in enumerate(lines):
            if "This Loop Header: Depth=2" in l:
                m = re.match(r"^\.(LBB\d+_\d+):", lines[i - 1]) or re.match(r"^\.(LBB\d+_\d+):", l)
                hdr = m.group(1)
                break
    assert hdr, "no depth-2 loop"
    tag = "B" + hdr[2:]  # LLVM's comments say Header=BB1_40 for label .LBB1_40
    body, inside = [], False
    for l in lines:
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", l):
            inside = l.startswith("." + hdr + ":") or f"Header={tag} " in l or f"Loop {tag} " in l
        if inside:
            body.append(l)
    return body


def test_k1_step_loop_spills_only_on_cold_paths(asm):
    """The one-workgroup kernels (every batch of at least 256 frames: the bench workloads): no spill
    reload on the step's hot path at all.  The split kernel (small batches): at most two (one per
    step at most, e.g. the previous quad's tag in the progress wait -- a v_readlane, no memory)."""
    for key, (name, lines) in _k1(asm).items():
        body = _step_loop(lines)
        assert len(_insts(body)) > 1500, (key, len(_insts(body)))  # the whole step body, not a spin loop
        hot = []
        for i, l in enumerate(body):
            if not re.match(r"^\s+v_(readlane|writelane)_b32", l):
                continue
            after = _insts(body[i:i + 40])[:20]
            cold = any(w.startswith("global_atomic_or") for w in after)  # the timeout's error report
            if key.endswith("ILb1ELb1"):  # the split kernel's part-boundary publish (every 4th column)
                cold |= any("wg-gprog-publish" in x for x in body[max(0, i - 20):i + 1])
            if not cold:
                hot.append(l.strip())
        assert len(hot) <= (2 if key.endswith("ILb1ELb1") else 0), (key, hot)


def test_k2_no_spills(asm):
    meta = _metadata(asm["k2"])
    names = [n for n in meta if "yuv_to_rgba_kernel" in n]
    assert len(names) == 4, names  # fancy / point x RGBA-only / every mode
    for n in names:
        md = meta[n]
        assert md["sgpr_spill_count"] == 0 and md["vgpr_spill_count"] == 0, (n, md)
        assert md["private_segment_fixed_size"] == 0, (n, md)


def test_split_handoff_order(asm):
    name, lines = _k1(asm)["vp8_recon_filter_kernelILb1ELb1"]
    pub = [i for i, l in enumerate(lines) if "wg-gprog-publish" in l]
    assert len(pub) == 1, pub
    i = pub[0]
    assert "s_waitcnt vmcnt(0)" in lines[i]
    # next vector-memory instruction after the marker: the flag store, sc1, nothing in between
    nxt = [l.strip() for l in lines[i + 1:] if re.match(r"^\s+(global_|buffer_|flat_|scratch_)", l)]
    assert nxt and nxt[0].startswith("global_store_dword ") and nxt[0].endswith(" sc1"), nxt[:2]
    polled = [j for j, l in enumerate(lines) if "wg-gprog-polled" in l]
    assert len(polled) == 1, polled
    j = polled[0]
    # the poll: the last sc1 global load before the marker, its value waited for (vmcnt(0)) before
    # the marker in program order
    loads = [k for k in range(j) if re.match(r"^\s+global_load_dword .* sc1$", lines[k])]
    assert loads, "no sc1 poll load before the poll marker"
    k = loads[-1]
    assert any(re.match(r"^\s+s_waitcnt vmcnt\(0\)", lines[x]) for x in range(k + 1, j)), lines[k:j]
