"""Static ISA guard for K7's round-4 synchronisation (device/vp8l_resolve.hip).

K7 stages each block's literal values straight into LDS (`buffer_load_dword ... lds`, issued
last in the previous block) and replaced `__syncthreads()` with a raw `s_waitcnt lgkmcnt(0);
s_barrier` (bar()), so two orderings rest on the machine code rather than on the source:

1. step 1's reads of the staged values (`vcur[wave * 256 + 64 j + lane]`: four `ds_read_b32`
   at offsets 0 / 256 / 512 / 768 from one address register) must not be reachable from an
   LDS-DMA load along any control-flow path without an `s_waitcnt vmcnt(0)` in between
   (gfx950 has one in-order vmcnt for loads and stores; the literal loads are the newest
   vector-memory operations at that point, so only vmcnt(0) covers them);
2. every `s_barrier` must be reached with no LDS operation outstanding (an `s_waitcnt` with
   lgkmcnt(0) after the last `ds_*` on every path), or another wave could read LDS data this
   wave has not finished writing.

The test compiles the kernel for gfx950 as the Makefile does, disassembles the code object
(llvm-objdump) and checks both properties by a forward data-flow pass over the control-flow
graph of each instantiation.  CPU only: hipcc cross-compiles.  The reference's loop this kernel
replaces is DecodeImageData, pkg/vp8/vp8l_dec.c.go:1105-1153."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "go-webp_amd", "csrc", "device", "vp8l_resolve.hip")
HIPCC = "/opt/rocm/bin/hipcc"
LLVM = "/opt/rocm/lib/llvm/bin"

_LINE = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):")
_SYM = re.compile(r"^[0-9a-f]+ <(\S+)>:$")


def _disassemble(tmp):
    co, elf = os.path.join(tmp, "k7.co"), os.path.join(tmp, "k7.elf")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-x", "hip", "-c",
                    SRC, "-o", co], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={co}", f"--output={elf}"],
                   check=True, capture_output=True)
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", elf], check=True,
                         capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = _SYM.match(line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = _LINE.match(line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return {k: v for k, v in funcs.items() if "vp8l_resolve_kernel" in k}


def _successors(insts):
    """Per instruction index, the indices control may pass to next."""
    index = {addr: i for i, (addr, _, _) in enumerate(insts)}
    succ = []
    for i, (addr, op, args) in enumerate(insts):
        nxt = [i + 1] if i + 1 < len(insts) else []
        if op == "s_endpgm" or op.startswith("s_setpc") or op.startswith("s_trap"):
            succ.append([])
            continue
        if op == "s_branch" or op.startswith("s_cbranch"):
            simm = int(args.split(",")[0].split()[0])
            if simm >= 0x8000:  # printed as an unsigned 16-bit field
                simm -= 0x10000
            tgt = index.get(addr + 4 + 4 * simm)
            assert tgt is not None, f"branch target outside the function at {addr:#x}: {op} {args}"
            succ.append([tgt] if op == "s_branch" else nxt + [tgt])
            continue
        succ.append(nxt)
    return succ


def _flow(insts, succ, gen, kill):
    """Forward may-analysis: state[i] = a `gen` instruction may have executed since the last
    `kill` on some path reaching instruction i (before it executes)."""
    state = [False] * len(insts)
    work = [0]
    seen = set()
    while work:
        i = work.pop()
        out = (state[i] or gen(insts[i])) and not kill(insts[i])
        for j in succ[i]:
            if (out and not state[j]) or j not in seen:
                seen.add(j)
                state[j] = state[j] or out
                work.append(j)
    return state


def _waits(inst, counter):
    op, args = inst[1], inst[2]
    return op == "s_waitcnt" and f"{counter}(0)" in args


def _staged_reads(insts):
    """Step 1's four reads of the staged literal values: ds_read_b32 from one address register
    at offsets 0, 256, 512 and 768 within a short stretch of code."""
    reads = {}
    for i, (_, op, args) in enumerate(insts):
        if op != "ds_read_b32":
            continue
        m = re.match(r"v\d+, (v\d+)(?: offset:(\d+))?$", args)
        if m:
            reads.setdefault(m.group(1), []).append((i, int(m.group(2) or 0)))
    groups = []
    for reg, lst in reads.items():
        for i, off in lst:
            if off != 768:
                continue
            near = [(j, o) for j, o in lst if i - 200 <= j <= i]
            offs = {o for _, o in near}
            if {0, 256, 512, 768} <= offs:
                groups.append([j for j, o in near if o in (0, 256, 512, 768)][-4:])
    return groups


@pytest.fixture(scope="module")
def k7_isa(tmp_path_factory):
    if not (os.path.exists(HIPCC) and os.path.exists(os.path.join(LLVM, "llvm-objdump"))):
        pytest.skip("hipcc / llvm-objdump not available")
    funcs = _disassemble(str(tmp_path_factory.mktemp("k7isa")))
    assert len(funcs) == 6, sorted(funcs)  # stage entry / batch, 32 / 64 mask words per key, + alpha bytes (rows / tiles)
    return funcs


def test_staged_literal_reads_wait_for_lds_dma(k7_isa):
    for name, insts in k7_isa.items():
        succ = _successors(insts)
        dma = [i for i, (_, op, args) in enumerate(insts) if op.startswith("buffer_load") and args.endswith(" lds")]
        # the prologue's block-0 loads plus one set per inlined block body (two register sets)
        assert len(dma) == 12, (name, len(dma))
        groups = _staged_reads(insts)
        assert len(groups) == 2, (name, groups)  # one per inlined block body
        pending = _flow(insts, succ, gen=lambda x: x[1].startswith("buffer_load") and x[2].endswith(" lds"),
                        kill=lambda x: _waits(x, "vmcnt"))
        for g in groups:
            for i in g:
                assert not pending[i], (
                    f"{name}: staged-literal read at {insts[i][0]:#x} ({insts[i][2]}) is reachable from an "
                    "LDS-DMA load without s_waitcnt vmcnt(0)")


def test_barriers_have_no_lds_outstanding(k7_isa):
    for name, insts in k7_isa.items():
        succ = _successors(insts)
        bars = [i for i, x in enumerate(insts) if x[1] == "s_barrier"]
        assert len(bars) >= 10, (name, len(bars))
        pending = _flow(insts, succ, gen=lambda x: x[1].startswith("ds_"), kill=lambda x: _waits(x, "lgkmcnt"))
        for i in bars:
            assert not pending[i], f"{name}: s_barrier at {insts[i][0]:#x} with an LDS operation possibly outstanding"
            assert insts[i - 1][1] == "s_waitcnt", f"{name}: s_barrier at {insts[i][0]:#x} not preceded by a wait"


def test_flow_analysis_catches_a_missing_wait():
    """The checker itself: a synthetic stream with an LDS-DMA load reaching a read around a loop
    back edge without a wait is flagged; with the wait it is not."""
    def prog(with_wait):
        body = [(0x0, "buffer_load_dword", "v1, s[0:3], 0 offen lds"),
                (0x8, "s_waitcnt", "vmcnt(0)" if with_wait else "lgkmcnt(0)"),
                (0xc, "ds_read_b32", "v2, v3"),
                (0x10, "s_cbranch_scc1", "65531"),  # -5: back to 0x0
                (0x14, "s_endpgm", "")]
        return body
    for with_wait in (True, False):
        insts = prog(with_wait)
        st = _flow(insts, _successors(insts), gen=lambda x: x[2].endswith(" lds"), kill=lambda x: _waits(x, "vmcnt"))
        assert st[2] == (not with_wait)
