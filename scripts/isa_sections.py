#!/usr/bin/env python3
"""Static instruction mix per section of the K1 loop body.

Copies vp8_recon_filter.hip with `asm volatile(";MARK name")` inserted before the section
comments listed below, compiles it for gfx950 and counts VALU/SALU/LDS/VMEM instructions
between markers.  Static counts (loops and both filter variants counted once), useful for
before/after comparisons of a change.  KERNEL (env) picks the instantiation: default the
product kernel of c3 / c3s (vp8_recon_filter_kernel<false, false>).
"""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "go-webp_amd", "csrc", "device", "vp8_recon_filter.hip")
MARKS = [("// ---- software pipeline", "prefetch"), ("// ---- wait for the previous quad", "wait"),
         ("// ---- ReconstructRow prologue", "prologue"), ("// ---- top samples", "top"),
         ("// ---- residuals of all blocks", "idct"), ("// ---- luma prediction + residual", "lumapred"),
         ("if (__any(act && i4))", "i4"), ("// ---- chroma prediction + residual", "chroma"),
         ("// ---- stash unfiltered bottom", "window"), ("// ---- loop filter on the window", "filter"),
         ("// ---- deposit final bottom rows", "deposit"), ("// ---- final pixels to HBM", "hbm"),
         ("// ---- rotate for the next MB", "rotate"), ("rc = rn;", "end")]


# Issue cost of a VALU instruction in SIMD-throughput units, measured by
# scripts/probes/valu_rate.hip (4 waves per SIMD): plain 2-operand integer ALU ops issue at
# one per ~1.07 ns per SIMD (1 unit); 3-operand ops, min/max, multiplies, compares,
# cndmask, DPP, SDWA and packed 16-bit ops at one per ~2.1 ns (2 units); v_ashr_pk_u8_i32 3.4.
FULL_RATE = re.compile(r"v_(add|sub|subrev)_(u32|co_u32|i32)(_e32|_e64)?$|v_(and|or|xor|not)_b32(_e32|_e64)?$|"
                       r"v_(lshrrev|lshlrev)_b32(_e32|_e64)?$|v_ashrrev_i32(_e32|_e64)?$|v_mov_b32(_e32|_e64)?$|"
                       r"v_(add|sub)_u16(_e32|_e64)?$|v_mul_lo_u16(_e32|_e64)?$")


def valu_units(op):
    if op.startswith("v_ashr_pk_u8"):
        return 3.4
    return 1.0 if FULL_RATE.match(op) else 2.0


def enc_bytes(op, line):
    """Encoded size of one instruction (GCN/CDNA formats): SOP*/VOP1/VOP2/VOPC 4 bytes, VOP3(P),
    SDWA, DPP, SMEM, DS and memory 8, plus 4 for a literal constant (a hex operand outside the
    inline range).  For code-size (instruction-cache footprint) comparisons."""
    if op.startswith("s_"):
        n = 8 if op.startswith(("s_load", "s_buffer", "s_store", "s_memtime", "s_memrealtime", "s_dcache",
                                "s_atomic")) else 4
    elif op.startswith("v_"):
        n = 4 if op.endswith("_e32") or (op.startswith(("v_mov_b32", "v_readfirstlane")) and "_e64" not in op) else 8
        if op.endswith(("_sdwa", "_dpp")) or op.startswith("v_pk_"):
            n = 8
    else:
        n = 8
    for m in re.findall(r"(?<![\w:])(-?0x[0-9a-fA-F]+|-?\d+)(?![\w.\]])", line.split(";")[0][len(op) + 1:]):
        try:
            v = int(m, 0)
        except ValueError:
            continue
        if not -16 <= v <= 64:
            n += 4
            break
    return n


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    d = os.path.dirname(os.path.abspath(src))
    s = open(src).read()
    for m, name in MARKS:
        if m in s:
            s = s.replace(m, 'asm volatile(";MARK %s");\n      ' % name + m, 1)
    for inc in re.findall(r'#include "([^"]+)"', s):
        s = s.replace(f'#include "{inc}"', f'#include "{os.path.normpath(os.path.join(d, inc))}"')
    with tempfile.TemporaryDirectory() as t:
        f = os.path.join(t, "k.hip")
        open(f, "w").write(s)
        subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x",
                               "hip", "-c", f, "--cuda-device-only", "-save-temps=obj", "-o",
                               os.path.join(t, "k.o")], cwd=t)
        asm = glob.glob(os.path.join(t, "*gfx950*.s"))[0]
        cur, cnt = "pre", collections.OrderedDict()
        meta = {}
        dump = os.environ.get("DUMP_SECTION")  # write that section's ISA to /tmp/isa_<name>.s
        out = open(f"/tmp/isa_{dump}.s", "w") if dump else None
        # one instantiation only (the c3 product kernel by default: no global columns, not split)
        want = os.environ.get("KERNEL", "vp8_recon_filter_kernelILb0ELb0E")
        inside = False
        for line in open(asm):
            if re.match(r"^_Z\w+:", line):
                inside = want in line
                cur = "pre"
                continue
            if line.startswith(".Lfunc_end"):
                inside = False
            if not inside:
                m = re.match(r"\s+\.(vgpr_count|sgpr_count|private_segment_fixed_size|sgpr_spill_count|vgpr_spill_count):\s+(\d+)", line)
                if m and meta.get("_name_ok"):
                    meta[m.group(1)] = m.group(2)
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m:
                    meta["_name_ok"] = want in m.group(1)
                continue
            m = re.search(r";MARK (\w+)", line)
            if m:
                cur = m.group(1)
                continue
            if out and cur == dump:
                out.write(line)
            tok = line.strip().split()
            if not tok or tok[0].startswith((".", ";")) or tok[0].endswith(":"):
                continue
            op = tok[0]
            cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_")
                   else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
            cnt.setdefault(cur, collections.Counter())[cls] += 1
            if op == "s_waitcnt":
                cnt[cur]["waitcnt"] += 1
            cnt[cur]["bytes"] += enc_bytes(op, line)
            if cls == "valu":
                cnt[cur]["units"] += valu_units(op)
                if op.startswith(("v_readlane", "v_writelane")):
                    cnt[cur]["spill"] += 1  # SGPR spills through VGPR lanes
    tot = collections.Counter()
    for k, v in cnt.items():
        print(f"{k:10s} " + " ".join(f"{c}={v[c]:g}" for c in ("valu", "units", "salu", "lds", "vmem", "waitcnt", "spill", "bytes")))
        tot += v
    meta.pop("_name_ok", None)
    print("total      " + " ".join(f"{c}={tot[c]:g}" for c in ("valu", "units", "salu", "lds", "vmem", "waitcnt", "spill", "bytes")),
          meta)


if __name__ == "__main__":
    main()
