#!/usr/bin/env python3
"""VALU issue ceilings per kernel -> profiles/valu_ceiling.json (read by bench.py's roofline).

The device probe scripts/probes/valu_rate.hip measured how fast one SIMD issues wave64 VALU
instructions with 4 waves resident: plain 2-operand integer ops (v_add/sub/and/or/shift/mov)
one per ~1.07 ns, 3-operand / "complex" ops (v_add3, v_med3, v_sad_u8, v_cndmask, v_cmp, DPP,
SDWA, packed 16-bit, 24-bit multiplies ...) one per ~2.1 ns, v_ashr_pk_u8_i32 one per ~3.6 ns
(DESIGN.md §4).  A kernel's ceiling is therefore set by its instruction mix: this script
compiles each device source for gfx950 (hipcc --save-temps), weights every VALU opcode of each
kernel's code by those costs (scripts/isa_sections.py's valu_units) and writes
ceiling = 1 / (1.07 ns * mean units per VALU instruction) in VALU wave-instructions per ns per
SIMD.  The mix is static (each instruction of the code counted once, not by how often it
runs), so the ceiling is an estimate; bench.py divides the measured issue rate
(SQ_INSTS_VALU per launch / (SIMDs * launch time)) by it."""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from isa_sections import valu_units  # noqa: E402

SOURCES = ["vp8_recon_filter.hip", "yuv_to_rgba.hip", "vp8l_transforms.hip", "vp8l_resolve.hip", "alpha.hip"]
KERNELS = ["vp8_recon_filter_kernel", "yuv_to_rgba_kernel", "vp8l_transforms_kernel", "vp8l_resolve_kernel",
           "alpha_kernel"]
PLAIN_NS = 1.07


def main():
    out = {}
    dev = os.path.join(ROOT, "go-webp_amd", "csrc", "device")
    with tempfile.TemporaryDirectory() as td:
        for src in SOURCES:
            subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip",
                                   "-c", os.path.join(dev, src), "-o", os.path.join(td, src + ".o"), "--save-temps",
                                   "-Wno-unused-parameter", "-Wno-unused-value", "-Wno-unused-result"], cwd=td,
                                  stderr=subprocess.DEVNULL)
        for s_path in glob.glob(os.path.join(td, "*gfx950*.s")):
            s = open(s_path).read()
            for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
                name = next((k for k in KERNELS if k in m.group(1)), None)
                if name is None:
                    continue
                body = s[m.end():s.index("s_endpgm", m.end())]
                ops = collections.Counter()
                for line in body.split("\n"):
                    line = line.strip()
                    if line.startswith("v_"):
                        ops[line.split()[0]] += 1
                n = sum(ops.values())
                units = sum(valu_units(op) * c for op, c in ops.items())
                e = out.setdefault(name, {"valu_static": 0, "units": 0.0, "variants": 0})
                e["valu_static"] += n
                e["units"] += units
                e["variants"] += 1
    for name, e in out.items():
        e["units_per_valu"] = round(e["units"] / e["valu_static"], 4)
        e["ceiling_valu_per_ns_per_simd"] = round(1.0 / (PLAIN_NS * e["units"] / e["valu_static"]), 4)
        e["units"] = round(e["units"], 1)
    out["_note"] = __doc__.split("\n\n")[1].replace("\n", " ")
    path = os.path.join(ROOT, "profiles", "valu_ceiling.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
