#!/usr/bin/env python3
"""Static instruction mix of every kernel in a gfx950 .s file (hipcc --save-temps):
VALU/SALU/LDS/VMEM counts and the most frequent VALU opcodes, for before/after checks."""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
    i = m.end()
    j = s.index('s_endpgm', i)
    c = collections.Counter()
    ops = collections.Counter()
    for l in s[i:j].split('\n'):
        l = l.strip()
        if not l or l.startswith(';') or l.startswith('.') or l.endswith(':'):
            continue
        op = l.split()[0]
        kind = ('VALU' if op.startswith('v_') else 'SALU' if op.startswith('s_') else
                'LDS' if op.startswith('ds_') else 'VMEM' if op.startswith(('global_', 'buffer_', 'flat_')) else 'other')
        c[kind] += 1
        if kind == 'VALU':
            ops[op] += 1
    print(m.group(1)[:90], dict(c))
    print('   ', ops.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 12))
