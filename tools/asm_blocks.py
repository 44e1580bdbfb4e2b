#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a device .s file (tools/asm_blocks.py file.s symbol_prefix)."""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split('\n')
start = [i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and l.rstrip().endswith(':') or l.startswith(sys.argv[2] + ':')][0]
end = [i for i, l in enumerate(lines) if i > start and l.startswith('.Lfunc_end')][0]
blocks, cur = [], ['entry', Counter(), 0]
blocks.append(cur)
for l in lines[start:end]:
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        cur = [m.group(1), Counter(), 0]
        blocks.append(cur)
        continue
    s = l.strip()
    if s and not s.startswith(';') and not s.startswith('.') and not s.endswith(':'):
        cur[1][s.split()[0]] += 1
        cur[2] += 1
minn = int(sys.argv[3]) if len(sys.argv) > 3 else 150
for name, c, n in blocks:
    sc = sum(v for k, v in c.items() if k.startswith('scratch'))
    if n >= minn or sc:
        print(name, n, 'scratch=%d' % sc, c.most_common(10))
