#!/bin/bash
# Kernel resource usage (VGPRs, spills, occupancy) of one translation unit: tools/kres.sh <file.hip>
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | python3 -c '
import sys, re
cur = None
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1); print(); print(cur[:60], end=" ")
        continue
    m = re.search(r"(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)", ln)
    if m: print(m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "") + "=" + m.group(2), end=" ")
print()'
