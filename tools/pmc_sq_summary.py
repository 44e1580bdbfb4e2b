#!/usr/bin/env python3
"""Summarise rocprofv3 SQ counter CSVs (tools/gpu/pmc_sq.sh) per kernel: issued VALU instructions,
wave cycles, the fraction of wave cycles with an instruction issued / waiting, and VALU instructions per
canonical MAC of the kernel when its work is known (bench.py's counts).

    python tools/pmc_sq_summary.py CSV [CSV ...] > profiles/r02_pmc_sq.txt
"""
import collections
import csv
import re
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = re.sub(r"^void fpai::", "", r["Kernel_Name"]).split("(")[0]
            if not k.startswith("k_"):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((path, r["Dispatch_Id"]))
    print("# kernel | dispatches | SQ_INSTS_VALU | SQ_WAVE_CYCLES | active_inst/wave_cycles | wait_any/wave_cycles |"
          " wait_inst_any/wave_cycles | LDS insts | SALU insts")
    for k in sorted(agg):
        c = agg[k]
        wc = c.get("SQ_WAVE_CYCLES", 0) or float("nan")
        print(f"{k} | {len(disp[k])} | {c.get('SQ_INSTS_VALU', 0):.4g} | {wc:.4g} | "
              f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} | {c.get('SQ_WAIT_ANY', 0) / wc:.3f} | "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} | {c.get('SQ_INSTS_LDS', 0):.4g} | {c.get('SQ_INSTS_SALU', 0):.4g}")


if __name__ == "__main__":
    main()
