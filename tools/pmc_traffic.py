#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs (separate passes) into per-launch HBM
bytes for one kernel, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reads
half of the bytes of a wide coalesced stream (so it is doubled); WRITE_SIZE is taken as is. Both are
in KiB. Writes profiles/pmc_<kernel>_latest.json, which bench.py reports as roofline.traffic -- only while the
library it loads is the one profiled: the file records the sha256 of libflexpai.so (lib_sha16).

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --kernel k_encrypt --n 1048576 --nb 2048 [-o out.json]
"""
import argparse
import csv
import hashlib
import re
import json
import os


def per_launch(path, counter, kernel):
    """Counter of the FIRST of the largest launches of `kernel` (the bench's full-size call on its main context;
    smaller launches come from the host-boundary legs, a later same-size launch from a second context, e.g. the
    library-default window). Rows of one dispatch are summed."""
    per, grid = {}, {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(r"\b%s\b" % re.escape(kernel), r["Kernel_Name"]):
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
            grid[d] = int(r["Grid_Size"])
    if not per:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    g = max(grid.values())
    return per[min(d for d in per if grid[d] == g)], len(per)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="k_encrypt")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--nb", type=int, required=True)
    ap.add_argument("--window", type=int, default=None, help="fixed-base digit window of the run (fixed-base kernels)")
    ap.add_argument("-o", default=None, help="default: profiles/pmc_<kernel>_latest.json (read by bench.py)")
    a = ap.parse_args()
    if a.o is None:
        a.o = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                           f"pmc_{a.kernel}_latest.json")
    f, nf = per_launch(a.fetch_csv, "FETCH_SIZE", a.kernel)
    w, nw = per_launch(a.write_csv, "WRITE_SIZE", a.kernel)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "ibond-flex_amd", "flex", "crypto", "paillier", "_native", "libflexpai.so")
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    out = {"kernel": a.kernel, "n": a.n, "nb": a.nb, "window": a.window, "lib_sha16": lib_sha,
           "fetch_size_kib_raw": f, "write_size_kib_raw": w, "launches": [nf, nw],
           "hbm_read_bytes_per_launch": 2 * f * 1024, "hbm_write_bytes_per_launch": w * 1024,
           "hbm_bytes_per_launch": (2 * f + w) * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), WRITE_SIZE x1; KiB -> bytes"}
    with open(a.o, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
