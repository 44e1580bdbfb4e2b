#!/usr/bin/env python3
"""Window sweep of the 1024-bit key holder's sampler (k_fbs<19>): bench.py's nb = 1024 leg at several table windows,
one JSON line per window (encrypt rate, k_fbs ms and fraction, table bytes and setup). Usage:
    python tools/gpu/nb1024_sweep.py [--windows 16,20,21,22,23] [--n 1048576]"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default="16,20,21,22,23")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from flex.crypto.paillier import _native
    lib = _native.load_library()
    stream = torch.cuda.current_stream(dev)
    x = torch.from_numpy(np.random.default_rng(0).standard_normal(a.n, dtype=np.float32)).to(dev)
    key = hashlib.sha256(b"nb1024-sweep").digest()
    for w in (int(v) for v in a.windows.split(",")):
        args = argparse.Namespace(fb_window=w, cpu_sample=1024)
        leg, _ = bench.nb1024_leg(args, dev, stream, lib, key, x, 0, 0, steps=a.steps)
        e = leg["encrypt"]
        print(json.dumps({"window_requested": w, "window": e["window_bits"], "digits": e["digits"], "value": e["value"],
                          "k_fbs_ms": e["stages"]["k_fbs"]["kernel_ms"], "k_fbs_frac": e["roofline"]["frac"],
                          "k_fbp_fin_ms": e["stages"]["k_fbp_fin"]["kernel_ms"], "table_bytes": e["table_bytes"],
                          "table_setup_ms": e["table_setup_ms"]}), flush=True)


if __name__ == "__main__":
    main()
