#!/usr/bin/env python3
"""Where the public fixed-base setup's time goes: the bench's order -- a key holder's W = 22 tables
(2 x 88 GB) built, then released (set_fb_window(16)), then a public-key-only context's W = 20 tables (139 GB) -- with
FLEXPAI_SETUP_TRACE=1 (flexpai.hip ensure_pfb's phases on stderr), and the same build on a device that never held the
key holder's tables. Usage: FLEXPAI_SETUP_TRACE=1 python tools/pfb_setup_trace.py [--no-holder] [--repeat N]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402,F401  (torch's HIP runtime first)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-holder", action="store_true")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--pfb-window", type=int, default=20)
    args = ap.parse_args()
    torch.cuda.init()
    from flex.crypto.paillier import _native
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk, sk = generate_paillier_keypair(2048, seed=1)
    holder = None
    if not args.no_holder:
        holder = _native.Context(pk.n, 0)
        holder.set_private(sk.p, sk.q)
        holder.set_fb_window(23)
        t0 = time.perf_counter()
        holder.prepare_fixed_base()
        print(f"holder tables W={holder.fb_window}: {(time.perf_counter() - t0) * 1e3:.0f} ms", flush=True)
        holder.set_fb_window(16)
        torch.cuda.synchronize()
    for r in range(args.repeat):
        free0 = torch.cuda.mem_get_info()[0]
        c = _native.Context(pk.n, 0)
        c.set_pfb_window(args.pfb_window)
        t0 = time.perf_counter()
        c.prepare_public_fixed_base()
        wall = (time.perf_counter() - t0) * 1e3
        print(f"public tables #{r}: {wall:.0f} ms (free before: {free0 / 1e9:.1f} GB)", flush=True)
        c.close()
        del c
    if holder is not None:
        holder.close()


if __name__ == "__main__":
    main()
