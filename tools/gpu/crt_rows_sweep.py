#!/usr/bin/env python3
"""Call-size sweep of the key holder's generic CRT encryption (device RNG, fixed bases off): k_crt_w on 16-lane rows
(kernels_crtw.hpp) against k_crt_a + k_crt_b_pair on lanes, and of decryption (k_dec_w against k_dec_pre/pow_pair), warm
calls, median of --reps, one JSON line per size; where the rows stop winning is PAI_OPT_ROWS_MAX's default. Usage:
    python tools/gpu/crt_rows_sweep.py [--nb 2048] [--sizes 256,1024,2048,4096,8192,16384] [--reps 3]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=2048)
    ap.add_argument("--sizes", default="256,1024,2048,4096,8192,16384")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = N.load_library()
    pk, sk = generate_paillier_keypair(a.nb, seed=4242)
    c = N.Context(pk.n, 0, sk.p, sk.q)
    c.set_fixed_base(False)
    c.set_stage_timing(True)
    stream = torch.cuda.current_stream(dev)
    W = 2 * a.nb // 32
    for n in (int(v) for v in a.sizes.split(",")):
        x = torch.randn(n, dtype=torch.float32, device=dev)
        ct = torch.empty((n, W), dtype=torch.int32, device=dev)
        ex = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        row = {"nb": a.nb, "n": n}
        outs = {}
        for name, cap in (("rows", n), ("lanes", 0)):
            c.set_rows_max(cap)
            wall, kern = [], []
            for rep in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0,
                                         bytes(32), 0, ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
                assert rc == 0, lib.pai_last_error()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if rep:
                    wall.append(1e3 * (t1 - t0))
                    kern.append([round(s, 3) for s in c.stage_times()])
            outs[name] = ct.clone()
            row[name] = {"wall_ms": round(statistics.median(wall), 3), "stages_ms": kern[len(kern) // 2]}
        row["identical"] = bool(torch.equal(outs["rows"], outs["lanes"]))
        val = torch.empty(n, dtype=torch.float64, device=dev)
        mant = torch.empty(n, dtype=torch.int64, device=dev)
        dst = torch.empty(n, dtype=torch.int32, device=dev)
        dec = {}
        for name, cap in (("rows", n), ("pairs", 0)):
            c.set_rows_max(cap)
            wall, kern = [], []
            for rep in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = lib.pai_decrypt_dev(c.handle, ct.data_ptr(), ex.data_ptr(), n, val.data_ptr(), mant.data_ptr(),
                                         dst.data_ptr(), None, stream.cuda_stream)
                assert rc == 0, lib.pai_last_error()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                if rep:
                    wall.append(1e3 * (t1 - t0))
                    kern.append([round(v, 3) for v in c.stage_times()])
            dec[name] = val.clone()
            row["dec_" + name] = {"wall_ms": round(statistics.median(wall), 3), "stages_ms": kern[len(kern) // 2]}
        row["dec_identical"] = bool(torch.equal(dec["rows"], dec["pairs"])) and bool(torch.equal(dec["rows"], x.double()))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
