#!/usr/bin/env python3
"""Protocol-sized call latency (warm context, device-resident, synchronised wall clock, median of 5): a public-key-only
party's encrypt (k_pe_* / k_encrypt), the key holder's encrypt and decrypt, at 1024/2048 bits and --n elements.
    python tools/gpu/latency_1k.py [--n 1000]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def timed(fn, reps=5):
    fn()
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(1e3 * (time.perf_counter() - t0))
    return round(statistics.median(out), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    a = ap.parse_args()
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = N.load_library()
    stream = torch.cuda.current_stream(dev)
    n = a.n
    x = torch.randn(n, dtype=torch.float32, device=dev)
    for nb in (1024, 2048, 4096):
        pk, sk = generate_paillier_keypair(nb, seed=77)
        W = 2 * nb // 32
        ct = torch.empty((n, W), dtype=torch.int32, device=dev)
        ex = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        val = torch.empty(n, dtype=torch.float64, device=dev)
        mant = torch.empty(n, dtype=torch.int64, device=dev)
        row = {"nb": nb, "n": n}
        for name, c in (("public", N.Context(pk.n, 0)), ("holder", N.Context(pk.n, 0, sk.p, sk.q))):
            c.set_stage_timing(True)
            if name == "holder":
                c.set_fixed_base(False)   # (a 4096-bit holder's first calls stay below the break-even count anyway)

            def enc():
                rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32),
                                         0, ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
                assert rc == 0, lib.pai_last_error()
            row[name + "_encrypt_ms"] = timed(enc)
            row[name + "_encrypt_stages_ms"] = [round(v, 3) for v in c.stage_times()]
            c.set_rows_max(0)
            row[name + "_encrypt_ms_without_rows"] = timed(enc)
            row[name + "_encrypt_stages_ms_without_rows"] = [round(v, 3) for v in c.stage_times()]
            c.set_rows_max(4096)
            if name == "holder":
                def dec():
                    rc = lib.pai_decrypt_dev(c.handle, ct.data_ptr(), ex.data_ptr(), n, val.data_ptr(), mant.data_ptr(),
                                             st.data_ptr(), None, stream.cuda_stream)
                    assert rc == 0, lib.pai_last_error()
                row["holder_decrypt_ms"] = timed(dec)
                c.set_rows_max(0)
                row["holder_decrypt_ms_without_rows"] = timed(dec)
                c.set_rows_max(4096)
                row["roundtrip_exact"] = bool(torch.equal(val, x.double()))
            c.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
