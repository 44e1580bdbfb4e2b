#!/usr/bin/env python3
"""Throughput of a 1024-bit public-key-only party on 1M float32 elements (device-resident, warm, device RNG, public
fixed bases off): the pair path (kernels_pe1.hpp) against the group engine's k_encrypt<2> (test build, $FLEXPAI_PAIR=0),
median of 3 calls, with the stage times; one JSON line."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def main():
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 1 << 20
    pk, _ = generate_paillier_keypair(1024, seed=5)
    x = torch.randn(n, dtype=torch.float32, device=dev)
    ct = {k: torch.empty((n, 64), dtype=torch.int32, device=dev) for k in ("pair", "group")}
    ex = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    row = {"nb": 1024, "n": n}
    for name in ("pair", "group"):
        os.environ["FLEXPAI_PAIR"] = "1" if name == "pair" else "0"
        lib = N.load_library(N.XCHECK_LIB_PATH) if name == "group" else N.load_library()
        c = N.Context(pk.n, 0, lib=lib if name == "group" else None)
        c.set_public_fixed_base(False)
        c.set_stage_timing(True)
        times = []
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32), 0,
                                     ct[name].data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
            assert rc == 0, lib.pai_last_error()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        ms = statistics.median(times[1:]) * 1e3
        row[name] = {"ms": round(ms, 2), "encrypts_per_s": round(n / ms * 1e3), "stages_ms": [round(v, 2) for v in c.stage_times()]}
        c.close()
    row["identical"] = bool(torch.equal(ct["pair"], ct["group"]))
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
