"""Measured inputs of the public-key break-even (flexpai.hip pfb_threshold): for a public-key
context at nb = 2048, the per-element rate of k_pe_* (no tables), and for each window the public fixed-base tables'
setup time (a fresh context per window: pai_ctx_public_fb_prepare, synchronised) and the sampler's rate on 1M
elements. Prints one JSON line.

    python tools/pfb_breakeven.py [--windows 12 16 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, nargs="+", default=[12, 16, 20])
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--n-pe", type=int, default=1 << 18)
    a = ap.parse_args()
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pk, _ = generate_paillier_keypair(2048, seed=7)
    x = torch.randn(a.n, dtype=torch.float32, device=dev)
    ct = torch.empty((a.n, 128), dtype=torch.int32, device=dev)
    ex = torch.empty(a.n, dtype=torch.int32, device=dev)
    st = torch.empty(a.n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    lib = N.load_library()

    def enc(c, n):
        rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32), 0,
                                 ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
        assert rc == 0, lib.pai_last_error()

    out = {}
    c = N.Context(pk.n, 0)
    c.set_public_fixed_base(False)
    enc(c, 4096)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc(c, a.n_pe)
    torch.cuda.synchronize()
    out["pe_per_s"] = a.n_pe / (time.perf_counter() - t0)
    c.close()
    for w in a.windows:
        c = N.Context(pk.n, 0)
        c.set_pfb_window(w)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.prepare_public_fixed_base()
        torch.cuda.synchronize()
        setup = time.perf_counter() - t0
        _, K, W, _ = c.public_fixed_base_info()
        enc(c, a.n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        enc(c, a.n)
        torch.cuda.synchronize()
        rate = a.n / (time.perf_counter() - t0)
        out[f"W{w}"] = {"setup_s": setup, "rows": K << W, "per_s": rate, "digits": K}
        c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
