"""Same-box A/B of the 1024/2048-bit decryption chain (k_dec_pow_pair): the factored B-free chain (the product,
k_dec_pow_pair<s, true>) against the general chain (the test build's k_dec_pow_pair<s, false>, $FLEXPAI_DECF=0), both
from libflexpai_xcheck.so, alternating, with the stage times of each device-resident decrypt of 1M elements.

    python tools/ab_decf.py [--reps 3] [--n 1048576] [--nb 2048]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--nb", type=int, default=2048)
    a = ap.parse_args()
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    xlib = N.load_library(N.XCHECK_LIB_PATH)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pk, sk = generate_paillier_keypair(a.nb, seed=1)
    W = 2 * a.nb // 32
    x = torch.randn(a.n, dtype=torch.float32, device=dev)
    ct = torch.empty((a.n, W), dtype=torch.int32, device=dev)
    ex = torch.empty(a.n, dtype=torch.int32, device=dev)
    st = torch.empty(a.n, dtype=torch.int32, device=dev)
    val = torch.empty(a.n, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctxs = {}
    for f in ("1", "0"):
        os.environ["FLEXPAI_DECF"] = f
        c = N.Context(pk.n, 0, sk.p, sk.q, lib=xlib)
        c.set_stage_timing(True)
        ctxs[f] = c
    os.environ.pop("FLEXPAI_DECF")
    c = ctxs["1"]
    rc = xlib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), a.n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32), 0,
                              ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
    assert rc == 0
    out = {"1": [], "0": []}
    for rep in range(a.reps + 1):
        for f in ("1", "0"):
            c = ctxs[f]
            rc = xlib.pai_decrypt_dev(c.handle, ct.data_ptr(), ex.data_ptr(), a.n, val.data_ptr(), None, st.data_ptr(),
                                      None, stream.cuda_stream)
            assert rc == 0, xlib.pai_last_error()
            torch.cuda.synchronize()
            assert torch.equal(val, x.double()), "round trip"
            if rep:
                out[f].append(c.stage_times())
    res = {("factored" if f == "1" else "general"): {"pow_ms": [round(s[1], 3) for s in v], "stages_ms": v[-1]} for f, v in out.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
