#!/usr/bin/env python3
"""Host-side operator throughput on ciphertext arrays received over the wire (pickled), for the
reference and for this package, on the same synthetic workload (VERDICT r1 Missing #1).

    python tools/host_ops_bench.py                                   # this package (default python3)
    PYTHONPATH=/root/reference /opt/conda/bin/python3.9 tools/host_ops_bench.py --ref   # the reference

Workload (nb = 2048 key, seed 1; ciphertexts are uniform residues < n^2 with N(0,1)-like exponents
{12: 4 %, 13: 86 %, 14: 9 %, 15: 1 %}, built directly as PaillierEncryptedNumber objects):
  * add8: 8 arrays of --n elements pickled and unpickled, then summed left to right with `+`
    (HE_SA_FT coordinator, he_sa_ft/train.py:66-69) -> pair-adds/s = 7 n / seconds;
  * dot: a pickled (32,) array times a (32, 6) float64 matrix with `.dot` (HE_OTP_LR,
    he_otp_lr_ft1/train.py:158-160) -> dots/s.
For this package, `--plain` pickles plain object ndarrays (the default pickle, and what an unmodified FLEX
peer sends); otherwise PaillierArray's bulk wire pickle (FLEXPAI_PICKLE_BULK=1). Prints one JSON line.
"""
import argparse
import json
import os
import pickle
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", action="store_true", help="running the reference (PYTHONPATH=/root/reference)")
    ap.add_argument("--plain", action="store_true", help="this package: pickle plain object ndarrays")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    if not args.ref:
        sys.path.insert(0, os.path.join(ROOT, "ibond-flex_amd"))
        if not args.plain:
            os.environ["FLEXPAI_PICKLE_BULK"] = "1"
    from flex.crypto.paillier.encrypted_number import PaillierEncryptedNumber
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk, _ = generate_paillier_keypair(2048, seed=1)
    rng = np.random.default_rng(0)
    nsq = pk.nsquare

    def make(n, seed):
        r = np.random.default_rng(seed)
        exps = r.choice([12, 13, 14, 15], size=n, p=[0.04, 0.86, 0.09, 0.01])
        objs = np.empty(n, dtype=object)
        objs[:] = [PaillierEncryptedNumber(pk, int.from_bytes(r.bytes(512), "little") % nsq, int(e)) for e in exps]
        if args.ref:
            return objs
        from flex.crypto.paillier.cipher_array import PaillierArray
        return PaillierArray(objs)

    arrays = [make(args.n, k) for k in range(8)]
    blobs = [pickle.dumps(a) for a in arrays]
    t_add = []
    for _ in range(args.reps):
        recv = [pickle.loads(b) for b in blobs]
        t0 = time.perf_counter()
        s = recv[0]
        for a in recv[1:]:
            s = s + a
        t_add.append(time.perf_counter() - t0)
    vec = make(32, 99)
    feats = rng.standard_normal((32, 6))
    blob = pickle.dumps(vec)
    t_dot = []
    for _ in range(args.reps):
        v = pickle.loads(blob)
        t0 = time.perf_counter()
        d = v.dot(feats)
        t_dot.append(time.perf_counter() - t0)
    assert len(d) == 6
    out = {"impl": "reference" if args.ref else ("flexpai-plain-pickle" if args.plain else "flexpai"),
           "received_type": type(pickle.loads(blobs[0])).__name__,
           "add8_pair_adds_per_s": 7 * args.n / min(t_add), "dot_32x6_per_s": 1.0 / min(t_dot), "n": args.n}
    if not args.ref:
        from flex.crypto.paillier import _bigint, _runtime
        out["gpu"] = _runtime.gpu_available()
        out["gmp_binding"] = _bigint._gmp is not None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
