"""Golden vectors for segmented sums (the per-bin sums of IV_FFS,
flex/tools/feature_iv_algo/hetero_bin.py:27-36, ``good = sum(y[i])``, ``bad = len(i) - sum(y[i])``)
FROM THE REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference /opt/conda/bin/python3.9 tests/golden/make_golden_seg.py

Bins: empty, single, 16, 17, 300 (three reduction levels), repeated and negative indices. Labels are 0/1
ints (exponent 0, as IV_FFS encrypts them); the float case holds values of 1e20 (exponent -4), which
Python's sum (starting from int 0) raises to exponent 0.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import enc_with_r, golden_r  # noqa: E402

from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor  # noqa: E402


def main():
    out = {"generator": "tests/golden/make_golden_seg.py", "numpy": np.__version__, "cases": {}}
    nb, cnt = 1024, 400
    pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
    n = pe.pub_key.n
    rng = np.random.default_rng(17)
    labels = rng.integers(0, 2, cnt).astype(np.int64)
    floats = rng.standard_normal(cnt)
    floats[::13] = 1e20
    bins = [[], [5], list(range(16)), list(range(20, 37)), rng.permutation(cnt)[:300].tolist(),
            [3, 3, 3, -1, -2], rng.integers(0, cnt, 40).tolist(), [0, 13, 26]]
    ct = lambda e: hex(e.ciphertext(be_secure=False))
    for name, vals in (("labels", labels), ("floats", floats)):
        enc = np.array([enc_with_r(pe, (int(v) if name == "labels" else float(v)), golden_r(n, 600, i))
                        for i, v in enumerate(vals)])
        good, bad = [], []
        for i in bins:
            g = sum(enc[i])
            b = len(i) - g
            good.append(None if isinstance(g, int) else [ct(g), int(g.exponent)])
            bad.append(None if isinstance(b, int) else [ct(b), int(b.exponent)])
        dec = [None if isinstance(g, int) else float(pd.decrypt(g)).hex() for g in (sum(enc[i]) for i in bins)]
        out["cases"][name] = {"c": [ct(e) for e in enc], "e": [int(e.exponent) for e in enc],
                              "good": good, "bad": bad, "good_dec": dec}
    out["bins"] = bins
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "paillier_golden_seg.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote paillier_golden_seg.json")


if __name__ == "__main__":
    main()
