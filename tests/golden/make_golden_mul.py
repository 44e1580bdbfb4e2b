"""Golden vectors for ciphertext x plaintext (f1: PaillierEncryptedNumber.__mul__ over arrays and the
encrypted-by-plain dot of he_otp_lr_ft1/train.py:160) FROM THE REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference /opt/conda/bin/python3.9 tests/golden/make_golden_mul.py

Every expected value comes from the reference's own objects under numpy 1.26: element-wise
``enc * x`` (encrypted_number.py:86-113, incl. the invert branch for negative scalars),
``enc.dot(features)`` (numpy's object dot over __mul__/__add__), ``(-1 / bs) * grad`` and ``enc / s``.
Inputs are encrypted with explicit obfuscators (make_golden.golden_r) so the bits are reproducible.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import enc_with_r, golden_r  # noqa: E402

from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor  # noqa: E402


def main():
    out = {"generator": "tests/golden/make_golden_mul.py", "numpy": np.__version__, "cases": {}}
    for nb, bs, d in [(1024, 40, 3), (2048, 20, 2)]:
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        n = pe.pub_key.n
        rng = np.random.default_rng(nb)
        y = (rng.standard_normal(bs) * 0.5).astype(np.float64)
        y[::7] = 0.0
        enc = np.array([enc_with_r(pe, v, golden_r(n, 400 + nb % 7, i)) for i, v in enumerate(y)])
        feats = rng.standard_normal((bs, d)) * (10.0 ** rng.integers(-3, 3, (bs, d)))
        feats[3, :] = 0.0
        feats[5, 0] = -1.0
        grad = enc.dot(feats)                              # he_otp_lr_ft1/train.py:160
        scaled = (-1 / bs) * grad
        elem = enc * feats[:, 0]
        ints = enc * np.array([(-1) ** i * (i * 37 % 11) for i in range(bs)], dtype=np.int64)
        div = enc / 3.0
        ct = lambda arr: [hex(e.ciphertext(be_secure=False)) for e in np.asarray(arr).reshape(-1)]
        ex = lambda arr: [int(e.exponent) for e in np.asarray(arr).reshape(-1)]
        out["cases"][str(nb)] = {
            "y": [float(v).hex() for v in y], "c": ct(enc), "e": ex(enc),
            "features": [[float(v).hex() for v in row] for row in feats],
            "dot_c": ct(grad), "dot_e": ex(grad), "dot_dec": [float(v).hex() for v in pd.decrypt(grad)],
            "scaled_c": ct(scaled), "scaled_e": ex(scaled),
            "elem_c": ct(elem), "elem_e": ex(elem),
            "ints": [(-1) ** i * (i * 37 % 11) for i in range(bs)], "ints_c": ct(ints), "ints_e": ex(ints),
            "div3_c": ct(div), "div3_e": ex(div),
        }
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "paillier_golden_mul.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote paillier_golden_mul.json")


if __name__ == "__main__":
    main()
