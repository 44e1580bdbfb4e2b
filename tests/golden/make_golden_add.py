"""Golden vectors for ciphertext + plaintext (f3: PaillierEncryptedNumber.__add__ / __sub__ / __rsub__
with a plain scalar or array, encrypted_number.py:65-78, 139-164, and parallel_ops.add) FROM THE
REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference /opt/conda/bin/python3.9 tests/golden/make_golden_add.py

Every expected value comes from the reference's own objects under numpy 1.26. The ``hi_*`` cases add
plain values to products (``enc * x``, exponents ~26-30), whose encodings exceed 64 bits, and the
``ovf`` case records the exception the reference raises when x * 16^E is not a finite double.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import enc_with_r, golden_r  # noqa: E402

from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor  # noqa: E402


def main():
    out = {"generator": "tests/golden/make_golden_add.py", "numpy": np.__version__, "cases": {}}
    for nb, cnt in [(1024, 40), (2048, 24)]:
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        n = pe.pub_key.n
        rng = np.random.default_rng(nb + 3)
        y = rng.standard_normal(cnt).astype(np.float32)
        y[::9] = 0.0
        enc = np.array([enc_with_r(pe, v, golden_r(n, 500 + nb % 11, i)) for i, v in enumerate(y)])
        plain = rng.standard_normal(cnt) * (10.0 ** rng.integers(-6, 7, cnt))
        plain[2] = 0.0
        plain[4] = 1e-210
        plain[6] = -2.5
        plain32 = plain.astype(np.float32)
        ints = np.array([(-1) ** i * (i * 7919 % 100003) for i in range(cnt)], dtype=np.int64)
        mulby = rng.standard_normal(cnt) * 100.0
        prod = enc * mulby                                  # exponents ~26-30
        ct = lambda arr: [hex(e.ciphertext(be_secure=False)) for e in np.asarray(arr).reshape(-1)]
        ex = lambda arr: [int(e.exponent) for e in np.asarray(arr).reshape(-1)]
        case = {"y": [float(v).hex() for v in y], "c": ct(enc), "e": ex(enc),
                "plain": [float(v).hex() for v in plain], "ints": [int(v) for v in ints],
                "mulby": [float(v).hex() for v in mulby], "prod_c": ct(prod), "prod_e": ex(prod)}
        results = {
            "add_f64": enc + plain, "add_f32": enc + plain32, "add_i64": enc + ints,
            "add_scalar_f": enc + 2.75, "add_scalar_i": enc + 3, "radd_scalar_f": 0.1 + enc,
            "sub_f64": enc - plain, "rsub_f64": plain - enc, "sub_scalar_i": enc - 5,
            "hi_add_f64": prod + plain, "hi_add_i64": prod + ints, "hi_add_scalar": prod + 1234.5,
        }
        for k, v in results.items():
            case[k + "_c"], case[k + "_e"] = ct(v), ex(v)
        case["hi_add_dec"] = [float(v).hex() for v in pd.decrypt(results["hi_add_f64"])]
        try:
            prod[0] + 1e300
            case["ovf"] = None
        except Exception as err:                            # noqa: BLE001 - recording the reference's type
            case["ovf"] = type(err).__name__
        out["cases"][str(nb)] = case
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "paillier_golden_add.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote paillier_golden_add.json")


if __name__ == "__main__":
    main()
