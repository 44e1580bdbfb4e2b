"""The oracle's restatement of ciphertext + plaintext (paillier_oracle.add_scalar / mul_scalar) against
the reference-generated vectors of tests/golden/make_golden_add.py: E(x) + y with float64, float32 and
int64 plain values and scalars, E(x) - y, y - E(x), and additions to products whose exponents (~26)
push the encoding far past 64 bits."""
import json
import os

import numpy as np
import pytest

from oracle import paillier_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gadd():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_add.json")) as f:
        return json.load(f)


def _case(golden, gadd, nb):
    k = golden["keys"][str(nb)]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    return key, gadd["cases"][str(nb)]


def expected_cases(g):
    """(result name, base ciphertexts name, per-element scalar, op) for every golden result."""
    plain = [float.fromhex(v) for v in g["plain"]]
    ints = [int(v) for v in g["ints"]]
    cnt = len(plain)
    return [
        ("add_f64", "", plain, "add"), ("add_f32", "", [np.float32(v) for v in plain], "add"),
        ("add_i64", "", [np.int64(v) for v in ints], "add"),
        ("add_scalar_f", "", [2.75] * cnt, "add"), ("add_scalar_i", "", [3] * cnt, "add"),
        ("radd_scalar_f", "", [0.1] * cnt, "add"), ("sub_f64", "", [-v for v in plain], "add"),
        ("rsub_f64", "", plain, "rsub"), ("sub_scalar_i", "", [-5] * cnt, "add"),
        ("hi_add_f64", "prod_", plain, "add"), ("hi_add_i64", "prod_", [np.int64(v) for v in ints], "add"),
        ("hi_add_scalar", "prod_", [1234.5] * cnt, "add"),
    ]


@pytest.mark.parametrize("nb", [1024, 2048])
def test_oracle_add_plain(golden, gadd, nb):
    key, g = _case(golden, gadd, nb)
    for name, base, ys, op in expected_cases(g):
        cs = [int(h, 16) for h in g[base + "c"]]
        es = g[base + "e"]
        for i, (c, e) in enumerate(zip(cs, es)):
            if op == "rsub":
                c, e = O.mul_scalar(c, e, -1, key)
            got = O.add_scalar(c, e, ys[i], key)
            assert (hex(got[0]), got[1]) == (g[name + "_c"][i], g[name + "_e"][i]), (name, i)


@pytest.mark.parametrize("nb", [1024, 2048])
def test_oracle_products_and_overflow(golden, gadd, nb):
    key, g = _case(golden, gadd, nb)
    for i, (c, e) in enumerate(zip(g["c"], g["e"])):
        got = O.mul_scalar(int(c, 16), e, float.fromhex(g["mulby"][i]), key)
        assert (hex(got[0]), got[1]) == (g["prod_c"][i], g["prod_e"][i])
    assert g["ovf"] == "OverflowError"
    with pytest.raises(OverflowError):
        O.add_scalar(int(g["prod_c"][0], 16), g["prod_e"][0], 1e300, key)
