"""The oracle's restatement of ciphertext x plaintext (paillier_oracle.mul_scalar / add_k) against
the reference-generated vectors of tests/golden/make_golden_mul.py: element-wise __mul__ (float,
int and negative scalars through the invert branch), the encrypted-by-plain dot of
he_otp_lr_ft1/train.py:160 and the (-1 / bs) scaling that follows it."""
import json
import os

import pytest

from oracle import paillier_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gmul():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_mul.json")) as f:
        return json.load(f)


def _case(golden, gmul, nb):
    k = golden["keys"][str(nb)]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    return key, gmul["cases"][str(nb)]


@pytest.mark.parametrize("nb", [1024, 2048])
def test_oracle_dot_and_scaling(golden, gmul, nb):
    key, g = _case(golden, gmul, nb)
    cs = [int(h, 16) for h in g["c"]]
    feats = [[float.fromhex(v) for v in row] for row in g["features"]]
    d = len(feats[0])
    for j in range(d):
        terms = [O.mul_scalar(c, e, feats[i][j], key) for i, (c, e) in enumerate(zip(cs, g["e"]))]
        C, E = O.add_k([t[0] for t in terms], [t[1] for t in terms], key)
        assert (hex(C), E) == (g["dot_c"][j], g["dot_e"][j]), j
        S, SE = O.mul_scalar(C, E, -1 / len(cs), key)
        assert (hex(S), SE) == (g["scaled_c"][j], g["scaled_e"][j]), j


@pytest.mark.parametrize("nb", [1024, 2048])
def test_oracle_elementwise(golden, gmul, nb):
    key, g = _case(golden, gmul, nb)
    cs = [int(h, 16) for h in g["c"]]
    for i, (c, e) in enumerate(zip(cs, g["e"])):
        x = float.fromhex(g["features"][i][0])
        assert tuple(map(lambda v: v, O.mul_scalar(c, e, x, key))) == (int(g["elem_c"][i], 16), g["elem_e"][i]), i
        assert O.mul_scalar(c, e, int(g["ints"][i]), key) == (int(g["ints_c"][i], 16), g["ints_e"][i]), i
        assert O.mul_scalar(c, e, 1 / 3.0, key) == (int(g["div3_c"][i], 16), g["div3_e"][i]), i
