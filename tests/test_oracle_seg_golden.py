"""The oracle's restatement of the per-bin sums of IV_FFS (hetero_bin.py:27-36: good = sum(y[i]),
bad = len(i) - good) against the reference-generated vectors of tests/golden/make_golden_seg.py:
sum() is the aligned k-way product plus the int 0 it starts from (which raises a negative exponent to 0)."""
import json
import os

import pytest

from oracle import paillier_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gseg():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_seg.json")) as f:
        return json.load(f)


def oracle_good_bad(cs, es, idx, key):
    """(good, bad) as (ciphertext, exponent) pairs, or None where the reference gets the int 0."""
    if not idx:
        return None, None
    C, E = O.add_k([cs[i] for i in idx], [es[i] for i in idx], key)
    C, E = O.add_scalar(C, E, 0, key)                 # sum() starts from the int 0
    nc, ne = O.mul_scalar(C, E, -1, key)              # len - g = len + (g * -1)
    return (C, E), O.add_scalar(nc, ne, len(idx), key)


@pytest.mark.parametrize("case", ["labels", "floats"])
def test_oracle_bin_sums(golden, gseg, case):
    k = golden["keys"]["1024"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    g = gseg["cases"][case]
    cs = [int(h, 16) for h in g["c"]]
    for b, idx in enumerate(gseg["bins"]):
        good, bad = oracle_good_bad(cs, g["e"], idx, key)
        want_g, want_b = g["good"][b], g["bad"][b]
        assert (good is None) == (want_g is None)
        if good is not None:
            assert (hex(good[0]), good[1]) == tuple(want_g), (case, b)
            assert (hex(bad[0]), bad[1]) == tuple(want_b), (case, b)
