"""Pin the public-key fixed-base sampler's restatement (oracle/paillier_oracle.py pfb_*) to THE REFERENCE:
tests/golden/paillier_golden_pfb.json holds the reference's own ciphertexts of pe.encrypt(x, random_value=r)
for r = prod_j g_j^e_j mod n (tests/golden/make_golden_pfb.py, gmpy2 2.0.8) at three digit windows."""
import pytest

from oracle import paillier_oracle as O


def _key(g):
    k = g["keys"]["2048"]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16)), [int(b, 16) for b in k["bases"]]


def test_pfb_bases(golden_pfb):
    key, bases = _key(golden_pfb)
    assert len(bases) == 1 + O.PFB_SHORT and all(1 < g < key.n for g in bases)
    assert O.jacobi(bases[0], key.n) == -1          # the publicly visible symbol of c mod n is uniform


@pytest.mark.parametrize("window", ["12", "16", "20"])
def test_pfb_r_matches_reference_ciphertexts(golden_pfb, window):
    key, bases = _key(golden_pfb)
    rk = bytes.fromhex(golden_pfb["rng_key"])
    base = golden_pfb["index_base"]
    W = int(window)
    for rec in golden_pfb["encrypt"]["2048"][window][:12]:
        gi = base + rec["i"]
        r = O.pfb_r(key.n, bases, rk, gi, W)
        assert hex(r) == rec["r"]
        x = O.f32_from_bits(rec["bits"])
        assert O.pfb_encrypt_value(x, key, bases, rk, gi, W) == (int(rec["c"], 16), rec["e"])
        assert float(O.decrypt_value(int(rec["c"], 16), rec["e"], key)).hex() == rec["dec"]


def test_pfb_layout():
    assert O.pfb_layout(2048, 16) == (132, 6)
    assert O.pfb_layout(2048, 20) == (106, 5)
    es = O.pfb_exponents(bytes(32), 5, 2048, 16)
    assert len(es) == 33 and es[0] < 1 << 2112 and all(e < 1 << 96 for e in es[1:])
    # the digit layout is the stream read in order: e_0's digits first, then each short exponent's
    es12 = O.pfb_exponents(bytes(32), 5, 2048, 12)
    assert es12[0] & ((1 << 2100) - 1) == es[0] & ((1 << 2100) - 1)


def test_jacobi_matches_euler():
    p = 1000003
    for a in (2, 3, 5, 10, 12345):
        assert O.jacobi(a, p) == (1 if pow(a, (p - 1) // 2, p) == 1 else -1)
