"""Pin the fixed-base sampler's restatement (oracle/paillier_oracle.py fb_*) to THE REFERENCE:
tests/golden/paillier_golden_fb.json holds the reference's own ciphertexts of
pe.encrypt(x, random_value=fb_r(...)) (tests/golden/make_golden_fb.py, gmpy2 2.0.8), so the
sampler's r^n is a real obfuscator of the reference's encryption (encryptor.py:61-67,
obfuscator.py:35-37) and fb_encrypt_value (the device's formula) gives its bits."""
import pytest

from oracle import paillier_oracle as O


def _key(g, nb):
    k = g["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16)), (k["g_p"], k["g_q"])


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_fb_bases_and_widths(golden_fb, nb):
    key, params = _key(golden_fb, nb)
    assert (O.fb_base(key.p), O.fb_base(key.q)) == params
    assert O.fb_raw_bits(key.p, key.q) == golden_fb["keys"][str(nb)]["raw_bits"]
    # the bases generate Z_h* as far as every prime factor of h - 1 below the trial bound can tell
    for P, g in ((key.p, params[0]), (key.q, params[1])):
        for l in (2, 3, 5, 7, 11, 13):
            if (P - 1) % l == 0:
                assert pow(g, (P - 1) // l, P) != 1


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_fb_r_matches_reference_ciphertexts(golden_fb, nb):
    key, params = _key(golden_fb, nb)
    rk = bytes.fromhex(golden_fb["rng_key"])
    base = golden_fb["index_base"]
    recs = golden_fb["encrypt"][str(nb)]
    if nb == 4096:
        recs = recs[:4]
    for rec in recs[:16]:
        gi = base + rec["i"]
        r = O.fb_r(key, rk, gi, params)
        assert hex(r) == rec["r"]
        x = O.f32_from_bits(rec["bits"])
        # the device's formula (G_h^a_h per half, CRT mod n^2) == the reference's encryption under r
        assert O.fb_encrypt_value(x, key, rk, gi, params) == (int(rec["c"], 16), rec["e"])
        assert O.encrypt_value(x, key, r) == (int(rec["c"], 16), rec["e"])
        assert float(O.decrypt_value(int(rec["c"], 16), rec["e"], key)).hex() == rec["dec"]


def test_fb_exponent_is_reduced(golden_fb):
    key, _ = _key(golden_fb, 2048)
    rk = bytes.fromhex(golden_fb["rng_key"])
    rb = O.fb_raw_bits(key.p, key.q)
    assert rb == 1024 + 64
    for i in range(8):
        a = O.fb_exponent(rk, i, 0, key.p - 1, rb)
        assert 0 <= a < key.p - 1
    assert O.fb_digits(key.p, key.q, 20) == 52 and O.fb_digits(key.p, key.q, 16) == 64
