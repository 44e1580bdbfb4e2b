"""Golden vectors that pin the engine's fixed-base (device-RNG, key-holder) encryption to THE REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference:/root/repo /opt/conda/bin/python3.9 tests/golden/make_golden_fb.py

The fixed-base sampler (ibond-flex_amd/csrc/kernels_fb.hpp) draws r^n mod n^2 as the CRT of
G_p^a_p and G_q^a_q, G_h = g_h^n mod h^2. That is r^n for the explicit obfuscator
r = CRT(g_p^a_p mod p, g_q^a_q mod q) (oracle.paillier_oracle.fb_r; r^n mod p^2 depends only on
r mod p). This script derives r per element from the ChaCha20 exponent stream (the oracle's
restatement of the engine's digit kernel), then lets the REFERENCE encrypt with it:
``pe.encrypt(np.float32(x), random_value=r)`` (encryptor.py:61-67 -> raw_encrypt.py:22-49 ->
obfuscator.py:35-37, gmpy2.powmod). The ciphertexts below are the reference's; the GPU test
(tests/test_gpu_fixed_base.py) compares k_fb's output against them bit-exactly at W = 16 and 20.
"""
import json
import sys

import numpy as np

from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
from flex.crypto.paillier.keypair import generate_paillier_keypair

from oracle import paillier_oracle as O

EDGE_F32 = [0.0, -0.0, 1e-45, -1e-45, 1e-30, -1e-30, 1.0, -1.0, 3.4e38, -3.4e38, -1.7, 65504.0]
RNG_KEY = bytes(range(101, 133))
INDEX_BASE = (1 << 33) + 12345


def f32_bits(x):
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


def main():
    out = {"generator": "tests/golden/make_golden_fb.py", "python": sys.version.split()[0],
           "numpy": np.__version__, "rng_key": RNG_KEY.hex(), "index_base": INDEX_BASE, "keys": {}, "encrypt": {}}
    import gmpy2
    out["gmpy2"] = gmpy2.version()
    for nb, K in [(1024, 64), (2048, 64), (4096, 16)]:
        pk, sk = generate_paillier_keypair(nb, seed=1)
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        key = O.Key(pk.n, sk.p, sk.q)
        gp, gq = O.fb_base(key.p), O.fb_base(key.q)
        out["keys"][str(nb)] = {"n": hex(pk.n), "p": hex(sk.p), "q": hex(sk.q), "g_p": gp, "g_q": gq,
                                "raw_bits": O.fb_raw_bits(key.p, key.q)}
        xs = EDGE_F32 + [float(v) for v in np.random.default_rng(nb + 7).standard_normal(K - len(EDGE_F32)).astype(np.float32)]
        recs = []
        for i, v in enumerate(xs):
            gi = INDEX_BASE + i
            r = O.fb_r(key, RNG_KEY, gi, (gp, gq))
            e = pe.encrypt(np.float32(v), random_value=r)
            c = e.ciphertext(be_secure=False)
            assert pow(r, pk.n, pk.nsquare) == O.fb_rn(key, RNG_KEY, gi, (gp, gq))
            recs.append({"i": i, "bits": f32_bits(v), "r": hex(r), "c": hex(c), "e": e.exponent,
                         "dec": float(pd.decrypt(e)).hex()})
        out["encrypt"][str(nb)] = recs
    with open(__file__.replace("make_golden_fb.py", "paillier_golden_fb.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote fixed-base golden vectors")


if __name__ == "__main__":
    main()
