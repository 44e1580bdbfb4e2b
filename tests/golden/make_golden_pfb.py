"""Golden vectors that pin the engine's PUBLIC-KEY fixed-base encryption (kernels_pfb.hpp) to THE REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference:/root/repo /opt/conda/bin/python3.9 tests/golden/make_golden_pfb.py

A party holding only the public key samples r = prod_j g_j^e_j mod n over 33 bases g_j and exponents read from
the element's ChaCha20 stream (oracle.paillier_oracle.pfb_r restates the digit layout); the engine computes
r^n mod n^2 as a product of table rows. This script fixes the bases (sha256-derived, g_0 with Jacobi symbol
-1, as the engine draws them), derives r per element, and lets the REFERENCE encrypt with it:
``pe.encrypt(np.float32(x), random_value=r)`` (encryptor.py:61-67 -> raw_encrypt.py:22-49 -> obfuscator.py:35-37,
gmpy2.powmod). The ciphertexts are the reference's; tests/test_gpu_public_fixed_base.py compares the engine's
output (bases set through pai_ctx_public_fb_set_bases) against them bit-exactly. r depends on the window W (the
digit layout of e_0), so there is one record set per window.
"""
import hashlib
import json
import sys

import numpy as np

from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
from flex.crypto.paillier.keypair import generate_paillier_keypair

from oracle import paillier_oracle as O

EDGE_F32 = [0.0, -0.0, 1e-45, -1e-45, 1e-30, -1e-30, 1.0, -1.0, 3.4e38, -3.4e38, -1.7, 65504.0]
RNG_KEY = bytes(range(151, 183))
INDEX_BASE = (1 << 34) + 777
WINDOWS = (12, 16, 20)


def f32_bits(x):
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


def derived_bases(n: int, tag: bytes):
    """33 bases in [2, n): sha256 counter stream, rejection-sampled like the engine's CSPRNG draw; g_0 is the
    first candidate with Jacobi symbol -1."""
    nbits = n.bit_length()
    ctr = 0

    def cand():
        nonlocal ctr
        while True:
            raw = b"".join(hashlib.sha256(tag + ctr.to_bytes(4, "little") + k.to_bytes(4, "little")).digest()
                           for k in range((nbits + 255) // 256))
            ctr += 1
            g = int.from_bytes(raw, "little") & ((1 << nbits) - 1)
            if 2 <= g < n:
                return g
    g0 = cand()
    while O.jacobi(g0, n) != -1:
        g0 = cand()
    return [g0] + [cand() for _ in range(O.PFB_SHORT)]


def main():
    out = {"generator": "tests/golden/make_golden_pfb.py", "python": sys.version.split()[0],
           "numpy": np.__version__, "rng_key": RNG_KEY.hex(), "index_base": INDEX_BASE, "keys": {}, "encrypt": {}}
    import gmpy2
    out["gmpy2"] = gmpy2.version()
    for nb, count in [(2048, 24)]:
        pk, sk = generate_paillier_keypair(nb, seed=1)
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        assert pe.pub_key.n == pk.n
        key = O.Key(pk.n, sk.p, sk.q)
        bases = derived_bases(pk.n, b"flexpai-pfb-golden")
        out["keys"][str(nb)] = {"n": hex(pk.n), "p": hex(sk.p), "q": hex(sk.q), "bases": [hex(g) for g in bases]}
        xs = EDGE_F32 + [float(v) for v in np.random.default_rng(nb + 11).standard_normal(count - len(EDGE_F32)).astype(np.float32)]
        out["encrypt"][str(nb)] = {}
        for W in WINDOWS:
            recs = []
            for i, v in enumerate(xs):
                gi = INDEX_BASE + i
                r = O.pfb_r(pk.n, bases, RNG_KEY, gi, W)
                e = pe.encrypt(np.float32(v), random_value=r)
                c = e.ciphertext(be_secure=False)
                recs.append({"i": i, "bits": f32_bits(v), "r": hex(r), "c": hex(c), "e": e.exponent,
                             "dec": float(pd.decrypt(e)).hex()})
            out["encrypt"][str(nb)][str(W)] = recs
    with open(__file__.replace("make_golden_pfb.py", "paillier_golden_pfb.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote public fixed-base golden vectors")


if __name__ == "__main__":
    main()
