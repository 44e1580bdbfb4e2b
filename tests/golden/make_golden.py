"""Generate the committed golden vectors for the Paillier hot path FROM THE REFERENCE.

Run in the survey container only (the reference never travels to the GPU box):

    PYTHONPATH=/root/reference /opt/conda/bin/python3.9 tests/golden/make_golden.py

That interpreter carries gmpy2 2.0.8 / GMP 6.2.1 (the pin of the reference's
requirements.txt:6) and numpy 1.26 (numpy-1.x encode semantics).
Everything in ``paillier_golden.json`` is produced by calling the reference's own
``flex.crypto.paillier`` objects; nothing here re-implements the algorithm.

Recipe: keys = generate_paillier_keypair(nb, seed=1); per-element
r_i = 1 + (SHA-256 stream(b"flexpai-r" | s | i) mod (n - 1)), stretched to nb+64 bits.
"""
import hashlib
import json
import math
import random
import sys

import numpy as np

from flex.crypto.paillier import obfuscator as ref_obfuscator
from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor, generate_paillier_decryptor
from flex.crypto.paillier.encrypted_number import PaillierEncryptedNumber
from flex.crypto.paillier.fixedpoint_number import FixedPointNumber
from flex.crypto.paillier.keypair import generate_paillier_keypair


def golden_r(n, s, i):
    nb = n.bit_length()
    want = (nb + 64 + 7) // 8
    out = b""
    ctr = 0
    while len(out) < want:
        out += hashlib.sha256(b"flexpai-r" + s.to_bytes(4, "little") + i.to_bytes(8, "little")
                              + ctr.to_bytes(4, "little")).digest()
        ctr += 1
    return 1 + int.from_bytes(out[:want], "little") % (n - 1)


EDGE_F32 = [0.0, -0.0, 1e-45, -1e-45, 1e-30, -1e-30, 3e-23, -3e-23, 1.0, -1.0,
            3.4e38, -3.4e38, -1.7, 0.5, 65504.0, -1e-38, 1.1754944e-38, 123456.789]


def f32_bits(x):
    return int(np.array([x], dtype=np.float32).view(np.uint32)[0])


def f64_hex(v):
    return float(v).hex()


def enc_with_r(pe, x, r):
    """Reference encrypt of one element with an explicit obfuscator (encryptor.py:48-69)."""
    return pe.encrypt(x, random_value=r)


def main():
    out = {"generator": "tests/golden/make_golden.py", "python": sys.version.split()[0],
           "numpy": np.__version__, "keys": {}, "encrypt": {}, "add8": {}, "encode": [],
           "keygen": [], "default_path": {}, "random_value_zero": {}, "scalar_ops": {}}
    import gmpy2
    out["gmpy2"] = gmpy2.version()

    # ---- keygen determinism (keypair.py:93-127, gmpy_math.py:77-87) ----
    for nb, seed in [(1024, 1), (1024, 2), (1024, 12345), (2048, 1), (4096, 7), (512, 99)]:
        pk, sk = generate_paillier_keypair(nb, seed=seed)
        out["keygen"].append({"nb": nb, "seed": seed, "p": hex(sk.p), "q": hex(sk.q), "n": hex(pk.n)})

    # ---- encode table (fixedpoint_number.py:46-90), key nb=1024 seed=1 ----
    pk, sk = generate_paillier_keypair(1024, seed=1)
    n, max_int = pk.n, pk.max_int
    rng = np.random.default_rng(2024)
    f32 = list(EDGE_F32) + [float(v) for v in rng.standard_normal(64).astype(np.float32)] \
        + [float(v) for v in (rng.standard_normal(32) * 10.0 ** rng.integers(-30, 30, 32)).astype(np.float32)]
    for v in f32:
        x = np.float32(v)
        fp = FixedPointNumber.encode(x, n, max_int)
        out["encode"].append({"dtype": "float32", "bits": f32_bits(v), "m": hex(fp.encoding), "e": fp.exponent})
    f64 = [0.1, -0.1, 1.0 / 3.0, 2.0 ** 60 + 1, -123.456, 1e-300, 5e-324, 1.7976931348623157e308 / 2 ** 1000,
           math.pi, -math.e] + [float(v) for v in rng.standard_normal(32)]
    for v in f64:
        fp = FixedPointNumber.encode(np.float64(v), n, max_int)
        out["encode"].append({"dtype": "float64", "hex": f64_hex(v), "m": hex(fp.encoding), "e": fp.exponent})
    for v in [0, 1, -1, 7, -7, 2 ** 40, -(2 ** 40), 2 ** 62, -(2 ** 62)]:
        fp = FixedPointNumber.encode(np.int64(v), n, max_int)
        out["encode"].append({"dtype": "int64", "int": str(v), "m": hex(fp.encoding), "e": fp.exponent})
    out["encode_key"] = {"n": hex(n)}

    # ---- encrypt / decrypt vectors per key size ----
    for nb, K in [(1024, 64), (2048, 64), (4096, 24)]:
        pk, sk = generate_paillier_keypair(nb, seed=1)
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        assert pe.pub_key.n == pk.n
        out["keys"][str(nb)] = {"p": hex(sk.p), "q": hex(sk.q), "n": hex(pk.n)}
        xs = [float(v) for v in np.random.default_rng(nb).standard_normal(K - len(EDGE_F32)).astype(np.float32)]
        xs = list(EDGE_F32) + xs
        recs = []
        for i, v in enumerate(xs):
            r = golden_r(pk.n, nb, i)
            e = enc_with_r(pe, np.float32(v), r)
            c = e.ciphertext(be_secure=False)
            dec = pd.decrypt(e)
            recs.append({"bits": f32_bits(v), "r": hex(r), "c": hex(c), "e": e.exponent, "dec": f64_hex(dec)})
        out["encrypt"][str(nb)] = recs

        # random_value = 0 -> no obfuscation at all (SURVEY.md §8b randomness contract)
        e0 = pe.encrypt(np.float32(1.25), random_value=0)
        out["random_value_zero"][str(nb)] = {"bits": f32_bits(1.25), "c": hex(e0.ciphertext(be_secure=False)),
                                             "e": e0.exponent}

    # ---- default (random_value=None) path with injected SystemRandom r (obfuscator.py:35) ----
    pk, sk = generate_paillier_keypair(1024, seed=1)
    pe, pd = generate_paillier_encryptor_decryptor(1024, seed=1)
    inj = []
    for i, v in enumerate([0.75, -2.5, 0.0, 1e-20]):
        r = golden_r(pk.n, 7, i)

        class FixedRandom:
            def randrange(self, a, b, _r=r):
                return _r
        saved = ref_obfuscator.random.SystemRandom
        ref_obfuscator.random.SystemRandom = FixedRandom
        try:
            e = pe.encrypt(np.float32(v))
        finally:
            ref_obfuscator.random.SystemRandom = saved
        inj.append({"bits": f32_bits(v), "r": hex(r), "c": hex(e.ciphertext(be_secure=False)), "e": e.exponent,
                    "is_obfuscator": bool(e._PaillierEncryptedNumber__is_obfuscator)})
    out["default_path"]["1024"] = inj

    # ---- 8-way homomorphic add (encrypted_number.py:166-185), left-to-right as HE_SA_FT coord ----
    for nb, K in [(1024, 32), (2048, 32)]:
        pk, sk = generate_paillier_keypair(nb, seed=1)
        pe, pd = generate_paillier_encryptor_decryptor(nb, seed=1)
        arrays = []
        for k in range(8):
            x = np.random.default_rng(k).standard_normal(K).astype(np.float32)
            # mixed magnitudes force exponent alignment (encrypted_number.py:115-137)
            x[: K // 4] *= np.float32(1000.0) if k % 2 else np.float32(0.001)
            arrays.append(x)
        cts = []
        for k, x in enumerate(arrays):
            row = []
            for i, v in enumerate(x):
                row.append(enc_with_r(pe, np.float32(v), golden_r(pk.n, 100 + k, i)))
            cts.append(np.array(row))
        acc = cts[0]
        for k in range(1, 8):
            acc = acc + cts[k]
        dec = pd.decrypt(acc)
        out["add8"][str(nb)] = {
            "x": [[f32_bits(float(v)) for v in x] for x in arrays],
            "c": [[hex(e.ciphertext(be_secure=False)) for e in row] for row in cts],
            "ce": [[e.exponent for e in row] for row in cts],
            "sum_c": [hex(e.ciphertext(be_secure=False)) for e in acc],
            "sum_e": [e.exponent for e in acc],
            "sum_dec": [f64_hex(v) for v in dec],
        }

    # ---- scalar ops ("next" rows f1/f3): enc*scalar, enc+scalar (deterministic given c) ----
    pk, sk = generate_paillier_keypair(1024, seed=1)
    pe, pd = generate_paillier_encryptor_decryptor(1024, seed=1)
    ops = []
    for i, (v, s) in enumerate([(0.5, 3), (-1.25, 2.5), (3.0, -0.125), (1e-3, 1000.0), (-7.5, -2)]):
        e = enc_with_r(pe, np.float32(v), golden_r(pk.n, 55, i))
        m = e * s
        a = e + s
        ops.append({"bits": f32_bits(v), "c": hex(e.ciphertext(be_secure=False)), "e": e.exponent,
                    "scalar": repr(s),
                    "mul_c": hex(m.ciphertext(be_secure=False)), "mul_e": m.exponent, "mul_dec": f64_hex(pd.decrypt(m)),
                    "add_c": hex(a.ciphertext(be_secure=False)), "add_e": a.exponent, "add_dec": f64_hex(pd.decrypt(a))})
    out["scalar_ops"]["1024"] = ops

    with open(__file__.replace("make_golden.py", "paillier_golden.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote golden vectors")


if __name__ == "__main__":
    main()
