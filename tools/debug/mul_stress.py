"""Debug: random 1024-bit keys, encrypt -> mul by scalar -> decrypt, each stage checked against the oracle."""
import os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
t0 = time.time()
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    pk, sk = generate_paillier_keypair(1024)
    key = O.Key(pk.n, sk.p, sk.q)
    ctx = N.Context(pk.n, 0, sk.p, sk.q)
    y = np.random.random(100).astype(np.float32)
    ct, ex, st = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=os.urandom(32))
    val, _, dst, _ = ctx.decrypt(ct, ex)
    ok_enc = np.array_equal(val, y.astype(np.float64))
    x = random.random()
    mo, me, mst = ctx.mul(ct, ex, np.array([x], dtype=np.float64))
    ints = N.words_to_ints(ct)
    got = N.words_to_ints(mo)
    bad = [i for i in range(100) if (got[i], int(me[i])) != O.mul_scalar(ints[i], int(ex[i]), x, key)]
    v2, _, d2, _ = ctx.decrypt(mo, me)
    print(trial, "enc_ok", ok_enc, "mul_bad", bad[:5], len(bad), "dec_status", sorted(set(d2.tolist())),
          "fb", ctx.fixed_base, "x", x, "p bits", sk.p.bit_length(), sk.q.bit_length(), flush=True)
    if bad or not ok_enc:
        print("KEY", hex(pk.n), hex(sk.p), hex(sk.q))
print("done", time.time() - t0)
