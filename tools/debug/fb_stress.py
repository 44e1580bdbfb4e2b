"""Debug: fixed-base encryption for random keys vs the oracle restatement; package path and direct path."""
import os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
for trial in range(int(sys.argv[1])):
    pk, sk = generate_paillier_keypair(nb)
    key = O.Key(pk.n, sk.p, sk.q)
    ctx = N.Context(pk.n, 0, sk.p, sk.q)
    y = np.random.random(64).astype(np.float32)
    y[::7] *= -1
    rk = os.urandom(32)
    ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=5)
    params = ctx.fixed_base_info()
    got = N.words_to_ints(ct)
    bad = [i for i in range(64) if (got[i], int(ex[i])) != O.fb_encrypt_value(y[i], key, rk, 5 + i, params)]
    val, _, st, _ = ctx.decrypt(ct, ex)
    print(trial, "bad", len(bad), bad[:6], "dec_ok", np.array_equal(val, y.astype(np.float64)), "params", params, flush=True)
    if bad:
        i = bad[0]
        print("  KEY p=%s q=%s rk=%s" % (hex(sk.p), hex(sk.q), rk.hex()))
        print("  x", y[i], "M,e", O.encode(y[i], key.n, key.max_int))
