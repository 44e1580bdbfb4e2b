import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
pk, sk = generate_paillier_keypair(1024, seed=1)
key = O.Key(pk.n, sk.p, sk.q)
ctx = N.Context(pk.n, 0, sk.p, sk.q)
n = 20000
y = np.random.default_rng(0).standard_normal(n).astype(np.float32)
rk = bytes(range(32))
params = ctx.fixed_base_info()
print("params", params)
for label, x in (("data", y), ("zeros", np.zeros(n, np.float32)), ("ones", np.ones(n, np.float32))):
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    ints = N.words_to_ints(ct)
    bad = [i for i in (1762, 1798, 0, 1) if ints[i] != O.fb_encrypt_value(x[i], key, rk, i, params)[0]]
    print(label, "bad among (1762,1798,0,1):", bad)
    for i in bad[:2]:
        want = O.fb_encrypt_value(x[i], key, rk, i, params)[0]
        print("   i", i, "mod p^2 ok", ints[i] % key.psquare == want % key.psquare, "mod q^2 ok", ints[i] % key.qsquare == want % key.qsquare)
# digits of the bad elements under each window
for w in (8, 12, 16, 20):
    ctx.set_fb_window(w)
    pr = ctx.fixed_base_info()
    ct, ex, _ = ctx.encrypt(y[:2000], obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    ints = N.words_to_ints(ct)
    bad = [i for i in range(2000) if ints[i] != O.fb_encrypt_value(y[i], key, rk, i, pr)[0]]
    print("window", w, "bad", bad)
