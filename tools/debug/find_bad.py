import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
nb = int(sys.argv[1]); n = int(sys.argv[2])
pk, sk = generate_paillier_keypair(nb, seed=1)
key = O.Key(pk.n, sk.p, sk.q)
ctx = N.Context(pk.n, 0, sk.p, sk.q)
y = np.random.default_rng(0).standard_normal(n).astype(np.float32)
rk = bytes(range(32))
for fb in (True, False):
    ctx.set_fixed_base(fb)
    ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    v, _, s, raw = ctx.decrypt(ct, ex, want_raw=True)
    bad = np.flatnonzero(v != y.astype(np.float64))
    print("fb", fb, "bad", bad.size, bad[:10].tolist(), flush=True)
    ints = N.words_to_ints(ct)
    params = ctx.fixed_base_info() if fb else None
    for i in bad[:4].tolist():
        m, e = O.encode(y[i], key.n, key.max_int)
        oc = O.fb_encrypt_value(y[i], key, rk, i, params) if fb else None
        print("  i", i, "x", repr(y[i]), "M", m if m < key.n // 2 else m - key.n, "e", e, "dev e", int(ex[i]),
              "ct==oracle", (ints[i], int(ex[i])) == oc if fb else None,
              "oracle dec of dev ct", O.decrypt_value(ints[i], int(ex[i]), key) if True else None,
              "dev val", v[i], "status", int(s[i]), flush=True)
