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
n = 4000
y = np.random.default_rng(0).standard_normal(20000).astype(np.float32)
rk = bytes(range(32))
params = ctx.fixed_base_info()
for v in (y[1762], y[1798], np.float32(1.0), np.float32(-1.5600872)):
    x = np.full(n, v, np.float32)
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    val, _, st, _ = ctx.decrypt(ct, ex)
    bad = np.flatnonzero(val != x.astype(np.float64))
    print("value", repr(v), "bad", bad.size, bad[:12].tolist(), flush=True)
# which elements of the data fail, over all 20000, and their M
ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
val, _, st, _ = ctx.decrypt(ct, ex)
bad = np.flatnonzero(val != y.astype(np.float64))
print("data bad", bad.tolist())
for i in bad.tolist():
    m, e = O.encode(y[i], key.n, key.max_int)
    print("  ", i, repr(y[i]), hex(m), e)
