"""Debug: repeat the same encrypt (fixed key, fixed rng key) and the same decrypt many times; any
difference between repetitions is a nondeterministic kernel."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
nb = int(sys.argv[1]); reps = int(sys.argv[2]); n = int(sys.argv[3])
pk, sk = generate_paillier_keypair(nb, seed=1)
ctx = N.Context(pk.n, 0, sk.p, sk.q)
y = np.random.default_rng(0).standard_normal(n).astype(np.float32)
rk = bytes(range(32))
ct0, ex0, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
v0, _, s0, _ = ctx.decrypt(ct0, ex0)
print("first", np.array_equal(v0, y.astype(np.float64)), flush=True)
t0 = time.time()
for r in range(reps):
    ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    de = np.flatnonzero(np.any(ct != ct0, axis=1))
    v, _, s, _ = ctx.decrypt(ct0, ex0)
    dd = np.flatnonzero(v != v0)
    if de.size or dd.size:
        print("rep", r, "enc diffs", de[:10], de.size, "dec diffs", dd[:10], dd.size, flush=True)
    if r % 20 == 0:
        print("rep", r, time.time() - t0, flush=True)
print("done", time.time() - t0)
