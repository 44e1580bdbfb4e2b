"""Debug: decrypt (lane and group engines) of encryptions / products vs the oracle, random 1024-bit keys."""
import os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
for trial in range(int(sys.argv[1])):
    pk, sk = generate_paillier_keypair(1024)
    key = O.Key(pk.n, sk.p, sk.q)
    ctx = N.Context(pk.n, 0, sk.p, sk.q)
    y = np.random.random(100).astype(np.float32)
    ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=os.urandom(32))
    x = random.random()
    mo, me, _ = ctx.mul(ct, ex, np.array([x], dtype=np.float64))
    res = []
    for nm, (c, e) in (("enc", (ct, ex)), ("mul", (mo, me))):
        ints = N.words_to_ints(c)
        want = [O.raw_decrypt(v, key) for v in ints]
        for lane in (True, False):
            ctx.set_lane_decrypt(lane)
            val, mant, st, raw = ctx.decrypt(c, e, want_raw=True)
            got = N.words_to_ints(raw)
            bad = [i for i in range(len(want)) if got[i] != want[i]]
            res.append((nm, "lane" if lane else "group", len(bad), bad[:4]))
        ctx.set_lane_decrypt(True)
    print(trial, res, "q>p" , sk.q > sk.p, "pbits", sk.p.bit_length(), sk.q.bit_length(), "nbits", pk.n.bit_length(), flush=True)
