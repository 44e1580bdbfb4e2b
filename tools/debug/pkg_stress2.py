"""Debug: package encrypt/decrypt over many random keys; on a failure, locate the faulty stage with the oracle."""
import os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
from flex.crypto.paillier import _native as N, _runtime
for trial in range(int(sys.argv[1])):
    pe, pd = generate_paillier_encryptor_decryptor()
    key = O.Key(pe.pub_key.n, pd.priv_key.p, pd.priv_key.q)
    x1 = random.random()
    ex1 = pe.encrypt(x1)
    y1 = np.random.random(100).astype(np.float32)
    ey1 = pe.encrypt(y1)
    ints = [e.ciphertext(False) for e in ey1]
    o_dec = [O.decrypt_value(c, e.exponent, key) if True else None for c, e in zip(ints, ey1)] if False else None
    bad_enc = []
    for i, (c, e) in enumerate(zip(ints, ey1)):
        try:
            v = O.decrypt_value(c, e.exponent, key)
        except Exception as exc:
            v = exc
        if not (isinstance(v, float) and v == float(y1[i])):
            bad_enc.append((i, repr(v)[:60]))
    try:
        d = pd.decrypt(ey1)
        dec_ok = np.array_equal(d, y1.astype(np.float64))
    except Exception as exc:
        dec_ok = repr(exc)
    ctx = _runtime.context(pe.pub_key)
    print(trial, "oracle-bad-enc", len(bad_enc), bad_enc[:3], "pkg dec", dec_ok, "fb", ctx.fixed_base, ctx.fb_ready,
          "ctxs", len(_runtime.cached_contexts()), flush=True)
