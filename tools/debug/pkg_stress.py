"""Debug: the test_gpu_package sequence (encrypt/add/mul/decrypt through the package API) over many
random keys, every result checked exactly against numpy / the oracle."""
import os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
from flex.crypto.paillier import _native as N
fails = 0
t0 = time.time()
for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    pe, pd = generate_paillier_encryptor_decryptor()
    key = O.Key(pe.pub_key.n, pd.priv_key.p, pd.priv_key.q)
    x1, x2 = random.random(), random.random()
    y1, y2 = np.random.random(100).astype(np.float32), np.random.random(100).astype(np.float32)
    ey1, ey2 = pe.encrypt(y1), pe.encrypt(y2)
    ok = {}
    try:
        ok["enc"] = np.array_equal(pd.decrypt(ey1), y1.astype(np.float64))
    except Exception as exc:
        ok["enc"] = repr(exc)
        ints = [e.ciphertext(False) for e in ey1]
        ob = []
        for i, (c, e) in enumerate(zip(ints, ey1)):
            try:
                v = O.decrypt_value(c, e.exponent, key)
            except Exception as exc2:
                v = repr(exc2)[:40]
            if v != float(y1[i]):
                ob.append((i, v))
        print("   oracle decrypt of the package ciphertexts: bad", len(ob), ob[:4], flush=True)
        from flex.crypto.paillier import _runtime
        ctx = _runtime.context(pe.pub_key)
        words = np.stack([np.frombuffer(c.to_bytes(ctx.ct_words * 4, "little"), dtype=np.uint32) for c in ints])
        val, _, st, raw = ctx.decrypt(words, np.array([e.exponent for e in ey1], dtype=np.int32), want_raw=True)
        print("   device decrypt statuses", sorted(set(st.tolist())), "raw ok",
              sum(1 for i, r in enumerate(N.words_to_ints(raw)) if r == O.raw_decrypt(ints[i], key)), flush=True)
    s = ey1 + ey2
    ok["add"] = np.array_equal(pd.decrypt(s), y1.astype(np.float64) + y2.astype(np.float64))
    s2 = ey1 + y2
    ok["add_plain"] = np.allclose(pd.decrypt(s2), y1.astype(np.float64) + y2, rtol=1e-15)
    ex1 = pe.encrypt(x1)
    ok["scalar_mul"] = abs(pd.decrypt(ex1 * x2) - x1 * x2) < 1e-12
    try:
        m = ey1 * x1
        ints = [e.ciphertext(False) for e in ey1]
        want = [O.mul_scalar(c, e.exponent, x1, key) for c, e in zip(ints, ey1)]
        bad = [i for i in range(100) if (m[i].ciphertext(False), m[i].exponent) != want[i]]
        ok["mul"] = not bad
        v = pd.decrypt(m)
        ok["mul_dec"] = np.allclose(v, y1.astype(np.float64) * x1, rtol=1e-12)
    except Exception as exc:
        ok["mul_exc"] = repr(exc)
        bad = "exc"
    m2 = ey1 * y2
    ok["mul_arr"] = np.allclose(pd.decrypt(m2), y1.astype(np.float64) * y2, rtol=1e-12)
    allok = all(v is True for v in ok.values())
    print(trial, "OK" if allok else ok, flush=True)
    if not allok:
        fails += 1
        print("KEY n=%s p=%s q=%s x1=%r bad=%s" % (hex(key.n), hex(key.p), hex(key.q), x1, bad if not isinstance(bad, str) else bad), flush=True)
print("done fails", fails, time.time() - t0)
