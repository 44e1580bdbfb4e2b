import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
pk, sk = generate_paillier_keypair(1024, seed=1)
key = O.Key(pk.n, sk.p, sk.q)
ctx = N.Context(pk.n, 0, sk.p, sk.q)
lib = N.load_library()
lib.pai_debug_fb_w.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
n = 2000
y = np.random.default_rng(0).standard_normal(20000).astype(np.float32)[:n]
rk = bytes(range(32))
params = ctx.fixed_base_info()
ct, ex, _ = ctx.encrypt(y, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
buf = np.zeros(2 * 37 * n, dtype=np.uint32)
nn, sb = ctypes.c_longlong(), ctypes.c_int()
assert lib.pai_debug_fb_w(ctx.handle, buf.ctypes.data, buf.size, ctypes.byref(nn), ctypes.byref(sb)) == 0
w = buf.reshape(2, 37, n)
def val(col): return sum(int(v) << (28 * j) for j, v in enumerate(col))
rb = O.fb_raw_bits(key.p, key.q)
badw = []
for i in range(n):
    m, e = O.encode(y[i], key.n, key.max_int)
    c0 = (1 + key.n * m) % key.nsquare
    for h, (P, gg) in enumerate(((key.p, params[0]), (key.q, params[1]))):
        P2 = P * P
        a = O.fb_exponent(rk, i, h, P - 1, rb)
        want = c0 * pow(pow(gg, key.n, P2), a, P2) % P2
        got = val(w[h, :, i])
        if got % P2 != want or got >= 2 * P2:
            badw.append((i, h, got >= 2 * P2))
ints = N.words_to_ints(ct)
badc = [i for i in range(n) if ints[i] != O.fb_encrypt_value(y[i], key, rk, i, params)[0]]
print("bad w (elem, half, >=2m):", badw[:10], len(badw))
print("bad ciphertexts:", badc[:10], len(badc))
# Garner on the device's own w values, in Python
P2, Q2 = key.p * key.p, key.q * key.q
R = 1 << (28 * 37)
for i in badc[:2]:
    wp, wq = val(w[0, :, i]), val(w[1, :, i])
    t = wp + 8 * P2 - wq
    hmont = t * (pow(Q2, -1, P2) * R % P2) * pow(R, -1, P2) % P2
    c = (wq % Q2) + Q2 * hmont
    print("elem", i, "python Garner == oracle", c == O.fb_encrypt_value(y[i], key, rk, i, params)[0],
          "device == python", ints[i] == c, "wp<2m", wp < 2 * P2, "wq<2q2", wq < 2 * Q2, "t bits", t.bit_length(),
          "h bits", hmont.bit_length(), "c bits", c.bit_length())
    # which words differ
    dw = [j for j in range(64) if ((ints[i] >> (32 * j)) & 0xffffffff) != ((c >> (32 * j)) & 0xffffffff)]
    print("   differing words", dw)
    print("   wq >= q2:", wq >= Q2, " wp >= p2:", wp >= P2)
