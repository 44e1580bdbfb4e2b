"""The p-adic pair kernels (bn_pair.hpp, bn_pgroup.hpp: k_fbp, k_fbgp, k_crt_b_pair, k_dec_*_pair, k_dec4_*)
against the kernels they replace, which live in the test-only build (libflexpai_xcheck.so) behind
$FLEXPAI_FB_PAIR=0 / $FLEXPAI_PAIR=0 (k_fb, k_fbg, k_crt_b, k_dec_pre/pow/fin, k_decrypt): bit-identical ciphertexts and plaintexts for the
device-RNG sampler, the generic CRT path (explicit r) and decryption, at every key size."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def _native():
    from flex.crypto.paillier import _native
    return _native


def _key(golden, nb):
    k = golden["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _ctx(monkeypatch, key, pair, lib=None):
    N = _native()
    monkeypatch.setenv("FLEXPAI_FB_PAIR", "1" if pair else "0")
    monkeypatch.setenv("FLEXPAI_PAIR", "1" if pair else "0")
    ctx = N.Context(key.n, 0, key.p, key.q, lib=lib)
    ctx.set_fb_window(12)
    ctx.prepare_fixed_base()
    return ctx


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_pair_kernels_match_the_kernels_they_replace(golden, monkeypatch, xlib, nb):
    N = _native()
    key = _key(golden, nb)
    a = _ctx(monkeypatch, key, True)
    b = _ctx(monkeypatch, key, False, xlib)
    assert a.fb_pair and not b.fb_pair
    assert (a.pair_paths & 1) and not (b.pair_paths & 1)
    n = 300 if nb < 4096 else 96
    rng = np.random.default_rng(nb)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(np.float32)
    x[::11] = 0.0
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=1000)
    ca, ea, _ = a.encrypt(x, **kw)          # fixed-base sampler: pairs
    cb, eb, _ = b.encrypt(x, **kw)          # fixed-base sampler: k_fb / k_fbg
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb)
    if nb < 4096:                           # generic CRT path (explicit r): k_crt_b_pair vs k_crt_b
        rs = [O.golden_r(key.n, 5, i) for i in range(n)]
        ga, _, _ = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        gb, _, _ = b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        assert np.array_equal(ga, gb)
        got = N.words_to_ints(ga[:8])
        for i in range(8):
            assert got[i] == O.encrypt_value(x[i], key, rs[i])[0], f"element {i}"
    da = a.decrypt(ca, ea, want_raw=True)
    db = b.decrypt(ca, ea, want_raw=True)
    for u, v in zip(da, db):
        assert np.array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
    assert np.array_equal(da[0], x.astype(np.float64))


def _prime(bits, rng):
    """A random prime of exactly `bits` bits (Miller-Rabin, 24 random bases)."""
    def probable(n):
        d, s = n - 1, 0
        while d % 2 == 0:
            d, s = d // 2, s + 1
        for _ in range(24):
            x = pow(int(rng.integers(2, 1 << 62)) % (n - 3) + 2, d, n)
            if x in (1, n - 1):
                continue
            for _ in range(s - 1):
                x = x * x % n
                if x == n - 1:
                    break
            else:
                return False
        return True
    while True:
        c = int.from_bytes(rng.bytes((bits + 7) // 8), "little") % (1 << bits) | (1 << (bits - 1)) | 1
        if all(c % sp for sp in (3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)) and probable(c):
            return c


def test_unbalanced_key_takes_the_generic_path():
    """Both fixed-base Garner kernels take w_q < q^2 as an operand mod p^2 (k_fbp_fin: A_q, B_q < 2p;
    k_fb_fin: w_p + 8 p^2 - w_q > 0), so a key with q > 2p (p of 1020 bits, q of 1024) gets no tables and
    encrypts on the generic CRT path with the ChaCha20 r, bit-exact against the oracle, and decrypts."""
    N = _native()
    rng = np.random.default_rng(2044)
    p, q = _prime(1020, rng), _prime(1024, rng)
    assert q > 2 * p
    key = O.Key(p * q, p, q)
    ctx = N.Context(key.n, 0, key.p, key.q)
    x = (rng.standard_normal(200) * 50).astype(np.float32)
    rk = bytes(range(100, 132))
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=9)
    assert not ctx.fixed_base and not ctx.fb_ready
    got = N.words_to_ints(ct)
    rbytes = ((key.n.bit_length() + 64 + 31) // 32) * 4
    for i in (0, 77, 199):
        r = O.device_r(rk, 9 + i, rbytes) % key.n
        c, e = O.encrypt_value(x[i], key, r)
        assert got[i] == c and int(ex[i]) == e, f"element {i}"
    assert np.array_equal(ctx.decrypt(ct, ex)[0], x.astype(np.float64))


def test_key_outside_pair_bounds_uses_the_general_kernels(xlib):
    """p, q of 1028 and 1030 bits (n of 2058 bits): R = 2^(28 * 37) is below 2^12 p_h, so no pair kernel applies.
    The product library then encrypts on the public-key group kernel (k_encrypt) and decrypts on the group engine
    (k_decrypt) -- its 2S-limb lane kernels live in the test build only -- bit-exact against the oracle and against
    the test build's 2S-limb CRT / lane path."""
    N = _native()
    rng = np.random.default_rng(2058)
    p, q = _prime(1028, rng), _prime(1030, rng)
    key = O.Key(p * q, min(p, q), max(p, q))
    ctx = N.Context(key.n, 0, key.p, key.q)
    assert not ctx.crt_available and not (ctx.pair_paths & 3) and not ctx.lane_decrypt
    xc = N.Context(key.n, 0, key.p, key.q, lib=xlib)
    assert xc.crt_available
    x = (rng.standard_normal(150) * 1e3).astype(np.float32)
    rs = [O.golden_r(key.n, 8, i) for i in range(x.size)]
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    cx, exx, _ = xc.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    assert np.array_equal(ct, cx) and np.array_equal(ex, exx)
    got = N.words_to_ints(ct)
    for i in (0, 75, 149):
        assert got[i] == O.encrypt_value(x[i], key, rs[i])[0], f"element {i}"
    rk = bytes(range(7, 39))
    a, ea, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=3)
    b, eb, _ = xc.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=3)
    assert np.array_equal(a, b) and np.array_equal(ea, eb)
    for d in (ctx.decrypt(a, ea), xc.decrypt(a, ea)):
        assert np.array_equal(d[0], x.astype(np.float64))
