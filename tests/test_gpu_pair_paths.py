"""The p-adic pair kernels (bn_pair.hpp, bn_pgroup.hpp: k_fbs, k_sgs/k_sgp, k_crt_b_pair, k_dec_*_pair, k_dec4_*) against
the reference's own encryption (the oracle, oracle/paillier_oracle.py) and against the independent group-engine kernels
the product also carries: the public-key k_encrypt and the group decryption k_decrypt, which the test build selects with
$FLEXPAI_PAIR=0. Bit-identical ciphertexts and plaintexts for the device-RNG sampler (against the oracle's restatement of
the sampler), the generic CRT path (explicit r) and decryption, at every key size. (Round 6: the round-1/2 generations
k_fb/k_fb_fin, k_fbg and the 2S-limb lane k_dec_* / k_crt_b that this test used to compare against were retired; the
reference goldens pin every sampler the product ships, tests/test_gpu_fixed_base*.py.)"""
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


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_pair_kernels_against_the_oracle_and_the_group_engine(golden, monkeypatch, xlib, nb):
    N = _native()
    key = _key(golden, nb)
    a = N.Context(key.n, 0, key.p, key.q)
    a.set_fb_window(12)
    a.prepare_fixed_base()
    monkeypatch.setenv("FLEXPAI_PAIR", "0")
    b = N.Context(key.n, 0, key.p, key.q, lib=xlib)      # group-engine decryption, public-key encryption
    monkeypatch.delenv("FLEXPAI_PAIR")
    assert a.fb_pair and (a.pair_paths & 1) and not (b.pair_paths & 3) and not b.lane_decrypt
    n = 300 if nb < 4096 else 96
    rng = np.random.default_rng(nb)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(np.float32)
    x[::11] = 0.0
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=1000)
    ca, ea, _ = a.encrypt(x, **kw)          # fixed-base sampler on pairs: the oracle's restatement of it
    params = a.fixed_base_info()
    got = N.words_to_ints(ca[[0, 1, n // 2, n - 1]])
    for j, i in enumerate([0, 1, n // 2, n - 1]):
        assert (got[j], int(ea[i])) == O.fb_encrypt_value(x[i], key, bytes(range(32)), 1000 + i, params), f"element {i}"
    if nb < 4096:                           # generic CRT path (explicit r): k_crt_b_pair vs the public-key kernel
        rs = [O.golden_r(key.n, 5, i) for i in range(n)]
        a.set_fixed_base(False)
        ga, _, _ = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        gb, _, _ = b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        assert np.array_equal(ga, gb)
        got = N.words_to_ints(ga[:8])
        for i in range(8):
            assert got[i] == O.encrypt_value(x[i], key, rs[i])[0], f"element {i}"
    da = a.decrypt(ca, ea, want_raw=True)   # pair kernels
    db = b.decrypt(ca, ea, want_raw=True)   # group engine
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


def test_key_outside_pair_bounds_uses_the_general_kernels():
    """p, q of 1028 and 1030 bits (n of 2058 bits): R = 2^(28 * 37) is below 2^12 p_h, so no pair kernel applies.
    The library then encrypts on the public-key group kernel (k_encrypt) and decrypts on the group engine (k_decrypt),
    bit-exact against the oracle, explicit r and device RNG alike."""
    N = _native()
    rng = np.random.default_rng(2058)
    p, q = _prime(1028, rng), _prime(1030, rng)
    key = O.Key(p * q, min(p, q), max(p, q))
    ctx = N.Context(key.n, 0, key.p, key.q)
    assert not ctx.crt_available and not (ctx.pair_paths & 3) and not ctx.lane_decrypt
    x = (rng.standard_normal(150) * 1e3).astype(np.float32)
    rs = [O.golden_r(key.n, 8, i) for i in range(x.size)]
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i in (0, 75, 149):
        assert got[i] == O.encrypt_value(x[i], key, rs[i])[0], f"element {i}"
    rk = bytes(range(7, 39))
    a, ea, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=3)
    got = N.words_to_ints(a)
    rbytes = ((key.n.bit_length() + 64 + 31) // 32) * 4
    for i in (0, 149):
        assert got[i] == O.encrypt_value(x[i], key, O.device_r(rk, 3 + i, rbytes) % key.n)[0], f"element {i}"
    assert np.array_equal(ctx.decrypt(a, ea)[0], x.astype(np.float64))
    assert np.array_equal(ctx.decrypt(ct, ex)[0], x.astype(np.float64))
