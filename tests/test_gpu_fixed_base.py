"""GPU parity of the fixed-base obfuscation sampler (kernels_fb.hpp), the default device-RNG
encryption for key holders: bit-exact against its CPU restatement (oracle/paillier_oracle.py
fb_rn: r^n mod h^2 = (g_h^n)^a_h, a_h from the ChaCha20 stream), decryptable, independent of the
launch geometry (index base, ragged sizes), and with the reference's randomizer statistics on the
publicly visible part (Jacobi symbol of c mod n, uniform +-1 like r^n for uniform r)."""
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


@pytest.fixture(scope="module")
def ctxs(golden):
    N = _native()
    out = {}
    for nb in (1024, 2048):
        key = _key(golden, nb)
        out[nb] = (N.Context(key.n, 0, key.p, key.q), key)
    return out


def _jacobi(a: int, n: int) -> int:
    a %= n
    res = 1
    while a:
        while a % 2 == 0:
            a //= 2
            if n % 8 in (3, 5):
                res = -res
        a, n = n, a
        if a % 4 == 3 and n % 4 == 3:
            res = -res
        a %= n
    return res if n == 1 else 0


@pytest.mark.parametrize("nb", [1024, 2048])
def test_fixed_base_params_match_oracle(ctxs, nb):
    ctx, key = ctxs[nb]
    assert ctx.fixed_base
    gp, gq, K, W = ctx.fixed_base_info()
    assert (gp, gq) == (O.fb_base(key.p), O.fb_base(key.q))
    assert W == ctx.fb_window and W in (8, 12, 16)
    assert K == O.fb_digits(key.p.bit_length(), key.q.bit_length(), W)


def test_fixed_base_needs_private_key(golden):
    N = _native()
    ctx = N.Context(_key(golden, 2048).n, 0)
    assert not ctx.fixed_base
    with pytest.raises(RuntimeError):
        ctx.fixed_base_info()


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count,base", [(1, 0), (255, 77), (257, 2 ** 33 + 5), (600, 123456)])
def test_fixed_base_bit_exact(ctxs, nb, count, base):
    N = _native()
    ctx, key = ctxs[nb]
    params = ctx.fixed_base_info()
    rk = bytes(range(7, 39))
    x = (np.random.default_rng(count).standard_normal(count) * 100).astype(np.float32)
    x[::13] = 0.0
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    for i in sorted({0, count // 3, count // 2, count - 1}):
        c, e = O.fb_encrypt_value(x[i], key, rk, base + i, params)
        assert got[i] == c and int(ex[i]) == e, f"element {i}"
    val, _, st2, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


def test_fixed_base_toggle_and_given_r_unaffected(ctxs, golden):
    """PAI_OBF_GIVEN keeps the explicit-r path (golden vectors); switching the sampler off returns
    the ChaCha r of the generic path."""
    N = _native()
    ctx, key = ctxs[2048]
    recs = golden["encrypt"]["2048"][:8]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=[int(r["r"], 16) for r in recs])
    assert [hex(c) for c in N.words_to_ints(ct)] == [r["c"] for r in recs]
    rk = b"\x01" * 32
    a = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)[0]
    ctx.set_fixed_base(False)
    try:
        assert not ctx.fixed_base
        b = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)[0]
    finally:
        ctx.set_fixed_base(True)
    assert not np.array_equal(a, b)
    r0 = O.device_r(rk, 0, ((2048 + 64 + 31) // 32) * 4) % key.n
    assert N.words_to_ints(b)[0] == O.encrypt_value(x[0], key, r0)[0]


def test_fixed_base_jacobi_statistics(ctxs):
    """c mod n = r^n mod n: its Jacobi symbol is uniform +-1 for uniform r; a sampler confined to a
    subgroup (e.g. bases that are squares mod p) would show a constant symbol."""
    N = _native()
    ctx, key = ctxs[2048]
    M = 2000
    ct, _, _ = ctx.encrypt(np.zeros(M, dtype=np.float32), obf_mode=N.PAI_OBF_RNG, rng_key=b"j" * 32)
    js = [_jacobi(c % key.n, key.n) for c in N.words_to_ints(ct)]
    plus = sum(1 for j in js if j == 1)
    assert all(j in (1, -1) for j in js)
    assert abs(plus - M / 2) < 5 * (M / 4) ** 0.5       # 5 sigma


@pytest.mark.parametrize("nb", [1024, 2048])
def test_fixed_base_windows(ctxs, nb):
    """Windows 8, 12, 16, 20 rebuild the tables; each is bit-exact against the oracle, and 8 and 16
    (same 1088-bit exponent for 2048-bit keys, 576-bit for 1024-bit) give identical ciphertexts."""
    N = _native()
    ctx, key = ctxs[nb]
    w0 = ctx.fb_window
    rk = bytes(range(40, 72))
    x = np.random.default_rng(nb).standard_normal(300).astype(np.float32)
    outs = {}
    try:
        for w in (8, 12, 16, 20):
            ctx.set_fb_window(w)
            params = ctx.fixed_base_info()
            assert params[3] == w
            ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=99)
            got = N.words_to_ints(ct)
            for i in (0, 150, 299):
                assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, 99 + i, params), (w, i)
            outs[w] = ct
        assert np.array_equal(outs[8], outs[16])
    finally:
        ctx.set_fb_window(w0)
    with pytest.raises(RuntimeError):
        ctx.set_fb_window(10)
