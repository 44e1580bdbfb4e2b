"""GPU parity of the CRT encryption path (kernels_crt.hpp) against the public-key kernel, the
reference golden vectors and the CPU oracle: same ciphertext bits for every obfuscator mode,
including obfuscators that share a factor with n and obfuscators as wide as n^2."""
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
def pairs(golden):
    """(crt context, public-only context, key) per key size."""
    N = _native()
    out = {}
    for nb in (1024, 2048):
        key = _key(golden, nb)
        crt = N.Context(key.n, 0, key.p, key.q)
        crt.set_fixed_base(False)   # generic r^n path here; the fixed-base sampler: test_gpu_fixed_base
        pub = N.Context(key.n, 0)
        out[nb] = (crt, pub, key)
    return out


@pytest.mark.parametrize("nb", [1024, 2048])
def test_crt_available_and_enabled(pairs, nb):
    crt, pub, _ = pairs[nb]
    assert crt.crt_available and crt.crt_enabled
    assert not pub.crt_available


def test_crt_not_available_4096(golden):
    N = _native()
    key = _key(golden, 4096)
    ctx = N.Context(key.n, 0, key.p, key.q)
    assert not ctx.crt_available


@pytest.mark.parametrize("nb", [1024, 2048])
def test_crt_golden_given_r(golden, pairs, nb):
    N = _native()
    crt, _, _ = pairs[nb]
    recs = golden["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    ct, ex, st = crt.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(ex[i])) == (rec["c"], rec["e"]), f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 255, 257, 1000])
def test_crt_rng_matches_public(pairs, nb, count):
    N = _native()
    crt, pub, key = pairs[nb]
    x = np.random.default_rng(count).standard_normal(count).astype(np.float32)
    rk = bytes(range(32))
    a = crt.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=12345)
    b = pub.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=12345)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    # and against the oracle on a few elements (r derived from the same ChaCha stream)
    got = N.words_to_ints(a[0])
    rbytes = ((nb + 64 + 31) // 32) * 4
    for i in {0, count // 2, count - 1}:
        r = O.device_r(rk, 12345 + i, rbytes)
        c, e = O.encrypt_value(x[i], key, r)
        assert got[i] == c and int(a[1][i]) == e


@pytest.mark.parametrize("nb", [1024, 2048])
def test_crt_edge_obfuscators(pairs, nb):
    """r = 1, r = n - 1, r a multiple of p or of q, r as wide as n^2 - 1, r = n (=> c = 0)."""
    N = _native()
    crt, pub, key = pairs[nb]
    n, p, q = key.n, key.p, key.q
    rs = [1, 2, n - 1, p, 3 * q, p * 7 + 0, n * n - 1, (n * n) // 3, n + 1, n]
    x = np.linspace(-5, 5, len(rs)).astype(np.float32)
    a = crt.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    b = pub.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(a[0])
    assert np.array_equal(a[0], b[0])
    for i, r in enumerate(rs):
        c, e = O.encrypt_value(x[i], key, r)
        assert got[i] == c, f"r index {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_crt_scalar_r_and_dtypes(pairs, nb):
    """random_value reused for every element (encryptor.py:92-95); float64 and int64 inputs."""
    N = _native()
    crt, pub, key = pairs[nb]
    r = 0x1234567890ABCDEF1234567 % key.n
    for x in (np.array([0.0, -0.0, 1.5, -2.25, 3e-30, -7e20], dtype=np.float64),
              np.array([0, 1, -1, 2 ** 40, -(2 ** 50), 123456789], dtype=np.int64)):
        a = crt.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        b = pub.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("nb", [2048])
def test_crt_toggle(pairs, nb):
    N = _native()
    crt, _, _ = pairs[nb]
    x = np.arange(300, dtype=np.float32) - 150.5
    rk = b"k" * 32
    crt.set_fixed_base(False)
    try:
        a = crt.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
        crt.set_crt(False)
        assert not crt.crt_enabled
        b = crt.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
    finally:
        crt.set_crt(True)
        crt.set_fixed_base(True)
    assert np.array_equal(a[0], b[0])
