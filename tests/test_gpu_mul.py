"""GPU parity of ciphertext x plaintext (kernels_mul.hpp: k_mul, batch inversion k_inv_*, and the
k_add reduction tree of pai_matmul) through the C ABI and the package, against the reference-generated
vectors (tests/golden/make_golden_mul.py) and the oracle (mul_scalar / add_k), bit-exact."""
import json
import os
import pickle

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def gmul():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_mul.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ctxs(golden):
    N = _native()
    out = {}
    for nb in (1024, 2048):
        k = golden["keys"][str(nb)]
        key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
        out[nb] = (N.Context(key.n, 0, key.p, key.q), key)
    return out


def _cts(ctx, g):
    N = _native()
    return N.ints_to_words([int(h, 16) for h in g["c"]], ctx.ct_words), np.array(g["e"], dtype=np.int32)


@pytest.mark.parametrize("nb", [1024, 2048])
def test_mul_reference_golden(ctxs, gmul, nb):
    N = _native()
    ctx, key = ctxs[nb]
    g = gmul["cases"][str(nb)]
    ct, ex = _cts(ctx, g)
    feats = np.array([[float.fromhex(v) for v in row] for row in g["features"]])
    for x, kc, ke in ((np.ascontiguousarray(feats[:, 0]), "elem_c", "elem_e"),
                      (np.array(g["ints"], dtype=np.int64), "ints_c", "ints_e"),
                      (np.array([1 / 3.0]), "div3_c", "div3_e")):
        out, oe, st = ctx.mul(ct, ex, x)
        assert [hex(v) for v in N.words_to_ints(out)] == g[kc] and list(oe) == g[ke], kc
        assert np.all(st == 0)


@pytest.mark.parametrize("nb", [1024, 2048])
def test_matmul_reference_golden(ctxs, gmul, nb):
    N = _native()
    ctx, key = ctxs[nb]
    g = gmul["cases"][str(nb)]
    ct, ex = _cts(ctx, g)
    feats = np.array([[float.fromhex(v) for v in row] for row in g["features"]])
    K, d = feats.shape
    out, oe = ctx.matmul(ct, ex, 1, K, feats, d)
    assert [hex(v) for v in N.words_to_ints(out)] == g["dot_c"] and list(oe) == g["dot_e"]
    s, se, _ = ctx.mul(out, oe, np.array([-1 / K]))
    assert [hex(v) for v in N.words_to_ints(s)] == g["scaled_c"] and list(se) == g["scaled_e"]
    val, _, _, _ = ctx.decrypt(out, oe)
    assert [float(v).hex() for v in val] == g["dot_dec"]


def _random_cts(key, count, seed):
    x = np.random.default_rng(seed).standard_normal(count).astype(np.float32)
    cs, es = [], []
    for i, v in enumerate(x):
        c, e = O.encrypt_value(v, key, O.golden_r(key.n, seed, i))
        cs.append(c)
        es.append(e)
    return cs, es


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 64, 65, 300])
def test_mul_vs_oracle_mixed_scalars(ctxs, nb, count):
    """Mixed signs, zeros, tiny and huge magnitudes, float32 / float64 / int64 scalars; ragged counts
    around the inversion segment (64) so the inversion tree has 1, 2 and 3 levels."""
    N = _native()
    ctx, key = ctxs[nb]
    cs, es = _random_cts(key, count, 11 + count)
    ct = N.ints_to_words(cs, ctx.ct_words)
    ex = np.array(es, dtype=np.int32)
    rng = np.random.default_rng(count)
    f64 = rng.standard_normal(count) * 10.0 ** rng.integers(-20, 20, count)
    f64[::5] = 0.0
    f64[1::9] = -1.0
    f32 = (rng.standard_normal(count) * 100).astype(np.float32)
    i64 = rng.integers(-(2 ** 62), 2 ** 62, count, dtype=np.int64)
    i64[::4] = 0
    for x in (f64, f32, i64, np.array([-0.5]), np.array([7], dtype=np.int64)):
        out, oe, _ = ctx.mul(ct, ex, x)
        got = N.words_to_ints(out)
        idx = sorted({0, count // 3, count // 2, count - 1} | set(range(0, count, max(1, count // 12))))
        for i in idx:
            s = x[i] if x.size == count else x[0]
            s = int(s) if x.dtype == np.int64 else (np.float32(s) if x.dtype == np.float32 else float(s))
            assert (got[i], int(oe[i])) == O.mul_scalar(cs[i], es[i], s, key), (x.dtype, i)


@pytest.mark.parametrize("m,K,d,dt", [(1, 70, 3, np.float64), (2, 5, 2, np.float64), (3, 33, 1, np.float32),
                                      (1, 257, 2, np.int64), (1, 16, 1, np.float64), (1, 17, 1, np.float64)])
def test_matmul_vs_oracle_shapes(ctxs, m, K, d, dt):
    """Reduction trees with and without chunking/padding (K around the chunk of 16, K = 257)."""
    N = _native()
    ctx, key = ctxs[1024]
    cs, es = _random_cts(key, m * K, 7 * K + d)
    ct = N.ints_to_words(cs, ctx.ct_words)
    ex = np.array(es, dtype=np.int32)
    rng = np.random.default_rng(K)
    if dt == np.int64:
        x = rng.integers(-1000, 1000, (K, d)).astype(np.int64)
    else:
        x = (rng.standard_normal((K, d)) * 10.0 ** rng.integers(-4, 4, (K, d))).astype(dt)
    out, oe = ctx.matmul(ct, ex, m, K, x, d)
    got = N.words_to_ints(out)
    for i in range(m):
        for j in range(d):
            s = (lambda v: int(v)) if dt == np.int64 else ((lambda v: np.float32(v)) if dt == np.float32 else float)
            terms = [O.mul_scalar(cs[i * K + k], es[i * K + k], s(x[k, j]), key) for k in range(K)]
            C, E = O.add_k([t[0] for t in terms], [t[1] for t in terms], key)
            assert (got[i * d + j], int(oe[i * d + j])) == (C, E), (i, j)


def test_mul_not_invertible_raises(ctxs):
    """A ciphertext sharing a factor with n has no inverse mod n^2: the reference raises
    ZeroDivisionError from gmpy_math.invert (gmpy_math.py:71-72) for a negative scalar."""
    N = _native()
    ctx, key = ctxs[1024]
    cs, es = _random_cts(key, 5, 3)
    cs[2] = key.p * 12345
    ct = N.ints_to_words(cs, ctx.ct_words)
    ex = np.array(es, dtype=np.int32)
    out, oe, _ = ctx.mul(ct, ex, np.array([2.0]))          # positive: fine
    assert N.words_to_ints(out)[2] == pow(cs[2], O.encode(2.0, key.n, key.max_int)[0], key.nsquare)
    with pytest.raises(ZeroDivisionError):
        ctx.mul(ct, ex, np.array([-2.0]))


def test_package_operators(ctxs):
    """PaillierArray * / dot / @ and parallel_ops.mul on the GPU, bit-exact with the reference's
    per-element object operators (the package's own scalar __mul__/__add__ on Python ints)."""
    from flex.crypto.paillier import parallel_ops
    from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
    pe, pd = generate_paillier_encryptor_decryptor(1024, seed=5)
    x = np.random.default_rng(1).standard_normal(50).astype(np.float32)
    enc = pe.encrypt(x)
    feats = np.random.default_rng(2).standard_normal((50, 4))
    plain = np.asarray(enc)                      # a plain object ndarray: numpy's per-object loop
    for got, want in ((enc * -0.25, plain * -0.25), (3 * enc, 3 * plain), (enc / 4.0, plain / 4.0),
                      (enc * feats[:, 1], plain * feats[:, 1]), (parallel_ops.mul(enc, feats[:, 2]), plain * feats[:, 2]),
                      (enc.dot(feats), plain.dot(feats)), (enc @ feats[:, 0], plain.dot(feats[:, 0])),
                      ((-1 / 50) * enc.dot(feats), (-1 / 50) * plain.dot(feats))):
        g = np.asarray(got).reshape(-1) if isinstance(got, np.ndarray) else np.array([got])
        w = np.asarray(want).reshape(-1) if isinstance(want, np.ndarray) else np.array([want])
        assert [(e.ciphertext(False), e.exponent) for e in g] == [(e.ciphertext(False), e.exponent) for e in w]
    out = pd.decrypt(enc.dot(feats))
    assert np.allclose(out, x.astype(np.float64).dot(feats), rtol=1e-9, atol=1e-9)
    assert pickle.loads(pickle.dumps(enc * 2.0)).dtype == object
