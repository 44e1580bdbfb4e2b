"""GPU parity of ciphertext + plaintext (kernels_mul.hpp k_plain + a 2-way k_add; pai_add_plain) through
the C ABI and the package, against the reference-generated vectors (tests/golden/make_golden_add.py)
and the oracle (add_scalar), bit-exact. Includes encodings far past 64 bits (plain values added to
products, exponents ~26) and the reference's OverflowError for x * 16^E beyond a double."""
import json
import os

import numpy as np
import pytest

from oracle import paillier_oracle as O
from tests.test_oracle_add_golden import expected_cases

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def gadd():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_add.json")) as f:
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


def _operand(ys):
    v = ys[0]
    if isinstance(v, np.float32):
        return np.array(ys, dtype=np.float32)
    if isinstance(v, (np.int64, int)) and not isinstance(v, bool):
        return np.array([int(y) for y in ys], dtype=np.int64)
    return np.array(ys, dtype=np.float64)


@pytest.mark.parametrize("nb", [1024, 2048])
def test_add_plain_reference_golden(ctxs, gadd, nb):
    N = _native()
    ctx, key = ctxs[nb]
    g = gadd["cases"][str(nb)]
    for name, base, ys, op in expected_cases(g):
        ct = N.ints_to_words([int(h, 16) for h in g[base + "c"]], ctx.ct_words)
        ex = np.array(g[base + "e"], dtype=np.int32)
        if op == "rsub":
            ct, ex, _ = ctx.mul(ct, ex, np.array([-1], dtype=np.int64))
        x = _operand(ys)
        if len(set(map(float, ys))) == 1:
            x = x[:1]                                  # the scalar form (x_stride 0)
        out, oe, st = ctx.add_plain(ct, ex, x)
        assert np.all(st == 0), name
        assert [hex(v) for v in N.words_to_ints(out)] == g[name + "_c"], name
        assert list(oe) == g[name + "_e"], name
    # decrypting the big-exponent sums gives the reference's floats
    ct = N.ints_to_words([int(h, 16) for h in g["hi_add_f64_c"]], ctx.ct_words)
    val, _, _, _ = ctx.decrypt(ct, np.array(g["hi_add_f64_e"], dtype=np.int32))
    assert [float(v).hex() for v in val] == g["hi_add_dec"]


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 63, 257])
def test_add_plain_vs_oracle_random(ctxs, nb, count):
    """Random exponents 0..40 (shifts across every limb offset of the c0 multiplier), mixed signs, zeros,
    tiny values, float32/float64/int64 (array elements reach the reference as Python ints/floats, so
    int64 * 16^E is exact); ragged counts."""
    N = _native()
    ctx, key = ctxs[nb]
    rng = np.random.default_rng(count + nb)
    cs = [O.raw_encrypt(int(m), key, O.golden_r(key.n, 77, i)) for i, m in enumerate(rng.integers(0, 1 << 60, count))]
    es = [int(e) for e in rng.integers(0, 41, count)]
    ct = N.ints_to_words(cs, ctx.ct_words)
    ex = np.array(es, dtype=np.int32)
    f64 = rng.standard_normal(count) * 10.0 ** rng.integers(-30, 30, count)
    f64[::5] = 0.0
    f64[1::7] = -1e-205
    f32 = (rng.standard_normal(count) * 1e3).astype(np.float32)
    i64 = rng.integers(-(2 ** 40), 2 ** 40, count, dtype=np.int64)
    i64[::4] = 0
    for x in (f64, f32, i64, np.array([-0.375]), np.array([9], dtype=np.int64)):
        out, oe, st = ctx.add_plain(ct, ex, x)
        got = N.words_to_ints(out)
        for i in range(count):
            s = x[i] if x.size == count else x[0]
            s = int(s) if x.dtype == np.int64 else (np.float32(s) if x.dtype == np.float32 else float(s))
            try:
                want = O.add_scalar(cs[i], es[i], s, key)
            except (OverflowError, ValueError):
                assert st[i] != 0, (x.dtype, i)
                continue
            assert st[i] == 0 and (got[i], int(oe[i])) == want, (x.dtype, i, es[i], s)


def test_add_plain_package_operators():
    """PaillierArray + - with plain arrays/scalars and parallel_ops.add on the GPU, bit-exact with the
    per-element object operators; the device-flagged elements (float overflow) raise like the
    reference."""
    from flex.crypto.paillier import parallel_ops
    from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
    pe, pd = generate_paillier_encryptor_decryptor(1024, seed=5)
    x = np.random.default_rng(3).standard_normal(40).astype(np.float32)
    enc = pe.encrypt(x)
    y = np.random.default_rng(4).standard_normal(40) * 10.0 ** np.random.default_rng(5).integers(-5, 5, 40)
    yi = np.arange(-20, 20, dtype=np.int64) * 99991
    yi32 = yi.astype(np.int32)
    plain = np.asarray(enc)
    prod = enc * (y * 3.0)
    pprod = np.asarray(prod)
    for got, want in ((enc + y, plain + y), (y + enc, y + plain), (enc + 1.5, plain + 1.5), (2 + enc, 2 + plain),
                      (enc - y, plain - y), (y - enc, y - plain), (enc - 4, plain - 4), (7.25 - enc, 7.25 - plain),
                      (enc + yi, plain + yi), (parallel_ops.add(enc, y), plain + y), (prod + y, pprod + y),
                      (prod + yi, pprod + yi), (enc + yi32, plain + yi32)):
        assert [(e.ciphertext(False), e.exponent) for e in np.asarray(got).reshape(-1)] == \
               [(e.ciphertext(False), e.exponent) for e in np.asarray(want).reshape(-1)]
    assert np.allclose(pd.decrypt(enc - y), x.astype(np.float64) - y, rtol=1e-9, atol=1e-9)
    with pytest.raises(OverflowError):
        prod + np.full(40, 1e300)
