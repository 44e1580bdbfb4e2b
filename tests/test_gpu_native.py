"""GPU parity of the HIP engine through the C ABI (libflexpai.so) against the golden vectors
generated from the reference (tests/golden/make_golden.py) and the CPU oracle."""
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
    for nb in (1024, 2048, 4096):
        key = _key(golden, nb)
        out[nb] = (N.Context(key.n, 0, key.p, key.q), key)
    return out


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_encrypt_given_r_bit_exact(golden, ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, rec in enumerate(recs):
        assert st[i] == 0
        assert (hex(got[i]), int(ex[i])) == (rec["c"], rec["e"]), f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_decrypt_bit_exact(golden, ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    cts = N.ints_to_words([int(r["c"], 16) for r in recs], ctx.ct_words)
    ex = np.array([r["e"] for r in recs], dtype=np.int32)
    val, mant, st, raw = ctx.decrypt(cts, ex, want_raw=True)
    raws = N.words_to_ints(raw)
    for i, rec in enumerate(recs):
        c = int(rec["c"], 16)
        assert raws[i] == O.raw_decrypt(c, key), f"raw plaintext {i}"
        assert float(val[i]).hex() == rec["dec"], f"decoded value {i} status {st[i]}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_add8_bit_exact(golden, ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    g = golden["add8"][str(nb)]
    cts = [N.ints_to_words([int(h, 16) for h in g["c"][k]], ctx.ct_words) for k in range(8)]
    exps = [np.array(g["ce"][k], dtype=np.int32) for k in range(8)]
    out, oe = ctx.add(cts, exps)
    got = N.words_to_ints(out)
    for i in range(len(g["sum_c"])):
        assert (hex(got[i]), int(oe[i])) == (g["sum_c"][i], g["sum_e"][i]), f"column {i}"
    val, mant, st, _ = ctx.decrypt(out, oe)
    assert [float(v).hex() for v in val] == g["sum_dec"]


@pytest.mark.parametrize("nb", [1024, 2048])
def test_random_value_zero(golden, ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    rec = golden["random_value_zero"][str(nb)]
    x = np.array([rec["bits"]], dtype=np.uint32).view(np.float32)
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_NONE)
    assert (hex(N.words_to_ints(ct)[0]), int(ex[0])) == (rec["c"], rec["e"])


@pytest.mark.parametrize("nb", [1024, 2048])
def test_device_rng_matches_oracle_stream(ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    rng_key = bytes(range(32))
    x = np.random.default_rng(5).standard_normal(40).astype(np.float32)
    fb = ctx.has_private
    if fb:
        ctx.set_fixed_base(False)   # r from the ChaCha stream (fixed-base sampler: test_gpu_fixed_base)
    try:
        ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rng_key, index_base=1000)
    finally:
        if fb:
            ctx.set_fixed_base(True)
    got = N.words_to_ints(ct)
    rbytes = ((nb + 64 + 31) // 32) * 4
    for i in range(len(x)):
        r = O.device_r(rng_key, 1000 + i, rbytes)
        c, e = O.encrypt_value(x[i], key, r % key.n)
        assert got[i] == c and ex[i] == e
    val, _, st, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


def test_encode_edge_values_and_ints(ctxs):
    N = _native()
    ctx, key = ctxs[1024]
    xs = np.array([0.0, -0.0, 1e-300, -1e-300, 5e-324, 2.0 ** 60 + 1, -123.456, 1.0 / 3.0], dtype=np.float64)
    rs = [O.golden_r(key.n, 9, i) for i in range(len(xs))]
    ct, ex, st = ctx.encrypt(xs, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, v in enumerate(xs):
        c, e = O.encrypt_value(np.float64(v), key, rs[i])
        assert (got[i], ex[i]) == (c, e), i
    ints = np.array([0, 1, -1, 2 ** 62, -(2 ** 62), 123456789], dtype=np.int64)
    ct, ex, st = ctx.encrypt(ints, obf_mode=N.PAI_OBF_GIVEN, r=rs[:6])
    got = N.words_to_ints(ct)
    for i, v in enumerate(ints):
        c, e = O.encrypt_value(np.int64(v), key, rs[i])
        assert (got[i], ex[i]) == (c, e), i
    val, mant, st, _ = ctx.decrypt(ct, ex)
    assert list(st) == [N.EL_INT] * 6 and list(mant) == list(ints)
