"""GPU parity of the lane-engine CRT decryption (kernels_dec.hpp: k_dec_pre / k_dec_pow /
k_dec_fin) against the reference golden vectors, the CPU oracle (decryptor.py:33-127 restated)
and the lane-group kernel (k_decrypt): same plaintext words, values, mantissas and statuses,
including ciphertexts the reference accepts but encryption never produces (c = 0, multiples of p
or q, c >= n^2, all-ones words)."""
import math

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
    return {nb: (N.Context(_key(golden, nb).n, 0, _key(golden, nb).p, _key(golden, nb).q), _key(golden, nb))
            for nb in (1024, 2048)}


def _both(ctx, ct, ex):
    """(lane result, group result) of decrypt with raw plaintext words."""
    ctx.set_lane_decrypt(True)
    assert ctx.lane_decrypt
    a = ctx.decrypt(ct, ex, want_raw=True)
    ctx.set_lane_decrypt(False)
    assert not ctx.lane_decrypt
    b = ctx.decrypt(ct, ex, want_raw=True)
    ctx.set_lane_decrypt(True)
    return a, b


def _same(a, b):
    for x, y in zip(a, b):
        if x is None or y is None:
            assert x is None and y is None
        else:
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_lane_decrypt_not_for_4096(golden):
    N = _native()
    key = _key(golden, 4096)
    ctx = N.Context(key.n, 0, key.p, key.q)
    assert not ctx.lane_decrypt


@pytest.mark.parametrize("nb", [1024, 2048])
def test_lane_decrypt_golden(golden, ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    ct = N.ints_to_words([int(r["c"], 16) for r in recs], ctx.ct_words)
    ex = np.array([r["e"] for r in recs], dtype=np.int32)
    a, b = _both(ctx, ct, ex)
    _same(a, b)
    val, mant, st, raw = a
    for i, r in enumerate(recs):
        want = float.fromhex(r["dec"]) if isinstance(r["dec"], str) else float(r["dec"])
        assert float(val[i]) == want, f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_lane_decrypt_edge_ciphertexts(ctxs, nb):
    N = _native()
    ctx, key = ctxs[nb]
    W = ctx.ct_words
    top = (1 << (32 * W)) - 1
    cs = [0, 1, 2, key.p, key.q, 3 * key.p, key.p * key.q, key.psquare, key.qsquare, key.nsquare - 1,
          key.nsquare, key.nsquare + 12345, top, top - 1, key.p * key.p * 7 + key.q,
          (key.n + 1) % key.nsquare, pow(key.n + 1, 5, key.nsquare)]
    rng = np.random.default_rng(nb)
    cs += [int.from_bytes(rng.bytes(4 * W), "little") for _ in range(47)]
    ct = N.ints_to_words(cs, W)
    ex = np.array([(i % 7) - 2 for i in range(len(cs))], dtype=np.int32)
    a, b = _both(ctx, ct, ex)
    raw = N.words_to_ints(a[3])
    for i, c in enumerate(cs):
        assert raw[i] == O.raw_decrypt(c, key), f"element {i} (c = {c:#x})"
    # the lane-group kernel agrees wherever c is a unit mod n (it does not special-case
    # c == 0 mod p, where the reference's floor division gives L = -1)
    unit = np.array([math.gcd(c, key.n) == 1 for c in cs])
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x)[unit].view(np.uint8), np.asarray(y)[unit].view(np.uint8))
    # decoded values and statuses follow the oracle's decode of the same plaintexts
    val, mant, st, _ = a
    for i, c in enumerate(cs):
        try:
            want = O.decode(raw[i], int(ex[i]), key.n, key.max_int)
        except OverflowError:
            assert st[i] in (N.EL_OVERFLOW, N.EL_FLOAT_OVF), f"element {i}"
            continue
        if isinstance(want, int):
            assert st[i] in (N.EL_INT, N.EL_INT_BIG), f"element {i}"
            if st[i] == N.EL_INT:
                assert int(mant[i]) == want, f"element {i}"
        else:
            assert st[i] == N.EL_OK and float(val[i]) == want, f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("n", [1, 255, 257, 1000])
def test_lane_decrypt_roundtrip_ragged(ctxs, nb, n):
    N = _native()
    ctx, key = ctxs[nb]
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    x[::17] = 0.0
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=7)
    a, b = _both(ctx, ct, ex)
    _same(a, b)
    assert np.array_equal(a[0], x.astype(np.float64))


@pytest.mark.parametrize("nb", [1024, 2048])
def test_lane_decrypt_decode_statuses(ctxs, nb):
    """Plaintexts across every decode branch: +/- mantissas, overflow band, exponents <= 0 with
    int64 and wider mantissas, floats whose rounding needs the sticky bit."""
    N = _native()
    ctx, key = ctxs[nb]
    n, mx = key.n, key.max_int
    ms = [0, 1, 5, mx, mx + 1, n - mx, n - mx - 1, n - 1, n // 2, (1 << 53) + 1, (1 << 64) + 3,
          ((1 << 54) + 3) << 60, n - ((1 << 63) - 1), n - (1 << 63), (1 << 1030) + 1 if nb > 1024 else (1 << 700) + 1]
    es = [0, -1, 3, 1, 0, 2, -3, 5, 1, 0, -2, 7, 0, 0, 260]
    rs = [O.golden_r(n, 99, i) for i in range(len(ms))]
    cs = [O.raw_encrypt(m % n, key, r) for m, r in zip(ms, rs)]
    ct = N.ints_to_words(cs, ctx.ct_words)
    ex = np.array(es, dtype=np.int32)
    a, b = _both(ctx, ct, ex)
    _same(a, b)
    val, mant, st, raw = a
    assert N.words_to_ints(raw) == [m % n for m in ms]
