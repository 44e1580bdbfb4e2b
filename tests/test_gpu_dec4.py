"""GPU parity of the 4096-bit split-pair decryption (kernels_dec4.hpp: k_dec4_pre / k_dec4_pow / k_dec4_L /
k_dec4_fin) against the reference golden vectors, the CPU oracle (decryptor.py:33-127 restated) and the
lane-group kernel k_decrypt (PAI_OPT_LANE_DECRYPT = 0 selects it): same plaintext words, values, mantissas
and statuses, including ciphertexts the reference accepts but encryption never produces."""
import math

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def ctx4(golden):
    N = _native()
    k = golden["keys"]["4096"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    return N.Context(key.n, 0, key.p, key.q), key


def _both(ctx, ct, ex):
    """(split-pair result, group-engine result)."""
    ctx.set_lane_decrypt(True)
    assert ctx.pair_paths & 1
    a = ctx.decrypt(ct, ex, want_raw=True)
    ctx.set_lane_decrypt(False)
    assert not ctx.pair_paths & 1
    b = ctx.decrypt(ct, ex, want_raw=True)
    ctx.set_lane_decrypt(True)
    return a, b


def test_dec4_golden(golden, ctx4):
    N = _native()
    ctx, key = ctx4
    recs = golden["encrypt"]["4096"]
    ct = N.ints_to_words([int(r["c"], 16) for r in recs], ctx.ct_words)
    ex = np.array([r["e"] for r in recs], dtype=np.int32)
    a, b = _both(ctx, ct, ex)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    raw = N.words_to_ints(a[3])
    for i, r in enumerate(recs):
        assert raw[i] == O.raw_decrypt(int(r["c"], 16), key), f"element {i}"
        assert float(a[0][i]).hex() == r["dec"], f"element {i}"


def test_dec4_edge_ciphertexts(ctx4):
    N = _native()
    ctx, key = ctx4
    W = ctx.ct_words
    top = (1 << (32 * W)) - 1
    cs = [0, 1, 2, key.p, key.q, 3 * key.p, key.p * key.q, key.psquare, key.qsquare, key.nsquare - 1,
          key.nsquare, key.nsquare + 12345, top, top - 1, key.p * key.p * 7 + key.q,
          (key.n + 1) % key.nsquare, pow(key.n + 1, 5, key.nsquare)]
    rng = np.random.default_rng(4096)
    cs += [int.from_bytes(rng.bytes(4 * W), "little") for _ in range(31)]
    ct = N.ints_to_words(cs, W)
    ex = np.array([(i % 7) - 2 for i in range(len(cs))], dtype=np.int32)
    a, b = _both(ctx, ct, ex)
    raw = N.words_to_ints(a[3])
    for i, c in enumerate(cs):
        assert raw[i] == O.raw_decrypt(c, key), f"element {i} (c = {c:#x})"
    unit = np.array([math.gcd(c, key.n) == 1 for c in cs])
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x)[unit].view(np.uint8), np.asarray(y)[unit].view(np.uint8))


@pytest.mark.parametrize("n", [1, 127, 129, 1000])
def test_dec4_roundtrip_ragged(ctx4, n):
    N = _native()
    ctx, key = ctx4
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    x[::13] = 0.0
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=11)
    val, mant, st, raw = ctx.decrypt(ct, ex, want_raw=True)
    assert np.array_equal(val, x.astype(np.float64))
    k = min(n, 24)
    got = N.words_to_ints(raw[:k])
    for i, c in enumerate(N.words_to_ints(ct[:k])):
        assert got[i] == O.raw_decrypt(c, key), f"element {i}"
