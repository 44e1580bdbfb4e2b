"""GPU parity of the Shoup-row sampler (kernels_fbs.hpp: k_fbs_fill builds the rows, k_fbs samples on split lane
pairs), the product's key-holder sampler at 1024/2048 bits: the same distribution and the same canonical pairs out as
k_fbp (Montgomery rows; the test build with $FLEXPAI_FBS=0), so the ciphertexts must be bit-identical to k_fbp's and
to the reference's own ciphertexts under the sampler's obfuscator (tests/golden/paillier_golden_fb.json, made by
tests/golden/make_golden_fb.py)."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

ROW_BYTES = {1024: 224, 2048: 448}   # a limbs (QA quads), a' limbs (QAP), b R words (QB): 5 + 5 + 4 and 10 + 10 + 8


def _key(golden, nb):
    k = golden["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _ctx(N, key, shoup, monkeypatch, window):
    """shoup: the product library; else the test build with $FLEXPAI_FBS=0 (k_fbp)."""
    if shoup:
        ctx = N.Context(key.n, 0, key.p, key.q)
    else:
        monkeypatch.setenv("FLEXPAI_FBS", "0")
        ctx = N.Context(key.n, 0, key.p, key.q, lib=N.load_library(N.XCHECK_LIB_PATH))
    ctx.set_fb_window(window)
    ctx.prepare_fixed_base()
    monkeypatch.delenv("FLEXPAI_FBS", raising=False)   # the choice is made at table build
    return ctx


@pytest.mark.parametrize("nb", [1024, 2048])
def test_shoup_rows_match_montgomery_rows_and_oracle(golden, monkeypatch, nb):
    from flex.crypto.paillier import _native as N
    key = _key(golden, nb)
    rk = bytes(range(90, 122))
    outs = {}
    for shoup in (False, True):
        ctx = _ctx(N, key, shoup, monkeypatch, 16)
        try:
            assert bool(ctx.split_sampler & 4) == shoup
            assert ctx.fb_pair == (19 if nb == 1024 else 37)
            gp, gq, K, W = params = ctx.fixed_base_info()
            if shoup:
                assert ctx.fixed_base_setup()[2] == 2 * K * (1 << W) * ROW_BYTES[nb]
            res = []
            for count, base in ((1, 0), (127, 5), (129, 2 ** 33 + 1), (5001, 777)):   # ragged against 128 pairs/block
                x = (np.random.default_rng(count).standard_normal(count) * 1000).astype(np.float32)
                x[::11] = 0.0
                x[3::17] *= -1e6
                ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
                assert np.all(st == 0)
                res.append((ct, ex))
                if shoup:
                    got = N.words_to_ints(ct)
                    for i in sorted({0, count // 2, count - 1}):
                        assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, base + i, params), (count, i)
                    val, _, _, _ = ctx.decrypt(ct, ex)
                    assert np.array_equal(val, x.astype(np.float64))
            outs[shoup] = res
        finally:
            ctx.close()
    for (a, ea), (b, eb) in zip(outs[False], outs[True]):
        assert np.array_equal(a, b) and np.array_equal(ea, eb)


@pytest.mark.parametrize("nb,window", [(1024, 20), (2048, 16), (2048, 20), (2048, 22)])
def test_shoup_rows_match_reference_goldens(golden, golden_fb, monkeypatch, nb, window):
    """The reference's own ciphertexts (window-independent: a_h is reduced mod p_h - 1 before it is cut into
    digits); W = 22 is the largest nb = 2048 window whose Shoup tables (2 x 88.3 GB) fit one MI355X."""
    from flex.crypto.paillier import _native as N
    key = _key(golden, nb)
    g = golden_fb["keys"][str(nb)]
    recs = golden_fb["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    ctx = _ctx(N, key, True, monkeypatch, window)
    try:
        assert ctx.split_sampler & 4
        gp, gq, K, W = ctx.fixed_base_info()
        assert (gp, gq, W) == (g["g_p"], g["g_q"], window)
        ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes.fromhex(golden_fb["rng_key"]),
                                index_base=golden_fb["index_base"])
        got = N.words_to_ints(ct)
        for i, r in enumerate(recs):
            assert (hex(got[i]), int(ex[i])) == (r["c"], r["e"]), f"element {i}"
        val, _, _, _ = ctx.decrypt(ct, ex)
        assert [float(v).hex() for v in val] == [r["dec"] for r in recs]
    finally:
        ctx.close()


def test_shoup_rows_full_size_1m(golden, monkeypatch):
    """configs[1]'s 1M elements at nb = 2048: Shoup rows at W = 22 bit-identical to k_fbp's Montgomery rows (at
    W = 16: the ciphertexts do not depend on the window), round trip exact."""
    from flex.crypto.paillier import _native as N
    key = _key(golden, 2048)
    n = 1 << 20
    x = np.random.default_rng(12).standard_normal(n).astype(np.float32)
    rk = bytes(range(200, 232))
    ctx = _ctx(N, key, False, monkeypatch, 16)
    try:
        ref, rex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=4096)
    finally:
        ctx.close()
    ctx = _ctx(N, key, True, monkeypatch, 22)
    try:
        assert ctx.split_sampler & 4 and ctx.fixed_base_info()[3] == 22
        ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=4096)
        assert np.all(st == 0)
        assert np.array_equal(ct, ref) and np.array_equal(ex, rex)
        val, _, dst, _ = ctx.decrypt(ct, ex)
        assert np.array_equal(val, x.astype(np.float64))
    finally:
        ctx.close()


@pytest.mark.parametrize("pbits", [(1020, 1021), (1016, 1017), (508, 509)])
def test_shoup_rows_short_primes(monkeypatch, pbits):
    """Primes below the full half size (n of 2041, 2033 and 1017 bits; 2033 is the shortest 2048-class n whose n^2
    still fills the 128-word rows the fixed-base path requires): Shoup's mu = floor(R^2 / p_h) takes more limbs and a'
    stays below R. Sampler bit-exact against the oracle and against k_fbp of the test build; decrypts."""
    from flex.crypto.paillier import _native as N
    from tests.test_gpu_pair_paths import _prime
    rng = np.random.default_rng(sum(pbits))
    while True:
        p, q = _prime(pbits[0], rng), _prime(pbits[1], rng)
        if p < q < 2 * p:
            break
    key = O.Key(p * q, p, q)
    x = (rng.standard_normal(300) * 100).astype(np.float32)
    rk = bytes(range(3, 35))
    outs = []
    for shoup in (True, False):
        ctx = _ctx(N, key, shoup, monkeypatch, 12)
        try:
            assert bool(ctx.split_sampler & 4) == shoup and ctx.fb_ready
            params = ctx.fixed_base_info()
            ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=17)
            assert np.all(st == 0)
            outs.append((ct, ex))
            if shoup:
                got = N.words_to_ints(ct)
                for i in (0, 150, 299):
                    assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, 17 + i, params), i
                assert np.array_equal(ctx.decrypt(ct, ex)[0], x.astype(np.float64))
        finally:
            ctx.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
