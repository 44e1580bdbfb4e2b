"""The table samplers under the test build's address guards (csrc/guard.hpp).

libflexpai_xcheck.so checks, in k_fb_digits, k_fbs_fill, k_fbs, k_sgp and k_fbp_fin, every index formed from a digit,
a row number or the element count against the size of the buffer it addresses (as flexpai.hip allocated it). A
violation is recorded, the index clamped (no access leaves its buffer, so no GPU fault) and the call fails with the
site. Here:

* ragged element counts around the 64-element tile and the 128-pair block -- 1, 63, 64, 65, 127, 129 -- through the
  key holder's sampler at S = 19 (nb = 1024) and S = 37 (nb = 2048), the 4096-bit key holder's k_sgp and the public
  fixed-base k_sgp, every element (or first/middle/last at 4096) against the oracle's restatement of the reference
  (oracle/paillier_oracle.py fb_encrypt_value / pfb_encrypt_value: `pe.encrypt(x, random_value=r)` for the
  sampler's r, obfuscator.py:35-37, raw_encrypt.py:37-45), then decrypted;
* the guard's self-test: $FLEXPAI_GUARD_INJECT=rows hands the kernels a one-row table, every row index trips, the
  call fails naming "k_fbs row index" (resp. "k_sgp row index") -- and the next call on the same context is clean;
  the product library ignores the variable.
"""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

COUNTS = [1, 63, 64, 65, 127, 129]


def _key(golden, nb):
    k = golden["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _x(count):
    x = (np.random.default_rng(1000 + count).standard_normal(count) * 1000).astype(np.float32)
    x[::7] = 0.0
    x[2::9] *= -1e5
    return x


@pytest.fixture(scope="module")
def holders(golden, xlib):
    from flex.crypto.paillier import _native as N
    out = {}
    for nb, w in ((1024, 8), (2048, 8), (4096, 12)):
        key = _key(golden, nb)
        ctx = N.Context(key.n, 0, key.p, key.q, lib=xlib)
        ctx.set_fb_window(w)
        ctx.prepare_fixed_base()        # k_fbs_fill (or the 4096 builders) under the guards
        out[nb] = (ctx, key, ctx.fixed_base_info())
    yield out
    for ctx, _, _ in out.values():
        ctx.close()


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", COUNTS)
def test_guarded_key_holder_sampler_ragged(holders, nb, count):
    from flex.crypto.paillier import _native as N
    ctx, key, params = holders[nb]
    assert ctx.split_sampler & 4 and ctx.fb_pair == (19 if nb == 1024 else 37)   # k_fbs on Shoup rows
    rk = bytes(range(17, 49))
    base = 3 * count + 11
    x = _x(count)
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    for i in range(count):
        assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, base + i, params), (nb, count, i)
    val, _, _, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


@pytest.mark.parametrize("count", COUNTS)
def test_guarded_4096_sampler_ragged(holders, count):
    from flex.crypto.paillier import _native as N
    ctx, key, params = holders[4096]
    rk = bytes(range(5, 37))
    base = 2 ** 32 + count
    x = _x(count)
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    for i in sorted({0, count // 2, count - 1}):
        assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, base + i, params), (count, i)
    val, _, _, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


@pytest.fixture(scope="module")
def public(golden, xlib):
    from flex.crypto.paillier import _native as N
    key = _key(golden, 2048)
    ctx = N.Context(key.n, 0, lib=xlib)
    ctx.set_pfb_window(12)
    ctx.prepare_public_fixed_base()
    dec = N.Context(key.n, 0, key.p, key.q)
    yield ctx, dec, key
    ctx.close()
    dec.close()


@pytest.mark.parametrize("count", COUNTS)
def test_guarded_public_sampler_ragged(public, count):
    from flex.crypto.paillier import _native as N
    ctx, dec, key = public
    bases, _, W, _ = ctx.public_fixed_base_info()
    rk = bytes(range(70, 102))
    base = 7 * count
    x = _x(count)
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    for i in sorted({0, count // 2, count - 1}):
        assert (got[i], int(ex[i])) == O.pfb_encrypt_value(x[i], key, bases, rk, base + i, W), (count, i)
    val, _, _, _ = dec.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


@pytest.mark.parametrize("nb,site", [(2048, "k_fbs row index"), (4096, "k_sgp row index")])
def test_guard_self_test_injected_row_limit(holders, monkeypatch, nb, site):
    from flex.crypto.paillier import _native as N
    ctx, key, params = holders[nb]
    rk = bytes(range(32))
    x = _x(65)
    monkeypatch.setenv("FLEXPAI_GUARD_INJECT", "rows")
    with pytest.raises(N.NativeError, match="address guard") as ei:
        ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=0)
    assert site in str(ei.value)
    monkeypatch.delenv("FLEXPAI_GUARD_INJECT")
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=0)   # the record was reset
    got = N.words_to_ints(ct)
    assert (got[64], int(ex[64])) == O.fb_encrypt_value(x[64], key, rk, 64, params)


def test_product_library_ignores_the_injection(golden, monkeypatch):
    from flex.crypto.paillier import _native as N
    key = _key(golden, 1024)
    ctx = N.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(8)
        ctx.prepare_fixed_base()
        monkeypatch.setenv("FLEXPAI_GUARD_INJECT", "rows")
        rk = bytes(range(32))
        x = _x(65)
        ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=0)
        got = N.words_to_ints(ct)
        params = ctx.fixed_base_info()
        assert (got[1], int(ex[1])) == O.fb_encrypt_value(x[1], key, rk, 1, params)
    finally:
        ctx.close()
