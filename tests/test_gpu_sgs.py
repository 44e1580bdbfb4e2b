"""GPU parity of the Shoup-row split-pair sampler for 4096-bit keys (kernels_sgs.hpp: k_sgs_conv, k_sgs, k_sgs_bfin;
the default where it prices below the factored rows, flexpai.hip fb_choose; $FLEXPAI_SGS=0 keeps k_sgp), VERDICT r4
item 3, reference semantics /root/reference/flex/crypto/paillier/obfuscator.py:36
(r^n mod n^2 with the sampler's r):

* the same ciphertexts and exponents as the Montgomery sampler (k_sgp, $FLEXPAI_SGS=0) from the same digits, at ragged
  counts (one element leaves 127 of a block's lane pairs clamped) and a non-zero index base;
* bit-exact against THE REFERENCE's own 4096-bit ciphertexts under the sampler's obfuscator
  (tests/golden/paillier_golden_fb.json) at W = 12 and 16;
* the test build's address guards (guard.hpp) on k_sgs's row / b-row DMA indices, digits and stores: zero hits."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

NB = 4096


def _native():
    from flex.crypto.paillier import _native
    return _native


def _key(golden):
    k = golden["keys"][str(NB)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _encrypt(key, x, window, sgs, monkeypatch, lib=None, base=7):
    N = _native()
    monkeypatch.setenv("FLEXPAI_SGS", "1" if sgs else "0")
    ctx = N.Context(key.n, 0, key.p, key.q, lib=lib) if lib is not None else N.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(window)
        ctx.prepare_fixed_base()
        assert ctx.fb_ready and ctx.split_sampler & 1
        assert bool(ctx.split_sampler & 8) == sgs
        ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(9, 41)), index_base=base)
        return ct, ex
    finally:
        ctx.close()


@pytest.mark.parametrize("count", [1, 63, 129, 1000])
def test_shoup_sampler_matches_montgomery_sampler(golden, monkeypatch, count):
    key = _key(golden)
    x = (np.random.default_rng(count + 5).standard_normal(count) * 1e4).astype(np.float64)
    x[::3] *= -1.0
    ca, ea = _encrypt(key, x, 8, True, monkeypatch, base=2 ** 32 - 5)
    cb, eb = _encrypt(key, x, 8, False, monkeypatch, base=2 ** 32 - 5)
    assert np.array_equal(ea, eb)
    assert np.array_equal(ca, cb)


@pytest.mark.parametrize("window", [12, 16])
def test_shoup_sampler_matches_reference_goldens(golden, golden_fb, monkeypatch, window):
    N = _native()
    key = _key(golden)
    g = golden_fb["keys"][str(NB)]
    assert (hex(key.n), hex(key.p), hex(key.q)) == (g["n"], g["p"], g["q"])
    recs = golden_fb["encrypt"][str(NB)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    monkeypatch.setenv("FLEXPAI_SGS", "1")
    ctx = N.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(window)
        ctx.prepare_fixed_base()
        assert ctx.split_sampler & 8
        ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes.fromhex(golden_fb["rng_key"]),
                                index_base=golden_fb["index_base"])
        got = N.words_to_ints(ct)
        for i, r in enumerate(recs):
            assert (hex(got[i]), int(ex[i])) == (r["c"], r["e"]), f"element {i}"
        val, _, _, _ = ctx.decrypt(ct, ex)
        assert [float(v).hex() for v in val] == [r["dec"] for r in recs]
    finally:
        ctx.close()


@pytest.mark.parametrize("count", [1, 129])
def test_shoup_sampler_guarded(golden, monkeypatch, xlib, count):
    """The test build (address guards on, guard.hpp): the Shoup sampler's indices stay inside their buffers, and its
    ciphertexts equal the product library's Montgomery sampler's."""
    key = _key(golden)
    x = (np.random.default_rng(count).standard_normal(count) * 1e3).astype(np.float32)
    ca, ea = _encrypt(key, x, 8, True, monkeypatch, lib=xlib)
    cb, eb = _encrypt(key, x, 8, False, monkeypatch)
    assert np.array_equal(ea, eb) and np.array_equal(ca, cb)


def test_shoup_rows_are_the_default_where_they_price_lower(golden, monkeypatch):
    """fb_choose: at W = 12 both tables fit, and 0.835 K(12) < K(12): Shoup rows without $FLEXPAI_SGS; with a budget
    that fits only the factored rows, k_sgp."""
    N = _native()
    key = _key(golden)
    monkeypatch.delenv("FLEXPAI_SGS", raising=False)
    ctx = N.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(12)
        ctx.prepare_fixed_base()
        assert ctx.split_sampler & 8
        K, W = ctx.fixed_base_info()[2:]
        assert W == 12 and ctx.fixed_base_setup()[2] == 2 * K * (1 << W) * (512 + 640)
    finally:
        ctx.close()
    monkeypatch.setenv("FLEXPAI_FB_MAX_BYTES", str(2 * 171 * (1 << 12) * 512 + 1000))
    ctx = N.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(12)
        ctx.prepare_fixed_base()
        assert ctx.fb_ready and not ctx.split_sampler & 8 and ctx.fixed_base_info()[3] == 12
    finally:
        ctx.close()
