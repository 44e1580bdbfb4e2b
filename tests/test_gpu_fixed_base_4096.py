"""GPU parity of the 4096-bit key holder's fixed-base sampler (kernels_grp.hpp: k_fbg on the lane-group
engine, recombined by k_crt_fin<8>), SURVEY.md §8 row (f) nb = 4096 / BASELINE configs[4]:

* bit-exact against THE REFERENCE's own 4096-bit ciphertexts under the sampler's obfuscator
  (tests/golden/paillier_golden_fb.json, made by tests/golden/make_golden_fb.py) at W = 12, 16 and 21 (the bench's);
* bit-exact against the CPU restatement (oracle/paillier_oracle.py fb_encrypt_value) at other index
  bases and ragged sizes, identical across windows, decryptable;
* the split-pair sampler (kernels_sgp.hpp: k_sgp, the default) and the pair-group k_fbgp (FLEXPAI_SGP=0) give
  identical ciphertexts from the same tables;
* round 5's lane kernels for the pairs -> w_h step and Garner's last product (k_sgp_w, k_sgp_fin) against the group
  kernels they replace (k_fbgp_w, k_fbg_fin; $FLEXPAI_SGP_FIN=0 in the test build) at counts 1, 2, 63, 129, 1000
  -- every element, so a store past an element's 256 words into its neighbour's shows;
* with the table memory capped, device-RNG encryption falls back to the public-key path (r = the ChaCha20
  stream, bit-identical to the explicit-r reference path) and decryption is unaffected."""
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


@pytest.fixture(scope="module")
def ctx4096(golden):
    N = _native()
    key = _key(golden)
    ctx = N.Context(key.n, 0, key.p, key.q)
    ctx.set_fb_window(12)               # 0.8 GB of tables: quick to build; W = 16 is tested once below
    return ctx, key


def test_fixed_base_4096_params(ctx4096):
    ctx, key = ctx4096
    assert ctx.fixed_base
    gp, gq, K, W = ctx.fixed_base_info()
    assert (gp, gq) == (O.fb_base(key.p), O.fb_base(key.q))
    assert W == 12 and K == O.fb_digits(key.p, key.q, W)
    _, _, nbytes = ctx.fixed_base_setup()
    # rows: the canonical pair as 2 x 64 32-bit words (+ 640-B Shoup rows for k_sgs, the default at this window)
    assert nbytes == 2 * K * (1 << W) * (128 * 4 + (640 if ctx.split_sampler & 8 else 0))


@pytest.mark.parametrize("window", [12, 16, 21])
def test_fixed_base_4096_matches_reference_goldens(ctx4096, golden_fb, window, monkeypatch):
    """W = 21: the factored rows' largest window on one MI355X (98 digits per half), on k_sgp ($FLEXPAI_SGS=0: Shoup
    rows beside them fit only W <= 20); W = 12, 16 on the default sampler."""
    N = _native()
    ctx, key = ctx4096
    if window == 21:
        monkeypatch.setenv("FLEXPAI_SGS", "0")
    g = golden_fb["keys"][str(NB)]
    assert (hex(key.n), hex(key.p), hex(key.q)) == (g["n"], g["p"], g["q"])
    recs = golden_fb["encrypt"][str(NB)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    try:
        ctx.set_fb_window(window)
        gp, gq, K, W = ctx.fixed_base_info()
        assert (gp, gq, W) == (g["g_p"], g["g_q"], window)
        ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes.fromhex(golden_fb["rng_key"]),
                                 index_base=golden_fb["index_base"])
    finally:
        ctx.set_fb_window(12)
    got = N.words_to_ints(ct)
    for i, r in enumerate(recs):
        assert (hex(got[i]), int(ex[i])) == (r["c"], r["e"]), f"element {i}"
    val, _, _, _ = ctx.decrypt(ct, ex)
    assert [float(v).hex() for v in val] == [r["dec"] for r in recs]


@pytest.mark.parametrize("count,base", [(1, 0), (63, 5), (65, 2 ** 33 + 1), (333, 4242)])
def test_fixed_base_4096_bit_exact(ctx4096, count, base):
    N = _native()
    ctx, key = ctx4096
    params = ctx.fixed_base_info()
    rk = bytes(range(3, 35))
    x = (np.random.default_rng(count).standard_normal(count) * 1e3).astype(np.float64)
    x[::7] = 0.0
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    val, _, _, _ = ctx.decrypt(ct, ex)
    for i in sorted({0, count // 2, count - 1}):
        assert (got[i], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, base + i, params), f"element {i}"
        assert val[i] == O.decrypt_value(got[i], int(ex[i]), key)
    # the reference's float64 encoding keeps 16^-e granularity (e = 10 here): not an exact round trip
    assert np.allclose(val, x, rtol=0, atol=2.0 ** -38)


def test_fixed_base_4096_windows_agree(ctx4096):
    """The exponent is reduced mod p_h - 1 before it is cut into digits: every window gives the same
    ciphertexts."""
    N = _native()
    ctx, _ = ctx4096
    rk = b"\x33" * 32
    x = np.random.default_rng(9).standard_normal(100).astype(np.float32)
    outs = []
    try:
        for w in (8, 12):
            ctx.set_fb_window(w)
            outs.append(ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=7)[0])
    finally:
        ctx.set_fb_window(12)
    assert np.array_equal(outs[0], outs[1])


def test_fixed_base_4096_memory_cap_falls_back(golden, monkeypatch):
    N = _native()
    key = _key(golden)
    monkeypatch.setenv("FLEXPAI_FB_MAX_BYTES", "1000000")
    monkeypatch.setenv("FLEXPAI_QUIET", "1")
    ctx = N.Context(key.n, 0, key.p, key.q)
    x = np.random.default_rng(6).standard_normal(40).astype(np.float32)
    rk = b"\x09" * 32
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=3)
    assert not ctx.fixed_base and not ctx.fb_ready
    got = N.words_to_ints(ct)
    rbytes = ((NB + 64 + 31) // 32) * 4
    for i in (0, 39):
        r = O.device_r(rk, 3 + i, rbytes) % key.n
        assert got[i] == O.encrypt_value(x[i], key, r)[0]
    val, _, _, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


def test_split_sampler_matches_group_engine(ctx4096, golden, monkeypatch, xlib):
    """k_sgp (kernels_sgp.hpp, split pairs: the default) and k_fbgp (pair groups, FLEXPAI_SGP=0 in the test build)
    read the same tables and give the same ciphertexts, ragged size, non-zero index base."""
    N = _native()
    ctx, key = ctx4096
    rk = bytes(range(40, 72))
    x = (np.random.default_rng(21).standard_normal(333) * 1e4).astype(np.float64)
    x[::5] *= -1.0
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=2 ** 32 - 3)
    assert ctx.split_sampler & 1
    monkeypatch.setenv("FLEXPAI_SGP", "0")
    ref = N.Context(key.n, 0, key.p, key.q, lib=xlib)
    ref.set_fb_window(12)
    ct2, ex2, _ = ref.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=2 ** 32 - 3)
    assert ref.fb_ready and not ref.split_sampler & 1
    assert np.array_equal(ct, ct2) and np.array_equal(ex, ex2)


@pytest.mark.parametrize("count", [1, 2, 63, 129, 1000])
def test_lane_garner_matches_group_garner(golden, monkeypatch, xlib, count):
    N = _native()
    key = _key(golden)
    rk = bytes(range(3, 35))
    x = (np.random.default_rng(count).standard_normal(count) * 1e3).astype(np.float32)
    out = []
    for fin in ("1", "0"):
        monkeypatch.setenv("FLEXPAI_SGP_FIN", fin)
        ctx = N.Context(key.n, 0, key.p, key.q, lib=xlib)
        try:
            ctx.set_fb_window(8)
            ctx.prepare_fixed_base()
            assert ctx.split_sampler & 1
            out.append(ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=7)[:2])
        finally:
            ctx.close()
    (ca, ea), (cb, eb) = out
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb)
    got = N.words_to_ints(ca[[0, count - 1]])
    assert got[0] < key.n * key.n and got[-1] < key.n * key.n
