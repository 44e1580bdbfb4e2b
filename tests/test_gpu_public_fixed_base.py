"""GPU parity of the public-key fixed-base sampler (kernels_pfb.hpp), device-RNG encryption for parties that
hold only the public key (HE_OTP_LR host, he_otp_lr_ft1/train.py:135,164; HE_LR_FP host, he_lr_fp/predict.py:
114,127):

* bit-exact against THE REFERENCE's own ciphertexts (tests/golden/paillier_golden_pfb.json: the reference's
  pe.encrypt(x, random_value=r) for r = prod_j g_j^e_j mod n, made by tests/golden/make_golden_pfb.py) at the
  windows 12, 16 and 20, with the golden's bases set through pai_ctx_public_fb_set_bases;
* bit-exact against the oracle's restatement (oracle/paillier_oracle.py pfb_*) with the bases the context drew
  itself (g_0 with Jacobi symbol -1), at ragged sizes and index bases; decryptable; the publicly visible Jacobi
  symbol of c mod n uniform +-1 (as for r uniform in Z_n*);
* the split-pair sampler (kernels_sgp.hpp: k_sgp, the default) and the pair-group k_pfb (FLEXPAI_SGP=0) give
  identical ciphertexts;
* below the break-even count a fresh public key encrypts on k_pe_* (ChaCha20 r, bit-exact vs the explicit-r
  reference path) and builds no tables; 1M elements round-trip exactly."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def _native():
    from flex.crypto.paillier import _native
    return _native


def _golden_key(g):
    k = g["keys"]["2048"]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16)), [int(b, 16) for b in k["bases"]]


@pytest.fixture(scope="module")
def pub(golden_pfb):
    N = _native()
    key, bases = _golden_key(golden_pfb)
    ctx = N.Context(key.n, 0)                     # the public key only
    dec = N.Context(key.n, 0, key.p, key.q)       # a key holder, for decryption checks
    return ctx, dec, key, bases


def _jacobi_stats(js):
    plus = sum(1 for j in js if j == 1)
    return plus, len(js)


@pytest.mark.parametrize("window", [12, 16, 20])
def test_public_fixed_base_matches_reference_goldens(pub, golden_pfb, window):
    N = _native()
    ctx, dec, key, bases = pub
    assert not ctx.has_private and ctx.public_fixed_base
    ctx.set_public_bases(bases)
    ctx.set_pfb_window(window)
    ctx.prepare_public_fixed_base()
    gb, K, W, K0 = ctx.public_fixed_base_info()
    assert gb == bases and W == window and (K0, (K - K0) // O.PFB_SHORT) == O.pfb_layout(2048, window)
    recs = golden_pfb["encrypt"]["2048"][str(window)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes.fromhex(golden_pfb["rng_key"]),
                             index_base=golden_pfb["index_base"])
    got = N.words_to_ints(ct)
    for i, r in enumerate(recs):
        assert (hex(got[i]), int(ex[i])) == (r["c"], r["e"]), f"element {i}"
    val, _, _, _ = dec.decrypt(ct, ex)
    assert [float(v).hex() for v in val] == [r["dec"] for r in recs]


@pytest.fixture(scope="module")
def drawn(golden):
    """A public context that draws its own bases (the library default, W = 16)."""
    N = _native()
    k = golden["keys"]["2048"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = N.Context(key.n, 0)
    ctx.prepare_public_fixed_base()
    return ctx, N.Context(key.n, 0, key.p, key.q), key


def test_drawn_bases(drawn):
    ctx, _, key = drawn
    bases, K, W, K0 = ctx.public_fixed_base_info()
    assert len(bases) == 1 + O.PFB_SHORT and len(set(bases)) == len(bases)
    assert all(1 < g < key.n for g in bases) and O.jacobi(bases[0], key.n) == -1
    assert W == 16 and (K0, (K - K0) // O.PFB_SHORT) == O.pfb_layout(2048, 16)


@pytest.mark.parametrize("count,base", [(1, 0), (63, 5), (65, 2 ** 33 + 1), (1000, 123457)])
def test_drawn_bases_bit_exact(drawn, count, base):
    N = _native()
    ctx, dec, key = drawn
    bases, _, W, _ = ctx.public_fixed_base_info()
    rk = bytes(range(60, 92))
    x = (np.random.default_rng(count).standard_normal(count) * 100).astype(np.float32)
    x[::11] = 0.0
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    for i in sorted({0, count // 2, count - 1}):
        assert (got[i], int(ex[i])) == O.pfb_encrypt_value(x[i], key, bases, rk, base + i, W), f"element {i}"
    val, _, _, _ = dec.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))


def test_public_fixed_base_jacobi_statistics(drawn):
    """c mod n = r^n mod n has Jacobi symbol (r | n): uniform +-1 for the reference's r; g_0's symbol is -1 and
    e_0 is uniform, so the sampler's symbol is uniform too."""
    N = _native()
    ctx, _, key = drawn
    M = 2000
    ct, _, _ = ctx.encrypt(np.zeros(M, dtype=np.float32), obf_mode=N.PAI_OBF_RNG, rng_key=b"q" * 32)
    plus, tot = _jacobi_stats([O.jacobi(c % key.n, key.n) for c in N.words_to_ints(ct)])
    assert abs(plus - M / 2) < 5 * (M / 4) ** 0.5


def test_public_fresh_key_small_call_uses_pe(golden, monkeypatch):
    """Below the break-even count a fresh public context builds no tables: k_pe_* with the ChaCha20 r,
    bit-exact against the reference path with that explicit r."""
    N = _native()
    monkeypatch.delenv("FLEXPAI_PFB_MIN_ELEMS", raising=False)
    k = golden["keys"]["2048"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = N.Context(key.n, 0)
    seen, thr = ctx.public_fixed_base_policy()
    assert seen == 0 and thr > 50_000
    x = np.random.default_rng(4).standard_normal(256).astype(np.float32)
    rk = bytes(range(32))
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=9)
    assert not ctx.pfb_ready and ctx.public_fixed_base_policy()[0] == 256
    got = N.words_to_ints(ct)
    rbytes = ((2048 + 64 + 31) // 32) * 4
    for i in (0, 255):
        assert got[i] == O.encrypt_value(x[i], key, O.device_r(rk, 9 + i, rbytes) % key.n)[0]


def test_public_full_size_roundtrip(drawn):
    N = _native()
    ctx, dec, key = drawn
    n = 1 << 20
    x = np.random.default_rng(1).standard_normal(n, dtype=np.float32)
    rk = bytes(range(1, 33))
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=0)
    assert np.all(st == 0)
    val, _, dst, _ = dec.decrypt(ct, ex)
    assert np.all(dst == 0) and np.array_equal(val, x.astype(np.float64))
    bases, _, W, _ = ctx.public_fixed_base_info()
    idx = [0, n // 2, n - 1]
    got = N.words_to_ints(ct[idx])
    for j, i in enumerate(idx):
        assert (got[j], int(ex[i])) == O.pfb_encrypt_value(x[i], key, bases, rk, i, W)
    half, _, _ = ctx.encrypt(x[n // 2:], obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=n // 2)
    assert np.array_equal(half, ct[n // 2:])


def test_split_sampler_matches_group_engine(pub, golden_pfb, monkeypatch, xlib):
    """k_sgp (split pairs, the default) and k_pfb (pair groups, FLEXPAI_SGP=0 in the test build) over the same bases
    and window: identical ciphertexts."""
    N = _native()
    ctx, dec, key, bases = pub
    rk = b"\x5a" * 32
    x = np.random.default_rng(33).standard_normal(257).astype(np.float32)
    outs = []
    for sgp in ("1", "0"):
        monkeypatch.setenv("FLEXPAI_SGP", sgp)
        c = N.Context(key.n, 0, lib=None if sgp == "1" else xlib)
        c.set_public_bases(bases)
        c.set_pfb_window(12)
        c.prepare_public_fixed_base()
        assert bool(c.split_sampler & 2) == (sgp == "1")
        outs.append(c.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=77)[:2])
        del c
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    val, _, st, _ = dec.decrypt(outs[0][0], outs[0][1])
    assert np.array_equal(np.asarray(val, dtype=np.float64), x.astype(np.float64))


def test_public_break_even_follows_the_measured_model(golden, monkeypatch):
    """pai_ctx_public_fb_policy's threshold is the measured model (tools/pfb_breakeven.py): build 0.114 s + 1.91 ns per
    row, saving 1/552 k - 1/rate(W) s per element (the factored k_pe chain against k_sgp at 3.93 M enc/s at the default
    W = 16; profiles/r06e_pfb_breakeven.json)."""
    N = _native()
    monkeypatch.delenv("FLEXPAI_PFB_MIN_ELEMS", raising=False)
    k = golden["keys"]["2048"]
    ctx = N.Context(int(k["n"], 16), 0)
    try:
        _, thr = ctx.public_fixed_base_policy()
        K0, KS = O.pfb_layout(2048, 16)
        rows = (K0 + O.PFB_SHORT * KS) << 16
        want = int((0.114 + rows * 1.91e-9) / (1 / 5.52e5 - 1 / 3.93e6)) + 1
        assert abs(thr - want) <= 1 and 90_000 < thr < 110_000
    finally:
        ctx.close()
