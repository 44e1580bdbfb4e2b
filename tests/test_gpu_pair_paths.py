"""The p-adic pair kernels (bn_pair.hpp, bn_pgroup.hpp: k_fbp, k_fbgp, k_crt_b_pair, k_dec_*_pair, k_dec4_*)
against the kernels they replace, which stay in the library behind $FLEXPAI_FB_PAIR=0 / $FLEXPAI_PAIR=0
(k_fb, k_fbg, k_crt_b, k_dec_pre/pow/fin, k_decrypt): bit-identical ciphertexts and plaintexts for the
device-RNG sampler, the generic CRT path (explicit r) and decryption, at every key size."""
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


def _ctx(monkeypatch, key, pair):
    N = _native()
    monkeypatch.setenv("FLEXPAI_FB_PAIR", "1" if pair else "0")
    monkeypatch.setenv("FLEXPAI_PAIR", "1" if pair else "0")
    ctx = N.Context(key.n, 0, key.p, key.q)
    ctx.set_fb_window(12)
    ctx.prepare_fixed_base()
    return ctx


@pytest.mark.parametrize("nb", [1024, 2048, 4096])
def test_pair_kernels_match_the_kernels_they_replace(golden, monkeypatch, nb):
    N = _native()
    key = _key(golden, nb)
    a = _ctx(monkeypatch, key, True)
    b = _ctx(monkeypatch, key, False)
    assert a.fb_pair and not b.fb_pair
    assert (a.pair_paths & 1) and not (b.pair_paths & 1)
    n = 300 if nb < 4096 else 96
    rng = np.random.default_rng(nb)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(np.float32)
    x[::11] = 0.0
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=1000)
    ca, ea, _ = a.encrypt(x, **kw)          # fixed-base sampler: pairs
    cb, eb, _ = b.encrypt(x, **kw)          # fixed-base sampler: k_fb / k_fbg
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb)
    if nb < 4096:                           # generic CRT path (explicit r): k_crt_b_pair vs k_crt_b
        rs = [O.golden_r(key.n, 5, i) for i in range(n)]
        ga, _, _ = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        gb, _, _ = b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
        assert np.array_equal(ga, gb)
        got = N.words_to_ints(ga[:8])
        for i in range(8):
            assert got[i] == O.encrypt_value(x[i], key, rs[i])[0], f"element {i}"
    da = a.decrypt(ca, ea, want_raw=True)
    db = b.decrypt(ca, ea, want_raw=True)
    for u, v in zip(da, db):
        assert np.array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
    assert np.array_equal(da[0], x.astype(np.float64))
