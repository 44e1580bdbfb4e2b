"""GPU parity of the 1024-bit public-key encryption on p-adic pairs (kernels_pe1.hpp: k_pe1_words, k_dec_pre_pair over
n, k_pe1_pow, k_pe1_fin; a party that holds only the public key of the reference protocols' default size,
sec_param.json:3) against the reference golden vectors (explicit r: encryptor.py:48-69), the CPU oracle (device ChaCha20
obfuscators, raw_encrypt.py:22-49, obfuscator.py:23-37) and the group-engine kernel it replaces (k_encrypt<2>,
$FLEXPAI_PAIR=0 in the test build): bit-identical ciphertexts, exponents and statuses."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def key1024(golden):
    k = golden["keys"]["1024"]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _ctxs(monkeypatch, key):
    """(pairs, k_encrypt<2>): the product's public context with the row kernels off, the test build's group engine."""
    N = _native()
    monkeypatch.setenv("FLEXPAI_PAIR", "1")
    a = N.Context(key.n, 0)
    a.set_rows_max(0)
    assert a.pair_paths & 4
    monkeypatch.setenv("FLEXPAI_PAIR", "0")
    b = N.Context(key.n, 0, lib=N.load_library(N.XCHECK_LIB_PATH))
    assert not b.pair_paths & 4
    return a, b


def _same(a, b):
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_pe1_golden_given_r(golden, key1024, monkeypatch):
    N = _native()
    a, b = _ctxs(monkeypatch, key1024)
    recs = golden["encrypt"]["1024"]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    ra = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    _same(ra, b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs))
    got = N.words_to_ints(ra[0])
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(ra[1][i])) == (rec["c"], rec["e"]), f"element {i}"


@pytest.mark.parametrize("count", [1, 63, 300, 5000])
def test_pe1_rng_matches_k_encrypt_and_oracle(key1024, monkeypatch, count):
    N = _native()
    a, b = _ctxs(monkeypatch, key1024)
    rng = np.random.default_rng(count)
    x = (rng.standard_normal(count) * 10.0 ** rng.integers(-30, 30, count)).astype(np.float32)
    x[::7] = 0.0
    x[1::9] = -x[1::9]
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(5, 37)), index_base=(1 << 33) + 3)
    a.set_stage_timing(True)
    ra = a.encrypt(x, **kw)
    assert len(a.stage_times()) == 3, "words + k_dec_pre_pair, k_pe1_pow, k_pe1_fin"
    _same(ra, b.encrypt(x, **kw))
    got = N.words_to_ints(ra[0][: min(count, 5)])
    rb = ((1024 + 64 + 31) // 32) * 4
    for i in range(min(count, 5)):
        c, e = O.encrypt_value(x[i], key1024, O.device_r(bytes(range(5, 37)), (1 << 33) + 3 + i, rb))
        assert (got[i], int(ra[1][i])) == (c, e), f"element {i}"


def test_pe1_edge_obfuscators_and_dtypes(key1024, monkeypatch):
    """r = 0, 1, 2, n - 1, n, n + 1, 5 p, n^2 - 1, the all-ones 64 words; a scalar r over float64 and int64 inputs."""
    N = _native()
    a, b = _ctxs(monkeypatch, key1024)
    k = key1024
    rs = [0, 1, 2, k.n - 1, k.n, k.n + 1, 5 * k.p, k.nsquare - 1, (1 << (32 * a.ct_words)) - 1]
    x = np.array([0.0, 1.0, -1.0, 3.5, -2.25, 1e-30, -1e30, 7.0, -0.0], dtype=np.float32)
    ra = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    _same(ra, b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs))
    got = N.words_to_ints(ra[0])
    for i, r in enumerate(rs):
        assert got[i] == O.encrypt_value(x[i], k, r)[0], f"r #{i}"
    r = 0x1234567890ABCDEF1234567 % k.n
    for x in (np.array([0.0, -0.0, 1.5, -2.25, 3e-30, -7e20], dtype=np.float64),
              np.array([0, 1, -1, 2 ** 40, -(2 ** 50), 123456789], dtype=np.int64)):
        _same(a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r), b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r))


def test_pe1_default_path_roundtrip(key1024):
    """At the library defaults a 10 000-element call runs the pair path (above the row kernels' 4 096) and decrypts to
    its input on the key holder's context."""
    N = _native()
    pub = N.Context(key1024.n, 0)
    pub.set_stage_timing(True)
    x = (np.random.default_rng(1).standard_normal(10000) * 1e4).astype(np.float32)
    ct, ex, st = pub.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(32), index_base=0)
    assert len(pub.stage_times()) == 3
    holder = N.Context(key1024.n, 0, key1024.p, key1024.q)
    val, _, _, _ = holder.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64))
