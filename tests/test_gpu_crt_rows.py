"""GPU parity of the 16-lane-row kernels (kernels_crtw.hpp: calls of at most PAI_OPT_ROWS_MAX elements) against the
kernels they stand in for (forced with rows_max = 0) and the CPU oracle (oracle/paillier_oracle.py: raw_encrypt.py:22-49,
obfuscator.py:23-37, decryptor.py:33-127 of the reference): the key holder's CRT encryption k_crt_w (against k_crt_a +
k_crt_b_pair) and decryption k_dec_w (against k_dec_pre/pow_pair), and a public-key-only party's encryption k_pe_w
(against k_pe_* at 2048 bits, k_encrypt at 1024). Bit-exact on every obfuscator mode, ragged counts and edge inputs."""
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
    for nb in (1024, 2048):
        key = _key(golden, nb)
        crt = N.Context(key.n, 0, key.p, key.q)
        crt.set_fixed_base(False)          # the generic r^n path (the sampler: test_gpu_fixed_base / test_gpu_fbs)
        pub = N.Context(key.n, 0)
        out[nb] = (crt, pub, key)
    return out


def _both(crt, *args, **kw):
    """(rows, lanes): the same call on k_crt_w and on k_crt_a + k_crt_b_pair, with the kernel count of each."""
    crt.set_stage_timing(True)
    try:
        a = crt.encrypt(*args, **kw)
        ka = len(crt.stage_times())
        old = crt.rows_max
        crt.set_rows_max(0)
        try:
            b = crt.encrypt(*args, **kw)
            kb = len(crt.stage_times())
        finally:
            crt.set_rows_max(old)
    finally:
        crt.set_stage_timing(False)
    assert (ka, kb) == (2, 3), "k_crt_w + k_crt_fin against k_crt_a + k_crt_b_pair + k_crt_fin"
    return a, b


def test_rows_default_threshold(ctxs):
    N = _native()
    crt, _, _ = ctxs[2048]
    assert crt.rows_max == 4096
    with pytest.raises(N.NativeError):
        crt.set_rows_max(-1)
    assert crt.rows_max == 4096


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 3, 4, 5, 17, 1000])
def test_rows_rng_matches_lanes_and_oracle(ctxs, nb, count):
    N = _native()
    crt, pub, key = ctxs[nb]
    x = np.random.default_rng(7 + count).standard_normal(count).astype(np.float32)
    rk = bytes(range(3, 35))
    base = (1 << 33) + 977                      # the element index's high word reaches the ChaCha nonce
    a, b = _both(crt, x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    got = N.words_to_ints(a[0])
    rbytes = ((nb + 64 + 31) // 32) * 4
    for i in sorted({0, count // 2, count - 1}):
        c, e = O.encrypt_value(x[i], key, O.device_r(rk, base + i, rbytes))
        assert got[i] == c and int(a[1][i]) == e, f"element {i}"
    if count == 17:
        p = pub.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
        assert np.array_equal(a[0], p[0])


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_golden_given_r(golden, ctxs, nb):
    N = _native()
    crt, _, _ = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    a, b = _both(crt, x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(a[0])
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(a[1][i])) == (rec["c"], rec["e"]), f"element {i}"
    assert np.array_equal(a[0], b[0])


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_edge_obfuscators(ctxs, nb):
    """r = 1, 2, n - 1, multiples of p and of q, r as wide as n^2 - 1, r = n + 1 and r = n (=> c = 0)."""
    N = _native()
    crt, _, key = ctxs[nb]
    n, p, q = key.n, key.p, key.q
    rs = [1, 2, n - 1, p, 3 * q, p * 7, n * n - 1, (n * n) // 3, n + 1, n, p - 1, q + 1]
    x = np.linspace(-5, 5, len(rs)).astype(np.float32)
    a, b = _both(crt, x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    assert np.array_equal(a[0], b[0])
    got = N.words_to_ints(a[0])
    for i, r in enumerate(rs):
        c, e = O.encrypt_value(x[i], key, r)
        assert got[i] == c, f"r index {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_scalar_r_and_dtypes(ctxs, nb):
    """random_value reused for every element (encryptor.py:92-95); float64 and int64 inputs."""
    N = _native()
    crt, pub, key = ctxs[nb]
    r = 0x1234567890ABCDEF1234567 % key.n
    for x in (np.array([0.0, -0.0, 1.5, -2.25, 3e-30, -7e20], dtype=np.float64),
              np.array([0, 1, -1, 2 ** 40, -(2 ** 50), 123456789], dtype=np.int64)):
        a, b = _both(crt, x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        c = pub.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        assert np.array_equal(a[0], c[0]) and np.array_equal(a[1], c[1])


def test_rows_threshold_boundary(ctxs):
    """rows_max elements run on rows, one more on the lane kernels; the bits agree."""
    N = _native()
    crt, _, key = ctxs[1024]
    old = crt.rows_max
    rk = b"t" * 32
    x = np.random.default_rng(3).standard_normal(65).astype(np.float32)
    crt.set_stage_timing(True)
    try:
        crt.set_rows_max(64)
        a = crt.encrypt(x[:64], obf_mode=N.PAI_OBF_RNG, rng_key=rk)
        assert len(crt.stage_times()) == 2
        b = crt.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk)
        assert len(crt.stage_times()) == 3
    finally:
        crt.set_rows_max(old)
        crt.set_stage_timing(False)
    assert np.array_equal(a[0], b[0][:64])


# ---------------------------------------------------------------- decryption on rows (k_dec_w + k_dec_fin_pair)
def _dboth(ctx, ct, ex):
    """(rows, pairs): decrypt with raw plaintext words on k_dec_w and on k_dec_pre/pow_pair, with the kernel counts."""
    ctx.set_stage_timing(True)
    try:
        a = ctx.decrypt(ct, ex, want_raw=True)
        ka = len(ctx.stage_times())
        old = ctx.rows_max
        ctx.set_rows_max(0)
        try:
            b = ctx.decrypt(ct, ex, want_raw=True)
            kb = len(ctx.stage_times())
        finally:
            ctx.set_rows_max(old)
    finally:
        ctx.set_stage_timing(False)
    assert (ka, kb) == (2, 3), "k_dec_w + k_dec_fin_pair against k_dec_pre_pair + k_dec_pow_pair + k_dec_fin_pair"
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    return a


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_decrypt_golden(golden, ctxs, nb):
    N = _native()
    crt, _, _ = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    ct = N.ints_to_words([int(r["c"], 16) for r in recs], crt.ct_words)
    ex = np.array([r["e"] for r in recs], dtype=np.int32)
    val = _dboth(crt, ct, ex)[0]
    for i, r in enumerate(recs):
        want = float.fromhex(r["dec"]) if isinstance(r["dec"], str) else float(r["dec"])
        assert float(val[i]) == want, f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_decrypt_edge_ciphertexts(ctxs, nb):
    """c = 0, multiples of p, q, p^2, q^2 (x_h = 0 or p_h^2 before the canonical step), c >= n^2, all-ones words."""
    N = _native()
    crt, _, key = ctxs[nb]
    W = crt.ct_words
    top = (1 << (32 * W)) - 1
    cs = [0, 1, 2, key.p, key.q, 3 * key.p, key.p * key.q, key.psquare, key.qsquare, key.psquare * 5 + key.q,
          key.nsquare - 1, key.nsquare, key.nsquare + 12345, top, top - 1, (key.n + 1) % key.nsquare,
          pow(key.n + 1, 5, key.nsquare)]
    rng = np.random.default_rng(nb + 1)
    cs += [int.from_bytes(rng.bytes(4 * W), "little") for _ in range(40)]
    ct = N.ints_to_words(cs, W)
    ex = np.array([(i % 5) - 1 for i in range(len(cs))], dtype=np.int32)
    raw = N.words_to_ints(_dboth(crt, ct, ex)[3])
    for i, c in enumerate(cs):
        assert raw[i] == O.raw_decrypt(c, key), f"element {i} (c = {c:#x})"


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 5, 1000])
def test_rows_decrypt_roundtrip(ctxs, nb, count):
    N = _native()
    crt, _, _ = ctxs[nb]
    rng = np.random.default_rng(count)
    x = (rng.standard_normal(count) * 10.0 ** rng.integers(-30, 30, count)).astype(np.float32)
    x[::7] = 0.0
    ct, ex, _ = crt.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=11)
    val = _dboth(crt, ct, ex)[0]
    assert np.array_equal(val, x.astype(np.float64))


# ---------------------------------------------------------------- public-key encryption on rows (k_pe_w)
def _pboth(pub, *args, **kw):
    """(rows, chain): a public-key-only party's call on k_pe_w and on k_pe_* (2048) / k_encrypt (1024)."""
    pub.set_stage_timing(True)
    try:
        a = pub.encrypt(*args, **kw)
        ka = len(pub.stage_times())
        old = pub.rows_max
        pub.set_rows_max(0)
        try:
            b = pub.encrypt(*args, **kw)
        finally:
            pub.set_rows_max(old)
    finally:
        pub.set_stage_timing(False)
    assert ka == 1, "one k_pe_w launch"
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    return a


@pytest.mark.parametrize("nb", [1024, 2048])
@pytest.mark.parametrize("count", [1, 5, 17, 1000])
def test_rows_public_rng_matches_chain_and_oracle(ctxs, nb, count):
    N = _native()
    _, pub, key = ctxs[nb]
    x = (np.random.default_rng(31 + count).standard_normal(count) * 10.0 ** np.random.default_rng(count).integers(-20, 20, count)).astype(np.float32)
    x[::6] = 0.0
    rk = bytes(range(9, 41))
    base = (1 << 32) + 5
    ct, ex, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    got = N.words_to_ints(ct)
    rbytes = ((nb + 64 + 31) // 32) * 4
    for i in sorted({0, count // 2, count - 1}):
        c, e = O.encrypt_value(x[i], key, O.device_r(rk, base + i, rbytes))
        assert got[i] == c and int(ex[i]) == e, f"element {i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_public_golden_and_edge_obfuscators(golden, ctxs, nb):
    """The reference goldens (explicit r), then r = 0, 1, 2, n - 1, n, n + 1, 5 p, n^2 - 1 and the all-ones word vector."""
    N = _native()
    _, pub, key = ctxs[nb]
    recs = golden["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    ct, ex, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_GIVEN, r=[int(r["r"], 16) for r in recs])
    got = N.words_to_ints(ct)
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(ex[i])) == (rec["c"], rec["e"]), f"element {i}"
    k = key
    rs = [0, 1, 2, k.n - 1, k.n, k.n + 1, 5 * k.p, k.nsquare - 1, (1 << (32 * pub.ct_words)) - 1]
    x = np.array([0.0, 1.0, -1.0, 3.5, -2.25, 1e-30, -1e30, 7.0, -0.0], dtype=np.float32)
    ct, _, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, r in enumerate(rs):
        assert got[i] == O.encrypt_value(x[i], k, r)[0], f"r #{i}"


@pytest.mark.parametrize("nb", [1024, 2048])
def test_rows_public_dtypes_and_scalar_r(ctxs, nb):
    N = _native()
    crt, pub, key = ctxs[nb]
    r = 0x1234567890ABCDEF1234567 % key.n
    for x in (np.array([0.0, -0.0, 1.5, -2.25, 3e-30, -7e20], dtype=np.float64),
              np.array([0, 1, -1, 2 ** 40, -(2 ** 50), 123456789], dtype=np.int64)):
        a = _pboth(pub, x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        b = crt.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r_scalar=r)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


# ---------------------------------------------------------------- 4096-bit keys on rows (k_crt_w<74, 148>, k_dec_w<74, 148>)
@pytest.fixture(scope="module")
def ctx4096(golden):
    N = _native()
    key = _key(golden, 4096)
    c = N.Context(key.n, 0, key.p, key.q)
    c.set_fixed_base(False)
    return c, key


def _counts(ctx, fn):
    ctx.set_stage_timing(True)
    try:
        r = fn()
        return r, len(ctx.stage_times())
    finally:
        ctx.set_stage_timing(False)


def _both4096(ctx, call):
    a, ka = _counts(ctx, call)
    old = ctx.rows_max
    ctx.set_rows_max(0)
    try:
        b, kb = _counts(ctx, call)
    finally:
        ctx.set_rows_max(old)
    return a, b, ka, kb


def test_rows_4096_encrypt_golden_and_rng(golden, ctx4096):
    """Against the reference goldens (explicit r) and, on the device stream, against the group engine's k_encrypt<8>
    and the oracle."""
    N = _native()
    ctx, key = ctx4096
    recs = golden["encrypt"]["4096"]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    a, b, ka, kb = _both4096(ctx, lambda: ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs))
    assert (ka, kb) == (2, 1), "k_crt_w + k_crt_fin against k_encrypt<8>"
    got = N.words_to_ints(a[0])
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(a[1][i])) == (rec["c"], rec["e"]), f"element {i}"
    assert np.array_equal(a[0], b[0])
    x = np.random.default_rng(4096).standard_normal(37).astype(np.float32)
    rk = bytes(range(5, 37))
    a, b, _, _ = _both4096(ctx, lambda: ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=99))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    got = N.words_to_ints(a[0])
    rbytes = ((4096 + 64 + 31) // 32) * 4
    for i in (0, 18, 36):
        assert got[i] == O.encrypt_value(x[i], key, O.device_r(rk, 99 + i, rbytes))[0], f"element {i}"


def test_rows_4096_edge_obfuscators(ctx4096):
    N = _native()
    ctx, key = ctx4096
    k = key
    rs = [1, 2, k.n - 1, k.n, k.n + 1, 5 * k.p, 3 * k.q, k.nsquare - 1, (1 << (32 * ctx.ct_words)) - 1]
    x = np.linspace(-3, 3, len(rs)).astype(np.float32)
    a, b, _, _ = _both4096(ctx, lambda: ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs))
    assert np.array_equal(a[0], b[0])
    got = N.words_to_ints(a[0])
    for i, r in enumerate(rs):
        assert got[i] == O.encrypt_value(x[i], k, r)[0], f"r #{i}"


def test_rows_4096_decrypt_edges_and_roundtrip(ctx4096):
    """k_dec_w<74, 148> + k_dec4_L + k_dec4_fin against the split-pair chain (k_dec4_pre/pow) and the oracle: c = 0,
    multiples of p, q, p^2, q^2, c >= n^2, all-ones words, random words, and a round trip."""
    N = _native()
    ctx, key = ctx4096
    W = ctx.ct_words
    top = (1 << (32 * W)) - 1
    cs = [0, 1, 2, key.p, key.q, 3 * key.p, key.p * key.q, key.psquare, key.qsquare, key.nsquare - 1, key.nsquare,
          top, (key.n + 1) % key.nsquare, pow(key.n + 1, 5, key.nsquare)]
    rng = np.random.default_rng(4097)
    cs += [int.from_bytes(rng.bytes(4 * W), "little") for _ in range(10)]
    ct = N.ints_to_words(cs, W)
    ex = np.array([(i % 5) - 1 for i in range(len(cs))], dtype=np.int32)
    a, b, ka, kb = _both4096(ctx, lambda: ctx.decrypt(ct, ex, want_raw=True))
    assert (ka, kb) == (2, 3), "k_dec_w + (k_dec4_L, k_dec4_fin) against k_dec4_pre/pow/L + fin"
    for u, v in zip(a, b):
        assert np.array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
    raw = N.words_to_ints(a[3])
    for i, c in enumerate(cs):
        assert raw[i] == O.raw_decrypt(c, key), f"element {i}"
    x = (rng.standard_normal(300) * 1e3).astype(np.float32)
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes(32), index_base=3)
    (val, _, _, _), _, _, _ = _both4096(ctx, lambda: ctx.decrypt(ct, ex))
    assert np.array_equal(val, x.astype(np.float64))


def test_rows_largest_call_all_kernels(ctxs):
    """rows_max elements (the largest call the rows take, 1024 of them per wave-row group of the grid) at nb = 1024:
    holder encryption, decryption and public encryption against the kernels they stand in for."""
    N = _native()
    crt, pub, _ = ctxs[1024]
    n = crt.rows_max
    x = (np.random.default_rng(n).standard_normal(n) * 100).astype(np.float32)
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(11, 43)), index_base=(1 << 40) - 7)
    a, b = _both(crt, x, **kw)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    val = _dboth(crt, a[0], a[1])[0]
    assert np.array_equal(val, x.astype(np.float64))
    _pboth(pub, x, **kw)


def test_rows_public_4096(golden):
    """k_pe_w<296> (the product loop rolled in groups of 19 steps) against k_encrypt<8>, the reference goldens and the
    oracle: explicit r, edge obfuscators and the device stream."""
    N = _native()
    key = _key(golden, 4096)
    pub = N.Context(key.n, 0)
    recs = golden["encrypt"]["4096"]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    ct, ex, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_GIVEN, r=[int(r["r"], 16) for r in recs])
    got = N.words_to_ints(ct)
    for i, rec in enumerate(recs):
        assert (hex(got[i]), int(ex[i])) == (rec["c"], rec["e"]), f"element {i}"
    k = key
    rs = [0, 1, k.n - 1, k.n, 5 * k.p, k.nsquare - 1, (1 << (32 * pub.ct_words)) - 1]
    x = np.array([0.0, 1.0, -1.0, 3.5, -2.25, 1e-30, -1e30], dtype=np.float32)
    ct, _, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, r in enumerate(rs):
        assert got[i] == O.encrypt_value(x[i], k, r)[0], f"r #{i}"
    x = np.random.default_rng(296).standard_normal(9).astype(np.float32)
    rk = bytes(range(2, 34))
    ct, ex, _ = _pboth(pub, x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=5)
    got = N.words_to_ints(ct)
    rbytes = ((4096 + 64 + 31) // 32) * 4
    for i in (0, 4, 8):
        assert got[i] == O.encrypt_value(x[i], key, O.device_r(rk, 5 + i, rbytes))[0], f"element {i}"
