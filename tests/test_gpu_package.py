"""The drop-in package on the GPU: the reference's own test_paillier.py cases
(test/crypto/paillier/test_paillier.py:31-113, one-sided almost_equal of test/utils.py:21-31 kept
AND tightened to exact equality where the math is exact), the HE_SA_FT encrypt -> coordinator
add -> decrypt flow (he_sa_ft/train.py:37-71), pickle interop and error behaviour."""
import pickle
import random

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def almost_equal(x, y, epsilon=1e-4):   # test/utils.py:21-31 (one-sided, as in the reference)
    if isinstance(x, (int, float)) and isinstance(y, (int, float)):
        return (x - y) < epsilon
    if isinstance(x, np.ndarray) and isinstance(y, np.ndarray) and x.shape == y.shape:
        return np.all(x - y < epsilon)
    return False


@pytest.fixture(scope="module")
def pe_pd():
    from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
    return generate_paillier_encryptor_decryptor()


def test_generator():
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk1, _ = generate_paillier_keypair(1024, seed=1)
    pk2, _ = generate_paillier_keypair(1024, seed=1)
    pk3, _ = generate_paillier_keypair(1024, seed=2)
    assert pk1.n.bit_length() == pk2.n.bit_length()
    assert pk1 == pk2 and pk1 != pk3


def test_encrypt_decrypt(pe_pd):
    pe, pd = pe_pd
    p1 = random.random()
    assert almost_equal(p1, pd.decrypt(pe.encrypt(p1)))
    key = O.Key(pe.pub_key.n)
    m, e = O.encode(p1, key.n, key.max_int)           # float64 scalars lose low bits (16^e scaling)
    assert pd.decrypt(pe.encrypt(p1)) == O.decode(m, e, key.n, key.max_int)
    a = np.random.random(100).astype(np.float32)
    enc = pe.encrypt(a)
    assert isinstance(enc, np.ndarray) and enc.shape == a.shape
    out = pd.decrypt(enc)
    assert almost_equal(a, out) and np.array_equal(out, a.astype(np.float64))
    b = np.random.random((128, 4)).astype(np.float32)
    out = pd.decrypt(pe.encrypt(b))
    assert out.shape == (128, 4) and np.array_equal(out, b.astype(np.float64))


def test_add(pe_pd):
    pe, pd = pe_pd
    x1, x2 = random.random(), random.random()
    y1, y2 = np.random.random(100).astype(np.float32), np.random.random(100).astype(np.float32)
    z1, z2 = np.random.random((128, 4)).astype(np.float32), np.random.random((128, 4)).astype(np.float32)
    ex1, ex2, ey1, ey2, ez1, ez2 = (pe.encrypt(v) for v in (x1, x2, y1, y2, z1, z2))
    assert almost_equal(pd.decrypt(ex1 + ex2), x1 + x2)
    assert almost_equal(pd.decrypt(ey1 + ey2), y1 + y2)
    assert almost_equal(pd.decrypt(ez1 + ez2), z1 + z2)
    assert almost_equal(pd.decrypt(ex1 + x2), x1 + x2)
    assert almost_equal(pd.decrypt(ey1 + y2), y1 + y2)
    assert almost_equal(pd.decrypt(ez1 + z2), z1 + z2)
    # exact: the float32 sums are exact in float64
    assert np.array_equal(pd.decrypt(ey1 + ey2), y1.astype(np.float64) + y2.astype(np.float64))


def test_mul(pe_pd):
    pe, pd = pe_pd
    x1, x2 = random.random(), random.random()
    y1, y2 = np.random.random(100).astype(np.float32), np.random.random(100).astype(np.float32)
    ex1, ey1 = pe.encrypt(x1), pe.encrypt(y1)
    assert almost_equal(pd.decrypt(ex1 * x2), x1 * x2)
    assert almost_equal(pd.decrypt(ey1 * x1), y1 * x1)
    assert almost_equal(pd.decrypt(ey1 * y2), y1 * y2)


def test_add_mul_numpy_parallel(pe_pd):
    from flex.crypto.paillier import parallel_ops
    pe, pd = pe_pd
    x = np.random.random(100).astype(np.float32)
    y = np.random.random(100).astype(np.float32)
    en_x, en_y = pe.encrypt(x), pe.encrypt(y)
    assert almost_equal(x + y, pd.decrypt(parallel_ops.add(en_x, y)))
    assert almost_equal(x + y, pd.decrypt(parallel_ops.add(en_x, en_y)))
    assert almost_equal(x * y, pd.decrypt(parallel_ops.mul(en_x, y)))


def test_he_sa_ft_flow_bit_exact_against_oracle(golden):
    """Two parties encrypt theta with the same DH-seeded key; the coordinator sums with `+`
    (onetime_pad/iterative_add.py:23-33); parties decrypt and average. Ciphertexts of the sum are
    compared bit-exactly with the oracle using the obfuscators the device drew."""
    from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
    pe, pd = generate_paillier_encryptor_decryptor(1024, seed=1234)
    theta = [np.random.default_rng(k).standard_normal((16, 3)).astype(np.float32) for k in range(2)]
    enc = [pe.encrypt(t) for t in theta]
    blob = pickle.dumps(enc)                       # ionic_bond ships pickles
    enc = pickle.loads(blob)
    s = enc[0]
    for e in enc[1:]:
        s = s + e
    avg = pd.decrypt(s) / 2.0
    assert np.array_equal(avg, (theta[0].astype(np.float64) + theta[1].astype(np.float64)) / 2.0)
    key = O.Key(pe.pub_key.n, pd.priv_key.p, pd.priv_key.q)
    for i in range(s.size):
        cs = [e.reshape(-1)[i].ciphertext(False) for e in enc]
        es = [e.reshape(-1)[i].exponent for e in enc]
        C, E = O.add_k(cs, es, key)
        assert s.reshape(-1)[i].ciphertext(False) == C and s.reshape(-1)[i].exponent == E


def test_random_value_semantics(golden):
    from flex.crypto.paillier.api import generate_paillier_decryptor
    from flex.crypto.paillier.encryptor import PaillierEncryptor
    from flex.crypto.paillier.keypair import PaillierPublicKey
    k = golden["keys"]["1024"]
    n = int(k["n"], 16)
    pe = PaillierEncryptor(PaillierPublicKey(n))
    rec = golden["random_value_zero"]["1024"]
    x = O.f32_from_bits(rec["bits"])
    e = pe.encrypt(np.array([x]), random_value=0)[0]
    assert hex(e.ciphertext(False)) == rec["c"] and not e._is_obfuscated()
    recs = golden["encrypt"]["1024"][:5]
    for r in recs:
        xv = O.f32_from_bits(r["bits"])
        e = pe.encrypt(np.array([xv], dtype=np.float32), random_value=int(r["r"], 16))[0]
        assert hex(e.ciphertext(False)) == r["c"] and e.exponent == r["e"]
        s = pe.encrypt(xv, random_value=int(r["r"], 16))     # scalar path
        assert hex(s.ciphertext(False)) == r["c"]
    pd = generate_paillier_decryptor(n, int(k["p"], 16), int(k["q"], 16))
    assert pd.decrypt(pe.encrypt(np.float32(2.5))) == 2.5


def test_int_arrays_and_precision(pe_pd):
    pe, pd = pe_pd
    ints = np.array([0, 1, -1, 7, -(2 ** 40), 123456789], dtype=np.int64)
    out = pd.decrypt(pe.encrypt(ints))
    assert out.dtype == np.int64 and list(out) == list(ints)
    x = np.array([0.123456, -1.5, 100.25, 3.0e9, -7.0e12], dtype=np.float64)
    key = O.Key(pe.pub_key.n)
    for prec in (1e-8, 0.5, 1e6):          # precision -> floor(log16(precision))
        out = pd.decrypt(pe.encrypt(x, precision=prec))
        want = [O.decode(*O.encode(np.float64(v), key.n, key.max_int, precision=prec), key.n, key.max_int)
                for v in x]
        assert [float(a) for a in out] == [float(b) for b in want], prec


def test_decrypt_errors(pe_pd, golden):
    from flex.crypto.paillier.api import generate_paillier_encryptor_decryptor
    pe, pd = pe_pd
    with pytest.raises(TypeError):
        pd.decrypt(np.array([1, 2], dtype=object))
    pe2, _ = generate_paillier_encryptor_decryptor(1024, seed=99)
    with pytest.raises(ValueError):
        pd.decrypt(pe2.encrypt(np.array([1.0], dtype=np.float32)))


def test_received_arrays_run_on_the_gpu(pe_pd, monkeypatch):
    """Arrays that arrive over the wire from flexpai senders that opted in to the bulk pickle
    (FLEXPAI_PICKLE_BULK=1; ion.py:150-178) unpickle as PaillierArray and the receiver's unchanged operators reach the device: the HE_SA_FT coordinator's `+`
    (he_sa_ft/train.py:66-69) -> pai_add, HE_LINEAR's `sum(...)` (he_linear_ft/train.py:64-65) ->
    pai_add_plain + pai_add, HE_OTP_LR's `(-1/bs) * enc.dot(features)` (he_otp_lr_ft1/train.py:158-160)
    -> pai_matmul + pai_mul. Bit-exact against the oracle's restatement of encrypted_number.py."""
    from flex.crypto.paillier import _runtime
    from flex.crypto.paillier.cipher_array import PaillierArray
    monkeypatch.setenv("FLEXPAI_PICKLE_BULK", "1")
    pe, pd = pe_pd
    key = O.Key(pe.pub_key.n, pd.priv_key.p, pd.priv_key.q)
    rng = np.random.default_rng(11)
    xs = [(rng.standard_normal(300) * (10.0 ** (k - 3))).astype(np.float32) for k in range(8)]
    recv = [pickle.loads(pickle.dumps(pe.encrypt(x))) for x in xs]
    assert all(type(r) is PaillierArray and r._valid_packed() is not None for r in recv)
    ctx = _runtime.context(pe.pub_key)
    c0 = dict(ctx.calls)
    s = recv[0]
    for r in recv[1:]:
        s = s + r
    assert ctx.calls["pai_add"] - c0.get("pai_add", 0) == 7
    for i in (0, 17, 299):
        C, E = O.add_k([r[i].ciphertext(False) for r in recv], [r[i].exponent for r in recv], key)
        assert (s[i].ciphertext(False), s[i].exponent) == (C, E)
    assert np.allclose(pd.decrypt(s), np.sum([x.astype(np.float64) for x in xs], axis=0), rtol=1e-12, atol=0)
    c1 = dict(ctx.calls)
    t = sum(recv)
    assert ctx.calls["pai_add_plain"] - c1.get("pai_add_plain", 0) == 1
    assert ctx.calls["pai_add"] - c1.get("pai_add", 0) == 7
    assert [(a.ciphertext(False), a.exponent) for a in t] == [(a.ciphertext(False), a.exponent) for a in s]
    v = pickle.loads(pickle.dumps(pe.encrypt(xs[3][:32])))
    feats = rng.standard_normal((32, 6))
    c2 = dict(ctx.calls)
    g = (-1 / 32) * v.dot(feats)
    assert ctx.calls["pai_matmul"] - c2.get("pai_matmul", 0) == 1
    assert ctx.calls["pai_mul"] - c2.get("pai_mul", 0) == 1
    for j in (0, 5):
        terms = [O.mul_scalar(v[i].ciphertext(False), v[i].exponent, float(feats[i, j]), key) for i in range(32)]
        C, E = O.add_k([a for a, _ in terms], [b for _, b in terms], key)
        C, E = O.mul_scalar(C, E, -1 / 32, key)
        assert (g[j].ciphertext(False), g[j].exponent) == (C, E)


def test_context_cache_is_bounded(monkeypatch):
    """contexts are held in a bounded LRU; a process cycling through keys does not keep
    every key's fixed-base tables resident."""
    from flex.crypto.paillier import _native, _runtime
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    monkeypatch.setenv("FLEXPAI_MAX_CONTEXTS", "2")
    monkeypatch.setenv("FLEXPAI_FB_WINDOW", "16")
    import gc
    gc.collect()
    free0, _ = _native.device_mem_info(0)
    for seed in range(21, 27):
        pk, sk = generate_paillier_keypair(1024, seed=seed)
        ctx = _runtime.context(pk, sk)
        ctx.prepare_fixed_base()                # ~0.5 GB of tables per 1024-bit key at W = 16
        assert ctx.fb_ready
        del ctx
        gc.collect()
    assert len(_runtime.cached_contexts()) <= 2
    free1, _ = _native.device_mem_info(0)
    assert free0 - free1 < 3 * 600 * 2 ** 20, (free0 - free1) / 2 ** 20


def test_encrypted_minus_encrypted_on_the_gpu(pe_pd):
    """`a - b` with both operands encrypted (encrypted_number.py:74-78, self + (other * -1)) runs as
    one pai_mul by -1 and one pai_add instead of numpy's per-object loop; bit-identical to the per-element
    operators (the reference's algorithm on the host) and decrypting to the differences. Also a plain received
    object ndarray on the left (PaillierArray.__rsub__) and a single PaillierEncryptedNumber on the right."""
    from flex.crypto.paillier import _runtime
    from flex.crypto.paillier.cipher_array import PaillierArray
    pe, pd = pe_pd
    rng = np.random.default_rng(21)
    xa = (rng.standard_normal((40, 3)) * 100).astype(np.float32)
    xb = rng.standard_normal((40, 3)).astype(np.float32)
    a, b = pe.encrypt(xa), pe.encrypt(xb)
    ctx = _runtime.context(pe.pub_key)
    c0 = dict(ctx.calls)
    d = a - b
    assert type(d) is PaillierArray
    assert ctx.calls["pai_mul"] - c0.get("pai_mul", 0) == 1 and ctx.calls["pai_add"] - c0.get("pai_add", 0) == 1
    fa, fb, fd = a.reshape(-1), b.reshape(-1), d.reshape(-1)
    for i in range(fa.size):
        want = fa[i] + (fb[i] * -1)                    # host per-element operators (the reference's code path)
        assert (fd[i].ciphertext(False), fd[i].exponent) == (want.ciphertext(False), want.exponent), i
    assert np.array_equal(pd.decrypt(d), xa.astype(np.float64) - xb.astype(np.float64))
    plain = np.asarray(a).view(np.ndarray).copy()      # an unpickled plain object ndarray minus a PaillierArray
    e = plain - b
    assert [(u.ciphertext(False), u.exponent) for u in e.reshape(-1)] == \
        [(u.ciphertext(False), u.exponent) for u in fd]
    s = fa[5]
    f = b - s                                          # array - single number
    for i in (0, 7, fb.size - 1):
        w1 = fb[i] + (s * -1)
        assert (f.reshape(-1)[i].ciphertext(False), f.reshape(-1)[i].exponent) == (w1.ciphertext(False), w1.exponent)
    assert np.array_equal(pd.decrypt(f), xb.astype(np.float64) - np.float64(xa.reshape(-1)[5]))
