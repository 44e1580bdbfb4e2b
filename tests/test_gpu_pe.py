"""GPU parity of the public-key encryption on split pairs (kernels_pe.hpp: k_pe_pre / k_pe_pow / k_pe_fin, the
path of every party that holds only the public key, 2048-bit n) against the reference golden vectors
(explicit r: encryptor.py:48-69 with random_value), the CPU oracle (device ChaCha20 obfuscators) and the
group-engine kernel it replaces (k_encrypt, $FLEXPAI_PAIR=0 in the test build): bit-identical ciphertexts, exponents, statuses.

Every case runs twice: on the general chain (k_pe_pow) and on the factored one (k_pe_pow_f: B-free multipliers, a batch
inversion of the bases, the closing Horner sum; round 5), the latter forced at small sizes by $FLEXPAI_PEF_MIN=0. The
edge obfuscators include non-units (r = 0, n, 5p): the batch inversion then finds no inverse and the chunk falls back
to the general chain -- same ciphertexts."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def key2048(golden):
    k = golden["keys"]["2048"]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


@pytest.fixture(params=["general", "factored"])
def chain(request, monkeypatch):
    monkeypatch.setenv("FLEXPAI_PEF_MIN", "0" if request.param == "factored" else str(1 << 40))
    return request.param


def _pub(monkeypatch, key, pair):
    from flex.crypto.paillier import _native as N
    monkeypatch.setenv("FLEXPAI_PAIR", "1" if pair else "0")
    ctx = N.Context(key.n, 0, lib=None if pair else N.load_library(N.XCHECK_LIB_PATH))
    assert bool(ctx.pair_paths & 4) == pair
    ctx.set_rows_max(0)   # the chains under test, not k_pe_w (tests/test_gpu_crt_rows.py)
    return ctx


def test_pe_given_r_matches_reference_goldens(golden, key2048, monkeypatch, chain):
    N = _native()
    ctx = _pub(monkeypatch, key2048, True)
    recs = golden["encrypt"]["2048"]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    got = N.words_to_ints(ct)
    for i, rec in enumerate(recs):
        assert st[i] == 0
        assert (hex(got[i]), int(ex[i])) == (rec["c"], rec["e"]), f"element {i}"


@pytest.mark.parametrize("n", [1, 127, 129, 300])
def test_pe_matches_k_encrypt_and_oracle(key2048, monkeypatch, n, chain):
    N = _native()
    a = _pub(monkeypatch, key2048, True)
    b = _pub(monkeypatch, key2048, False)
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32)
    x[::7] = 0.0
    x[1::9] = -x[1::9]
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(32)), index_base=77)
    ca, ea, sa = a.encrypt(x, **kw)
    cb, eb, sb = b.encrypt(x, **kw)
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb) and np.array_equal(sa, sb)
    got = N.words_to_ints(ca[: min(n, 6)])
    rb = ((2048 + 64 + 31) // 32) * 4       # bytes of the ChaCha20 stream k_encrypt and k_pe_pre draw
    for i in range(min(n, 6)):
        c, e = O.encrypt_value(x[i], key2048, O.device_r(bytes(range(32)), 77 + i, rb))
        assert (got[i], int(ea[i])) == (c, e), f"element {i}"


def test_pe_edge_obfuscators(key2048, monkeypatch, chain):
    """r = 0, 1, n - 1, n, n + 1, a multiple of p, r >= n^2 (explicit, like random_value)."""
    N = _native()
    a = _pub(monkeypatch, key2048, True)
    b = _pub(monkeypatch, key2048, False)
    k = key2048
    rs = [0, 1, 2, k.n - 1, k.n, k.n + 1, 5 * k.p, k.nsquare - 1, (1 << (32 * a.ct_words)) - 1]
    x = np.array([0.0, 1.0, -1.0, 3.5, -2.25, 1e-30, -1e30, 7.0, -0.0], dtype=np.float32)
    ca, ea, _ = a.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    cb, eb, _ = b.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb)
    got = N.words_to_ints(ca)
    for i, r in enumerate(rs):
        assert got[i] == O.encrypt_value(x[i], k, r)[0], f"r #{i}"


def test_pe_factored_chain_above_threshold_matches_general(key2048, monkeypatch):
    """At the default threshold a 20 000-element call runs the factored chain; the test build's general chain
    ($FLEXPAI_PEF=0) on the same device RNG gives the same ciphertexts, and both decrypt to the input."""
    N = _native()
    monkeypatch.delenv("FLEXPAI_PEF_MIN", raising=False)
    a = _pub(monkeypatch, key2048, True)
    monkeypatch.setenv("FLEXPAI_PEF", "0")
    b = N.Context(key2048.n, 0, lib=N.load_library(N.XCHECK_LIB_PATH))
    monkeypatch.delenv("FLEXPAI_PEF")
    a.set_public_fixed_base(False)
    b.set_public_fixed_base(False)
    n = 20000
    x = (np.random.default_rng(5).standard_normal(n) * 1000).astype(np.float32)
    kw = dict(obf_mode=N.PAI_OBF_RNG, rng_key=bytes(range(3, 35)), index_base=2 ** 34)
    ca, ea, _ = a.encrypt(x, **kw)
    cb, eb, _ = b.encrypt(x, **kw)
    assert np.array_equal(ca, cb) and np.array_equal(ea, eb)
    got = N.words_to_ints(ca[[0, n // 2, n - 1]])
    rb = ((2048 + 64 + 31) // 32) * 4
    for j, i in enumerate([0, n // 2, n - 1]):
        assert got[j] == O.encrypt_value(x[i], key2048, O.device_r(bytes(range(3, 35)), 2 ** 34 + i, rb))[0]
    d = N.Context(key2048.n, 0, key2048.p, key2048.q)
    val, _, _, _ = d.decrypt(ca, ea)
    assert np.array_equal(val, x.astype(np.float64))


def test_pe_dev_call_is_asynchronous_on_a_side_stream(key2048, monkeypatch):
    """pai_encrypt_dev on the factored public-key chain (>= 16 384 elements) queues its batch inversion's host
    step as a host function instead of synchronising the stream. On a non-default torch stream that is still busy with
    ~0.5 s of earlier work, the call returns at once; its ciphertexts equal the general chain's."""
    import time
    import torch
    N = _native()
    monkeypatch.delenv("FLEXPAI_PEF_MIN", raising=False)
    a = _pub(monkeypatch, key2048, True)
    a.set_public_fixed_base(False)
    lib = N.load_library()
    n = 20000
    dev = torch.device("cuda", 0)
    x = torch.from_numpy((np.random.default_rng(9).standard_normal(n) * 100).astype(np.float32)).to(dev)
    W = a.ct_words
    ct = torch.empty((n, W), dtype=torch.int32, device=dev)
    ex = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    key = bytes(range(7, 39))
    s = torch.cuda.Stream(dev)
    # calibrate torch's spin kernel, then keep the side stream busy for ~0.5 s
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        torch.cuda._sleep(10 ** 7)
        e1.record(s)
    torch.cuda.synchronize()
    cyc_per_ms = 10 ** 7 / max(e0.elapsed_time(e1), 1e-3)
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(500 * cyc_per_ms))
    t0 = time.perf_counter()
    rc = lib.pai_encrypt_dev(a.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, key, 11,
                             ct.data_ptr(), ex.data_ptr(), st.data_ptr(), s.cuda_stream)
    t_call = time.perf_counter() - t0
    assert rc == 0, lib.pai_last_error().decode()
    busy = not s.query()
    torch.cuda.synchronize()
    assert busy and t_call < 0.25, f"the call blocked the host for {t_call * 1e3:.0f} ms"
    monkeypatch.setenv("FLEXPAI_PEF_MIN", str(1 << 40))       # the general chain on the same inputs
    cg, eg, _ = a.encrypt(x.cpu().numpy(), obf_mode=N.PAI_OBF_RNG, rng_key=key, index_base=11)
    assert np.array_equal(ct.cpu().numpy().view(np.uint32), cg) and np.array_equal(ex.cpu().numpy(), eg)
