"""One context shared by several threads (VERDICT r3 "lock the context"): every
entry point holds the context's mutex and a *_dev call's stream waits for the device work of the
context's previous call (flexpai.hip CtxLock). Four threads encrypting, adding and decrypting under one
key -- host-buffer entry points, and *_dev entry points each on its own HIP stream -- give outputs
bit-identical to the same calls run serially, to the reference's golden ciphertexts (explicit r) and to
the inputs after decryption. The reference never shares this state: it pickles the key into pool
processes (flex/crypto/paillier/encryptor.py:89-96, decryptor.py:106-111)."""
import hashlib
import threading

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

NTHREADS = 4


def _key(golden, nb):
    k = golden["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def _run_threads(fn, n=NTHREADS):
    out, errs = [None] * n, []
    barrier = threading.Barrier(n)

    def body(t):
        try:
            barrier.wait()
            out[t] = fn(t)
        except BaseException as e:   # noqa: BLE001 - re-raised in the main thread
            errs.append(e)

    th = [threading.Thread(target=body, args=(t,)) for t in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th), "a thread did not finish"
    if errs:
        raise errs[0]
    return out


@pytest.fixture(scope="module")
def shared(golden):
    from flex.crypto.paillier import _native as N
    key = _key(golden, 2048)
    ctx = N.Context(key.n, 0, key.p, key.q)
    return N, ctx, key


def _work(N, ctx, t, n=40_000):
    """Encrypt (device RNG: the fixed-base sampler), 3-way add, decrypt: one thread's share."""
    rng = np.random.default_rng(100 + t)
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(3)]
    key = hashlib.sha256(b"threads-%d" % t).digest()
    cts = [ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=key, index_base=j * n) for j, x in enumerate(xs)]
    s, se = ctx.add([c for c, _, _ in cts], [e for _, e, _ in cts])
    val, _, st, _ = ctx.decrypt(s, se)
    return [c.copy() for c, _, _ in cts], s, se, val, st, xs


def test_threads_share_one_context_host_entry_points(shared):
    N, ctx, _ = shared
    ctx.prepare_fixed_base()
    serial = [_work(N, ctx, t) for t in range(NTHREADS)]
    for _ in range(2):
        conc = _run_threads(lambda t: _work(N, ctx, t))
        for t in range(NTHREADS):
            cs, s, se, val, st, xs = conc[t]
            cs0, s0, se0, val0, _, _ = serial[t]
            for a, b in zip(cs, cs0):
                assert np.array_equal(a, b), f"thread {t}: ciphertexts differ from the serial run"
            assert np.array_equal(s, s0) and np.array_equal(se, se0), f"thread {t}: sums differ"
            assert np.array_equal(val, val0) and np.all(st == 0)
            want = xs[0].astype(np.float64) + xs[1].astype(np.float64) + xs[2].astype(np.float64)
            assert np.max(np.abs(val - want)) < 1e-5


def test_threads_explicit_r_match_reference_goldens(golden, shared):
    N, ctx, key = shared
    recs = golden["encrypt"]["2048"]
    x = np.array([r["bits"] for r in recs], dtype=np.uint32).view(np.float32)
    rs = [int(r["r"], 16) for r in recs]
    want = [(r["c"], r["e"]) for r in recs]

    def fn(t):
        res = []
        for _ in range(5):
            ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_GIVEN, r=rs)
            res.append([(hex(c), int(e)) for c, e in zip(N.words_to_ints(ct), ex)])
            val, _, st2, _ = ctx.decrypt(ct, ex)
            assert [float(v).hex() for v in val] == [r["dec"] for r in recs]
        return res

    for res in _run_threads(fn):
        for r in res:
            assert r == want


def test_threads_dev_entry_points_on_own_streams(shared):
    """Each thread launches on its own torch stream into its own buffers; the context's scratch and work
    buffers are shared, so without the cross-stream ordering the kernels of two calls would overlap on them."""
    import torch
    N, ctx, _ = shared
    lib = N.load_library()
    dev = torch.device("cuda", 0)
    n, W = 200_000, ctx.ct_words
    xs = [np.random.default_rng(7 + t).standard_normal(n).astype(np.float32) for t in range(NTHREADS)]
    keys = [hashlib.sha256(b"dev-threads-%d" % t).digest() for t in range(NTHREADS)]

    def fn(t, stream_per_thread=True):
        s = torch.cuda.Stream(dev) if stream_per_thread else torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            dx = torch.from_numpy(xs[t]).to(dev, non_blocking=False)
            ct = torch.empty((n, W), dtype=torch.int32, device=dev)
            ex = torch.empty(n, dtype=torch.int32, device=dev)
            st = torch.empty(n, dtype=torch.int32, device=dev)
            val = torch.empty(n, dtype=torch.float64, device=dev)
            dst = torch.empty(n, dtype=torch.int32, device=dev)
        s.synchronize()
        outs = []
        for rep in range(3):
            rc = lib.pai_encrypt_dev(ctx.handle, N.PAI_F32, dx.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0,
                                     keys[t], rep * n, ct.data_ptr(), ex.data_ptr(), st.data_ptr(), s.cuda_stream)
            assert rc == 0, lib.pai_last_error().decode()
            rc = lib.pai_decrypt_dev(ctx.handle, ct.data_ptr(), ex.data_ptr(), n, val.data_ptr(), None,
                                     dst.data_ptr(), None, s.cuda_stream)
            assert rc == 0, lib.pai_last_error().decode()
            s.synchronize()
            outs.append((ct.cpu().numpy().view(np.uint32).copy(), val.cpu().numpy().copy(), dst.cpu().numpy().copy()))
        return outs

    serial = [fn(t, stream_per_thread=False) for t in range(NTHREADS)]
    conc = _run_threads(fn)
    for t in range(NTHREADS):
        for rep in range(3):
            c0, v0, s0 = serial[t][rep]
            c1, v1, s1 = conc[t][rep]
            assert np.array_equal(c0, c1), f"thread {t} rep {rep}: ciphertexts differ"
            assert np.all(s1 == 0) and np.array_equal(v1, xs[t].astype(np.float64)), f"thread {t} rep {rep}"
