"""GPU parity of the host-buffer entry points (pai_encrypt / pai_add / pai_decrypt): the operands cross
PCIe in chunks (HOST_CHUNK_MIN = 2^17 elements) that overlap the kernels. Chunking must not change a
single bit: ciphertexts at and around the chunk seams equal the CPU restatement (oracle/paillier_oracle.py,
keyed by the global element index), the k-way sums equal the oracle's add_k, decryption round-trips."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

CHUNK_MIN = 1 << 17


def _native():
    from flex.crypto.paillier import _native
    return _native


@pytest.fixture(scope="module")
def ctx1024(golden):
    N = _native()
    k = golden["keys"]["1024"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    return N.Context(key.n, 0, key.p, key.q), key


def _seams(n):
    nch = max(1, min(16, n // CHUNK_MIN))
    ch = -(-n // nch)
    idx = {0, n - 1}
    for i in range(1, nch):
        idx.update({i * ch - 1, i * ch})
    return sorted(i for i in idx if 0 <= i < n), nch


@pytest.mark.parametrize("fixed_base", [True, False])
def test_host_encrypt_chunked_bit_exact(ctx1024, fixed_base):
    N = _native()
    ctx, key = ctx1024
    n = 3 * CHUNK_MIN + 12345                      # 3 chunks, ragged
    x = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    rk = bytes(range(100, 132))
    ctx.set_fixed_base(fixed_base)
    try:
        ct, ex, st = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=1000)
        params = ctx.fixed_base_info() if fixed_base else None
    finally:
        ctx.set_fixed_base(True)
    idx, nch = _seams(n)
    assert nch == 3
    got = N.words_to_ints(ct[idx])
    rbytes = ((1024 + 64 + 31) // 32) * 4
    for j, i in enumerate(idx):
        if fixed_base:
            want = O.fb_encrypt_value(x[i], key, rk, 1000 + i, params)
        else:
            want = O.encrypt_value(x[i], key, O.device_r(rk, 1000 + i, rbytes) % key.n)
        assert (got[j], int(ex[i])) == want, f"element {i}"
    val, _, st2, _ = ctx.decrypt(ct, ex)
    assert np.array_equal(val, x.astype(np.float64)) and int((st2 > 1).sum()) == 0


def test_host_add_chunked_matches_oracle(ctx1024):
    N = _native()
    ctx, key = ctx1024
    n = 2 * CHUNK_MIN + 777
    xs = [np.random.default_rng(10 + j).standard_normal(n) * 10 ** j for j in range(3)]   # mixed exponents
    enc = [ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=bytes([j]) * 32) for j, x in enumerate(xs)]
    cts, exps = [e[0] for e in enc], [e[1] for e in enc]
    s_ct, s_ex = ctx.add(cts, exps)
    idx, nch = _seams(n)
    assert nch == 2
    got = N.words_to_ints(s_ct[idx])
    for j, i in enumerate(idx):
        ops = N.words_to_ints(np.stack([c[i] for c in cts]))
        assert (got[j], int(s_ex[i])) == O.add_k(ops, [int(e[i]) for e in exps], key), f"element {i}"
    val, _, _, _ = ctx.decrypt(s_ct, s_ex)
    want = xs[0] + xs[1] + xs[2]
    assert np.allclose(val, want, rtol=1e-12, atol=1e-9)
