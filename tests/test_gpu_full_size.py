"""GPU parity at BASELINE.json's full sizes (configs[1], configs[2]: 1 048 576 elements, nb = 2048; configs[3]:
16 777 216 elements as 8 shards; configs[4]: one rank's 524 288-element shard at nb = 4096),
through the C ABI, checked by size-independent properties plus a bit-exact oracle sample:

* decrypt(encrypt(x)) == x exactly for every element (fixed-base key-holder path, the bench's timed
  path), with every status OK; a sample of ciphertexts equals the oracle's restatement;
* one 8-way add of 8 encrypted 1M arrays: the decrypted sums equal the exact sums (checked against the
  float64 sums within one ulp, and bit-exactly against the oracle on a sample of ciphertexts)."""
import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu
N = 1 << 20


@pytest.fixture(scope="module")
def ctx2048(golden):
    from flex.crypto.paillier import _native
    k = golden["keys"]["2048"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    return _native.Context(key.n, 0, key.p, key.q), key


@pytest.mark.parametrize("window", [16, 22])
def test_full_size_roundtrip(ctx2048, window):
    """At the library default window and at the bench's timed one (W = 22, 2 x 88.3 GB of Shoup tables)."""
    from flex.crypto.paillier import _native as Nn
    ctx, key = ctx2048
    x = np.random.default_rng(0).standard_normal(N, dtype=np.float32)
    rk = bytes(range(200, 232))
    try:
        ctx.set_fb_window(window)
        ctx.prepare_fixed_base()
        assert ctx.fixed_base_info()[3] == window
        ct, ex, st = ctx.encrypt(x, obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=0)
        params = ctx.fixed_base_info()
    finally:
        ctx.set_fb_window(16)
    assert np.all(st == 0)
    val, _, dst, _ = ctx.decrypt(ct, ex)
    assert np.all(dst == 0) and np.array_equal(val, x.astype(np.float64))
    idx = [0, 1, N // 3, N - 1]
    got = Nn.words_to_ints(ct[idx])
    for j, i in enumerate(idx):
        assert (got[j], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, i, params)


def test_full_size_add8(ctx2048):
    from flex.crypto.paillier import _native as Nn
    ctx, key = ctx2048
    xs = [np.random.default_rng(k).standard_normal(N, dtype=np.float32) for k in range(8)]
    rk = bytes(range(32))
    cts, exs = [], []
    for k, x in enumerate(xs):
        ct, ex, _ = ctx.encrypt(x, obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=(k + 1) * N)
        cts.append(ct)
        exs.append(ex)
    s, es = ctx.add(cts, exs)
    val, _, st, _ = ctx.decrypt(s, es)
    assert np.all(st == 0)
    ref = np.sum([x.astype(np.float64) for x in xs], axis=0)
    assert np.all(np.abs(val - ref) <= np.spacing(np.abs(ref)))
    idx = [0, 12345, N - 1]
    got = Nn.words_to_ints(s[idx])
    for j, i in enumerate(idx):
        C, E = O.add_k([Nn.words_to_ints(c[i:i + 1])[0] for c in cts], [int(e[i]) for e in exs], key)
        assert (got[j], int(es[i])) == (C, E)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_encrypt_equals_single(ctx2048, world):
    """configs[3]'s contract on one GPU: the contiguous shards of `world` ranks (sharding.shard_bounds, each
    encrypting with index_base = its first global index, as bench.py does) reassemble into exactly the
    ciphertexts of one unsharded call -- ciphertexts do not depend on the GPU count."""
    from flex.crypto.paillier import _native as Nn
    from flex.crypto.paillier.sharding import shard_bounds
    ctx, _ = ctx2048
    total = 3 * 65536 + 17                                  # ragged: the last shard is shorter
    x = np.random.default_rng(3).standard_normal(total, dtype=np.float32)
    rk = bytes(range(50, 82))
    whole, wex, _ = ctx.encrypt(x, obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=0)
    parts, pex = [], []
    for r in range(world):
        lo, hi = shard_bounds(total, world, r)
        c, e, _ = ctx.encrypt(x[lo:hi], obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=lo)
        parts.append(c)
        pex.append(e)
    assert np.array_equal(np.concatenate(parts), whole) and np.array_equal(np.concatenate(pex), wex)


def test_full_size_4096_sample(golden):
    """configs[4]'s key (nb = 4096) on 262 144 elements of the fixed-base group path: exact round trip,
    oracle sample, and the chunk-independent ciphertexts of a split call."""
    from flex.crypto.paillier import _native as Nn
    k = golden["keys"]["4096"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = Nn.Context(key.n, 0, key.p, key.q)
    ctx.set_fb_window(16)
    n = 1 << 18
    x = np.random.default_rng(4).standard_normal(n, dtype=np.float32)
    rk = bytes(range(9, 41))
    ct, ex, st = ctx.encrypt(x, obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=7)
    assert np.all(st == 0)
    val, _, dst, _ = ctx.decrypt(ct, ex)
    assert np.all(dst == 0) and np.array_equal(val, x.astype(np.float64))
    params = ctx.fixed_base_info()
    idx = [0, n // 2, n - 1]
    got = Nn.words_to_ints(ct[idx])
    for j, i in enumerate(idx):
        assert (got[j], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, 7 + i, params)
    half, _, _ = ctx.encrypt(x[n // 2:], obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=7 + n // 2)
    assert np.array_equal(half, ct[n // 2:])


def _dev_encrypt(lib, Nn, ctx, dx, n, rk, base, ct, ex, st, stream):
    rc = lib.pai_encrypt_dev(ctx.handle, Nn.PAI_F32, dx, n, 0, 0, Nn.PAI_OBF_RNG, None, 0, 0, rk, base, ct, ex, st, stream)
    assert rc == 0, lib.pai_last_error().decode()


def test_config3_full_size_sharded(ctx2048):
    """configs[3] at its full size on one GPU: 16 777 216 elements (nb = 2048) at the bench's window W = 22,
    encrypted as the 8 contiguous shards of an 8-GPU run (index_base = the shard's first global index,
    sharding.shard_bounds) into one buffer -- the all-gather's output layout -- equal bit for bit to ONE
    unsharded call; the oracle's restatement of the sampler matches at every shard seam (first and last
    element of each shard); decryption reproduces all 16M inputs exactly with every status OK. Reference
    semantics: flex/crypto/paillier/encryptor.py:71-97 (element-wise, order independent), obfuscator.py:35-37."""
    import torch
    from flex.crypto.paillier import _native as Nn
    from flex.crypto.paillier.sharding import shard_bounds
    ctx, key = ctx2048
    lib = Nn.load_library()
    total, world, W = 16 << 20, 8, ctx.ct_words
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    x = np.random.default_rng(33).standard_normal(total, dtype=np.float32)
    rk = bytes(range(100, 132))
    try:
        ctx.set_fb_window(22)
        ctx.prepare_fixed_base()
        params = ctx.fixed_base_info()
        assert params[3] == 22
        dx = torch.from_numpy(x).to(dev)
        whole = torch.empty((total, W), dtype=torch.int32, device=dev)
        wex = torch.empty(total, dtype=torch.int32, device=dev)
        st = torch.empty(total, dtype=torch.int32, device=dev)
        _dev_encrypt(lib, Nn, ctx, dx.data_ptr(), total, rk, 0, whole.data_ptr(), wex.data_ptr(), st.data_ptr(), s)
        assert int(torch.count_nonzero(st).item()) == 0
        shards = torch.empty_like(whole)
        sex = torch.empty_like(wex)
        seams = []
        for r in range(world):
            lo, hi = shard_bounds(total, world, r)
            _dev_encrypt(lib, Nn, ctx, dx[lo:].data_ptr(), hi - lo, rk, lo, shards[lo:].data_ptr(), sex[lo:].data_ptr(),
                         st[lo:].data_ptr(), s)
            seams += [lo, hi - 1]
        assert torch.equal(shards, whole) and torch.equal(sex, wex), "sharded != unsharded"
        del shards, sex
        got = Nn.words_to_ints(whole[seams].cpu().numpy().view(np.uint32))
        gex = wex[seams].cpu().numpy()
        for j, i in enumerate(seams):
            assert (got[j], int(gex[j])) == O.fb_encrypt_value(x[i], key, rk, i, params), f"seam element {i}"
        val = torch.empty(total, dtype=torch.float64, device=dev)
        rc = lib.pai_decrypt_dev(ctx.handle, whole.data_ptr(), wex.data_ptr(), total, val.data_ptr(), None,
                                 st.data_ptr(), None, s)
        assert rc == 0, lib.pai_last_error().decode()
        # integer-valued inputs (this sample holds 0.0, -0.0 and 1.0) decode with exponent <= 0: PAI_EL_INT, value
        # still in val_out (fixedpoint_number.py decode); everything else PAI_EL_OK
        ints = torch.from_numpy(np.nonzero(x == np.round(x))[0]).to(dev)
        assert bool(torch.all(st[ints] <= Nn.EL_INT).item())
        st[ints] = 0
        assert int(torch.count_nonzero(st).item()) == 0
        assert torch.equal(val, dx.double()), "16M round trip"
    finally:
        torch.cuda.synchronize()
        ctx.set_fb_window(16)
        torch.cuda.empty_cache()


def test_config4_shard_full_size_4096(golden):
    """configs[4]'s per-rank shard at N = 8 (4M / 8 = 524 288 elements, nb = 4096) at the bench's window
    (asked 21: W = 20 with the Shoup rows beside the factored rows, k_sgs -- flexpai.hip fb_choose -- or 21 without):
    exact round trip, every status OK, the oracle's restatement of the sampler on a sample (first, seams, last)."""
    from flex.crypto.paillier import _native as Nn
    k = golden["keys"]["4096"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = Nn.Context(key.n, 0, key.p, key.q)
    try:
        ctx.set_fb_window(21)
        ctx.prepare_fixed_base()
        params = ctx.fixed_base_info()
        assert params[3] == (20 if ctx.split_sampler & 8 else 21)
        n = 1 << 19
        base = 3 * n                                       # rank 3's shard of the 4M vector
        x = np.random.default_rng(44).standard_normal(n, dtype=np.float32)
        rk = bytes(range(60, 92))
        ct, ex, st = ctx.encrypt(x, obf_mode=Nn.PAI_OBF_RNG, rng_key=rk, index_base=base)
        assert np.all(st == 0)
        val, _, dst, _ = ctx.decrypt(ct, ex)
        assert np.all(dst == 0) and np.array_equal(val, x.astype(np.float64))
        idx = [0, 1, n // 2 - 1, n // 2, n - 1]
        got = Nn.words_to_ints(ct[idx])
        for j, i in enumerate(idx):
            assert (got[j], int(ex[i])) == O.fb_encrypt_value(x[i], key, rk, base + i, params), f"element {i}"
    finally:
        ctx.close()
