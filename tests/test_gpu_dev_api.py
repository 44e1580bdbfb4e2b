"""Device-resident entry points (pai_*_dev on torch device buffers and the current stream) agree
bit-for-bit with the host-buffer entry points and the oracle: encrypt -> mul -> add_plain -> add ->
segment_add -> decrypt without leaving HBM."""
import hashlib

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu


def test_device_resident_chain(golden):
    import torch
    from flex.crypto.paillier import _native as N
    k = golden["keys"]["1024"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = N.Context(key.n, 0, key.p, key.q)
    lib = N.load_library()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    n, W = 300, ctx.ct_words
    rng = np.random.default_rng(8)
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n) * 10.0 ** rng.integers(-3, 3, n)
    sc = rng.standard_normal(n)
    rk = hashlib.sha256(b"dev-api").digest()

    def chk(rc):
        assert rc == 0, lib.pai_last_error().decode()

    dx = torch.from_numpy(x).to(dev)
    dy = torch.from_numpy(y).to(dev)
    dsc = torch.from_numpy(sc).to(dev)
    ct = torch.empty((n, W), dtype=torch.int32, device=dev)
    ex = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    chk(lib.pai_encrypt_dev(ctx.handle, N.PAI_F32, dx.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, rk, 0,
                            ct.data_ptr(), ex.data_ptr(), st.data_ptr(), s))
    m_ct, m_ex = torch.empty_like(ct), torch.empty_like(ex)
    chk(lib.pai_mul_dev(ctx.handle, ct.data_ptr(), ex.data_ptr(), n, N.PAI_F64, dsc.data_ptr(), 1,
                        m_ct.data_ptr(), m_ex.data_ptr(), st.data_ptr(), s))
    a_ct, a_ex = torch.empty_like(ct), torch.empty_like(ex)
    chk(lib.pai_add_plain_dev(ctx.handle, m_ct.data_ptr(), m_ex.data_ptr(), n, N.PAI_F64, dy.data_ptr(), 1,
                              a_ct.data_ptr(), a_ex.data_ptr(), st.data_ptr(), s))
    assert int(st.abs().sum().item()) == 0
    # host-buffer entry points on the same data give the same words
    h_ct, h_ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=0)
    h_m, h_me, _ = ctx.mul(h_ct, h_ex, sc)
    h_a, h_ae, _ = ctx.add_plain(h_m, h_me, y)
    torch.cuda.synchronize()
    assert np.array_equal(a_ct.cpu().numpy().view(np.uint32), h_a) and np.array_equal(a_ex.cpu().numpy(), h_ae)
    # oracle on a few elements
    got = N.words_to_ints(h_a)
    base = N.words_to_ints(h_ct)
    for i in (0, 1, 150, n - 1):
        c, e = O.mul_scalar(base[i], int(h_ex[i]), float(sc[i]), key)
        assert (got[i], int(h_ae[i])) == O.add_scalar(c, e, float(y[i]), key), i
    # segmented sum on the device, then decrypt on the device
    bins = [np.arange(0, 17), np.array([], dtype=np.int64), np.arange(17, n)]
    idx = np.concatenate(bins).astype(np.int64)
    off = np.array([0, 17, 17, n], dtype=np.int64)
    g_ct = torch.empty((3, W), dtype=torch.int32, device=dev)
    g_ex = torch.empty(3, dtype=torch.int32, device=dev)
    chk(lib.pai_segment_add_dev(ctx.handle, a_ct.data_ptr(), a_ex.data_ptr(), n, idx.ctypes.data, off.ctypes.data, 3,
                                g_ct.data_ptr(), g_ex.data_ptr(), s))
    val = torch.empty(3, dtype=torch.float64, device=dev)
    dst = torch.empty(3, dtype=torch.int32, device=dev)
    chk(lib.pai_decrypt_dev(ctx.handle, g_ct.data_ptr(), g_ex.data_ptr(), 3, val.data_ptr(), None,
                            dst.data_ptr(), None, s))
    torch.cuda.synchronize()
    want = x.astype(np.float64) * sc + y
    v = val.cpu().numpy()
    assert abs(v[0] - want[:17].sum()) <= 1e-9 * max(1.0, abs(want[:17].sum()))
    assert abs(v[2] - want[17:].sum()) <= 1e-9 * max(1.0, abs(want[17:].sum()))
    h_s, h_se = ctx.segment_add(h_a, h_ae, idx, off)
    assert np.array_equal(g_ct.cpu().numpy().view(np.uint32), h_s) and np.array_equal(g_ex.cpu().numpy(), h_se)
