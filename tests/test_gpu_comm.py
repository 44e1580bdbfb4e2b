"""GPU check of the C ABI's RCCL shard all-gather (pai_comm_* / pai_allgather_*, comm.hip) at world size 1
on the one-GPU box: the communicator comes up from a unique id, the grouped all-gather of ciphertext words
and exponents reproduces the shard bit for bit, and the byte all-gather likewise. The N > 1 exchange is the
driver's 8-GPU bench (bench.py configs[3]/[4] gather through torch.distributed/RCCL); its shard/index
logic is covered on CPU by tests/test_dist_shards.py (gloo, world size 2)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_allgather_world1_bit_exact(golden):
    import torch
    from flex.crypto.paillier import _native as N
    from oracle import paillier_oracle as O
    k = golden["keys"]["1024"]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    ctx = N.Context(key.n, 0, key.p, key.q)
    x = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=b"\x05" * 32)
    dev = torch.device("cuda", 0)
    d_ct = torch.from_numpy(ct.view(np.int32)).to(dev)
    d_ex = torch.from_numpy(ex).to(dev)
    o_ct = torch.zeros_like(d_ct)
    o_ex = torch.zeros_like(d_ex)
    comm = N.Comm(N.Comm.unique_id(), world=1, rank=0, device=0)
    try:
        s = torch.cuda.current_stream(dev)
        comm.allgather_shards(d_ct.data_ptr(), d_ex.data_ptr(), x.size, ctx.ct_words, o_ct.data_ptr(),
                              o_ex.data_ptr(), s.cuda_stream)
        raw = torch.arange(256, dtype=torch.uint8, device=dev)
        got = torch.zeros_like(raw)
        from flex.crypto.paillier._native import _check
        _check(comm.lib.pai_allgather_dev(comm._h, raw.data_ptr(), 256, got.data_ptr(), s.cuda_stream))
        torch.cuda.synchronize()
    finally:
        comm.close()
    assert torch.equal(o_ct, d_ct) and torch.equal(o_ex, d_ex) and torch.equal(got, raw)
    with pytest.raises(ValueError):
        N.Comm(b"short", 1, 0)
