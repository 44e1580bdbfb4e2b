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


CHILD = r'''
import os, sys, json
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/ibond-flex_amd"]
import numpy as np, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2], RANK="0", WORLD_SIZE="1")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.sharding import gather_shards_async
g = json.load(open(sys.argv[1] + "/tests/golden/paillier_golden.json"))["keys"]["2048"]
ctx = N.Context(int(g["n"], 16), 0, int(g["p"], 16), int(g["q"], 16))
lib = N.load_library()
n, W = 65536, ctx.ct_words
x = torch.from_numpy(np.random.default_rng(3).standard_normal(n, dtype=np.float32)).to(dev)
outs = []
bufs = [(torch.empty((n, W), dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(2)]
gath = [(torch.empty((n, W), dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(2)]
st = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev)
works = []
for step in range(4):   # bench.py's double-buffered encrypt + asynchronous gather, on RCCL
    b = step % 2
    for w in [w for (bb, w) in works if bb == b]:
        w.wait()
    works = [(bb, w) for (bb, w) in works if bb != b]
    ct, ex = bufs[b]
    assert lib.pai_encrypt_dev(ctx.handle, N.PAI_F32, x.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, b"\x09" * 32,
                               1000 * step, ct.data_ptr(), ex.data_ptr(), st.data_ptr(), s.cuda_stream) == 0
    for t, o in zip(bufs[b], gath[b]):
        _, w = gather_shards_async(t, n, 1, out=o)
        works.append((b, w))
for _, w in works:
    w.wait()
torch.cuda.synchronize()
ok = all(torch.equal(bufs[b][i], gath[b][i]) for b in range(2) for i in range(2))
dist.destroy_process_group()
print(json.dumps({"ok": ok}))
'''


def test_torch_distributed_rccl_gather_world1():
    """bench.py's multi-GPU step at world size 1 on real RCCL ("nccl" backend, device tensors): double-buffered
    pai_encrypt_dev outputs all-gathered asynchronously with sharding.gather_shards_async into preallocated
    receive buffers, every gathered block equal to its shard. (N > 1 needs one GPU per rank: the driver's run.)"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", CHILD, root, "29517"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["ok"]
