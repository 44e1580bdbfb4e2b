"""Several ranks on the one GPU of the test box: bench.py's sharded step through libflexpai in separate
processes -- contiguous shards (sharding.shard_bounds), obfuscators keyed by the GLOBAL element index, a native
context and fixed-base tables per process -- with the shards gathered by gloo on host copies
(sharding.gather_shards; RCCL needs one device per rank, the driver's 8-GPU run covers it). The reassembled
ciphertexts are bit-identical to one process encrypting the whole array, for the fixed-base sampler and for the
generic CRT path, at world 2 and 3 (ragged shards), and decrypt to the input (encryptor.py:89-96 maps elements
independently, which is what makes the split legal)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NB = 1024
TOTAL = 1001
KEY32 = bytes(range(7, 39))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _context(fixed_base):
    from flex.crypto.paillier import _native
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk, sk = generate_paillier_keypair(NB, seed=1)
    ctx = _native.Context(pk.n, 0, sk.p, sk.q)
    ctx.set_fixed_base(fixed_base)
    if fixed_base:
        ctx.set_fb_window(12)
        ctx.prepare_fixed_base()
    return ctx


def _worker(rank, world, port, fixed_base, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXPAI_QUIET="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flex.crypto.paillier.sharding import gather_shards, shard_bounds
        ctx = _context(fixed_base)
        x = np.random.default_rng(11).standard_normal(TOTAL).astype(np.float32)
        s0, s1 = shard_bounds(TOTAL, world, rank)
        ct, ex, st = ctx.encrypt(x[s0:s1], rng_key=KEY32, index_base=s0)
        assert not st.any()
        full = gather_shards(torch.from_numpy(ct.view(np.int32)), TOTAL, world)
        fe = gather_shards(torch.from_numpy(ex), TOTAL, world)
        if rank == 0:
            q.put((full.numpy().view(np.uint32).copy(), fe.numpy().copy(), ctx.fb_ready))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fixed_base", [True, False])
@pytest.mark.parametrize("world", [2, 3])
def test_ranks_sharing_the_gpu_equal_one_process(world, fixed_base):
    ctx = _context(fixed_base)
    x = np.random.default_rng(11).standard_normal(TOTAL).astype(np.float32)
    want_ct, want_ex, st = ctx.encrypt(x, rng_key=KEY32, index_base=0)
    assert not st.any() and ctx.fb_ready == fixed_base
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_worker, args=(r, world, port, fixed_base, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got_ct, got_ex, ready = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert ready == fixed_base
    assert np.array_equal(got_ct, want_ct) and np.array_equal(got_ex, want_ex)
    val, _, st2, _ = ctx.decrypt(got_ct, got_ex)
    assert not np.asarray(st2).any() and np.array_equal(np.asarray(val, dtype=np.float64), x.astype(np.float64))
