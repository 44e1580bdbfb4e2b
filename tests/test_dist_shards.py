"""World-size-2 gloo test (CPU) of the multi-GPU sharding logic used by bench.py
(flex/crypto/paillier/sharding.py): contiguous shards, obfuscators keyed by the global index,
all-gather; the reassembled ciphertexts equal a single-process encryption bit for bit. The
per-shard encryption here is the CPU oracle (no GPU in this test); on the GPU box the same
sharding drives libflexpai."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import paillier_oracle as O

NB = 1024
TOTAL = 9          # ragged: ceil(9 / 2) = 5 -> shards of 5 and 4
KEY32 = bytes(range(32))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _encrypt_range(key, x, start, stop):
    from flex.crypto.paillier._native import ints_to_words
    W = (2 * key.n.bit_length() + 31) // 32
    rb = ((NB + 64 + 31) // 32) * 4
    cts = []
    for g in range(start, stop):
        c, _ = O.encrypt_value(x[g], key, O.device_r(KEY32, g, rb))
        cts.append(c)
    return ints_to_words(cts, W) if cts else np.zeros((0, W), np.uint32)


def _worker(rank, world, port, keyt, x, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flex.crypto.paillier.sharding import gather_shards, gather_shards_async, shard_bounds
        key = O.Key(*keyt)
        s0, s1 = shard_bounds(TOTAL, world, rank)
        local = torch.from_numpy(_encrypt_range(key, x, s0, s1).view(np.int32).copy())
        full = gather_shards(local, TOTAL, world)
        full2, work = gather_shards_async(local, TOTAL, world)
        if work is not None:
            work.wait()
        assert torch.equal(full, full2)
        # preallocated receive buffer reused across steps (bench.py double-buffers these)
        per = -(-TOTAL // world)
        buf = torch.zeros((world * per,) + tuple(local.shape[1:]), dtype=local.dtype)
        for _ in range(2):
            full3, work = gather_shards_async(local, TOTAL, world, out=buf)
            if work is not None:
                work.wait()
            assert torch.equal(full, full3) and full3.data_ptr() == buf.data_ptr()
        if rank == 0:
            q.put(full.numpy().view(np.uint32).copy())
    finally:
        dist.destroy_process_group()


def test_shard_bounds():
    from flex.crypto.paillier.sharding import shard_bounds
    assert [shard_bounds(9, 2, r) for r in range(2)] == [(0, 5), (5, 9)]
    assert [shard_bounds(16, 8, r) for r in range(8)] == [(2 * r, 2 * r + 2) for r in range(8)]
    assert shard_bounds(3, 4, 3) == (3, 3)
    with pytest.raises(ValueError):
        shard_bounds(3, 2, 2)


def test_gloo_world2_gather_matches_serial(golden):
    k = golden["keys"][str(NB)]
    keyt = (int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    key = O.Key(*keyt)
    x = np.random.default_rng(5).standard_normal(TOTAL).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, keyt, x, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _encrypt_range(key, x, 0, TOTAL)
    assert np.array_equal(got, want)
