"""Multi-GPU sharding of a Paillier array: one process per GPU, contiguous shards,
obfuscators keyed by the GLOBAL element index (so the ciphertexts do not depend on the number of
GPUs), one all-gather to reassemble. Elements are independent (flex/crypto/paillier/encryptor.py:71-97
maps element-wise), so there is no other communication. The collective is torch.distributed:
RCCL over xGMI on GPUs ("nccl" backend), gloo in the CPU tests.
"""
from __future__ import annotations

from typing import Tuple


def shard_bounds(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, stop) of rank's contiguous block of ceil(total / world) elements (the last may be short)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-total // world)
    start = min(rank * per, total)
    return start, min(start + per, total)


def gather_shards(local, total: int, world: int, group=None):
    """All-gather equal-size (padded) shards of a [rows, ...] tensor into the [total, ...] array."""
    import torch
    import torch.distributed as dist
    per = -(-total // world)
    if local.shape[0] > per:
        raise ValueError("shard larger than ceil(total / world)")
    if local.shape[0] < per:
        pad = torch.zeros((per - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.is_cuda:
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, local.contiguous(), group=group)
        out = torch.cat(parts)
    return out[:total]


def gather_shards_async(local, total: int, world: int, group=None, out=None):
    """Like gather_shards, but the collective is issued asynchronously: returns (out, work). On GPUs
    the RCCL all-gather runs on the process group's own stream (ordered after the work already queued
    on the current stream), so the caller can launch the next shard's kernels on the compute stream
    while it runs, and calls work.wait() before reusing `local` or reading `out`. work is None when
    the gather completed synchronously. `out` (optional, [world * ceil(total / world), ...])
    is a preallocated receive buffer reused across steps instead of a fresh allocation per call. On CPU tensors (gloo,
    the multi-rank CPU tests) the gather is asynchronous too: gloo writes the world's shards into views of `out`
    in the background until work.wait()."""
    import torch
    import torch.distributed as dist
    per = -(-total // world)
    if local.shape[0] > per:
        raise ValueError("shard larger than ceil(total / world)")
    if local.shape[0] < per:
        pad = torch.zeros((per - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    shape = (world * per,) + tuple(local.shape[1:])
    if out is None:
        out = torch.empty(shape, dtype=local.dtype, device=local.device)
    elif tuple(out.shape) != shape or out.dtype != local.dtype:
        raise ValueError(f"receive buffer {tuple(out.shape)} {out.dtype} != {shape} {local.dtype}")
    if local.is_cuda:
        work = dist.all_gather_into_tensor(out, local.contiguous(), group=group, async_op=True)
    else:
        work = dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group, async_op=True)
    return out[:total], work
