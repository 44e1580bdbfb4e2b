"""parallel_ops — same API as flex/crypto/paillier/parallel_ops.py:23-129.

enc + enc arrays run as one batched GPU add (cipher_array.add_encrypted) and enc * plain as one
batched GPU multiply (cipher_array.mul_plain) instead of one ProcessPoolExecutor task per element;
enc + plain as one batched GPU encode + add (cipher_array.add_plain)."""
from typing import Union

import numpy as np

from .cipher_array import PaillierArray, add_encrypted, add_plain, mul_plain


def mul(x: np.ndarray, y: Union[np.ndarray, float, int]) -> np.ndarray:
    return calculate(x, y, 'mul')


def add(x: np.ndarray, y: Union[np.ndarray, float, int]) -> np.ndarray:
    return calculate(x, y, 'add')


def _add(x, y):
    return x + y


def _mul(x, y):
    return x * y


def calculate(x: np.ndarray, y: Union[np.ndarray, float, int], method: str) -> np.ndarray:
    if not isinstance(x, np.ndarray):
        # the reference raises ValueError(msg=...), which Python turns into a TypeError
        raise TypeError(f"{type(x)} * {type(y)} not supported")
    if method == 'add':
        func = _add
    elif method == 'mul':
        func = _mul
    else:
        raise NotImplementedError(method)
    if isinstance(y, np.ndarray) and x.shape != y.shape:
        raise TypeError(f"{x.shape} != {y.shape}")
    if method == 'add' and isinstance(y, np.ndarray) and y.dtype == object:
        res = add_encrypted(x, y)
        if res is not NotImplemented:
            return res.reshape(x.shape)
    if method == 'add' and (isinstance(y, (int, float)) or (isinstance(y, np.ndarray) and y.dtype != object)):
        res = add_plain(x, y)                    # one encode launch + one 2-way k_add
        if res is not NotImplemented:
            return res.reshape(x.shape)
    if method == 'mul' and (isinstance(y, (int, float)) or (isinstance(y, np.ndarray) and y.dtype != object)):
        res = mul_plain(x, y)                    # one GPU launch instead of a task per element
        if res is not NotImplemented:
            return res.reshape(x.shape)
    xf = np.asarray(x).reshape(-1)
    if isinstance(y, (int, float)):
        out = [func(a, y) for a in xf]
    else:
        yf = np.asarray(y).reshape(-1)
        out = [func(a, b) for a, b in zip(xf, yf)]
    return np.array(out).reshape(x.shape)


def segment_sum(x: np.ndarray, index_lists) -> list:
    """``[sum(x[i]) for i in index_lists]`` (the per-bin sums of hetero_bin.py:28-36) as ONE segmented
    k-way add on the GPU (pai_segment_add) followed by ``0 + S`` (one batched add_plain, which raises a
    segment whose exponent is negative to 0 exactly like Python's sum starting from int 0). Empty
    segments give the int 0, as ``sum([])`` does."""
    from . import _runtime
    from .cipher_array import _encrypted_operand, materialize, pack
    lists = [np.asarray(i).reshape(-1) for i in index_lists]
    flat = np.asarray(x).reshape(-1)
    A, pk = _encrypted_operand(flat)
    if A is None:
        return [sum(flat[i]) for i in lists]
    sizes = np.array([len(i) for i in lists], dtype=np.int64)
    idx = np.concatenate(lists).astype(np.int64) if sizes.sum() else np.zeros(0, dtype=np.int64)
    idx = np.where(idx < 0, idx + flat.size, idx)          # numpy negative indices, like x[i]
    seg_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    words, exps, _ = pack(x, pk)
    ctx = _runtime.context(pk)
    out, oe = ctx.segment_add(words, exps, idx, seg_off)
    nz = np.flatnonzero(sizes)
    res = [0] * len(lists)
    if nz.size:
        sums = materialize(pk, out[nz], oe[nz], (nz.size,), obfuscated=False)
        total = add_plain(sums, 0)                          # Python's sum starts from the int 0
        for k, s in zip(nz.tolist(), np.asarray(total).reshape(-1)):
            res[k] = s
    return res


def good_bad_calc(y: np.ndarray, index_lists):
    """HeteroBin.en_good_bad_calc (hetero_bin.py:27-36) on the GPU: good_s = sum(y[i]), bad_s = len(i) -
    good_s for every bin; returns the two numpy arrays the reference builds."""
    good = segment_sum(y, index_lists)
    lens = np.array([len(np.asarray(i).reshape(-1)) for i in index_lists], dtype=np.int64)
    enc = [k for k, g in enumerate(good) if not isinstance(g, (int, np.integer))]
    bad = [int(n) - g if isinstance(g, (int, np.integer)) else None for n, g in zip(lens, good)]
    if enc:
        objs = np.empty(len(enc), dtype=object)
        objs[:] = [good[k] for k in enc]
        neg = mul_plain(objs, -1)                            # len - g = len + (g * -1)  (encrypted_number.py:77-78)
        b = add_plain(neg, lens[enc])
        for k, v in zip(enc, np.asarray(b).reshape(-1)):
            bad[k] = v
    return np.array(good), np.array(bad)
