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
