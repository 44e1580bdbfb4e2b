"""ctypes wrapper of oracle/_build/libgmp_oracle.so (GMP restatement of the reference CPU path).
TEST / BASELINE INFRASTRUCTURE ONLY — see oracle/gmp_oracle.c."""
import ctypes
import os

import numpy as np

_LIB = None
PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libgmp_oracle.so")


def available() -> bool:
    return os.path.exists(PATH)


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(PATH)
        P, S, I, U64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        _LIB.oracle_encrypt_f32_chacha.argtypes = [P, S, P, S, P, U64, P, P, I]
        _LIB.oracle_decrypt_raw.argtypes = [P, P, S, P, S, P, I]
    return _LIB


def encrypt_f32_chacha(n: int, x: np.ndarray, key32: bytes, index_base: int = 0, nthreads: int = 1):
    x = np.ascontiguousarray(x, dtype=np.float32)
    nb = n.bit_length()
    ctw = (2 * nb + 31) // 32
    ct = np.zeros((x.size, ctw), dtype=np.uint32)
    ex = np.zeros(x.size, dtype=np.int32)
    nbytes = (nb + 7) // 8
    lib().oracle_encrypt_f32_chacha(n.to_bytes(nbytes, "little"), nbytes, x.ctypes.data, x.size, key32,
                                    index_base, ct.ctypes.data, ex.ctypes.data, nthreads)
    return ct, ex


def decrypt_raw(p: int, q: int, ct: np.ndarray, nthreads: int = 1) -> np.ndarray:
    ct = np.ascontiguousarray(ct, dtype=np.uint32)
    hb = max(p.bit_length(), q.bit_length()) // 8 + 1
    n = p * q
    ptw = (n.bit_length() + 31) // 32
    out = np.zeros((ct.shape[0], ptw), dtype=np.uint32)
    lib().oracle_decrypt_raw(p.to_bytes(hb, "little"), q.to_bytes(hb, "little"), hb, ct.ctypes.data, ct.shape[0],
                             out.ctypes.data, nthreads)
    return out
