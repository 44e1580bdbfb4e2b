"""CiphertextBuffer: ciphertext arrays in the packed device format, with no Python object per element.

A PaillierArray (cipher_array.py) is an object ndarray so that every reference caller keeps working; the
price is one PaillierEncryptedNumber and one Python int per element (~1 us each to build).
A party that only forwards, sums or scales ciphertexts -- the HE_SA_FT coordinator summing the parties'
gradients (he_sa_ft/train.py:64-71), a relay between two ionic_bond peers -- never needs those objects.
CiphertextBuffer keeps the words ([N, W] little-endian uint32), the exponents and the obfuscation flags
as numpy arrays, and runs the array operators straight on the GPU:

    buf = from_wire(received_bytes, lazy=True)      # no objects: validated words + exponents
    total = add_buffers([buf, other, third])        # ONE k-way k_add launch (encrypted_number.py:166-185)
    scaled = total * 0.5                            # ONE k_mul launch (encrypted_number.py:86-113)
    send(scaled.to_wire())                          # same bulk format, straight from the words
    values = decryptor.decrypt(scaled)              # ONE decrypt launch (decryptor.py:91-112)

Results are bit-identical to the per-object operators (same kernels as PaillierArray's). Conversions:
CiphertextBuffer.from_array(PaillierArray or object ndarray), .to_array() -> PaillierArray,
PaillierEncryptor.encrypt_to_buffer(ndarray).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .encrypted_number import PaillierEncryptedNumber


class CiphertextBuffer(object):
    __slots__ = ("public_key", "words", "exps", "obfuscated", "shape")

    def __init__(self, public_key, words: np.ndarray, exps: np.ndarray, obfuscated=None, shape=None):
        W = (2 * public_key.n.bit_length() + 31) // 32
        words = np.ascontiguousarray(words, dtype=np.uint32)
        exps = np.ascontiguousarray(exps, dtype=np.int32).reshape(-1)
        N = exps.size
        if words.shape != (N, W):
            raise ValueError(f"ciphertext words {words.shape} do not match ({N}, {W}) for this key")
        self.public_key = public_key
        self.words = words
        self.exps = exps
        if obfuscated is None:
            obfuscated = np.zeros(N, dtype=np.uint8)
        self.obfuscated = np.broadcast_to(np.asarray(obfuscated, dtype=np.uint8), (N,)).copy()
        self.shape = tuple(shape) if shape is not None else (N,)
        if int(np.prod(self.shape)) != N:
            raise ValueError("shape does not match the number of ciphertexts")

    # ---------------------------------------------------------------- conversions
    @classmethod
    def from_array(cls, arr) -> "CiphertextBuffer":
        """Pack a PaillierArray / object ndarray of PaillierEncryptedNumber (one public key)."""
        from .cipher_array import _encrypted_operand, pack
        A, pk = _encrypted_operand(arr)
        if A is None:
            raise TypeError("from_array needs a non-empty array of PaillierEncryptedNumber with one public key")
        words, exps, _ = pack(arr, pk)
        obf = np.fromiter((e._is_obfuscated() for e in A.reshape(-1)), dtype=np.uint8, count=A.size)
        return cls(pk, words, exps, obf, A.shape)

    def to_array(self):
        """PaillierArray of PaillierEncryptedNumber (materialises one object per element)."""
        from .cipher_array import materialize
        return materialize(self.public_key, self.words, self.exps, self.shape, obfuscated=self.obfuscated != 0)

    def to_wire(self) -> bytes:
        from .cipher_array import _wire_bytes
        return _wire_bytes(self.public_key.n, self.shape, self.exps, self.obfuscated, self.words)

    def reshape(self, *shape) -> "CiphertextBuffer":
        shape = shape[0] if len(shape) == 1 and isinstance(shape[0], (tuple, list)) else shape
        shape = tuple(np.empty(self.size, dtype=np.uint8).reshape(shape).shape)
        return CiphertextBuffer(self.public_key, self.words, self.exps, self.obfuscated, shape)

    @property
    def size(self) -> int:
        return self.exps.size

    def __len__(self) -> int:
        return self.shape[0] if self.shape else 1

    def __repr__(self) -> str:
        return f"CiphertextBuffer(shape={self.shape}, key_bits={self.public_key.n.bit_length()})"

    def _ctx(self):
        from . import _runtime
        if not _runtime.gpu_available():
            raise RuntimeError("CiphertextBuffer operators need a GPU (use .to_array() for the host operators)")
        return _runtime.context(self.public_key)

    def _like(self, words, exps, obfuscated=0, shape=None) -> "CiphertextBuffer":
        return CiphertextBuffer(self.public_key, words, exps, obfuscated, shape or self.shape)

    def _coerce(self, other) -> Optional["CiphertextBuffer"]:
        if isinstance(other, CiphertextBuffer):
            b = other
        elif isinstance(other, np.ndarray) and other.dtype == object:
            b = CiphertextBuffer.from_array(other)
        else:
            return None
        if b.public_key != self.public_key:
            raise ValueError("add two numbers have different public key!")    # encrypted_number.py:169-170
        if b.shape != self.shape:
            raise ValueError(f"shapes {self.shape} and {b.shape} differ")
        return b

    # ---------------------------------------------------------------- operators (GPU)
    def __add__(self, other):
        b = self._coerce(other)
        if b is not None:
            return add_buffers([self, b])
        if isinstance(other, PaillierEncryptedNumber):
            return add_buffers([self, CiphertextBuffer.from_array(np.full(self.shape, other, dtype=object))])
        return self._add_plain(other)

    __radd__ = __add__

    def __sub__(self, other):
        # self + (other * -1), encrypted_number.py:74-75: an encrypted operand is scaled by -1 on the GPU
        # (k_mul with the batch inversion) and added by k_add; a plain one is negated and added as plain
        if isinstance(other, PaillierEncryptedNumber):
            other = CiphertextBuffer.from_array(np.full(self.shape, other, dtype=object))
        b = self._coerce(other)
        if b is not None:
            return add_buffers([self, b * -1])
        return self._add_plain(_plain(other, self.size) * -1)

    def __rsub__(self, other):
        if isinstance(other, PaillierEncryptedNumber):
            return CiphertextBuffer.from_array(np.full(self.shape, other, dtype=object)) - self
        return (self * -1)._add_plain(other)                    # other + (self * -1), encrypted_number.py:77-78

    def _add_plain(self, y):
        x = _plain(y, self.size)
        out, oe, st = self._ctx().add_plain(self.words, self.exps, x)
        bad = np.flatnonzero(st)
        if bad.size:
            # values the device flags (float overflow, |M| near max_int): the per-element operator, which
            # raises the reference's exception where it does
            out = out.copy()
            oe = oe.copy()
            ints = _ints(self.words[bad])
            for j, i in enumerate(bad.tolist()):
                r = PaillierEncryptedNumber(self.public_key, ints[j], int(self.exps[i])) + _item(y, i)
                out[i] = _words(r.ciphertext(False), self.words.shape[1])
                oe[i] = r.exponent
        return self._like(out, oe)

    def __mul__(self, y):
        if isinstance(y, (PaillierEncryptedNumber, CiphertextBuffer)):
            raise ValueError("PaillierEncryptedNumber * PaillierEncryptedNumber is not allowed.")
        out, oe, _ = self._ctx().mul(self.words, self.exps, _plain(y, self.size))
        return self._like(out, oe)

    __rmul__ = __mul__

    def __truediv__(self, s):
        return self * (1 / s)

    def dot(self, b):
        """(K,) or (m, K) encrypted @ (K,) or (K, d) plain, numpy semantics (he_otp_lr_ft1/train.py:160)."""
        x = np.asarray(b)
        if len(self.shape) not in (1, 2) or x.ndim not in (1, 2) or x.shape[0] != self.shape[-1]:
            raise ValueError(f"dot: shapes {self.shape} and {x.shape} not aligned")
        from .cipher_array import _plain_array
        xs = _plain_array(x)
        if xs is None:
            raise TypeError(f"dot: unsupported operand dtype {x.dtype}")
        m = self.shape[0] if len(self.shape) == 2 else 1
        d = x.shape[1] if x.ndim == 2 else 1
        out, oe = self._ctx().matmul(self.words, self.exps, m, self.shape[-1], np.ascontiguousarray(xs).reshape(-1), d)
        shape = tuple(([m] if len(self.shape) == 2 else []) + ([d] if x.ndim == 2 else []))
        return self._like(out, oe, 0, shape if shape else (1,))

    __matmul__ = dot


def add_buffers(bufs: Sequence[CiphertextBuffer]) -> CiphertextBuffer:
    """Element-wise sum of k buffers of one key and shape in ONE k-way add launch (the reference's
    left-to-right __add__ chain gives the same ciphertexts: each sum is the product of the operands
    aligned to the largest exponent)."""
    bufs = list(bufs)
    if not bufs:
        raise ValueError("add_buffers needs at least one buffer")
    a = bufs[0]
    for b in bufs[1:]:
        a._coerce(b)
    if len(bufs) == 1:
        return a
    out, oe = a._ctx().add([b.words for b in bufs], [b.exps for b in bufs])
    return a._like(out, oe)


def _plain(y, N: int) -> np.ndarray:
    from .cipher_array import _plain_array, _plain_scalar
    if isinstance(y, np.ndarray):
        x = _plain_array(y.reshape(-1))
        if x is None or x.size not in (1, N):
            raise TypeError(f"unsupported plain operand {y.dtype}{y.shape}")
        return x
    dt = _plain_scalar(y)
    if dt is None:
        raise TypeError(f"unsupported plain operand {type(y)}")
    return np.array([y], dtype=dt)


def _item(y, i):
    return y.reshape(-1)[i if y.size > 1 else 0] if isinstance(y, np.ndarray) else y


def _ints(words):
    from . import _runtime
    return _runtime.words_to_ints(words)


def _words(v: int, W: int) -> np.ndarray:
    from . import _runtime
    return _runtime.ints_to_words([v], W)[0]
