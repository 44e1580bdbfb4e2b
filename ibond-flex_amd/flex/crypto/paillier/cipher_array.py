"""PaillierArray: the ndarray the array entry points return.

It IS an ``np.ndarray`` of ``PaillierEncryptedNumber`` objects (dtype=object), so
``flex/tools/iterative_apply.py:26-41`` (which type-checks ``np.ndarray``) and every caller that
indexes, reshapes or pickles the result keep working unchanged. Two additions:

* it remembers the packed device format of its ciphertexts (little-endian uint32 words [N, W]
  plus int32 exponents), validated by object identity before use, so chained array operations
  do not re-serialise Python ints;
* ``a + b`` between two encrypted arrays (the HE_SA_FT coordinator's ``iterative_add``,
  he_sa_ft/train.py:64-71, and ``sum(...)`` callers) runs as ONE batched k-way add on the GPU
  instead of numpy's per-object loop (encrypted_number.py:166-185);
* ``a + y``, ``y + a``, ``a - y``, ``y - a`` with a plain scalar or array (encrypted_number.py:65-78,
  139-164: encode y with max_exponent = e_x, raw-encrypt with r = 1, align, multiply) run as ONE encode
  launch plus ONE 2-way k_add;
* ``a * s``, ``s * a``, ``a / s`` with a plain scalar or array (encrypted_number.py:80-113) run as ONE
  GPU launch (negative scalars: one batch inversion for the whole array), and ``a.dot(x)`` /
  ``a @ x`` with a plain matrix (he_otp_lr_ft1/train.py:160) as one launch plus a reduction tree.

Pickling (ionic_bond ships pickles, ion.py:150-178) writes, by default, exactly what the reference
writes: a plain object ndarray of PaillierEncryptedNumber (same class path and slot state), which an
unmodified FLEX peer's ``pickle.load`` (ion.py:201) reads. Deployments where every party runs this
package opt in to the bulk wire format below with ``FLEXPAI_PICKLE_BULK=1`` on the senders: the pickle
then unpickles into a PaillierArray with its packed words cached, so an array received from a flexpai
peer goes straight back to the GPU for the receiver's ``+``, ``sum``, ``.dot`` and ``*`` (HE_SA_FT
coordinator he_sa_ft/train.py:66-69, HE_OTP_LR he_otp_lr_ft1/train.py:158-160, HE_LINEAR
he_linear_ft/train.py:64-65). Plain object ndarrays (the default, and what unmodified peers send) run
the reference's per-element operators on the package's GMP binding (_bigint.py).

On a host without a GPU (e.g. a CPU-only protocol coordinator) the operators on existing ciphertext
arrays fall back to numpy's per-element loop over PaillierEncryptedNumber, i.e. exactly the reference's
computation on GMP; encryption and decryption still require the GPU and raise without one.
"""
from __future__ import annotations

import contextlib
import gc
import operator
import os
from typing import Optional, Tuple

import numpy as np

from .encrypted_number import PaillierEncryptedNumber

_CT = "_PaillierEncryptedNumber__ciphertext"

try:                                        # bulk slot construction and checks (csrc/hostgmp.c), when built
    from ._gmp import make_numbers as _make_numbers, packed_valid as _packed_valid, pack_numbers as _pack_numbers
except ImportError:                         # pragma: no cover - build() always builds it
    _make_numbers = _packed_valid = _pack_numbers = None


class _Packed:
    __slots__ = ("n", "words", "exps", "ints")

    def __init__(self, n: int, words: np.ndarray, exps: np.ndarray, ints: list):
        self.n, self.words, self.exps, self.ints = n, words, exps, ints


def bulk_pickle_enabled() -> bool:
    """FLEXPAI_PICKLE_BULK=1: pickle PaillierArray through the bulk wire format (all peers run flexpai).
    Default: the reference's plain object-ndarray pickle."""
    return os.environ.get("FLEXPAI_PICKLE_BULK", "0").strip() not in ("", "0")


class PaillierArray(np.ndarray):
    def __new__(cls, objs: np.ndarray, packed: Optional[_Packed] = None):
        obj = np.asarray(objs, dtype=object).view(cls)
        obj._packed = packed
        return obj

    def __array_finalize__(self, obj):
        self._packed = None

    def __reduce__(self):
        plain = np.asarray(self).view(np.ndarray).__reduce__
        if not bulk_pickle_enabled():
            return plain()
        try:
            return (_from_pickle, (to_wire(self),))
        except (TypeError, ValueError):      # empty, mixed keys or non-ciphertext elements
            return plain()

    def __setitem__(self, key, value):
        self._packed = None
        super().__setitem__(key, value)

    # ---------------------------------------------------------------- packed view
    def _valid_packed(self) -> Optional[_Packed]:
        pk = getattr(self, "_packed", None)
        if pk is None:
            return None
        flat = np.asarray(self).reshape(-1)
        if flat.size != pk.exps.size:
            return None
        if _packed_valid is not None:            # the same identity check in C (csrc/hostgmp.c), ~ns/element
            return pk if _packed_valid(PaillierEncryptedNumber, flat, pk.ints, pk.exps) else None
        try:
            cur = [getattr(e, _CT) for e in flat]
            exps = [e.exponent for e in flat]
        except AttributeError:
            return None
        if not all(map(operator.is_, cur, pk.ints)):
            return None
        if not np.array_equal(np.asarray(exps, dtype=np.int64), pk.exps):
            return None
        return pk

    def __add__(self, other):
        res = add_encrypted(self, other)
        if res is NotImplemented:
            res = add_plain(self, other)
        if res is NotImplemented:
            return np.ndarray.__add__(np.asarray(self), other)
        return res

    def __radd__(self, other):
        res = add_encrypted(self, other)
        if res is NotImplemented:
            res = add_plain(self, other)
        if res is NotImplemented:
            return np.ndarray.__radd__(np.asarray(self), other)
        return res

    def __sub__(self, other):
        # PaillierEncryptedNumber.__sub__: self + (other * -1) (encrypted_number.py:74-75)
        res = NotImplemented
        if _plain_operand(other):
            res = add_plain(self, other * -1)
        elif _encrypted_like(other):
            res = sub_encrypted(self, other)
        if res is NotImplemented:
            return np.ndarray.__sub__(np.asarray(self), other)
        return res

    def __rsub__(self, other):
        # other + (self * -1) (encrypted_number.py:77-78)
        res = NotImplemented
        if _plain_operand(other):
            neg = mul_plain(self, -1)
            if neg is not NotImplemented:
                res = add_plain(neg, other)
        elif _encrypted_like(other):
            res = sub_encrypted(other, self)
        if res is NotImplemented:
            return np.ndarray.__rsub__(np.asarray(self), other)
        return res

    def __mul__(self, other):
        res = mul_plain(self, other)
        if res is NotImplemented:
            return np.ndarray.__mul__(np.asarray(self), other)
        return res

    def __rmul__(self, other):
        res = mul_plain(self, other)
        if res is NotImplemented:
            return np.ndarray.__rmul__(np.asarray(self), other)
        return res

    def __truediv__(self, other):
        # PaillierEncryptedNumber.__truediv__ multiplies by 1 / scalar (encrypted_number.py:83-84)
        if _plain_scalar(other) is not None and other != 0:
            res = mul_plain(self, 1 / other)
            if res is not NotImplemented:
                return res
        return np.ndarray.__truediv__(np.asarray(self), other)

    def dot(self, b, out=None):
        res = dot_plain(self, b) if out is None else NotImplemented
        if res is NotImplemented:
            return np.asarray(self).dot(b, out) if out is not None else np.asarray(self).dot(b)
        return res

    def __matmul__(self, b):
        res = dot_plain(self, b)
        if res is NotImplemented:
            return np.ndarray.__matmul__(np.asarray(self), b)
        return res


def _all_encrypted(flat) -> bool:
    return all(isinstance(e, PaillierEncryptedNumber) for e in flat)


def pack(arr: np.ndarray, public_key) -> Tuple[np.ndarray, np.ndarray, list]:
    """Packed device format of an object array of PaillierEncryptedNumber (ciphertext(False))."""
    from . import _runtime
    if isinstance(arr, PaillierArray):
        pk = arr._valid_packed()
        if pk is not None and pk.n == public_key.n:
            return pk.words, pk.exps.astype(np.int32), pk.ints
    flat = np.asarray(arr).reshape(-1)
    W = (2 * public_key.n.bit_length() + 31) // 32
    got = pack_checked(flat, public_key, W)
    if got is not None:
        return got
    ints = [e.ciphertext(False) for e in flat]
    words = _runtime.ints_to_words(ints, W)
    exps = np.fromiter((e.exponent for e in flat), dtype=np.int64, count=flat.size)
    return words, exps.astype(np.int32), ints


def pack_checked(flat: np.ndarray, public_key, W: int, want_words: bool = True):
    """One C pass over a flat object array (csrc/hostgmp.c pack_numbers): the reference's per-element check
    (every element a PaillierEncryptedNumber under `public_key`, decryptor.py:73-79), the exponents, the
    ciphertext ints and -- with want_words -- their [N, W] words. None when an element fails a check or does
    not fit (the caller's per-element path then raises the reference's exception)."""
    if _pack_numbers is None:
        return None
    got = _pack_numbers(PaillierEncryptedNumber, flat, public_key, W, want_words)
    if got is None:
        return None
    words, exps, ints = got
    w = np.frombuffer(words, dtype="<u4").reshape(len(ints), W) if words is not None else None
    return w, np.frombuffer(exps, dtype=np.int32), ints


def materialize(public_key, words: np.ndarray, exps: np.ndarray, shape, obfuscated) -> PaillierArray:
    """Device output -> PaillierArray of PaillierEncryptedNumber (+ packed cache). `obfuscated` is one
    flag for all elements or a per-element flag array."""
    from . import _runtime
    with _gc_paused():
        return _materialize(_runtime, public_key, words, exps, shape, obfuscated)


@contextlib.contextmanager
def _gc_paused():
    """Bulk construction of acyclic objects: the cyclic collector would rescan every survivor each time
    the allocation count crosses its threshold (measured: ~4x the construction cost at 256k numbers)."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _materialize(_runtime, public_key, words, exps, shape, obfuscated):
    ints = _runtime.words_to_ints(words)
    if _make_numbers is not None:
        flags = np.ascontiguousarray(obfuscated, dtype=np.uint8) if isinstance(obfuscated, np.ndarray) else bool(obfuscated)
        el = _make_numbers(PaillierEncryptedNumber, public_key, ints, np.ascontiguousarray(exps, dtype=np.int32), flags)
    else:
        make = PaillierEncryptedNumber._make
        if isinstance(obfuscated, np.ndarray):
            el = [make(public_key, c, int(e), bool(o)) for c, e, o in zip(ints, exps.tolist(), obfuscated.tolist())]
        else:
            el = [make(public_key, c, int(e), obfuscated) for c, e in zip(ints, exps.tolist())]
    objs = np.fromiter(el, dtype=object, count=len(el))     # (`objs[:] = el` probes every element: ~10x)
    return PaillierArray(objs.reshape(shape), _Packed(public_key.n, words, exps.astype(np.int64), ints))


def add_encrypted(a, b):
    """Batched GPU add of two encrypted arrays (broadcasting like numpy). Returns NotImplemented
    when either side is not entirely PaillierEncryptedNumber (or there is no GPU)."""
    from . import _runtime
    if not _runtime.gpu_available():
        return NotImplemented
    A = np.asarray(a, dtype=object) if not isinstance(a, PaillierEncryptedNumber) else None
    if A is None or A.size == 0:
        return NotImplemented
    if isinstance(b, PaillierEncryptedNumber):
        B = np.empty(A.shape, dtype=object)
        B[...] = b
    elif isinstance(b, np.ndarray) and b.dtype == object:
        B = b
    else:
        return NotImplemented
    try:
        Ab, Bb = np.broadcast_arrays(A, B)
    except ValueError:
        return NotImplemented
    fa, fb = Ab.reshape(-1), Bb.reshape(-1)
    if not (_all_encrypted(fa) and _all_encrypted(fb)):
        return NotImplemented
    pk = fa[0].public_key
    for e in (fa, fb):
        for x in e:
            if x.public_key != pk:
                raise ValueError("add two numbers have different public key!")
    if Ab.shape == np.shape(a):
        wa, ea, _ = pack(a, pk)
    else:
        wa, ea, _ = pack(np.ascontiguousarray(Ab), pk)
    if isinstance(b, np.ndarray) and Bb.shape == b.shape:
        wb, eb, _ = pack(b, pk)
    else:
        wb, eb, _ = pack(np.ascontiguousarray(Bb), pk)
    ctx = _runtime.context(pk)
    out, oe = ctx.add([wa, wb], [ea, eb])
    # __raw_add builds fresh, not-yet-obfuscated numbers (encrypted_number.py:180-185)
    return materialize(pk, out, oe, Ab.shape, obfuscated=False)


def _encrypted_like(y) -> bool:
    return isinstance(y, PaillierEncryptedNumber) or (isinstance(y, np.ndarray) and y.dtype == object)


def sub_encrypted(a, b):
    """a - b with both operands encrypted (a PaillierEncryptedNumber or an object array of them, numpy
    broadcasting): a + (b * -1) per element (encrypted_number.py:74-78) as ONE k_mul by -1 (invert(c), the
    reference's negative-scalar branch, encrypted_number.py:97-101) and ONE 2-way k_add. The add is order
    independent, so a scalar left operand is added on the right. NotImplemented when an operand is not
    entirely PaillierEncryptedNumber (or there is no GPU): the caller falls back to numpy's per-element loop."""
    if isinstance(b, PaillierEncryptedNumber):
        # a must be an encrypted array under b's key before b's inverse is paid for: otherwise the
        # caller's per-element loop recomputes everything
        if isinstance(a, PaillierEncryptedNumber):
            return NotImplemented
        A, pk = _encrypted_operand(a)
        if A is None or pk != b.public_key:
            return NotImplemented
        neg = b * -1
    else:
        neg = mul_plain(b, -1)
        if neg is NotImplemented:
            return NotImplemented
    if isinstance(a, PaillierEncryptedNumber):
        return add_encrypted(neg, a) if isinstance(neg, np.ndarray) else NotImplemented
    return add_encrypted(a, neg)


# ------------------------------------------------------------------ ciphertext x plaintext
_DEV_FLOAT = {np.dtype(np.float64): np.float64, np.dtype(np.float32): np.float32, np.dtype(np.float16): np.float32}
_DEV_INT = (np.dtype(np.int16), np.dtype(np.int32), np.dtype(np.int64))


def _plain_scalar(y):
    """The device dtype for a plain scalar operand, following FixedPointNumber.encode's type rules
    (fixedpoint_number.py:63-77), or None (bools, unsigned, big ints, other objects: host path)."""
    if isinstance(y, (bool, np.bool_)):
        return None
    if type(y) is float or isinstance(y, np.float64):
        return np.float64
    if isinstance(y, (np.float32, np.float16)):
        return np.float32
    if (type(y) is int and -(1 << 63) < y < (1 << 63)) or isinstance(y, (np.int16, np.int32, np.int64)):
        return np.int64
    return None


def _plain_array(y: np.ndarray):
    if y.dtype in _DEV_FLOAT:
        return y.astype(_DEV_FLOAT[y.dtype])
    if y.dtype in _DEV_INT:
        return y.astype(np.int64)
    return None


def _encrypted_operand(a):
    """(flat object array, public key) when `a` is entirely PaillierEncryptedNumber of one key."""
    A = np.asarray(a, dtype=object)
    flat = A.reshape(-1)
    if flat.size == 0 or not _all_encrypted(flat):
        return None, None
    pk = flat[0].public_key
    for e in flat:
        if e.public_key != pk:
            return None, None
    return A, pk


def mul_plain(a, y):
    """Encrypted array times a plain scalar or array on the GPU (PaillierEncryptedNumber.__mul__
    per element, encrypted_number.py:86-113, with numpy broadcasting). NotImplemented when an
    operand is not of a device type (the caller then falls back to the per-element operators)."""
    from . import _runtime
    if isinstance(y, PaillierEncryptedNumber):
        raise ValueError("PaillierEncryptedNumber * PaillierEncryptedNumber is not allowed.")
    if not _runtime.gpu_available():
        return NotImplemented
    A, pk = _encrypted_operand(a)
    if A is None:
        return NotImplemented
    if isinstance(y, np.ndarray):
        if y.dtype == object:
            return NotImplemented
        x = _plain_array(y)
        if x is None:
            return NotImplemented
        try:
            Ab, xb = np.broadcast_arrays(A, x)
        except ValueError:
            return NotImplemented
        shape = Ab.shape
        if shape != A.shape:
            A = np.ascontiguousarray(Ab)
        xs = np.ascontiguousarray(xb).reshape(-1)
    else:
        dt = _plain_scalar(y)
        if dt is None:
            return NotImplemented
        shape = A.shape
        xs = np.array([y], dtype=dt)
    words, exps, _ = pack(a if A is a else A, pk)
    ctx = _runtime.context(pk)
    out, oe, st = ctx.mul(words, exps, xs)
    # __mul__ returns fresh, not-yet-obfuscated numbers (encrypted_number.py:113)
    return materialize(pk, out, oe, shape, obfuscated=False)


def dot_plain(a, b):
    """numpy dot / matmul of an encrypted (K,) or (m, K) array with a plain (K,) or (K, d) array on
    the GPU: every output is sum_k a[.., k] * b[k, ..] with the reference's exponent alignment
    (bit-identical to numpy's object loop over __mul__ and __add__). NotImplemented otherwise."""
    from . import _runtime
    if not isinstance(b, np.ndarray) or b.dtype == object or b.ndim not in (1, 2) or not _runtime.gpu_available():
        return NotImplemented
    A, pk = _encrypted_operand(a)
    if A is None or A.ndim not in (1, 2):
        return NotImplemented
    x = _plain_array(b)
    if x is None:
        return NotImplemented
    K = A.shape[-1]
    if K == 0 or x.shape[0] != K:
        return NotImplemented
    m = A.shape[0] if A.ndim == 2 else 1
    d = x.shape[1] if x.ndim == 2 else 1
    words, exps, _ = pack(a if A is a else A, pk)
    ctx = _runtime.context(pk)
    out, oe = ctx.matmul(words, exps, m, K, np.ascontiguousarray(x).reshape(-1), d)
    shape = tuple(([m] if A.ndim == 2 else []) + ([d] if x.ndim == 2 else []))
    res = materialize(pk, out, oe, shape if shape else (1,), obfuscated=False)
    return res.reshape(-1)[0] if not shape else res


# ------------------------------------------------------------------ ciphertext + plaintext
# numpy's object add loop casts int arrays to object, so every integer is a Python int (exact) and every
# float a Python float; the device encoder is exact for both.
_ADD_DEV = (np.dtype(np.float16), np.dtype(np.float32), np.dtype(np.float64),
            np.dtype(np.int16), np.dtype(np.int32), np.dtype(np.int64))


def _plain_operand(y) -> bool:
    if isinstance(y, np.ndarray):
        return y.dtype in _ADD_DEV
    return _plain_scalar(y) is not None


def add_plain(a, y):
    """Encrypted array plus a plain scalar or array on the GPU (PaillierEncryptedNumber.__add__ with a
    scalar per element, encrypted_number.py:65-72, 139-164, with numpy broadcasting). Elements the device
    flags (see pai_add_plain in include/flexpai.h: float overflow, |M| near max_int) are
    redone by the per-element operator, which raises the reference's exception where it does.
    NotImplemented when an operand is not of a device type."""
    from . import _runtime
    if isinstance(y, PaillierEncryptedNumber) or not _plain_operand(y) or not _runtime.gpu_available():
        return NotImplemented
    A, pk = _encrypted_operand(a)
    if A is None:
        return NotImplemented
    if isinstance(y, np.ndarray):
        x = y.astype(np.float32) if y.dtype == np.float16 else (y.astype(np.int64) if y.dtype.kind == "i" else y)
        try:
            Ab, xb = np.broadcast_arrays(A, x)
            _, yb = np.broadcast_arrays(A, y)
        except ValueError:
            return NotImplemented
        shape = Ab.shape
        if shape != A.shape:
            A = np.ascontiguousarray(Ab)
        xs = np.ascontiguousarray(xb).reshape(-1)
        ys = yb.reshape(-1)
    else:
        shape = A.shape
        xs = np.array([y], dtype=_plain_scalar(y))
        ys = None
    words, exps, _ = pack(a if A is a else A, pk)
    ctx = _runtime.context(pk)
    out, oe, st = ctx.add_plain(words, exps, xs)
    # __raw_add returns a fresh, not-yet-obfuscated number (encrypted_number.py:180-185)
    res = materialize(pk, out, oe, shape, obfuscated=False)
    bad = np.flatnonzero(st)
    if bad.size:
        flat_a = np.asarray(A).reshape(-1)
        flat_r = np.asarray(res).reshape(-1)
        for i in bad.tolist():
            flat_r[i] = flat_a[i] + (y if ys is None else ys[i])
        res._packed = None
    return res


# ------------------------------------------------------------------ bulk wire format
# The reference ships ciphertext arrays as pickled object ndarrays (Ion._send, ion.py:150-178): ~543 B
# and one Python object per element at nb = 2048. The bulk format is the packed device layout itself:
#   magic "FPAW1\0" | u32 ndim | i64 shape[ndim] | u32 n_bytes | n (little-endian) | u32 W |
#   i32 exponents[N] | u8 obfuscated[N] | u32 words[N][W]
# i.e. 4 W + 5 bytes per element plus a header; ciphertext i = int.from_bytes(words[i], "little").
# PaillierArray pickles through this format when FLEXPAI_PICKLE_BULK=1 (see the module docstring);
# from_wire(lazy=True) reads it into a CiphertextBuffer without per-element objects.
_WIRE_MAGIC = b"FPAW1\0"


def _wire_bytes(n: int, shape, exps, obf, words) -> bytes:
    nb = (n.bit_length() + 7) // 8
    head = [_WIRE_MAGIC, np.uint32(len(shape)).tobytes(), np.asarray(shape, dtype="<i8").tobytes(),
            np.uint32(nb).tobytes(), n.to_bytes(nb, "little"), np.uint32(words.shape[1]).tobytes()]
    return b"".join(head + [np.ascontiguousarray(exps, dtype="<i4").tobytes(),
                            np.ascontiguousarray(obf, dtype=np.uint8).tobytes(),
                            np.ascontiguousarray(words, dtype="<u4").tobytes()])


def to_wire(arr) -> bytes:
    """Serialise an array of PaillierEncryptedNumber (one public key), or a CiphertextBuffer, into the
    bulk format."""
    from .cipher_buffer import CiphertextBuffer
    if isinstance(arr, CiphertextBuffer):
        return arr.to_wire()
    A, pk = _encrypted_operand(arr)
    if A is None:
        raise TypeError("to_wire needs a non-empty array of PaillierEncryptedNumber with one public key")
    words, exps, _ = pack(arr if isinstance(arr, PaillierArray) else A, pk)
    obf = np.fromiter((e._is_obfuscated() for e in A.reshape(-1)), dtype=np.uint8, count=A.size)
    return _wire_bytes(pk.n, A.shape, exps, obf, words)


def _rows_below(words: np.ndarray, limit: int) -> bool:
    """True when every row of little-endian words, read as an integer, is < limit (vectorised: the most
    significant word where a row differs from the limit decides)."""
    N, W = words.shape
    lw = np.frombuffer(limit.to_bytes(4 * W, "little"), dtype="<u4")
    step = max(1, (1 << 24) // max(W, 1))
    for o in range(0, N, step):
        w = words[o:o + step]
        ne = w != lw
        if not ne.any(axis=1).all():
            return False                                  # a row equal to the limit
        j = W - 1 - np.argmax(ne[:, ::-1], axis=1)
        if not (w[np.arange(w.shape[0]), j] < lw[j]).all():
            return False
    return True


def from_wire(buf, public_key=None, lazy: bool = False):
    """Inverse of to_wire. `public_key` (optional) must match the key in the buffer (ValueError
    otherwise, like encrypted_number.py:169-170); without it a PaillierPublicKey is rebuilt from n.
    lazy=True returns a CiphertextBuffer (cipher_buffer.py): the validated words and exponents, no
    Python object per element."""
    from .keypair import PaillierPublicKey
    mv = memoryview(buf).cast("B")
    bad = ValueError("corrupted ciphertext array")
    if len(mv) < 14 or bytes(mv[:6]) != _WIRE_MAGIC:
        raise ValueError("not a flexpai ciphertext array")
    o = 6
    ndim = int(np.frombuffer(mv, "<u4", 1, o)[0]); o += 4
    if ndim > 32 or len(mv) < o + 8 * ndim + 4:
        raise bad
    shape = tuple(int(v) for v in np.frombuffer(mv, "<i8", ndim, o)); o += 8 * ndim
    nb = int(np.frombuffer(mv, "<u4", 1, o)[0]); o += 4
    if any(v < 0 for v in shape) or nb == 0 or len(mv) < o + nb + 4:
        raise bad
    n = int.from_bytes(mv[o:o + nb], "little"); o += nb
    W = int(np.frombuffer(mv, "<u4", 1, o)[0]); o += 4
    if n < 3 or W != (2 * n.bit_length() + 31) // 32:     # the key's ciphertext width, not the sender's word
        raise bad
    N = int(np.prod(shape)) if shape else 1
    if len(mv) != o + N * (4 * W + 5):
        raise ValueError("corrupted ciphertext array (length mismatch)")
    exps = np.frombuffer(mv, "<i4", N, o).astype(np.int32); o += 4 * N
    obf = np.frombuffer(mv, np.uint8, N, o).copy(); o += N
    words = np.frombuffer(mv, "<u4", N * W, o).reshape(N, W).copy(); o += 4 * N * W
    if public_key is None:
        public_key = PaillierPublicKey(n)
    elif public_key.n != n:
        raise ValueError("ciphertext array was encrypted under a different public key")
    if not _rows_below(words, public_key.nsquare):
        raise ValueError("corrupted ciphertext array (ciphertext >= n^2)")
    if lazy:
        from .cipher_buffer import CiphertextBuffer
        return CiphertextBuffer(public_key, words, exps, obf, shape)
    return materialize(public_key, words, exps, shape, obfuscated=obf != 0)


def _from_pickle(buf) -> PaillierArray:
    """Unpickling hook of PaillierArray (see the module docstring)."""
    return from_wire(buf)
