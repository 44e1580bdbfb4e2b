"""PaillierEncryptor — same API as flex/crypto/paillier/encryptor.py:32-114.

Arrays are encrypted in ONE fused GPU launch (encode -> c0 = 1 + n*m -> c0 * r^n mod n^2) instead
of the reference's per-element gmpy2 powmods in a fork pool (encryptor.py:71-97). The encryptor
pickles as {'pub_key': ...} like the reference; the GPU context is per process and lazy."""
from __future__ import annotations

import math
from typing import Union

import numpy as np

from .encrypted_number import PaillierEncryptedNumber
from .fixedpoint_number import FixedPointNumber
from .keypair import PaillierPublicKey
from .raw_encrypt import raw_encrypt

_FLOAT_DT = (np.float16, np.float32, np.float64)
_INT_DT = (np.int16, np.int32, np.int64)


def _device_input(flat: np.ndarray):
    """Map an array onto a device input dtype following fixedpoint_number.py:63-77's type rules.
    Returns (array, None) or (None, offending_type)."""
    dt = flat.dtype
    if dt == np.float32 or dt == np.float16:
        return flat.astype(np.float32), None
    if dt == np.float64:
        return flat, None
    if dt in (np.dtype(np.int16), np.dtype(np.int32), np.dtype(np.int64)):
        return flat.astype(np.int64), None
    if dt == object:
        vals = list(flat)
        if all(type(v) is float or isinstance(v, np.float64) for v in vals):
            return np.array(vals, dtype=np.float64), None
        if all(isinstance(v, (np.float32, np.float16)) for v in vals):
            return np.array(vals, dtype=np.float32), None
        if all((type(v) is int and -(1 << 63) <= v < (1 << 63)) or isinstance(v, _INT_DT) for v in vals):
            return np.array(vals, dtype=np.int64), None
        return None, "mixed"
    return None, type(flat.reshape(-1)[0]) if flat.size else dt.type


class PaillierEncryptor(object):
    def __init__(self, pub_key: PaillierPublicKey):
        self.pub_key = pub_key

    def __raw_encrypt(self, plaintext: int, random_value: int = None) -> int:
        return raw_encrypt(plaintext, self.pub_key, random_value)

    def _encrypt(self, value: Union[int, float], precision: int = None,
                 random_value: int = None) -> PaillierEncryptedNumber:
        """encryptor.py:48-69 for one value (c0 on the host, r^n on the GPU)."""
        encoding = FixedPointNumber.encode(value, self.pub_key.n, self.pub_key.max_int, precision)
        obfuscator = random_value or 1
        ciphertext = self.__raw_encrypt(encoding.encoding, random_value=obfuscator)
        encryptednumber = PaillierEncryptedNumber(self.pub_key, ciphertext, encoding.exponent)
        if random_value is None:
            encryptednumber.apply_obfuscation()
        return encryptednumber

    def _encrypt_numpy(self, values_numpy: np.ndarray, precision: int = None, random_value: int = None) -> np.ndarray:
        """encryptor.py:71-97, one batched GPU launch."""
        from . import _native, _runtime
        from .cipher_array import PaillierArray, materialize
        s = values_numpy.shape
        flat = values_numpy.reshape(-1)
        if flat.size == 0:
            return PaillierArray(np.array([], dtype=object).reshape(s))
        x, bad = _device_input(flat)
        if x is None:
            # mixed object arrays and non-numeric dtypes: per-element semantics of the reference
            # (raises the same TypeError for unsupported element types)
            el = [self._encrypt(v, precision, random_value) for v in flat]
            objs = np.empty(len(el), dtype=object)
            objs[:] = el
            return PaillierArray(objs.reshape(s))
        exp_mode, fixed_exp = _native.PAI_EXP_AUTO, 0
        if precision is not None:
            exp_mode, fixed_exp = _native.PAI_EXP_FIXED, math.floor(math.log(precision, FixedPointNumber.BASE))
        ctx = _runtime.context(self.pub_key)
        if random_value is None:
            ct, ex, st = ctx.encrypt(x, exp_mode, fixed_exp, _native.PAI_OBF_RNG)
            obfuscated = True
        elif random_value:
            ct, ex, st = ctx.encrypt(x, exp_mode, fixed_exp, _native.PAI_OBF_GIVEN,
                                     r_scalar=int(random_value) % self.pub_key.nsquare)
            obfuscated = False
        else:
            ct, ex, st = ctx.encrypt(x, exp_mode, fixed_exp, _native.PAI_OBF_NONE)
            obfuscated = False
        out = materialize(self.pub_key, ct, ex, s, obfuscated)
        bad_idx = np.nonzero(st != _native.EL_OK)[0]
        if bad_idx.size:
            # |int_fixpoint| beyond the device's 64-bit fixed-point range: encode exactly on the host
            # (raises the reference's ValueError when out of range), obfuscate on the GPU.
            objs = np.asarray(out).reshape(-1)
            for i in bad_idx:
                objs[i] = self._encrypt(flat[i], precision, random_value)
            out = PaillierArray(objs.reshape(s))
        return out

    def encrypt_to_buffer(self, values: np.ndarray, precision: int = None):
        """Encrypt an array into a CiphertextBuffer (cipher_buffer.py): the device words, exponents and
        obfuscation flags, no PaillierEncryptedNumber per element. Same ciphertext distribution as
        encrypt(values); for callers that ship (to_wire) or sum ciphertexts without touching them."""
        from . import _native, _runtime
        from .cipher_buffer import CiphertextBuffer
        values = np.asarray(values)
        s = values.shape
        x, _ = _device_input(values.reshape(-1))
        if x is None:
            raise TypeError(f"encrypt_to_buffer: unsupported input dtype {values.dtype}")
        exp_mode, fixed_exp = _native.PAI_EXP_AUTO, 0
        if precision is not None:
            exp_mode, fixed_exp = _native.PAI_EXP_FIXED, math.floor(math.log(precision, FixedPointNumber.BASE))
        ctx = _runtime.context(self.pub_key)
        ct, ex, st = ctx.encrypt(x, exp_mode, fixed_exp, _native.PAI_OBF_RNG)
        bad_idx = np.nonzero(st != _native.EL_OK)[0]
        if bad_idx.size:
            # beyond the device's 64-bit fixed-point range: the host encoder (raises like the reference)
            ct = ct.copy()
            ex = ex.copy()
            for i in bad_idx.tolist():
                e = self._encrypt(values.reshape(-1)[i], precision)
                ct[i] = _runtime.ints_to_words([e.ciphertext(False)], ct.shape[1])[0]
                ex[i] = e.exponent
        return CiphertextBuffer(self.pub_key, ct, ex, 1, s)

    def encrypt(self, value, precision: int = None, random_value: int = None):
        """encryptor.py:99-114"""
        if isinstance(value, np.ndarray):
            return self._encrypt_numpy(value, precision, random_value)
        return self._encrypt(value, precision, random_value)
