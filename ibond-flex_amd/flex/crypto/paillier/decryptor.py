"""PaillierDecryptor — same API and errors as flex/crypto/paillier/decryptor.py:28-127.

Arrays decrypt in ONE device call: both CRT half-exponentiations c^(p-1) mod p^2 and c^(q-1) mod q^2,
the L-function, the CRT recombination and the fixed-point decode to float64 run on the GPU -- the
lane-engine kernels k_dec_pre / k_dec_pow / k_dec_fin (kernels_dec.hpp) for 1024- and 2048-bit keys,
the lane-group kernel k_decrypt (kernels.hpp) for larger ones. A CiphertextBuffer (cipher_buffer.py)
decrypts straight from its words, without per-element objects."""
from __future__ import annotations

from typing import Union

import numpy as np

from .encrypted_number import PaillierEncryptedNumber
from .fixedpoint_number import FixedPointNumber
from .keypair import PaillierPrivateKey, PaillierPublicKey


class PaillierDecryptor(object):
    def __init__(self, pub_key: PaillierPublicKey, priv_key: PaillierPrivateKey):
        self.pub_key = pub_key
        self.priv_key = priv_key
        from . import _runtime
        _runtime.register_private(pub_key, priv_key)

    def __setstate__(self, state):
        # unpickled in another process (the reference pickles decryptors into pool workers)
        self.__dict__.update(state)
        from . import _runtime
        _runtime.register_private(self.pub_key, self.priv_key)

    def _check(self, encrypted_number):
        if not isinstance(encrypted_number, PaillierEncryptedNumber):          # decryptor.py:73-75
            raise TypeError("encrypted_number should be an PaillierEncryptedNumber, \
                             not: %s" % type(encrypted_number))
        if self.pub_key != encrypted_number.public_key:                        # decryptor.py:77-79
            raise ValueError("encrypted_number was encrypted against a different key!")

    def _decrypt(self, encrypted_number: PaillierEncryptedNumber) -> Union[int, float]:
        """decryptor.py:65-89"""
        self._check(encrypted_number)
        out = np.array([encrypted_number], dtype=object)
        v = self._decrypt_numpy(out).reshape(-1)[0]
        return v.item() if isinstance(v, np.generic) else v

    def _decrypt_numpy(self, encrypted_number_numpy: np.ndarray) -> np.ndarray:
        """decryptor.py:91-112, one batched GPU launch. The per-element _check and the packing of the
        ciphertexts run as one C pass (cipher_array.pack_checked; a PaillierArray whose packed words are
        still valid only checks); the reference's exceptions come from the per-element path when it fails."""
        from .cipher_array import PaillierArray, pack, pack_checked
        s = encrypted_number_numpy.shape
        flat = np.asarray(encrypted_number_numpy).reshape(-1)
        if flat.size == 0:
            return np.array([]).reshape(s)
        W = (2 * self.pub_key.n.bit_length() + 31) // 32
        cached = encrypted_number_numpy._valid_packed() if isinstance(encrypted_number_numpy, PaillierArray) else None
        if cached is not None and cached.n == self.pub_key.n:
            if pack_checked(flat, self.pub_key, W, want_words=False) is not None:
                return self._decrypt_words(cached.words, cached.exps.astype(np.int32), s)
        else:
            got = pack_checked(flat, self.pub_key, W)
            if got is not None:
                return self._decrypt_words(got[0], got[1], s)
        for e in flat:
            self._check(e)
        words, exps, _ = pack(encrypted_number_numpy, self.pub_key)
        return self._decrypt_words(words, exps, s)

    def _decrypt_words(self, words: np.ndarray, exps: np.ndarray, s) -> np.ndarray:
        from . import _native, _runtime
        ctx = _runtime.context(self.pub_key, self.priv_key)
        val, mant, st, _ = ctx.decrypt(words, exps)
        if np.all(st == _native.EL_OK):
            return val.reshape(s)
        for code, exc, msg in ((_native.EL_OVERFLOW, OverflowError, 'Overflow detected in decode number'),
                               (_native.EL_FLOAT_OVF, OverflowError, 'int too large to convert to float')):
            if np.any(st == code):
                raise exc(msg)
        raw = None
        if np.any(st == _native.EL_INT_BIG):
            _, _, _, raw_words = ctx.decrypt(words, exps, want_raw=True)
            raw = _runtime.words_to_ints(raw_words)
        values = []
        for i in range(exps.size):
            if st[i] == _native.EL_OK:
                values.append(float(val[i]))
            elif st[i] == _native.EL_INT:
                values.append(int(mant[i]))
            else:   # exact integer too wide for int64: decode the exact plaintext
                values.append(FixedPointNumber(raw[i], int(exps[i]), self.pub_key.n, self.pub_key.max_int).decode())
        return np.array(values).reshape(s)

    def decrypt(self, encrypted_number):
        """decryptor.py:114-127 (plus CiphertextBuffer, cipher_buffer.py)"""
        from .cipher_buffer import CiphertextBuffer
        if isinstance(encrypted_number, CiphertextBuffer):
            if encrypted_number.public_key != self.pub_key:
                raise ValueError("encrypted_number was encrypted against a different key!")
            if encrypted_number.size == 0:
                return np.array([]).reshape(encrypted_number.shape)
            return self._decrypt_words(encrypted_number.words, encrypted_number.exps, encrypted_number.shape)
        if isinstance(encrypted_number, np.ndarray):
            return self._decrypt_numpy(encrypted_number)
        return self._decrypt(encrypted_number)
