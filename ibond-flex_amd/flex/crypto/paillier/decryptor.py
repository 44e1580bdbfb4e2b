"""PaillierDecryptor — same API and errors as flex/crypto/paillier/decryptor.py:28-127.

Arrays decrypt in ONE GPU launch: both CRT half-exponentiations c^(p-1) mod p^2 and
c^(q-1) mod q^2, the L-function, the CRT recombination and the fixed-point decode to float64
run on the device (kernels.hpp k_decrypt)."""
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
        """decryptor.py:91-112, one batched GPU launch."""
        from . import _native, _runtime
        from .cipher_array import pack
        s = encrypted_number_numpy.shape
        flat = np.asarray(encrypted_number_numpy).reshape(-1)
        if flat.size == 0:
            return np.array([]).reshape(s)
        for e in flat:
            self._check(e)
        words, exps, _ = pack(encrypted_number_numpy, self.pub_key)
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
        for i in range(flat.size):
            if st[i] == _native.EL_OK:
                values.append(float(val[i]))
            elif st[i] == _native.EL_INT:
                values.append(int(mant[i]))
            else:   # exact integer too wide for int64: decode the exact plaintext
                values.append(FixedPointNumber(raw[i], int(exps[i]), self.pub_key.n, self.pub_key.max_int).decode())
        return np.array(values).reshape(s)

    def decrypt(self, encrypted_number):
        """decryptor.py:114-127"""
        if isinstance(encrypted_number, np.ndarray):
            return self._decrypt_numpy(encrypted_number)
        return self._decrypt(encrypted_number)
