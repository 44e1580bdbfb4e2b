"""PaillierEncryptedNumber — same class path, __slots__ and pickle layout as
flex/crypto/paillier/encrypted_number.py:26-185, so objects round-trip through pickle between
this engine and unmodified FLEX peers (ionic_bond ships them pickled).

Scalar object operators compute with Python ints on the host, exactly as the reference does
through gmpy_math; whole-array operations go to the GPU (cipher_array.PaillierArray)."""
from typing import Union

from . import _bigint as gmpy_math
from .fixedpoint_number import FixedPointNumber
from .obfuscator import apply_obfuscation
from .raw_encrypt import raw_encrypt


class PaillierEncryptedNumber(object):
    __slots__ = ('public_key', 'exponent', '__ciphertext', '__is_obfuscator')

    def __init__(self, public_key, ciphertext: int, exponent: int = 0):
        self.public_key = public_key
        self.__ciphertext = ciphertext
        self.exponent = exponent
        self.__is_obfuscator = False

    def ciphertext(self, be_secure: bool = True) -> int:
        """encrypted_number.py:50-56"""
        if be_secure and not self.__is_obfuscator:
            self.apply_obfuscation()
        return self.__ciphertext

    def apply_obfuscation(self) -> None:
        """encrypted_number.py:58-63 (fresh r^n from the device CSPRNG)"""
        self.__ciphertext = apply_obfuscation(self.__ciphertext, self.public_key)
        self.__is_obfuscator = True

    # fast construction used by the array paths (no per-object __init__ dispatch)
    @classmethod
    def _make(cls, public_key, ciphertext: int, exponent: int, obfuscated: bool):
        obj = cls.__new__(cls)
        obj.public_key = public_key
        obj.__ciphertext = ciphertext
        obj.exponent = exponent
        obj.__is_obfuscator = obfuscated
        return obj

    def _is_obfuscated(self) -> bool:
        return self.__is_obfuscator

    def __add__(self, other):
        if isinstance(other, __class__):
            return self.__add_encryptednumber(other)
        return self.__add_scalar(other)

    def __radd__(self, other):
        return self.__add__(other)

    def __sub__(self, other):
        return self + (other * -1)

    def __rsub__(self, other):
        return other + (self * -1)

    def __rmul__(self, scalar):
        return self.__mul__(scalar)

    def __truediv__(self, scalar):
        return self.__mul__(1 / scalar)

    def __mul__(self, scalar: Union[int, float]):
        """encrypted_number.py:86-113"""
        if isinstance(scalar, PaillierEncryptedNumber):
            raise ValueError("PaillierEncryptedNumber * PaillierEncryptedNumber is not allowed.")
        encode = FixedPointNumber.encode(scalar, self.public_key.n, self.public_key.max_int)
        plaintext = encode.encoding
        if plaintext < 0 or plaintext >= self.public_key.n:
            raise ValueError("Scalar out of bounds: %i" % plaintext)
        # (c^-1)^(n - plaintext) for the "very large" plaintexts, c^plaintext otherwise; scalar_pow shares the
        # squarings of a ciphertext multiplied by several scalars (enc.dot(features))
        if plaintext >= self.public_key.n - self.public_key.max_int:
            ciphertext = gmpy_math.scalar_pow(self.ciphertext(False), self.public_key.n - plaintext,
                                              self.public_key.nsquare, True)
        else:
            ciphertext = gmpy_math.scalar_pow(self.ciphertext(False), plaintext, self.public_key.nsquare)
        exponent = self.exponent + encode.exponent
        return PaillierEncryptedNumber(self.public_key, ciphertext, exponent)

    def _increase_exponent_to(self, new_exponent: int):
        """encrypted_number.py:115-127"""
        if new_exponent < self.exponent:
            raise ValueError("New exponent %i should be great than old exponent %i" % (new_exponent, self.exponent))
        factor = pow(FixedPointNumber.BASE, new_exponent - self.exponent)
        if factor <= self.public_key.max_int:
            # __mul__(factor) for an int factor in range: encode gives (factor, exponent 0), so it is
            # c^factor mod n^2 (encrypted_number.py:107-109); out-of-range factors take __mul__ and raise
            c = gmpy_math.powmod(self.ciphertext(False), factor, self.public_key.nsquare)
            return PaillierEncryptedNumber(self.public_key, c, new_exponent)
        new_encryptednumber = self.__mul__(factor)
        new_encryptednumber.exponent = new_exponent
        return new_encryptednumber

    def _align_exponent(self, x, y):
        """encrypted_number.py:129-137"""
        if x.exponent < y.exponent:
            x = x._increase_exponent_to(y.exponent)
        elif x.exponent > y.exponent:
            y = y._increase_exponent_to(x.exponent)
        return x, y

    def __add_scalar(self, scalar):
        """encrypted_number.py:139-146"""
        encoded = FixedPointNumber.encode(scalar, self.public_key.n, self.public_key.max_int,
                                          max_exponent=self.exponent)
        return self.__add_fixpointnumber(encoded)

    def __add_fixpointnumber(self, encoded):
        """encrypted_number.py:148-164"""
        if self.public_key.n != encoded.n:
            raise ValueError("Attempted to add numbers encoded against different public keys!")
        x, y = self._align_exponent(self, encoded)
        encrypted_scalar = raw_encrypt(y.encoding, x.public_key, 1)
        return self.__raw_add(x.ciphertext(False), encrypted_scalar, x.exponent)

    def __add_encryptednumber(self, other):
        """encrypted_number.py:166-178"""
        if self.public_key != other.public_key:
            raise ValueError("add two numbers have different public key!")
        x, y = self._align_exponent(self, other)
        return self.__raw_add(x.ciphertext(False), y.ciphertext(False), x.exponent)

    def __raw_add(self, e_x, e_y, exponent):
        """encrypted_number.py:180-185"""
        ciphertext = gmpy_math.mulmod(e_x, e_y, self.public_key.nsquare)
        return PaillierEncryptedNumber(self.public_key, ciphertext, exponent)
