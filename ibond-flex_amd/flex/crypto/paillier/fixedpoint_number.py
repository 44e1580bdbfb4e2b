"""FixedPointNumber — same API as flex/crypto/paillier/fixedpoint_number.py:25-270.

Arrays are encoded on the GPU (inside the encrypt kernel); this class serves the scalar
object operators. Semantics follow numpy 1.x (exact scaling), which is what the
reference pins (requirements.txt:1)."""
import math
import sys

import numpy as np

from . import _bigint as gmpy_math


def _scaled_round(scalar, exponent: int) -> int:
    """int(round(scalar * 16**exponent)) evaluated exactly (fixedpoint_number.py:84)."""
    if isinstance(scalar, (int, np.integer)):
        if exponent >= 0:
            return int(scalar) * 16 ** exponent
        return int(round(int(scalar) * pow(16, exponent)))
    fr = float(scalar)
    # numpy 1.x multiplies floats in double (float32/float16 promote): a product that is not a finite
    # double ends in OverflowError (round(inf), or int -> float of 16^E >= 2^1024)
    if exponent >= 256 or (fr != 0.0 and math.frexp(fr)[1] + 4 * exponent > 1024):
        raise OverflowError("cannot convert float infinity to integer")
    if exponent >= 0:
        num, den = fr.as_integer_ratio()
        num <<= 4 * exponent
        q, r = divmod(num, den)
        if 2 * r > den or (2 * r == den and q & 1):
            q += 1
        return q
    return int(round(fr * pow(16, exponent)))


class FixedPointNumber(object):
    BASE = 16
    LOG2_BASE = math.log(BASE, 2)
    FLOAT_MANTISSA_BITS = sys.float_info.mant_dig
    Q = 293973345475167247070445277780365744413

    def __init__(self, encoding, exponent, n=None, max_int=None):
        self.n = n
        if self.n is None:
            self.n = self.Q
            self.max_int = self.Q // 3 - 1
        else:
            self.max_int = max_int
        self.encoding = encoding
        self.exponent = exponent

    @classmethod
    def encode(cls, scalar, n=None, max_int=None, precision=None, max_exponent=None):
        """fixedpoint_number.py:46-90"""
        if isinstance(scalar, (np.unsignedinteger, np.bool_)):
            raise TypeError("Don't know the precision of type %s." % type(scalar))
        if abs(float(scalar)) < 1e-200:
            scalar = 0
        if n is None:
            n = cls.Q
            max_int = cls.Q // 3 - 1
        if max_int is None:
            max_int = cls.Q // 3 - 1
        if precision is None:
            if isinstance(scalar, (int, np.int16, np.int32, np.int64)):
                exponent = 0
            elif isinstance(scalar, (float, np.float16, np.float32, np.float64)):
                flt_exponent = math.frexp(scalar)[1]
                lsb_exponent = cls.FLOAT_MANTISSA_BITS - flt_exponent
                exponent = math.floor(lsb_exponent / cls.LOG2_BASE)
            else:
                raise TypeError("Don't know the precision of type %s." % type(scalar))
        else:
            exponent = math.floor(math.log(precision, cls.BASE))
        if max_exponent is not None:
            exponent = max(max_exponent, exponent)
        int_fixpoint = _scaled_round(scalar, exponent)
        if abs(int_fixpoint) > max_int:
            raise ValueError('Integer needs to be within +/- %d but got %d' % (max_int, int_fixpoint))
        return cls(int_fixpoint % n, exponent, n, max_int)

    def decode(self):
        """fixedpoint_number.py:92-107"""
        if self.encoding >= self.n:
            raise ValueError('Attempted to decode corrupted number')
        elif self.encoding <= self.max_int:
            mantissa = self.encoding
        elif self.encoding >= self.n - self.max_int:
            mantissa = self.encoding - self.n
        else:
            raise OverflowError('Overflow detected in decode number')
        return mantissa * pow(self.BASE, -self.exponent)

    def increase_exponent_to(self, new_exponent):
        if new_exponent < self.exponent:
            raise ValueError('New exponent %i should be greater than'
                             'old exponent %i' % (new_exponent, self.exponent))
        factor = pow(self.BASE, new_exponent - self.exponent)
        new_encoding = gmpy_math.mulmod(self.encoding, factor, self.n)
        return FixedPointNumber(new_encoding, new_exponent, self.n, self.max_int)

    def _align_exponent(self, x, y):
        if x.exponent < y.exponent:
            x = x.increase_exponent_to(y.exponent)
        elif x.exponent > y.exponent:
            y = y.increase_exponent_to(x.exponent)
        return x, y

    def _truncate(self, a):
        return FixedPointNumber.encode(a.decode())

    def __add__(self, other):
        if isinstance(other, FixedPointNumber):
            return self._add_fixpointnumber(other)
        return self._add_fixpointnumber(self.encode(other))

    def __radd__(self, other):
        return self.__add__(other)

    def __sub__(self, other):
        scalar = -1 * (other.decode() if isinstance(other, FixedPointNumber) else other)
        return self._add_fixpointnumber(self.encode(scalar))

    def __rsub__(self, other):
        x = self.__sub__(other)
        return self.encode(-1 * x.decode())

    def __rmul__(self, other):
        return self.__mul__(other)

    def __mul__(self, other):
        if not isinstance(other, FixedPointNumber):
            other = self.encode(other)
        # fixedpoint_number.py:261-266 squares self (reference quirk) — kept
        encoding = gmpy_math.mulmod(self.encoding, self.encoding, self.Q)
        return self._truncate(FixedPointNumber(encoding, self.exponent + other.exponent))

    def __truediv__(self, other):
        scalar = other.decode() if isinstance(other, FixedPointNumber) else other
        return self.__mul__(1 / scalar)

    def __rtruediv__(self, other):
        return FixedPointNumber.encode(1.0 / self.__truediv__(other).decode())

    def _cmp_value(self, other):
        return other.decode() if isinstance(other, FixedPointNumber) else other

    def __lt__(self, other):
        return self.decode() < self._cmp_value(other)

    def __gt__(self, other):
        return self.decode() > self._cmp_value(other)

    def __le__(self, other):
        return self.decode() <= self._cmp_value(other)

    def __ge__(self, other):
        return self.decode() >= self._cmp_value(other)

    def __eq__(self, other):
        return self.decode() == self._cmp_value(other)

    def __ne__(self, other):
        return self.decode() != self._cmp_value(other)

    def _add_fixpointnumber(self, other):
        x, y = self._align_exponent(self, other)
        encoding = (x.encoding + y.encoding) % self.Q
        return FixedPointNumber(encoding, x.exponent)
