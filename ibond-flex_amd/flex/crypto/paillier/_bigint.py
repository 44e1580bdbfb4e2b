"""Host-side big-integer helpers for one-time key setup (keygen) and for the scalar object
operators. Restates flex/crypto/gmpy_math.py:27-93 on the package's own GMP binding (_gmp.so,
csrc/hostgmp.c, the library gmpy2 wraps), or on Python ints where that binding is not built.
Array paths never use these: they go to the GPU through _runtime.py."""
from __future__ import annotations

import random

try:
    from . import _gmp
except ImportError:          # not built: same results through Python ints (slower)
    _gmp = None

POWMOD_GMP_SIZE = 1 << 64

_SMALL_PRIMES = [p for p in range(3, 2000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


def mul(a: int, b: int) -> int:                      # gmpy_math.py:27-28
    return a * b


def crt(mp: int, mq: int, p: int, q: int, q_inverse: int, n: int) -> int:   # gmpy_math.py:31-40
    u = (mp - mq) * q_inverse % p
    return (mq + u * q) % n


def mulmod(a: int, b: int, c: int) -> int:           # gmpy_math.py:43-48
    if _gmp is not None and c >= POWMOD_GMP_SIZE:
        return _gmp.mulmod(a, b, c)
    return a * b % c


def powmod(a: int, b: int, c: int) -> int:           # gmpy_math.py:51-63
    if a == 1:
        return 1
    if _gmp is not None and max(a, b, c) >= POWMOD_GMP_SIZE:
        return _gmp.powmod(a, b, c)
    return pow(a, b, c)


def scalar_pow(c: int, k: int, m: int, neg: bool = False) -> int:
    """c^k mod m, or (c^-1)^k mod m when neg -- powmod(c, k, m) / powmod(invert(c, m), k, m) as
    encrypted_number.py:99-109 computes them, for 0 < k < 2^64. On the GMP binding a ciphertext that is
    multiplied again keeps its table of squarings (hostgmp.c scalar_pow): same values, fewer products."""
    if _gmp is not None and m >= POWMOD_GMP_SIZE and 0 <= k < POWMOD_GMP_SIZE:
        return _gmp.scalar_pow(c, k, m, neg)
    return powmod(invert(c, m), k, m) if neg else powmod(c, k, m)


def invert(a: int, b: int) -> int:                   # gmpy_math.py:66-74
    if _gmp is not None:
        return _gmp.invert(a, b)
    try:
        x = pow(a, -1, b)
    except ValueError:
        x = 0
    if x == 0:
        raise ZeroDivisionError('invert(a, b) no inverse exists')
    return x


def is_probable_prime(x: int) -> bool:
    if x < 2:
        return False
    for p in _SMALL_PRIMES:
        if x % p == 0:
            return x == p
    d, s = x - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in _SMALL_PRIMES[:40]:
        y = pow(a, d, x)
        if y == 1 or y == x - 1:
            continue
        for _ in range(s - 1):
            y = y * y % x
            if y == x - 1:
                break
        else:
            return False
    return True


def next_prime(x: int) -> int:
    """gmpy2.next_prime: the smallest (probable) prime strictly greater than x."""
    c = x + 1
    if c <= 2:
        return 2
    if c % 2 == 0:
        c += 1
    while not is_probable_prime(c):
        c += 2
    return c


def getprimeover(n: int, seed=None) -> int:          # gmpy_math.py:77-87
    if not seed:
        r = random.SystemRandom().getrandbits(n)
    else:
        random.seed(seed)
        r = random.getrandbits(n)
    r |= 1 << (n - 1)
    return next_prime(r)


def isqrt(n: int) -> int:                            # gmpy_math.py:90-93
    import math
    return math.isqrt(n)
