#  Portions of this file (the seeded key-generation loop of generate_paillier_keypair and the classes' slot
#  lists) follow flex/crypto/paillier/keypair.py of iBond-flex so that seeded keys and pickles match it bit
#  for bit: Copyright 2020 The FLEX Authors, licensed under the Apache License, Version 2.0
#  (http://www.apache.org/licenses/LICENSE-2.0). Distributed on an "AS IS" BASIS, WITHOUT WARRANTIES OR
#  CONDITIONS OF ANY KIND, either express or implied.
"""Paillier keys — same classes, slots and behaviour as flex/crypto/paillier/keypair.py:20-127.

Key generation is host-side and one-time; the seeded path reproduces the
reference's keys (random.seed + getrandbits + next_prime), checked against golden vectors."""
from . import _bigint as gmpy_math


class PaillierPublicKey(object):
    """keypair.py:20-39"""
    __slots__ = ['g', 'n', 'nsquare', 'max_int']

    def __init__(self, n):
        self.g = n + 1
        self.n = n
        self.nsquare = gmpy_math.mul(n, n)
        self.max_int = n // 3 - 1

    def __repr__(self):
        hashcode = hex(hash(self))[2:]
        return "<PaillierPublicKey {}>".format(hashcode[:10])

    def __eq__(self, other):
        return self.n == other.n

    def __hash__(self):
        return hash(self.n)


class PaillierPrivateKey(object):
    """keypair.py:42-90"""
    __slots__ = ['public_key', 'p', 'q', 'psquare', 'qsquare', 'q_inverse', 'hp', 'hq']

    def __init__(self, public_key, p, q):
        if not gmpy_math.mul(p, q) == public_key.n:
            raise ValueError("given public key does not match the given p and q")
        if p == q:
            raise ValueError("p and q have to be different")
        self.public_key = public_key
        if q < p:
            self.p, self.q = q, p
        else:
            self.p, self.q = p, q
        self.psquare = gmpy_math.mul(self.p, self.p)
        self.qsquare = gmpy_math.mul(self.q, self.q)
        self.q_inverse = gmpy_math.invert(self.q, self.p)
        self.hp = self._h_func(self.p, self.psquare)
        self.hq = self._h_func(self.q, self.qsquare)

    def __eq__(self, other):
        return self.p == other.p and self.q == other.q

    def __hash__(self):
        return hash((self.p, self.q))

    def __repr__(self):
        hashcode = hex(hash(self))[2:]
        return "<PaillierPrivateKey {}>".format(hashcode[:10])

    def _h_func(self, x, xsquare):
        # keypair.py:81-90; g^(x-1) mod x^2 = 1 + (x-1) n mod x^2 for g = n + 1
        gx = (1 + (x - 1) * self.public_key.n) % xsquare
        return gmpy_math.invert((gx - 1) // x, x)


def generate_paillier_keypair(n_length: int = 1024, seed: int = None):
    """keypair.py:93-127: returns (PaillierPublicKey, PaillierPrivateKey)."""
    p = q = n = None
    n_len = 0
    i = 1
    while n_len != n_length:
        if seed:
            p = gmpy_math.getprimeover(n_length // 2, seed)
        else:
            p = gmpy_math.getprimeover(n_length // 2)
        q = p
        while q == p:
            if seed:
                q = gmpy_math.getprimeover(n_length // 2, seed + i)
                i += 1
            else:
                q = gmpy_math.getprimeover(n_length // 2)
        n = gmpy_math.mul(p, q)
        n_len = n.bit_length()
    public_key = PaillierPublicKey(n)
    private_key = PaillierPrivateKey(public_key, p, q)
    return public_key, private_key
