"""raw_encrypt — same signature and errors as flex/crypto/paillier/raw_encrypt.py:22-49.
c0 = 1 + n*m mod n^2 (the reference's inverse branch yields the same value); the obfuscation
r^n mod n^2 runs on the GPU (obfuscator.py)."""
from .keypair import PaillierPublicKey
from .obfuscator import apply_obfuscation


def raw_encrypt(plaintext: int, pub_key: PaillierPublicKey, random_value: int = None) -> int:
    if not isinstance(plaintext, int):
        raise TypeError("plaintext should be int, but got: %s" % type(plaintext))
    ciphertext = (pub_key.n * plaintext + 1) % pub_key.nsquare
    return apply_obfuscation(ciphertext, pub_key, random_value)
