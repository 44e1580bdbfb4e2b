"""apply_obfuscation — same signature as flex/crypto/paillier/obfuscator.py:23-37.

c * r^n mod n^2. The modular exponentiation r^n mod n^2 (~99 % of the reference's encryption
time) runs on the GPU: it is the device encryption of the integer 0 (c0 = 1) with obfuscator r
(given) or with a fresh device-CSPRNG r (random_value None)."""
import numpy as np

from . import _bigint as gmpy_math


def obfuscator_power(pub_key, random_value: int = None) -> int:
    """r^n mod n^2 computed on the GPU."""
    from . import _native, _runtime
    ctx = _runtime.context(pub_key)
    zero = np.zeros(1, dtype=np.int64)
    if random_value:
        ct, _, _ = ctx.encrypt(zero, obf_mode=_native.PAI_OBF_GIVEN, r_scalar=int(random_value) % pub_key.nsquare)
    else:
        ct, _, _ = ctx.encrypt(zero, obf_mode=_native.PAI_OBF_RNG)
    return _native.words_to_ints(ct)[0]


def apply_obfuscation(ciphertext: int, pub_key, random_value: int = None) -> int:
    if random_value == 1:
        return gmpy_math.mulmod(ciphertext, 1, pub_key.nsquare)     # gmpy_math.powmod(1, ...) == 1
    obfuscator = obfuscator_power(pub_key, random_value)
    return gmpy_math.mulmod(ciphertext, obfuscator, pub_key.nsquare)
