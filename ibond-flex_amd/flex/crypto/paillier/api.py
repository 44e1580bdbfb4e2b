#  The three factory signatures below are the boundary contract of flex/crypto/paillier/api.py of iBond-flex, which
#  callers reach unchanged: Copyright 2020 The FLEX Authors, licensed under the Apache License, Version 2.0
#  (http://www.apache.org/licenses/LICENSE-2.0). Distributed on an "AS IS" BASIS, WITHOUT WARRANTIES OR
#  CONDITIONS OF ANY KIND, either express or implied.
"""Factory API — same names and signatures as flex/crypto/paillier/api.py:17-34."""
from .decryptor import PaillierDecryptor
from .encryptor import PaillierEncryptor
from .keypair import PaillierPrivateKey, PaillierPublicKey, generate_paillier_keypair


def generate_paillier_encryptor_decryptor(n_length: int = 1024, seed: int = None):
    public_key, private_key = generate_paillier_keypair(n_length, seed)
    return PaillierEncryptor(public_key), PaillierDecryptor(public_key, private_key)


def generate_paillier_encryptor(n: int) -> PaillierEncryptor:
    return PaillierEncryptor(PaillierPublicKey(n))


def generate_paillier_decryptor(n: int, p: int, q: int) -> PaillierDecryptor:
    public_key = PaillierPublicKey(n)
    private_key = PaillierPrivateKey(public_key, p, q)
    return PaillierDecryptor(public_key, private_key)
