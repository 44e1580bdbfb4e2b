"""Bulk ciphertext-array wire format (cipher_array.to_wire / from_wire): round trip of
ciphertexts, exponents, obfuscation flags and shape; key checks; pickling a PaillierArray goes through the
wire format (a PaillierArray comes back), and with FLEXPAI_PICKLE_PLAIN=1 it produces the plain object
ndarray unmodified FLEX peers load. CPU only (no kernel calls)."""
import pickle

import numpy as np
import pytest

from oracle import paillier_oracle as O


def _array(golden, shape, nb=1024):
    from flex.crypto.paillier.cipher_array import PaillierArray
    from flex.crypto.paillier.encrypted_number import PaillierEncryptedNumber
    from flex.crypto.paillier.keypair import PaillierPublicKey
    k = golden["keys"][str(nb)]
    key = O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))
    pk = PaillierPublicKey(key.n)
    cnt = int(np.prod(shape))
    x = np.random.default_rng(cnt).standard_normal(cnt).astype(np.float32)
    el = []
    for i, v in enumerate(x):
        c, e = O.encrypt_value(v, key, O.golden_r(key.n, 31, i))
        el.append(PaillierEncryptedNumber._make(pk, c, e, bool(i % 3)))
    objs = np.empty(cnt, dtype=object)
    objs[:] = el
    return PaillierArray(objs.reshape(shape)), pk


@pytest.mark.parametrize("shape", [(1,), (7,), (3, 5)])
def test_wire_round_trip(golden, shape):
    from flex.crypto.paillier.cipher_array import from_wire, to_wire
    arr, pk = _array(golden, shape)
    buf = to_wire(arr)
    W = 2 * 1024 // 32
    assert len(buf) < arr.size * (4 * W + 5) + 256
    back = from_wire(buf, pk)
    assert back.shape == arr.shape and isinstance(back, np.ndarray)
    for a, b in zip(np.asarray(arr).reshape(-1), np.asarray(back).reshape(-1)):
        assert (a.ciphertext(False), a.exponent, a._is_obfuscated()) == (b.ciphertext(False), b.exponent, b._is_obfuscated())
    assert from_wire(buf).reshape(-1)[0].public_key.n == pk.n


def test_wire_errors_and_pickle(golden, monkeypatch):
    from flex.crypto.paillier.cipher_array import from_wire, to_wire
    from flex.crypto.paillier.keypair import PaillierPublicKey
    arr, pk = _array(golden, (4,))
    buf = to_wire(arr)
    with pytest.raises(ValueError):
        from_wire(buf, PaillierPublicKey(pk.n + 2))
    with pytest.raises(ValueError):
        from_wire(buf[:-1])
    with pytest.raises(ValueError):
        from_wire(b"nonsense" + buf)
    with pytest.raises(TypeError):
        to_wire(np.array([1.0, 2.0]))
    back = pickle.loads(pickle.dumps(arr))
    assert type(back) is type(arr) and back._valid_packed() is not None
    assert [(a.ciphertext(False), a.exponent, a._is_obfuscated()) for a in arr] == \
        [(b.ciphertext(False), b.exponent, b._is_obfuscated()) for b in back]
    monkeypatch.setenv("FLEXPAI_PICKLE_PLAIN", "1")
    plain = pickle.loads(pickle.dumps(arr))
    assert type(plain) is np.ndarray and plain.dtype == object
