"""Bulk ciphertext-array wire format (cipher_array.to_wire / from_wire): round trip of
ciphertexts, exponents, obfuscation flags and shape; key checks; pickling a PaillierArray produces, by default, the plain object
ndarray unmodified FLEX peers load, and with FLEXPAI_PICKLE_BULK=1 goes through the wire format (a
PaillierArray comes back). CPU only (no kernel calls)."""
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
    plain = pickle.loads(pickle.dumps(arr))           # default: the reference's object-ndarray pickle
    assert type(plain) is np.ndarray and plain.dtype == object
    monkeypatch.setenv("FLEXPAI_PICKLE_BULK", "1")
    back = pickle.loads(pickle.dumps(arr))
    assert type(back) is type(arr) and back._valid_packed() is not None
    assert [(a.ciphertext(False), a.exponent, a._is_obfuscated()) for a in arr] == \
        [(b.ciphertext(False), b.exponent, b._is_obfuscated()) for b in back]


def test_lazy_from_wire_buffer_round_trip(golden):
    """from_wire(lazy=True) -> CiphertextBuffer: the same words / exponents / flags / shape without objects;
    its to_wire is byte-identical; to_array / from_array convert both ways; ciphertexts >= n^2 and rows
    equal to n^2 are rejected (vectorised check)."""
    from flex.crypto.paillier.cipher_array import from_wire, to_wire
    from flex.crypto.paillier.cipher_buffer import CiphertextBuffer
    arr, pk = _array(golden, (3, 4))
    buf = to_wire(arr)
    cb = from_wire(buf, pk, lazy=True)
    assert isinstance(cb, CiphertextBuffer) and cb.shape == (3, 4) and cb.size == 12
    assert cb.to_wire() == buf and to_wire(cb) == buf
    assert CiphertextBuffer.from_array(arr).to_wire() == buf
    back = cb.to_array()
    assert back.shape == arr.shape
    for a, b in zip(np.asarray(arr).reshape(-1), np.asarray(back).reshape(-1)):
        assert (a.ciphertext(False), a.exponent, a._is_obfuscated()) == (b.ciphertext(False), b.exponent, b._is_obfuscated())
    assert cb.reshape(12).shape == (12,) and cb.reshape(4, 3).to_wire() != buf
    W = cb.words.shape[1]
    nsq = pk.nsquare
    for bad in (nsq, nsq + 1, (1 << (32 * W)) - 1):
        t = bytearray(buf)
        t[-4 * W:] = bad.to_bytes(4 * W, "little")
        with pytest.raises(ValueError):
            from_wire(bytes(t), lazy=True)
    t = bytearray(buf)
    t[-4 * W:] = (nsq - 1).to_bytes(4 * W, "little")
    assert from_wire(bytes(t), lazy=True).size == 12
    with pytest.raises(ValueError):
        CiphertextBuffer(pk, cb.words[:, :-1], cb.exps)


def test_buffer_operators_need_gpu_without_one(golden, monkeypatch):
    from flex.crypto.paillier import _runtime
    from flex.crypto.paillier.cipher_array import from_wire, to_wire
    arr, pk = _array(golden, (5,))
    cb = from_wire(to_wire(arr), lazy=True)
    monkeypatch.setattr(_runtime, "gpu_available", lambda: False)
    with pytest.raises(RuntimeError):
        cb + cb
    with pytest.raises(ValueError):
        cb * cb
