"""GPU parity of the object-free ciphertext path (cipher_buffer.py): encrypt_to_buffer ->
to_wire -> from_wire(lazy) -> add_buffers / * / dot / + plain -> to_wire -> decrypt, with no
PaillierEncryptedNumber built anywhere in the chain, bit-identical to the object path (PaillierArray
operators, themselves pinned to the reference's per-element operators by test_gpu_package.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def keys():
    from flex.crypto.paillier.decryptor import PaillierDecryptor
    from flex.crypto.paillier.encryptor import PaillierEncryptor
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk, sk = generate_paillier_keypair(1024, seed=7)
    return pk, PaillierEncryptor(pk), PaillierDecryptor(pk, sk)


@pytest.fixture
def no_objects(monkeypatch):
    """Any PaillierEncryptedNumber construction inside the block fails the test."""
    from flex.crypto.paillier.encrypted_number import PaillierEncryptedNumber

    def boom(*a, **k):
        raise AssertionError("a PaillierEncryptedNumber was built on the object-free path")
    monkeypatch.setattr(PaillierEncryptedNumber, "_make", classmethod(boom))
    monkeypatch.setattr(PaillierEncryptedNumber, "__init__", boom)
    monkeypatch.setattr("flex.crypto.paillier.cipher_array._make_numbers", boom)   # the C bulk constructor


def test_wire_add_chain_without_objects(keys, no_objects):
    from flex.crypto.paillier.cipher_array import from_wire
    from flex.crypto.paillier.cipher_buffer import CiphertextBuffer, add_buffers
    pk, enc, dec = keys
    n = 5000
    xs = [np.random.default_rng(j).standard_normal(n) * 10 ** (j - 1) for j in range(3)]
    wires = [enc.encrypt_to_buffer(x).to_wire() for x in xs]              # three parties
    recv = [from_wire(w, pk, lazy=True) for w in wires]                   # the coordinator
    assert all(isinstance(b, CiphertextBuffer) for b in recv)
    total = add_buffers(recv)
    back = from_wire(total.to_wire(), pk, lazy=True)                      # and back to a party
    val = dec.decrypt(back)
    assert np.allclose(val, xs[0] + xs[1] + xs[2], rtol=1e-12, atol=1e-9)
    assert np.array_equal(back.words, total.words) and not back.obfuscated.any()


def test_buffer_ops_bit_identical_to_object_path(keys):
    from flex.crypto.paillier.cipher_array import pack, to_wire
    from flex.crypto.paillier.cipher_buffer import add_buffers
    pk, enc, dec = keys
    n = 333
    x = np.random.default_rng(3).standard_normal(n).astype(np.float32)    # float32: exact round trip
    b1 = enc.encrypt_to_buffer(x)
    b2 = enc.encrypt_to_buffer(x[::-1].copy() * 100)
    a1, a2 = b1.to_array(), b2.to_array()
    assert np.array_equal(dec.decrypt(b1), x.astype(np.float64))
    assert np.array_equal(dec.decrypt(a1), x.astype(np.float64))

    def same(buf, arr):
        words, exps, _ = pack(arr, pk)
        return np.array_equal(buf.words, words) and np.array_equal(buf.exps, exps)
    assert same(add_buffers([b1, b2]), a1 + a2)
    assert same(b1 + b2, a1 + a2)
    assert same(b1 * 0.5, a1 * 0.5)
    assert same(b1 * -3, a1 * -3)
    y = np.random.default_rng(4).standard_normal(n)
    assert same(b1 + y, a1 + y)
    assert same(b1 - 2.5, a1 - 2.5)
    # E(x) - E(y) = E(x) + E(y) * -1 (encrypted_number.py:74-75) against numpy's per-object loop
    assert same(b1 - b2, np.asarray(a1) - np.asarray(a2))
    assert same(b1 - a2[7], np.asarray(a1) - a2[7])
    m = np.random.default_rng(5).standard_normal((n, 3))
    d_buf, d_arr = b1.dot(m), a1.dot(m)
    assert d_buf.shape == (3,) and same(d_buf, d_arr)
    assert np.allclose(dec.decrypt(d_buf), x.astype(np.float64) @ m, rtol=1e-9, atol=1e-9)
    # to_wire of a buffer equals to_wire of the array it materialises to
    s = b1 + b2
    assert s.to_wire() == to_wire(s.to_array())


def test_buffer_2048_large_through_host_pipeline():
    """2048-bit, 300k elements: encrypt_to_buffer, 2 x wire, k-way add, decrypt (chunked host transfers)."""
    from flex.crypto.paillier.cipher_array import from_wire
    from flex.crypto.paillier.cipher_buffer import add_buffers
    from flex.crypto.paillier.decryptor import PaillierDecryptor
    from flex.crypto.paillier.encryptor import PaillierEncryptor
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    pk, sk = generate_paillier_keypair(2048, seed=11)
    enc, dec = PaillierEncryptor(pk), PaillierDecryptor(pk, sk)
    n = 300_000
    xs = [np.random.default_rng(20 + j).standard_normal(n).astype(np.float32) for j in range(4)]
    bufs = [from_wire(enc.encrypt_to_buffer(x).to_wire(), pk, lazy=True) for x in xs]
    total = add_buffers(bufs)
    val = dec.decrypt(from_wire(total.to_wire(), pk, lazy=True))
    want = sum(x.astype(np.float64) for x in xs)
    assert np.allclose(val, want, rtol=1e-12, atol=1e-12)
