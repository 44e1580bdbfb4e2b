"""Pin the C/GMP oracle (used for the CPU baseline and large-N sampled parity) to the Python
oracle and, through it, to the reference golden vectors."""
import numpy as np
import pytest

from oracle import gmp_oracle as G
from oracle import paillier_oracle as O

pytestmark = pytest.mark.skipif(not G.available(), reason="oracle/_build/libgmp_oracle.so not built")


def _key(golden, nb):
    k = golden["keys"][str(nb)]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


@pytest.mark.parametrize("nb", [1024, 2048])
def test_gmp_encrypt_matches_python_oracle(golden, nb):
    key = _key(golden, nb)
    rec = golden["encrypt"][str(nb)]
    x = np.array([r["bits"] for r in rec], dtype=np.uint32).view(np.float32)[:24]
    k32 = bytes(range(32))
    ct, ex = G.encrypt_f32_chacha(key.n, x, k32, index_base=77, nthreads=4)
    rb = ((nb + 64 + 31) // 32) * 4
    for i in range(len(x)):
        r = O.device_r(k32, 77 + i, rb) % key.n
        c, e = O.encrypt_value(x[i], key, r)
        got = int.from_bytes(ct[i].tobytes(), "little")
        assert (got, ex[i]) == (c, e)


@pytest.mark.parametrize("nb", [1024, 2048])
def test_gmp_decrypt_golden(golden, nb):
    key = _key(golden, nb)
    rec = golden["encrypt"][str(nb)]
    ctw = (2 * nb) // 32
    cts = np.frombuffer(b"".join(int(r["c"], 16).to_bytes(ctw * 4, "little") for r in rec), dtype=np.uint32)
    pt = G.decrypt_raw(key.p, key.q, cts.reshape(len(rec), ctw), nthreads=4)
    for i, r in enumerate(rec):
        x = int.from_bytes(pt[i].tobytes(), "little")
        assert float(O.decode(x, r["e"], key.n, key.max_int)).hex() == r["dec"]
