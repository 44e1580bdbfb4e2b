"""The factored 4096-bit decryption chain (kernels_dec4.hpp d4f_run, flexpai.hip build_dec4f_program): a value-level
model (tools/dec4f_model.py) of its B-free window multipliers, the chain over p - 2 whose result is the Fermat
inverse, and the closing Horner sum, checked against c^(p-1) mod p^2 directly -- random ciphertexts and the edge
cases c = 0, c == 0 mod p, 1, n^2 - 1. CPU only; the kernel itself is checked bit-exactly by tests/test_gpu_dec4.py."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import dec4f_model as DM  # noqa: E402


@pytest.mark.parametrize("key,S", [("4096", 74), ("2048", 37)])
def test_factored_chain_matches_direct_power(golden, key, S):
    rnd = random.Random(int(key))
    p, q = int(golden["keys"][key]["p"], 16), int(golden["keys"][key]["q"], 16)
    n2 = (p * q) ** 2
    cs = [rnd.randrange(n2) for _ in range(5)] + [0, p * rnd.randrange(1, q * q), 1, n2 - 1, p * p + 3]
    for c in cs:
        assert DM.run(p, c, S) == pow(c, p - 1, p * p), hex(c)[:24]


def test_k_constants_count_every_multiply(golden):
    """The K_t weights reproduce the exponent: (2 first + 1) 2^(all squares) + sum_t (2t + 1) K_t == p - 2."""
    p = int(golden["keys"]["4096"]["p"], 16)
    e = p - 2
    first, ops = DM.sliding_schedule(e)
    K = [0] * 16
    after = 0
    for nsq, idx in reversed(ops):
        if idx is not None:
            K[idx] += 1 << after
        after += nsq
    assert (2 * first + 1) * (1 << after) + sum((2 * t + 1) * K[t] for t in range(16)) == e
