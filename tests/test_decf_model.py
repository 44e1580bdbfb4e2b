"""The factored 1024/2048-bit decryption chain (kernels_pair.hpp decf_run, flexpai.hip build_decf_lane_program): the
value-level model (tools/decf_model.py) of its full-pair window table, B-free chain multipliers over p - 2 and closing
Horner sum (slot 1's weight + 1 for the closing (A~, 0)), checked against c^(p-1) mod p^2 directly on the reference's
seeded keys -- random ciphertexts and the edge cases c = 0, c == 0 mod p, 1, n^2 - 1. CPU only; the kernel itself is
checked bit-exactly by the -m gpu decrypt tests (goldens, oracle, edge ciphertexts, the 16M round trip)."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import decf_model as FM  # noqa: E402


@pytest.mark.parametrize("key,S", [("1024", 19), ("2048", 37)])
def test_factored_lane_chain_matches_direct_power(golden, key, S):
    rnd = random.Random(int(key) + 5)
    for p, q in ((int(golden["keys"][key]["p"], 16), int(golden["keys"][key]["q"], 16)),
                 (int(golden["keys"][key]["q"], 16), int(golden["keys"][key]["p"], 16))):
        n2 = (p * q) ** 2
        cs = [rnd.randrange(n2) for _ in range(4)] + [0, p * rnd.randrange(1, q * q), 1, n2 - 1, p * p + 3]
        for c in cs:
            assert FM.run(p, c, S) == pow(c, p - 1, p * p), hex(c)[:24]


def test_slot_one_weight_includes_the_closing_multiply(golden):
    p = int(golden["keys"]["2048"]["p"], 16)
    R = 1 << (28 * 37)
    first, ops, Kp = FM.kconsts(p - 2, p, R)
    K = [0] * 16
    after = 0
    for nsq, idx in reversed(ops):
        if idx is not None:
            K[idx] += 1 << after
        after += nsq
    assert Kp[0] == (K[0] + 1) * R % p and all(Kp[t] == K[t] * R % p for t in range(1, 16))
