"""The p-adic pair product mod p^2 (ibond-flex_amd/csrc/bn_pair.hpp, used by k_fbp, k_dec_*_pair and
k_crt_b_pair): a limb-level model of the kernel's two lock-step CIOS rows (tools/pair_model.py) checked
against plain modular arithmetic, including the accumulator bounds the kernels rely on (the signed second
row stays inside int64, outputs stay < 2p) at worst-case operands. CPU only; the kernels themselves are
checked bit-exactly through the C ABI by the -m gpu suite."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import pair_model as PM  # noqa: E402


@pytest.mark.parametrize("pbits,S", [(512, 19), (1024, 37)])
def test_pair_product_and_square_match_montgomery_mod_p2(pbits, S):
    rng = random.Random(pbits)
    R = 1 << (PM.LB * S)
    for _ in range(40):
        p = rng.getrandbits(pbits) | (1 << (pbits - 1)) | 1
        p2 = p * p
        Rinv = pow(R, -1, p2)
        cases = [(rng.randrange(2 * p), rng.randrange(2 * p), rng.randrange(p), rng.randrange(p)),
                 (2 * p - 1, 2 * p - 1, p - 1, p - 1)]             # the bound's worst case
        for A1, B1, A2, B2 in cases:
            U, Bn = PM.pair_mul(PM.limbs(A1, S), PM.limbs(B1, S), PM.limbs(A2, S), PM.limbs(B2, S), p, S)
            U, Bn = PM.val(U), PM.val(Bn)
            assert U < 2 * p and Bn < 2 * p
            assert (U + p * Bn) % p2 == (A1 + p * B1) * (A2 + p * B2) * Rinv % p2
            U, Bn = PM.pair_mul(PM.limbs(A1, S), PM.limbs(B1, S), PM.limbs(A1, S), PM.limbs(B1, S), p, S, sqr=True)
            U, Bn = PM.val(U), PM.val(Bn)
            assert U < 2 * p and Bn < 2 * p
            assert (U + p * Bn) % p2 == pow(A1 + p * B1, 2, p2) * Rinv % p2


def test_first_fixed_base_product_takes_the_unreduced_c0_pair():
    """k_fbp's accumulator starts at (1, B0) with B0 an unreduced chunk sum < 2^11 p (kernels_fbp.hpp)."""
    rng = random.Random(7)
    S, pbits = 37, 1024
    R = 1 << (PM.LB * S)
    for _ in range(40):
        p = rng.getrandbits(pbits) | (1 << (pbits - 1)) | 1
        B0 = (1 << 11) * p - 1 - rng.randrange(p)
        A2, B2 = p - 1 - rng.randrange(8), p - 1 - rng.randrange(8)
        U, Bn = PM.pair_mul(PM.limbs(1, S), PM.limbs(B0, S), PM.limbs(A2, S), PM.limbs(B2, S), p, S)
        U, Bn = PM.val(U), PM.val(Bn)
        assert U < 2 * p and Bn < 2 * p
        assert (U + p * Bn) % (p * p) == (1 + p * B0) * (A2 + p * B2) * pow(R, -1, p * p) % (p * p)
