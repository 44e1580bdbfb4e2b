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


@pytest.mark.parametrize("pbits", [1024, 2048])
def test_split_sampler_radix_fold(pbits):
    """k_sgp (kernels_sgp.hpp): the factored rows hold T R mod p^2 with R = 2^(28*76) (built by the pair-group
    engine) while the split CIOS runs at R' = 2^(28*74). Modelled at the limb level for the products (pair_mul with
    the row (a, 0), S = 74) and exactly for the rest: start (C_A, C_B + gamma C_A), C = 2^(-56 K) mod p^2, the b sum
    of the b R words, z = REDC'(A bs) 2^-56 by two zero-digit REDC steps. The result is c0 prod_k T_k mod p^2 with
    A < 2p and B < 4p (what k_fbgp_w / k_pe_fin take)."""
    rng = random.Random(pbits + 3)
    S, ST = 74, 76
    R, Rt = 1 << (PM.LB * S), 1 << (PM.LB * ST)
    for trial in range(3):
        p = rng.getrandbits(pbits) | (1 << (pbits - 1)) | 1
        while any(p % q == 0 for q in (3, 5, 7, 11, 13)):
            p += 2
        p2 = p * p
        K = 5 + trial
        rows, want = [], 1
        for _ in range(K):
            T = rng.randrange(1, p2)
            while T % p == 0:
                T = rng.randrange(1, p2)
            want = want * T % p2
            Tp = T * Rt % p2
            a = Tp % p
            b = (Tp // p) * pow(a, -1, p) % p
            rows.append((a, b * Rt % p))
        M = rng.getrandbits(62) * rng.choice((1, -1))
        want = want * (1 + p * M) % p2                        # c0 = (1, gamma), gamma = M (the public sampler's w = 1)
        C = pow(pow(2, 56 * K, p2), -1, p2)
        ca, cb = C % p, C // p
        nmc = [(1 << (16 * c)) * ca % p for c in range(4)]
        mag = abs(M)
        xs = sum(nmc[c] * ((mag >> (16 * c)) & 0xFFFF) for c in range(4))
        B = cb + ((p << 20) - xs if M < 0 else xs)
        A = ca
        assert B < (1 << 21) * p
        for a, _ in rows:
            Al, Bl = PM.pair_mul(PM.limbs(A, S), PM.limbs(B, S), PM.limbs(a, S), [0] * S, p, S)
            A, B = PM.val(Al), PM.val(Bl)
            assert A < 2 * p and B < 2 * p
        bs = sum(br for _, br in rows)
        mp = pow(-p, -1, R)
        z1 = (A * bs + (A * bs * mp % R) * p) // R            # REDC'(A bs R)
        assert z1 < 2 * p
        z = (z1 + (z1 * pow(-p, -1, 1 << 56) % (1 << 56)) * p) >> 56   # two zero-digit steps: 2^-56
        assert z < 2 * p
        B += z
        assert A < 2 * p and B < 4 * p
        assert (A + p * B) % p2 == want
