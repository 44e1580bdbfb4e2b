"""Limb-level model of the p-adic pair arithmetic mod p^2 (bn_pair.hpp), for checking the algebra
and the accumulator bounds on the host before the kernels change. Not test infrastructure for the
product; run directly: python tools/pair_model.py

A number v mod p^2 is held as a pair (A, B), 0 <= A, B < 2p, with v = A + p B (mod p^2). With
R = 2^(28 S) (S limbs of p), the CIOS product A1 A2 = U R - m p (m the q-digits of the reduction), so
  (A1 + p B1)(A2 + p B2) R^-1 = U + p (A1 B2 + A2 B1 - m) R^-1   (mod p^2)
i.e. the Montgomery product mod p^2 (radix R) is (U, REDC_p(A1 B2 + A2 B1 - m)): 5 S^2 MACs at S limbs
instead of 2 (2S)^2 for a Montgomery product over the 2S limbs of p^2.
"""
import random

LB = 28
MASK = (1 << LB) - 1
I64 = 1 << 64


def limbs(x, S):
    return [(x >> (LB * i)) & MASK for i in range(S)]


def val(l):
    return sum(v << (LB * i) for i, v in enumerate(l))


def wrap64(v):
    v &= I64 - 1
    return v - I64 if v >= (1 << 63) else v


def pair_mul(A1, B1, A2, B2, p, S, sqr=False):
    """Lockstep CIOS over j: P1 <- A1 A2 (+ q1 p), P2 <- B1 A2 + A1 B2 - q1 (+ q2 p). As the kernels do
    (bn_pair.hpp red2), q1 is not subtracted: q2 = (P2_J - q1) pinv makes position J equal q1 mod 2^28 and the
    retiring shift drops it, so P2 stays non-negative (unsigned 64-bit accumulators)."""
    pl = limbs(p, S)
    pinv = (-pow(p, -1, 1 << LB)) % (1 << LB)
    P1 = [0] * S
    P2 = [0] * S
    mx1 = mx2 = 0
    for J in range(S):
        a2j, b2j = A2[J], B2[J]
        if sqr:
            P1[(2 * J) % S] += A1[J] * A1[J]
            for i in range(J + 1, S):
                P1[(i + J) % S] += A1[i] * (2 * A1[J])
            for i in range(S):
                P2[(i + J) % S] += A1[i] * (2 * B1[J])
        else:
            for i in range(S):
                P1[(i + J) % S] += A1[i] * a2j
                P2[(i + J) % S] += B1[i] * a2j + A1[i] * b2j
        q1 = ((P1[J] & MASK) * pinv) & MASK
        for i in range(S):
            P1[(i + J) % S] += q1 * pl[i]
        assert P1[J] & MASK == 0
        P1[(J + 1) % S] += P1[J] >> LB
        P1[J] = 0
        q2 = ((((P2[J] & 0xFFFFFFFF) - q1) & 0xFFFFFFFF) * pinv) & MASK
        for i in range(S):
            P2[(i + J) % S] += q2 * pl[i]
        assert P2[J] >= 0 and P2[J] & MASK == q1
        P2[(J + 1) % S] += P2[J] >> LB   # drops q1: the subtraction of m
        P2[J] = 0
        mx1 = max(mx1, max(P1))
        mx2 = max(mx2, max(P2))
    assert mx1 < (1 << 64) and mx2 < (1 << 64), (mx1.bit_length(), mx2.bit_length())

    def norm(P):
        c, r = 0, []
        for v in P:
            v += c
            r.append(v & MASK)
            c = v >> LB
        assert c == 0, c
        return r
    return norm(P1), norm(P2)


def check(pbits, trials=200, seed=1):
    rng = random.Random(seed)
    S = (pbits + 4 + LB - 1) // LB if pbits == 512 else -(-(pbits + 12) // LB)
    S = {512: 19, 1024: 37, 2048: 74}[pbits]
    R = 1 << (LB * S)
    for _ in range(trials):
        p = rng.getrandbits(pbits) | (1 << (pbits - 1)) | 1
        p2 = p * p
        Rinv = pow(R, -1, p2)
        for sqr in (False, True):
            A1, B1 = rng.randrange(2 * p), rng.randrange(2 * p)
            if sqr:
                A2, B2 = A1, B1
            else:
                A2, B2 = rng.randrange(p), rng.randrange(p)
            U, Bn = pair_mul(limbs(A1, S), limbs(B1, S), limbs(A2, S), limbs(B2, S), p, S, sqr)
            U, Bn = val(U), val(Bn)
            assert U < 2 * p and Bn < 2 * p, (U / p, Bn / p)
            want = (A1 + p * B1) * (A2 + p * B2) * Rinv % p2
            assert (U + p * Bn) % p2 == want
        # first product with the unreduced c0 chunk sum as B1 (< 2^10 p)
        A1, B1 = 1, rng.randrange(1 << 10) * p + rng.randrange(p)
        A2, B2 = rng.randrange(p), rng.randrange(p)
        U, Bn = pair_mul(limbs(A1, S), limbs(B1, S), limbs(A2, S), limbs(B2, S), p, S)
        U, Bn = val(U), val(Bn)
        assert U < 2 * p and Bn < 2 * p
        assert (U + p * Bn) % p2 == (A1 + p * B1) * (A2 + p * B2) * Rinv % p2
    print(f"pbits={pbits} S={S}: {trials} x (mul, sqr, c0-first) ok")


if __name__ == "__main__":
    check(512)
    check(1024)
    check(2048, trials=20)
