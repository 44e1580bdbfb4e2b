"""Limb-level model of the Shoup-form fixed-base sampler (kernels_fbs.hpp) for 28-bit limbs, checking the
algebra, the truncated quotient and every accumulator bound on the host before the kernel changes. Not test
infrastructure for the product; run directly: python tools/shoup_model.py

A table entry T = T_k[d] mod p^2 (plain, not Montgomery form) is stored factored as T = a (1 + p b) with
a = T mod p, together with Shoup's precomputed quotient a' = floor(a R / p), R = 2^(28 S). The running pair
(A, B), V = A + p B (mod p^2), is multiplied by a in two passes per component (A then B):
  step 1: Q = floor(X / R) from the columns >= S - 1 of X = A a' only (the dropped columns are worth < S R,
          so Q is at most S + 1 below floor(A a' / R));
  step 2: r = A a - Q p, computed as the low S limbs (columns 0 .. S-1, signed accumulators: the A a products
          added, the Q p products subtracted), exact because 0 <= r < R.
Shoup: A a / p - A a' / R lies in [0, A / R), so r < (A / R + S + 3) p; the B pass adds the A pass's quotient
(V a = r_A + p (Q_A + B a)), B' = Q_A + B a - Q_B p. With A < ALPHA p, B < BETA p both stay bounded.
MACs per product: 2 (S (S+1) / 2 + S (S+1)) = 3 S^2 + 3 S against 4 S^2 for the Montgomery pair product by
(a, 0) (kernels_fbp.hpp).
"""
import random

LB = 28
MASK = (1 << LB) - 1
I64 = 1 << 64


def limbs(x, S):
    return [(x >> (LB * i)) & MASK for i in range(S)]


def val(l):
    return sum(v << (LB * i) for i, v in enumerate(l))


class Stats:
    def __init__(self):
        self.acc1 = self.acc2 = 0
        self.alpha = self.beta = 0.0
        self.qerr = 0


def shoup_pass(X, a, ap, p, S, init, st):
    """One component: Q from the columns >= S-1 of X a' (unsigned), r = (init + X a - Q p) mod R from the
    columns 0..S-1 (signed). Returns (r, Q)."""
    Xl, al, apl, pl = limbs(X, S), limbs(a, S), limbs(ap, S), limbs(p, S)
    # step 1: columns k >= S - 1 of X a' (digits j descending, i >= S - 1 - j)
    P1 = [0] * (2 * S)
    for j in range(S - 1, -1, -1):
        for i in range(max(0, S - 1 - j), S):
            P1[i + j] += Xl[i] * apl[j]
            assert P1[i + j] < I64
    st.acc1 = max(st.acc1, max(P1))
    c = 0
    Ql = []
    for k in range(S - 1, 2 * S):
        v = P1[k] + c
        if k >= S:
            Ql.append(v & MASK)
        c = v >> LB
    assert c == 0
    Q = val(Ql)
    st.qerr = max(st.qerr, (X * ap) // (1 << (LB * S)) - Q)
    assert 0 <= (X * ap) // (1 << (LB * S)) - Q <= S + 1
    # step 2: columns 0..S-1 of init + X a - Q p (signed 64-bit accumulators)
    P2 = [0] * S
    il = limbs(init, S)
    for k in range(S):
        P2[k] = il[k]
    Qlm = Ql[:S]
    for j in range(S):
        for i in range(S - j):
            P2[i + j] += Xl[i] * al[j] - Qlm[i] * pl[j]
            assert -(1 << 63) <= P2[i + j] < (1 << 63)
    st.acc2 = max(st.acc2, max(abs(v) for v in P2))
    c = 0
    rl = []
    for k in range(S):
        v = P2[k] + c
        rl.append(v & MASK)
        c = v >> LB          # arithmetic shift (Python's >> floors)
    r = val(rl)
    R = 1 << (LB * S)
    assert r == (init + X * a - Q * p) % R
    assert r == init + X * a - Q * p, "r must be exact (0 <= r < R)"
    return r, Q


def check(pbits, S, K=47, trials=40, seed=7):
    rng = random.Random(seed)
    st = Stats()
    R = 1 << (LB * S)
    for t in range(trials):
        while True:
            p = rng.getrandbits(pbits) | (1 << (pbits - 1)) | 1
            if pow(3, p - 1, p) == 1:
                break
        p2 = p * p
        # start: c0 = (1, gamma), gamma an unreduced chunk sum < 2^11 p (kernels_fbp.hpp fbp_c0)
        A, B = 1, rng.randrange(0, (1 << 11) * p)
        V = (A + p * B) % p2
        bs = 0
        for k in range(K):
            T = rng.randrange(1, p2)
            if T % p == 0:
                continue
            a = T % p
            b = ((T - a) // p) * pow(a, -1, p) % p
            assert T % p2 == a * (1 + p * b) % p2
            ap = a * R // p
            A, QA = shoup_pass(A, a, ap, p, S, 0, st)
            B, _ = shoup_pass(B, a, ap, p, S, QA, st)
            bs += b
            V = V * a % p2
            assert (A + p * B) % p2 == V
            st.alpha = max(st.alpha, A / p)
            st.beta = max(st.beta, B / p)
            assert A < R and B < R
        # (A + p B)(1 + p bs) == prod T_k c0: the b sum applied once
        W = (A + p * (B + A * bs)) % p2
        assert W == V * (1 + p * bs) % p2
    return st


if __name__ == "__main__":
    for pbits, S in ((512, 19), (1024, 37)):
        st = check(pbits, S)
        print(f"p {pbits} bits, S = {S}: max A/p = {st.alpha:.1f}, max B/p = {st.beta:.1f}, quotient shortfall <= {st.qerr}, "
              f"step-1 accumulator < 2^{st.acc1.bit_length()}, step-2 |accumulator| < 2^{st.acc2.bit_length()}")
