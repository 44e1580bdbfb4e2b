"""Value-level model of the factored 1024/2048-bit decryption exponentiation (k_dec_pow_pair, kernels_pair.hpp decf_run;
flexpai.hip build_decf_lane_program) -- the lane-engine port of dec4f_model.py's chain.

Unlike the 4096-bit split-pair kernel, the lane engine keeps its window table of FULL pairs: P_1 = c~ = (A~, B_c) and
P_{2k+1} = mm(P_{2k-1}, mm(c~, c~)) (one square + 15 general pair products, as before), because there a general pair
product costs 5 S^2 MACs against 4 S^2 for a B-free one, not twice. Only the chain's window multipliers are B-free:
each entry is factored P_t = a_t (1 + p b_t) (b_t = H_t / a_t, H_t its B component, which now carries the
ciphertext's u = B_c / A~ t times) and the chain multiplies by (a_t, 0). The dropped factors total 1 + p s,
s = sum_t K_t b_t (K_t: the chain's multiplies by t weighted by 2^(squares after them)); the closing multiply by the
B-free (A~, 0) instead of c~ drops one more factor (1 + p u) = (1 + p b_1), so slot 1's weight is K_1 + 1. The chain
runs p - 2, so its result's A component is iota = A~^-1 R^2 mod p (Fermat) and a_t^-1 = iota^t (up to the R scaling
the Horner weights K'_t = K_t R absorb):

  Y' = chain over p - 2 with multipliers (a_t, 0) (first load: the full pair P_first)
  1 + p G = mm(mm(Y', (A~, 0)), (1, 0))
  delta = REDC(acc iota), acc = Horner over j = 15..0 of REDC(H_{2j+1} K'_{2j+1}) in w R^-1, w = REDC(iota iota)
  c^(p-1) mod p^2 = (1 + p G)(1 + p delta): the output pair (A, G + delta)
"""
import dec4f_model as D

LB = D.LB


def kconsts(e, p, R):
    """K'_t = R (K_t + [t == 1]) mod p: the chain's weights, plus the closing (A~, 0) for entry 1."""
    first, ops = D.sliding_schedule(e)
    K = [0] * 16
    after = 0
    for nsq, idx in reversed(ops):
        if idx is not None:
            K[idx] += 1 << after
        after += nsq
    K[0] += 1
    return first, ops, [(k * R) % p for k in K]


def run(p, c, S):
    R = 1 << (LB * S)
    p2 = p * p
    Ri2 = pow(R, -1, p2)
    Rip = pow(R, -1, p)
    mm = lambda x, y: x * y * Ri2 % p2
    mp = lambda x, y: x * y * Rip % p
    xt = c * R % p2                       # k_dec_pre_pair's pair, as a value
    A = xt % p
    # table of full pairs: P_1 = c~, x2 = mm(c~, c~), P_{t+2} = mm(P_t, x2)
    x2 = mm(xt, xt)
    P = {1: xt}
    for t in range(3, 32, 2):
        P[t] = mm(P[t - 2], x2)
    a = {t: P[t] % p for t in P}
    H = {t: P[t] // p for t in P}
    first, ops, Kp = kconsts(p - 2, p, R)
    y = P[2 * first + 1]                  # the first load takes the full pair
    for nsq, idx in ops:
        for _ in range(nsq):
            y = mm(y, y)
        if idx is not None:
            y = mm(y, a[2 * idx + 1])     # B-free multiplier
    iota = y % p
    g = mm(mm(y, A), 1)
    assert g % p == 1 % p or A == 0
    G = g // p
    w = mp(iota, iota)
    acc = 0
    for j in range(15, -1, -1):
        v = H[2 * j + 1] * Kp[j] * Rip % p
        acc = (v + acc * w) * Rip % p
    delta = mp(acc, iota)
    return (g + p * delta) % p2


if __name__ == "__main__":
    import random
    import sys
    rnd = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    bad = 0
    for bits, S in ((1024, 37), (1020, 37), (512, 19)):
        for trial in range(4):
            p = D.rand_prime(bits, rnd)
            q = D.rand_prime(bits, rnd)
            n2 = (p * q) ** 2
            cs = [rnd.randrange(n2) for _ in range(6)] + [0, p * rnd.randrange(1, q * q), 1, n2 - 1]
            for c in cs:
                if run(p, c, S) != pow(c, p - 1, p * p):
                    bad += 1
                    print("MISMATCH", bits, hex(c)[:20])
    print("ok" if bad == 0 else f"{bad} mismatches")
