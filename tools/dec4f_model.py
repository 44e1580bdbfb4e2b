"""Value-level model of the factored 4096-bit decryption exponentiation (k_dec4_pow, kernels_dec4.hpp).

c^(p-1) mod p^2 on p-adic pairs with B-free multipliers: the window table P_t (mm-powers of the B-free base
(A~, 0)) is factored P_t = a_t (1 + p b_t), the chain multiplies by (a_t, 0) only (one pass on both lanes), and
the dropped factors are restored at the end from the chain's own Fermat inverse (the chain runs p - 2):

  c~ = A~ + p B_c = A~ (1 + p u),  u = B_c / A~
  Y' = chain over p - 2 with multipliers (a_t, 0);  iota = Y' mod p = A~^-1 R^2
  s' - u = REDC(acc iota),  acc = Horner_w(c_j),  w = REDC(iota iota),  c_j = REDC(REDC(H_t K'_t) + ...)
  c^(p-1) mod p^2 = (1 + p G)(1 + p (s' - u)),  1 + p G = mm(mm(Y', A~), 1)

Checks L = (c^(p-1) mod p^2 - 1) / p against the direct computation for random primes and ciphertexts.
"""
import random
import sys

LB = 28


def sliding_schedule(e, K=5):
    """Mirror of flexpai.hip sliding_schedule: (first, [(nsq, idx | None), ...])."""
    bit = lambda b: (e >> b) & 1
    i = e.bit_length() - 1

    def window(hi):
        lo = max(hi - K + 1, 0)
        while not bit(lo):
            lo += 1
        v = 0
        for b in range(hi, lo - 1, -1):
            v = (v << 1) | bit(b)
        return lo, v

    lo, v = window(i)
    first = (v - 1) // 2
    i = lo - 1
    ops, nsq = [], 0
    while i >= 0:
        if not bit(i):
            nsq += 1
            i -= 1
            continue
        lo, v = window(i)
        nsq += i - lo + 1
        ops.append((nsq, (v - 1) // 2))
        nsq = 0
        i = lo - 1
    if nsq:
        ops.append((nsq, None))
    return first, ops


def kconsts(e, p, R):
    """K'_t = R * sum over the chain's multiplies by table entry t of 2^(squarings after it), mod p; slot 0 = -R."""
    first, ops = sliding_schedule(e)
    K = [0] * 16
    after = 0
    for nsq, idx in reversed(ops):
        if idx is not None:
            K[idx] += 1 << after
        after += nsq
    Kp = [(k * R) % p for k in K]
    Kp[0] = (-R) % p
    return first, ops, Kp


def run(p, c, S):
    R = 1 << (LB * S)
    p2 = p * p
    Ri2 = pow(R, -1, p2)
    Rip = pow(R, -1, p)
    mm = lambda x, y: x * y * Ri2 % p2
    mp = lambda x, y: x * y * Rip % p
    xt = c * R % p2                       # k_dec4_pre's pair, as a value
    A, Bc = xt % p, xt // p               # its components (the kernel's may be non-canonical: same algebra)
    # table: P_1 = (A, 0), P_{t+1} = mm(P_t, (A, 0))
    P = {1: A}
    for t in range(2, 32):
        P[t] = mm(P[t - 1], A)
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
    z = mm(y, A)
    g = mm(z, 1)
    assert g % p == 1 % p or A == 0
    G = g // p
    w = mp(iota, iota)
    acc = 0
    for j in range(15, -1, -1):
        h = Bc if j == 0 else H[2 * j + 1]
        v = h * Kp[j] * Rip % p           # pass 1: REDC(H K')
        acc = (v + acc * w) * Rip % p     # pass 2: REDC(V + acc w)
    delta = mp(acc, iota)
    return (g + p * delta) % p2           # k_dec4_pow's output pair A + p (G + delta)


def is_prime(n, rnd):
    if n < 4:
        return n in (2, 3)
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for _ in range(8):
        x = pow(rnd.randrange(2, n - 1), d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def rand_prime(bits, rnd):
    while True:
        v = rnd.getrandbits(bits) | (1 << (bits - 1)) | 1
        if is_prime(v, rnd):
            return v


if __name__ == "__main__":
    rnd = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    bad = 0
    for bits, S in ((2048, 74), (2040, 74), (1024, 37), (512, 19)):
        for trial in range(4):
            p = rand_prime(bits, rnd)
            q = rand_prime(bits, rnd)
            n2 = (p * q) ** 2
            cs = [rnd.randrange(n2) for _ in range(6)] + [0, p * rnd.randrange(1, q * q), 1, n2 - 1]
            for c in cs:
                got = run(p, c, S)
                want = pow(c, p - 1, p * p)
                if got != want:
                    bad += 1
                    print("MISMATCH", bits, hex(c)[:20])
    print("ok" if bad == 0 else f"{bad} mismatches")
