"""Vectors and checker for tools/microbench/sgp_shoup_pass.hip (the S = 74 Shoup-pass feasibility measurement,
DESIGN.md section 8.2).

  python tools/microbench/sgp_shoup_vec.py gen  <vec.bin>
  python tools/microbench/sgp_shoup_vec.py check <vec.bin> <out_prefix> <K>
  python tools/microbench/sgp_shoup_vec.py check_sgs <vec.bin> <out.bin>   (tools/microbench/sgs_stream.hip check)

gen: a random 2048-bit odd modulus m (so m > 2^(28 * 73), the Shoup estimate's condition), two rows a0, a1 < m with
their Shoup quotients a' = floor(a R / m), R = 2^(28 * 74), the rows again as packed 32-bit words (the Montgomery
pass's layout), and 64 starting pairs (A, B) < m.  check: the pairs the GPU wrote after K products (row k & 1 for
product k) against V_K = V_0 a0^ceil(K/2) a1^floor(K/2) (Shoup: plain products) and the same times R^-K (Montgomery)
mod m^2, V = A + m B.
"""
import random
import struct
import sys

S, LB = 74, 28
R = 1 << (LB * S)
PAIRS = 64


def limbs(x, n=S):
    return [(x >> (LB * i)) & ((1 << LB) - 1) for i in range(n)]


def words(x, n):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def unlimbs(v):
    return sum(int(d) << (LB * i) for i, d in enumerate(v))


def gen(path):
    rng = random.Random(20261018)
    m = rng.getrandbits(2048) | (1 << 2047) | 1
    mprime = (-pow(m, -1, 1 << LB)) % (1 << LB)
    a = [rng.randrange(1, m) for _ in range(2)]
    ap = [(x * R) // m for x in a]
    out = limbs(m) + [mprime]
    for x in a:
        out += limbs(x)
    for x in ap:
        out += limbs(x)
    for x in a:
        out += words(x, 64)
    for _ in range(PAIRS):
        out += limbs(rng.randrange(m)) + limbs(rng.randrange(m))
    with open(path, "wb") as f:
        f.write(struct.pack("<%dI" % len(out), *out))


def read(path):
    b = open(path, "rb").read()
    return list(struct.unpack("<%dI" % (len(b) // 4), b))


def check(vec_path, prefix, K):
    v = read(vec_path)
    m = unlimbs(v[:S])
    o = S + 1
    a = [unlimbs(v[o:o + S]), unlimbs(v[o + S:o + 2 * S])]
    o += 4 * S + 128
    x0 = []
    for p in range(PAIRS):
        x0.append((unlimbs(v[o:o + S]), unlimbs(v[o + S:o + 2 * S])))
        o += 2 * S
    m2 = m * m
    f = pow(a[0], (K + 1) // 2, m2) * pow(a[1], K // 2, m2) % m2
    rinv = pow(R, -K, m2)
    ok = True
    for name, fac in (("shoup", f), ("mont", f * rinv % m2)):
        try:
            g = read("%s_%s.bin" % (prefix, name))
        except FileNotFoundError:
            print(name, "missing")
            continue
        bad = 0
        for p in range(PAIRS):
            A = unlimbs(g[(2 * p) * S:(2 * p + 1) * S])
            B = unlimbs(g[(2 * p + 1) * S:(2 * p + 2) * S])
            want = (x0[p][0] + m * x0[p][1]) * fac % m2
            if (A + m * B) % m2 != want:
                bad += 1
        print("%s: %d/%d pairs exact" % (name, PAIRS - bad, PAIRS))
        ok = ok and bad == 0
    return ok


def check_sgs(vec_path, out_path, K=9):
    """tools/microbench/sgs_stream.hip check: element e's pair = prod_k a_((k + e) & 1) mod m^2 (row 0 the start)"""
    v = read(vec_path)
    m = unlimbs(v[:S])
    o = S + 1
    a = [unlimbs(v[o:o + S]), unlimbs(v[o + S:o + 2 * S])]
    m2 = m * m
    g = read(out_path)
    # the b halves sgs_stream.hip wrote: word j of b_d = 0x9E3779B9 (2 j + d + 1) ^ 0xA5A5A5A5 d (32-bit)
    b = [sum((((0x9E3779B9 * (2 * j + d + 1)) & 0xFFFFFFFF) ^ ((0xA5A5A5A5 * d) & 0xFFFFFFFF)) << (32 * j) for j in range(64))
         for d in range(2)]
    bad = badb = 0
    ob = PAIRS * 2 * S
    for e in range(PAIRS):
        want = 1
        for k in range(K):
            want = want * a[(k + e) & 1] % m2
        A = unlimbs(g[(2 * e) * S:(2 * e + 1) * S])
        B = unlimbs(g[(2 * e + 1) * S:(2 * e + 2) * S])
        bad += (A + m * B) % m2 != want
        w = g[ob + 66 * e:ob + 66 * e + 66]
        got = sum(w[j] << (32 * j) for j in range(64)) + (w[64] << (32 * 32)) + (w[65] << (32 * 64))
        badb += got != sum(b[(k + e) & 1] for k in range(K))
    print("k_sgs: %d/%d pairs exact, %d/%d b sums exact" % (PAIRS - bad, PAIRS, PAIRS - badb, PAIRS))
    return bad == 0 and badb == 0


if __name__ == "__main__":
    if sys.argv[1] == "gen":
        gen(sys.argv[2])
    elif sys.argv[1] == "check_sgs":
        sys.exit(0 if check_sgs(sys.argv[2], sys.argv[3]) else 1)
    else:
        sys.exit(0 if check(sys.argv[2], sys.argv[3], int(sys.argv[4])) else 1)
