"""The Shoup-row sampler's intermediates for one 4096-bit element against the oracle (debug aid, test build):
$FLEXPAI_DEBUG_SGS_STAGE=1 leaves k_sgs's pairs (expected prod_k (T_k R mod p^2 mod p) mod p^2, R = 2^(28 76)),
=2 the pairs after k_sgs_bfin (expected c0 G^a mod p^2); the Montgomery sampler's (k_sgp) pairs at stage 2 too."""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from oracle import paillier_oracle as O
from flex.crypto.paillier import _native as N
g = json.load(open(os.path.join(ROOT, "tests/golden/paillier_golden.json")))["keys"]["4096"]
key = O.Key(int(g["n"], 16), int(g["p"], 16), int(g["q"], 16))
xlib = N.load_library(N.XCHECK_LIB_PATH)
W, base = 8, 7
rk = bytes(range(9, 41))
x = np.array([1234.5, -77.25, 3.0], dtype=np.float64)
S = 74
R = 1 << (28 * 76)


def run(sgs, stage):
    os.environ["FLEXPAI_DEBUG_SGS_STAGE"] = str(stage)
    if sgs:
        os.environ["FLEXPAI_SGS"] = "1"
    else:
        os.environ.pop("FLEXPAI_SGS", None)
    ctx = N.Context(key.n, 0, key.p, key.q, lib=xlib)
    ctx.set_fb_window(W)
    ctx.prepare_fixed_base()
    assert bool(ctx.split_sampler & 8) == sgs
    ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    n = len(x)
    buf = (ctypes.c_uint32 * (2 * 148 * n))()
    nn, sb = ctypes.c_longlong(), ctypes.c_int()
    rc = xlib.pai_debug_fb_w(ctx._h, buf, ctypes.c_size_t(len(buf)), ctypes.byref(nn), ctypes.byref(sb))
    assert rc == 0, rc
    a = np.frombuffer(buf, dtype=np.uint32).reshape(2, 148, n)
    ctx.close()
    out = []
    for h in range(2):
        P = (key.p, key.q)[h]
        A = sum(int(a[h, i, 0]) << (28 * i) for i in range(S))
        B = sum(int(a[h, S + i, 0]) << (28 * i) for i in range(S))
        out.append((A, B, (A + P * B) % (P * P)))
    return out


params = None
gp, gq = O.fb_base(key.p), O.fb_base(key.q)
rb = O.fb_raw_bits(key.p, key.q)
K = O.fb_digits(key.p, key.q, W)
m_enc, _ = O.encode(float(x[0]), key.n, key.max_int)
for h in range(2):
    P = (key.p, key.q)[h]
    P2 = P * P
    G = pow((gp, gq)[h], key.n, P2)
    a_h = O.fb_exponent(rk, base, h, P - 1, rb)
    digits = [(a_h >> (W * k)) & ((1 << W) - 1) for k in range(K)]
    vraw = 1
    for k, d in enumerate(digits):
        T = pow(G, d << (W * k), P2)
        vraw = vraw * ((T * R % P2) % P) % P2
    c0 = (1 + key.n * m_enc) % P2
    vfin = c0 * pow(G, a_h, P2) % P2
    s1 = run(True, 1)[h]
    s2 = run(True, 2)[h]
    m2 = run(False, 2)[h]
    print("half", h, "k_sgs raw ok", s1[2] == vraw, "A<77P", s1[0] < 77 * P, "B<154P", s1[1] < 154 * P)
    print("half", h, "after bfin ok", s2[2] == vfin, "A<P", s2[0] < P, "B<P", s2[1] < P)
    print("half", h, "k_sgp ok", m2[2] == vfin)
    if s1[2] != vraw:
        print("  raw/expected ratio mod P:", s1[2] * pow(vraw, -1, P2) % P2 % P == 1)
    # which factor is off: A of the final pair against V_raw c_A (mod P), then the b-sum scalar
    Ci = pow(pow(2, 28 * 76 * K, P2), -1, P2)
    cA, cB = Ci % P, Ci // P
    beta = cB * pow(cA, -1, P) % P
    gam = (key.n // P) * m_enc % P
    base_v = s1[2] * cA % P2
    print("  A part ok", s2[2] % P == base_v % P)
    inv_base = pow(base_v, -1, P2)
    S_exp = ((vfin * inv_base % P2) - 1) // P % P
    S_act = ((s2[2] * inv_base % P2) - 1) // P % P
    for name, v in (("gamma", gam), ("beta", beta), ("gamma+beta", gam + beta), ("-beta", -beta), ("2beta", 2 * beta)):
        if (S_act - S_exp - v) % P == 0:
            print("  actual b scalar = expected +", name)
        if (S_exp - S_act - v) % P == 0:
            print("  actual b scalar = expected -", name)
    print("  diff", hex((S_act - S_exp) % P)[:40])
    # the b sum itself: b_k = B_k A_k^-1 mod P for the pair (A_k, B_k) of T_k R mod P^2
    sb = 0
    bints = []
    for k, d in enumerate(digits):
        TR = pow(G, d << (W * k), P2) * R % P2
        Ak, Bk = TR % P, TR // P
        bk = Bk * pow(Ak, -1, P) % P
        bints.append(bk * R % P)
        sb += bk
    print("  S_exp == gamma + beta + sum b:", (S_exp - gam - beta - sb) % P == 0)
    dint = (S_act - S_exp) * R % P
    for wpos in (0, 32, 64):
        c = dint * pow(2, -32 * wpos, P) % P
        c2 = (-dint) * pow(2, -32 * wpos, P) % P
        print("  diff at word", wpos, ":", c if c < 2 ** 40 else "-", "/ neg", c2 if c2 < 2 ** 40 else "-")
    for name, v in (("b_0", bints[0]), ("b_last", bints[-1]), ("gammaR", gam * R % P), ("betaR", beta * R % P)):
        if dint == v % P or (-dint) % P == v % P:
            print("  diff = +-", name)
    s3 = None
    os.environ["FLEXPAI_DEBUG_SGS_STAGE"] = "3"
    os.environ["FLEXPAI_SGS"] = "1"
    ctx = N.Context(key.n, 0, key.p, key.q, lib=xlib)
    ctx.set_fb_window(W)
    ctx.prepare_fixed_base()
    ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    buf = (ctypes.c_uint32 * (2 * 148 * len(x)))()
    nn, sbb = ctypes.c_longlong(), ctypes.c_int()
    assert xlib.pai_debug_fb_w(ctx._h, buf, ctypes.c_size_t(len(buf)), ctypes.byref(nn), ctypes.byref(sbb)) == 0
    ctx.close()
    a3 = np.frombuffer(buf, dtype=np.uint32).reshape(2, 148, len(x))
    bs_act = sum(int(a3[h, w_, 0]) << (32 * w_) for w_ in range(68))
    bs_sum = sum(bints)
    gR = gam * R % P
    print("  bs words == sum b_k R + gamma R + beta R (as integers mod P):", (bs_act - bs_sum - gR - beta * R) % P == 0)
    print("  bs - sum b_k R (mod P) == gammaR+betaR:", (bs_act - bs_sum) % P == (gR + beta * R) % P, " == gammaR:", (bs_act - bs_sum) % P == gR)
    print("  bs - gammaR - betaR == sum b (int):", bs_act - bs_sum, "bits", (bs_act - bs_sum).bit_length())
    os.environ["FLEXPAI_DEBUG_SGS_STAGE"] = "4"
    ctx = N.Context(key.n, 0, key.p, key.q, lib=xlib)
    ctx.set_fb_window(W)
    ctx.prepare_fixed_base()
    ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=base)
    assert xlib.pai_debug_fb_w(ctx._h, buf, ctypes.c_size_t(len(buf)), ctypes.byref(nn), ctypes.byref(sbb)) == 0
    ctx.close()
    a4 = np.frombuffer(buf, dtype=np.uint32).reshape(2, 148, len(x))
    A1 = sum(int(a4[h, i, 0]) << (28 * i) for i in range(S))
    B1 = sum(int(a4[h, S + i, 0]) << (28 * i) for i in range(S))
    print("  after the c_A pass: V == V_raw c_A mod P^2:", (A1 + P * B1) % P2 == base_v, "A1<2P", A1 < 2 * P, "B1 < 4P", B1 < 4 * P,
          "B1/P", B1 // P)
    # final from these by the formula
    t_ = A1 // P
    A1r = A1 - t_ * P
    Sb = (bs_act * pow(R, -1, P)) % P
    Bf = (B1 + t_ + A1r * Sb) % P
    print("  formula final == expected:", (A1r + P * Bf) % P2 == vfin, " kernel final B == formula B:", s2[1] == Bf, "kernel A == A1r", s2[0] == A1r)
    # simulate kernels_sgp.hpp sgp_step on both lanes for (A_raw, B_raw) times y = c_A R' mod P
    def limbs(v):
        return [(v >> (28 * i)) & ((1 << 28) - 1) for i in range(S)]
    mm = limbs(P)
    mpr = (-pow(P, -1, 1 << 28)) % (1 << 28)
    y = cA * (1 << (28 * S)) % P
    yd = limbs(y)
    xa, xb = limbs(s1[0]), limbs(s1[1])
    PA, PB = [0] * S, [0] * S
    for J in range(S):
        for i in range(S):
            PA[(i + J) % S] += xa[i] * yd[J]
            PB[(i + J) % S] += xb[i] * yd[J]
        q0a = (PA[J] * mpr) & ((1 << 28) - 1)
        q1 = q0a
        qa = q0a
        qb = (((PB[J] & 0xFFFFFFFF) - q1) * mpr) & ((1 << 28) - 1)
        for i in range(S):
            PA[(i + J) % S] += qa * mm[i]
            PB[(i + J) % S] += qb * mm[i]
        PA[(J + 1) % S] += PA[J] >> 28
        PB[(J + 1) % S] += PB[J] >> 28
        PA[J] = PB[J] = 0
    def norm(Pv):
        c = 0
        out = 0
        for i in range(S):
            v = Pv[i] + c
            out |= (v & ((1 << 28) - 1)) << (28 * i)
            c = v >> 28
        return out, c
    As, ca_ = norm(PA)
    Bs, cb_ = norm(PB)
    print("  sim: A == kernel A1", As == A1, "B == kernel B1", Bs == B1, "sim V ok", (As + P * Bs) % P2 == base_v, "top carries", ca_, cb_)
