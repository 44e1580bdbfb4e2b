"""GPU parity of segmented sums (pai_segment_add: gather-indexed 16-operand k_add reduction tree) and of
parallel_ops.segment_sum / good_bad_calc (the per-bin sums of hetero_bin.py:27-36) against the
reference-generated vectors (tests/golden/make_golden_seg.py) and the oracle, bit-exact."""
import json
import os

import numpy as np
import pytest

from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gseg():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_seg.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def key(golden):
    k = golden["keys"]["1024"]
    return O.Key(int(k["n"], 16), int(k["p"], 16), int(k["q"], 16))


def test_segment_add_golden_and_package(gseg, key):
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier import parallel_ops
    from flex.crypto.paillier.cipher_array import materialize
    from flex.crypto.paillier.keypair import PaillierPublicKey
    ctx = N.Context(key.n, 0, key.p, key.q)
    pub = PaillierPublicKey(key.n)
    for case in ("labels", "floats"):
        g = gseg["cases"][case]
        cs = [int(h, 16) for h in g["c"]]
        words = N.ints_to_words(cs, ctx.ct_words)
        exps = np.array(g["e"], dtype=np.int32)
        bins = gseg["bins"]
        # raw segmented add through the C ABI vs the oracle's aligned product
        idx = np.array([i % len(cs) for b in bins for i in b], dtype=np.int64)
        off = np.concatenate([[0], np.cumsum([len(b) for b in bins])]).astype(np.int64)
        out, oe = ctx.segment_add(words, exps, idx, off)
        got = N.words_to_ints(out)
        for s, b in enumerate(bins):
            if b:
                assert (got[s], int(oe[s])) == O.add_k([cs[i] for i in b], [g["e"][i] for i in b], key), (case, s)
            else:
                assert got[s] == 1 and int(oe[s]) == np.iinfo(np.int32).min
        # the package API vs the reference's good/bad numbers
        enc = materialize(pub, words, exps, (len(cs),), obfuscated=True)
        good, bad = parallel_ops.good_bad_calc(enc, [np.array(b, dtype=np.int64) for b in bins])
        for s in range(len(bins)):
            if g["good"][s] is None:
                assert good[s] == 0 and bad[s] == 0
                continue
            assert (hex(good[s].ciphertext(False)), good[s].exponent) == tuple(g["good"][s]), (case, s)
            assert (hex(bad[s].ciphertext(False)), bad[s].exponent) == tuple(g["bad"][s]), (case, s)


@pytest.mark.parametrize("sizes", [[0, 1, 2, 15, 16, 17, 255, 256, 257, 1000], [4096], [1] * 300])
def test_segment_add_vs_oracle_levels(key, sizes):
    """Segments that need 1, 2, 3 and 4 reduction levels side by side, random exponents 0..20."""
    from flex.crypto.paillier import _native as N
    ctx = N.Context(key.n, 0, key.p, key.q)
    rng = np.random.default_rng(len(sizes))
    M = 3000
    cs = [O.raw_encrypt(int(m), key, O.golden_r(key.n, 91, i)) for i, m in enumerate(rng.integers(0, 1 << 50, M))]
    es = rng.integers(0, 21, M).astype(np.int32)
    words = N.ints_to_words(cs, ctx.ct_words)
    members = [rng.integers(0, M, s) for s in sizes]
    idx = np.concatenate(members).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    out, oe = ctx.segment_add(words, es, idx, off)
    got = N.words_to_ints(out)
    for s, mem in enumerate(members):
        if len(mem):
            assert (got[s], int(oe[s])) == O.add_k([cs[i] for i in mem], [int(es[i]) for i in mem], key), s
