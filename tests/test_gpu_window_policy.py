"""FLEXPAI_FB_WINDOW=auto (include/flexpai.h PAI_OPT_FB_WINDOW): a process holding ONE private key
takes the largest fixed-base window whose tables fit FLEXPAI_FB_AUTO_FRAC of the free HBM, a process holding
several keys the default 16; the public tables take 20 in a one-context process. Each case runs in a child
process of its own, so the memory it sees and the keys it holds are its own. Plus the checks on caller-supplied
public bases."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/ibond-flex_amd"]
from flex.crypto.paillier import _native as N
g = json.load(open(sys.argv[1] + "/tests/golden/paillier_golden.json"))
k = g["keys"]["2048"]
n, p, q = int(k["n"], 16), int(k["p"], 16), int(k["q"], 16)
mode = sys.argv[2]
out = {}
free0, tot = N.device_mem_info(0)
out["free"], out["total"] = free0, tot
ctx = N.Context(n, 0, p, q)
if mode == "two_keys":
    k2 = g["keys"]["1024"]
    other = N.Context(int(k2["n"], 16), 0, int(k2["p"], 16), int(k2["q"], 16))
if mode in ("one_key", "two_keys"):
    ctx.prepare_fixed_base()
    out["window"] = ctx.fb_window
    out["table_bytes"] = ctx.fixed_base_setup()[2]
if mode == "public":
    pub = N.Context(n, 0)
    del ctx
    import gc; gc.collect()
    pub.prepare_public_fixed_base()
    out["pfb_window"] = pub.public_fixed_base_info()[2]
print(json.dumps(out))
'''


def _child(mode, **env):
    # the device as an idle MI355X: this (parent) process hands the chunks of tables earlier tests released back to the
    # driver first (csrc/table_arena.hpp keeps them for its own rebuilds until its last context is destroyed)
    from flex.crypto.paillier import _native as N
    N.release_table_cache()
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, mode], env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _fb_bytes(W, nb=2048):
    K = -(-(nb // 2) // W)                      # digits of p_h - 1 (1024 bits for the golden key)
    return 2 * K * (1 << W) * 448               # Shoup rows (kernels_fbs.hpp): 10 + 10 + 8 quads


def test_auto_window_one_key_takes_the_largest_that_fits():
    out = _child("one_key", FLEXPAI_FB_WINDOW="auto", FLEXPAI_FB_MIN_ELEMS="0")
    free, tot = out["free"], out["total"]
    budget = min(free - max(4 << 30, tot // 12), int(0.75 * free))
    want = max(w for w in (8, 12, 16, 20, 21, 22, 23, 24) if _fb_bytes(w) <= budget)
    assert out["window"] == want, out
    assert out["table_bytes"] == _fb_bytes(want)
    if free > 280e9:                            # an otherwise idle MI355X: the bench's window
        assert out["window"] == 22


def test_auto_window_fraction_caps_the_tables():
    out = _child("one_key", FLEXPAI_FB_WINDOW="auto", FLEXPAI_FB_AUTO_FRAC="0.2", FLEXPAI_FB_MIN_ELEMS="0")
    budget = min(out["free"] - max(4 << 30, out["total"] // 12), int(0.2 * out["free"]))
    assert _fb_bytes(out["window"]) <= budget < _fb_bytes(out["window"] + (1 if out["window"] >= 20 else 4))


def test_auto_window_several_keys_keep_the_default():
    out = _child("two_keys", FLEXPAI_FB_WINDOW="auto", FLEXPAI_FB_MIN_ELEMS="0")
    assert out["window"] == 16


def test_auto_window_public_tables():
    out = _child("public", FLEXPAI_FB_WINDOW="auto", FLEXPAI_PFB_MIN_ELEMS="0")
    assert out["pfb_window"] == 20


def test_default_window_is_16_without_auto():
    env = {k: v for k, v in os.environ.items() if k != "FLEXPAI_FB_WINDOW"}
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, "one_key"], env=dict(env, FLEXPAI_FB_MIN_ELEMS="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["window"] == 16


def test_public_bases_are_validated(golden_pfb):
    from flex.crypto.paillier import _native as N
    from oracle import paillier_oracle as O
    k = golden_pfb["keys"]["2048"]
    n = int(k["n"], 16)
    bases = [int(h, 16) for h in k["bases"]]
    ctx = N.Context(n, 0)
    ctx.set_public_bases(bases)                  # the golden bases satisfy every condition
    bad = list(bases)
    bad[3] = bad[7]
    with pytest.raises(N.NativeError, match="repeated"):
        ctx.set_public_bases(bad)
    bad = list(bases)
    bad[5] = int(k["p"], 16)                     # not a unit mod n
    with pytest.raises(N.NativeError, match="unit"):
        ctx.set_public_bases(bad)
    g0 = 2
    while O.jacobi(g0, n) != 1:
        g0 += 1
    bad = [g0] + bases[1:]
    with pytest.raises(N.NativeError, match="Jacobi"):
        ctx.set_public_bases(bad)
    with pytest.raises(N.NativeError):
        ctx.set_pfb_window(8)                    # only the golden-pinned windows 12, 16, 20
    ctx.set_pfb_window(12)
