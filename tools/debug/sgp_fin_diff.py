"""k_sgp_fin against k_fbg_fin (test build, $FLEXPAI_SGP_FIN=0) on the same device RNG: which elements differ (debug aid)."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
from flex.crypto.paillier import _native as N
g = json.load(open(os.path.join(ROOT, "tests/golden/paillier_golden.json")))["keys"]["4096"]
n, p, q = int(g["n"], 16), int(g["p"], 16), int(g["q"], 16)
xlib = N.load_library(N.XCHECK_LIB_PATH)
rk = bytes(range(3, 35))
res = {}
for fin in ("1", "0"):
    os.environ["FLEXPAI_SGP_FIN"] = fin
    ctx = N.Context(n, 0, p, q, lib=xlib)
    ctx.set_fb_window(8)
    ctx.prepare_fixed_base()
    for count in (1, 2, 31, 32, 33, 63, 64, 129, 1000):
        x = (np.random.default_rng(count).standard_normal(count) * 1e3).astype(np.float32)
        ct, ex, _ = ctx.encrypt(x, obf_mode=N.PAI_OBF_RNG, rng_key=rk, index_base=7)
        res[(fin, count)] = ct.copy()
    ctx.close()
for count in (1, 2, 31, 32, 33, 63, 64, 129, 1000):
    a, b = res[("1", count)], res[("0", count)]
    bad = np.nonzero((a != b).any(axis=1))[0]
    words = sorted(set(np.nonzero((a != b))[1].tolist()))[:12] if len(bad) else []
    print("count", count, "bad", len(bad), bad[:12].tolist(), "words", words, flush=True)
