"""Diagnostic: does torch's HIP runtime still initialise after libflexpai contexts exist (with and without
threads, with the context still alive)? Prints one line per case."""
import sys, threading, os, json
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "ibond-flex_amd")]
import numpy as np
mode = sys.argv[1]
if mode.startswith("ti_"):
    import torch  # noqa: F401 - imported (not initialised) before flexpai: the loader starts torch's runtime
from flex.crypto.paillier import _native as N
root = sys.path[0]
g = json.load(open(root + "/tests/golden/paillier_golden.json"))
k = g["keys"]["2048"]
ctx = N.Context(int(k["n"], 16), 0, int(k["p"], 16), int(k["q"], 16))
x = np.ones(1000, np.float32)
if mode in ("threads", "threads_close"):
    th = [threading.Thread(target=lambda: ctx.encrypt(x)) for _ in range(4)]
    [t.start() for t in th]; [t.join() for t in th]
else:
    ctx.encrypt(x)
if mode.endswith("close"):
    ctx.close()
import torch
try:
    torch.cuda.init()
    print(mode, "torch ok", torch.cuda.device_count())
except Exception as e:
    print(mode, "torch FAILED", e)
