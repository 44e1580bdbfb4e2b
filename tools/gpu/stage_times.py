"""Alternating encrypt / decrypt on one 1M-element vector with per-kernel HIP-event timing, to
compare kernels under the same clock/thermal state (diagnostic, not part of the bench contract)."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "ibond-flex_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from flex.crypto.paillier import _native  # noqa: E402
from flex.crypto.paillier.keypair import generate_paillier_keypair  # noqa: E402

nb = int(os.environ.get("NB", "2048"))
N = int(os.environ.get("N", str(1 << 20)))
reps = int(os.environ.get("REPS", "3"))
pk, sk = generate_paillier_keypair(nb, seed=1)
ctx = _native.Context(pk.n, 0, sk.p, sk.q)
ctx.set_stage_timing(True)
lib = _native.load_library()
dev = torch.device("cuda", 0)
x = torch.from_numpy(np.random.default_rng(0).standard_normal(N, dtype=np.float32)).to(dev)
ct = torch.empty((N, ctx.ct_words), dtype=torch.int32, device=dev)
ex = torch.empty(N, dtype=torch.int32, device=dev)
val = torch.empty(N, dtype=torch.float64, device=dev)
st = torch.empty(N, dtype=torch.int32, device=dev)
key = hashlib.sha256(b"k").digest()
s = torch.cuda.current_stream(dev).cuda_stream
out = []
for r in range(reps):
    assert lib.pai_encrypt_dev(ctx.handle, 0, x.data_ptr(), N, 0, 0, 2, None, 0, 0, key, 0, ct.data_ptr(),
                               ex.data_ptr(), None, s) == 0
    e = ctx.stage_times()
    assert lib.pai_decrypt_dev(ctx.handle, ct.data_ptr(), ex.data_ptr(), N, val.data_ptr(), None, st.data_ptr(),
                               None, s) == 0
    d = ctx.stage_times()
    out.append({"rep": r, "encrypt_ms": e, "decrypt_ms": d})
    print(json.dumps(out[-1]), flush=True)
torch.cuda.synchronize()
assert torch.equal(val, x.double())
