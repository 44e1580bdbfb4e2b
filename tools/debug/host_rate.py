"""Where does the host-buffer encrypt time go (debug aid): first-touch of the output, the device call, the
pipelined host call."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]
import torch
from flex.crypto.paillier import _native as N
from flex.crypto.paillier.keypair import generate_paillier_keypair
pk, sk = generate_paillier_keypair(2048, seed=1)
ctx = N.Context(pk.n, 0, sk.p, sk.q)
ctx.set_fb_window(20)
ctx.prepare_fixed_base()
n = 1 << 20
x = np.random.default_rng(0).standard_normal(n).astype(np.float32)
print("thp:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(), flush=True)
for rep in range(3):
    t = time.perf_counter(); a = np.empty((n, 128), np.uint32); a.fill(1); t_touch = time.perf_counter() - t
    t = time.perf_counter(); a[:] = 2; t_rewrite = time.perf_counter() - t
    t = time.perf_counter(); ct, ex, st = ctx.encrypt(x, rng_key=b"k" * 32); t_enc = time.perf_counter() - t
    print(f"touch 512MiB {t_touch*1e3:.1f} ms, rewrite {t_rewrite*1e3:.1f} ms, host encrypt {t_enc*1e3:.1f} ms "
          f"({n / t_enc / 1e6:.2f} M/s)", flush=True)
d = torch.device("cuda", 0)
xd = torch.from_numpy(x).to(d)
ctd = torch.empty((n, 128), dtype=torch.int32, device=d)
exd = torch.empty(n, dtype=torch.int32, device=d)
std = torch.empty(n, dtype=torch.int32, device=d)
lib = N.load_library()
for rep in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    lib.pai_encrypt_dev(ctx.handle, N.PAI_F32, xd.data_ptr(), n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, b"k" * 32, 0,
                        ctd.data_ptr(), exd.data_ptr(), std.data_ptr(), None)
    torch.cuda.synchronize(); t_dev = time.perf_counter() - t
    pin = torch.empty((n, 128), dtype=torch.int32, pin_memory=True)
    t = time.perf_counter(); pin.copy_(ctd); torch.cuda.synchronize(); t_d2h = time.perf_counter() - t
    print(f"device encrypt {t_dev*1e3:.1f} ms, D2H pinned 512MiB {t_d2h*1e3:.1f} ms", flush=True)
# pipeline alone: caller buffers allocated and touched once, reused
ct = np.ones((n, 128), np.uint32); ex = np.ones(n, np.int32); st = np.ones(n, np.int32)
for rep in range(3):
    t = time.perf_counter()
    rc = lib.pai_encrypt(ctx.handle, N.PAI_F32, x.ctypes.data, n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, b"k" * 32, 0,
                         ct.ctypes.data, ex.ctypes.data, st.ctypes.data)
    t_p = time.perf_counter() - t
    print(f"pai_encrypt into touched buffers {t_p*1e3:.1f} ms ({n / t_p / 1e6:.2f} M/s) rc={rc}", flush=True)
