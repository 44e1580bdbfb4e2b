"""Fresh-key breakdown: a new keypair per call, as HE_SA_FT does per exchange
(/root/reference/flex/federated_training/secure_aggregation/he_sa_ft/train.py:38-39): Context, set_private, and the
first device-RNG encrypt of a 1M float32 vector (which builds the W = 16 tables past the break-even count), each timed
on the host clock with the device synchronised, with $FLEXPAI_SETUP_TRACE's per-step lines from the library on stderr.

    python tools/fresh_key_trace.py [--keys 3] [--n 1048576] [--nb 2048] [--rows-max N]

--rows-max sets PAI_OPT_ROWS_MAX (0: the lane kernels k_crt_a + k_crt_b_pair for every call size).
"""
import argparse
import os
import sys
import time

os.environ.setdefault("FLEXPAI_SETUP_TRACE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ibond-flex_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--nb", type=int, default=2048)
    ap.add_argument("--rows-max", type=int, default=None)
    a = ap.parse_args()
    from flex.crypto.paillier import _native as N
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    x = torch.randn(a.n, dtype=torch.float32, device=dev)
    W = 2 * a.nb // 32
    ct = torch.empty((a.n, W), dtype=torch.int32, device=dev)
    ex = torch.empty(a.n, dtype=torch.int32, device=dev)
    st = torch.empty(a.n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    lib = N.load_library()
    keys = [generate_paillier_keypair(a.nb, seed=100 + i) for i in range(a.keys)]
    for i, (pk, sk) in enumerate(keys):
        torch.cuda.synchronize()
        print(f"--- key {i}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        c = N.Context(pk.n, 0)
        t1 = time.perf_counter()
        c.set_private(sk.p, sk.q)
        if a.rows_max is not None:
            c.set_rows_max(a.rows_max)
        t2 = time.perf_counter()
        c.set_stage_timing(True)
        rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), a.n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32), 0,
                                 ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
        assert rc == 0, lib.pai_last_error()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        stages = c.stage_times()
        rc = lib.pai_encrypt_dev(c.handle, N.PAI_F32, x.data_ptr(), a.n, 0, 0, N.PAI_OBF_RNG, None, 0, 0, bytes(32), 0,
                                 ct.data_ptr(), ex.data_ptr(), st.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"key {i}: ctx {1e3 * (t1 - t0):.1f} ms, set_private {1e3 * (t2 - t1):.1f} ms, first call "
              f"{1e3 * (t3 - t2):.1f} ms (kernels {sum(stages):.1f} ms: {[round(s, 2) for s in stages]}), total "
              f"{1e3 * (t3 - t0):.1f} ms = {a.n / (t3 - t0) / 1e6:.2f} M enc/s incl setup; warm call {1e3 * (t4 - t3):.1f} ms; "
              f"tables {c.fb_ready} W = {c.fb_window if c.fb_ready else None}", flush=True)
        c.close()


if __name__ == "__main__":
    main()
