#!/usr/bin/env python3
"""bench.py — Paillier-2048 array encryption on MI355X (BASELINE.json metric).

A step = one device-resident encryption of the rank's 1M-element float32 vector (encode ->
c0 -> c0 * r^n mod n^2 with a device ChaCha20 obfuscator r per element), then, for N > 1, one
RCCL all-gather of the ciphertext shards so every rank holds the whole encrypted vector.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, weak scaling)

Rank 0 prints ONE JSON line. `value` = encrypts/s over all ranks (max-over-ranks wall clock of the
K timed steps). `roofline` is for the dominant kernel (k_encrypt), timed with HIP events on the
stream it is launched on; `cpu_baseline` is the GMP restatement of the reference's CPU path
(oracle/gmp_oracle.c) timed on this host on a bounded sample of the same workload.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "ibond-flex_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

INT_MAC_PEAK = 31.94e12      # measured v_mad_u64_u32 issue rate, profiles/r01_step0_int_throughput.txt
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)


def canonical_w_enc(nb: int) -> float:
    """SURVEY.md §8d canonical algorithmic work of one encryption in 32x32->64 MACs."""
    s = nb // 16
    M = 2 * s * s + s
    P = (nb - 1) + (nb + 3) // 4 + 16
    return float((P + 1) * M)


def canonical_w_dec(nb: int) -> float:
    s = nb // 32
    M = 2 * s * s + s
    b = nb // 2
    P = (b - 1) + (b + 3) // 4 + 16
    return float(2 * (P + 2) * M)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 20, help="elements per GPU")
    ap.add_argument("--nb", type=int, default=2048, help="Paillier key bits")
    ap.add_argument("--cpu-sample", type=int, default=16384)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decrypt", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from flex.crypto.paillier import _native
    from flex.crypto.paillier.keypair import generate_paillier_keypair

    pk, sk = generate_paillier_keypair(args.nb, seed=1)
    ctx = _native.Context(pk.n, local_rank, sk.p, sk.q)
    lib = _native.load_library()
    N, W = args.n, ctx.ct_words
    x_host = np.random.default_rng(rank).standard_normal(N, dtype=np.float32)
    x = torch.from_numpy(x_host).to(dev)
    ct = torch.empty((N, W), dtype=torch.int32, device=dev)
    ex = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)
    rng_key = hashlib.sha256(b"flexpai-bench-key").digest()
    index_base = rank * N
    stream = torch.cuda.current_stream(dev)
    gathered = None
    if world > 1:
        gathered = torch.empty((world * N, W), dtype=torch.int32, device=dev)

    def encrypt():
        rc = lib.pai_encrypt_dev(ctx.handle, _native.PAI_F32, x.data_ptr(), N, 0, 0, _native.PAI_OBF_RNG,
                                 None, 0, 0, rng_key, index_base, ct.data_ptr(), ex.data_ptr(), st.data_ptr(),
                                 stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    def step():
        encrypt()
        if world > 1:
            dist.all_gather_into_tensor(gathered, ct)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        encrypt()
        ev[k][1].record(stream)
        if world > 1:
            dist.all_gather_into_tensor(gathered, ct)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    # correctness on the timed output: decrypt on the device and compare with the input exactly
    extra = {}
    if not args.no_decrypt:
        val = torch.empty(N, dtype=torch.float64, device=dev)
        stt = torch.empty(N, dtype=torch.int32, device=dev)
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record(stream)
        rc = lib.pai_decrypt_dev(ctx.handle, ct.data_ptr(), ex.data_ptr(), N, val.data_ptr(), None,
                                 stt.data_ptr(), None, stream.cuda_stream)
        d1.record(stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())
        torch.cuda.synchronize()
        dec_ms = d0.elapsed_time(d1)
        ok = bool(torch.equal(val, x.double())) and int((stt > 1).sum().item()) == 0
        extra["decrypt_per_s_per_gpu"] = N / (dec_ms * 1e-3)
        extra["decrypt_kernel_ms"] = dec_ms
        extra["roundtrip_exact"] = ok
        extra["decrypt_int_mac_frac"] = (N * canonical_w_dec(args.nb) / (dec_ms * 1e-3)) / INT_MAC_PEAK
        if not ok:
            raise SystemExit("decrypt(encrypt(x)) != x on the device")

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    value = world * N * args.steps / elapsed
    w_enc = canonical_w_enc(args.nb)
    achieved_mac = N * w_enc / (kern_ms * 1e-3)
    alg_bytes = 4 + W * 4 + 4     # x in, ciphertext out, exponent out (r generated on device)
    achieved_gbs = N * alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_encrypt_latest.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("n") == N and pm.get("nb") == args.nb:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if not args.no_cpu_baseline:
        from oracle import gmp_oracle
        if gmp_oracle.available():
            S = min(args.cpu_sample, N)
            th = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            t1 = time.perf_counter()
            cct, cex = gmp_oracle.encrypt_f32_chacha(pk.n, x_host[:S], rng_key, index_base, th)
            cdt = time.perf_counter() - t1
            # the sample doubles as a bit-exact parity check of the timed GPU output
            gct = ct[:S].cpu().numpy().view(np.uint32)
            same = bool(np.array_equal(gct, cct) and np.array_equal(ex[:S].cpu().numpy(), cex))
            cpu = {"value": S / cdt, "unit": "encrypts/s", "cores": th, "kind": "port",
                   "sample": f"first {S} elements of the rank-0 vector, same ChaCha20 r stream; "
                             f"GMP 6.2.1 mpz_powm per element (the library gmpy2 2.0.8 wraps), "
                             f"{th} worker threads like the reference's Pool(cpu_count())",
                   "gpu_bit_exact_on_sample": same}
            if not same:
                raise SystemExit("GPU ciphertexts differ from the GMP oracle on the CPU sample")

    out = {
        "metric": "Paillier-2048 encrypts/sec (device-resident), 1M-elem float32 array" if args.nb == 2048
        else f"Paillier-{args.nb} encrypts/sec (device-resident)",
        "value": value,
        "unit": "encrypts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: numpy default_rng(rank).standard_normal float32; seeded key generate_paillier_keypair(nb, seed=1)",
        "config": {"workload": f"Paillier n={args.nb} encrypt of a {N}-element float32 vector per GPU, "
                               f"device-resident, device ChaCha20 obfuscators"
                               + (", RCCL all-gather of ciphertext shards" if world > 1 else ""),
                   "key_bits": args.nb, "elements_per_gpu": N, "parallelism": f"dp{world}"},
        "roofline": {"bound": "valu-int-mac", "achieved": achieved_mac / 1e12, "peak": INT_MAC_PEAK / 1e12,
                     "unit": "TMAC/s", "frac": achieved_mac / INT_MAC_PEAK, "traffic": traffic,
                     "kernel": "k_encrypt", "kernel_ms": kern_ms,
                     "work_per_unit": f"{w_enc:.4g} 32x32->64 MAC per encrypt (SURVEY.md §8d canonical)"},
        "roofline_hbm": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_unit": alg_bytes},
        "cpu_baseline": cpu,
        "extra": extra,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
