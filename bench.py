#!/usr/bin/env python3
"""bench.py — Paillier-2048 array encryption on MI355X (BASELINE.json metric).

A step = one device-resident encryption of the rank's 1M-element float32 vector: fixed-point
encode -> c0 = 1 + n*m -> c0 * r^n mod n^2 with a device ChaCha20 obfuscator r per element
(flex/crypto/paillier/encryptor.py:71-114 semantics), then, for N > 1 GPUs, one RCCL all-gather of
the ciphertext shards so every rank holds the whole encrypted vector (weak scaling).

The workload (BASELINE.json configs[1]: "encrypt+decrypt on 1 MI355X") holds the private key, so
the default path is the key holder's: r^n sampled through fixed-base tables per CRT half
(kernels_fb.hpp, `--obf fixedbase`, digit window `--fb-window`, default 20) and recombined with c0
(k_crt_fin). The generic CRT path (`--obf generic`: r from the ChaCha20 stream, r^n by half-size
exponentiations, bit-identical to the public-key kernel and GMP), the public-key-only kernel,
device decryption, the configs[2] leg (8 arrays, 8-way add, decrypt) and the host-boundary rates
are measured on the same input in the same run, outside the timed region, under `extra`.
For N > 1 the ciphertext and exponent shards are double-buffered and step i's all-gather overlaps
step i+1's encryption.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--path crt|public] [--obf fixedbase|generic]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

Rank 0 prints ONE JSON line. `value` = encrypts/s over all ranks (max-over-ranks wall clock of the
K timed steps). `roofline` is for the dominant kernel of the timed path, timed live with HIP events
recorded on the launch stream between the kernels of every timed encrypt call; its work figure is
the SURVEY.md §8d canonical 32x32->64 MAC count. `cpu_baseline` is the
GMP restatement of the reference CPU path (oracle/gmp_oracle.c) on this host's cores, on a bounded
sample of the same workload, which doubles as a bit-exact check of the GPU output.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "ibond-flex_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# Peak 32x32->64 multiply-accumulate issue rate of one MI355X: v_mad_u64_u32 lanes/s measured by
# tools/microbench/int_throughput.hip, 16 independent chains, 32 waves/CU, 3.9 ms runs
# (profiles/r01_step0_int_throughput_long.txt).
INT_MAC_PEAK = float(os.environ.get("FLEXPAI_INT_MAC_PEAK", "35.13e12"))
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)


# ------------------------------------------------------------- canonical work
def _M(s: int) -> int:
    """Montgomery product of s 32-bit limbs: 2 s^2 + s MACs."""
    return 2 * s * s + s


def _P(b: int) -> int:
    """Products of a fixed-window-4 exponentiation with a b-bit exponent."""
    return (b - 1) + (b + 3) // 4 + 14 + 2


def work_enc_public(nb: int) -> float:
    return float((_P(nb) + 1) * _M(nb // 16))


def work_crt(nb: int) -> dict:
    """Per-element canonical MACs of the CRT encryption stages."""
    h = nb // 2
    return {"k_crt_a": float(2 * (_P(h) + 1) * _M(nb // 64)),      # (r mod p_h)^(e_h) mod p_h, both halves
            "k_crt_b": float(2 * (_P(h) + 2) * _M(nb // 32)),      # y^(p_h) * coef mod p_h^2, both halves
            "k_crt_fin": float(3 * _M(nb // 16))}                  # (u_p q^2 + u_q p^2) * c0 mod n^2


def fb_digit_count(nb: int, window: int) -> int:
    """Exponent digits K of the fixed-base sampler: window-bit digits of a_h mod (p_h - 1) (nb/2 bits)."""
    return -(-(nb // 2) // window)


def work_fb(nb: int, digits: int) -> dict:
    """Per-element MACs of the fixed-base path (kernels_fb.hpp), counted like SURVEY.md §8d (32-bit limbs,
    M(s) = 2 s^2 + s per Montgomery product): k_fb = K table products mod p_h^2 per half (the first one
    takes c0), no squarings; k_fb_fin (Garner) = one product mod p^2 + one plain (nb/32)^2 product; the
    ChaCha digit kernel does no MACs. This is NOT the public-key W_enc of §8d (a different algorithm)."""
    s = nb // 32
    return {"k_fb_digits": 0.0,
            "k_fb": float(2 * digits * _M(s)),
            "k_fb_fin": float(_M(s) + s * s)}


def work_dec(nb: int) -> float:
    return float(2 * (_P(nb // 2) + 2) * _M(nb // 32))


def load_traffic(kernel: str, n: int, nb: int):
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel}_latest.json")
    try:
        with open(path) as f:
            pm = json.load(f)
        if pm.get("n") == n and pm.get("nb") == nb:
            return pm.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 20, help="elements per GPU")
    ap.add_argument("--nb", type=int, default=2048, help="Paillier key bits")
    ap.add_argument("--path", choices=("crt", "public"), default="crt")
    ap.add_argument("--obf", choices=("fixedbase", "generic"), default="fixedbase",
                    help="device-RNG sampler of r^n on the CRT path (kernels_fb.hpp vs r from ChaCha20)")
    ap.add_argument("--fb-window", type=int, default=20, choices=(8, 12, 16, 20),
                    help="digit window of the fixed-base tables (20: 55 products per half, 17.5 GB table per half)")
    ap.add_argument("--cpu-sample", type=int, default=16384)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decrypt", action="store_true")
    ap.add_argument("--no-public", action="store_true", help="skip timing the public-key path beside CRT")
    ap.add_argument("--no-add8", action="store_true", help="skip the configs[2] leg (encrypt 8 arrays, 8-way add, decrypt)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-boundary (PCIe, Python objects) rates")
    ap.add_argument("--host-sample", type=int, default=1 << 16,
                    help="elements for the Python-object (PaillierEncryptor.encrypt) rate")
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
    from flex.crypto.paillier.sharding import gather_shards_async, shard_bounds

    pk, sk = generate_paillier_keypair(args.nb, seed=1)
    ctx = _native.Context(pk.n, local_rank, sk.p, sk.q)
    use_crt = args.path == "crt" and ctx.crt_available
    ctx.set_crt(use_crt)
    use_fb = use_crt and args.obf == "fixedbase"
    ctx.set_fixed_base(use_fb)
    use_fb = use_fb and ctx.fixed_base
    if use_fb:
        ctx.set_fb_window(args.fb_window)     # a dedicated encrypt GPU: 2 x 17.5 GB of tables at W = 20
    fb_info = ctx.fixed_base_info() if use_fb else None
    ctx.set_stage_timing(True)
    lib = _native.load_library()
    N, W = args.n, ctx.ct_words
    x_host = np.random.default_rng(rank).standard_normal(N, dtype=np.float32)
    x = torch.from_numpy(x_host).to(dev)
    ct = torch.empty((N, W), dtype=torch.int32, device=dev)
    ex = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)
    rng_key = hashlib.sha256(b"flexpai-bench-key").digest()
    total = world * N                 # weak scaling: N elements per GPU
    index_base, _ = shard_bounds(total, world, rank)   # obfuscators keyed by the GLOBAL element index
    stream = torch.cuda.current_stream(dev)

    def encrypt(out, exo=ex):
        rc = lib.pai_encrypt_dev(ctx.handle, _native.PAI_F32, x.data_ptr(), N, 0, 0, _native.PAI_OBF_RNG,
                                 None, 0, 0, rng_key, index_base, out.data_ptr(), exo.data_ptr(), st.data_ptr(),
                                 stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    # N > 1: double-buffered shards; step i's RCCL all-gather (ciphertexts + exponents) runs on the process
    # group's stream while step i+1 encrypts on the compute stream
    bufs = [(ct, ex)] + ([(torch.empty_like(ct), torch.empty_like(ex))] if world > 1 else [])
    works = [[] for _ in bufs]

    def step(i):
        b = i % len(bufs)
        for w in works[b]:
            w.wait()                   # the gather that last read this buffer is done
        works[b] = []
        encrypt(*bufs[b])
        if world > 1:
            for t in bufs[b]:
                _, w = gather_shards_async(t, total, world)
                if w is not None:
                    works[b].append(w)

    def drain():
        for b in range(len(bufs)):
            for w in works[b]:
                w.wait()
            works[b] = []

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stage_ms = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
        stage_ms.append(ctx.stage_times())     # HIP events recorded between this call's kernels
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ct, ex = bufs[(args.steps - 1) % len(bufs)]   # the last timed step's output (checked below)
    stage_avg = [float(np.mean([s[i] for s in stage_ms])) for i in range(len(stage_ms[0]))]
    S_chk = min(N, args.cpu_sample)
    ct_timed_check = ct[:S_chk].cpu().numpy().view(np.uint32).copy()
    ex_timed_check = ex[:S_chk].cpu().numpy().copy()

    extra = {}
    # Fixed-base sampling (kernels_fb.hpp) draws r^n directly, so its ciphertexts are not the ones of
    # the ChaCha r stream; the generic CRT path on the same input (untimed) is the bit-reproducible
    # reference the public-key kernel and the GMP CPU baseline are compared with.
    ct_ref = ct
    if use_fb:
        ct_ref = torch.empty_like(ct)
        ctx.set_fixed_base(False)
        encrypt(ct_ref)
        encrypt(ct_ref)
        gen_ms = ctx.stage_times()
        ctx.set_fixed_base(True)
        torch.cuda.synchronize()
        wc = work_crt(args.nb)
        extra["generic_crt_path"] = {
            "value": N / (sum(gen_ms) * 1e-3), "unit": "encrypts/s per GPU",
            "note": "r from the ChaCha20 stream and r^n by CRT exponentiation (kernels_crt.hpp); "
                    "bit-identical to the public-key kernel and the GMP baseline",
            "stages_ms": dict(zip(["k_crt_a", "k_crt_b", "k_crt_fin"], gen_ms)),
            "k_crt_b_int_mac_frac": N * wc["k_crt_b"] / (gen_ms[1] * 1e-3) / INT_MAC_PEAK if len(gen_ms) > 1 else None}
    ct_host_check = ct_ref[:S_chk].cpu().numpy().view(np.uint32).copy()
    ex_host_check = ex[:S_chk].cpu().numpy().copy()

    # the public-key path on the same input (untimed region), for the record and as a parity check
    if use_crt and not args.no_public:
        ct2 = torch.empty_like(ct)
        ctx.set_crt(False)
        encrypt(ct2)
        pub_ms = ctx.stage_times()[0]
        ctx.set_crt(True)
        torch.cuda.synchronize()
        same = bool(torch.equal(ct2, ct_ref))
        extra["public_key_path"] = {"value": N / (pub_ms * 1e-3), "unit": "encrypts/s per GPU",
                                    "kernel": "k_encrypt", "kernel_ms": pub_ms,
                                    "int_mac_frac": N * work_enc_public(args.nb) / (pub_ms * 1e-3) / INT_MAC_PEAK,
                                    "bit_identical_to_crt": same}
        del ct2
        if not same:
            raise SystemExit("CRT and public-key ciphertexts differ")

    # correctness of the timed output: decrypt on the device and compare with the input exactly
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
        dst = ctx.stage_times()
        if ctx.lane_decrypt and len(dst) == 3:
            wd = work_dec(args.nb)
            extra["decrypt_stages"] = {
                "k_dec_pre": {"kernel_ms": dst[0]},
                "k_dec_pow": {"kernel_ms": dst[1], "work_mac_per_elem": wd,
                              "achieved_tmac_s": N * wd / (dst[1] * 1e-3) / 1e12},
                "k_dec_fin": {"kernel_ms": dst[2]}}
        extra["decrypt_path"] = "lane" if ctx.lane_decrypt else "group"
        ok = bool(torch.equal(val, x.double())) and int((stt > 1).sum().item()) == 0
        extra["decrypt_per_s_per_gpu"] = N / (dec_ms * 1e-3)
        extra["decrypt_kernel_ms"] = dec_ms
        extra["decrypt_int_mac_frac"] = N * work_dec(args.nb) / (dec_ms * 1e-3) / INT_MAC_PEAK
        extra["roundtrip_exact"] = ok
        if not ok:
            raise SystemExit("decrypt(encrypt(x)) != x on the device")

    # configs[2]: encrypt 8 arrays (default_rng(k), k = 0..7), one 8-way homomorphic add (k_add), decrypt the
    # sum; device-resident, HIP events on the launch stream; the decrypted sum is checked against float64
    if not args.no_add8 and not args.no_decrypt:
        K8 = 8
        xs8 = torch.stack([torch.from_numpy(np.random.default_rng(k).standard_normal(N, dtype=np.float32))
                           for k in range(K8)]).to(dev)
        cts8 = torch.empty((K8, N, W), dtype=torch.int32, device=dev)
        exs8 = torch.empty((K8, N), dtype=torch.int32, device=dev)
        sum_ct = torch.empty((N, W), dtype=torch.int32, device=dev)
        sum_ex = torch.empty(N, dtype=torch.int32, device=dev)
        val8 = torch.empty(N, dtype=torch.float64, device=dev)
        st8 = torch.empty(N, dtype=torch.int32, device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        torch.cuda.synchronize()
        t8 = time.perf_counter()
        ev[0].record(stream)
        for k in range(K8):
            rc = lib.pai_encrypt_dev(ctx.handle, _native.PAI_F32, xs8[k].data_ptr(), N, 0, 0, _native.PAI_OBF_RNG,
                                     None, 0, 0, rng_key, index_base + (k + 1) * total, cts8[k].data_ptr(),
                                     exs8[k].data_ptr(), st.data_ptr(), stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(lib.pai_last_error().decode())
        ev[1].record(stream)
        rc = lib.pai_add_dev(ctx.handle, cts8.data_ptr(), exs8.data_ptr(), K8, N, sum_ct.data_ptr(),
                             sum_ex.data_ptr(), stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())
        ev[2].record(stream)
        rc = lib.pai_decrypt_dev(ctx.handle, sum_ct.data_ptr(), sum_ex.data_ptr(), N, val8.data_ptr(), None,
                                 st8.data_ptr(), None, stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())
        ev[3].record(stream)
        torch.cuda.synchronize()
        wall8 = time.perf_counter() - t8
        ref = xs8.double().sum(0)
        err = float((val8 - ref).abs().max().item())
        add_ms = ev[1].elapsed_time(ev[2])
        # canonical add work: (k-1) products + 4 d squarings per operand aligned by d
        E = exs8.max(0).values
        sq = int((4 * (E.unsqueeze(0) - exs8)).sum().item())
        add_work = (N * (K8 - 1) + sq) * _M(args.nb // 16)
        extra["config3_add8"] = {
            "workload": "configs[2]: encrypt 8 x 1M float32 arrays, one 8-way add, decrypt the sum (device-resident)",
            "elements_per_s": N / wall8, "wall_s": wall8,
            "encrypt8_ms": ev[0].elapsed_time(ev[1]), "k_add_ms": add_ms, "decrypt_ms": ev[2].elapsed_time(ev[3]),
            "k_add_int_mac_frac": add_work / (add_ms * 1e-3) / INT_MAC_PEAK,
            "k_add_alignment_squarings_per_elem": sq / N,
            "max_abs_err_vs_float64_sum": err, "statuses_ok": int((st8 > 1).sum().item()) == 0}
        del xs8, cts8, exs8, sum_ct, sum_ex, val8, st8
        torch.cuda.empty_cache()

    # host boundary (DESIGN.md §Host boundary): plaintexts start in host numpy and ciphertexts leave as
    # host buffers / PaillierEncryptedNumber objects; never part of `value`
    if not args.no_host and rank == 0:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hct, hex_, _ = ctx.encrypt(x_host, obf_mode=_native.PAI_OBF_RNG, rng_key=rng_key, index_base=index_base)
        t_host = time.perf_counter() - t1
        hb = {"host_buffers_encrypts_per_s": N / t_host,
              "host_buffers_note": "pai_encrypt: H2D float32 x, kernels, D2H ciphertext words "
                                   f"({N * W * 4 / 2**20:.0f} MiB), pageable host memory",
              "host_buffers_bit_identical": bool(np.array_equal(hct[: len(ct_timed_check)], ct_timed_check))}
        from flex.crypto.paillier import _runtime
        from flex.crypto.paillier.encryptor import PaillierEncryptor
        _runtime.register_private(pk, sk)        # this process holds the key (CRT path, as above)
        enc = PaillierEncryptor(pk)
        hs = min(args.host_sample, N)
        t1 = time.perf_counter()
        objs = enc.encrypt(x_host[:hs])
        t_obj = time.perf_counter() - t1
        hb["python_objects_encrypts_per_s"] = hs / t_obj
        hb["python_objects_note"] = (f"PaillierEncryptor.encrypt(ndarray[{hs}]) -> object ndarray of "
                                     "PaillierEncryptedNumber (encryptor.py:99-114 API), incl. materialisation")
        del objs
        extra["host_boundary"] = hb

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    value = world * N * args.steps / elapsed
    if use_crt:
        if use_fb:
            names = ["k_fb_digits", "k_fb", "k_fb_fin"]
            works = work_fb(args.nb, fb_info[2])
        else:
            names = ["k_crt_a", "k_crt_b", "k_crt_fin"]
            works = work_crt(args.nb)
        stages = {nm: {"kernel_ms": ms, "work_mac_per_elem": works[nm],
                       "achieved_tmac_s": N * works[nm] / (ms * 1e-3) / 1e12}
                  for nm, ms in zip(names, stage_avg)}
        dom = max(names, key=lambda nm: stages[nm]["kernel_ms"])
        dom_ms, dom_work = stages[dom]["kernel_ms"], works[dom]
        extra["stages"] = stages
        total_work = sum(works.values())
    else:
        dom, dom_ms, dom_work = "k_encrypt", stage_avg[0], work_enc_public(args.nb)
        total_work = dom_work
    achieved = N * dom_work / (dom_ms * 1e-3)
    alg_bytes = 4 + W * 4 + 4     # x in, ciphertext out, exponent out (r generated on the device)
    extra["path"] = ("crt-fixedbase" if use_fb else "crt") if use_crt else "public"
    if use_fb:
        extra["fixed_base"] = {"g_p": fb_info[0], "g_q": fb_info[1], "digits": fb_info[2],
                               "window_bits": fb_info[3] if len(fb_info) > 3 else 8}
    extra["encrypt_call_ms"] = float(sum(stage_avg))
    extra["path_int_mac_frac"] = N * total_work / (sum(stage_avg) * 1e-3) / INT_MAC_PEAK
    extra["hbm_algorithmic_gbs"] = N * alg_bytes / (sum(stage_avg) * 1e-3) / 1e9

    cpu = None
    if not args.no_cpu_baseline:
        from oracle import gmp_oracle
        if gmp_oracle.available():
            S = min(args.cpu_sample, N)
            th = max(1, min(args.cpu_threads, os.cpu_count() or 1))
            t1 = time.perf_counter()
            cct, cex = gmp_oracle.encrypt_f32_chacha(pk.n, x_host[:S], rng_key, index_base, th)
            cdt = time.perf_counter() - t1
            same = bool(np.array_equal(ct_host_check[:S], cct) and np.array_equal(ex_host_check[:S], cex))
            cpu = {"value": S / cdt, "unit": "encrypts/s", "cores": th, "kind": "port",
                   "sample": f"first {S} elements of the rank-0 vector with the same ChaCha20 obfuscators; "
                             f"GMP 6.2.1 mpz_powm(r, n, n^2) per element (the library gmpy2 2.0.8 wraps, "
                             f"obfuscator.py:36), {th} worker threads like the reference's Pool(cpu_count())",
                   "gpu_bit_exact_on_sample": same}
            if not same:
                raise SystemExit("GPU ciphertexts differ from the GMP oracle on the CPU sample")
            if use_fb:
                # the timed (fixed-base) ciphertexts against the oracle's restatement of the sampler
                from oracle import paillier_oracle as O
                okey = O.Key(pk.n, sk.p, sk.q)
                idx = sorted({0, 1, S_chk // 2, S_chk - 1})
                got = _native.words_to_ints(ct_timed_check[idx])
                fb_ok = all(O.fb_encrypt_value(x_host[i], okey, rng_key, index_base + i, fb_info)
                            == (got[j], int(ex_timed_check[i])) for j, i in enumerate(idx))
                cpu["fixed_base_bit_exact_vs_oracle"] = {"elements": idx, "ok": fb_ok}
                if not fb_ok:
                    raise SystemExit("fixed-base ciphertexts differ from the oracle restatement")

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
        "data": "synthetic: numpy default_rng(rank).standard_normal float32; seeded key "
                "generate_paillier_keypair(nb, seed=1); device ChaCha20 obfuscators keyed by global index",
        "config": {"workload": f"Paillier n={args.nb} encrypt of a {N}-element float32 vector per GPU, "
                               f"device-resident, key holder ({('CRT, fixed-base r^n sampler' if use_fb else 'CRT') if use_crt else 'public-key'} path)"
                               + (", RCCL all-gather of ciphertext shards" if world > 1 else ""),
                   "key_bits": args.nb, "elements_per_gpu": N, "parallelism": f"dp{world}"},
        "roofline": {"bound": "valu-int-mac", "achieved": achieved / 1e12, "peak": INT_MAC_PEAK / 1e12,
                     "unit": "TMAC/s", "frac": achieved / INT_MAC_PEAK,
                     "traffic": load_traffic(dom, N, args.nb),
                     "kernel": dom, "kernel_ms": dom_ms,
                     "work_per_unit": f"{dom_work:.4g} canonical 32x32->64 MAC per element (SURVEY.md §8d)"},
        "roofline_hbm": {"bound": "hbm", "achieved": extra["hbm_algorithmic_gbs"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": extra["hbm_algorithmic_gbs"] / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_unit": alg_bytes},
        "cpu_baseline": cpu,
        "extra": extra,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
