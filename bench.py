#!/usr/bin/env python3
"""bench.py — Paillier array encryption on MI355X (BASELINE.json metric and configs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {0,1,2,3,4}] ...
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL over xGMI)

`--gpus N > 1` without a torch.distributed launcher (no WORLD_SIZE in the environment) starts the N rank
processes itself, before anything touches the GPU (launch_ranks), and exits with the first failing rank's
code; under torchrun the ranks come from the environment.

Workloads (BASELINE.json configs; synthetic float32 N(0,1) vectors, seeded keys):
  --config 1 (default at every N): nb = 2048, 1 048 576 elements per GPU, device-resident encryption
             (the headline metric "Paillier-2048 encrypts/sec (device-resident), 1M-elem float32 array");
             weak scaling, no data-path collective (elements are independent). The same run times the
             configs[3] leg below as `extra.config3_strong` unless --no-strong;
  --config 3: nb = 2048, 16 777 216 elements in total, sharded over the N ranks
             (strong scaling: 2M per GPU at N = 8), ciphertext shards reassembled on every rank by an
             RCCL all-gather inside the timed step (double-buffered: step i's gather overlaps step i+1);
  --config 4: nb = 4096, 4 194 304 elements in total, sharded like config 3;
  --config 2: nb = 2048, 1M elements: a step = encrypt 8 arrays + one 8-way homomorphic add + decrypt;
  --config 0: nb = 1024, 1000 elements (the reference's plumbing case; its CPU leg is timed in full).
A step = one pass of the hot path over the rank's shard, obfuscators from the device ChaCha20 stream
keyed by the GLOBAL element index (ciphertexts do not depend on N). A key holder encrypts through the
fixed-base sampler (kernels_fb.hpp; its tables are built, and timed under `setup`, before the timed
region). `value` = elements of the whole job per second over the K timed steps (barrier + synchronize
on both sides, max over ranks).

Rank 0 prints ONE JSON line. `roofline` is for the dominant kernel of the timed path, its duration
timed live with HIP events recorded on the launch stream between the kernels of every timed call; its
work figure is that kernel's own MAC count (the fixed-base count for k_fb, NOT SURVEY.md §8d's public-
key W_enc, which is reported beside it as `w_enc_equivalent`). `cpu_baseline` (N = 1 only) is the GMP
restatement of the reference CPU path (oracle/gmp_oracle.c; threads = the process's CPU share -- its
affinity mask capped by the cgroup CPU quota, which on a shared GPU box is far below os.cpu_count() -- like
the reference's Pool(cpu_count())) on a bounded sample of the same workload, which doubles as a bit-exact
check of the GPU output; a one-thread run of the first elements gives the per-core rate and
`cores_effective` = threaded rate / per-core rate; `extra.config0_cpu` times configs[0] (nb = 1024, 1k elements) in full.
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

# Peak 32x32->64 multiply-accumulate issue rate of one MI355X: v_mad_u64_u32 lanes/s measured by
# tools/microbench/int_throughput.hip, 16 independent chains, 32 waves/CU, 3.9 ms runs
# (profiles/r01_step0_int_throughput_long.txt).
INT_MAC_PEAK = float(os.environ.get("FLEXPAI_INT_MAC_PEAK", "35.13e12"))
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    0: {"nb": 1024, "total": 1000, "shard": "strong",
        "desc": "configs[0]: Paillier n=1024, 1k-element float32 vector (the reference's CPU plumbing case)"},
    1: {"nb": 2048, "total": 1 << 20, "shard": "weak",
        "desc": "configs[1]: Paillier n=2048, 1M-element float32 vector per GPU, device-resident encrypt (+decrypt)"},
    2: {"nb": 2048, "total": 1 << 20, "shard": "weak",
        "desc": "configs[2]: Paillier n=2048, encrypt 8 x 1M float32 arrays + one 8-way homomorphic add + decrypt"},
    3: {"nb": 2048, "total": 16 << 20, "shard": "strong",
        "desc": "configs[3]: Paillier n=2048, 16M-element float32 vector sharded over the GPUs, RCCL all-gather"},
    4: {"nb": 4096, "total": 4 << 20, "shard": "strong",
        "desc": "configs[4]: Paillier n=4096, 4M-element float32 vector sharded over the GPUs, RCCL all-gather"},
}


# ------------------------------------------------------------- canonical work
def _M(s: int) -> int:
    """Montgomery product of s 32-bit limbs: 2 s^2 + s MACs."""
    return 2 * s * s + s


def _P(b: int) -> int:
    """Products of a fixed-window-4 exponentiation with a b-bit exponent."""
    return (b - 1) + (b + 3) // 4 + 14 + 2


def work_enc_public(nb: int) -> float:
    """SURVEY.md §8d W_enc: the public-key encryption's canonical MACs per element."""
    return float((_P(nb) + 1) * _M(nb // 16))


def work_crt(nb: int) -> dict:
    """Per-element canonical MACs of the generic CRT encryption stages."""
    h = nb // 2
    return {"k_crt_a": float(2 * (_P(h) + 1) * _M(nb // 64)),      # (r mod p_h)^(e_h) mod p_h, both halves
            "k_crt_b": float(2 * (_P(h) + 2) * _M(nb // 32)),      # y^(p_h) * coef mod p_h^2, both halves
            "k_crt_fin": float(3 * _M(nb // 16))}                  # (u_p q^2 + u_q p^2) * c0 mod n^2


def work_fb(nb: int, digits: int) -> dict:
    """Per-element MACs of the fixed-base path (kernels_fb.hpp), counted like SURVEY.md §8d (32-bit limbs,
    M(s) = 2 s^2 + s per Montgomery product): k_fb = K table products mod p_h^2 per half (the first one
    takes c0), no squarings; k_fb_fin (Garner) = one product mod p^2 + one plain (nb/32)^2 product; the
    ChaCha digit kernel does no MACs. This is NOT the public-key W_enc of §8d (a different algorithm)."""
    s = nb // 32
    return {"k_fb_digits": 0.0, "k_fb": float(2 * digits * _M(s)), "k_fb_fin": float(_M(s) + s * s)}


def _Mp(s: int) -> int:
    """Pair product mod p^2 over s 32-bit limbs of p (bn_pair.hpp): A1 A2 + q1 p, and B1 A2 + A1 B2 + q2 p,
    5 s^2 MACs, + 2 s for the two digit reductions (the analogue of M(s)'s + s)."""
    return 5 * s * s + 2 * s


def work_fbp(nb: int, digits: int) -> dict:
    """Per-element MACs of the pair fixed-base path (kernels_fbp.hpp): k_fbp = K products by factored rows (a_k, 0)
    per half (s = nb/64 limbs of p_h, 4 s^2 + 2 s each) + the c0 chunk sum (s^2) + the b-sum correction
    B += REDC(A bs) (one s-limb Montgomery product, M(s)); k_fbp_fin = Garner on pairs: q B_q (4 s^2, B row
    zero), h (5 s^2), c = A_q + q B_q + q^2 H_A + p q^2 H_B (6 s^2)."""
    s = nb // 64
    return {"k_fb_digits": 0.0, "k_fbp": float(2 * (digits * _Mf(s) + s * s + _M(s))), "k_fbp_fin": float(15 * s * s)}


def work_fbs(nb: int, digits: int) -> dict:
    """The pair fixed-base path on Shoup rows (kernels_fbs.hpp): k_fbs = K - 1 Shoup products per half (the first row
    is the start (a_0, 0), c0's gamma R joins the b sum; s = nb/64 limbs of p_h; per component a quotient from the top
    s (s + 1) / 2 columns of X a' and the low s (s + 1) / 2 columns of X a and of Q p: 3 s^2 + 3 s per pair) + the c0
    chunk sum (s^2) + the b-sum correction (M(s)); k_fbp_fin: Y = w_q q^-2 in one two-operand pass (6 s^2) and the
    final sum (6 s^2)."""
    s = nb // 64
    return {"k_fb_digits": 0.0, "k_fbs": float(2 * ((digits - 1) * (3 * s * s + 3 * s) + s * s + _M(s))),
            "k_fbp_fin": float(12 * s * s)}


def work_fbg(nb: int, digits: int) -> dict:
    """Per-element MACs of the 4096-bit key holder's fixed-base path (kernels_grp.hpp), counted like work_fb:
    k_fbg = K table products mod p_h^2 per half (c0 folded into the first); Garner = one product mod p^2
    (k_fbg_garner) + one product mod n^2 (k_fbg_fin), timed together."""
    s = nb // 32
    return {"k_fb_digits": 0.0, "k_fbg": float(2 * digits * _M(s)), "k_fbg_fin": float(_M(s) + _M(nb // 16))}


def _Mf(s: int) -> int:
    """Pair product by a factored row (a, 0) (kernels_grp_pair.hpp): A a + q1 p, B a + q2 p: 4 s^2 + 2 s."""
    return 4 * s * s + 2 * s


def work_fbgp(nb: int, digits: int) -> dict:
    """The 4096-bit sampler on pair groups with factored rows (kernels_grp_pair.hpp): K products by (a_k, 0) per half
    over the nb/64 32-bit limbs of p_h, plus the correction B += REDC(A bs) (one s-limb Montgomery product, M(s));
    the fin stage adds k_fbgp_w's product mod p_h^2 per half to the Garner work."""
    s = nb // 64
    return {"k_fb_digits": 0.0, "k_fbgp": float(2 * (digits * _Mf(s) + _M(s))),
            "k_fbg_fin": float(2 * _M(nb // 32) + _M(nb // 32) + _M(nb // 16))}


def work_sgs(nb: int, digits: int) -> float:
    """The 4096-bit sampler on Shoup rows ($FLEXPAI_SGS=1, kernels_sgs.hpp): K - 1 Shoup products per half (3 s^2 + 3 s
    over the nb/64 32-bit limbs of p_h, as k_fbs's count) and k_sgs_bfin's split pass by the constant c_A (4 s^2 + 2 s)
    and b-sum product M(s)."""
    s = nb // 64
    return float(2 * ((digits - 1) * (3 * s * s + 3 * s) + _Mf(s) + _M(s)))


def work_sgp_fin(nb: int) -> float:
    """The 4096-bit split-pair path's fin stage (round 5): k_sgp_w's plain product p_h B per half ((nb/64)^2 each),
    k_fbg_garner's product mod p^2 (M(nb/32)) and k_sgp_fin's two plain products by q (q h: (nb/64)(nb/32), q t:
    (nb/64)(3 nb/64)), canonical 32-bit limbs."""
    s = nb // 64
    return float(2 * s * s + _M(nb // 32) + s * (2 * s) + s * (3 * s))


def work_pfb(nb: int, digits: int) -> float:
    """Public fixed bases (kernels_pfb.hpp): K products by factored rows over the nb/32 32-bit limbs of n, plus the
    correction (one Montgomery product mod n)."""
    s = nb // 32
    return float(digits * _Mf(s) + _M(s))


def work_dec(nb: int) -> float:
    return float(2 * (_P(nb // 2) + 2) * _M(nb // 32))


def work_dec_pair(nb: int) -> float:
    """W_dec with every product mod p_h^2 a pair product over the nb/64 32-bit limbs of p_h (kernels_pair.hpp;
    squarings counted as products, like §8d's W_dec)."""
    return float(2 * (_P(nb // 2) + 2) * _Mp(nb // 64))


def work_add(exps: "torch.Tensor", nb: int) -> float:
    """Canonical k-way add work over [k][N] exponents: per element (k - 1) products plus
    4 d squarings per operand aligned by d (the reference's per-operand alignment)."""
    k, n = exps.shape
    E = exps.max(0).values
    sq = int((4 * (E.unsqueeze(0) - exps)).sum().item())
    return float((n * (k - 1) + sq) * _M(nb // 16))


# ------------------------------------------------------------- per-rank HBM plan
FB_ROW_BYTES = {1024: 224, 2048: 448, 4096: 512}   # Shoup rows (k_fbs) at 1024/2048, factored word rows at 4096 (+ 640-B
                                                    # Shoup rows beside them for k_sgs, fb_table_bytes)
FB_WINDOWS = (24, 23, 22, 21, 20, 16, 12, 8)        # the library's ladder (flexpai.hip ensure_fb)
GiB = 1 << 30


def sgs_enabled() -> bool:
    """The 4096-bit key holder's Shoup-row sampler (kernels_sgs.hpp; off with $FLEXPAI_SGS=0), whose 640-B rows sit
    beside the factored rows: at the windows a dedicated MI355X allows the library takes them (flexpai.hip fb_choose:
    W = 20 with them prices below W = 21 without)."""
    return os.environ.get("FLEXPAI_SGS", "") != "0"


def fb_table_bytes(nb: int, w: int) -> int:
    """Both halves' fixed-base tables at window w: 2 x K x 2^w rows, K = ceil(bits(p_h - 1) / w) (fb_digit_count)."""
    row = FB_ROW_BYTES[nb] + (640 if nb == 4096 and sgs_enabled() else 0)
    return 2 * (-(-(nb // 2) // w)) * (1 << w) * row


def fb_reserve(device_bytes: int) -> int:
    """What the library keeps free beside its tables (flexpai.hip fb_budget): max(4 GiB, 1/12 of the device)."""
    return max(4 * GiB, device_bytes // 12)


def rank_memory_plan(cfg_id: int, world: int, nb: int, strong_leg: bool = True) -> dict:
    """Bytes one rank allocates beside the fixed-base tables for the timed legs of bench.py: the shard outputs
    (double-buffered at N > 1) and the all-gather receive buffers, the library's per-chunk work (digits + pairs of at
    most CRT_CHUNK = 4M elements), the decrypt check, and an allowance for RCCL and the torch context."""
    W = 2 * nb // 32                         # ciphertext words
    ctb = W * 4 + 4                          # ciphertext + exponent bytes per element
    K = -(-(nb // 2) // 16)                  # digits per half at the smallest window the legs might see (upper bound)
    S2 = 2 * (nb // 64 + 5)                  # words of a pair (2 S limbs) per half, rounded up
    work = 2 * K * 4 + 2 * S2 * 4            # library work per element of a chunk: digits + pairs
    if nb == 4096 and sgs_enabled():
        work += 2 * (16 * 16 + 2 * 4)        # + k_sgs's b sums
    dec = 8 + 4 + 2 * 2 * S2 * 4             # decrypt check: value + status + the library's pair outputs

    def leg(total, shard):
        n = -(-total // world) if shard == "strong" else total
        nb_ = 2 if world > 1 else 1
        return {"shard_outputs": nb_ * n * ctb + 8 * n,                     # + input and status
                "gathered_outputs": nb_ * world * n * ctb if world > 1 else 0,
                "library_work": min(n, 4 << 20) * work,
                "decrypt_check": min(n, 2 << 20) * dec}

    plan = {f"config{cfg_id}": leg(CONFIGS[cfg_id]["total"], CONFIGS[cfg_id]["shard"])}
    if cfg_id == 1 and strong_leg and nb == 2048:
        plan["config3_leg"] = leg(CONFIGS[3]["total"], "strong")
    plan["rccl_and_runtime_allowance"] = 3 * GiB
    return plan


def plan_total(plan: dict) -> int:
    return sum(v if isinstance(v, int) else sum(v.values()) for v in plan.values())


def preflight_window(cfg_id: int, world: int, nb: int, fb_window: int, device_bytes: int, strong_leg: bool = True) -> dict:
    """The window the tables can have on this device beside every leg: the largest w <= fb_window of the library's
    ladder with tables + the legs' plan + the library's reserve <= device memory; and the window the tables alone
    would get. bench.py refuses to run (SystemExit) when the legs would force a smaller window than the tables alone,
    or when the library then builds a smaller one than planned: a silently smaller W is a different measurement."""
    legs = plan_total(rank_memory_plan(cfg_id, world, nb, strong_leg))
    res = fb_reserve(device_bytes)
    alone = next((w for w in FB_WINDOWS if w <= fb_window and fb_table_bytes(nb, w) + res <= device_bytes), None)
    both = next((w for w in FB_WINDOWS if w <= fb_window and fb_table_bytes(nb, w) + max(res, legs) <= device_bytes), None)
    return {"window": both, "window_tables_alone": alone, "legs_bytes": legs, "reserve_bytes": res,
            "tables_bytes": fb_table_bytes(nb, both) if both else None, "device_bytes": device_bytes,
            "ok": both is not None and both == alone}


def lib_sha16() -> str:
    """sha256 (16 hex digits) of the libflexpai.so this process runs."""
    from flex.crypto.paillier import _native
    with open(_native.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(kernel: str, n: int, nb: int, window=None):
    """Measured HBM bytes per launch of `kernel` (profiles/pmc_<kernel>_latest.json, tools/pmc_traffic.py),
    only when that profile was taken at the same size, key and fixed-base window AND of the same library binary
    (lib_sha16): a profile of an older build is not reported as this build's traffic."""
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel}_latest.json")
    try:
        with open(path) as f:
            pm = json.load(f)
        if (pm.get("n") == n and pm.get("nb") == nb and pm.get("window") == window
                and pm.get("lib_sha16") == lib_sha16()):
            return pm.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota() -> dict:
    """The CPU share this process may use: the cgroup CPU quota (v2 cpu.max, or v1 cfs_quota_us /
    cfs_period_us) of its own cgroup, and the affinity mask. os.cpu_count() counts the whole machine, which on
    a shared GPU box is many times the process's share (256 threads delivered ~17 cores of work)."""
    out = {"os_cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "cgroup_quota_cores": None, "cgroup_quota_source": None}
    rel = {}
    try:
        with open("/proc/self/cgroup") as f:
            for line in f:
                _, ctrl, path = line.rstrip("\n").split(":", 2)
                for c in (ctrl.split(",") if ctrl else [""]):
                    rel[c] = path
    except OSError:
        pass
    cands = []
    if "" in rel:                                    # cgroup v2: walk up from our group to the root
        p = rel[""]
        while True:
            cands.append(("v2", os.path.join("/sys/fs/cgroup", p.lstrip("/"), "cpu.max")))
            if p in ("/", ""):
                break
            p = os.path.dirname(p)
    for key in ("cpu", "cpu,cpuacct"):
        if key in rel:
            for base in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
                cands.append(("v1", os.path.join(base, rel[key].lstrip("/"))))
                cands.append(("v1", base))
    best = None
    for kind, path in cands:
        try:
            if kind == "v2":
                with open(path) as f:
                    q, per = f.read().split()[:2]
                if q != "max":
                    v = int(q) / int(per)
                    best = (v, path) if best is None or v < best[0] else best
            else:
                with open(os.path.join(path, "cpu.cfs_quota_us")) as f:
                    q = int(f.read())
                with open(os.path.join(path, "cpu.cfs_period_us")) as f:
                    per = int(f.read())
                if q > 0:
                    v = q / per
                    best = (v, path) if best is None or v < best[0] else best
        except (OSError, ValueError):
            continue
    if best is not None:
        out["cgroup_quota_cores"], out["cgroup_quota_source"] = round(best[0], 2), best[1]
    return out


def cpu_threads_default() -> int:
    """Worker threads for the CPU baseline: the affinity mask, capped by the cgroup quota when one is set."""
    q = cpu_quota()
    n = q["affinity_cpus"] or 1
    if q["cgroup_quota_cores"]:
        n = min(n, max(1, int(q["cgroup_quota_cores"] + 0.5)))
    return n


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`--gpus n` with no launcher: start n fresh rank processes of this script (RANK = LOCAL_RANK = r,
    WORLD_SIZE = n, MASTER_ADDR = 127.0.0.1) and wait for them. Called before any GPU call in this process
    (importing torch and parsing arguments touch no device). The first rank that fails ends the others
    (their exact PIDs) and its exit code is returned; rank 0 prints the JSON line."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


# ------------------------------------------------------------- the timed step of the sharded legs
def step_base(rank_base: int, stride: int, i: int) -> int:
    """The obfuscator index base of step i: the rank's first global index + i x the job's elements per step, so that no
    two steps of a run encrypt under the same obfuscators (nothing in the timed region could be served from a cache)
    and the ciphertexts still do not depend on the number of ranks."""
    return rank_base + i * stride


def job_units(shard: str, total: int, world: int, n: int, steps: int) -> int:
    """Elements of the whole job over `steps` steps: strong = the fixed total, weak = n per rank."""
    return (total if shard == "strong" else world * n) * steps


class ShardSteps:
    """The step of configs[1]/[3]/[4] and of the configs[3] leg, the same code at every world size and on every backend.

    Step i encrypts this rank's shard (`encrypt(out_words, out_exps, base)`, base = step_base(rank_base, stride, i))
    into output buffer i % nbuf; at world > 1 it then starts the all-gather of that buffer's words and exponents into
    the matching receive buffers (`gather_async(local, rows, world, out=recv) -> (view, work|None)`, sharding.
    gather_shards_async: RCCL on the process group's stream on GPUs, gloo in the CPU tests). With two buffers step i's
    gather runs while step i + 1 encrypts; a buffer is written again only after the gather that read it has completed
    (the waits at the top of step). `rows` = world x the per-rank row count (the last shard is padded)."""

    def __init__(self, encrypt, bufs, recv, world, rank_base, stride, gather_async=None):
        if world > 1 and len(recv) != len(bufs):
            raise ValueError("one receive pair per output buffer")
        self.encrypt, self.bufs, self.recv, self.world = encrypt, bufs, recv, world
        self.rank_base, self.stride, self.gather_async = rank_base, stride, gather_async
        self.works = [[] for _ in bufs]
        self.rows = bufs[0][0].shape[0] * world
        self.last_i = None

    def base(self, i: int) -> int:
        return step_base(self.rank_base, self.stride, i)

    def buffer(self, i: int) -> int:
        return i % len(self.bufs)

    def step(self, i: int) -> None:
        b = self.buffer(i)
        for w in self.works[b]:
            w.wait()                         # the gather that last read this buffer is done
        self.works[b] = []
        self.encrypt(self.bufs[b][0], self.bufs[b][1], self.base(i))
        if self.world > 1:
            for t, o in zip(self.bufs[b], self.recv[b]):
                _, w = self.gather_async(t, self.rows, self.world, out=o)
                if w is not None:
                    self.works[b].append(w)
        self.last_i = i

    def drain(self) -> None:
        for b in range(len(self.bufs)):
            for w in self.works[b]:
                w.wait()
            self.works[b] = []

    def pending(self, b: int) -> int:
        return len(self.works[b])

    def last_output(self):
        """(words, exponents) of the last step, and its receive pair at world > 1 (None at world 1)."""
        b = self.buffer(self.last_i)
        return self.bufs[b], (self.recv[b] if self.world > 1 else None)

    def own_shard_identical(self, rank: int) -> bool:
        """This rank's block of the last step's gathered arrays equals its own output (call after drain)."""
        (ct, ex), rv = self.last_output()
        n = ct.shape[0]
        return all(bool(torch.equal(g[rank * n:(rank + 1) * n], t)) for g, t in zip(rv, (ct, ex)))


def run_timed(stepper, steps: int, warmup: int, sync, barrier, max_over_ranks, after_step=None) -> float:
    """`warmup` untimed steps, then exactly `steps` timed ones bracketed by drain + sync + barrier + sync on both sides;
    returns the MAX over ranks of the timed region's wall time. Timed step i runs as stepper.step(warmup + i), so its
    obfuscators differ from every warmup step's. after_step() (host bookkeeping, e.g. reading the stage events) runs
    after each timed step."""
    for i in range(warmup):
        stepper.step(i)
    stepper.drain()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        stepper.step(warmup + i)
        if after_step is not None:
            after_step()
    stepper.drain()
    sync()
    barrier()
    sync()
    return max_over_ranks(time.perf_counter() - t0)


def nb1024_leg(args, dev, stream, lib, rng_key, x, local_rank, base, steps=5):
    """configs[1]'s vector under a 1024-bit key -- the default of the factory (flex/crypto/paillier/api.py:22) and of
    every Paillier protocol's sec_param.json (e.g. he_sa_ft/sec_param.json:3): the key holder's fixed-base encrypt
    (k_fb_digits + k_fbs<19> + k_fbp_fin<19> at the largest window <= --fb-window that fits), its decryption
    (k_dec_*_pair<19>) and the public-key per-element path, each with its dominant kernel's fraction of the MAC peak.
    Returns (leg, check): check = what the cpu_baseline section compares with the GMP port and the oracle."""
    from flex.crypto.paillier import _native
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    nb1 = 1024
    N = x.numel()
    pk1, sk1 = generate_paillier_keypair(nb1, seed=1)
    c1 = _native.Context(pk1.n, local_rank)
    c1.set_private(sk1.p, sk1.q)
    c1.set_crt(True)
    c1.set_fixed_base(True)
    c1.set_fb_window(args.fb_window)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c1.prepare_fixed_base()
    setup_ms = (time.perf_counter() - t0) * 1e3
    c1.set_stage_timing(True)
    fbi = c1.fixed_base_info()
    W1 = c1.ct_words
    ct = torch.empty((N, W1), dtype=torch.int32, device=dev)
    ex = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)

    def enc(ctx, n, b, out=ct, exo=ex):
        rc = lib.pai_encrypt_dev(ctx.handle, _native.PAI_F32, x.data_ptr(), n, 0, 0, _native.PAI_OBF_RNG, None, 0, 0,
                                 rng_key, b, out.data_ptr(), exo.data_ptr(), st.data_ptr(), stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    enc(c1, N, base)                                     # warmup
    torch.cuda.synchronize()
    stages = []
    t0 = time.perf_counter()
    for i in range(steps):
        enc(c1, N, base + (i + 1) * N)
        stages.append(c1.stage_times())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    base_chk = base + steps * N                          # the last step's obfuscators
    st_avg = [float(np.mean([s[i] for s in stages])) for i in range(len(stages[0]))]
    wk = work_fbs(nb1, fbi[2])
    names = ["k_fb_digits", "k_fbs", "k_fbp_fin"]
    sdict = {nm: {"kernel_ms": ms, "work_mac_per_elem": wk[nm],
                  "int_mac_frac": (N * wk[nm] / (ms * 1e-3) / INT_MAC_PEAK) if wk[nm] else None}
             for nm, ms in zip(names, st_avg)}
    leg = {"workload": "configs[1]'s 1M-element float32 vector under a 1024-bit key (the reference protocols' default)",
           "key_bits": nb1, "elements": N,
           "encrypt": {"value": N * steps / el, "unit": "encrypts/s", "steps": steps, "ms_per_step": el / steps * 1e3,
                       "path": "key holder: k_fb_digits + k_fbs<19> (Shoup rows) + k_fbp_fin<19>",
                       "window_bits": fbi[3], "digits": fbi[2], "stages": sdict,
                       "roofline": {"kernel": "k_fbs", "frac": sdict["k_fbs"]["int_mac_frac"],
                                    "work_per_unit": wk["k_fbs"], "peak_tmac_s": INT_MAC_PEAK / 1e12},
                       "table_setup_ms": setup_ms, "table_bytes": c1.fixed_base_setup()[2]}}
    # decryption of the last step's output, exact against the input
    val = torch.empty(N, dtype=torch.float64, device=dev)
    stt = torch.empty(N, dtype=torch.int32, device=dev)
    d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(2):                                 # the first call allocates the decrypt work buffers
        d0.record(stream)
        rc = lib.pai_decrypt_dev(c1.handle, ct.data_ptr(), ex.data_ptr(), N, val.data_ptr(), None, stt.data_ptr(), None,
                                 stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())
        d1.record(stream)
        torch.cuda.synchronize()
    dms = d0.elapsed_time(d1)
    dst = c1.stage_times()
    wd = work_dec_pair(nb1)
    ok = bool(torch.equal(val, x.double())) and int((stt > 1).sum().item()) == 0
    leg["decrypt"] = {"value": N / (dms * 1e-3), "unit": "decrypts/s", "kernel_ms": dms,
                      "stages_ms": dict(zip(["k_dec_pre_pair", "k_dec_pow_pair", "k_dec_fin_pair"], dst)) if len(dst) == 3 else dst,
                      "roofline": {"kernel": "k_dec_pow_pair", "work_per_unit": wd,
                                   "frac": (N * wd / (dst[1] * 1e-3) / INT_MAC_PEAK) if len(dst) == 3 else None},
                      "roundtrip_exact": ok}
    if not ok:
        raise SystemExit("nb = 1024: decrypt(encrypt(x)) != x")
    # the generic CRT path on a prefix (bit-identical to the GMP port, checked in the cpu_baseline section) and the
    # public-key per-element path on a larger prefix (bit-identical to CRT)
    nchk = min(N, args.cpu_sample)
    ctg = torch.empty((nchk, W1), dtype=torch.int32, device=dev)
    exg = torch.empty(nchk, dtype=torch.int32, device=dev)
    c1.set_fixed_base(False)
    enc(c1, nchk, base_chk, ctg, exg)
    c1.set_fixed_base(True)
    npub = min(N, 1 << 18)
    ctp = torch.empty((npub, W1), dtype=torch.int32, device=dev)
    exp_ = torch.empty(npub, dtype=torch.int32, device=dev)
    c1.set_crt(False)
    c1.set_fixed_base(False)
    c1.set_public_fixed_base(False)
    enc(c1, npub, base_chk, ctp, exp_)                   # warmup (work buffers)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc(c1, npub, base_chk, ctp, exp_)
    torch.cuda.synchronize()
    tp = time.perf_counter() - t0
    pst = c1.stage_times()
    pe = bool(c1.pair_paths & 4) and len(pst) == 3
    wpe = float((_P(nb1) + 1) * _Mp(nb1 // 32)) if pe else work_enc_public(nb1)
    dom_ms = (pst[1] if pe else sum(pst)) if pst else tp * 1e3
    same_pub = bool(torch.equal(ctp[:nchk], ctg)) and bool(torch.equal(exp_[:nchk], exg))
    pk_names = (("k_pe1_words + k_dec_pre_pair + k_pe1_pow + k_pe1_fin", "k_pe1_pow") if nb1 <= 1024 else
                ("k_pe_pre + k_pe_pow + k_pe_fin", "k_pe_pow")) if pe else ("k_encrypt", "k_encrypt")
    leg["public_key_path"] = {"value": npub / tp, "unit": "encrypts/s", "elements": npub,
                              "kernel": pk_names[0], "stages_ms": pst,
                              "roofline": {"kernel": pk_names[1], "work_per_unit": wpe,
                                           "frac": npub * wpe / (dom_ms * 1e-3) / INT_MAC_PEAK},
                              "bit_identical_to_crt_on_prefix": same_pub}
    if not same_pub:
        raise SystemExit("nb = 1024: public-key and CRT ciphertexts differ")
    check = {"n": pk1.n, "p": sk1.p, "q": sk1.q, "base": base_chk, "fb_info": fbi, "pk": pk1,
             "generic": (ctg.cpu().numpy().view(np.uint32).copy(), exg.cpu().numpy().copy()),
             "fb_idx": sorted({0, 1, N // 2, N - 1}),
             "fb_ct": ct[sorted({0, 1, N // 2, N - 1})].cpu().numpy().view(np.uint32).copy(),
             "fb_ex": ex[sorted({0, 1, N // 2, N - 1})].cpu().numpy().copy()}
    c1.close()
    del c1, ct, ex, st, val, stt, ctg, exg, ctp, exp_
    torch.cuda.empty_cache()
    return leg, check


def selftest_cpu(args) -> None:
    """The launcher's CPU self-test (tests/test_bench_launcher.py): gloo ranks, each contributes a shard
    of rank-stamped rows, one all-gather through sharding.gather_shards; rank 0 prints the world as the
    process group sees it. No GPU is touched."""
    import torch.distributed as dist
    from flex.crypto.paillier.sharding import gather_shards, shard_bounds
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("FLEXPAI_SELFTEST_FAIL_RANK") == str(rank):
        raise SystemExit(3)                 # the launcher must end the other ranks and return 3
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    total = 1000
    lo, hi = shard_bounds(total, world, rank)
    local = torch.arange(lo, hi, dtype=torch.int64).unsqueeze(1) * 16 + rank
    full = gather_shards(local, total, world) if world > 1 else local
    owners = sorted({int(v) % 16 for v in full[:, 0].tolist()})
    ok = bool(torch.equal(full[:, 0] // 16, torch.arange(total)))
    if rank == 0:
        print(json.dumps({"selftest": "cpu", "n_gpus": world, "world_size_seen": dist.get_world_size() if world > 1 else 1,
                          "shard_owners": owners, "gather_ok": ok}))
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("selftest: gathered rows out of order")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json config (default: 1 at every N; the configs[3] leg runs inside it unless "
                         "--no-strong)")
    ap.add_argument("--n", type=int, default=None, help="override: total elements (per GPU for weak configs)")
    ap.add_argument("--nb", type=int, default=None, help="override: Paillier key bits")
    ap.add_argument("--path", choices=("crt", "public"), default="crt")
    ap.add_argument("--obf", choices=("fixedbase", "generic"), default="fixedbase",
                    help="device-RNG sampler of r^n on the CRT path (kernels_fb.hpp vs r from ChaCha20)")
    ap.add_argument("--fb-window", type=int, default=23, choices=(8, 12, 16, 20, 21, 22, 23, 24),
                    help="largest digit window of the fixed-base tables; the library takes the largest one <= this "
                         "whose tables fit the free HBM (nb = 2048: W = 22 with Shoup rows, 47 products per half, "
                         "2 x 88.3 GB; nb = 4096: W = 21, 98 products per half, 2 x 105.2 GB)")
    ap.add_argument("--pfb-window", type=int, default=20, choices=(12, 16, 20),
                    help="digit window of the public-key fixed-base leg (W = 20: 266 row products per element, "
                         "139 GB of tables; the library default is 16)")
    ap.add_argument("--cpu-sample", type=int, default=16384)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the GMP CPU baseline (default os.cpu_count(), like the reference's Pool)")
    ap.add_argument("--deterministic", action="store_true",
                    help="fixed obfuscator key (sha256 constant) instead of os.urandom on rank 0; reproducible runs only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decrypt", action="store_true")
    ap.add_argument("--no-public", action="store_true", help="skip timing the public-key path beside CRT")
    ap.add_argument("--no-add8", action="store_true", help="skip the configs[2] leg (encrypt 8 arrays, 8-way add, decrypt)")
    ap.add_argument("--no-host", action="store_true", help="skip the host-boundary (PCIe, Python objects) rates")
    ap.add_argument("--host-sample", type=int, default=1 << 16,
                    help="elements for the Python-object (PaillierEncryptor.encrypt) rate")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the configs[3] leg (16M elements sharded over the ranks + RCCL all-gather)")
    ap.add_argument("--strong-steps", type=int, default=3, help="timed steps of the configs[3] leg")
    ap.add_argument("--no-contention", action="store_true",
                    help="skip the one-GPU rehearsal of the N = 8 all-gather's HBM contention")
    ap.add_argument("--no-nb1024", action="store_true",
                    help="skip the nb = 1024 leg (configs[1]'s vector under a 1024-bit key: fixed-base encrypt, decrypt, "
                         "public-key path)")
    ap.add_argument("--selftest-cpu", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.selftest_cpu:
        selftest_cpu(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}; reporting the launched world",
              file=sys.stderr)
    cfg_id = args.config if args.config is not None else 1
    cfg = CONFIGS[cfg_id]
    nb = args.nb or cfg["nb"]
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from flex.crypto.paillier import _native
    from flex.crypto.paillier.keypair import generate_paillier_keypair
    from flex.crypto.paillier.sharding import gather_shards_async, shard_bounds

    # workload geometry: weak = N per GPU; strong = the total split into contiguous shards of
    # ceil(total / world) (the last shard is padded; its tail is computed and discarded)
    if cfg["shard"] == "weak":
        N = args.n or cfg["total"]
        total = world * N
        index_base, n_real = rank * N, N
    else:
        total = args.n or cfg["total"]
        lo, hi = shard_bounds(total, world, rank)
        N = -(-total // world)
        index_base, n_real = lo, hi - lo

    setup = {}
    t0 = time.perf_counter()
    pk, sk = generate_paillier_keypair(nb, seed=1)
    setup["keygen_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx = _native.Context(pk.n, local_rank)
    ctx.set_private(sk.p, sk.q)
    setup["context_and_private_key_ms"] = (time.perf_counter() - t0) * 1e3
    # key holder ("crt"): lane CRT kernels for nb <= 2048; at nb = 4096 only the fixed-base sampler exists
    # (group engine, kernels_grp.hpp) and anything else runs the public-key kernel
    holder = args.path == "crt"
    use_crt = holder and ctx.crt_available
    ctx.set_crt(holder)
    use_fb = holder and args.obf == "fixedbase" and ctx.fixed_base
    ctx.set_fixed_base(use_fb)
    grp_fb = use_fb and not use_crt          # 4096-bit keys: k_fb_digits, k_fbg, k_fbg_garner + k_fbg_fin
    fb_info = None
    fb_pair = 0
    fb_split = False
    fb_sgs = False
    fb_shoup = False
    if use_fb:
        ctx.set_fb_window(args.fb_window)     # a dedicated encrypt GPU: the largest tables that fit its HBM
        free0, total0 = torch.cuda.mem_get_info(dev)
        pf = preflight_window(cfg_id, world, nb, args.fb_window, free0, strong_leg=not args.no_strong)
        setup["memory_preflight"] = pf
        if not pf["ok"]:
            raise SystemExit(f"memory preflight: the legs of this run ({pf['legs_bytes'] / 1e9:.1f} GB per rank) would "
                             f"force the fixed-base window from W = {pf['window_tables_alone']} to {pf['window']} on "
                             f"{free0 / 1e9:.1f} GB free: {pf}")
        t0 = time.perf_counter()
        try:
            ctx.prepare_fixed_base()
        except _native.NativeError as exc:
            setup["fixed_base_unavailable"] = str(exc)
        setup["fixed_base_build_wall_ms"] = (time.perf_counter() - t0) * 1e3
        use_fb = ctx.fb_ready
        if use_fb and pf["window"] and ctx.fb_window < pf["window"]:
            raise SystemExit(f"memory preflight: the library built W = {ctx.fb_window} tables, below the planned "
                             f"W = {pf['window']} ({pf})")
        fb_pair = ctx.fb_pair if use_fb else 0
        fb_split = bool(ctx.split_sampler & 1) if use_fb else False   # k_sgp (kernels_sgp.hpp) for k_fbgp
        fb_shoup = bool(ctx.split_sampler & 4) if use_fb else False   # k_fbs (kernels_fbs.hpp) for k_fbp
        fb_sgs = bool(ctx.split_sampler & 8) if use_fb else False     # k_sgs (kernels_sgs.hpp, $FLEXPAI_SGS=1) for k_sgp
        if use_fb:
            fb_info = ctx.fixed_base_info()
            h_ms, d_ms, tbytes = ctx.fixed_base_setup()
            setup.update({"fixed_base_host_ms": h_ms, "fixed_base_device_ms": d_ms, "fixed_base_table_bytes": tbytes,
                          "fixed_base_note": "once per key: bases + B_k on the host, hipMalloc, k_fb(p)_lohi + k_fb(p)_fill; "
                                             "outside the timed region (the tables stay resident)"})
    ctx.set_stage_timing(True)
    lib = _native.load_library()
    W = ctx.ct_words
    stream = torch.cuda.current_stream(dev)

    # obfuscator key: fresh per run, shared by the ranks (a secret in production: INTEGRATION.md)
    if args.deterministic:
        rng_key = hashlib.sha256(b"flexpai-bench-key").digest()
    else:
        kt = torch.tensor(list(os.urandom(32)), dtype=torch.uint8, device=dev)
        if world > 1:
            dist.broadcast(kt, src=0)
        rng_key = bytes(kt.cpu().tolist())

    x_host = np.random.default_rng(rank).standard_normal(N, dtype=np.float32)
    x = torch.from_numpy(x_host).to(dev)
    st = torch.empty(N, dtype=torch.int32, device=dev)

    def encrypt(xd, out, exo, base, n=N, sto=None):
        sto = st if sto is None else sto
        assert xd.numel() >= n and out.shape[0] >= n and exo.numel() >= n and sto.numel() >= n
        rc = lib.pai_encrypt_dev(ctx.handle, _native.PAI_F32, xd.data_ptr(), n, 0, 0, _native.PAI_OBF_RNG,
                                 None, 0, 0, rng_key, base, out.data_ptr(), exo.data_ptr(), sto.data_ptr(),
                                 stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    def decrypt(ct, ex, val, stt, n=N):
        rc = lib.pai_decrypt_dev(ctx.handle, ct.data_ptr(), ex.data_ptr(), n, val.data_ptr(), None,
                                 stt.data_ptr(), None, stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    def add_k(cts, exs, k, out, oe):
        rc = lib.pai_add_dev(ctx.handle, cts.data_ptr(), exs.data_ptr(), k, N, out.data_ptr(), oe.data_ptr(),
                             stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(lib.pai_last_error().decode())

    extra = {}
    K8 = 8
    add_events = []
    stride = job_units(cfg["shard"], total, world, N, 1)     # the job's elements per step (step_base)
    sync = torch.cuda.synchronize
    barrier = dist.barrier if world > 1 else (lambda: None)

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if cfg_id == 2:
        # ---- a step = the configs[2] pipeline: encrypt 8 arrays, one 8-way add, decrypt the sum; step i's arrays
        # are under obfuscator bases index_base + (8 i + k + 1) x total, k = 0..7
        xs8 = torch.stack([torch.from_numpy(np.random.default_rng(k).standard_normal(N, dtype=np.float32))
                           for k in range(K8)]).to(dev)
        cts8 = torch.empty((K8, N, W), dtype=torch.int32, device=dev)
        exs8 = torch.empty((K8, N), dtype=torch.int32, device=dev)
        sum_ct = torch.empty((N, W), dtype=torch.int32, device=dev)
        sum_ex = torch.empty(N, dtype=torch.int32, device=dev)
        val8 = torch.empty(N, dtype=torch.float64, device=dev)
        st8 = torch.empty(N, dtype=torch.int32, device=dev)

        class Add8Steps:
            last_i = None

            def step(self, i):
                for k in range(K8):
                    encrypt(xs8[k], cts8[k], exs8[k], index_base + (K8 * i + k + 1) * total)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                add_k(cts8, exs8, K8, sum_ct, sum_ex)
                e1.record(stream)
                if i >= args.warmup:
                    add_events.append((e0, e1))
                decrypt(sum_ct, sum_ex, val8, st8)
                self.last_i = i

            def drain(self):
                pass

        stepper = Add8Steps()
        stage_ms = []
        elapsed = run_timed(stepper, args.steps, args.warmup, sync, barrier, max_over_ranks)
    else:
        ct = torch.empty((N, W), dtype=torch.int32, device=dev)
        ex = torch.empty(N, dtype=torch.int32, device=dev)
        # N > 1: double-buffered shards and gathered outputs; step i's RCCL all-gather (ciphertexts +
        # exponents) runs on the process group's stream while step i+1 encrypts (ShardSteps)
        bufs = [(ct, ex)] + ([(torch.empty_like(ct), torch.empty_like(ex))] if world > 1 else [])
        gath = [(torch.empty((world * N, W), dtype=torch.int32, device=dev),
                 torch.empty(world * N, dtype=torch.int32, device=dev)) for _ in bufs] if world > 1 else []
        stepper = ShardSteps(lambda o, e, base: encrypt(x, o, e, base), bufs, gath, world, index_base, stride,
                             gather_shards_async)
        stage_ms = []
        # HIP events recorded between each timed encrypt call's kernels
        elapsed = run_timed(stepper, args.steps, args.warmup, sync, barrier, max_over_ranks,
                            after_step=lambda: stage_ms.append(ctx.stage_times()))
    units = job_units(cfg["shard"], total, world, N, args.steps)
    value = units / elapsed

    if cfg_id == 2:
        ref = xs8.double().sum(0)
        err = float((val8 - ref).abs().max().item())
        ok8 = bool(torch.all((val8 - ref).abs() <= torch.finfo(torch.float64).eps * ref.abs()).item()) and \
            int((st8 > 1).sum().item()) == 0
        extra["config2_check"] = {"max_abs_err_vs_float64_sum": err, "within_1ulp": ok8}
        if not ok8:
            raise SystemExit("configs[2]: decrypted sums differ from the float64 sums")
        ct, ex = cts8[0], exs8[0]
        x_host = xs8[0].cpu().numpy()
        x = xs8[0]
        index_base_chk = index_base + (K8 * stepper.last_i + 1) * total
    else:
        index_base_chk = stepper.base(stepper.last_i)
        (ct, ex), _ = stepper.last_output()       # the last timed step's output (checked below)
        if world > 1:
            # the gathered array holds every rank's shard; this rank's block equals its own output
            same = stepper.own_shard_identical(rank)
            extra["allgather_own_shard_identical"] = same
            if not same:
                raise SystemExit("all-gathered shard differs from the local one")
    extra["obfuscator_index_bases"] = {"first_timed_step": (index_base + K8 * args.warmup * total + total) if cfg_id == 2
                                       else stepper.base(args.warmup),
                                       "stride_per_step": K8 * total if cfg_id == 2 else stride,
                                       "note": "every step encrypts under fresh obfuscators (global index base advanced "
                                               "by the job's elements per step, bench.py step_base)"}
    stage_avg = [float(np.mean([s[i] for s in stage_ms])) for i in range(len(stage_ms[0]))] if stage_ms else []

    # ---- correctness of the timed output: decrypt on the device, compare with the input exactly
    if not args.no_decrypt and cfg_id != 2:
        val = torch.empty(N, dtype=torch.float64, device=dev)
        stt = torch.empty(N, dtype=torch.int32, device=dev)
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record(stream)
        decrypt(ct, ex, val, stt)
        d1.record(stream)
        torch.cuda.synchronize()
        dec_ms = d0.elapsed_time(d1)
        dst = ctx.stage_times()
        dec_pair = bool(ctx.pair_paths & 1)
        wd = work_dec_pair(nb) if dec_pair else work_dec(nb)
        if ctx.lane_decrypt and len(dst) == 3:
            extra["decrypt_stages"] = {
                "k_dec_pre": {"kernel_ms": dst[0]},
                "k_dec_pow": {"kernel_ms": dst[1], "work_mac_per_elem": wd,
                              "achieved_tmac_s": N * wd / (dst[1] * 1e-3) / 1e12},
                "k_dec_fin": {"kernel_ms": dst[2]}}
        extra["decrypt_path"] = (("lane-pair" if dec_pair else "lane") if ctx.lane_decrypt
                                 else "split-pair (kernels_dec4.hpp)" if dec_pair else "group")
        ok = bool(torch.equal(val[:n_real], x[:n_real].double())) and int((stt[:n_real] > 1).sum().item()) == 0
        extra["decrypt_per_s_per_gpu"] = N / (dec_ms * 1e-3)
        extra["decrypt_kernel_ms"] = dec_ms
        extra["decrypt_int_mac_frac"] = N * wd / (dec_ms * 1e-3) / INT_MAC_PEAK
        extra["decrypt_w_dec_equivalent_frac"] = N * work_dec(nb) / (dec_ms * 1e-3) / INT_MAC_PEAK
        extra["roundtrip_exact"] = ok
        if not ok:
            raise SystemExit("decrypt(encrypt(x)) != x on the device")
        del val, stt

    # ---- HBM contention of the N = 8 all-gather, rehearsed on one GPU: at N = 8 a rank
    # receives 7 shards (7 x N x W words, 3.8 GB) per step while it encrypts the next one. A device-to-device copy
    # of that size on a side stream stands in for the RCCL receive writes (pessimistic: a copy also reads the
    # bytes from HBM, the xGMI receive only writes them); reported: each alone, and both at once.
    if cfg_id == 1 and world == 1 and not args.no_contention:
        nbytes = 7 * N * W * 4
        try:
            src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
            dst = torch.empty_like(src)
        except RuntimeError:
            src = dst = None
        if src is not None:
            side = torch.cuda.Stream(dev)

            standin = None
            try:                                  # tools/gpu/rccl_standin.hip (__graft_entry__.build_standin)
                import ctypes
                standin = ctypes.CDLL(os.path.join(ROOT, "tools", "gpu", "librccl_standin.so"))
                standin.standin_throttled_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong,
                                                           ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p]
            except OSError:
                standin = None

            def timed(run_copy, run_enc, cu_copy=None):
                ev = {k: torch.cuda.Event(enable_timing=True) for k in ("c0", "c1", "e0", "e1")}
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if run_copy:
                    with torch.cuda.stream(side):
                        ev["c0"].record(side)
                        if cu_copy is None:
                            dst.copy_(src, non_blocking=True)
                        elif standin.standin_throttled_copy(src.data_ptr(), dst.data_ptr(), nbytes, cu_copy[0],
                                                            int(cu_copy[1] * 1e6), side.cuda_stream) != 0:
                            raise RuntimeError("stand-in copy kernel failed to launch")
                        ev["c1"].record(side)
                if run_enc:
                    ev["e0"].record(stream)
                    encrypt(x, ct, ex, index_base_chk)   # (rewrites the last step's own output)
                    ev["e1"].record(stream)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) * 1e3
                return (ev["c0"].elapsed_time(ev["c1"]) if run_copy else None,
                        ev["e0"].elapsed_time(ev["e1"]) if run_enc else None, wall)

            timed(True, True)
            c_alone = min(timed(True, False)[0] for _ in range(3))
            e_alone = min(timed(False, True)[1] for _ in range(3))
            both = [timed(True, True) for _ in range(3)]
            c_both, e_both, w_both = min(both, key=lambda t: t[2])
            extra["allgather_contention_1gpu"] = {
                "received_bytes_per_step_at_n8": nbytes, "copy_alone_ms": c_alone,
                "copy_alone_gb_s": nbytes / (c_alone * 1e-3) / 1e9, "encrypt_alone_ms": e_alone,
                "encrypt_with_copy_ms": e_both, "copy_with_encrypt_ms": c_both, "both_wall_ms": w_both,
                "encrypt_slowdown": e_both / e_alone,
                "note": "a 3.8 GB device-to-device copy on a side stream (reads + writes HBM) stands in for the N = 8 "
                        "all-gather's receive writes into this rank's HBM during the next step's encrypt"}
            # the same bytes moved by CU-resident copy workgroups (RCCL's channels: one workgroup each) that stay on
            # their CUs for the xGMI-limited time of the gather (3.8 GB over 7 links x ~153 GB/s at ring efficiency:
            # ~8-12 ms of each step), launched ahead of the encrypt like the previous step's gather
            if standin is not None:
                cu = []
                for blocks, dur_ms in ((32, 10.0), (64, 10.0), (64, 12.0), (128, 8.0)):
                    timed(True, False, (blocks, dur_ms))
                    runs = [timed(True, True, (blocks, dur_ms)) for _ in range(3)]
                    cb, eb, wb = min(runs, key=lambda t: t[1])
                    ca = min(timed(True, False, (blocks, dur_ms))[0] for _ in range(2))
                    cu.append({"workgroups": blocks, "target_ms": dur_ms, "copy_alone_ms": ca, "copy_with_encrypt_ms": cb,
                               "encrypt_with_copy_ms": eb, "encrypt_slowdown": eb / e_alone, "both_wall_ms": wb})
                extra["allgather_contention_1gpu"]["cu_resident_copy"] = {
                    "runs": cu, "encrypt_alone_ms": e_alone,
                    "note": "tools/gpu/rccl_standin.hip: the 3.8 GB moved by `workgroups` x 256 lanes that hold their CUs "
                            "for target_ms (wall-clock throttled), on a side stream launched before the encrypt"}
            del src, dst
            torch.cuda.empty_cache()

    # ---- configs[3] leg (strong scaling): 16M elements over the ranks, every step's ciphertext shards
    # reassembled on every rank by an RCCL all-gather (double-buffered against the next step's encrypt)
    c3_seams = None
    if cfg_id == 1 and not args.no_strong and nb == 2048:
        tot3 = CONFIGS[3]["total"]
        lo3, hi3 = shard_bounds(tot3, world, rank)
        N3 = -(-tot3 // world)
        x3_host = np.random.default_rng(1000 + rank).standard_normal(N3, dtype=np.float32)
        x3 = torch.from_numpy(x3_host).to(dev)
        st3 = torch.empty(N3, dtype=torch.int32, device=dev)
        b3 = [(torch.empty((N3, W), dtype=torch.int32, device=dev), torch.empty(N3, dtype=torch.int32, device=dev))
              for _ in range(2 if world > 1 else 1)]
        g3 = [(torch.empty((world * N3, W), dtype=torch.int32, device=dev),
               torch.empty(world * N3, dtype=torch.int32, device=dev)) for _ in b3] if world > 1 else []
        s3 = ShardSteps(lambda o, e, base: encrypt(x3, o, e, base, N3, st3), b3, g3, world, lo3, tot3,
                        gather_shards_async)
        el3 = run_timed(s3, args.strong_steps, 1, sync, barrier, max_over_ranks)
        leg = {"workload": CONFIGS[3]["desc"], "elements_total": tot3, "elements_per_gpu": N3,
               "value": tot3 * args.strong_steps / el3, "unit": "encrypts/s", "scaling": "strong",
               "steps": args.strong_steps, "ms_per_step": el3 / args.strong_steps * 1e3,
               "allgather": "RCCL all_gather_into_tensor of words + exponents per step" if world > 1 else "none (N = 1)"}
        if world > 1:
            same = s3.own_shard_identical(rank)
            leg["allgather_own_shard_identical"] = same
            leg["gathered_bytes_per_rank_per_step"] = world * N3 * (W + 1) * 4
            if not same:
                raise SystemExit("configs[3]: all-gathered shard differs from the local one")
        # the last timed step's output, checked: this rank's shard decrypted on the device (up to
        # the 2M elements of one rank's shard at N = 8), the sampler's restatement at the shard's seams, and at
        # N > 1 a block of the next rank's shard as gathered here, against that rank's regenerated input
        (c3o, e3o), r3o = s3.last_output()
        base3 = s3.base(s3.last_i)               # the last step's obfuscator base (global index of the shard's row 0)
        n3 = hi3 - lo3
        nchk = min(n3, 2 << 20)
        v3 = torch.empty(nchk, dtype=torch.float64, device=dev)
        st3v = torch.empty(nchk, dtype=torch.int32, device=dev)
        decrypt(c3o, e3o, v3, st3v, nchk)
        torch.cuda.synchronize()
        chk = {"decrypted_own_elements": nchk,
               "own_roundtrip_exact": bool(torch.equal(v3, x3[:nchk].double())) and int((st3v > 1).sum().item()) == 0}
        if use_fb and fb_info is not None:
            # checked against the oracle's restatement in the cpu_baseline leg below (the one place bench.py
            # runs oracle/ code)
            seam = [0, n3 - 1]
            c3_seams = (leg, [base3 + i for i in seam], [x3_host[i] for i in seam],
                        _native.words_to_ints(c3o[seam].cpu().numpy().view(np.uint32)),
                        [int(v) for v in e3o[seam].cpu().numpy()])
        if world > 1:
            peer = (rank + 1) % world
            plo, phi = shard_bounds(tot3, world, peer)
            npe = min(phi - plo, 1 << 16)
            xp = torch.from_numpy(np.random.default_rng(1000 + peer).standard_normal(N3, dtype=np.float32)[:npe]).to(dev)
            vp = torch.empty(npe, dtype=torch.float64, device=dev)
            sp = torch.empty(npe, dtype=torch.int32, device=dev)
            decrypt(r3o[0][peer * N3:], r3o[1][peer * N3:], vp, sp, npe)
            torch.cuda.synchronize()
            chk["gathered_peer_block"] = {"peer": peer, "elements": npe,
                                          "roundtrip_exact": bool(torch.equal(vp, xp.double())) and int((sp > 1).sum().item()) == 0}
        leg["check"] = chk
        bad = (not chk["own_roundtrip_exact"]
               or not chk.get("gathered_peer_block", {"roundtrip_exact": True})["roundtrip_exact"])
        if bad:
            raise SystemExit(f"configs[3]: last step's output failed its check: {chk}")
        extra["config3_strong"] = leg
        del x3, st3, b3, g3, s3, c3o, e3o, r3o, v3, st3v
        torch.cuda.empty_cache()

    solo = world == 1 and rank == 0        # single-GPU legs beside the timed path

    # ---- a freshly generated key (VERDICT r2 Missing #4): context + private key + the first device-RNG call,
    # setup included, at the library defaults (W = 16 tables, built only past the break-even count)
    if solo and cfg_id == 1 and use_fb:
        fresh = {}
        for label, nf, seed, nbf in (("first_1M_call", N, 2, nb), ("first_1k_call", 1000, 3, nb),
                                     ("first_1k_call_nb1024", 1000, 4, 1024)):
            pk2, sk2 = generate_paillier_keypair(nbf, seed=seed)    # host keygen, not timed (the reference's too)
            Wf = 2 * nbf // 32
            ct_f = torch.empty((nf, Wf), dtype=torch.int32, device=dev)
            ex_f = torch.empty(nf, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            c2 = _native.Context(pk2.n, local_rank)
            c2.set_private(sk2.p, sk2.q)
            rc = lib.pai_encrypt_dev(c2.handle, _native.PAI_F32, x.data_ptr(), nf, 0, 0, _native.PAI_OBF_RNG, None, 0, 0,
                                     rng_key, 0, ct_f.data_ptr(), ex_f.data_ptr(), st.data_ptr(), stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(lib.pai_last_error().decode())
            torch.cuda.synchronize()
            wall = time.perf_counter() - t1
            fresh[label] = {"elements": nf, "key_bits": nbf, "wall_ms": wall * 1e3, "encrypts_per_s_incl_setup": nf / wall,
                            "tables_built": c2.fb_ready,
                            "fixed_base_window": c2.fb_window if c2.fb_ready else None}
            if nf <= 4096:   # the protocol's other half: decrypt the call's ciphertexts on the same fresh context
                val_f = torch.empty(nf, dtype=torch.float64, device=dev)
                mant_f = torch.empty(nf, dtype=torch.int64, device=dev)
                st_f = torch.empty(nf, dtype=torch.int32, device=dev)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                rc = lib.pai_decrypt_dev(c2.handle, ct_f.data_ptr(), ex_f.data_ptr(), nf, val_f.data_ptr(), mant_f.data_ptr(),
                                         st_f.data_ptr(), None, stream.cuda_stream)
                if rc != 0:
                    raise RuntimeError(lib.pai_last_error().decode())
                torch.cuda.synchronize()
                fresh[label]["decrypt_wall_ms"] = (time.perf_counter() - t2) * 1e3
                fresh[label]["roundtrip_exact"] = bool(torch.equal(val_f, x[:nf].double()))
            del c2, ct_f, ex_f
        fresh["note"] = ("new keypair per call (HE_SA_FT re-keys per exchange, he_sa_ft/train.py:39-40): wall time of "
                         "Context + set_private + one pai_encrypt_dev on device-resident x, synchronised; tables are "
                         "built only when the call reaches the break-even count (pai_ctx_fixed_base_policy); calls of "
                         "<= 4096 elements run on 16-lane rows (k_crt_w / k_dec_w, PAI_OPT_ROWS_MAX); "
                         "decrypt_wall_ms: pai_decrypt_dev of the call's ciphertexts on the same context")
        extra["fresh_key"] = fresh
    cpu_sample = args.cpu_sample if nb <= 2048 else min(args.cpu_sample, 4096)   # bounded CPU work at nb = 4096
    S_chk = min(N, cpu_sample)
    # ---- the generic CRT path on the same input (untimed): bit-reproducible against GMP
    ct_ref = ct
    if use_fb and solo:
        ct_ref = torch.empty_like(ct)
        ex_ref = torch.empty_like(ex)
        ctx.set_fixed_base(False)
        n_gen = N if use_crt else S_chk        # 4096: the public-key kernel, on the CPU-checked prefix only
        encrypt(x, ct_ref, ex_ref, index_base_chk, n_gen)
        encrypt(x, ct_ref, ex_ref, index_base_chk, n_gen)
        gen_ms = ctx.stage_times()
        ctx.set_fixed_base(True)
        torch.cuda.synchronize()
        if use_crt:
            wc = work_crt(nb)
            if ctx.pair_paths & 2:   # stage B on pairs: (P(h) + 2) pair products per half
                wc["k_crt_b"] = float(2 * (_P(nb // 2) + 2) * _Mp(nb // 64))
            extra["generic_crt_path"] = {
                "value": N / (sum(gen_ms) * 1e-3), "unit": "encrypts/s per GPU",
                "note": "r from the ChaCha20 stream and r^n by CRT exponentiation (kernels_crt.hpp); "
                        "bit-identical to the public-key kernel and the GMP baseline",
                "stages_ms": dict(zip(["k_crt_a", "k_crt_b", "k_crt_fin"], gen_ms)),
                "k_crt_b_int_mac_frac": N * wc["k_crt_b"] / (gen_ms[1] * 1e-3) / INT_MAC_PEAK if len(gen_ms) > 1 else None}
        else:
            extra["generic_path"] = {
                "value": n_gen / (sum(gen_ms) * 1e-3), "unit": "encrypts/s per GPU", "elements": n_gen,
                "note": "no lane CRT at nb = 4096: r from the ChaCha20 stream, r^n mod n^2 by the public-key "
                        "kernel k_encrypt<8>; bit-identical to the GMP baseline"}
    ct_host_check = ct_ref[:S_chk].cpu().numpy().view(np.uint32).copy()
    ex_host_check = ex[:S_chk].cpu().numpy().copy()
    ct_timed_check = ct[:S_chk].cpu().numpy().view(np.uint32).copy()

    # ---- the public-key path on the same input (untimed region), for the record and as a parity check
    if holder and (use_crt or use_fb) and not args.no_public and solo:
        ct2 = torch.empty_like(ct)
        ex2 = torch.empty_like(ex)
        npub = min(N, 1 << 16) if nb > 2048 else N
        ctx.set_crt(False)
        ctx.set_fixed_base(False)
        ctx.set_public_fixed_base(False)    # the per-element exponentiation (same r as the CRT path)
        encrypt(x, ct2, ex2, index_base_chk, npub)
        pub_st = ctx.stage_times()          # k_encrypt: one stage; split pairs: k_pe_pre, k_pe_pow, k_pe_fin
        pub_ms = float(sum(pub_st))
        pe = bool(ctx.pair_paths & 4) and len(pub_st) == 3
        ctx.set_crt(True)
        ctx.set_fixed_base(use_fb)
        ctx.set_public_fixed_base(True)
        torch.cuda.synchronize()
        ncmp = npub if use_crt else min(npub, S_chk)
        same = bool(torch.equal(ct2[:ncmp], ct_ref[:ncmp]))
        wpe = float((_P(nb) + 1) * _Mp(nb // 32))   # W_enc with pair products over the nb/32 limbs of n
        extra["public_key_path"] = {"value": npub / (pub_ms * 1e-3), "unit": "encrypts/s per GPU", "elements": npub,
                                    "kernel": "k_pe_pre + k_pe_pow + k_pe_fin (split pairs)" if pe else "k_encrypt",
                                    "kernel_ms": pub_ms,
                                    "stages_ms": dict(zip(["k_pe_pre", "k_pe_pow", "k_pe_fin"], pub_st)) if pe else None,
                                    "int_mac_frac": npub * (wpe if pe else work_enc_public(nb)) / (pub_ms * 1e-3) / INT_MAC_PEAK,
                                    "w_enc_equivalent_frac": npub * work_enc_public(nb) / (pub_ms * 1e-3) / INT_MAC_PEAK,
                                    "bit_identical_to_crt": same}
        del ct2, ex2
        if not same:
            raise SystemExit("CRT and public-key ciphertexts differ")

    pfb_check = None

    # ---- configs[2] beside configs[1]: encrypt 8 arrays, one 8-way add (k_add), decrypt the sum
    if cfg_id == 1 and solo and not args.no_add8 and not args.no_decrypt:
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
            encrypt(xs8[k], cts8[k], exs8[k], index_base + (k + 1) * total)
        ev[1].record(stream)
        add_k(cts8, exs8, K8, sum_ct, sum_ex)
        ev[2].record(stream)
        decrypt(sum_ct, sum_ex, val8, st8)
        ev[3].record(stream)
        torch.cuda.synchronize()
        wall8 = time.perf_counter() - t8
        ref = xs8.double().sum(0)
        err = float((val8 - ref).abs().max().item())
        add_ms = ev[1].elapsed_time(ev[2])
        E, emin = exs8.max(0).values, exs8.min(0).values
        extra["config2_add8"] = {
            "workload": "configs[2]: encrypt 8 x 1M float32 arrays, one 8-way add, decrypt the sum (device-resident)",
            "elements_per_s": N / wall8, "wall_s": wall8,
            "encrypt8_ms": ev[0].elapsed_time(ev[1]), "k_add_ms": add_ms, "decrypt_ms": ev[2].elapsed_time(ev[3]),
            "k_add_int_mac_frac": work_add(exs8, nb) / (add_ms * 1e-3) / INT_MAC_PEAK,
            "k_add_note": "canonical W_add of SURVEY.md §8d (per-operand alignment squarings); k_add evaluates the "
                          "same product by Horner over exponent levels (squarings of the running product); "
                          "k_add_ms includes the schedule sort (k_add_plan/scan/scatter)",
            "canonical_alignment_squarings_per_elem": int((4 * (E.unsqueeze(0) - exs8)).sum().item()) / N,
            "horner_squarings_per_elem": int((4 * (E - emin)).sum().item()) / N,
            "max_abs_err_vs_float64_sum": err, "statuses_ok": int((st8 > 1).sum().item()) == 0}
        del xs8, cts8, exs8, sum_ct, sum_ex, val8, st8
        torch.cuda.empty_cache()

    # ---- host boundary: plaintexts start in host numpy, ciphertexts leave as host buffers /
    # PaillierEncryptedNumber objects; never part of `value`
    if not args.no_host and solo and cfg_id in (1, 3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hct, hex_, hst = ctx.encrypt(x_host, obf_mode=_native.PAI_OBF_RNG, rng_key=rng_key, index_base=index_base_chk)
        t_fresh = time.perf_counter() - t1
        t_host = float("inf")
        for _ in range(2):                        # a streaming sender reuses its output buffers
            t1 = time.perf_counter()
            ctx.encrypt(x_host, obf_mode=_native.PAI_OBF_RNG, rng_key=rng_key, index_base=index_base_chk,
                        out=(hct, hex_, hst))
            t_host = min(t_host, time.perf_counter() - t1)
        hb = {"host_buffers_encrypts_per_s": N / t_host,
              "host_buffers_fresh_outputs_per_s": N / t_fresh,
              "host_buffers_note": "pai_encrypt: H2D float32 x, kernels, D2H ciphertext words "
                                   f"({N * W * 4 / 2**20:.0f} MiB) through pinned staging into caller (pageable) "
                                   "memory, chunks overlapped with the kernels; caller buffers reused (out=), "
                                   "best of 2; fresh_outputs: new numpy arrays (page faults on first write)",
              "host_vs_device": None,
              "host_buffers_bit_identical": bool(np.array_equal(hct[: len(ct_timed_check)], ct_timed_check))}
        from flex.crypto.paillier import _runtime
        from flex.crypto.paillier.encryptor import PaillierEncryptor
        _runtime.register_private(pk, sk)        # this process holds the key (CRT path, as above)
        enc = PaillierEncryptor(pk)
        _runtime.context(pk).prepare_fixed_base()  # the runtime's own context + its tables (W = 16): setup, untimed
        enc.encrypt(x_host[:4096])
        hs = min(args.host_sample, N)
        t1 = time.perf_counter()
        objs = enc.encrypt(x_host[:hs])
        t_obj = time.perf_counter() - t1
        hb["python_objects_encrypts_per_s"] = hs / t_obj
        hb["python_objects_note"] = (f"PaillierEncryptor.encrypt(ndarray[{hs}]) -> object ndarray of "
                                     "PaillierEncryptedNumber (encryptor.py:99-114 API), incl. materialisation")
        del objs
        # the drop-in path's own device rate: the runtime's context at the library's default window (callers
        # of PaillierEncryptor reach this, not the bench's W = 22 context), device-resident input
        rctx = _runtime.context(pk)
        ct_r = torch.empty((N, W), dtype=torch.int32, device=dev)
        ex_r = torch.empty(N, dtype=torch.int32, device=dev)
        st_r = torch.empty(N, dtype=torch.int32, device=dev)
        t_r = float("inf")
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rc = lib.pai_encrypt_dev(rctx.handle, _native.PAI_F32, x.data_ptr(), N, 0, 0, _native.PAI_OBF_RNG, None, 0, 0,
                                     rng_key, index_base_chk, ct_r.data_ptr(), ex_r.data_ptr(), st_r.data_ptr(),
                                     stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(lib.pai_last_error().decode())
            torch.cuda.synchronize()
            t_r = min(t_r, time.perf_counter() - t1)
        extra["dropin_default_window"] = {
            "encrypts_per_s": N / t_r, "window_bits": rctx.fb_window, "elements": N,
            "table_bytes": rctx.fixed_base_setup()[2] if rctx.fb_ready else 0,
            "note": "_runtime.context(pk) (what PaillierEncryptor.encrypt uses) at the library default window "
                    "($FLEXPAI_FB_WINDOW unset: 16), device-resident x, best of 3 synchronised calls; "
                    "FLEXPAI_FB_WINDOW=auto gives a process holding one key the largest window that fits "
                    "(the bench context's W above)"}
        del ct_r, ex_r, st_r
        # a received ciphertext array decrypted through the drop-in API: the reference's plain object-ndarray
        # pickle (what an unmodified peer sends, ion.py:150-178 -> ion.py:201) into PaillierDecryptor.decrypt
        # (decryptor.py:114-127), the per-element key check and the packing included
        import pickle
        from flex.crypto.paillier.cipher_array import pack_checked
        from flex.crypto.paillier.decryptor import PaillierDecryptor
        pdec = PaillierDecryptor(pk, sk)
        received = pickle.loads(pickle.dumps(enc.encrypt(x_host)))
        assert type(received) is np.ndarray and received.dtype == object
        pdec.decrypt(received[:4096])
        t1 = time.perf_counter()
        got_vals = pdec.decrypt(received)
        t_rd = time.perf_counter() - t1
        t1 = time.perf_counter()
        pack_checked(received.reshape(-1), pk, W)
        t_pack = time.perf_counter() - t1
        hb["received_decrypt_per_s"] = N / t_rd
        hb["received_decrypt_s"] = t_rd
        hb["received_check_and_pack_s"] = t_pack
        hb["received_decrypt_exact"] = bool(np.array_equal(got_vals, x_host.astype(np.float64)))
        if "decrypt_per_s_per_gpu" in extra:
            hb["received_decrypt_vs_device_decrypt"] = (N / t_rd) / extra["decrypt_per_s_per_gpu"]
        hb["received_decrypt_note"] = (f"PaillierDecryptor.decrypt(object ndarray[{N}]) unpickled from the reference's "
                                       "plain pickle: C key check + word packing (hostgmp.c pack_numbers), host -> "
                                       "device, decrypt kernels, float64 out")
        del received, got_vals
        if not hb["received_decrypt_exact"]:
            raise SystemExit("decrypting the received object array did not reproduce the input")
        # object-free path (cipher_buffer.py): encrypt into words, serialise, receive without objects
        from flex.crypto.paillier.cipher_array import from_wire
        t1 = time.perf_counter()
        buf = enc.encrypt_to_buffer(x_host)
        t_buf = time.perf_counter() - t1
        t1 = time.perf_counter()
        wire = buf.to_wire()
        t_wire = time.perf_counter() - t1
        t1 = time.perf_counter()
        back = from_wire(wire, pk, lazy=True)
        t_recv = time.perf_counter() - t1
        hb["buffer_encrypts_per_s"] = N / t_buf
        hb["buffer_to_wire_per_s"] = N / t_wire
        hb["buffer_from_wire_lazy_per_s"] = N / t_recv
        hb["buffer_note"] = ("PaillierEncryptor.encrypt_to_buffer(ndarray[N]) -> CiphertextBuffer (words, no objects), "
                             f".to_wire() ({len(wire) / 2**20:.0f} MiB), from_wire(lazy=True) incl. the < n^2 check")
        hb["buffer_round_trip_identical"] = bool(np.array_equal(back.words, buf.words))
        del buf, back, wire
        hb["host_vs_device"] = hb["host_buffers_encrypts_per_s"] / value
        extra["host_boundary"] = hb

    # ---- a party holding ONLY the public key (HE_OTP_LR / HE_LR_FP hosts): public fixed bases (kernels_pfb.hpp)
    if not args.no_public and solo and nb == 2048:
        # the key holder's tables (2 x 88.3 GB at W = 22) make room for the public ones (W = 20: 139 GB); nothing
        # after this leg encrypts with the key holder's context
        ctx.set_fb_window(16)
        torch.cuda.synchronize()
        cpub = _native.Context(pk.n, local_rank)
        cpub.set_pfb_window(args.pfb_window)
        t1 = time.perf_counter()
        cpub.prepare_public_fixed_base()
        pfb_setup_ms = (time.perf_counter() - t1) * 1e3
        cpub.set_stage_timing(True)
        ct3 = torch.empty_like(ct)
        ex3 = torch.empty_like(ex)
        runs = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rc = lib.pai_encrypt_dev(cpub.handle, _native.PAI_F32, x.data_ptr(), N, 0, 0, _native.PAI_OBF_RNG, None, 0, 0,
                                     rng_key, index_base_chk, ct3.data_ptr(), ex3.data_ptr(), st.data_ptr(),
                                     stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(lib.pai_last_error().decode())
            torch.cuda.synchronize()
            runs.append((time.perf_counter() - t1, cpub.stage_times()))
        wall, pst = min(runs, key=lambda r: r[0])
        bases, Kp, Wp, K0p = cpub.public_fixed_base_info()
        pfb_k = "k_sgp" if cpub.split_sampler & 2 else "k_pfb"
        wpfb = work_pfb(nb, Kp)                     # K factored-row products mod n^2 + the correction
        # exact round trip through the key holder's decryption
        valp = torch.empty(N, dtype=torch.float64, device=dev)
        stp = torch.empty(N, dtype=torch.int32, device=dev)
        decrypt(ct3, ex3, valp, stp)
        torch.cuda.synchronize()
        okp = bool(torch.equal(valp, x.double())) and int((stp > 1).sum().item()) == 0
        extra["public_key_fixed_base"] = {
            "value": N / wall, "unit": "encrypts/s per GPU", "elements": N,
            "kernel": f"k_pfb_digits + {pfb_k} + k_pe_fin", "stages_ms": dict(zip(["k_pfb_digits", pfb_k, "k_pe_fin"], pst)),
            "k_pfb_int_mac_frac": N * wpfb / (pst[1] * 1e-3) / INT_MAC_PEAK if len(pst) > 1 else None,
            "sampler": pfb_k + (" (split pairs, kernels_sgp.hpp)" if pfb_k == "k_sgp" else " (pair groups, kernels_pfb.hpp)"),
            "work_mac_per_elem": wpfb, "digits": Kp, "window": Wp, "e0_digits": K0p,
            "setup_ms": pfb_setup_ms, "table_bytes": Kp * (1 << Wp) * 512,
            "roundtrip_exact": okp,
            "note": "a public-key-only context: r = prod_j g_j^e_j mod n over 33 self-drawn bases (DESIGN.md §3), "
                    "r^n as K table-row products; ciphertexts are the reference's encryption under that r"}
        pfb_check = (bases, Wp, ct3[:4].cpu().numpy().view(np.uint32).copy(), ex3[:4].cpu().numpy().copy())
        del ct3, ex3, valp, stp, cpub
        torch.cuda.empty_cache()
        if not okp:
            raise SystemExit("public fixed-base ciphertexts do not decrypt to the input")

    # ---- the 1024-bit key every reference protocol defaults to (VERDICT r5 Missing #2)
    nb1_check = None
    if cfg_id == 1 and solo and nb == 2048 and not args.no_nb1024 and use_fb:
        ctx.set_fb_window(16)                 # (the key holder's big tables are not needed after the timed region)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        extra["nb1024"], nb1_check = nb1024_leg(args, dev, stream, lib, rng_key, x, local_rank, index_base_chk + 7 * total)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel of the timed path
    alg_bytes = 4 + W * 4 + 4     # x in, ciphertext out, exponent out (r generated on the device)
    if cfg_id == 2:
        add_ms = float(np.mean([a.elapsed_time(b) for a, b in add_events]))
        dom, dom_ms, dom_work = "k_add", add_ms, work_add(exs8, nb) / N
        achieved = N * dom_work / (dom_ms * 1e-3)
        extra["k_add_ms"] = add_ms
    else:
        if grp_fb and fb_pair:
            names, works = ["k_fb_digits", "k_fbgp", "k_fbg_fin"], work_fbgp(nb, fb_info[2])
            if fb_split:   # same tables, same count, the split-pair kernel; Garner on lanes (k_sgp_w, k_sgp_fin)
                names[1] = "k_sgp"
                works["k_sgp"] = works.pop("k_fbgp")
                names[2] = "k_sgp_w+garner+fin"
                works.pop("k_fbg_fin")
                works[names[2]] = work_sgp_fin(nb)
                if fb_sgs:   # Shoup rows: k_sgs + k_sgs_bfin in the sampler stage
                    names[1] = "k_sgs+bfin"
                    works.pop("k_sgp")
                    works["k_sgs+bfin"] = work_sgs(nb, fb_info[2])
        elif grp_fb:
            names, works = ["k_fb_digits", "k_fbg", "k_fbg_fin"], work_fbg(nb, fb_info[2])
        elif use_crt and use_fb and fb_pair and fb_shoup:
            names, works = ["k_fb_digits", "k_fbs", "k_fbp_fin"], work_fbs(nb, fb_info[2])
        elif use_crt and use_fb and fb_pair:
            names, works = ["k_fb_digits", "k_fbp", "k_fbp_fin"], work_fbp(nb, fb_info[2])
        elif use_crt and use_fb:
            names, works = ["k_fb_digits", "k_fb", "k_fb_fin"], work_fb(nb, fb_info[2])
        elif use_crt:
            names, works = ["k_crt_a", "k_crt_b", "k_crt_fin"], work_crt(nb)
        else:
            names, works = ["k_encrypt"], {"k_encrypt": work_enc_public(nb)}
        stages = {nm: {"kernel_ms": ms, "work_mac_per_elem": works[nm],
                       "achieved_tmac_s": N * works[nm] / (ms * 1e-3) / 1e12}
                  for nm, ms in zip(names, stage_avg)}
        dom = max(stages, key=lambda nm: stages[nm]["kernel_ms"])
        dom_ms, dom_work = stages[dom]["kernel_ms"], works[dom]
        extra["stages"] = stages
        achieved = N * dom_work / (dom_ms * 1e-3)
        enc_ms = float(sum(stage_avg))
        extra["path"] = (("crt-fixedbase-shoup" if fb_shoup else "crt-fixedbase-pair") if fb_pair else "crt-fixedbase") \
            if use_fb else "crt" if use_crt else "public"
        if use_fb:
            extra["fixed_base"] = {"g_p": fb_info[0], "g_q": fb_info[1], "digits": fb_info[2], "window_bits": fb_info[3]}
        extra["encrypt_call_ms"] = enc_ms
        extra["path_int_mac_frac"] = N * sum(works.values()) / (enc_ms * 1e-3) / INT_MAC_PEAK
        extra["hbm_algorithmic_gbs"] = N * alg_bytes / (enc_ms * 1e-3) / 1e9
        # SURVEY.md §8d prices every encryption at the public-key work W_enc; the fraction it implies
        extra["w_enc_equivalent"] = {
            "frac_of_peak": (N / (enc_ms * 1e-3)) * work_enc_public(nb) / INT_MAC_PEAK,
            "note": "encrypt rate x SURVEY.md §8d W_enc / peak: > 1 means the path does less work than the "
                    "canonical public-key exponentiation, not a faster multiplier"}

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        from oracle import gmp_oracle
        if gmp_oracle.available():
            quota = cpu_quota()
            th = max(1, args.cpu_threads if args.cpu_threads else cpu_threads_default())
            cores = {**quota, "cpu_model": cpu_model()}
            # one thread first: the per-core rate, against which the threaded run's parallelism is measured
            S1 = min(S_chk, 256 if nb <= 2048 else 32)
            t1 = time.perf_counter()
            c1, e1 = gmp_oracle.encrypt_f32_chacha(pk.n, x_host[:S1], rng_key, index_base_chk, 1)
            single = S1 / (time.perf_counter() - t1)
            S = S_chk
            t1 = time.perf_counter()
            cct, cex = gmp_oracle.encrypt_f32_chacha(pk.n, x_host[:S], rng_key, index_base_chk, th)
            cdt = time.perf_counter() - t1
            same = bool(np.array_equal(ct_host_check[:S], cct) and np.array_equal(ex_host_check[:S], cex)
                        and np.array_equal(c1, cct[:S1]) and np.array_equal(e1, cex[:S1]))
            eff = (S / cdt) / single
            throttled = eff < 0.7 * th
            cpu = {"value": S / cdt, "unit": "encrypts/s", "cores": th, "kind": "port",
                   "kind_detail": ("port (oracle/gmp_oracle.c); " +
                                   (f"THROTTLED: {th} threads delivered {eff:.1f} cores of work" if throttled
                                    else f"{th} threads delivered {eff:.1f} cores of work")),
                   "single_thread_per_s": single, "single_thread_sample": S1,
                   "cores_effective": eff, "throttled": throttled,
                   "sample": f"first {S} elements of the rank-0 vector with the same ChaCha20 obfuscators; "
                             f"GMP 6.2.1 mpz_powm(r, n, n^2) per element (the library gmpy2 2.0.8 wraps, "
                             f"obfuscator.py:36), {th} worker threads like the reference's Pool(cpu_count()), "
                             f"capped by the cgroup quota; the first {S1} also on one thread",
                   "extrapolated_full_job_s": N / (S / cdt),
                   "per_core_extrapolated_full_job_s": N / single,
                   "gpu_bit_exact_on_sample": same, **cores}
            if not same:
                raise SystemExit("GPU ciphertexts differ from the GMP oracle on the CPU sample")
            if use_fb:
                # the timed (fixed-base) ciphertexts against the oracle's restatement of the sampler
                from oracle import paillier_oracle as O
                okey = O.Key(pk.n, sk.p, sk.q)
                idx = sorted({0, 1, S_chk // 2, S_chk - 1})
                got = _native.words_to_ints(ct_timed_check[idx])
                fb_ok = all(O.fb_encrypt_value(x_host[i], okey, rng_key, index_base_chk + i, fb_info)
                            == (got[j], int(ex_host_check[i])) for j, i in enumerate(idx))
                cpu["fixed_base_bit_exact_vs_oracle"] = {"elements": idx, "ok": fb_ok}
                if not fb_ok:
                    raise SystemExit("fixed-base ciphertexts differ from the oracle restatement")
            if c3_seams is not None:
                # the configs[3] leg's last step at its shard seams
                from oracle import paillier_oracle as O
                leg3, gidx, xs3, got3, ex3 = c3_seams
                okey = O.Key(pk.n, sk.p, sk.q)
                ok3 = all(O.fb_encrypt_value(xv, okey, rng_key, gi, fb_info) == (cv, ev)
                          for gi, xv, cv, ev in zip(gidx, xs3, got3, ex3))
                leg3["check"]["seams_vs_oracle"] = {"global_index": gidx, "ok": ok3}
                if not ok3:
                    raise SystemExit("configs[3]: seam ciphertexts differ from the oracle restatement")
            if pfb_check is not None:
                from oracle import paillier_oracle as O
                bases, Wp, cts, exs = pfb_check
                okey = O.Key(pk.n, sk.p, sk.q)
                got = _native.words_to_ints(cts)
                pok = all(O.pfb_encrypt_value(x_host[i], okey, bases, rng_key, index_base_chk + i, Wp)
                          == (got[i], int(exs[i])) for i in range(len(got)))
                cpu["public_fixed_base_bit_exact_vs_oracle"] = {"elements": list(range(len(got))), "ok": pok}
                if not pok:
                    raise SystemExit("public fixed-base ciphertexts differ from the oracle restatement")
            if nb1_check is not None:
                # the nb = 1024 leg: its generic CRT prefix against the GMP port, its fixed-base outputs against the
                # oracle's restatement of the sampler
                from oracle import paillier_oracle as O
                g1, e1g = nb1_check["generic"]
                s1 = len(g1)
                x1 = x_host[:s1]
                cc1, ce1 = gmp_oracle.encrypt_f32_chacha(nb1_check["n"], x1, rng_key, nb1_check["base"], th)
                ok1 = bool(np.array_equal(g1, cc1) and np.array_equal(e1g, ce1))
                okey1 = O.Key(nb1_check["n"], nb1_check["p"], nb1_check["q"])
                got1 = _native.words_to_ints(nb1_check["fb_ct"])
                okf = all(O.fb_encrypt_value(x_host[i], okey1, rng_key, nb1_check["base"] + i, nb1_check["fb_info"])
                          == (got1[j], int(nb1_check["fb_ex"][j])) for j, i in enumerate(nb1_check["fb_idx"]))
                extra["nb1024"]["check"] = {"generic_prefix_bit_exact_vs_gmp": {"elements": s1, "ok": ok1},
                                            "fixed_base_bit_exact_vs_oracle": {"elements": nb1_check["fb_idx"], "ok": okf}}
                if not (ok1 and okf):
                    raise SystemExit(f"nb = 1024 leg differs from the GMP port / oracle: {extra['nb1024']['check']}")
            # configs[0] timed in full: nb = 1024, 1000 elements, encrypt + decrypt, threads = os.cpu_count()
            pk0, sk0 = generate_paillier_keypair(1024, seed=1)
            x0 = np.random.default_rng(0).standard_normal(1000, dtype=np.float32)
            t1 = time.perf_counter()
            c0, _ = gmp_oracle.encrypt_f32_chacha(pk0.n, x0, rng_key, 0, th)
            t_e0 = time.perf_counter() - t1
            t1 = time.perf_counter()
            gmp_oracle.decrypt_raw(sk0.p, sk0.q, c0, th)
            t_d0 = time.perf_counter() - t1
            extra["config0_cpu"] = {"workload": CONFIGS[0]["desc"], "encrypt_per_s": 1000 / t_e0,
                                    "decrypt_per_s": 1000 / t_d0, "encrypt_s": t_e0, "decrypt_s": t_d0,
                                    "threads": th, **cores, "kind": "port (oracle/gmp_oracle.c)"}

    path_label = (("key holder: fixed-base r^n sampler on the lane-group engine" if grp_fb
                   else "key holder: CRT, fixed-base r^n sampler") if use_fb
                  else "key holder: CRT" if use_crt else "public-key")
    metric = {1: "Paillier-2048 encrypts/sec (device-resident), 1M-elem float32 array",
              2: "Paillier-2048 encrypt + 8-way add + decrypt, elements/sec (device-resident), 1M-elem arrays"}
    out = {
        "metric": metric.get(cfg_id, f"Paillier-{nb} encrypts/sec (device-resident)") if nb == cfg["nb"]
        else f"Paillier-{nb} encrypts/sec (device-resident)",
        "value": value,
        "unit": "encrypts/s" if cfg_id != 2 else "elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": cfg["shard"],
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: numpy default_rng(rank).standard_normal float32; seeded key "
                "generate_paillier_keypair(nb, seed=1); device ChaCha20 obfuscators keyed by global index",
        "config": {"workload": cfg["desc"] + " (" + path_label + " path"
                               + (", RCCL all-gather of ciphertext shards in the step" if world > 1 else "") + ")",
                   "baseline_config": cfg_id, "key_bits": nb,
                   "elements_total": total if cfg["shard"] == "strong" else world * N,
                   "elements_per_gpu": N, "parallelism": f"dp{world}",
                   "world_size_seen": dist.get_world_size() if world > 1 else 1},
        "roofline": {"bound": "valu-int-mac", "achieved": achieved / 1e12, "peak": INT_MAC_PEAK / 1e12,
                     "unit": "TMAC/s", "frac": achieved / INT_MAC_PEAK,
                     "traffic": load_traffic("k_sgs" if dom == "k_sgs+bfin" else dom, N, nb,   # (k_sgs's launch: the rows)
                                             fb_info[3] if (use_fb and dom in ("k_fb", "k_fbp", "k_fbs", "k_fbg", "k_fbgp", "k_sgp",
                                                                               "k_sgs+bfin")) else None),
                     "kernel": dom, "kernel_ms": dom_ms,
                     "work_per_unit": (f"{dom_work:.4g} MAC per element: the Shoup-row count (K - 1 = {fb_info[2] - 1} Shoup products "
                                       f"mod p_h^2 per half (the first of K rows is the start), 3 s^2 + 3 s each over s = nb/64 32-bit limbs of p_h, + the c0 sum "
                                       f"and the b-sum correction, kernels_fbs.hpp), not SURVEY.md §8d's W_enc"
                                       if dom == "k_fbs" else
                                       f"{dom_work:.4g} MAC per element: the Shoup-row count at nb = 4096 (K - 1 = {fb_info[2] - 1} Shoup "
                                       f"products mod p_h^2 per half, 3 s^2 + 3 s each over s = nb/64 32-bit limbs of p_h, + k_sgs_bfin's "
                                       f"pass by the constant c_A and b-sum product, kernels_sgs.hpp), not SURVEY.md §8d's W_enc"
                                       if dom == "k_sgs+bfin" else
                                       f"{dom_work:.4g} MAC per element: the fixed-base count (K = {fb_info[2]} products by "
                                       f"factored rows (a, 0) mod p_h^2 per half, 4 s^2 + 2 s each over s = nb/64 32-bit limbs "
                                       f"of p_h, + the c0 sum and the b-sum correction, "
                                       f"{'kernels_fbp.hpp' if dom == 'k_fbp' else 'kernels_sgp.hpp' if dom == 'k_sgp' else 'kernels_grp_pair.hpp'}), not SURVEY.md §8d's W_enc"
                                       if dom in ("k_fbp", "k_fbgp", "k_sgp") else
                                       f"{dom_work:.4g} MAC per element: the fixed-base count (K = {fb_info[2]} table "
                                       f"products per half, 32-bit limbs, kernels_fb.hpp), not SURVEY.md §8d's W_enc"
                                       if dom in ("k_fb", "k_fbg") else f"{dom_work:.4g} canonical 32x32->64 MAC per element (SURVEY.md §8d)")},
        "roofline_hbm": {"bound": "hbm", "achieved": extra.get("hbm_algorithmic_gbs"), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": (extra["hbm_algorithmic_gbs"] / HBM_PEAK_GBS) if "hbm_algorithmic_gbs" in extra else None,
                         "algorithmic_bytes_per_unit": alg_bytes},
        "cpu_baseline": cpu,
        "setup": setup,
        "extra": extra,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
