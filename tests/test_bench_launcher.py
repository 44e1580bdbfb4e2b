"""bench.py --gpus N without torchrun starts the N rank processes itself (bench.py:launch_ranks); the CPU
self-test runs them on gloo and reports the world the process group sees. The reference splits the same
array element-wise over a process pool (flex/crypto/paillier/encryptor.py:89-96)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest-cpu"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout       # only rank 0 prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_launcher_spawns_ranks(n):
    d = _run(n)
    assert d["n_gpus"] == n and d["world_size_seen"] == n
    assert d["shard_owners"] == list(range(n)) and d["gather_ok"]


def test_launcher_propagates_failure():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FLEXPAI_SELFTEST_FAIL_RANK"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--selftest-cpu"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 3
