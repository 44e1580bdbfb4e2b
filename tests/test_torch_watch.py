"""The late-torch warning of _native.load_library: a process that starts libflexpai's HIP runtime
and imports torch afterwards gets one RuntimeWarning at that import when torch.cuda then sees no GPU (the two HIP
runtimes of one process: the first to open the device keeps it). Run in fresh interpreters: torch must not be
imported yet. On this CPU container torch.cuda.is_available() is False, which is exactly the condition reported."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ibond-flex_amd")

SCRIPT = r"""
import sys, warnings
sys.path[:0] = [{root!r}, {pkg!r}]
from flex.crypto.paillier import _native as N
assert "torch" not in sys.modules
N.load_library()                      # torch absent: the watch is armed
assert N._torch_watch is not None
N._runtime_started = {started}        # as after the first context (no GPU here to create one)
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    import torch
assert N._torch_watch is None         # one shot
import importlib.machinery
assert not any(isinstance(f, N._LateTorchWatch) for f in sys.meta_path)
hits = [str(x.message) for x in w if issubclass(x.category, RuntimeWarning) and "imported after libflexpai" in str(x.message)]
print("HITS", len(hits), torch.cuda.is_available())
"""


def _run(started):
    out = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT, pkg=PKG, started=started)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout.strip().splitlines()[-1]


def test_late_torch_import_warns_once_after_the_runtime_started():
    assert _run(True) == "HITS 1 False"


def test_late_torch_import_is_silent_before_any_context():
    assert _run(False) == "HITS 0 False"
