import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ibond-flex_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# The parity tests pin the fixed-base sampler's outputs on small inputs (a few to a few hundred elements),
# below the library's build break-even (include/flexpai.h pai_ctx_fixed_base_policy): build the tables on
# the first device-RNG call, as before the policy existed. The policy itself is tested with this unset
# (test_gpu_fixed_base.py::test_fresh_key_small_call_skips_tables).
os.environ.setdefault("FLEXPAI_FB_MIN_ELEMS", "0")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """PyTorch-ROCm ships its own HIP and HSA runtimes; in one process the runtime that opens the device first
    wins, and torch's fails ("No HIP GPUs are available") once libflexpai's has started. GPU test sessions that
    use torch buffers therefore start torch's runtime before any flexpai call (PyTorch)."""
    mark = request.config.getoption("-m") or ""
    if "gpu" in mark and "not gpu" not in mark:
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:   # noqa: BLE001 - a session without a usable torch still runs the C-ABI tests
            pass
    yield


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_fb():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_fb.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_pfb():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "paillier_golden_pfb.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def xlib():
    """The test-only build of the C ABI (libflexpai_xcheck.so, __graft_entry__.build): the product kernels plus the
    generations they replaced, selected by $FLEXPAI_FB_PAIR=0 / $FLEXPAI_SGP=0 / $FLEXPAI_PAIR=0, for the
    cross-checks. Contexts on it: _native.Context(..., lib=xlib)."""
    from flex.crypto.paillier import _native
    return _native.load_library(_native.XCHECK_LIB_PATH)
