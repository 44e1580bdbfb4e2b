"""ctypes binding of libflexpai.so, the MI355X Paillier engine (C ABI: include/flexpai.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950)
and is REQUIRED: there is no CPU fallback. Loading fails loudly if it is missing.
"""
from __future__ import annotations

import collections
import ctypes
import os
import sys
import threading
import warnings
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLEXPAI_LIB") or os.path.join(_HERE, "libflexpai.so")   # override: experiments only
# the test-only build (FLEXPAI_XCHECK): also holds the kernel generations the tests still cross-check against
# (k_fbgp, k_pfb, k_fbp), selected by $FLEXPAI_SGP=0 / $FLEXPAI_FBS=0, and honours $FLEXPAI_PAIR=0
XCHECK_LIB_PATH = os.path.join(_HERE, "libflexpai_xcheck.so")

PAI_F32, PAI_F64, PAI_I64 = 0, 1, 2
PAI_OBF_NONE, PAI_OBF_GIVEN, PAI_OBF_RNG = 0, 1, 2
PAI_EXP_AUTO, PAI_EXP_FIXED = 0, 1
EL_OK, EL_INT, EL_INT_BIG, EL_OVERFLOW, EL_FLOAT_OVF, EL_ENC_RANGE = 0, 1, 2, 3, 4, 5

PAI_OPT_CRT_ENCRYPT, PAI_OPT_CRT_AVAILABLE, PAI_OPT_STAGE_TIMING, PAI_OPT_LANE_DECRYPT = 1, 2, 3, 4
PAI_OPT_FIXED_BASE, PAI_OPT_FB_WINDOW, PAI_OPT_FB_READY, PAI_OPT_FB_PAIR, PAI_OPT_PAIR = 5, 6, 7, 8, 9
PAI_OPT_SPLIT_SAMPLER, PAI_OPT_ROWS_MAX = 13, 14
PAI_OPT_PUBLIC_FB, PAI_OPT_PFB_READY, PAI_OPT_PFB_WINDOW = 10, 11, 12
PFB_NBASES = 33

EXPORTED = ("pai_device_count", "pai_device_mem_info", "pai_ctx_create", "pai_ctx_set_private", "pai_ctx_destroy", "pai_ctx_info", "pai_last_error",
            "pai_ctx_set_option", "pai_ctx_get_option", "pai_ctx_stage_times", "pai_ctx_fixed_base_info",
            "pai_ctx_fixed_base_prepare", "pai_ctx_fixed_base_setup", "pai_ctx_fixed_base_policy",
            "pai_ctx_public_fb_prepare", "pai_ctx_public_fb_set_bases", "pai_ctx_public_fb_info",
            "pai_ctx_public_fb_policy",
            "pai_encrypt", "pai_add", "pai_decrypt", "pai_encrypt_dev", "pai_add_dev", "pai_decrypt_dev",
            "pai_mul", "pai_mul_dev", "pai_matmul", "pai_matmul_dev", "pai_add_plain", "pai_add_plain_dev",
            "pai_segment_add", "pai_segment_add_dev", "pai_comm_unique_id", "pai_comm_create", "pai_comm_destroy",
            "pai_allgather_dev", "pai_allgather_shards_dev", "pai_release_table_cache")
PAI_COMM_ID_BYTES = 128

_lib = None
_libs = {}
_lib_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libflexpai.so (or another build of the C ABI, e.g. XCHECK_LIB_PATH) and declare the C signatures.
    Raises if the library is absent."""
    global _lib
    with _lib_lock:
        if path in _libs:
            return _libs[path]
        if not os.path.exists(path):
            raise NativeError(f"flexpai native library not found at {path}; run __graft_entry__.build() "
                              f"(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        _start_torch_runtime_first()
        if "torch" not in sys.modules:
            _watch_late_torch_import()
        lib = ctypes.CDLL(path)
        P, S, I, U64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        lib.pai_device_count.argtypes = [P]
        lib.pai_device_mem_info.argtypes = [I, P, P]
        lib.pai_ctx_create.argtypes = [P, S, I, ctypes.POINTER(ctypes.c_void_p)]
        lib.pai_ctx_set_private.argtypes = [P, P, P, S]
        lib.pai_ctx_destroy.argtypes = [P]
        lib.pai_ctx_destroy.restype = None
        lib.pai_ctx_info.argtypes = [P, P, P, P]
        lib.pai_last_error.restype = ctypes.c_char_p
        lib.pai_ctx_set_option.argtypes = [P, I, I]
        lib.pai_ctx_get_option.argtypes = [P, I, P]
        lib.pai_ctx_stage_times.argtypes = [P, P, I, P]
        lib.pai_ctx_fixed_base_info.argtypes = [P, P, P, P, P]
        lib.pai_ctx_fixed_base_prepare.argtypes = [P]
        lib.pai_ctx_fixed_base_setup.argtypes = [P, P, P, P]
        lib.pai_ctx_fixed_base_policy.argtypes = [P, P, P]
        lib.pai_ctx_public_fb_prepare.argtypes = [P]
        lib.pai_ctx_public_fb_set_bases.argtypes = [P, P, S, I]
        lib.pai_ctx_public_fb_info.argtypes = [P, P, S, P, P, P, P]
        lib.pai_ctx_public_fb_policy.argtypes = [P, P, P]
        lib.pai_encrypt.argtypes = [P, I, P, S, I, ctypes.c_int32, I, P, S, S, P, U64, P, P, P]
        lib.pai_add.argtypes = [P, P, P, I, S, P, P]
        lib.pai_decrypt.argtypes = [P, P, P, S, P, P, P, P]
        lib.pai_encrypt_dev.argtypes = [P, I, P, S, I, ctypes.c_int32, I, P, S, S, P, U64, P, P, P, P]
        lib.pai_add_dev.argtypes = [P, P, P, I, S, P, P, P]
        lib.pai_decrypt_dev.argtypes = [P, P, P, S, P, P, P, P, P]
        lib.pai_mul.argtypes = [P, P, P, S, I, P, S, P, P, P]
        lib.pai_mul_dev.argtypes = [P, P, P, S, I, P, S, P, P, P, P]
        lib.pai_add_plain.argtypes = [P, P, P, S, I, P, S, P, P, P]
        lib.pai_add_plain_dev.argtypes = [P, P, P, S, I, P, S, P, P, P, P]
        lib.pai_segment_add.argtypes = [P, P, P, S, P, P, S, P, P]
        lib.pai_segment_add_dev.argtypes = [P, P, P, S, P, P, S, P, P, P]
        lib.pai_matmul.argtypes = [P, P, P, S, S, I, P, S, P, P]
        lib.pai_matmul_dev.argtypes = [P, P, P, S, S, I, P, S, P, P, P]
        lib.pai_comm_unique_id.argtypes = [P]
        lib.pai_comm_create.argtypes = [P, I, I, I, ctypes.POINTER(ctypes.c_void_p)]
        lib.pai_comm_destroy.argtypes = [P]
        lib.pai_comm_destroy.restype = None
        lib.pai_allgather_dev.argtypes = [P, P, S, P, P]
        lib.pai_allgather_shards_dev.argtypes = [P, P, P, S, I, P, P, P]
        lib.pai_release_table_cache.argtypes = []
        lib.pai_release_table_cache.restype = None
        for name in EXPORTED:
            if name not in ("pai_ctx_destroy", "pai_last_error", "pai_comm_destroy", "pai_release_table_cache"):
                getattr(lib, name).restype = ctypes.c_int
        _libs[path] = lib
        if path == LIB_PATH:
            _lib = lib
        return lib


def release_table_cache() -> None:
    """Give the device memory of released fixed-base tables back to the driver now (csrc/table_arena.hpp: the library
    keeps it for the process's next table build until its last context is destroyed)."""
    load_library().pai_release_table_cache()


def _start_torch_runtime_first() -> None:
    """PyTorch-ROCm wheels bundle their own HIP and HSA runtimes. In one process only the runtime that opens the
    GPU first works: once libflexpai's (/opt/rocm) runtime has started, torch.cuda fails with "No HIP GPUs are
    available". A process that has already imported torch (device buffers for the *_dev entry points, a
    torch.distributed job) gets torch's runtime started here, before flexpai's first HIP call; torch is never
    imported by this package. See INTEGRATION.md (PyTorch)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or os.environ.get("FLEXPAI_NO_TORCH_INIT"):
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:   # noqa: BLE001 - torch without a usable GPU: flexpai's own runtime still works
        pass


_runtime_started = False   # a context was created: libflexpai's HIP runtime holds the GPU
_torch_watch = None


class _LateTorchWatch:
    """sys.meta_path finder armed when libflexpai loads before torch: when torch is imported later, after
    libflexpai's runtime has opened the GPU, torch's own HIP runtime cannot (torch.cuda.is_available() is False).
    Warn once at that import instead of leaving the caller to find the failure. One shot:
    the finder removes itself at torch's import and never changes what is imported."""

    def find_spec(self, name, path=None, target=None):
        if name != "torch":
            return None
        _disarm_torch_watch()
        import importlib.machinery
        spec = importlib.machinery.PathFinder.find_spec(name, path)
        loader = getattr(spec, "loader", None)
        if loader is None or not hasattr(loader, "exec_module"):
            return spec
        inner = loader.exec_module

        def exec_module(module):
            inner(module)
            _check_torch_after_flexpai(module)

        loader.exec_module = exec_module   # (this loader instance only: it loads torch's __init__ and nothing else)
        return spec


def _watch_late_torch_import() -> None:
    global _torch_watch
    if _torch_watch is None and not os.environ.get("FLEXPAI_NO_TORCH_INIT"):
        _torch_watch = _LateTorchWatch()
        sys.meta_path.insert(0, _torch_watch)


def _disarm_torch_watch() -> None:
    global _torch_watch
    if _torch_watch is not None:
        try:
            sys.meta_path.remove(_torch_watch)
        except ValueError:
            pass
        _torch_watch = None


def _check_torch_after_flexpai(torch) -> bool:
    """True (and a RuntimeWarning) when torch was imported after libflexpai started the GPU and torch cannot see it."""
    if not _runtime_started:
        return False
    try:
        ok = bool(torch.cuda.is_available())
    except Exception:   # noqa: BLE001 - a torch without a HIP build: nothing of ours to report
        return False
    if ok:
        return False
    warnings.warn("flexpai: torch was imported after libflexpai started the GPU, and torch.cuda now reports no GPU "
                  "(two HIP runtimes in one process: the first to open the device keeps it). Import torch before "
                  "the first Paillier call; see INTEGRATION.md (PyTorch).", RuntimeWarning, stacklevel=2)
    return True


def device_count() -> int:
    """GPUs visible to the engine (0 without one). Raises when libflexpai.so is missing."""
    n = ctypes.c_int()
    _check(load_library().pai_device_count(ctypes.byref(n)))
    return n.value


def device_mem_info(device: int = 0):
    """(free, total) device memory in bytes, through the engine's own HIP runtime."""
    fr, tot = ctypes.c_uint64(), ctypes.c_uint64()
    _check(load_library().pai_device_mem_info(device, ctypes.byref(fr), ctypes.byref(tot)))
    return fr.value, tot.value


class Comm:
    """RCCL communicator of the C ABI's shard all-gather (pai_comm_*): one per rank, one process per GPU.
    Rank 0 makes the id (Comm.unique_id()) and passes it to the others over any channel."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * PAI_COMM_ID_BYTES)()
        _check(load_library().pai_comm_unique_id(buf))
        return bytes(buf)

    def _chk(self, rc: int):
        _check(rc, self.lib)

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        if len(uid) != PAI_COMM_ID_BYTES:
            raise ValueError("communicator id must be %d bytes" % PAI_COMM_ID_BYTES)
        self.lib = load_library()
        h = ctypes.c_void_p()
        self._chk(self.lib.pai_comm_create(uid, world, rank, device, ctypes.byref(h)))
        self._h, self.world, self.rank = h, world, rank

    def allgather_shards(self, d_ct: int, d_exp: int, n_per_rank: int, ct_words: int, d_ct_all: int,
                         d_exp_all: int, stream: int = 0):
        """Device pointers (e.g. torch tensor .data_ptr()); asynchronous on `stream`."""
        self._chk(self.lib.pai_allgather_shards_dev(self._h, d_ct, d_exp, n_per_rank, ct_words, d_ct_all, d_exp_all,
                                                 stream or None))

    def close(self):
        if getattr(self, "_h", None):
            self.lib.pai_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _check(rc: int, lib=None):
    if rc != 0:
        msg = (lib or load_library()).pai_last_error().decode(errors="replace")
        if rc == -5:
            raise ZeroDivisionError(msg)          # gmpy_math.invert (gmpy_math.py:71-72)
        if rc == -4 and ("does not match" in msg or "have to be different" in msg):
            raise ValueError(msg)
        raise NativeError(f"flexpai error {rc}: {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def int_to_le(v: int, nbytes: int) -> bytes:
    return int(v).to_bytes(nbytes, "little")


class Context:
    """One key on one GPU. Created lazily by the Python layer (never pickled, never forked)."""

    def __init__(self, n: int, device: int = 0, p: Optional[int] = None, q: Optional[int] = None, lib=None):
        """lib: another build of the C ABI (load_library(XCHECK_LIB_PATH) in the cross-check tests)."""
        self.lib = lib or load_library()
        self.n = n
        nbytes = (n.bit_length() + 7) // 8
        buf = int_to_le(n, nbytes)
        h = ctypes.c_void_p()
        self._chk(self.lib.pai_ctx_create(buf, nbytes, device, ctypes.byref(h)))
        global _runtime_started
        _runtime_started = True
        self._h = h
        kb, cw, pw = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.pai_ctx_info(h, ctypes.byref(kb), ctypes.byref(cw), ctypes.byref(pw)))
        self.key_bits, self.ct_words, self.pt_words = kb.value, cw.value, pw.value
        self.has_private = False
        self.calls = collections.Counter()     # C-ABI entry points this context has run (tests, stats)
        if p is not None:
            self.set_private(p, q)

    def _chk(self, rc: int):
        _check(rc, self.lib)

    @property
    def handle(self):
        return self._h

    def set_private(self, p: int, q: int):
        hb = max(p.bit_length(), q.bit_length()) // 8 + 1
        self._chk(self.lib.pai_ctx_set_private(self._h, int_to_le(p, hb), int_to_le(q, hb), hb))
        self.has_private = True
        if os.environ.get("FLEXPAI_CRT", "1").strip() == "0":
            self.set_crt(False)

    def _get_option(self, opt: int) -> int:
        v = ctypes.c_int()
        self._chk(self.lib.pai_ctx_get_option(self._h, opt, ctypes.byref(v)))
        return v.value

    @property
    def crt_available(self) -> bool:
        """True when the private key is set and the CRT encryption kernels fit this key size."""
        return bool(self._get_option(PAI_OPT_CRT_AVAILABLE))

    @property
    def crt_enabled(self) -> bool:
        return bool(self._get_option(PAI_OPT_CRT_ENCRYPT))

    def set_stage_timing(self, enabled: bool):
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_STAGE_TIMING, 1 if enabled else 0))

    def stage_times(self):
        """Kernel durations (ms) of the last encrypt call (needs set_stage_timing(True))."""
        buf = (ctypes.c_float * 8)()
        cnt = ctypes.c_int()
        self._chk(self.lib.pai_ctx_stage_times(self._h, buf, 8, ctypes.byref(cnt)))
        return [float(buf[i]) for i in range(cnt.value)]

    @property
    def rows_max(self) -> int:
        """Largest CRT encryption / decryption call (elements) that runs on 16-lane rows (k_crt_w / k_dec_w)."""
        return int(self._get_option(PAI_OPT_ROWS_MAX))

    def set_rows_max(self, n: int):
        """0 keeps every CRT encryption / decryption on the lane kernels (k_crt_a + k_crt_b_pair, k_dec_*_pair); same bits."""
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_ROWS_MAX, int(n)))

    def set_crt(self, enabled: bool):
        """Encrypt through the private-key CRT kernels (default when available) or the public-key one.
        The ciphertext bits are identical either way."""
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_CRT_ENCRYPT, 1 if enabled else 0))

    @property
    def lane_decrypt(self) -> bool:
        """True when decrypt runs on the lane engine (kernels_dec.hpp), False for the lane-group kernel."""
        return bool(self._get_option(PAI_OPT_LANE_DECRYPT))

    def set_lane_decrypt(self, enabled: bool):
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_LANE_DECRYPT, 1 if enabled else 0))

    @property
    def fixed_base(self) -> bool:
        """True when device-RNG encryption samples r^n through the fixed bases (kernels_fb.hpp)."""
        return bool(self._get_option(PAI_OPT_FIXED_BASE))

    def set_fixed_base(self, enabled: bool):
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_FIXED_BASE, 1 if enabled else 0))

    def fixed_base_info(self):
        """(g_p, g_q, K, W): the generators, the exponent digit count and the digit window (bits) of
        the fixed-base path."""
        gp, gq, k, w = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.pai_ctx_fixed_base_info(self._h, ctypes.byref(gp), ctypes.byref(gq), ctypes.byref(k),
                                                ctypes.byref(w)))
        return gp.value, gq.value, k.value, w.value

    @property
    def fb_window(self) -> int:
        """Window of the resident fixed-base tables (else the requested one)."""
        return self._get_option(PAI_OPT_FB_WINDOW)

    def set_fb_window(self, bits: int):
        """Digit window of the fixed-base tables (8, 12, 16 or 20 .. 24); the tables are rebuilt lazily."""
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_FB_WINDOW, int(bits)))

    @property
    def fb_ready(self) -> bool:
        """True when the fixed-base tables are resident on the device."""
        return bool(self._get_option(PAI_OPT_FB_READY))

    @property
    def fb_pair(self) -> int:
        """Limbs of p_h of the resident pair tables (kernels_fbs.hpp: k_fbs; kernels_fbp.hpp: k_fbp in the test build),
        0 for k_fb tables or none."""
        return int(self._get_option(PAI_OPT_FB_PAIR))

    @property
    def split_sampler(self) -> int:
        """Bit 0: the 4096-bit key-holder tables, bit 1: the public tables are sampled by k_sgp (kernels_sgp.hpp);
        bit 2: the 1024/2048-bit key-holder tables hold Shoup rows sampled by k_fbs (kernels_fbs.hpp)."""
        return int(self._get_option(PAI_OPT_SPLIT_SAMPLER))

    @property
    def pair_paths(self) -> int:
        """Bit 0: decryption, bit 1: CRT encryption stage B on p-adic pairs (kernels_pair.hpp)."""
        return int(self._get_option(PAI_OPT_PAIR))

    def prepare_fixed_base(self):
        """Build the fixed-base tables now (NativeError with the reason when unavailable)."""
        self._chk(self.lib.pai_ctx_fixed_base_prepare(self._h))

    def fixed_base_setup(self):
        """(host_ms, device_ms, table_bytes) of the last table build."""
        hm, dm, tb = ctypes.c_float(), ctypes.c_float(), ctypes.c_uint64()
        self._chk(self.lib.pai_ctx_fixed_base_setup(self._h, ctypes.byref(hm), ctypes.byref(dm), ctypes.byref(tb)))
        return float(hm.value), float(dm.value), int(tb.value)

    def fixed_base_policy(self):
        """(seen, threshold): device-RNG elements encrypted under this key so far, and the count at which
        the fixed-base tables get built (0 once resident or unavailable); include/flexpai.h."""
        seen, thr = ctypes.c_longlong(), ctypes.c_longlong()
        self._chk(self.lib.pai_ctx_fixed_base_policy(self._h, ctypes.byref(seen), ctypes.byref(thr)))
        return int(seen.value), int(thr.value)

    # ------------------------------------------------------ public-key fixed bases (kernels_pfb.hpp)
    @property
    def public_fixed_base(self) -> bool:
        """True when device-RNG encryption without the private key may use the public fixed bases."""
        return bool(self._get_option(PAI_OPT_PUBLIC_FB))

    def set_public_fixed_base(self, enabled: bool):
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_PUBLIC_FB, 1 if enabled else 0))

    @property
    def pfb_ready(self) -> bool:
        return bool(self._get_option(PAI_OPT_PFB_READY))

    def set_pfb_window(self, bits: int):
        """Digit window of the public tables: 12, 16 or 20 (the windows pinned to the reference's goldens)."""
        self._chk(self.lib.pai_ctx_set_option(self._h, PAI_OPT_PFB_WINDOW, int(bits)))

    def prepare_public_fixed_base(self):
        self._chk(self.lib.pai_ctx_public_fb_prepare(self._h))

    def set_public_bases(self, bases: Sequence[int]):
        """Fix the 33 bases g_0..g_32 instead of drawing them (tests, reproducible runs). Each must be a unit
        in (1, n), all distinct, and g_0 must have Jacobi symbol -1 mod n (else NativeError)."""
        nb = (self.n.bit_length() + 7) // 8
        buf = b"".join(int_to_le(g, nb) for g in bases)
        self._chk(self.lib.pai_ctx_public_fb_set_bases(self._h, buf, nb, len(bases)))

    def public_fixed_base_info(self):
        """(bases, K, W, K0) of the resident public tables."""
        nb = (self.n.bit_length() + 7) // 8
        buf = (ctypes.c_uint8 * (nb * PFB_NBASES))()
        nbs, k, w, k0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.pai_ctx_public_fb_info(self._h, buf, nb, ctypes.byref(nbs), ctypes.byref(k), ctypes.byref(w),
                                               ctypes.byref(k0)))
        raw = bytes(buf)
        bases = [int.from_bytes(raw[j * nb:(j + 1) * nb], "little") for j in range(nbs.value)]
        return bases, k.value, w.value, k0.value

    def public_fixed_base_policy(self):
        seen, thr = ctypes.c_longlong(), ctypes.c_longlong()
        self._chk(self.lib.pai_ctx_public_fb_policy(self._h, ctypes.byref(seen), ctypes.byref(thr)))
        return int(seen.value), int(thr.value)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.pai_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_words(self, ct: np.ndarray, exp: np.ndarray, N: int):
        """Host buffers must be exactly [N, ct_words] words and N exponents: the C ABI reads N * ct_words."""
        if ct.dtype != np.uint32 or ct.shape != (N, self.ct_words) or exp.shape != (N,):
            raise ValueError(f"ciphertext buffer shape {ct.shape} / exponents {exp.shape} do not match "
                             f"({N}, {self.ct_words})")

    # ----------------------------------------------------------------- host-buffer ops
    def encrypt(self, x: np.ndarray, exp_mode: int = PAI_EXP_AUTO, fixed_exp: int = 0,
                obf_mode: int = PAI_OBF_RNG, r: Optional[Sequence[int]] = None, r_scalar: Optional[int] = None,
                rng_key: Optional[bytes] = None, index_base: int = 0,
                out: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Host buffers in and out. `out` = (ct [N, W] uint32, exp [N] int32, status [N] int32) to reuse
        caller buffers (a streaming sender's), else fresh arrays."""
        x = np.ascontiguousarray(x)
        if x.dtype == np.float32:
            dt = PAI_F32
        elif x.dtype == np.float64:
            dt = PAI_F64
        elif x.dtype == np.int64:
            dt = PAI_I64
        else:
            raise TypeError(f"unsupported dtype {x.dtype}")
        N = x.size
        if out is not None:
            ct, ex, st = out
            if not (ct.dtype == np.uint32 and ct.shape == (N, self.ct_words) and ct.flags.c_contiguous and
                    ex.dtype == np.int32 and ex.shape == (N,) and ex.flags.c_contiguous and
                    st.dtype == np.int32 and st.shape == (N,) and st.flags.c_contiguous):
                raise ValueError("out must be C-contiguous (uint32 [N, ct_words], int32 [N], int32 [N])")
        else:
            ct = np.empty((N, self.ct_words), dtype=np.uint32)
            ex = np.empty(N, dtype=np.int32)
            st = np.empty(N, dtype=np.int32)
        r_buf, r_stride, r_bytes = None, 0, 0
        if obf_mode == PAI_OBF_GIVEN:
            r_bytes = self.ct_words * 4
            if r_scalar is not None:
                r_buf = np.frombuffer(int_to_le(r_scalar, r_bytes), dtype=np.uint8).copy()
                r_stride = 0
            else:
                r_buf = np.frombuffer(b"".join(int_to_le(v, r_bytes) for v in r), dtype=np.uint8).copy()
                r_stride = r_bytes
        key = rng_key if rng_key is not None else os.urandom(32)
        self.calls["pai_encrypt"] += 1
        self._chk(self.lib.pai_encrypt(self._h, dt, _ptr(x), N, exp_mode, fixed_exp, obf_mode,
                                    _ptr(r_buf) if r_buf is not None else None, r_stride, r_bytes,
                                    key, index_base, _ptr(ct), _ptr(ex), _ptr(st)))
        return ct, ex, st

    def add(self, cts: Sequence[np.ndarray], exps: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray]:
        k = len(cts)
        cts = [np.ascontiguousarray(c, dtype=np.uint32) for c in cts]
        exps = [np.ascontiguousarray(e, dtype=np.int32) for e in exps]
        N = exps[0].size
        for c, e in zip(cts, exps):
            self._check_words(c, e, N)
        self.calls["pai_add"] += 1
        ct_ptrs = (ctypes.c_void_p * k)(*[_ptr(c) for c in cts])
        ex_ptrs = (ctypes.c_void_p * k)(*[_ptr(e) for e in exps])
        out = np.empty((N, self.ct_words), dtype=np.uint32)
        oe = np.empty(N, dtype=np.int32)
        self._chk(self.lib.pai_add(self._h, ct_ptrs, ex_ptrs, k, N, _ptr(out), _ptr(oe)))
        return out, oe

    def mul(self, ct: np.ndarray, exp: np.ndarray, x: np.ndarray):
        """Element-wise ct_i (x) x_i (x of size 1: one scalar for every element); returns
        (ciphertext words, exponents, statuses). PaillierEncryptedNumber.__mul__ semantics."""
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        exp = np.ascontiguousarray(exp, dtype=np.int32)
        x = np.ascontiguousarray(x)
        N = exp.size
        self._check_words(ct, exp, N)
        if x.size not in (1, N):
            raise ValueError("scalar operand must have 1 or N elements")
        self.calls["pai_mul"] += 1
        out = np.empty((N, self.ct_words), dtype=np.uint32)
        oe = np.empty(N, dtype=np.int32)
        st = np.empty(N, dtype=np.int32)
        self._chk(self.lib.pai_mul(self._h, _ptr(ct), _ptr(exp), N, scalar_dtype(x), _ptr(x), 1 if x.size == N and N > 1 else 0,
                                _ptr(out), _ptr(oe), _ptr(st)))
        return out, oe, st

    def add_plain(self, ct: np.ndarray, exp: np.ndarray, x: np.ndarray):
        """Element-wise ct_i (+) x_i (x of size 1: one scalar for every element); returns (ciphertext
        words, exponents, statuses). PaillierEncryptedNumber.__add__(scalar) semantics."""
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        exp = np.ascontiguousarray(exp, dtype=np.int32)
        x = np.ascontiguousarray(x)
        N = exp.size
        self._check_words(ct, exp, N)
        if x.size not in (1, N):
            raise ValueError("plain operand must have 1 or N elements")
        self.calls["pai_add_plain"] += 1
        out = np.empty((N, self.ct_words), dtype=np.uint32)
        oe = np.empty(N, dtype=np.int32)
        st = np.empty(N, dtype=np.int32)
        self._chk(self.lib.pai_add_plain(self._h, _ptr(ct), _ptr(exp), N, scalar_dtype(x), _ptr(x),
                                      1 if x.size == N and N > 1 else 0, _ptr(out), _ptr(oe), _ptr(st)))
        return out, oe, st

    def segment_add(self, ct: np.ndarray, exp: np.ndarray, index: np.ndarray, seg_off: np.ndarray):
        """Per-segment k-way sums: segment s = ct[index[seg_off[s]:seg_off[s+1]]]. Returns (words [nseg, W],
        exponents [nseg]); an empty segment gives ciphertext 1 and exponent INT32_MIN."""
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        exp = np.ascontiguousarray(exp, dtype=np.int32)
        index = np.ascontiguousarray(index, dtype=np.int64)
        seg_off = np.ascontiguousarray(seg_off, dtype=np.int64)
        nseg = seg_off.size - 1
        self._check_words(ct, exp, exp.size)
        self.calls["pai_segment_add"] += 1
        out = np.empty((max(nseg, 0), self.ct_words), dtype=np.uint32)
        oe = np.empty(max(nseg, 0), dtype=np.int32)
        if nseg <= 0:
            return out, oe
        self._chk(self.lib.pai_segment_add(self._h, _ptr(ct), _ptr(exp), exp.size, _ptr(index), _ptr(seg_off), nseg,
                                        _ptr(out), _ptr(oe)))
        return out, oe

    def matmul(self, ct: np.ndarray, exp: np.ndarray, m: int, K: int, x: np.ndarray, d: int):
        """(m x K encrypted) @ (K x d plain) -> (m d ciphertext words, m d exponents), row-major."""
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        exp = np.ascontiguousarray(exp, dtype=np.int32)
        x = np.ascontiguousarray(x)
        if exp.size != m * K or x.size != K * d:
            raise ValueError("matmul: shape mismatch")
        self._check_words(ct, exp, m * K)
        self.calls["pai_matmul"] += 1
        out = np.empty((m * d, self.ct_words), dtype=np.uint32)
        oe = np.empty(m * d, dtype=np.int32)
        self._chk(self.lib.pai_matmul(self._h, _ptr(ct), _ptr(exp), m, K, scalar_dtype(x), _ptr(x), d, _ptr(out), _ptr(oe)))
        return out, oe

    def decrypt(self, ct: np.ndarray, exp: np.ndarray, want_raw: bool = False):
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        exp = np.ascontiguousarray(exp, dtype=np.int32)
        N = exp.size
        self._check_words(ct, exp, N)
        self.calls["pai_decrypt"] += 1
        val = np.empty(N, dtype=np.float64)
        mant = np.empty(N, dtype=np.int64)
        st = np.empty(N, dtype=np.int32)
        raw = np.empty((N, self.pt_words), dtype=np.uint32) if want_raw else None
        self._chk(self.lib.pai_decrypt(self._h, _ptr(ct), _ptr(exp), N, _ptr(val), _ptr(mant), _ptr(st),
                                    _ptr(raw) if raw is not None else None))
        return val, mant, st, raw


def scalar_dtype(x: np.ndarray) -> int:
    if x.dtype == np.float32:
        return PAI_F32
    if x.dtype == np.float64:
        return PAI_F64
    if x.dtype == np.int64:
        return PAI_I64
    raise TypeError(f"unsupported dtype {x.dtype}")


try:                                        # the package's C conversions (csrc/hostgmp.c), when built
    from .._gmp import ints_to_words as _c_ints_to_words, words_to_ints as _c_words_to_ints
except ImportError:                         # pragma: no cover - build() always builds it
    _c_ints_to_words = _c_words_to_ints = None


def words_to_ints(words: np.ndarray):
    """[N, W] little-endian uint32 words -> list of Python ints."""
    w = np.ascontiguousarray(words, dtype="<u4")
    if w.ndim != 2:
        w = w.reshape(len(w), -1)
    if _c_words_to_ints is not None and w.size:
        return _c_words_to_ints(w, w.shape[1])
    b = w.tobytes()
    step = w.shape[1] * 4
    return [int.from_bytes(b[i * step:(i + 1) * step], "little") for i in range(w.shape[0])]


def ints_to_words(vals, nwords: int) -> np.ndarray:
    vals = list(vals)
    if _c_ints_to_words is not None:
        buf = _c_ints_to_words(vals, nwords)
    else:
        nbytes = nwords * 4
        buf = b"".join(int(v).to_bytes(nbytes, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), nwords).copy()
