"""Process-local GPU runtime for the Paillier package: one native context per (key, device,
process). Contexts are created lazily, never pickled and never shared across a fork (a forked
child builds its own), so PaillierEncryptor/PaillierDecryptor stay picklable exactly like the
reference's (encryptor.py / decryptor.py are sent to peers, e.g. he_otp_lr_ft1/train.py:70).

Device selection: $FLEXPAI_DEVICE, else $LOCAL_RANK, else 0.

Private keys known to this process (a PaillierDecryptor was built, or the factory
generate_paillier_encryptor_decryptor made the pair) are registered here so that the context
of that key can encrypt through the CRT kernels (same ciphertext bits, ~4x fewer multiplies);
the registry is process-local and never pickled. $FLEXPAI_CRT=0 disables CRT encryption.

Contexts live in a bounded LRU ($FLEXPAI_MAX_CONTEXTS, default 4): a process that cycles through
keys (a new keypair per round, or several simulated parties) drops the least recently used context,
whose device memory (constants, fixed-base tables) is released when the last reference goes, and the
registered private key of that public key with it; the private-key registry is bounded by the same
limit. A PaillierDecryptor always passes its own key, so eviction only costs a later encryption under an
evicted key the CRT path (it then runs the public-key kernels, same ciphertext distribution).
"""
from __future__ import annotations

import collections
import os
import threading
from typing import Optional, Tuple

import numpy as np

from . import _native

_lock = threading.Lock()
_ctxs: "collections.OrderedDict[Tuple[int, int, int], _native.Context]" = collections.OrderedDict()
_private: "collections.OrderedDict[int, object]" = collections.OrderedDict()
_gpus: Optional[Tuple[int, int]] = None     # (pid, device count)


def max_contexts() -> int:
    try:
        return max(1, int(os.environ.get("FLEXPAI_MAX_CONTEXTS", "4")))
    except ValueError:
        return 4


def gpu_available() -> bool:
    """True when this process sees a GPU (raises when libflexpai.so is missing: no silent fallback).
    Without one, operators on existing ciphertext arrays use the reference's per-element computation
    (cipher_array.py); encryption and decryption raise."""
    global _gpus
    pid = os.getpid()
    if _gpus is None or _gpus[0] != pid:
        _gpus = (pid, _native.device_count())
    return _gpus[1] > 0


_evict_warned = False


def register_private(public_key, private_key) -> None:
    """Remember this process's private key for `public_key` (enables CRT encryption)."""
    global _evict_warned
    with _lock:
        _private[public_key.n] = private_key
        _private.move_to_end(public_key.n)
        while len(_private) > max_contexts():    # bounded like the contexts (HE_SA_FT re-keys per exchange)
            n_old, _ = _private.popitem(last=False)
            # a context of that key still cached keeps its private part (set_private is never undone), but a
            # context created for it later encrypts on the public-key kernels: say so once
            if not _evict_warned and not os.environ.get("FLEXPAI_QUIET"):
                import sys
                print(f"flexpai: more than FLEXPAI_MAX_CONTEXTS={max_contexts()} private keys registered; the least "
                      "recently registered one is dropped, and a later context for it encrypts through the slower "
                      "public-key kernels (results unchanged). Raise FLEXPAI_MAX_CONTEXTS to keep it.", file=sys.stderr)
                _evict_warned = True


def _evict_lru() -> None:
    """Drop the least recently used contexts beyond max_contexts(), and with each the private key of its
    public key unless another cached context (another device) still uses it. Caller holds _lock."""
    while len(_ctxs) > max_contexts():
        (n_old, _, _), _ = _ctxs.popitem(last=False)        # freed once no caller holds it any more
        if not any(k[0] == n_old for k in _ctxs):
            _private.pop(n_old, None)


def device_index() -> int:
    for var in ("FLEXPAI_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            return int(v)
    return 0


def context(public_key, private_key=None) -> "_native.Context":
    """The native context of `public_key` on this process's device (private part attached when
    `private_key` is given)."""
    dev = device_index()
    k = (public_key.n, dev, os.getpid())
    with _lock:
        if private_key is None:
            private_key = _private.get(public_key.n)
        ctx = _ctxs.get(k)
        if ctx is None:
            ctx = _native.Context(public_key.n, dev)
            _ctxs[k] = ctx
            _evict_lru()
        else:
            _ctxs.move_to_end(k)
        if public_key.n in _private:
            _private.move_to_end(public_key.n)
        if private_key is not None and not ctx.has_private:
            ctx.set_private(private_key.p, private_key.q)
    return ctx


def cached_contexts():
    """The contexts currently cached (most recently used last)."""
    with _lock:
        return list(_ctxs.values())


def ints_to_words(vals, nwords: int) -> np.ndarray:
    return _native.ints_to_words(vals, nwords)


def words_to_ints(words: np.ndarray):
    return _native.words_to_ints(words)
