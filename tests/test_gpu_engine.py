"""Unit tests of the lane-group big-number engine (bn_group.hpp) through pai_debug_engine (k_debug), which is in
the test build (libflexpai_xcheck.so) only; the product library refuses the call."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(ctx, op, a_vals, b_vals):
    from flex.crypto.paillier import _native as N
    lib = ctx.lib
    lib.pai_debug_engine.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    A = N.ints_to_words(a_vals, ctx.ct_words)
    B = N.ints_to_words(b_vals, ctx.ct_words)
    out = np.zeros_like(A)
    flag = np.zeros(len(a_vals), dtype=np.int32)
    rc = lib.pai_debug_engine(ctx.handle, op, A.ctypes.data, B.ctypes.data, len(a_vals), out.ctypes.data,
                              flag.ctypes.data)
    assert rc == 0, lib.pai_last_error()
    return N.words_to_ints(out), flag


@pytest.fixture(scope="module", params=[1024, 2048, 4096])
def setup(request, golden, xlib):
    from flex.crypto.paillier import _native as N
    k = golden["keys"][str(request.param)]
    n = int(k["n"], 16)
    ctx = N.Context(n, 0, lib=xlib)
    S = 37 * {1024: 2, 2048: 4, 4096: 8}[request.param]   # L = 37 limbs per lane (bn_group.hpp)
    return ctx, n, n * n, 28 * S


def test_roundtrip_words(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(1)
    a = [rnd.getrandbits(N2.bit_length()) % N2 for _ in range(37)]
    got, _ = _run(ctx, 1, a, a)
    assert got == a


def test_normalize_add(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(2)
    a = [rnd.getrandbits(N2.bit_length() - 1) for _ in range(37)]
    b = [rnd.getrandbits(N2.bit_length() - 1) for _ in range(37)]
    a[0] = (1 << (N2.bit_length() - 1)) - 1
    b[0] = 1
    got, _ = _run(ctx, 7, a, b)
    assert got == [x + y for x, y in zip(a, b)]


def test_sub_and_condsub(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(3)
    a = [rnd.getrandbits(N2.bit_length()) for _ in range(37)]
    b = [rnd.getrandbits(N2.bit_length()) for _ in range(37)]
    a[1] = b[1]
    got, flag = _run(ctx, 6, a, b)
    for i in range(37):
        assert flag[i] == (a[i] < b[i]), i
        if a[i] >= b[i]:
            assert got[i] == a[i] - b[i], i
    a2 = [rnd.randrange(2 * N2) for _ in range(37)] + [N2, N2 - 1, 0]
    got, _ = _run(ctx, 5, a2, a2)
    assert got == [x % N2 for x in a2]


def test_montmul(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(4)
    a = [rnd.randrange(2 * N2) for _ in range(37)]
    b = [rnd.randrange(2 * N2) for _ in range(37)]
    Rinv = pow(1 << Rb, -1, N2)
    got, _ = _run(ctx, 0, a, b)
    for i in range(37):
        assert got[i] % N2 == a[i] * b[i] * Rinv % N2, i
        assert got[i] < 2 * N2


def test_mont_roundtrip(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(5)
    a = [rnd.randrange(N2) for _ in range(37)]
    got, _ = _run(ctx, 3, a, a)
    assert [g % N2 for g in got] == a


def test_c0(setup):
    ctx, n, N2, Rb = setup
    Ms = [0, 1, -1, 5, -5, 2 ** 53 - 1, -(2 ** 53), 2 ** 62, -(2 ** 63)]
    a = [M & ((1 << 64) - 1) for M in Ms]
    got, _ = _run(ctx, 2, a, a)
    assert got == [(1 + n * (M % n)) % N2 for M in Ms]


def test_modexp_n(setup):
    ctx, n, N2, Rb = setup
    rnd = random.Random(6)
    a = [rnd.randrange(1, n) for _ in range(11)]
    got, _ = _run(ctx, 4, a, a)
    assert got == [pow(x, n, N2) for x in a]


def test_product_library_refuses_the_debug_hook(golden):
    from flex.crypto.paillier import _native as N
    ctx = N.Context(int(golden["keys"]["1024"]["n"], 16), 0)
    lib = N.load_library()
    lib.pai_debug_engine.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    A = N.ints_to_words([5], ctx.ct_words)
    out = np.zeros_like(A)
    flag = np.zeros(1, dtype=np.int32)
    assert lib.pai_debug_engine(ctx.handle, 1, A.ctypes.data, A.ctypes.data, 1, out.ctypes.data, flag.ctypes.data) != 0
    assert b"test build" in lib.pai_last_error()
