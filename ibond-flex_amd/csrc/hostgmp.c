/* _gmp: the package's own GMP binding for the per-element host operators (CPython extension).
 *
 * The reference reaches GMP through gmpy2 (flex/crypto/gmpy_math.py:27-74: mul, mulmod, powmod,
 * invert). Object-level operators on single PaillierEncryptedNumber values (encrypted_number.py:65-185)
 * -- numpy's per-element loop over an object ndarray received from an unmodified FLEX peer, or scalar
 * code -- run on the host; with this module they cost what gmpy2 costs instead of Python's builtin
 * pow (~9x slower at 2048 bits). Whole-array operations never come here: they go to the
 * GPU through libflexpai.so.
 *
 * Conversions repack CPython's 30-bit long digits straight into / out of 64-bit mpz limbs, as gmpy2
 * does (mpz_import with nails is a slow generic loop). Built by __graft_entry__.build() against GMP 6.2.1
 * (/opt/conda, the library gmpy2 2.0.8 wraps).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <longintrepr.h>
#include <gmp.h>
#include <stdint.h>
#include <string.h>

/* Work registers, allocated once and reused (every call holds the GIL, so they are never shared
 * concurrently); results go to a register distinct from the inputs, so GMP needs no temporaries. */
static mpz_t A, B, C, T;

static int to_mpz(PyObject* o, mpz_t z) {
  if (!PyLong_Check(o)) {
    PyErr_Format(PyExc_TypeError, "expected int, got %s", Py_TYPE(o)->tp_name);
    return -1;
  }
  PyLongObject* l = (PyLongObject*)o;
  const Py_ssize_t size = Py_SIZE(l), n = size < 0 ? -size : size;
  if (n == 0) {
    mpz_set_ui(z, 0);
    return 0;
  }
  /* pack the 30-bit digits into 64-bit limbs directly (mpz_import with nails is a slow generic loop) */
  const size_t nl = ((size_t)n * PyLong_SHIFT + GMP_NUMB_BITS - 1) / GMP_NUMB_BITS;
  mp_limb_t* w = mpz_limbs_write(z, (mp_size_t)nl);
  mp_limb_t acc = 0;
  int have = 0;
  size_t k = 0;
  for (Py_ssize_t i = 0; i < n; ++i) {
    const mp_limb_t d = l->ob_digit[i];
    acc |= d << have;
    have += PyLong_SHIFT;
    if (have >= GMP_NUMB_BITS) {
      w[k++] = acc;
      have -= GMP_NUMB_BITS;
      acc = have ? d >> (PyLong_SHIFT - have) : 0;
    }
  }
  if (have) w[k++] = acc;
  while (k > 0 && w[k - 1] == 0) --k;
  mpz_limbs_finish(z, size < 0 ? -(mp_size_t)k : (mp_size_t)k);
  return 0;
}

static PyObject* from_mpz(const mpz_t z) {
  const int sgn = mpz_sgn(z);
  if (sgn == 0) return PyLong_FromLong(0);
  const size_t nl = mpz_size(z);
  const mp_limb_t* w = mpz_limbs_read(z);
  const size_t bits = mpz_sizeinbase(z, 2);
  const size_t n = (bits + PyLong_SHIFT - 1) / PyLong_SHIFT;
  PyLongObject* l = _PyLong_New((Py_ssize_t)n);
  if (!l) return NULL;
  const digit mask = ((digit)1 << PyLong_SHIFT) - 1;
  size_t k = 0;
  int have = 0;          /* unread bits left in w[k] past position `pos` */
  int pos = 0;
  for (size_t i = 0; i < n; ++i) {
    mp_limb_t v = k < nl ? w[k] >> pos : 0;
    have = GMP_NUMB_BITS - pos;
    if (have < PyLong_SHIFT && k + 1 < nl) v |= w[k + 1] << have;
    l->ob_digit[i] = (digit)(v & mask);
    pos += PyLong_SHIFT;
    if (pos >= GMP_NUMB_BITS) {
      pos -= GMP_NUMB_BITS;
      ++k;
    }
  }
  Py_SET_SIZE(l, sgn < 0 ? -(Py_ssize_t)n : (Py_ssize_t)n);
  return (PyObject*)l;
}

/* mulmod(a, b, c) = (a * b) % c, Python floor semantics (gmpy_math.py:43-48) */
static PyObject* g_mulmod(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "mulmod(a, b, c)");
    return NULL;
  }
  if (to_mpz(args[0], A) || to_mpz(args[1], B) || to_mpz(args[2], C)) return NULL;
  if (mpz_sgn(C) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "mulmod by zero");
    return NULL;
  }
  mpz_mul(T, A, B);
  mpz_fdiv_r(A, T, C);
  return from_mpz(A);
}

/* powmod(a, b, c) (gmpy_math.py:51-63): 1 for a == 1; b < 0 means powers of the inverse */
static PyObject* g_powmod(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "powmod(a, b, c)");
    return NULL;
  }
  if (to_mpz(args[0], A) || to_mpz(args[1], B) || to_mpz(args[2], C)) return NULL;
  if (mpz_cmp_ui(A, 1) == 0) return PyLong_FromLong(1);
  if (mpz_sgn(C) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "powmod by zero");
    return NULL;
  }
  if (mpz_sgn(B) < 0) {
    if (!mpz_invert(T, A, C)) {
      PyErr_SetString(PyExc_ZeroDivisionError, "powmod: base not invertible");
      return NULL;
    }
    mpz_swap(T, A);
    mpz_neg(B, B);
  }
  mpz_powm(T, A, B, C);
  return from_mpz(T);
}

/* invert(a, b) (gmpy_math.py:66-74): ZeroDivisionError when no inverse exists */
static PyObject* g_invert(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "invert(a, b)");
    return NULL;
  }
  if (to_mpz(args[0], A) || to_mpz(args[1], B)) return NULL;
  if (mpz_sgn(B) == 0 || !mpz_invert(T, A, B) || mpz_sgn(T) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "invert(a, b) no inverse exists");
    return NULL;
  }
  return from_mpz(T);
}

/* mul(a, b) (gmpy_math.py:27-28) */
static PyObject* g_mul(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "mul(a, b)");
    return NULL;
  }
  if (to_mpz(args[0], A) || to_mpz(args[1], B)) return NULL;
  mpz_mul(T, A, B);
  return from_mpz(T);
}

/* PyLong from nl little-endian 64-bit limbs (non-negative), repacking into 30-bit digits directly */
static PyObject* long_from_limbs(const uint64_t* w, size_t nl) {
  while (nl > 0 && w[nl - 1] == 0) --nl;
  if (nl == 0) return PyLong_FromLong(0);
  const int top = 64 - __builtin_clzll(w[nl - 1]);
  const size_t bits = (nl - 1) * 64 + (size_t)top;
  const size_t n = (bits + PyLong_SHIFT - 1) / PyLong_SHIFT;
  PyLongObject* l = _PyLong_New((Py_ssize_t)n);
  if (!l) return NULL;
  const digit mask = ((digit)1 << PyLong_SHIFT) - 1;
  size_t k = 0;
  int pos = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t v = k < nl ? w[k] >> pos : 0;
    const int have = 64 - pos;
    if (have < PyLong_SHIFT && k + 1 < nl) v |= w[k + 1] << have;
    l->ob_digit[i] = (digit)(v & mask);
    pos += PyLong_SHIFT;
    if (pos >= 64) {
      pos -= 64;
      ++k;
    }
  }
  return (PyObject*)l;
}

/* words_to_ints(buf, nwords): rows of `nwords` little-endian 32-bit words -> list of non-negative ints
 * (the device ciphertext layout; one C loop instead of a Python slice + int.from_bytes per row) */
static PyObject* g_words_to_ints(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "words_to_ints(buf, nwords)");
    return NULL;
  }
  const Py_ssize_t nw = PyLong_AsSsize_t(args[1]);
  if (nw <= 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "nwords must be positive");
    return NULL;
  }
  Py_buffer view;
  if (PyObject_GetBuffer(args[0], &view, PyBUF_C_CONTIGUOUS) < 0) return NULL;
  const Py_ssize_t row = 4 * nw;
  if (view.len % row != 0) {
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "buffer length is not a multiple of the row size");
    return NULL;
  }
  const Py_ssize_t n = view.len / row;
  PyObject* out = PyList_New(n);
  if (!out) {
    PyBuffer_Release(&view);
    return NULL;
  }
  const unsigned char* b = (const unsigned char*)view.buf;
  const size_t nl = (size_t)(nw + 1) / 2;
  uint64_t stackbuf[256];
  uint64_t* limbs = nl <= 256 ? stackbuf : (uint64_t*)PyMem_Malloc(nl * sizeof(uint64_t));
  if (!limbs) {
    Py_DECREF(out);
    PyBuffer_Release(&view);
    return PyErr_NoMemory();
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    limbs[nl - 1] = 0;
    memcpy(limbs, b + i * row, (size_t)row);          /* little-endian host: words pair into limbs */
    PyObject* v = long_from_limbs(limbs, nl);
    if (!v) {
      if (limbs != stackbuf) PyMem_Free(limbs);
      Py_DECREF(out);
      PyBuffer_Release(&view);
      return NULL;
    }
    PyList_SET_ITEM(out, i, v);
  }
  if (limbs != stackbuf) PyMem_Free(limbs);
  PyBuffer_Release(&view);
  return out;
}

/* ints_to_words(seq, nwords) -> bytes of len(seq) rows of `nwords` little-endian 32-bit words
 * (OverflowError when a value does not fit, ValueError for negatives) */
static PyObject* g_ints_to_words(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "ints_to_words(seq, nwords)");
    return NULL;
  }
  const Py_ssize_t nw = PyLong_AsSsize_t(args[1]);
  if (nw <= 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "nwords must be positive");
    return NULL;
  }
  PyObject* seq = PySequence_Fast(args[0], "ints_to_words: expected a sequence");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  const Py_ssize_t row = 4 * nw;
  PyObject* out = PyBytes_FromStringAndSize(NULL, n * row);
  if (!out) {
    Py_DECREF(seq);
    return NULL;
  }
  unsigned char* b = (unsigned char*)PyBytes_AS_STRING(out);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* v = items[i];
    if (!PyLong_Check(v)) {
      v = PyNumber_Index(v);
      if (!v) goto fail;
    } else {
      Py_INCREF(v);
    }
    const int rc = _PyLong_AsByteArray((PyLongObject*)v, b + i * row, (size_t)row, 1, 0);
    Py_DECREF(v);
    if (rc < 0) goto fail;
  }
  Py_DECREF(seq);
  return out;
fail:
  Py_DECREF(seq);
  Py_DECREF(out);
  return NULL;
}

static PyMethodDef methods[] = {
    {"words_to_ints", (PyCFunction)(void (*)(void))g_words_to_ints, METH_FASTCALL, "rows of LE 32-bit words -> ints"},
    {"ints_to_words", (PyCFunction)(void (*)(void))g_ints_to_words, METH_FASTCALL, "ints -> rows of LE 32-bit words"},
    {"mulmod", (PyCFunction)(void (*)(void))g_mulmod, METH_FASTCALL, "(a * b) % c"},
    {"powmod", (PyCFunction)(void (*)(void))g_powmod, METH_FASTCALL, "a ** b % c (GMP mpz_powm)"},
    {"invert", (PyCFunction)(void (*)(void))g_invert, METH_FASTCALL, "a^-1 mod b"},
    {"mul", (PyCFunction)(void (*)(void))g_mul, METH_FASTCALL, "a * b"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_gmp", "GMP binding for the host operators", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__gmp(void) {
  mpz_init2(A, 8192);
  mpz_init2(B, 8192);
  mpz_init2(C, 8192);
  mpz_init2(T, 16384);
  PyObject* m = PyModule_Create(&moddef);
  if (m) PyModule_AddStringConstant(m, "gmp_version", gmp_version);
  return m;
}
