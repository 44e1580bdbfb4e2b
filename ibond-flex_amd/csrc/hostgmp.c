/* _gmp: the package's own GMP binding for the per-element host operators (CPython extension).
 *
 * The reference reaches GMP through gmpy2 (flex/crypto/gmpy_math.py:27-74: mul, mulmod, powmod,
 * invert). Object-level operators on single PaillierEncryptedNumber values (encrypted_number.py:65-185)
 * -- numpy's per-element loop over an object ndarray received from an unmodified FLEX peer, or scalar
 * code -- run on the host; with this module they cost what gmpy2 costs instead of Python's builtin
 * pow (~9x slower at 2048 bits). Whole-array operations never come here: they go to the
 * GPU through libflexpai.so.
 *
 * Conversions copy CPython's 30-bit long digits straight into / out of mpz limbs (mpz_import /
 * mpz_export with 2 nail bits), as gmpy2 does. Built by __graft_entry__.build() against GMP 6.2.1
 * (/opt/conda, the library gmpy2 2.0.8 wraps).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <longintrepr.h>
#include <gmp.h>

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
  mpz_import(z, (size_t)n, -1, sizeof(digit), 0, sizeof(digit) * 8 - PyLong_SHIFT, l->ob_digit);
  if (size < 0) mpz_neg(z, z);
  return 0;
}

static PyObject* from_mpz(const mpz_t z) {
  const int sgn = mpz_sgn(z);
  if (sgn == 0) return PyLong_FromLong(0);
  const size_t bits = mpz_sizeinbase(z, 2);
  const size_t n = (bits + PyLong_SHIFT - 1) / PyLong_SHIFT;
  PyLongObject* l = _PyLong_New((Py_ssize_t)n);
  if (!l) return NULL;
  size_t count = 0;
  mpz_export(l->ob_digit, &count, -1, sizeof(digit), 0, sizeof(digit) * 8 - PyLong_SHIFT, z);
  for (size_t i = count; i < n; ++i) l->ob_digit[i] = 0;
  Py_SET_SIZE(l, sgn < 0 ? -(Py_ssize_t)count : (Py_ssize_t)count);
  return (PyObject*)l;
}

/* mulmod(a, b, c) = (a * b) % c, Python floor semantics (gmpy_math.py:43-48) */
static PyObject* g_mulmod(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "mulmod(a, b, c)");
    return NULL;
  }
  mpz_t a, b, c;
  mpz_inits(a, b, c, NULL);
  PyObject* r = NULL;
  if (to_mpz(args[0], a) || to_mpz(args[1], b) || to_mpz(args[2], c)) goto done;
  if (mpz_sgn(c) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "mulmod by zero");
    goto done;
  }
  mpz_mul(a, a, b);
  mpz_fdiv_r(a, a, c);
  r = from_mpz(a);
done:
  mpz_clears(a, b, c, NULL);
  return r;
}

/* powmod(a, b, c) (gmpy_math.py:51-63): 1 for a == 1; b < 0 means powers of the inverse */
static PyObject* g_powmod(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "powmod(a, b, c)");
    return NULL;
  }
  mpz_t a, b, c;
  mpz_inits(a, b, c, NULL);
  PyObject* r = NULL;
  if (to_mpz(args[0], a) || to_mpz(args[1], b) || to_mpz(args[2], c)) goto done;
  if (mpz_cmp_ui(a, 1) == 0) {
    r = PyLong_FromLong(1);
    goto done;
  }
  if (mpz_sgn(c) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "powmod by zero");
    goto done;
  }
  if (mpz_sgn(b) < 0) {
    if (!mpz_invert(a, a, c)) {
      PyErr_SetString(PyExc_ZeroDivisionError, "powmod: base not invertible");
      goto done;
    }
    mpz_neg(b, b);
  }
  mpz_powm(a, a, b, c);
  r = from_mpz(a);
done:
  mpz_clears(a, b, c, NULL);
  return r;
}

/* invert(a, b) (gmpy_math.py:66-74): ZeroDivisionError when no inverse exists */
static PyObject* g_invert(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "invert(a, b)");
    return NULL;
  }
  mpz_t a, b;
  mpz_inits(a, b, NULL);
  PyObject* r = NULL;
  if (to_mpz(args[0], a) || to_mpz(args[1], b)) goto done;
  if (mpz_sgn(b) == 0 || !mpz_invert(a, a, b) || mpz_sgn(a) == 0) {
    PyErr_SetString(PyExc_ZeroDivisionError, "invert(a, b) no inverse exists");
    goto done;
  }
  r = from_mpz(a);
done:
  mpz_clears(a, b, NULL);
  return r;
}

/* mul(a, b) (gmpy_math.py:27-28) */
static PyObject* g_mul(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "mul(a, b)");
    return NULL;
  }
  mpz_t a, b;
  mpz_inits(a, b, NULL);
  PyObject* r = NULL;
  if (to_mpz(args[0], a) || to_mpz(args[1], b)) goto done;
  mpz_mul(a, a, b);
  r = from_mpz(a);
done:
  mpz_clears(a, b, NULL);
  return r;
}

static PyMethodDef methods[] = {
    {"mulmod", (PyCFunction)(void (*)(void))g_mulmod, METH_FASTCALL, "(a * b) % c"},
    {"powmod", (PyCFunction)(void (*)(void))g_powmod, METH_FASTCALL, "a ** b % c (GMP mpz_powm)"},
    {"invert", (PyCFunction)(void (*)(void))g_invert, METH_FASTCALL, "a^-1 mod b"},
    {"mul", (PyCFunction)(void (*)(void))g_mul, METH_FASTCALL, "a * b"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_gmp", "GMP binding for the host operators", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__gmp(void) {
  PyObject* m = PyModule_Create(&moddef);
  if (m) PyModule_AddStringConstant(m, "gmp_version", gmp_version);
  return m;
}
