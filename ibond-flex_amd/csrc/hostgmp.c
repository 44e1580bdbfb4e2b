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
#if PY_VERSION_HEX >= 0x030C0000
/* 3.12 moved the sign of a PyLong into lv_tag: the digit-level conversions below read ob_digit with the
 * sign in Py_SIZE (the layout of 3.6 - 3.11). Refuse to build rather than build wrong ints. */
#error "hostgmp.c reads the PyLong digit layout of CPython <= 3.11"
#elif PY_VERSION_HEX >= 0x030B0000
#include <cpython/longintrepr.h>
#else
#include <longintrepr.h>
#endif
#include <structmember.h>
#include <pthread.h>
#include <unistd.h>

#define W2I_THREADS_MAX 16                                 /* the GPU box grants 16 cores per GPU */
#define W2I_ROWS_MIN 8192                                  /* rows per thread below which one thread does it */
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

/* scalar_pow(c, k, m, neg): c^k mod m (neg: (c^k)^-1 mod m == (c^-1)^k, the reference's inverse trick,
 * encrypted_number.py:99-106) for 0 <= k < 2^SQ_BITS -- the multiplication of a ciphertext by an encoded scalar
 * (encrypted_number.py:86-113) and the exponent alignment (:115-127). A ciphertext multiplied by several scalars
 * (HE_OTP_LR's enc.dot(features), he_otp_lr_ft1/train.py:160: every element times six feature columns) keeps the
 * table of its squarings c^(2^j): from its second multiplication on, c^k costs popcount(k) products instead of an
 * mpz_powm (~bits(k) squarings). A ciphertext seen once takes mpz_powm: a table would not pay for one use. Keys are
 * the int objects themselves (a strong reference is held while cached, so an address is never reused by another
 * int); the modulus is compared by value. Same values as mpz_powm / mpz_invert. */
#define SQ_BITS 64
#define SQ_CACHE 64
#define SQ_SEEN 256
typedef struct {
  PyObject* key;
  mpz_t mod;
  int nsq;                 /* squarings held: sq[0 .. nsq) = c^(2^j) mod m */
  mpz_t sq[SQ_BITS];
  unsigned long long used;
} SqEntry;
static SqEntry sqc[SQ_CACHE];
static const PyObject* sq_seen[SQ_SEEN];
static int sq_seen_at = 0;
static unsigned long long sq_clock = 0;

static SqEntry* sq_find(PyObject* key, const mpz_t m) {
  for (int i = 0; i < SQ_CACHE; ++i)
    if (sqc[i].key == key && mpz_cmp(sqc[i].mod, m) == 0) return &sqc[i];
  return NULL;
}
static SqEntry* sq_insert(PyObject* key, const mpz_t c, const mpz_t m) {
  int v = 0;
  for (int i = 1; i < SQ_CACHE; ++i)
    if (sqc[i].used < sqc[v].used) v = i;
  SqEntry* e = &sqc[v];
  if (!e->key) {
    mpz_init(e->mod);
    for (int j = 0; j < SQ_BITS; ++j) mpz_init(e->sq[j]);
  }
  Py_XDECREF(e->key);
  Py_INCREF(key);
  e->key = key;
  mpz_set(e->mod, m);
  mpz_mod(e->sq[0], c, m);
  e->nsq = 1;
  return e;
}
static int sq_seen_before(const PyObject* key) {
  for (int i = 0; i < SQ_SEEN; ++i)
    if (sq_seen[i] == key) return 1;
  sq_seen[sq_seen_at] = key;
  sq_seen_at = (sq_seen_at + 1) % SQ_SEEN;
  return 0;
}

static PyObject* g_scalar_pow(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "scalar_pow(c, k, m, neg)");
    return NULL;
  }
  const int neg = PyObject_IsTrue(args[3]);
  if (neg < 0) return NULL;
  if (to_mpz(args[1], B) || to_mpz(args[2], C)) return NULL;
  if (mpz_sgn(C) <= 0 || mpz_sgn(B) < 0 || mpz_sizeinbase(B, 2) > SQ_BITS) {
    PyErr_SetString(PyExc_ValueError, "scalar_pow: 0 <= k < 2^64 and m > 0");
    return NULL;
  }
  SqEntry* e = sq_find(args[0], C);
  if (!e && !sq_seen_before(args[0])) {
    if (to_mpz(args[0], A)) return NULL;
    mpz_powm(T, A, B, C);
  } else {
    if (!e) {
      if (to_mpz(args[0], A)) return NULL;
      e = sq_insert(args[0], A, C);
    }
    e->used = ++sq_clock;
    const int bits = mpz_sgn(B) ? (int)mpz_sizeinbase(B, 2) : 0;
    for (; e->nsq < bits; ++e->nsq) {
      mpz_mul(T, e->sq[e->nsq - 1], e->sq[e->nsq - 1]);
      mpz_mod(e->sq[e->nsq], T, C);
    }
    int first = 1;
    for (int j = 0; j < bits; ++j) {
      if (!mpz_tstbit(B, j)) continue;
      if (first) {
        mpz_set(A, e->sq[j]);
        first = 0;
      } else {
        mpz_mul(T, A, e->sq[j]);
        mpz_mod(A, T, C);
      }
    }
    if (first) mpz_set_ui(A, 1);
    mpz_mod(T, A, C);   /* 1 mod 1 == 0, as mpz_powm */
  }
  if (neg) {
    if (!mpz_invert(A, T, C)) {
      PyErr_SetString(PyExc_ZeroDivisionError, "invert(a, b) no inverse exists");
      return NULL;
    }
    return from_mpz(A);
  }
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

/* repack nl limbs into the n 30-bit digits of an allocated PyLong (no Python API: thread-safe) */
static void fill_digits(digit* d, size_t n, const uint64_t* w, size_t nl) {
  const digit mask = ((digit)1 << PyLong_SHIFT) - 1;
  size_t k = 0;
  int pos = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t v = k < nl ? w[k] >> pos : 0;
    const int have = 64 - pos;
    if (have < PyLong_SHIFT && k + 1 < nl) v |= w[k + 1] << have;
    d[i] = (digit)(v & mask);
    pos += PyLong_SHIFT;
    if (pos >= 64) {
      pos -= 64;
      ++k;
    }
  }
}

/* words_to_ints fill phase: rows [lo, hi) of the word buffer into the PyLongs allocated for them */
typedef struct {
  const unsigned char* b;
  Py_ssize_t row, lo, hi;
  size_t nl;
  PyObject** items;
} w2i_job;

static void* w2i_fill(void* arg) {
  const w2i_job* j = (const w2i_job*)arg;
  uint64_t limbs[256];
  for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
    PyLongObject* l = (PyLongObject*)j->items[i];
    const Py_ssize_t n = Py_SIZE(l);
    if (n == 0) continue;                                 /* the shared small int 0 */
    limbs[j->nl - 1] = 0;
    memcpy(limbs, j->b + i * j->row, (size_t)j->row);
    fill_digits(l->ob_digit, (size_t)n, limbs, j->nl);
  }
  return NULL;
}

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
  if (nl > 256) {
    Py_DECREF(out);
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "words_to_ints: at most 512 words per row");
    return NULL;
  }
  /* phase 1 (GIL): size and allocate every PyLong -- allocation needs the interpreter; phase 2 (no GIL,
   * threads): repack the rows into the digits, the part that scales with the key size */
  uint64_t top[2];
  for (Py_ssize_t i = 0; i < n; ++i) {
    const unsigned char* r = b + i * row;
    size_t k = nl;
    size_t nd;
    for (;;) {                                           /* highest non-zero limb decides the digit count */
      if (k == 0) {
        nd = 0;
        break;
      }
      top[0] = 0;
      top[1] = 0;
      const size_t off = (k - 1) * 8;
      memcpy(top, r + off, (size_t)row - off < 8 ? (size_t)row - off : 8);
      if (top[0]) {
        const int tb = 64 - __builtin_clzll(top[0]);
        nd = ((k - 1) * 64 + (size_t)tb + PyLong_SHIFT - 1) / PyLong_SHIFT;
        break;
      }
      --k;
    }
    PyObject* v = nd ? (PyObject*)_PyLong_New((Py_ssize_t)nd) : PyLong_FromLong(0);
    if (!v) {
      Py_DECREF(out);                                    /* digits of the allocated longs are never read */
      PyBuffer_Release(&view);
      return NULL;
    }
    PyList_SET_ITEM(out, i, v);
  }
  PyObject** items = ((PyListObject*)out)->ob_item;
  long nt = sysconf(_SC_NPROCESSORS_ONLN);
  if (nt > W2I_THREADS_MAX) nt = W2I_THREADS_MAX;
  if (nt > n / W2I_ROWS_MIN) nt = (long)(n / W2I_ROWS_MIN);
  if (nt < 1) nt = 1;
  w2i_job jobs[W2I_THREADS_MAX];
  pthread_t th[W2I_THREADS_MAX];
  int started[W2I_THREADS_MAX] = {0};
  const Py_ssize_t per = (n + nt - 1) / nt;
  for (long t = 0; t < nt; ++t) {
    jobs[t].b = b;
    jobs[t].row = row;
    jobs[t].lo = t * per < n ? t * per : n;
    jobs[t].hi = (t + 1) * per < n ? (t + 1) * per : n;
    jobs[t].nl = nl;
    jobs[t].items = items;
  }
  Py_BEGIN_ALLOW_THREADS
  for (long t = 1; t < nt; ++t) started[t] = pthread_create(&th[t], NULL, w2i_fill, &jobs[t]) == 0;
  w2i_fill(&jobs[0]);
  for (long t = 1; t < nt; ++t) {
    if (started[t]) pthread_join(th[t], NULL);
    else w2i_fill(&jobs[t]);                             /* no thread: do its rows here */
  }
  Py_END_ALLOW_THREADS
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

/* make_numbers(cls, public_key, ints, exps, obf) -> list of cls instances with the slots public_key,
 * exponent, _<cls>__ciphertext, _<cls>__is_obfuscator set directly (PaillierEncryptedNumber._make without a
 * Python call per element). exps: int32 buffer of len(ints); obf: uint8 buffer of len(ints), or a bool for
 * every element. */
static Py_ssize_t slot_offset(PyObject* cls, const char* name) {
  PyObject* d = PyObject_GetAttrString(cls, name);
  if (!d) return -1;
  Py_ssize_t off = -1;
  if (Py_TYPE(d) == &PyMemberDescr_Type) off = ((PyMemberDescrObject*)d)->d_member->offset;
  else PyErr_Format(PyExc_TypeError, "%s is not a slot", name);
  Py_DECREF(d);
  return off;
}

static PyObject* g_make_numbers(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 5 || !PyType_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "make_numbers(cls, public_key, ints, exps, obf)");
    return NULL;
  }
  PyTypeObject* cls = (PyTypeObject*)args[0];
  const char* cname = cls->tp_name;
  const char* dot = strrchr(cname, '.');
  if (dot) cname = dot + 1;
  char nct[256], nob[256];
  snprintf(nct, sizeof nct, "_%s__ciphertext", cname);
  snprintf(nob, sizeof nob, "_%s__is_obfuscator", cname);
  Py_ssize_t o_pk, o_ex, o_ct, o_ob;
  if ((o_pk = slot_offset(args[0], "public_key")) < 0 || (o_ex = slot_offset(args[0], "exponent")) < 0 ||
      (o_ct = slot_offset(args[0], nct)) < 0 || (o_ob = slot_offset(args[0], nob)) < 0)
    return NULL;
  PyObject* ints = PySequence_Fast(args[2], "make_numbers: ints must be a sequence");
  if (!ints) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(ints);
  Py_buffer ev, ov;
  if (PyObject_GetBuffer(args[3], &ev, PyBUF_C_CONTIGUOUS) < 0) {
    Py_DECREF(ints);
    return NULL;
  }
  const int obf_all = PyBool_Check(args[4]);
  if (!obf_all && PyObject_GetBuffer(args[4], &ov, PyBUF_C_CONTIGUOUS) < 0) {
    PyBuffer_Release(&ev);
    Py_DECREF(ints);
    return NULL;
  }
  PyObject* out = NULL;
  if (ev.len != n * 4 || (!obf_all && ov.len != n)) {
    PyErr_SetString(PyExc_ValueError, "make_numbers: exps / obf do not match the number of ciphertexts");
    goto done;
  }
  out = PyList_New(n);
  if (!out) goto done;
  const int32_t* e = (const int32_t*)ev.buf;
  const uint8_t* ob = obf_all ? NULL : (const uint8_t*)ov.buf;
  PyObject** it = PySequence_Fast_ITEMS(ints);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* obj = cls->tp_alloc(cls, 0);
    PyObject* ex = PyLong_FromLong(e[i]);
    if (!obj || !ex) {
      Py_XDECREF(obj);
      Py_XDECREF(ex);
      Py_CLEAR(out);
      goto done;
    }
    PyObject* flag = (obf_all ? PyObject_IsTrue(args[4]) : ob[i] != 0) ? Py_True : Py_False;
    Py_INCREF(args[1]);
    Py_INCREF(it[i]);
    Py_INCREF(flag);
    *(PyObject**)((char*)obj + o_pk) = args[1];
    *(PyObject**)((char*)obj + o_ex) = ex;
    *(PyObject**)((char*)obj + o_ct) = it[i];
    *(PyObject**)((char*)obj + o_ob) = flag;
    /* the slots hold two ints, a bool and the public key: no cycle can pass through the number, so it
     * stays out of the collector (which otherwise rescans every survivor as the list grows). Objects built
     * here are therefore NOT tracked by the cyclic GC: a caller that later stores a container in one of
     * their slots (nothing in the package or the reference does) would have to re-track it. */
    if (PyObject_IS_GC(obj)) PyObject_GC_UnTrack(obj);
    PyList_SET_ITEM(out, i, obj);
  }
done:
  PyBuffer_Release(&ev);
  if (!obf_all) PyBuffer_Release(&ov);
  Py_DECREF(ints);
  return out;
}

/* packed_valid(cls, objs, ints, exps) -> bool: every objs[i] is a `cls` whose ciphertext slot IS ints[i]
 * (object identity) and whose exponent equals exps[i] (int64 buffer) -- the check that a PaillierArray's
 * cached device words still describe its elements (cipher_array.PaillierArray._valid_packed). Elements can
 * change in place (apply_obfuscation replaces the ciphertext, callers may assign .exponent), so the check
 * is per element, done here at a few ns per element instead of two Python attribute reads. */
static PyObject* g_packed_valid(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 4 || !PyType_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "packed_valid(cls, objs, ints, exps)");
    return NULL;
  }
  PyTypeObject* cls = (PyTypeObject*)args[0];
  const char* cname = cls->tp_name;
  const char* dot = strrchr(cname, '.');
  if (dot) cname = dot + 1;
  char nct[256];
  snprintf(nct, sizeof nct, "_%s__ciphertext", cname);
  Py_ssize_t o_ex, o_ct;
  if ((o_ex = slot_offset(args[0], "exponent")) < 0 || (o_ct = slot_offset(args[0], nct)) < 0) return NULL;
  PyObject* objs = PySequence_Fast(args[1], "packed_valid: objs must be a sequence");
  if (!objs) return NULL;
  PyObject* ints = PySequence_Fast(args[2], "packed_valid: ints must be a sequence");
  if (!ints) {
    Py_DECREF(objs);
    return NULL;
  }
  Py_buffer ev;
  if (PyObject_GetBuffer(args[3], &ev, PyBUF_C_CONTIGUOUS) < 0) {
    Py_DECREF(objs);
    Py_DECREF(ints);
    return NULL;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(objs);
  int ok = n == PySequence_Fast_GET_SIZE(ints) && ev.len == n * 8;
  PyObject** it = PySequence_Fast_ITEMS(objs);
  PyObject** iv = PySequence_Fast_ITEMS(ints);
  const int64_t* e = (const int64_t*)ev.buf;
  for (Py_ssize_t i = 0; ok && i < n; ++i) {
    PyObject* o = it[i];
    if (Py_TYPE(o) != cls) {
      ok = 0;
      break;
    }
    PyObject* ct = *(PyObject**)((char*)o + o_ct);
    PyObject* ex = *(PyObject**)((char*)o + o_ex);
    if (ct != iv[i] || !ex || !PyLong_CheckExact(ex)) {
      ok = 0;
      break;
    }
    int over = 0;
    const long long v = PyLong_AsLongLongAndOverflow(ex, &over);
    if (over || v != e[i]) ok = 0;
  }
  PyBuffer_Release(&ev);
  Py_DECREF(objs);
  Py_DECREF(ints);
  if (PyErr_Occurred()) return NULL;
  return PyBool_FromLong(ok);
}

/* pack_numbers(cls, objs, public_key, nwords, want_words) -> (words, exps, ints) or None
 *
 * The received-array half of PaillierDecryptor.decrypt and of the array operators (decryptor.py:53-55 and
 * cipher_array.pack): for an object array of PaillierEncryptedNumber in one pass
 *   - the reference's per-element _check (decryptor.py:73-79): every element is a `cls` (subclasses too) and its
 *     public_key IS `public_key` or compares equal to it (PaillierPublicKey.__eq__; the last equal object is
 *     remembered, and an unpickled array shares one key object, so this is an identity test per element);
 *   - the exponents (int32 bytes) and the ciphertext slots (a list of the ints, for the packed cache);
 *   - with want_words, the ciphertexts as rows of `nwords` little-endian 32-bit words (bytes): the GIL pass
 *     only collects the int objects; the digit repacking runs on up to 16 threads without the GIL.
 * Returns None when any element fails a check or a value does not fit (negative, too wide, exponent beyond
 * int32): the caller then runs the reference's per-element path, which raises the reference's exception. */
typedef struct {
  PyObject** ints;
  unsigned char* out;
  Py_ssize_t lo, hi, nw;
  int bad;
} i2w_job;

static void* i2w_fill(void* arg) {
  i2w_job* j = (i2w_job*)arg;
  for (Py_ssize_t i = j->lo; i < j->hi; ++i) {
    const PyLongObject* l = (const PyLongObject*)j->ints[i];
    const Py_ssize_t nd = Py_SIZE(l);
    uint32_t* w = (uint32_t*)(j->out + (size_t)i * 4 * j->nw);
    memset(w, 0, (size_t)4 * j->nw);
    if (nd < 0) {
      j->bad = 1;
      continue;
    }
    uint64_t acc = 0;
    int have = 0;
    Py_ssize_t k = 0;
    for (Py_ssize_t d = 0; d < nd; ++d) {
      acc |= (uint64_t)l->ob_digit[d] << have;
      have += PyLong_SHIFT;
      while (have >= 32) {
        if (k >= j->nw) {
          if ((uint32_t)acc) j->bad = 1;
        } else {
          w[k] = (uint32_t)acc;
        }
        ++k;
        acc >>= 32;
        have -= 32;
      }
    }
    if (have > 0 && acc) {
      if (k >= j->nw) j->bad = 1;
      else w[k] = (uint32_t)acc;
    }
  }
  return NULL;
}

static PyObject* g_pack_numbers(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  if (nargs != 5 || !PyType_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "pack_numbers(cls, objs, public_key, nwords, want_words)");
    return NULL;
  }
  PyTypeObject* cls = (PyTypeObject*)args[0];
  const char* cname = cls->tp_name;
  const char* dot = strrchr(cname, '.');
  if (dot) cname = dot + 1;
  char nct[256];
  snprintf(nct, sizeof nct, "_%s__ciphertext", cname);
  Py_ssize_t o_pk, o_ex, o_ct;
  if ((o_pk = slot_offset(args[0], "public_key")) < 0 || (o_ex = slot_offset(args[0], "exponent")) < 0 ||
      (o_ct = slot_offset(args[0], nct)) < 0)
    return NULL;
  const Py_ssize_t nw = PyLong_AsSsize_t(args[3]);
  if (nw <= 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "nwords must be positive");
    return NULL;
  }
  const int want = PyObject_IsTrue(args[4]);
  if (want < 0) return NULL;
  PyObject* objs = PySequence_Fast(args[1], "pack_numbers: objs must be a sequence");
  if (!objs) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(objs);
  PyObject** it = PySequence_Fast_ITEMS(objs);
  PyObject* key = args[2];
  PyObject* same_key = key;            /* the last key object found equal to `key` */
  PyObject *ints = NULL, *exps = NULL, *words = NULL, *res = NULL;
  int ok = 1;
  ints = PyList_New(n);
  exps = PyBytes_FromStringAndSize(NULL, n * 4);
  if (!ints || !exps) goto done;
  int32_t* e = (int32_t*)PyBytes_AS_STRING(exps);
  for (Py_ssize_t i = 0; i < n && ok; ++i) {
    PyObject* o = it[i];
    if (!PyObject_TypeCheck(o, cls)) {
      ok = 0;
      break;
    }
    PyObject* pk = *(PyObject**)((char*)o + o_pk);
    if (!pk) {
      ok = 0;
      break;
    }
    if (pk != key && pk != same_key) {
      const int eq = PyObject_RichCompareBool(pk, key, Py_EQ);
      if (eq < 0) goto done;
      if (!eq) {
        ok = 0;
        break;
      }
      same_key = pk;
    }
    PyObject* ct = *(PyObject**)((char*)o + o_ct);
    PyObject* ex = *(PyObject**)((char*)o + o_ex);
    if (!ct || !ex || !PyLong_CheckExact(ct) || !PyLong_Check(ex)) {
      ok = 0;
      break;
    }
    int over = 0;
    const long long v = PyLong_AsLongLongAndOverflow(ex, &over);
    if (over || v < INT32_MIN || v > INT32_MAX) {
      if (PyErr_Occurred()) goto done;
      ok = 0;
      break;
    }
    e[i] = (int32_t)v;
    Py_INCREF(ct);
    PyList_SET_ITEM(ints, i, ct);
  }
  if (!ok) {
    res = Py_None;
    Py_INCREF(res);
    goto done;
  }
  if (want) {
    words = PyBytes_FromStringAndSize(NULL, n * 4 * nw);
    if (!words) goto done;
    PyObject** iv = ((PyListObject*)ints)->ob_item;
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    if (nt > W2I_THREADS_MAX) nt = W2I_THREADS_MAX;
    if (nt > n / W2I_ROWS_MIN) nt = (long)(n / W2I_ROWS_MIN);
    if (nt < 1) nt = 1;
    i2w_job jobs[W2I_THREADS_MAX];
    pthread_t th[W2I_THREADS_MAX];
    int started[W2I_THREADS_MAX] = {0};
    const Py_ssize_t per = (n + nt - 1) / nt;
    for (long t = 0; t < nt; ++t) {
      jobs[t].ints = iv;
      jobs[t].out = (unsigned char*)PyBytes_AS_STRING(words);
      jobs[t].lo = t * per < n ? t * per : n;
      jobs[t].hi = (t + 1) * per < n ? (t + 1) * per : n;
      jobs[t].nw = nw;
      jobs[t].bad = 0;
    }
    /* the ints are referenced by `ints` (immutable objects): reading their digits needs no GIL */
    Py_BEGIN_ALLOW_THREADS
    for (long t = 1; t < nt; ++t) started[t] = pthread_create(&th[t], NULL, i2w_fill, &jobs[t]) == 0;
    i2w_fill(&jobs[0]);
    for (long t = 1; t < nt; ++t) {
      if (started[t]) pthread_join(th[t], NULL);
      else i2w_fill(&jobs[t]);
    }
    Py_END_ALLOW_THREADS
    for (long t = 0; t < nt; ++t)
      if (jobs[t].bad) {
        res = Py_None;
        Py_INCREF(res);
        goto done;
      }
  } else {
    words = Py_None;
    Py_INCREF(words);
  }
  res = PyTuple_Pack(3, words, exps, ints);
done:
  Py_XDECREF(words);
  Py_XDECREF(exps);
  Py_XDECREF(ints);
  Py_DECREF(objs);
  return res;
}

static PyMethodDef methods[] = {
    {"pack_numbers", (PyCFunction)(void (*)(void))g_pack_numbers, METH_FASTCALL, "checks + words of received numbers"},
    {"packed_valid", (PyCFunction)(void (*)(void))g_packed_valid, METH_FASTCALL, "cached words still match"},
    {"make_numbers", (PyCFunction)(void (*)(void))g_make_numbers, METH_FASTCALL, "bulk slot construction"},
    {"words_to_ints", (PyCFunction)(void (*)(void))g_words_to_ints, METH_FASTCALL, "rows of LE 32-bit words -> ints"},
    {"ints_to_words", (PyCFunction)(void (*)(void))g_ints_to_words, METH_FASTCALL, "ints -> rows of LE 32-bit words"},
    {"mulmod", (PyCFunction)(void (*)(void))g_mulmod, METH_FASTCALL, "(a * b) % c"},
    {"powmod", (PyCFunction)(void (*)(void))g_powmod, METH_FASTCALL, "a ** b % c (GMP mpz_powm)"},
    {"invert", (PyCFunction)(void (*)(void))g_invert, METH_FASTCALL, "a^-1 mod b"},
    {"scalar_pow", (PyCFunction)(void (*)(void))g_scalar_pow, METH_FASTCALL, "c^k mod m (neg: inverse) with cached squarings"},
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
