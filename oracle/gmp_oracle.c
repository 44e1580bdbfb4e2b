/*
 * CPU ORACLE (C + GMP) for the Paillier hot path — TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library.
 * It restates the reference's per-element CPU path of tongdun/iBond-flex on the same
 * arithmetic library the reference reaches through gmpy2 2.0.8 (GMP 6.2.1, requirements.txt:6):
 *   encode        flex/crypto/paillier/fixedpoint_number.py:46-90
 *   c0 = 1 + n*m  flex/crypto/paillier/raw_encrypt.py:37-45
 *   r^n mod n^2   flex/crypto/paillier/obfuscator.py:36  (gmpy_math.powmod -> mpz_powm, gmpy_math.py:51-63)
 *   c0 * r^n      flex/crypto/paillier/obfuscator.py:37  (gmpy_math.mulmod, gmpy_math.py:43-48)
 *   decrypt (CRT) flex/crypto/paillier/decryptor.py:33-63, gmpy_math.crt gmpy_math.py:31-40
 * and parallelises over elements with a pool of worker threads, as the reference does with
 * multiprocessing.Pool(cpu_count()) (encryptor.py:89-96, decryptor.py:106-111).
 * The per-element obfuscator is the same ChaCha20 stream the device CSPRNG uses
 * (oracle/paillier_oracle.py:device_r), so outputs are bit-comparable with the GPU.
 * Parity pinning: tests/test_gmp_oracle.py checks it against the reference golden vectors.
 */
#include <gmp.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void chacha20_block(const uint32_t key[8], uint32_t counter, uint32_t n0, uint32_t n1, uint32_t n2,
                           uint32_t out[16]) {
#define ROTL(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)  \
  a += b; d = ROTL(d ^ a, 16); \
  c += d; b = ROTL(b ^ c, 12); \
  a += b; d = ROTL(d ^ a, 8);  \
  c += d; b = ROTL(b ^ c, 7);
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4], key[5], key[6], key[7], counter, n0, n1, n2};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
  for (int r = 0; r < 10; ++r) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
#undef QR
#undef ROTL
}

/* encode a finite float value (precision=None); returns 0 on success */
static int encode_double(double v, int64_t* M, int* e) {
  if (fabs(v) < 1e-200) { *M = 0; *e = 0; return 0; }
  int fe;
  (void)frexp(v, &fe);
  int a = 53 - fe;
  *e = a >= 0 ? a / 4 : -((-a + 3) / 4);
  double s = rint(ldexp(v, 4 * (*e)));
  if (!(fabs(s) < 9.223372036854775e18)) return -1;
  *M = (int64_t)s;
  return 0;
}

typedef struct {
  mpz_t n, nsq;
  int ct_words, r_words;
  uint32_t key[8];
  uint64_t index_base;
  const float* x;
  uint32_t* ct_out;
  int32_t* exp_out;
  size_t N;
  size_t next;
  pthread_mutex_t lock;
} enc_job;

static void* enc_worker(void* arg) {
  enc_job* J = (enc_job*)arg;
  mpz_t r, c, c0, m, t;
  mpz_inits(r, c, c0, m, t, NULL);
  uint32_t rbuf[256];
  for (;;) {
    pthread_mutex_lock(&J->lock);
    size_t i = J->next;
    J->next += 16;
    pthread_mutex_unlock(&J->lock);
    if (i >= J->N) break;
    size_t end = i + 16 < J->N ? i + 16 : J->N;
    for (; i < end; ++i) {
      int64_t M;
      int e;
      encode_double((double)J->x[i], &M, &e);
      /* m = M mod n; c0 = (n*m + 1) mod n^2 */
      mpz_set_si(m, 0);
      if (M >= 0) mpz_set_ui(m, (unsigned long)M);
      else { mpz_set_ui(t, (unsigned long)(-(uint64_t)M)); mpz_sub(m, J->n, t); }
      mpz_mul(c0, J->n, m);
      mpz_add_ui(c0, c0, 1);
      mpz_mod(c0, c0, J->nsq);
      /* r from the ChaCha20 stream of element index_base + i */
      uint64_t g = J->index_base + i;
      for (int b = 0; b * 16 < J->r_words; ++b) chacha20_block(J->key, (uint32_t)b, (uint32_t)g, (uint32_t)(g >> 32), 0x66786169u, rbuf + 16 * b);
      mpz_import(r, J->r_words, -1, 4, 0, 0, rbuf);
      mpz_mod(r, r, J->n);
      mpz_powm(t, r, J->n, J->nsq);
      mpz_mul(c, c0, t);
      mpz_mod(c, c, J->nsq);
      uint32_t* out = J->ct_out + i * (size_t)J->ct_words;
      memset(out, 0, 4 * (size_t)J->ct_words);
      mpz_export(out, NULL, -1, 4, 0, 0, c);
      J->exp_out[i] = e;
    }
  }
  mpz_clears(r, c, c0, m, t, NULL);
  return NULL;
}

/* Encrypt N float32 values with obfuscators r_i = ChaCha20(key, index_base + i) mod n. */
int oracle_encrypt_f32_chacha(const uint8_t* n_le, size_t n_bytes, const float* x, size_t N, const uint8_t* key32,
                              uint64_t index_base, uint32_t* ct_out, int32_t* exp_out, int nthreads) {
  enc_job J;
  mpz_init(J.n);
  mpz_init(J.nsq);
  mpz_import(J.n, n_bytes, -1, 1, 0, 0, n_le);
  mpz_mul(J.nsq, J.n, J.n);
  int nb = (int)mpz_sizeinbase(J.n, 2);
  J.ct_words = (2 * nb + 31) / 32;
  J.r_words = (nb + 64 + 31) / 32;
  memcpy(J.key, key32, 32);
  J.index_base = index_base;
  J.x = x;
  J.ct_out = ct_out;
  J.exp_out = exp_out;
  J.N = N;
  J.next = 0;
  pthread_mutex_init(&J.lock, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, enc_worker, &J);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&J.lock);
  mpz_clear(J.n);
  mpz_clear(J.nsq);
  return 0;
}

typedef struct {
  mpz_t n, p, q, psq, qsq, hp, hq, qinv;
  int ct_words, pt_words;
  const uint32_t* ct;
  uint32_t* pt_out;
  size_t N, next;
  pthread_mutex_t lock;
} dec_job;

static void* dec_worker(void* arg) {
  dec_job* J = (dec_job*)arg;
  mpz_t c, mp, mq, u, x, pm1, qm1;
  mpz_inits(c, mp, mq, u, x, pm1, qm1, NULL);
  mpz_sub_ui(pm1, J->p, 1);
  mpz_sub_ui(qm1, J->q, 1);
  for (;;) {
    pthread_mutex_lock(&J->lock);
    size_t i = J->next;
    J->next += 16;
    pthread_mutex_unlock(&J->lock);
    if (i >= J->N) break;
    size_t end = i + 16 < J->N ? i + 16 : J->N;
    for (; i < end; ++i) {
      mpz_import(c, J->ct_words, -1, 4, 0, 0, J->ct + i * (size_t)J->ct_words);
      mpz_powm(mp, c, pm1, J->psq);
      mpz_sub_ui(mp, mp, 1);
      mpz_fdiv_q(mp, mp, J->p);
      mpz_mul(mp, mp, J->hp);
      mpz_mod(mp, mp, J->p);
      mpz_powm(mq, c, qm1, J->qsq);
      mpz_sub_ui(mq, mq, 1);
      mpz_fdiv_q(mq, mq, J->q);
      mpz_mul(mq, mq, J->hq);
      mpz_mod(mq, mq, J->q);
      mpz_sub(u, mp, mq);
      mpz_mul(u, u, J->qinv);
      mpz_mod(u, u, J->p);
      mpz_mul(x, u, J->q);
      mpz_add(x, x, mq);
      mpz_mod(x, x, J->n);
      uint32_t* out = J->pt_out + i * (size_t)J->pt_words;
      memset(out, 0, 4 * (size_t)J->pt_words);
      mpz_export(out, NULL, -1, 4, 0, 0, x);
    }
  }
  mpz_clears(c, mp, mq, u, x, pm1, qm1, NULL);
  return NULL;
}

/* Raw CRT decryption (decryptor.py:33-63): plaintext words (N x pt_words). */
int oracle_decrypt_raw(const uint8_t* p_le, const uint8_t* q_le, size_t half_bytes, const uint32_t* ct, size_t N,
                       uint32_t* pt_out, int nthreads) {
  dec_job J;
  mpz_inits(J.n, J.p, J.q, J.psq, J.qsq, J.hp, J.hq, J.qinv, NULL);
  mpz_import(J.p, half_bytes, -1, 1, 0, 0, p_le);
  mpz_import(J.q, half_bytes, -1, 1, 0, 0, q_le);
  if (mpz_cmp(J.q, J.p) < 0) mpz_swap(J.p, J.q);
  mpz_mul(J.n, J.p, J.q);
  mpz_mul(J.psq, J.p, J.p);
  mpz_mul(J.qsq, J.q, J.q);
  mpz_invert(J.qinv, J.q, J.p);
  /* hp = L(g^(p-1) mod p^2)^-1 mod p with g = n + 1 (keypair.py:81-90) */
  mpz_t g, t;
  mpz_inits(g, t, NULL);
  mpz_add_ui(g, J.n, 1);
  mpz_sub_ui(t, J.p, 1);
  mpz_powm(t, g, t, J.psq);
  mpz_sub_ui(t, t, 1);
  mpz_fdiv_q(t, t, J.p);
  mpz_invert(J.hp, t, J.p);
  mpz_sub_ui(t, J.q, 1);
  mpz_powm(t, g, t, J.qsq);
  mpz_sub_ui(t, t, 1);
  mpz_fdiv_q(t, t, J.q);
  mpz_invert(J.hq, t, J.q);
  mpz_clears(g, t, NULL);
  int nb = (int)mpz_sizeinbase(J.n, 2);
  J.ct_words = (2 * nb + 31) / 32;
  J.pt_words = (nb + 31) / 32;
  J.ct = ct;
  J.pt_out = pt_out;
  J.N = N;
  J.next = 0;
  pthread_mutex_init(&J.lock, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int k = 0; k < nthreads; ++k) pthread_create(&th[k], NULL, dec_worker, &J);
  for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
  free(th);
  pthread_mutex_destroy(&J.lock);
  mpz_clears(J.n, J.p, J.q, J.psq, J.qsq, J.hp, J.hq, J.qinv, NULL);
  return 0;
}
