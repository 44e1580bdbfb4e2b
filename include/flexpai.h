/*
 * flexpai — MI355X-native Paillier array engine, C ABI.
 *
 * Drop-in boundary for tongdun/iBond-flex `flex.crypto.paillier` (Python). Each entry point
 * replaces the per-element gmpy2 work that the reference does on the CPU:
 *
 *   pai_ctx_create        <- PaillierPublicKey(n)                  flex/crypto/paillier/keypair.py:20-39
 *   pai_ctx_set_private   <- PaillierPrivateKey(pk, p, q)          flex/crypto/paillier/keypair.py:42-90
 *   pai_ctx_set_option    <- (no reference counterpart: selects the CRT encryption kernels)
 *   pai_encrypt[_dev]     <- PaillierEncryptor.encrypt(ndarray)    flex/crypto/paillier/encryptor.py:71-114
 *                            (FixedPointNumber.encode fixedpoint_number.py:46-90, raw_encrypt
 *                             raw_encrypt.py:22-49, apply_obfuscation obfuscator.py:23-37 ->
 *                             gmpy_math.powmod/mulmod gmpy_math.py:43-63)
 *   pai_add[_dev]         <- sum of PaillierEncryptedNumber arrays encrypted_number.py:65-69,
 *                            115-137, 166-185 (k-way, order independent)
 *   pai_decrypt[_dev]     <- PaillierDecryptor.decrypt(ndarray)    flex/crypto/paillier/decryptor.py:33-127
 *                            (+ FixedPointNumber.decode fixedpoint_number.py:92-107)
 *   pai_mul[_dev]         <- PaillierEncryptedNumber.__mul__ / __rmul__ over arrays (encrypted_number.py:80-113;
 *                            parallel_ops.mul parallel_ops.py:23-44): c^s, or invert(c)^(n-s) for negatives
 *   pai_add_plain[_dev]   <- PaillierEncryptedNumber + plain scalar over arrays (encrypted_number.py:65-72,
 *                            139-164 __add_scalar/__add_fixpointnumber; parallel_ops.add parallel_ops.py:47-72)
 *   pai_segment_add[_dev] <- per-bin sums sum(y[i]) over index lists (hetero_bin.py:28-36, IV_FFS
 *                            iv_ffs/compute.py:77-93): one k-way aligned product per segment
 *   pai_matmul[_dev]      <- ndarray.dot of encrypted by plain (he_otp_lr_ft1/train.py:160,
 *                            he_otp_lr_ft2/train.py:188): per output sum_k c_ik (x) x_kj, i.e. __mul__ then
 *                            __add__ (encrypted_number.py:65-69, 86-113, 166-185)
 *   pai_comm_* / pai_allgather_*  <- (no reference counterpart: the reference encrypts on one host's CPU
 *                            pool, encryptor.py:71-97) reassembly of ciphertext shards encrypted on
 *                            several GPUs, one RCCL all-gather over xGMI
 *
 * Conventions
 *   - Integers cross the boundary as little-endian bytes (key material) or little-endian 32-bit
 *     words, one ciphertext contiguous (AoS): ciphertext i occupies words [i*W, (i+1)*W) with
 *     W = pai_ct_words(ctx) = 2*key_bits/32. This is zero-copy with Python int.to_bytes(...,'little').
 *   - Host-buffer entry points are synchronous and never retain caller memory.
 *   - *_dev entry points take device pointers and a hipStream_t (as void*) and are asynchronous.
 *   - Return value 0 = success; negative = error, message in pai_last_error() (thread local).
 *   - Per-element outcomes are reported in an int32 status array (PAI_EL_*), mapped by the Python
 *     layer onto the reference's exceptions.
 *   - Threads: a context may be shared by several threads. Every entry point that takes a pai_ctx holds
 *     the context's (recursive) mutex for the whole call, and a *_dev call's stream first waits for the
 *     device work of the context's previous call, whatever stream that was on (the context's scratch,
 *     work and table buffers are shared by all its calls). Calls on one context therefore run one after
 *     the other; contexts of different keys run concurrently. pai_ctx_destroy must not race other calls
 *     on the same context. (The reference never shares this state: it pickles the key into pool
 *     processes, encryptor.py:89-96.)
 *   - Reproducibility: PAI_OBF_RNG ciphertexts depend only on (rng_key, global index) for a given sampler,
 *     but the sampler is chosen per context: the fixed-base tables are built only once a context has seen
 *     the break-even element count (pai_ctx_fixed_base_policy). Two process layouts (one process vs
 *     sharded ranks, whose shards may sit below the threshold) give the same bits only when the tables are
 *     built up front (pai_ctx_fixed_base_prepare / pai_ctx_public_fb_prepare) or $FLEXPAI_FB_MIN_ELEMS /
 *     $FLEXPAI_PFB_MIN_ELEMS = 0; otherwise the outputs differ in bits but decrypt identically and have
 *     the same distribution.
 */
#ifndef FLEXPAI_H
#define FLEXPAI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pai_ctx pai_ctx;
typedef struct pai_comm pai_comm;

/* return codes */
#define PAI_OK 0
#define PAI_ERR_ARG (-1)
#define PAI_ERR_HIP (-2)
#define PAI_ERR_NOPRIV (-3)
#define PAI_ERR_KEY (-4)
#define PAI_ERR_NOINV (-5)  /* a ciphertext has no inverse mod n^2 (gmpy_math.invert ZeroDivisionError) */

/* input dtypes for pai_encrypt */
#define PAI_F32 0
#define PAI_F64 1
#define PAI_I64 2

/* obfuscation modes (SURVEY.md §8b randomness contract) */
#define PAI_OBF_NONE 0   /* random_value == 0 : c = 1 + n*m                      (encryptor.py:61-67) */
#define PAI_OBF_GIVEN 1  /* explicit r per element (r_stride 0 = one r for all)  (obfuscator.py:35)  */
#define PAI_OBF_RNG 2    /* device ChaCha20 CSPRNG keyed by rng_key, nonce = global element index    */

/* exponent modes for encode (fixedpoint_number.py:63-82) */
#define PAI_EXP_AUTO 0   /* precision=None: exponent from frexp / 0 for ints */
#define PAI_EXP_FIXED 1  /* precision given: exponent = fixed_exp for every element */

/* per-element status */
#define PAI_EL_OK 0           /* float result in val_out                                            */
#define PAI_EL_INT 1          /* exponent <= 0: exact integer mant_out * 16^(-exp) (fits int64)      */
#define PAI_EL_INT_BIG 2      /* exponent <= 0 and the mantissa does not fit int64 (use raw_out)     */
#define PAI_EL_OVERFLOW 3     /* OverflowError('Overflow detected in decode number')  :104-105     */
#define PAI_EL_FLOAT_OVF 4    /* OverflowError: int too large to convert to float (e > 0)           */
#define PAI_EL_ENC_RANGE 5    /* encode ValueError (fixedpoint_number.py:86-88) / beyond int64      */

/* context options */
#define PAI_OPT_CRT_ENCRYPT 1    /* 1 (default): encrypt via the private-key CRT path when available */
#define PAI_OPT_CRT_AVAILABLE 2  /* read-only: 1 when the private key is set and the CRT kernels fit */
#define PAI_OPT_STAGE_TIMING 3   /* 1: record HIP events between the kernels of each encrypt/decrypt call */
#define PAI_OPT_LANE_DECRYPT 4   /* 1 (default): decrypt on the lane engine when the key halves fit it;
                                    0: lane-group kernel. Read back: 1 when the lane path is in use  */
#define PAI_OPT_FIXED_BASE 5     /* 1 (default): PAI_OBF_RNG encryption with the private key set samples
                                    r^n through fixed bases (G_p^a_p, G_q^a_q: same distribution as
                                    r^n for uniform r, see pai_ctx_fixed_base_info); 0: r from the
                                    ChaCha20 stream and r^n by exponentiation. Read back: 1 when used */
#define PAI_OPT_FB_WINDOW 6      /* digit window of the fixed-base tables: 8, 12, 16 or 20 .. 24 bits (default 16, or
                                    $FLEXPAI_FB_WINDOW); setting it drops the tables (rebuilt lazily). Read
                                    back: the window of the resident tables, which is the largest one <= the
                                    requested window whose 2 K 2^W rows fit $FLEXPAI_FB_MAX_BYTES (default:
                                    free device memory less max(4 GiB, 1/12 of the device)).
                                    $FLEXPAI_FB_WINDOW=auto: a process holding ONE private key asks for 24 and
                                    gets the largest window whose tables fit $FLEXPAI_FB_AUTO_FRAC (default
                                    0.75) of the free memory (W = 22 at nb = 2048, 21 at nb = 4096 on an idle
                                    MI355X); a process holding several keys gets 16                          */
#define PAI_OPT_FB_READY 7       /* read-only: 1 when the fixed-base tables are resident                    */
#define PAI_OPT_FB_PAIR 8        /* read-only: limbs of p_h (19, 37; 76 for the 4096-bit pair-group tables)
                                    when the resident tables are pair tables (kernels_fbp.hpp,
                                    kernels_grp_pair.hpp: the default; round 1's k_fb / k_fbg were retired in round 6),
                                    else 0                                                                     */
#define PAI_OPT_PAIR 9           /* read-only: bit 0 = decryption, bit 1 = CRT encryption (stage B), bit 2 =
                                    public-key encryption (2048-bit n, and n of at most 1024 bits) run on
                                    p-adic pairs (kernels_pair.hpp, kernels_dec4.hpp, kernels_pe.hpp,
                                    kernels_pe1.hpp: the default; $FLEXPAI_PAIR=0 at context creation selects
                                    the kernels they replace)                                                  */
#define PAI_OPT_PUBLIC_FB 10     /* 1 (default): PAI_OBF_RNG encryption WITHOUT the private key (2048-bit n) samples
                                  * r^n through the public fixed bases (kernels_pfb.hpp) once the break-even count
                                  * is reached (pai_ctx_public_fb_policy); get: 1 when the path is enabled and not
                                  * known unavailable                                                          */
#define PAI_OPT_PFB_READY 11     /* read-only: 1 when the public fixed-base tables are resident               */
#define PAI_OPT_PFB_WINDOW 12    /* digit window of the public tables: 12, 16 or 20 (the windows pinned to the
                                  * reference's goldens; default 16: 324 rows of 512 B per element, 10.9 GB of
                                  * tables; $FLEXPAI_FB_WINDOW=auto: 20 for a process with one context)       */
#define PAI_OPT_SPLIT_SAMPLER 13 /* read-only: bit 0 = the resident 4096-bit key-holder tables, bit 1 = the resident
                                  * public tables are sampled on split pairs (kernels_sgp.hpp: k_sgp, the default;
                                  * $FLEXPAI_SGP=0 at table build selects k_fbgp / k_pfb); bit 2 = the resident
                                  * 1024/2048-bit key-holder tables hold Shoup rows sampled on split pairs
                                  * (kernels_fbs.hpp: k_fbs, the default; $FLEXPAI_FBS=0 in the test build keeps
                                  * k_fbp's Montgomery rows); bit 3 = the resident 4096-bit key-holder tables add
                                  * Shoup rows (kernels_sgs.hpp: k_sgs, the default where they price lower than the
                                  * factored rows at their window; $FLEXPAI_SGS=0 keeps k_sgp, =1 takes them
                                  * whenever they fit)                                                        */
#define PAI_OPT_ROWS_MAX 14      /* calls of at most this many elements (default 4096) run their exponentiations with
                                  * each residue on a 16-lane row (kernels_crtw.hpp: the key holder's CRT encryption
                                  * k_crt_w and decryption k_dec_w, a public-key-only party's encryption k_pe_w; the
                                  * latency of protocol-sized calls) instead of one lane / lane pair each; 0
                                  * disables. Same bits either way                                               */

/* Number of visible GPUs (0 when there is none or the runtime cannot start). */
int pai_device_count(int* count);
/* Free and total device memory of `device` (bytes). */
int pai_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes);
int pai_ctx_create(const uint8_t* n_le, size_t n_bytes, int device, pai_ctx** out);
int pai_ctx_set_private(pai_ctx* ctx, const uint8_t* p_le, const uint8_t* q_le, size_t half_bytes);
void pai_ctx_destroy(pai_ctx* ctx);
/* Fixed-base tables live in device memory the library keeps when they are released (a window change, a context's
 * end): the next table build in the process maps it again instead of waiting for the driver to wipe released memory
 * (csrc/table_arena.hpp). It goes back to the driver when the process's last context is destroyed, or now with this
 * call (no context may be building tables concurrently). $FLEXPAI_TABLE_POOL=0: plain hipMalloc / hipFree. */
void pai_release_table_cache(void);
/* Encryption with the private key set uses CRT over p^2, q^2 (same ciphertext bits, ~4x fewer
 * multiply-accumulates); PAI_OPT_CRT_ENCRYPT = 0 forces the public-key kernel. */
int pai_ctx_set_option(pai_ctx* ctx, int option, int value);
int pai_ctx_get_option(const pai_ctx* ctx, int option, int* value);
/* With PAI_OPT_STAGE_TIMING on: kernel durations (ms) of the last encrypt call, summed over all its chunks
 * (a host-buffer call's chunks included; past 64 chunks the recorded ones are folded into running sums,
 * which waits for them), in launch order (CRT: stage A, stage B, finish; public key on pairs: k_pe_pre, k_pe_pow, k_pe_fin; other public-key
 * paths: the one encrypt kernel). Waits for them. */
int pai_ctx_stage_times(pai_ctx* ctx, float* ms_out, int max_out, int* count);
/* key bits, 32-bit words per ciphertext (2*key_bits/32), words per plaintext (key_bits/32) */
int pai_ctx_info(const pai_ctx* ctx, int* key_bits, int* ct_words, int* pt_words);
const char* pai_last_error(void);
/* Fixed-base obfuscation parameters (PAI_OPT_FIXED_BASE): the bases g_p, g_q (generators of Z_p*,
 * Z_q*, p < q) with G_h = g_h^n mod h^2, the digit count K and the window W. Element i's exponent is
 * a_h = raw_h mod (h - 1), raw_h = the little-endian integer of the first max(bits(p-1), bits(q-1)) + 64
 * bits of the ChaCha20 stream (rng_key, counter 0.., nonce = (index lo, index hi, 0x66786230 + h));
 * r^n mod h^2 is G_h^a_h, i.e. the ciphertext is the reference's encryption under the obfuscator
 * r = CRT(g_p^a_p mod p, g_q^a_q mod q). Builds the tables if they are not resident (like
 * pai_ctx_fixed_base_prepare); PAI_ERR_KEY with the reason when the path is unavailable.          */
int pai_ctx_fixed_base_info(pai_ctx* ctx, uint32_t* g_p, uint32_t* g_q, int* digits, int* window);
/* Build the fixed-base tables now (otherwise on the first PAI_OBF_RNG encryption with the private key).
 * 0 when they are resident; PAI_ERR_KEY / PAI_ERR_NOPRIV with the reason otherwise (encryption then
 * uses the generic CRT path; decryption is never affected).                                       */
int pai_ctx_fixed_base_prepare(pai_ctx* ctx);
/* Cost of the last table build: host ms (bases, B_k, constants, hipMalloc), device ms (table kernels),
 * resident table bytes.                                                                            */
int pai_ctx_fixed_base_setup(const pai_ctx* ctx, float* host_ms, float* device_ms, uint64_t* table_bytes);
/* Fixed-base break-even: a device-RNG encryption builds the tables only once the device-RNG
 * elements encrypted under this context (the current call included) reach `threshold` (estimated build
 * time / per-element saving against the generic path; $FLEXPAI_FB_MIN_ELEMS overrides); smaller calls
 * take the generic path (same ciphertext distribution). `seen`: elements counted so far. threshold = 0
 * once the tables are resident or known unavailable. Replaces nothing in the reference (its obfuscator,
 * obfuscator.py:23-37, has no per-key state); protects re-keying callers (he_sa_ft/train.py:39-40).  */
int pai_ctx_fixed_base_policy(pai_ctx* ctx, long long* seen, long long* threshold);

/* Public-key fixed bases (DESIGN.md §3 "Fixed bases without the private key"; replaces, for a party holding
 * only n, the per-element gmpy2.powmod(r, n, n^2) of obfuscator.py:35-36). The context draws 33 bases
 * g_0..g_32 in [2, n) from the OS CSPRNG (g_0 with Jacobi symbol (g_0 | n) = -1); element i's obfuscator is
 * r = prod_j g_j^e_j mod n with the exponents read from its ChaCha20 stream (rng_key, counter 0.., nonce =
 * (index lo, index hi, 0x70666230)) cut into W-bit digits: digits [0, K0) are e_0 (K0 = ceil((nb + 64) / W)),
 * then 32 runs of KS = ceil(96 / W) digits are e_1..e_32, each little-endian. The ciphertext is the
 * reference's encryption of x under that r.                                                            */
int pai_ctx_public_fb_prepare(pai_ctx* ctx);
/* Use these bases (nbases = 33, each base_bytes little-endian, 1 < g < n) instead of random ones; drops
 * resident public tables (rebuilt lazily). For reproducible runs and the parity tests. PAI_ERR_ARG unless
 * every base is a unit mod n, the bases are distinct and g_0 has Jacobi symbol (g_0 | n) = -1: the
 * conditions of the distribution argument that a caller can check.                      */
int pai_ctx_public_fb_set_bases(pai_ctx* ctx, const uint8_t* bases_le, size_t base_bytes, int nbases);
/* The resident public tables' bases (nbases x base_bytes, nullable), digit count K, window W, and K0.
 * PAI_ERR_KEY when the tables are not resident.                                                        */
int pai_ctx_public_fb_info(pai_ctx* ctx, uint8_t* bases_le, size_t base_bytes, int* nbases, int* digits,
                           int* window, int* e0_digits);
/* Break-even of the public tables, like pai_ctx_fixed_base_policy ($FLEXPAI_PFB_MIN_ELEMS overrides).  */
int pai_ctx_public_fb_policy(pai_ctx* ctx, long long* seen, long long* threshold);

/* Encrypt N plaintexts. dtype PAI_F32/F64/I64. obf_mode PAI_OBF_*.
 *   r_le:      PAI_OBF_GIVEN only: r values as little-endian byte strings of r_bytes each, element i
 *              at r_le + i*r_stride_bytes (stride 0 = the same r for every element). 1 <= r < n^2.
 *   rng_key32: PAI_OBF_RNG only: 32-byte ChaCha20 key; element i uses nonce (index_base + i).
 * Outputs: ct_out N*W words, exp_out N exponents, status_out N statuses (nullable).           */
int pai_encrypt(pai_ctx* ctx, int dtype, const void* x, size_t N, int exp_mode, int32_t fixed_exp,
                int obf_mode, const uint8_t* r_le, size_t r_stride_bytes, size_t r_bytes,
                const uint8_t* rng_key32, uint64_t index_base,
                uint32_t* ct_out, int32_t* exp_out, int32_t* status_out);

/* k-way homomorphic add: out_i = prod_j ct_j,i^(16^(E_i - e_j,i)) mod n^2, E_i = max_j e_j,i. */
int pai_add(pai_ctx* ctx, const uint32_t* const* cts, const int32_t* const* exps, int k, size_t N,
            uint32_t* ct_out, int32_t* exp_out);

/* Decrypt + decode. val_out: float64 value (status OK/INT), mant_out: signed mantissa when it
 * fits int64 (nullable), status_out (required), raw_out: N * pt_words canonical plaintexts
 * m = D(c) in [0, n) (nullable).                                                              */
int pai_decrypt(pai_ctx* ctx, const uint32_t* ct, const int32_t* exp, size_t N, double* val_out,
                int64_t* mant_out, int32_t* status_out, uint32_t* raw_out);

/* Ciphertext x plaintext, element-wise: out_i = ct_i (x) x_(i*x_stride) (x_stride 0: one scalar for all,
 * 1: one per element), x of dtype PAI_F32/F64/I64 encoded like FixedPointNumber.encode; exponent
 * exp_i + e(x). Negative scalars: invert(ct)^|m|, computed as ONE batch inversion for the array.
 * status_out (nullable): PAI_EL_ENC_RANGE where the scalar does not fit the 64-bit encoder.      */
int pai_mul(pai_ctx* ctx, const uint32_t* ct, const int32_t* exp, size_t N, int dtype, const void* x, size_t x_stride,
            uint32_t* ct_out, int32_t* exp_out, int32_t* status_out);
/* Ciphertext + plaintext, element-wise: out_i = ct_i (+) x_(i*x_stride), x encoded like
 * FixedPointNumber.encode(x, max_exponent=exp_i) (fixedpoint_number.py:81-84) and raw-encrypted with r = 1,
 * exponent max(exp_i, e(x)). status_out (nullable): PAI_EL_FLOAT_OVF where x * 16^E is not a finite double
 * (OverflowError), PAI_EL_ENC_RANGE where |M| >= 2^(nb-3) (the exact |M| > max_int test is the caller's);
 * those outputs are undefined and the caller redoes them. Integers are exact (numpy's object add loop sees
 * Python ints), so int64 * 16^E never wraps. */
int pai_add_plain(pai_ctx* ctx, const uint32_t* ct, const int32_t* exp, size_t N, int dtype, const void* x,
                  size_t x_stride, uint32_t* ct_out, int32_t* exp_out, int32_t* status_out);
/* Segmented k-way add: out_s = prod over t in [seg_off[s], seg_off[s+1]) of ct[index[t]] aligned to the
 * segment's maximum exponent (same as pai_add over the members). index and seg_off (nseg + 1 offsets,
 * seg_off[0] = 0, non-decreasing) are host arrays in both variants. An empty segment yields ciphertext 1
 * with exponent INT32_MIN. The _dev variant synchronises `stream` once per reduction level. */
int pai_segment_add(pai_ctx* ctx, const uint32_t* ct, const int32_t* exp, size_t N, const int64_t* index,
                    const int64_t* seg_off, size_t nseg, uint32_t* ct_out, int32_t* exp_out);
/* Encrypted (m x K, row-major ciphertexts + exponents) times plain (K x d, row-major, dtype as above):
 * out[i][j] = sum_k ct[i][k] (x) x[k][j] with the reference's exponent alignment (bit-identical to
 * numpy's object dot over PaillierEncryptedNumber, whose sums are order independent). */
int pai_matmul(pai_ctx* ctx, const uint32_t* ct, const int32_t* exp, size_t m, size_t K, int dtype, const void* x,
               size_t d, uint32_t* ct_out, int32_t* exp_out);

/* Device-resident variants (device pointers, asynchronous on `stream`, a hipStream_t; pai_mul_dev and
 * pai_matmul_dev synchronise `stream` once, for the single host-side inversion of the batch). pai_encrypt_dev never
 * waits on the host: the public-key chain's batch inversion (chunks of >= 16384 elements) inverts its one top value
 * in a host function queued on `stream` (hipLaunchHostFunc), so the call stays asynchronous and capturable; only
 * the first device-RNG call that BUILDS a key's fixed-base tables synchronises the device (per-key setup). */
int pai_encrypt_dev(pai_ctx* ctx, int dtype, const void* d_x, size_t N, int exp_mode, int32_t fixed_exp,
                    int obf_mode, const uint32_t* d_r_words, size_t r_stride_words, size_t r_words,
                    const uint8_t* rng_key32, uint64_t index_base,
                    uint32_t* d_ct, int32_t* d_exp, int32_t* d_status, void* stream);
/* d_cts: k consecutive [N][W] ciphertext arrays; d_exps: k consecutive [N] exponent arrays. */
int pai_add_dev(pai_ctx* ctx, const uint32_t* d_cts, const int32_t* d_exps, int k, size_t N,
                uint32_t* d_out, int32_t* d_exp_out, void* stream);
int pai_decrypt_dev(pai_ctx* ctx, const uint32_t* d_ct, const int32_t* d_exp, size_t N, double* d_val,
                    int64_t* d_mant, int32_t* d_status, uint32_t* d_raw, void* stream);
int pai_mul_dev(pai_ctx* ctx, const uint32_t* d_ct, const int32_t* d_exp, size_t N, int dtype, const void* d_x,
                size_t x_stride, uint32_t* d_out, int32_t* d_exp_out, int32_t* d_status, void* stream);
int pai_add_plain_dev(pai_ctx* ctx, const uint32_t* d_ct, const int32_t* d_exp, size_t N, int dtype,
                      const void* d_x, size_t x_stride, uint32_t* d_out, int32_t* d_exp_out, int32_t* d_status,
                      void* stream);
int pai_segment_add_dev(pai_ctx* ctx, const uint32_t* d_ct, const int32_t* d_exp, size_t N, const int64_t* index,
                        const int64_t* seg_off, size_t nseg, uint32_t* d_out, int32_t* d_exp_out, void* stream);
int pai_matmul_dev(pai_ctx* ctx, const uint32_t* d_ct, const int32_t* d_exp, size_t m, size_t K, int dtype,
                   const void* d_x, size_t d, uint32_t* d_out, int32_t* d_exp_out, void* stream);

/* Multi-GPU: ciphertext shards -> every rank (RCCL, opened with dlopen on first use; one process per GPU).
 * Rank 0 calls pai_comm_unique_id and hands the PAI_COMM_ID_BYTES bytes to the other ranks over any
 * channel; every rank then calls pai_comm_create (collective). */
#define PAI_COMM_ID_BYTES 128
int pai_comm_unique_id(uint8_t* id_out);
int pai_comm_create(const uint8_t* id, int world, int rank, int device, pai_comm** out);
void pai_comm_destroy(pai_comm* comm);
/* d_recv[r * bytes_per_rank ...] <- rank r's d_send; asynchronous on `stream` (a hipStream_t). */
int pai_allgather_dev(pai_comm* comm, const void* d_send, size_t bytes_per_rank, void* d_recv, void* stream);
/* Both halves of a ciphertext shard (words [n_per_rank][ct_words], exponents [n_per_rank]) in one grouped
 * launch: d_ct_all [world * n_per_rank][ct_words], d_exp_all [world * n_per_rank]. */
int pai_allgather_shards_dev(pai_comm* comm, const uint32_t* d_ct, const int32_t* d_exp, size_t n_per_rank,
                             int ct_words, uint32_t* d_ct_all, int32_t* d_exp_all, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FLEXPAI_H */
