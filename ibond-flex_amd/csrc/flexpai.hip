// flexpai: host context + C ABI for the MI355X Paillier engine (see include/flexpai.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <sys/random.h>
#include <thread>
#include <array>
#include <vector>
#include <optional>

#include "flexpai.h"
#include "host_bignum.hpp"
#include "table_arena.hpp"
#include "kernels.hpp"
#include "kernels_crt.hpp"
#include "engine_dec.hpp"
#include "engine_lane.hpp"
#include "engine_fb.hpp"
#include "engine_fbp.hpp"
#include "engine_fbs.hpp"

// FLEXPAI_XCHECK (the test-only library libflexpai_xcheck.so, __graft_entry__.build): the kernel generations the
// pair kernels replaced -- k_fbgp, k_pfb, k_fbp (k_fb/k_fb_fin, k_fbg and the 2S-limb k_dec_* / k_crt_b were retired in
// round 6) -- and k_debug, selected by $FLEXPAI_SGP=0 / $FLEXPAI_FBS=0 ($FLEXPAI_PAIR=0: the group-engine decryption and
// the public-key encryption kernels of the product), so that the tests can cross-check the shipping
// kernels against them. The product library (FLEXPAI_XCHECK 0) does not contain them and ignores those variables.
#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0
#endif
static const char* xcheck_env(const char* name) {
#if FLEXPAI_XCHECK
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
#include "engine_pair.hpp"
#include "engine_dec4.hpp"
#include "engine_grp_pair.hpp"
#include "engine_pe.hpp"
#include "engine_pfb.hpp"
#include "engine_sgp.hpp"
#include "engine_sgs.hpp"
#include "engine_grp.hpp"
#include "engine_mul.hpp"
#include "engine_crtw.hpp"
#include "engine_pe1.hpp"

using namespace fpai;

static thread_local std::string g_last_error;

static int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail(PAI_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

// Largest call (elements) whose CRT exponentiations run on 16-lane rows (k_crt_w) instead of lanes / lane pairs
// (k_crt_a + k_crt_b_pair): below it the lane kernels leave the chip mostly idle and take one lane's whole chain.
// The test build keeps 0, so that its contexts -- the cross-checks' references -- stay on the kernels the rows stand in for.
constexpr long long CRTW_DEFAULT_MAX = FLEXPAI_XCHECK ? 0 : 4096;

struct pai_ctx {
  int device = 0;
  int nb = 0;
  int tpi_e = 0, S_e = 0;
  int tpi_d = 0, S_d = 0;
  int ct_words = 0, pt_words = 0;
  HBig n, N;
  uint32_t mprime_N = 0;
  uint32_t *d_N = nullptr, *d_R2 = nullptr, *d_nl = nullptr;
  uint32_t* d_pew_prog = nullptr;   // op list over n for k_pe_w (public-key encryption on 16-lane rows)
  int pew_nprog = 0;
  uint32_t* d_prog = nullptr;   // Montgomery program for x^n (run_program, kernels.hpp)
  int nprog = 0;
  uint32_t* d_oneR = nullptr;   // R mod n^2
  uint32_t* d_RS = nullptr;     // [ADD_KMAX + 2][ct_words]: R^s mod n^2 (k_add's Montgomery corrections)
  void* d_addplan = nullptr;    // k_add schedule sort: buckets, permutation, histogram
  size_t addplan_bytes = 0;
  // private key material
  bool has_priv = false;
  DecHalf* d_halves = nullptr;
  uint32_t *d_qinvR = nullptr, *d_nlimb = nullptr, *d_qRn = nullptr, *d_maxint = nullptr;
  uint32_t nprime_d = 0;
  int nwin = 0, n_limbs = 0;
  // CRT encryption (kernels_crt.hpp): available when the private key is set and the halves fit
  bool crt_ok = false;
  bool fbg_ok = false;        // 4096-bit keys: fixed-base sampler on the group engine (engine_grp), no lane CRT
  bool crt_enabled = true;
  // calls of up to crtw_max elements run the CRT exponentiations on 16-lane rows (kernels_crtw.hpp: latency of
  // protocol-sized calls); PAI_OPT_ROWS_MAX
  long long crtw_max = CRTW_DEFAULT_MAX;
  int crt_sa = 0, crt_sb = 0;
  int rows_sa = 0;   // 74: a 4096-bit key's row-kernel constants (k_crt_w<74, 148>, k_dec_w<74, 148>; setup_rows4096)
  CrtHalf* d_crt_a = nullptr;   // [2] stage A halves
  CrtHalf* d_crt_b = nullptr;   // [2] stage B halves
  uint32_t *d_kq = nullptr, *d_kp = nullptr;
  // lane-engine CRT decryption (kernels_dec.hpp): same sizes as the CRT encryption halves
  bool dec_lane_ok = false;
  bool dec_lane_enabled = true;
  // p-adic pair exponentiations (kernels_pair.hpp): decryption and CRT stage B on the S limbs of p_h;
  // the default for 1024/2048-bit keys ($FLEXPAI_PAIR=0 selects the 2S-limb lane kernels)
  bool dec_pair_ok = false, crt_pair_ok = false;
  DecPairHalf* d_decp_halves = nullptr;
  CrtHalf* d_decp_pow = nullptr;   // decryption halves; c0: the factored chain's K'_t ([16][S], decf)
  bool decf = false;                // the factored (B-free) decryption chain (kernels_pair.hpp decf_run)
  CrtHalf* d_crtp_b = nullptr;
  CrtHalf* d_decw = nullptr;   // [2] k_dec_w's halves (kernels_crtw.hpp): p_h^2, R^(K+1), 1, op list over p_h - 1
  int decw_kchunks = 0;
  uint32_t *d_decp_nl = nullptr, *d_decp_maxint = nullptr;
  int decp_kchunks = 0;
  // 4096-bit keys: decryption on split pairs (kernels_dec4.hpp), the default; the group k_decrypt otherwise
  bool dec4_ok = false;
  Dec4Half* d_dec4_halves = nullptr;
  int dec4_kchunks = 0;
  // public-key encryption on split pairs (kernels_pe.hpp): 2048-bit n, the default ($FLEXPAI_PAIR=0: k_encrypt)
  bool pe_ok = false;
  // public-key encryption of n <= 1024 bits on pairs over the 37 limbs of n (kernels_pe1.hpp)
  bool pe1_ok = false;
  DecPairHalf* d_pe1_half = nullptr;   // n, the pair of R^3 mod n^2 (k_dec_pre_pair's constants)
  uint32_t *d_pe1_n = nullptr, *d_pe1_one = nullptr, *d_pe1_prog = nullptr, *d_pe1_r2n = nullptr;
  int pe1_nprog = 0;
  uint32_t pe1_mprime = 0;
  bool pef_ok = false;          // the factored public-key chain (k_pe_pow_f) is set up ($FLEXPAI_PEF=0, test build: off)
  PeConst* d_pe = nullptr;
  uint32_t *d_pe_n = nullptr, *d_pe_r2 = nullptr, *d_pe_oneR = nullptr;   // n, R^2, R mod n (R = 2^(28 74)): the batch
  uint32_t pe_mprime = 0;                                                 //   inversion of the bases mod n (TPI = 2)
  uint32_t *d_dec_p = nullptr, *d_dec_q = nullptr, *d_dec_qinvR = nullptr;   // (k_dec_fin_pair's CRT constants)
  uint32_t dec_pprime = 0;
  // fixed-base obfuscation (kernels_fb.hpp): device-RNG encryption for key holders. Built lazily on
  // the first PAI_OBF_RNG encryption (or pai_ctx_fixed_base_prepare); any failure (key shape, table
  // memory) leaves the generic CRT path in charge and never affects decryption.
  enum { FB_UNTRIED = 0, FB_READY = 1, FB_UNAVAILABLE = 2 };
  int fb_state = FB_UNTRIED;
  std::string fb_reason;        // why the fixed-base path is unavailable
  bool fb_enabled = true;
  int fb_K = 0;
  int fb_W = 0;                 // digit window (bits); 0 = not chosen yet ($FLEXPAI_FB_WINDOW, default 16)
  int fb_W_used = 0;            // window of the resident tables (may be below fb_W under a memory cap)
  int fb_raw_bits = 0;
  FbHalf* d_fb_halves = nullptr;
  FbpHalf* d_fbp_halves = nullptr;  // pair tables (kernels_fbp.hpp): the default for 1024/2048-bit keys
  uint32_t *d_fbp_fin_cs = nullptr, *d_fbp_fin_p = nullptr;   // k_fbp_fin: its 12 S constant words, p
  uint32_t fbp_fin_mprime = 0;
  int fb_pair_s = 0;            // limbs of p_h of the resident pair tables; 0 = k_fb tables
  bool fb_shoup = false;        // the pair tables hold Shoup rows (kernels_fbs.hpp, k_fbs) instead of Montgomery rows
  FbsConst* d_fbs_cst = nullptr;   // [2] k_fbs_fill's constants (table construction only)
  FbgpHalf* d_fbgp_halves = nullptr;  // 4096-bit keys: pair-group tables (kernels_grp_pair.hpp)
  bool fb_gpair = false;
  SgpHalf* d_sgp_fb = nullptr;  // 4096-bit keys: the split-pair sampler over the same tables (kernels_sgp.hpp)
  SgsHalf* d_sgs_fb = nullptr;  //   ... on Shoup rows ($FLEXPAI_SGS=1, kernels_sgs.hpp)
  const uint32_t* d_sgp_q = nullptr;   //   q's S limbs (k_sgp_fin)
  FbRed* d_fb_red = nullptr;
  uint32_t *d_fb_m8 = nullptr, *d_fb_coefR = nullptr, *d_fb_q2 = nullptr, *d_fb_m0 = nullptr;
  uint32_t* d_fb_q2Rn = nullptr;  // 4096-bit keys: q^2 R mod n^2 (k_fbg_fin)
  uint32_t fb_mprime0 = 0;      // p^2 (Garner)
  uint32_t fb_g[2] = {0, 0};   // the bases g_p, g_q (generators of Z_p*, Z_q*)
  std::vector<void*> fb_mem;    // the tables' constants and build scratch (rebuilt when the window changes)
  std::vector<void*> fb_tables; // the tables themselves (TableArena: pooled device memory)
  HBig fb_p, fb_q;              // p < q
  float fb_host_ms = 0.f, fb_dev_ms = 0.f;
  uint32_t* fb_last_w = nullptr;  // debugging: k_fb output of the last chunk ([2][SB][fb_last_n])
  long long fb_last_n = 0;
  uint64_t fb_table_bytes = 0;
  GuardRec* d_guard = nullptr;  // test build: the address guards' record (guard.hpp); null in the product
#if defined(FBS_AB) && (FBS_AB & 4)
  FbDigitParams* d_abdig = nullptr;   // measurement build: k_fbs's digit parameters
#endif
  // public-key fixed-base obfuscators (kernels_pfb.hpp): device-RNG encryption without the private key.
  // Built lazily past the break-even count (or pai_ctx_public_fb_prepare); never needed for correctness.
  int pfb_state = FB_UNTRIED;
  std::string pfb_reason;
  bool pfb_enabled = true;
  int pfb_W = 0, pfb_W_used = 0, pfb_K = 0, pfb_K0 = 0, pfb_KS = 0;
  std::vector<HBig> pfb_bases;  // g_0 .. g_PFB_SHORT (chosen at the first build unless set)
  PfbConst* d_pfb = nullptr;
  SgpHalf* d_sgp_pfb = nullptr;  // the split-pair sampler over the public tables (kernels_sgp.hpp)
  std::vector<void*> pfb_mem;
  std::vector<void*> pfb_tables;  // (TableArena)
  long long pfb_seen = 0;
  float pfb_host_ms = 0.f, pfb_dev_ms = 0.f;
  uint64_t pfb_table_bytes = 0;
  long long fb_seen = 0;        // device-RNG elements encrypted under this key before the tables exist
  int fb_call = 0;              // host-buffer call in progress: its one fixed-base decision (+1 / -1), else 0
  int pfb_call = 0;             // the same for the public fixed-base sampler
  bool stage_keep = false;      // host-buffer calls: stage timing spans all chunks of the call
  std::vector<void*> allocs;
  std::vector<void*> priv_allocs;   // private-key constants: all freed together if set_private fails
  bool in_priv = false;             // upload() targets priv_allocs
  // scratch (exponent tables), grown on demand
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  void* d_work = nullptr;       // CRT intermediates (y, u)
  size_t work_bytes = 0;
  void* d_mul = nullptr;        // ciphertext x plaintext terms, flags, reduction partials
  size_t mul_bytes = 0;
  void* d_seg = nullptr;        // segmented sums: gather rows and the partial sums of each level
  size_t seg_bytes = 0;
  void* d_plain = nullptr;      // ciphertext + plaintext: the two k_add operands and their exponents
  size_t plain_bytes = 0;
  void* d_inv = nullptr;        // batch-inversion prefix products and segment products
  size_t inv_bytes = 0;
  std::vector<uint32_t> inv_host;   // top of the inversion tree (host side of an async copy)
  // the public-key chain's inversion without a host wait (batch_invert_async): the top value goes device -> pinned
  // words, a host function in stream order inverts it mod n there, and the result (+ a no-inverse flag) goes back
  struct AsyncInv {
    HBig mod;
    int W = 0;
    uint32_t* pin = nullptr;     // [W] words of the top value, then its inverse; [W]: 1 = no inverse exists
  };
  AsyncInv* inv_async = nullptr;
  int cus = 0;
  // optional per-stage timing of the last encrypt call (PAI_OPT_STAGE_TIMING)
  bool timing = false;
  // HIP events between the kernels of each chunk of the last encrypt / decrypt call; the stage times
  // are summed over its chunks (a call of more than CRT_CHUNK elements runs several)
  std::vector<std::array<hipEvent_t, 4>> ev;   // per chunk of the timed call; grown on demand, read at the query
  int nev = 0, nchunk_ev = 0;
  // host-buffer entry points (pai_encrypt / pai_decrypt / pai_add): device copies of the operands, a
  // compute and a copy stream, one event per chunk (host_pipe below)
  void* d_hostio = nullptr;
  size_t hostio_bytes = 0;
  hipStream_t s_comp = nullptr, s_copy = nullptr;
  std::vector<hipEvent_t> hev, pev;   // per chunk: kernels done / staging copy done
  void* h_pin[2] = {nullptr, nullptr};  // pinned staging slots (PCIe at full rate, truly asynchronous)
  size_t pin_bytes = 0;
  // thread safety (CtxLock below): one call at a time per context, and the device work of successive calls
  // ordered through tail_ev even when they come on different streams
  mutable std::recursive_mutex mu;
  hipEvent_t tail_ev = nullptr;
  bool counted = false, holder = false;   // in g_contexts / g_key_holders
  ~pai_ctx();
};

static std::atomic<int> g_contexts{0}, g_key_holders{0};

// $FLEXPAI_SETUP_TRACE=1: wall time of each per-key setup step on stderr ("flexpai-trace <step> <ms>"), and the count
// and time of the constant uploads (the fresh-key analysis of DESIGN §5; tools/fresh_key_trace.py)
static bool setup_trace_on() {
  static const bool on = getenv("FLEXPAI_SETUP_TRACE") != nullptr;
  return on;
}
static std::atomic<long> g_upload_n{0};
static std::atomic<long long> g_upload_ns{0};
struct SetupTrace {
  const char* name;
  std::chrono::steady_clock::time_point t0;
  explicit SetupTrace(const char* n) : name(n), t0(std::chrono::steady_clock::now()) {}
  ~SetupTrace() {
    if (setup_trace_on())
      fprintf(stderr, "flexpai-trace %-32s %10.3f ms\n", name,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};
static void trace_uploads(const char* where) {
  if (!setup_trace_on()) return;
  fprintf(stderr, "flexpai-trace %-32s %10.3f ms (%ld uploads)\n", where, (double)g_upload_ns.exchange(0) * 1e-6,
          g_upload_n.exchange(0));
}

pai_ctx::~pai_ctx() {
  if (counted) --g_contexts;
  if (holder) --g_key_holders;
  (void)hipSetDevice(device);
  if (tail_ev) {
    (void)hipEventSynchronize(tail_ev);
    (void)hipEventDestroy(tail_ev);
  }
  for (auto& ch : ev)
    for (auto& e : ch)
      if (e) (void)hipEventDestroy(e);
  for (auto& e : hev) (void)hipEventDestroy(e);
  for (auto& e : pev) (void)hipEventDestroy(e);
  for (void* p : h_pin)
    if (p) (void)hipHostFree(p);
  if (s_comp) (void)hipStreamDestroy(s_comp);
  if (s_copy) (void)hipStreamDestroy(s_copy);
  if (d_hostio) (void)hipFree(d_hostio);
  if (d_guard) (void)hipFree(d_guard);
  for (void* p : allocs) (void)hipFree(p);
  for (void* p : priv_allocs) (void)hipFree(p);
  for (void* p : fb_mem) (void)hipFree(p);
  for (void* p : pfb_mem) (void)hipFree(p);
  for (void* p : fb_tables) TableArena::get().free(p);
  for (void* p : pfb_tables) TableArena::get().free(p);
  if (counted && g_contexts.load() == 0) TableArena::get().trim();   // the process's last context: pooled chunks go back
  if (d_scratch) (void)hipFree(d_scratch);
  if (d_work) (void)hipFree(d_work);
  if (d_mul) (void)hipFree(d_mul);
  if (d_inv) (void)hipFree(d_inv);
  if (inv_async) {
    if (inv_async->pin) (void)hipHostFree(inv_async->pin);
    delete inv_async;
  }
  if (d_plain) (void)hipFree(d_plain);
  if (d_seg) (void)hipFree(d_seg);
  if (d_addplan) (void)hipFree(d_addplan);
}

// Held by every entry point that takes a context, for the whole call (recursive: the host-buffer entry points
// call the *_dev ones). A context's device buffers -- scratch, work, fixed-base tables, host-io carve-outs --
// are shared by all its calls, so a *_dev call's stream first waits for the device work of the context's
// previous call (whatever stream that was on) and the call's own work becomes the new tail. Two threads may
// therefore share one context: their calls run one after the other, on the host and on the device (SURVEY.md
// §8(b)(iv); the reference isolates its state per process instead, encryptor.py:89-96).
struct CtxLock {
  pai_ctx* c;
  hipStream_t st = nullptr;
  bool dev = false;
  std::unique_lock<std::recursive_mutex> lk;
  explicit CtxLock(const pai_ctx* ctx) : c(const_cast<pai_ctx*>(ctx)), lk(ctx->mu) {}
  CtxLock(pai_ctx* ctx, hipStream_t s) : c(ctx), st(s), dev(true), lk(ctx->mu) {
    (void)hipSetDevice(c->device);
    if (c->tail_ev) (void)hipStreamWaitEvent(st, c->tail_ev, 0);
  }
  ~CtxLock() {
    if (!dev) return;
    if (!c->tail_ev && hipEventCreateWithFlags(&c->tail_ev, hipEventDisableTiming) != hipSuccess) {
      c->tail_ev = nullptr;
      (void)hipGetLastError();
      return;
    }
    (void)hipEventRecord(c->tail_ev, st);
  }
};

template <typename T>
static int upload(pai_ctx* c, const std::vector<T>& v, T** out) {
  const auto t0 = std::chrono::steady_clock::now();
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(T)));
  (c->in_priv ? c->priv_allocs : c->allocs).push_back(p);
  if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (T*)p;
  ++g_upload_n;
  g_upload_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

static int tpi_for_bits(size_t need_bits, int min_tpi) {
  for (int t : {1, 2, 4, 8})
    if (t >= min_tpi && (size_t)LB * L * t >= need_bits) return t;
  return 0;
}

// left-to-right sliding window (k = 5) over the fixed public exponent n
static void sliding_schedule(const HBig& e, std::vector<uint16_t>& ops, int& first) {
  const int K = 5;
  int i = (int)e.bits() - 1;
  auto window = [&](int hi, int& lo, uint32_t& val) {
    lo = std::max(hi - K + 1, 0);
    while (!e.bit(lo)) ++lo;
    val = 0;
    for (int b = hi; b >= lo; --b) val = (val << 1) | (uint32_t)e.bit(b);
  };
  int lo;
  uint32_t v;
  window(i, lo, v);
  first = (int)(v - 1) / 2;
  i = lo - 1;
  int nsq = 0;
  while (i >= 0) {
    if (!e.bit(i)) {
      ++nsq;
      --i;
      continue;
    }
    window(i, lo, v);
    nsq += i - lo + 1;
    ops.push_back((uint16_t)nsq);
    ops.push_back((uint16_t)((v - 1) / 2));
    nsq = 0;
    i = lo - 1;
  }
  if (nsq) {
    ops.push_back((uint16_t)nsq);
    ops.push_back(0xFFFF);
  }
}

// Op list for run_program: x~ = x R (the caller puts R^2 in the slot), odd powers x~^(2k+1) into
// tiles k = 0..15, then the left-to-right sliding-window chain over e. The kernel appends the final
// product with tile T_FINAL.
static bool build_modexp_program(const HBig& e, std::vector<uint32_t>& prog) {
  std::vector<uint16_t> sched;
  int first = 0;
  sliding_schedule(e, sched, first);
  auto op = [](uint32_t flags, int bidx, int aidx, int sidx) {
    return flags | ((uint32_t)bidx << 8) | ((uint32_t)aidx << 16) | ((uint32_t)sidx << 24);
  };
  prog.clear();
  prog.push_back(op(OP_STORE, 0, 0, 0));                                  // x~ = x R        -> T0
  prog.push_back(op(OP_B_FROM_A, 0, 0, 0));                               // x~^2
  prog.push_back(op(OP_B_FROM_A | OP_A_FROM_T | OP_STORE, 0, 0, 1));      // x~^3           -> T1
  for (int k = 2; k < TABLE_ODD; ++k) prog.push_back(op(OP_STORE, 0, 0, k));   // x~^(2k+1) -> Tk
  bool loaded = false;   // accumulator still to be taken from tile `first`
  for (size_t i = 0; i + 1 < sched.size(); i += 2) {
    const int nsq = sched[i], idx = sched[i + 1];
    for (int t = 0; t < nsq; ++t) {
      prog.push_back(loaded ? op(OP_B_FROM_A, 0, 0, 0) : op(OP_B_FROM_T | OP_A_FROM_T, first, first, 0));
      loaded = true;
    }
    if (idx != 0xFFFF) {
      prog.push_back(loaded ? op(OP_B_FROM_A | OP_A_FROM_T, 0, idx, 0) : op(OP_B_FROM_T | OP_A_FROM_T, first, idx, 0));
      loaded = true;
    }
  }
  return loaded;   // false only for single-window exponents, which n (odd, >= 64 bits) never is
}

// Op list for run_lane_program (kernels_crt.hpp): the kernel stores x~ in tile 0; odd powers into
// tiles 0..15 (x~^2 kept as the LDS multiplier), then the sliding-window chain over e.
static bool build_lane_program(const HBig& e, std::vector<uint32_t>& prog) {
  if (e.bits() < 8) return false;
  std::vector<uint16_t> sched;
  int first = 0;
  sliding_schedule(e, sched, first);
  auto op = [](uint32_t flags, int bidx, int aidx, int sidx) {
    return flags | ((uint32_t)bidx << 8) | ((uint32_t)aidx << 16) | ((uint32_t)sidx << 24);
  };
  prog.clear();
  prog.push_back(op(LOP_SQR | LOP_B_SET, 0, 0, 0));                       // x~^2 -> LDS multiplier
  prog.push_back(op(LOP_A_FROM_T | LOP_B_READY | LOP_STORE, 0, 0, 1));    // x~ * x~^2  -> T1
  for (int k = 2; k < 16; ++k) prog.push_back(op(LOP_STORE | LOP_B_READY, 0, 0, k));   // multiplier x~^2 kept
  bool loaded = false;
  size_t first_sq = SIZE_MAX;   // first squaring since the last multiply (prefetch slot)
  for (size_t i = 0; i + 1 < sched.size(); i += 2) {
    const int nsq = sched[i], idx = sched[i + 1];
    for (int t = 0; t < nsq; ++t) {
      if (first_sq == SIZE_MAX) first_sq = prog.size();
      prog.push_back(loaded ? op(LOP_SQR, 0, 0, 0) : op(LOP_SQR | LOP_A_FROM_T, 0, first, 0));
      loaded = true;
    }
    if (idx != 0xFFFF) {
      if (first_sq != SIZE_MAX) {
        prog[first_sq] |= LOP_PREFETCH | ((uint32_t)idx << 8);
        prog.push_back(op(LOP_B_READY, idx, 0, 0));
      } else {
        prog.push_back(loaded ? op(0, idx, 0, 0) : op(LOP_A_FROM_T, idx, first, 0));
      }
      loaded = true;
      first_sq = SIZE_MAX;
    }
  }
  return loaded;
}

// K_t: for each table entry t, the sum over the chain's multiplies by it of 2^(squares after that multiply)
static std::vector<HBig> chain_weights(const HBig& ph, const std::vector<uint16_t>& sched) {
  std::vector<HBig> K(LANE_NTILE, HBig(0));
  size_t after = 0;
  for (size_t i = sched.size(); i >= 2; i -= 2) {
    const int nsq = sched[i - 2], idx = sched[i - 1];
    if (idx != 0xFFFF) K[idx] = mod(add(K[idx], mul_pow2_mod(HBig(1), after, ph)), ph);
    after += (size_t)nsq;
  }
  return K;
}

// Op list of the factored 1024/2048-bit decryption (decf_run, kernels_pair.hpp; tools/decf_model.py): the table of
// full pairs as build_lane_program (x~^2 general, kept in the column; odd powers into tiles 0..15), the chain over
// e = p_h - 2 with B-free multipliers (LOP_BFREE), then Y' (A~, 0) (iota put into the column before it) and the
// product with (1, 0). kf: the closing Horner sum's K'_t = R (K_t + [t == 0]) mod p_h, S limbs each (entry 1's
// weight + 1: the closing (A~, 0) drops its (1 + p b_1)).
static bool build_decf_lane_program(const HBig& ph, size_t RS, int S, std::vector<uint32_t>& prog, std::vector<uint32_t>& kf) {
  const HBig e = sub(ph, HBig(2));
  if (e.bits() < 8) return false;
  std::vector<uint16_t> sched;
  int first = 0;
  sliding_schedule(e, sched, first);
  auto op = [](uint32_t flags, int bidx, int aidx, int sidx) {
    return flags | ((uint32_t)bidx << 8) | ((uint32_t)aidx << 16) | ((uint32_t)sidx << 24);
  };
  prog.clear();
  prog.push_back(op(LOP_SQR | LOP_B_SET, 0, 0, 0));                       // x~^2 -> LDS multiplier
  prog.push_back(op(LOP_A_FROM_T | LOP_B_READY | LOP_STORE, 0, 0, 1));    // x~ * x~^2  -> T1
  for (int k = 2; k < LANE_NTILE; ++k) prog.push_back(op(LOP_STORE | LOP_B_READY, 0, 0, k));
  bool loaded = false;
  size_t first_sq = SIZE_MAX;
  for (size_t i = 0; i + 1 < sched.size(); i += 2) {
    const int nsq = sched[i], idx = sched[i + 1];
    for (int t = 0; t < nsq; ++t) {
      if (first_sq == SIZE_MAX) first_sq = prog.size();
      prog.push_back(loaded ? op(LOP_SQR, 0, 0, 0) : op(LOP_SQR | LOP_A_FROM_T, 0, first, 0));
      loaded = true;
    }
    if (idx != 0xFFFF) {
      if (first_sq != SIZE_MAX) {
        prog[first_sq] |= LOP_PREFETCH | ((uint32_t)idx << 8);
        prog.push_back(op(LOP_B_READY | LOP_BFREE, idx, 0, 0));
      } else {
        prog.push_back(loaded ? op(LOP_BFREE, idx, 0, 0) : op(LOP_A_FROM_T | LOP_BFREE, idx, first, 0));
      }
      loaded = true;
      first_sq = SIZE_MAX;
    }
  }
  if (!loaded) return false;
  prog.push_back(op(LOP_IOTA | LOP_BFREE, 0, 0, 0));      // Z = Y' (A~, 0), iota = Y' mod p -> the column
  prog.push_back(op(LOP_B_CONST | LOP_BFREE, 0, 0, 0));   // (1 + p G) = Z (1, 0)
  std::vector<HBig> K = chain_weights(ph, sched);
  K[0] = mod(add(K[0], HBig(1)), ph);
  kf.clear();
  for (int t = 0; t < LANE_NTILE; ++t) {
    const std::vector<uint32_t> l = mul_pow2_mod(K[t], RS, ph).limbs(S, LB);
    kf.insert(kf.end(), l.begin(), l.end());
  }
  return true;
}

// Op list of the factored public-key chain (d4f_run<S, true>, kernels_pe.hpp k_pe_pow_f): the table's 30 one-pass
// products by the kept (A_r, 0) (odd powers into tiles 0..15, tile 0 = (A_r, 0)), the sliding-window chain over n with
// B-free multipliers, then the product with (1, 0) into tile D4F_G. kf: K'_t = R K_t mod n (entry 1 is B-free: H_1 = 0).
static bool build_pef_program(const HBig& n, size_t RS, std::vector<uint32_t>& prog, std::vector<uint32_t>& kf) {
  if (n.bits() < 8) return false;
  std::vector<uint16_t> sched;
  int first = 0;
  sliding_schedule(n, sched, first);
  auto op = [](uint32_t flags, int bidx, int aidx, int sidx) {
    return flags | ((uint32_t)bidx << 8) | ((uint32_t)aidx << 16) | ((uint32_t)sidx << 24);
  };
  prog.clear();
  for (int t = 2; t < 2 * LANE_NTILE; ++t) prog.push_back(op(LOP_B_READY | ((t & 1) ? LOP_STORE : 0u), 0, 0, (t - 1) / 2));
  bool loaded = false;
  size_t first_sq = SIZE_MAX;
  for (size_t i = 0; i + 1 < sched.size(); i += 2) {
    const int nsq = sched[i], idx = sched[i + 1];
    for (int t = 0; t < nsq; ++t) {
      if (first_sq == SIZE_MAX) first_sq = prog.size();
      prog.push_back(loaded ? op(LOP_SQR, 0, 0, 0) : op(LOP_SQR | LOP_A_FROM_T, 0, first, 0));
      loaded = true;
    }
    if (idx != 0xFFFF) {
      if (first_sq != SIZE_MAX) {
        prog[first_sq] |= LOP_PREFETCH | ((uint32_t)idx << 8);
        prog.push_back(op(LOP_B_READY, idx, 0, 0));
      } else {
        prog.push_back(loaded ? op(0, idx, 0, 0) : op(LOP_A_FROM_T, idx, first, 0));
      }
      loaded = true;
      first_sq = SIZE_MAX;
    }
  }
  if (!loaded) return false;
  prog.push_back(op(LOP_B_CONST | LOP_STORE, 0, 0, D4F_G));   // Z = Y' (1, 0)
  const std::vector<HBig> K = chain_weights(n, sched);
  kf.clear();
  for (int t = 0; t < LANE_NTILE; ++t) {
    const std::vector<uint32_t> l = mul_pow2_mod(K[t], RS, n).limbs(D4_S, LB);
    kf.insert(kf.end(), l.begin(), l.end());
  }
  return true;
}

// Op list of the factored 4096-bit decryption (d4f_run, kernels_dec4.hpp): the table's 30 one-pass products by the
// kept (A~, 0) (odd powers stored in tiles 0..15), the sliding-window chain over e = p_h - 2 with B-free multipliers,
// then Y' (A~, 0) (iota taken before it) and the product with (1, 0) into tile D4F_G. kf gets the closing sum's
// constants: K'_t = R sum over the chain's multiplies by entry t of 2^(squares after it) mod p_h, slot 0 = -R mod
// p_h (entry 1 is B-free, its slot carries the ciphertext's B_c term). tools/dec4f_model.py restates the algebra.
static bool build_dec4f_program(const HBig& ph, size_t RS, std::vector<uint32_t>& prog, std::vector<uint32_t>& kf) {
  const HBig e = sub(ph, HBig(2));
  if (e.bits() < 8) return false;
  std::vector<uint16_t> sched;
  int first = 0;
  sliding_schedule(e, sched, first);
  auto op = [](uint32_t flags, int bidx, int aidx, int sidx) {
    return flags | ((uint32_t)bidx << 8) | ((uint32_t)aidx << 16) | ((uint32_t)sidx << 24);
  };
  prog.clear();
  for (int t = 2; t < 2 * LANE_NTILE; ++t) prog.push_back(op(LOP_B_READY | ((t & 1) ? LOP_STORE : 0u), 0, 0, (t - 1) / 2));
  bool loaded = false;
  size_t first_sq = SIZE_MAX;
  for (size_t i = 0; i + 1 < sched.size(); i += 2) {
    const int nsq = sched[i], idx = sched[i + 1];
    for (int t = 0; t < nsq; ++t) {
      if (first_sq == SIZE_MAX) first_sq = prog.size();
      prog.push_back(loaded ? op(LOP_SQR, 0, 0, 0) : op(LOP_SQR | LOP_A_FROM_T, 0, first, 0));
      loaded = true;
    }
    if (idx != 0xFFFF) {
      if (first_sq != SIZE_MAX) {
        prog[first_sq] |= LOP_PREFETCH | ((uint32_t)idx << 8);
        prog.push_back(op(LOP_B_READY, idx, 0, 0));
      } else {
        prog.push_back(loaded ? op(0, idx, 0, 0) : op(LOP_A_FROM_T, idx, first, 0));
      }
      loaded = true;
      first_sq = SIZE_MAX;
    }
  }
  if (!loaded) return false;
  prog.push_back(op(LOP_IOTA, 0, 0, 0));                      // Z = Y' (A~, 0), A~ = tile 0's even component
  prog.push_back(op(LOP_B_CONST | LOP_STORE, 0, 0, D4F_G));   // (1 + p G) = Z (1, 0)
  const std::vector<HBig> K = chain_weights(ph, sched);
  kf.clear();
  for (int t = 0; t < LANE_NTILE; ++t) {
    const HBig v = t == 0 ? sub(ph, mul_pow2_mod(HBig(1), RS, ph)) : mul_pow2_mod(K[t], RS, ph);
    const std::vector<uint32_t> l = v.limbs(D4_S, LB);
    kf.insert(kf.end(), l.begin(), l.end());
  }
  return true;
}

template <typename K>
static int grid_for(pai_ctx* c, K kernel, size_t lds, long long units, int per_block) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, BLOCK, lds) != hipSuccess || occ < 1) occ = 1;
  long long want = (units + per_block - 1) / per_block;
  long long cap = (long long)occ * c->cus;
  return (int)std::max<long long>(1, std::min(want, cap));
}

static int ensure_scratch(pai_ctx* c, size_t bytes) {
  if (bytes <= c->scratch_bytes) return 0;
  if (c->d_scratch) HIPCHK(hipFree(c->d_scratch));
  c->d_scratch = nullptr;
  c->scratch_bytes = 0;
  HIPCHK(hipMalloc(&c->d_scratch, bytes));
  c->scratch_bytes = bytes;
  return 0;
}

static size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

// hipMalloc that, when the device is full, first hands the released tables' pooled chunks (table_arena.hpp) back to the
// driver and tries again: pooled memory serves table rebuilds, never at the expense of a call's working buffers
static hipError_t dev_malloc(void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory && TableArena::get().pooled_any()) {
    (void)hipGetLastError();
    TableArena::get().trim();
    e = hipMalloc(p, bytes);
  }
  return e;
}

static int ensure_buf(void** buf, size_t* have, size_t bytes) {
  if (bytes <= *have) return 0;
  if (*buf) HIPCHK(hipFree(*buf));
  *buf = nullptr;
  *have = 0;
  HIPCHK(dev_malloc(buf, bytes));
  *have = bytes;
  return 0;
}

static int ensure_work(pai_ctx* c, size_t bytes) {
  if (bytes <= c->work_bytes) return 0;
  if (c->d_work) HIPCHK(hipFree(c->d_work));
  c->d_work = nullptr;
  c->work_bytes = 0;
  HIPCHK(dev_malloc(&c->d_work, bytes));
  c->work_bytes = bytes;
  return 0;
}

static void stage_reset(pai_ctx* c) {
  if (c->stage_keep) return;   // inside a host-buffer call: its entry point reset once for all chunks
  c->nev = 0;
  c->nchunk_ev = 0;
}
// The events of a new chunk (nullptr when timing is off). The event table grows with the chunks of a call and is
// read only by pai_ctx_stage_times: recording a stage never waits on the device (folding the slots of a
// long call synchronised mid-call and removed the copy/compute overlap being timed).
static hipEvent_t* stage_chunk(pai_ctx* c) {
  if (!c->timing) return nullptr;
  if (c->nchunk_ev >= (int)c->ev.size()) c->ev.push_back({nullptr, nullptr, nullptr, nullptr});
  hipEvent_t* e = c->ev[c->nchunk_ev++].data();
  for (int i = 0; i < 4; ++i)
    if (!e[i]) (void)hipEventCreate(&e[i]);
  return e;
}
// mark i (0..3) of the current chunk; mark 0 opens a new chunk
static void stage_mark(pai_ctx* c, int i, hipStream_t st) {
  if (!c->timing || i >= 4) return;
  if (i == 0 && !stage_chunk(c)) return;
  if (c->nchunk_ev == 0) return;
  (void)hipEventRecord(c->ev[c->nchunk_ev - 1][i], st);
  c->nev = std::max(c->nev, i + 1);
}

template <typename K>
static int blocks_per_cu(K kernel, int threads, size_t lds) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds) != hipSuccess || occ < 1) occ = 1;
  return occ;
}

// C-linkage comes from the declarations in flexpai.h.
const char* pai_last_error(void) { return g_last_error.c_str(); }

namespace fpai {
int set_error(int code, const char* msg) { return fail(code, msg); }   // for the other translation units
}

int pai_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes) {
  HIPCHK(hipSetDevice(device));
  size_t fr = 0, tot = 0;
  HIPCHK(hipMemGetInfo(&fr, &tot));
  if (free_bytes) *free_bytes = fr;
  if (total_bytes) *total_bytes = tot;
  return 0;
}

int pai_device_count(int* count) {
  if (!count) return fail(PAI_ERR_ARG, "null argument");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  *count = n;
  return 0;
}

static int setup_pe(pai_ctx* c, const HBig& n);
static int setup_pe1(pai_ctx* c, const HBig& n);

int pai_ctx_create(const uint8_t* n_le, size_t n_bytes, int device, pai_ctx** out) {
  if (!n_le || !out || n_bytes == 0) return fail(PAI_ERR_ARG, "pai_ctx_create: null argument");
  SetupTrace tr("pai_ctx_create");
  HBig n = HBig::from_le_bytes(n_le, n_bytes);
  if (!n.is_odd() || n.bits() < 64) return fail(PAI_ERR_KEY, "pai_ctx_create: n must be odd and >= 64 bits");
  auto* c = new pai_ctx();
  c->device = device;
  c->counted = true;
  ++g_contexts;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return fail(PAI_ERR_HIP, "pai_ctx_create: hipSetDevice failed");
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    delete c;
    return fail(PAI_ERR_HIP, "pai_ctx_create: hipGetDeviceProperties failed");
  }
  c->cus = prop.multiProcessorCount;
  c->n = n;
  c->nb = (int)n.bits();
  c->N = mul(n, n);
  c->tpi_e = tpi_for_bits(2 * (size_t)c->nb + 2, 2);
  c->tpi_d = tpi_for_bits((size_t)c->nb + 3, 1);
  if (!c->tpi_e || !c->tpi_d) {
    delete c;
    return fail(PAI_ERR_KEY, "pai_ctx_create: key size not supported (max 4096 bits)");
  }
  c->S_e = L * c->tpi_e;
  c->S_d = L * c->tpi_d;
  c->ct_words = (2 * c->nb + 31) / 32;
  c->pt_words = (c->nb + 31) / 32;
  c->mprime_N = mont_prime(c->N, LB);
  const size_t Rbits = (size_t)LB * c->S_e;
  HBig R2 = mul_pow2_mod(HBig(1), 2 * Rbits, c->N);
  std::vector<uint32_t> prog;
  if (!build_modexp_program(n, prog)) {
    delete c;
    return fail(PAI_ERR_KEY, "pai_ctx_create: degenerate exponent schedule");
  }
  c->nprog = (int)prog.size();
  HBig oneR = mul_pow2_mod(HBig(1), Rbits, c->N);
  std::vector<uint32_t> rs;
  {
    HMont M(c->N);
    HBig x(1);
    for (int s = 0; s <= ADD_KMAX + 1; ++s) {
      const std::vector<uint32_t> v = x.words(c->ct_words);
      rs.insert(rs.end(), v.begin(), v.end());
      x = M.mul(M.mul(x, oneR), M.r2);   // x R mod N
    }
  }
  int rc;
  if ((rc = upload(c, rs, &c->d_RS)) || (rc = upload(c, c->N.limbs(c->S_e, LB), &c->d_N)) ||
      (rc = upload(c, R2.limbs(c->S_e, LB), &c->d_R2)) ||
      (rc = upload(c, n.limbs(c->S_e, LB), &c->d_nl)) || (rc = upload(c, prog, &c->d_prog)) ||
      (rc = upload(c, oneR.limbs(c->S_e, LB), &c->d_oneR)) || (rc = (SetupTrace("  setup_pe"), setup_pe(c, n))) ||
      (rc = setup_pe1(c, n))) {
    delete c;
    return rc;
  }
  if (c->S_e == 74 || c->S_e == 148 || c->S_e == 296) {   // public-key encryption of protocol-sized calls on rows (k_pe_w)
    std::vector<uint32_t> pw;
    if (build_lane_program(n, pw)) {
      if ((rc = upload(c, pw, &c->d_pew_prog))) {
        delete c;
        return rc;
      }
      c->pew_nprog = (int)pw.size();
    }
  }
#if FLEXPAI_XCHECK
  if (hipMalloc(&c->d_guard, sizeof(GuardRec)) != hipSuccess || hipMemset(c->d_guard, 0, sizeof(GuardRec)) != hipSuccess) {
    delete c;
    return fail(PAI_ERR_HIP, "pai_ctx_create: guard record");
  }
#endif
  *out = c;
  return 0;
}

// The test build's address guards (guard.hpp): the sizes the samplers' indices must stay below, as allocated here.
// $FLEXPAI_GUARD_INJECT=rows (test build only) passes a table of one row, so that every row index trips the guard:
// the self-test of the mechanism (tests/test_gpu_guard.py).
static GuardArgs guard_args(const pai_ctx* c, unsigned long long rows, unsigned long long digits, unsigned long long out,
                            unsigned long long in) {
  const char* inj = xcheck_env("FLEXPAI_GUARD_INJECT");
  if (inj && std::strcmp(inj, "rows") == 0) rows = 1;
  return GuardArgs{c->d_guard, rows, digits, out, in};
}
// after the guarded launches of a call: a violation fails the call with the first one's site, value and limit
static int guard_collect(pai_ctx* c, hipStream_t st) {
  if (!c->d_guard) return 0;
  HIPCHK(hipStreamSynchronize(st));
  GuardRec g{};
  HIPCHK(hipMemcpy(&g, c->d_guard, sizeof(g), hipMemcpyDeviceToHost));
  if (!g.hits) return 0;
  HIPCHK(hipMemset(c->d_guard, 0, sizeof(GuardRec)));
  return fail(PAI_ERR_HIP, std::string("address guard: ") + std::to_string(g.hits) + " violation(s), first at " +
                               guard_site_name(g.site) + ": index " + std::to_string(g.val) + " >= limit " +
                               std::to_string(g.lim) + " (element " + std::to_string(g.elem) + ")");
}

// Fixed-base obfuscation setup (kernels_fb.hpp): the smallest g >= 2 that generates Z_P* as far as
// the prime factors of P - 1 below 2^24 can tell (g^((P-1)/l) != 1 for each); a prime factor l of
// P - 1 above the bound that g misses has probability about 1/l < 2^-24. G = g^n mod P^2.
constexpr uint32_t FB_TRIAL_BOUND = 1u << 24;   // = oracle/paillier_oracle.py FB_TRIAL_BOUND

// The primes below FB_TRIAL_BOUND in chunks of 4096 with each chunk's product (a product tree on GMP), built once
// per process: the small prime factors of P - 1 are then found chunk by chunk as gcd(prod_j mod (P - 1), P - 1)
// (~0.3 k GMP operations per key instead of 1.08 M single-precision remainders: 66 -> a few ms per half, round 5).
struct PrimeChunks {
  std::vector<uint32_t> primes;
  std::vector<size_t> start;                  // chunk j = primes[start[j] .. start[j + 1])
  std::vector<std::unique_ptr<Mpz>> prod;
};
static void prime_product(const std::vector<uint32_t>& pr, size_t lo, size_t hi, mpz_t out) {
  if (hi - lo <= 16) {
    mpz_set_ui(out, 1);
    for (size_t i = lo; i < hi; ++i) mpz_mul_ui(out, out, pr[i]);
    return;
  }
  const size_t mid = (lo + hi) / 2;
  Mpz a, b;
  prime_product(pr, lo, mid, a.v);
  prime_product(pr, mid, hi, b.v);
  mpz_mul(out, a.v, b.v);
}
static const PrimeChunks& prime_chunks() {
  static const PrimeChunks pc = [] {
    PrimeChunks c;
    c.primes = small_primes(FB_TRIAL_BOUND);
    constexpr size_t CH = 4096;
    for (size_t s = 0; s < c.primes.size(); s += CH) {
      c.start.push_back(s);
      c.prod.emplace_back(new Mpz());
      prime_product(c.primes, s, std::min(s + CH, c.primes.size()), c.prod.back()->v);
    }
    c.start.push_back(c.primes.size());
    return c;
  }();
  return pc;
}

static uint32_t fb_base(const HBig& P) {
  const PrimeChunks& pc = prime_chunks();
  Mpz p(P), pm1, t, g;
  mpz_sub_ui(pm1.v, p.v, 1);
  std::vector<uint32_t> fac;
  for (size_t j = 0; j < pc.prod.size(); ++j) {
    mpz_mod(t.v, pc.prod[j]->v, pm1.v);
    mpz_gcd(g.v, t.v, pm1.v);
    if (mpz_cmp_ui(g.v, 1) == 0) continue;
    for (size_t i = pc.start[j]; i < pc.start[j + 1]; ++i)
      if (mpz_divisible_ui_p(g.v, pc.primes[i])) fac.push_back(pc.primes[i]);
  }
  std::vector<std::unique_ptr<Mpz>> cof;
  for (uint32_t l : fac) {
    cof.emplace_back(new Mpz());
    mpz_divexact_ui(cof.back()->v, pm1.v, l);
  }
  Mpz gb, r;
  for (uint32_t cand = 2; cand < 1000000u; ++cand) {
    bool ok = true;
    for (size_t k = 0; k < fac.size() && ok; ++k) {
      if (fac[k] == 2) {   // g^((P-1)/2) == 1 iff g is a square mod P (Euler's criterion)
        mpz_set_ui(gb.v, cand);
        ok = mpz_jacobi(gb.v, p.v) != 1;
      } else {
        mpz_set_ui(gb.v, cand);
        mpz_powm(r.v, gb.v, cof[k]->v, p.v);
        ok = mpz_cmp_ui(r.v, 1) != 0;
      }
    }
    if (ok) return cand;
  }
  return 0;
}


// Public-key encryption on split pairs (kernels_pe.hpp) for n of 1537..2048 bits: S = 74 limbs of n, R =
// 2^(28 S) >= 2^24 n. Constants: n, (1 - R) and (1 - R^2) mod n, the pair of R^3 mod n^2, the op list for n.
static int setup_pe(pai_ctx* c, const HBig& n) {
  bool pair = true;
  if (const char* e = xcheck_env("FLEXPAI_PAIR")) pair = atoi(e) != 0;
  const size_t RS = (size_t)LB * D4_S;
  if (!pair || n.bits() + 24 > RS || n.bits() <= 1536) return 0;
  std::vector<uint32_t> prog;
  if (!build_lane_program(n, prog)) return 0;
  const HBig n2 = mul(n, n);
  auto one_minus = [&](const HBig& r) { return mod(sub(add(n, HBig(1)), r), n); };   // (1 - r) mod n, 0 < r < n
  const HBig r3 = mul_pow2_mod(HBig(1), 3 * RS, n2);
  const HBig qt = div_big(r3, n), rm = sub(r3, mul(qt, n));
  std::vector<uint32_t> ck = rm.limbs(D4_S, LB), b = qt.limbs(D4_S, LB);
  ck.insert(ck.end(), b.begin(), b.end());
  uint32_t *dn, *dx1, *dxk, *dck, *dprog;
  int rc;
  if ((rc = upload(c, n.limbs(D4_S, LB), &dn)) ||
      (rc = upload(c, one_minus(mul_pow2_mod(HBig(1), RS, n)).limbs(D4_S, LB), &dx1)) ||
      (rc = upload(c, one_minus(mul_pow2_mod(HBig(1), 2 * RS, n)).limbs(D4_S, LB), &dxk)) ||
      (rc = upload(c, ck, &dck)) || (rc = upload(c, prog, &dprog)))
    return rc;
  std::vector<PeConst> pc{PeConst{dn, dx1, dxk, dck, dprog, (int)prog.size(), mont_prime(n, LB)}};
  // the factored chain (kernels_pe.hpp k_pe_pow_f): its program and Horner weights, R^2 mod n; R mod n for the batch
  // inversion of the bases mod n on the TPI = 2 group engine (same radix R = 2^(28 74))
  std::vector<uint32_t> progf, kf;
  const bool pef = !(xcheck_env("FLEXPAI_PEF") && atoi(xcheck_env("FLEXPAI_PEF")) == 0);
  if (pef && tpi_for_bits((size_t)c->nb + 3, 1) == 2 && build_pef_program(n, RS, progf, kf)) {
    uint32_t *dpf, *dkf, *dr2, *done;
    if ((rc = upload(c, progf, &dpf)) || (rc = upload(c, kf, &dkf)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), 2 * RS, n).limbs(D4_S, LB), &dr2)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), RS, n).limbs(D4_S, LB), &done)))
      return rc;
    pc[0].progf = dpf;
    pc[0].nprogf = (int)progf.size();
    pc[0].kf = dkf;
    pc[0].r2n = dr2;
    c->d_pe_n = dn;
    c->d_pe_r2 = dr2;
    c->d_pe_oneR = done;
    c->pe_mprime = mont_prime(n, LB);
    c->pef_ok = true;
  }
  if ((rc = upload(c, pc, &c->d_pe))) return rc;
  c->pe_ok = true;
  return 0;
}

// Public-key encryption on pairs over the S = 37 limbs of n for n <= 1024 bits (kernels_pe1.hpp; R = 2^1036 >= 2^12 n):
// n, the pair of R^3 mod n^2 (r's two digit chunks, k_dec_pre_pair), the pair (1, 0), the op list over n, R^2 mod n.
static int setup_pe1(pai_ctx* c, const HBig& n) {
  bool pair = true;
  if (const char* e = xcheck_env("FLEXPAI_PAIR")) pair = atoi(e) != 0;
  const size_t RS = (size_t)LB * PE1_S;
  if (!pair || n.bits() + 12 > RS || c->ct_words > 64) return 0;
  std::vector<uint32_t> prog;
  if (!build_lane_program(n, prog)) return 0;
  const HBig n2 = mul(n, n);
  const HBig r3 = mul_pow2_mod(HBig(1), 3 * RS, n2);
  const HBig qt = div_big(r3, n), rm = sub(r3, mul(qt, n));
  std::vector<uint32_t> ck = rm.limbs(PE1_S, LB), b = qt.limbs(PE1_S, LB), one(2 * PE1_S, 0);
  ck.insert(ck.end(), b.begin(), b.end());
  one[0] = 1;
  uint32_t *dn, *dck, *done, *dprog, *dr2;
  int rc;
  if ((rc = upload(c, n.limbs(PE1_S, LB), &dn)) || (rc = upload(c, ck, &dck)) || (rc = upload(c, one, &done)) ||
      (rc = upload(c, prog, &dprog)) || (rc = upload(c, mul_pow2_mod(HBig(1), 2 * RS, n).limbs(PE1_S, LB), &dr2)))
    return rc;
  const uint32_t mp = mont_prime(n, LB);
  std::vector<DecPairHalf> h{DecPairHalf{dn, dck, nullptr, nullptr, mp, 0u}};
  if ((rc = upload(c, h, &c->d_pe1_half))) return rc;
  c->d_pe1_n = dn;
  c->d_pe1_one = done;
  c->d_pe1_prog = dprog;
  c->pe1_nprog = (int)prog.size();
  c->d_pe1_r2n = dr2;
  c->pe1_mprime = mp;
  c->pe1_ok = true;
  return 0;
}

template <typename T>
static int upload_fb(pai_ctx* c, const std::vector<T>& v, T** out) {
  const auto t0 = std::chrono::steady_clock::now();
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(T)));
  c->fb_mem.push_back(p);
  if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (T*)p;
  ++g_upload_n;
  g_upload_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

// Split-pair sampler (kernels_sgp.hpp) over the pair-group tables of modulus P (rows T R, R = 2^(28 FBGP_S)): C =
// 2^(-56 K) mod P^2 as (C mod P, C div P), the chunk weights w 2^(16 c) C_A mod P of c0 = (1, w |M|), and 2^20 P.
// FLEXPAI_SGP=0 keeps the group-engine samplers (k_fbgp, k_pfb).
static bool sgp_enabled() {
  const char* e = xcheck_env("FLEXPAI_SGP");
  return !e || atoi(e) != 0;
}
// Shoup rows for the 4096-bit key holder's split-pair sampler (kernels_sgs.hpp). Their 640-B rows sit beside the
// factored rows (whose b halves they keep using): 1152 B per entry against 512, so they fit one window lower (W = 20
// at nb = 4096 on a 288-GB device, 249 GB, against the factored rows' W = 21, 205 GB). fb_choose takes them when the
// product count at their window, priced at the measured 0.835 of a Montgomery row product
// (profiles/r05_ab_sgs_prototype_stream.txt), is below the factored rows' at theirs. $FLEXPAI_SGS=0 never takes them,
// $FLEXPAI_SGS=1 whenever they fit.
static int sgs_mode() {
  const char* e = getenv("FLEXPAI_SGS");
  return !e || !*e ? -1 : atoi(e) != 0 ? 1 : 0;
}
// Garner's last step on lanes (k_sgp_fin); the test build's $FLEXPAI_SGP_FIN=0 keeps the group kernel k_fbg_fin
static bool sgp_fin_enabled() {
  const char* e = xcheck_env("FLEXPAI_SGP_FIN");
  return !e || atoi(e) != 0;
}

template <class Upload>
static int sgp_make_half(const HBig& P, const HBig& w, int K, const void* table, Upload&& up, SgpHalf* out) {
  const HBig P2 = mul(P, P);
  const HBig C = inv_mod(mul_pow2_mod(HBig(1), (size_t)LB * (FBGP_S - SGP_S) * K, P2), P2);
  if (C.is_zero()) return fail(PAI_ERR_KEY, "split-pair sampler: 2 not invertible mod P^2");
  const HBig cb = div_big(C, P), ca = sub(C, mul(cb, P));
  std::vector<uint32_t> nmc;
  for (int k = 0; k < 4; ++k) {
    const std::vector<uint32_t> v = mod(mul(mul_pow2_mod(mod(w, P), (size_t)16 * k, P), ca), P).limbs(SGP_S, LB);
    nmc.insert(nmc.end(), v.begin(), v.end());
  }
  uint32_t *dp, *dca, *dcb, *dnmc, *dpb;
  int rc;
  if ((rc = up(P.limbs(SGP_S, LB), &dp)) || (rc = up(ca.limbs(SGP_S, LB), &dca)) || (rc = up(cb.limbs(SGP_S, LB), &dcb)) ||
      (rc = up(nmc, &dnmc)) || (rc = up(mul(P, pow2(20)).limbs(SGP_S, LB), &dpb)))
    return rc;
  *out = SgpHalf{(const uint4*)table, dp, dca, dcb, dnmc, dpb, mont_prime(P, LB)};
  return 0;
}

// The Shoup rows of both halves from their factored rows t[h] (kernels_sgs.hpp k_sgs_conv) and the constants of
// k_sgs_bfin: w 2^(16 c) R mod P (R = 2^(28 FBGP_S), the b rows' radix; w = the other prime) and mu = floor(2^(56 S) / P).
// The row memory at[h] was reserved before the factored tables were built (ensure_fb), so that a device without room for
// both never ends up on the factored rows at the Shoup rows' lower window. Any failure here leaves the Montgomery sampler
// k_sgp in place over the complete factored tables (returns nonzero with the reason in pai_last_error; the caller frees
// at[] and keeps the fixed-base path).
template <class Ctx>
static int sgs_build(Ctx* c, const HBig* primes, int K, int W, void* const* t, const SgpHalf* sv, uint4* const* at) {
  SgsHalf sh[2];
  const size_t rows = (size_t)K << W;
  for (int h = 0; h < 2; ++h) {
    const HBig& P = primes[h];
    std::vector<uint32_t> nmr;
    for (int k = 0; k < 4; ++k) {
      const std::vector<uint32_t> v = mul_pow2_mod(mod(primes[1 - h], P), (size_t)16 * k + (size_t)LB * FBGP_S, P).limbs(SGP_S, LB);
      nmr.insert(nmr.end(), v.begin(), v.end());
    }
    const HBig mu = div_big(pow2((size_t)2 * LB * SGP_S), P);
    if (mu.bits() > (size_t)LB * (SGP_S + 1)) return fail(PAI_ERR_KEY, "Shoup rows: mu exceeds S + 1 limbs");
    // R^-K mod P^2 = c_A (1 + P beta): the rows' Montgomery factor R = 2^(28 FBGP_S), once per row product
    const HBig P2 = mul(P, P);
    const HBig Ci = inv_mod(mul_pow2_mod(HBig(1), (size_t)LB * FBGP_S * K, P2), P2);
    if (Ci.is_zero()) return fail(PAI_ERR_KEY, "Shoup rows: 2 not invertible mod P^2");
    const HBig cB = div_big(Ci, P), cA = sub(Ci, mul(cB, P));
    const HBig cAi = inv_mod(cA, P);
    if (cAi.is_zero()) return fail(PAI_ERR_KEY, "Shoup rows: c_A not invertible");
    // the pass multiplies by the integer y = c_A R' mod P, and y R'^-1 = c_A (1 + P delta)^-1 mod P^2 with Y = c_A R'
    // mod P^2 = y (1 + P delta): delta joins the b sum with beta
    const HBig Y = mul_pow2_mod(cA, (size_t)LB * SGP_S, P2);
    const HBig yB = div_big(Y, P), y = sub(Y, mul(yB, P));
    const HBig yi = inv_mod(y, P);
    if (yi.is_zero()) return fail(PAI_ERR_KEY, "Shoup rows: y not invertible");
    const HBig delta = mod(mul(yB, yi), P);
    const HBig beta = mod(add(mul(cB, cAi), delta), P);
    uint32_t *dn, *dmu, *dcy, *dbr;
    int rc;
    if ((rc = upload_fb(c, nmr, &dn)) || (rc = upload_fb(c, mu.limbs(SGP_S + 2, LB), &dmu)) ||
        (rc = upload_fb(c, y.words(FBGP_PW), &dcy)) ||
        (rc = upload_fb(c, mul_pow2_mod(beta, (size_t)LB * FBGP_S, P).limbs(SGP_S, LB), &dbr)))
      return rc;
    sh[h] = SgsHalf{at[h], (const uint4*)t[h], sv[h].p, dn, sv[h].pbig, dmu, dcy, dbr, sv[h].mprime};
  }
  SgsHalf* d = nullptr;
  std::vector<SgsHalf> shv(sh, sh + 2);
  int rc;
  if ((rc = upload_fb(c, shv, &d))) return rc;
  if (sgs_launch_conv(d, rows, at[0], at[1], nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipGetLastError();
    return fail(PAI_ERR_HIP, "Shoup row conversion failed");
  }
  c->d_sgs_fb = d;
  return 0;
}

// Digit windows the table builder supports (lo/hi half-digit tables of at most FB_LO entries)
static bool fb_window_ok(int w) { return w == 8 || w == 12 || w == 16 || (w >= 20 && w <= 24); }

// g_contexts, g_key_holders (above): contexts of this process, and those holding a private key.
static bool fb_window_auto() {
  const char* e = getenv("FLEXPAI_FB_WINDOW");
  return e && strcmp(e, "auto") == 0;
}

// Window of the key holder's tables: $FLEXPAI_FB_WINDOW, default 16 (2 x 1.07 GB at nb = 2048: a process may hold
// several keys). "auto": a process whose only private key is this one asks for the largest window (24) and
// gets the largest whose tables fit auto's share of the free HBM (fb_budget), i.e. W = 22 at nb = 2048 (2 x 88.3 GB of
// 448-B Shoup rows) and W = 21 at nb = 4096 on an otherwise empty MI355X; a process holding several keys gets 16.
static int fb_default_window() {
  if (fb_window_auto()) return g_key_holders.load() <= 1 ? 24 : 16;
  const char* e = getenv("FLEXPAI_FB_WINDOW");
  const int w = e ? atoi(e) : 16;
  return fb_window_ok(w) ? w : 16;
}

// Windows of the public-key tables: the ones pinned to reference goldens (12, 16, 20; tests/golden/
// make_golden_pfb.py). Their K = K0 + 32 KS rows keep k_sgp's b sum within its bound (K <= 512; W = 8 would
// need 648). "auto": 20 for a process with one context, else 16.
static bool pfb_window_ok(int w) { return w == 12 || w == 16 || w == 20; }

static int pfb_default_window() {
  if (fb_window_auto()) return g_contexts.load() <= 1 ? 20 : 16;
  const char* e = getenv("FLEXPAI_FB_WINDOW");
  const int w = e ? atoi(e) : 16;
  return pfb_window_ok(w) ? w : w > 20 ? 20 : 16;
}

// 32-bit words of one table row: packed words for the lane kernels, S canonical limbs for the group kernel
static int fb_row_words(int sb) {
  return sb == 37 ? FbGeom<37>::TW : sb == 74 ? FbGeom<74>::TW : sb == GRP_TPI * L ? GRP_TPI * L : 0;
}

// 4096-bit keys: the pair-group sampler (kernels_grp_pair.hpp) runs when both p_h fit its 76 limbs with
// R >= 2^24 p_h; its rows are the canonical pair as 2 x 64 words
static bool fb_gpair_possible(const pai_ctx* c) {
  if (c->crt_sb != GRP_TPI * L) return false;
  for (const HBig* h : {&c->fb_p, &c->fb_q})
    if (h->bits() + 24 > (size_t)LB * FBGP_S || h->bits() > (size_t)LB * FBGP_SP || h->bits() > (size_t)32 * FBGP_PW)
      return false;
  return true;
}

static int fb_row_words(const pai_ctx* c) { return fb_gpair_possible(c) ? 4 * FBGP_ROW4 : fb_row_words(c->crt_sb); }

// 1024/2048-bit keys: the pair tables (kernels_fbp.hpp) need p_h < 2^(32 PW) and R = 2^(28 S) >= 2^12 p_h (bounds of
// the first product, kernels_fbp.hpp). Returns S (19 or 37), or 0.
static int fb_pair_possible(const pai_ctx* c) {
  const int sb = c->crt_sb;
  const int ps = sb == 37 ? 19 : sb == 74 ? 37 : 0;
  if (!ps) return 0;
  const int pw = ps == 19 ? FbpGeom<19>::PW : FbpGeom<37>::PW;
  for (const HBig* h : {&c->fb_p, &c->fb_q})
    if (h->bits() > (size_t)32 * pw || h->bits() + FBP_PB + 1 > (size_t)LB * ps) return 0;
  return ps;
}

// Shoup rows (kernels_fbs.hpp, k_fbs) on the pair path: the product's sampler for 1024/2048-bit keys. The test build
// keeps k_fbp's Montgomery rows behind $FLEXPAI_FBS=0 for the cross-checks. Shoup's a' = floor(a R / p_h) < R and
// k_fbs_fill's mu = floor(R^2 / p_h) must fit S + 1 limbs: p_h > 2^(28 (S - 1)).
static bool fb_shoup_possible(const pai_ctx* c) {
  const int ps = fb_pair_possible(c);
  if (!ps) return false;
  const char* e = xcheck_env("FLEXPAI_FBS");
  if (e && atoi(e) == 0) return false;
  for (const HBig* h : {&c->fb_p, &c->fb_q})
    if (h->bits() <= (size_t)LB * (ps - 1)) return false;
  return true;
}

// 32-bit words of one resident table row (fb_row_words is the ciphertext half's word count for the Garner
// kernels; the Shoup rows are longer: a, a', b R)
static int fb_table_row_words(const pai_ctx* c) {
  if (fb_shoup_possible(c)) return fbs_row_bytes(fb_pair_possible(c)) / 4;
  return fb_row_words(c);
}

static int fb_digit_count(const pai_ctx* c, int W) {
  const size_t kb = std::max(sub(c->fb_p, HBig(1)).bits(), sub(c->fb_q, HBig(1)).bits());
  return (int)((kb + W - 1) / W);
}

static uint64_t fb_bytes(const pai_ctx* c, int W, bool sgs = false) {
  return 2ull * (uint64_t)fb_digit_count(c, W) * (1ull << W) * ((uint64_t)fb_table_row_words(c) + (sgs ? 4ull * SGS_ROW_Q : 0ull)) *
         4ull;
}

// The window of the tables (<= c->fb_W, within budget) and whether Shoup rows join them (sgs_mode, above)
static int fb_choose(const pai_ctx* c, uint64_t budget, bool* sgs, bool allow_sgs = true) {
  static const int ladder[] = {24, 23, 22, 21, 20, 16, 12, 8};
  int wm = 0, ws = 0;
  for (int w : ladder)
    if (w <= c->fb_W && fb_bytes(c, w) <= budget) {
      wm = w;
      break;
    }
  const int mode = allow_sgs ? sgs_mode() : 0;
  if (mode != 0 && fb_gpair_possible(c) && sgp_enabled())
    for (int w : ladder)
      if (w <= c->fb_W && fb_bytes(c, w, true) <= budget) {
        ws = w;
        break;
      }
  *sgs = ws && (mode == 1 || (wm && 0.835 * fb_digit_count(c, ws) < (double)fb_digit_count(c, wm)));
  return *sgs ? ws : wm;
}

// Budget for the two tables: $FLEXPAI_FB_MAX_BYTES, else the free device memory less a reserve of
// max(4 GiB, 1/12 of the device) -- 24 GB on a 288 GB MI355X -- kept for what the context (and others in
// the process) allocate after the tables: host-pipeline buffers for larger calls, decryption work and
// scratch, k_add's schedule, a configs[3] shard with its all-gather receive buffers.
// With FLEXPAI_FB_WINDOW=auto the budget is further capped at $FLEXPAI_FB_AUTO_FRAC (default 0.75) of the free
// memory, so an automatic choice never takes the whole device (W = 22 at nb = 2048 is 177 GB of 287 GB free; W = 23's
// Shoup rows, 338 GB, do not fit).
static uint64_t fb_budget(const pai_ctx* c) {
  if (const char* e = getenv("FLEXPAI_FB_MAX_BYTES")) return (uint64_t)strtod(e, nullptr);
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
  fr += TableArena::get().pooled_bytes(c->device);   // released tables' chunks, held for reuse (table_arena.hpp)
  const uint64_t reserve = std::max<uint64_t>(4ull << 30, (uint64_t)tot / 12);
  uint64_t b = fr > reserve ? fr - reserve : 0;
  if (fb_window_auto()) {
    const char* f = getenv("FLEXPAI_FB_AUTO_FRAC");
    double frac = f ? atof(f) : 0.75;
    if (!(frac > 0.0 && frac <= 1.0)) frac = 0.75;
    b = std::min<uint64_t>(b, (uint64_t)(frac * (double)fr));
  }
  return b;
}

// Fixed-base break-even: the tables cost a one-time build (host bases + k_fb*_lohi/fill over 2 K 2^W rows,
// ~2.1 ns per 256-B row on one MI355X, profiles/r02_bench_v13.log setup) and save, per element, the
// difference between the generic path and the sampler (nb = 2048: 1/1.63 M - 1/40 M s = 0.59 us; nb = 4096
// against the public-key kernel: 1/37 k - 1/4.2 M s = 27 us; nb = 1024: ~0.08 us). A fresh key builds them
// only once the device-RNG elements of this context (this call included) reach the break-even count --
// a re-keying caller (HE_SA_FT, he_sa_ft/train.py:39-40) encrypting a few hundred elements per key never
// pays the build. $FLEXPAI_FB_MIN_ELEMS overrides the count; pai_ctx_fixed_base_prepare builds at once.
static long long fb_break_even(const pai_ctx* c, int W, int K, int row_bytes) {
  if (const char* e = getenv("FLEXPAI_FB_MIN_ELEMS")) return atoll(e);
  const double build_s = 0.05 + 2.0 * K * (double)(1ull << W) * 2.1e-9 * (row_bytes / 256.0);
  const double save_s = c->nb > 2048 ? 27e-6 : c->nb > 1024 ? 0.59e-6 : 0.08e-6;
  return (long long)(build_s / save_s) + 1;
}

static bool fb_wanted(pai_ctx* c, long long n);
static bool pfb_supported(const pai_ctx* c);
static void pfb_release(pai_ctx* c);

static void fb_release(pai_ctx* c) {
  for (void* p : c->fb_mem) (void)hipFree(p);
  c->fb_mem.clear();
  for (void* p : c->fb_tables) TableArena::get().free(p);
  c->fb_tables.clear();
  c->d_fb_halves = nullptr;
  c->d_fbp_halves = nullptr;
  c->d_fbp_fin_cs = c->d_fbp_fin_p = nullptr;
  c->fb_pair_s = 0;
  c->fb_shoup = false;
  c->d_fbs_cst = nullptr;
  c->d_fbgp_halves = nullptr;
  c->fb_gpair = false;
  c->d_sgp_fb = nullptr;
  c->d_sgs_fb = nullptr;
  c->d_fb_red = nullptr;
}

static int fb_unavailable(pai_ctx* c, const std::string& why) {
  fb_release(c);
  (void)hipGetLastError();   // clear a failed allocation / launch so later calls start clean
  c->fb_state = pai_ctx::FB_UNAVAILABLE;
  c->fb_reason = why;
  static bool warned = false;
  if (!warned && !getenv("FLEXPAI_QUIET")) {
    fprintf(stderr, "flexpai: fixed-base obfuscation unavailable (%s); encrypting through the generic CRT path\n",
            why.c_str());
    warned = true;
  }
  return 0;
}

// 28-bit limbs (device) -> HBig
static HBig from_limbs(const uint32_t* l, int nl) {
  HBig r;
  r.w.assign(((size_t)nl * LB + 31) / 32 + 2, 0);
  for (int i = 0; i < nl; ++i) {
    const size_t bit = (size_t)LB * i;
    const uint64_t v = (uint64_t)l[i] << (bit % 32);
    r.w[bit / 32] |= (uint32_t)v;
    r.w[bit / 32 + 1] |= (uint32_t)(v >> 32);
  }
  r.trim();
  return r;
}

// The host step of the factored rows' batch inversion (kernels_grp_pair.hpp): the nv chain products v_i
// (R-forms, < 2m, S limbs each at d_cval) -> v_i^-1 R_dev^2 mod m, R_dev = 2^(28 S), in place. Montgomery's
// trick over the nv values and one binary extended-Euclid inversion: m may be composite (n).
static int pair_host_invert(const HBig& m, uint32_t* d_cval, int nv, int S) {
  std::vector<uint32_t> buf((size_t)nv * S);
  HIPCHK(hipMemcpy(buf.data(), d_cval, buf.size() * 4, hipMemcpyDeviceToHost));
  HMont M(m);
  std::vector<HBig> xm(nv), pre(nv);
  for (int i = 0; i < nv; ++i) {
    HBig v = from_limbs(&buf[(size_t)i * S], S);
    while (cmp(v, m) >= 0) v = sub(v, m);
    if (v.is_zero()) return fail(PAI_ERR_KEY, "table construction: a zero chain product");
    xm[i] = M.mul(v, M.r2);                       // host Montgomery form
    pre[i] = i ? M.mul(pre[i - 1], xm[i]) : xm[i];
  }
  const HBig ti = inv_mod(M.from(pre[nv - 1]), m);
  if (ti.is_zero()) return fail(PAI_ERR_KEY, "table construction: a chain product is not invertible");
  const HBig rdm = M.mul(mul_pow2_mod(HBig(1), 2 * (size_t)LB * S, m), M.r2);   // R_dev^2, host Montgomery form
  HBig I = M.mul(ti, M.r2);
  for (int i = nv - 1; i >= 0; --i) {
    const HBig inv = i ? M.mul(I, pre[i - 1]) : I;
    if (i) I = M.mul(I, xm[i]);
    const std::vector<uint32_t> l = M.from(M.mul(inv, rdm)).limbs(S, LB);
    std::copy(l.begin(), l.end(), buf.begin() + (size_t)i * S);
  }
  HIPCHK(hipMemcpy(d_cval, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
  return 0;
}

// Builds everything the fixed-base path needs for window c->fb_W (or the largest smaller window within
// the memory budget). Returns 1 when the path is ready, 0 when it is unavailable (reason in fb_reason);
// never fails the caller.
static int ensure_fb(pai_ctx* c) {
  if (c->fb_state == pai_ctx::FB_READY) return 1;
  if (c->fb_state == pai_ctx::FB_UNAVAILABLE) return 0;
  if (!c->crt_ok && !c->fbg_ok) return fb_unavailable(c, "needs the private key and the CRT kernels");
  const int sb = c->crt_sb, TW = fb_row_words(c);
  if (!TW) return fb_unavailable(c, "key size not supported by the fixed-base kernels");
  const bool grp = sb == GRP_TPI * L;   // group-engine rows (limbs), recombined by k_crt_fin
  const HBig sq[2] = {mul(c->fb_p, c->fb_p), mul(c->fb_q, c->fb_q)};
  if (!grp && (sq[0].bits() > (size_t)32 * TW || sq[1].bits() > (size_t)32 * TW || c->ct_words != 2 * TW))
    return fb_unavailable(c, "unbalanced primes: p^2 or q^2 exceeds the table row");
  if (!c->fb_W) c->fb_W = fb_default_window();
  const uint64_t budget = fb_budget(c);
  bool sgs = false;
  int W = fb_choose(c, budget, &sgs);
  if (!W) return fb_unavailable(c, "tables do not fit the device memory budget");
  // the 4096-bit Shoup rows' memory is taken first: without room for it the tables are built at the factored rows'
  // own (higher) window instead of at the one chosen for both
  uint4* sgs_rows[2] = {nullptr, nullptr};
  if (sgs) {
    const size_t rows = (size_t)fb_digit_count(c, W) << W;
    for (int h = 0; h < 2 && sgs; ++h)
      if (!(sgs_rows[h] = (uint4*)TableArena::get().alloc(c->device, rows * SGS_ROW_Q * sizeof(uint4)))) sgs = false;
    if (!sgs) {
      for (uint4*& r : sgs_rows)
        if (r) TableArena::get().free(r), r = nullptr;
      W = fb_choose(c, fb_budget(c), &sgs, false);
      if (!W) return fb_unavailable(c, "tables do not fit the device memory budget");
      if (setup_trace_on()) fprintf(stderr, "flexpai-trace Shoup rows: no room; factored rows at W = %d\n", W);
    } else {
      for (uint4* r : sgs_rows) c->fb_tables.push_back(r);
    }
  }
  SetupTrace tr_all("ensure_fb");
  const auto t0 = std::chrono::steady_clock::now();
  const size_t kb[2] = {sub(c->fb_p, HBig(1)).bits(), sub(c->fb_q, HBig(1)).bits()};
  const int raw_bits = (int)std::max(kb[0], kb[1]) + 64;
  if ((raw_bits + 31) / 32 > FB_RAW_MAX - 2) return fb_unavailable(c, "exponent too wide");
  const int K = fb_digit_count(c, W);
  const size_t RB = (size_t)LB * sb;
  const HBig primes[2] = {c->fb_p, c->fb_q};
  // both Garner kernels take w_q < q^2 as an operand mod p^2 (k_fb_fin: w_p + 8 p^2 - w_q > 0; k_fbp_fin:
  // A_q, B_q < 2p): keys with q >= 2p encrypt on the generic CRT path
  if (cmp(primes[1], shl1(primes[0])) >= 0) return fb_unavailable(c, "q >= 2p: fixed-base Garner bounds");
  // pair products (kernels_fbp.hpp) over the S limbs of p_h (fb_pair_possible), on Shoup rows when
  // fb_shoup_possible (kernels_fbs.hpp)
  const int ps = grp ? 0 : fb_pair_possible(c);
  const bool pair_ok = ps != 0;
  const bool shoup = pair_ok && fb_shoup_possible(c);
#if FLEXPAI_XCHECK
  if (!grp && !pair_ok) return fb_unavailable(c, "key outside the pair sampler's bounds");
#else
  if (!grp && !shoup) return fb_unavailable(c, "key outside the pair sampler's bounds");
#endif
  // 4096-bit keys: pair products on lane groups of 4 x 19 limbs (kernels_grp_pair.hpp), R = 2^(28 76) >= 2^24 p_h
  const bool gpair_ok = grp && fb_gpair_possible(c);
#if FLEXPAI_XCHECK
  if (grp && !gpair_ok) return fb_unavailable(c, "key outside the pair-group sampler's bounds");
#else
  if (grp && !(gpair_ok && sgp_enabled())) return fb_unavailable(c, "key outside the split-pair sampler's bounds");
#endif
  const int lohi_limbs = pair_ok ? std::max(sb, 2 * ps) : gpair_ok ? std::max(sb, 2 * FBGP_S) : sb;
  FbgpHalf gv[2];
  SgpHalf sv[2];
  FbpHalf pv[2];
  std::vector<uint32_t> fcst_host[2];   // Shoup rows: mu = floor(R^2 / p_h) (S + 2 limbs), R^2 mod p_h (S limbs)
  FbHalf hv[2];
  FbRed red[2];
  std::memset(red, 0, sizeof(red));
  int rc;
  void* t[2] = {nullptr, nullptr};
  void* lohi[2] = {nullptr, nullptr};
  std::vector<void*> fb_scratch;   // further build scratch (freed with lohi)
  uint32_t* gcval[2] = {nullptr, nullptr};
  uint32_t* pcval[2] = {nullptr, nullptr};
  // The per-half host work that needs no device -- the generator search, G = g^n mod p_h^2 (ONE powm) and the digit
  // bases B_k by squarings in the form the resident sampler's build takes -- for both halves at once on two threads (a
  // fresh key's setup, HE_SA_FT re-keys per exchange; round 6: the pair paths had computed G and the B_k twice)
  struct HalfPrep {
    uint32_t g = 0;
    std::vector<uint32_t> bases_p;
  };
  HalfPrep hp[2];
  {
    SetupTrace tr_hp("  host prep (generator, G, B_k; both halves)");
    auto split_into = [](const HBig& v, const HBig& P, int limbs, std::vector<uint32_t>& out) {
      const HBig qt = div_big(v, P), rm = sub(v, mul(qt, P));
      const std::vector<uint32_t> a = rm.limbs(limbs, LB), b = qt.limbs(limbs, LB);
      out.insert(out.end(), a.begin(), a.end());
      out.insert(out.end(), b.begin(), b.end());
    };
    auto prep = [&](int h) {
      HalfPrep& o = hp[h];
      o.g = c->fb_g[h] ? c->fb_g[h] : fb_base(primes[h]);
      if (!o.g) return;
      const HBig& m2 = sq[h];
      HMont M2(m2);
      const HBig G = M2.to(M2.pow(HBig(o.g), c->n));
      // pair constants: (x mod p_h, x div p_h) of Montgomery-form values x = v R mod p_h^2: B_k R and B_k^(2^LO) R
      const HBig& P = primes[h];
      const int limbs = pair_ok ? ps : FBGP_S;
      const size_t RS = (size_t)LB * limbs;
      HBig y = G;
      for (int k = 0; k < K; ++k) {
        split_into(mul_pow2_mod(M2.from(y), RS, m2), P, limbs, o.bases_p);
        split_into(mul_pow2_mod(M2.from(M2.sqr_k(y, (size_t)(W / 2))), RS, m2), P, limbs, o.bases_p);
        y = M2.sqr_k(y, (size_t)W);
      }
    };
    std::thread t1(prep, 1);
    prep(0);
    t1.join();
  }
  for (int h = 0; h < 2; ++h) {
    if (!(c->fb_g[h] = hp[h].g)) return fb_unavailable(c, "no base found");
    SetupTrace tr_h("  host prep (one half)");
    const HBig& m2 = sq[h];
    const std::vector<uint32_t> bl(sb, 0u);   // FbHalf::bases: no sampler left reads them (a placeholder row)
    // c0 folding: n 2^(CB c) mod p_h^2 (c < NC) and 2^PB p_h^2 (the group kernel uses 74's geometry:
    // 16-bit chunks, PB = 20)
    std::vector<uint32_t> nm;
    const int CB = sb == 37 ? FbGeom<37>::CB : FbGeom<74>::CB, NC = sb == 37 ? FbGeom<37>::NC : FbGeom<74>::NC;
    const int PB = sb == 37 ? FbGeom<37>::PB : FbGeom<74>::PB;
    {
      const HBig nmod = mod(c->n, m2);
      for (int k = 0; k < NC; ++k) {
        const std::vector<uint32_t> v = mul_pow2_mod(nmod, (size_t)CB * k, m2).limbs(sb, LB);
        nm.insert(nm.end(), v.begin(), v.end());
      }
    }
    uint32_t *dm, *dR2, *done, *dbases, *dlohi, *dnm, *dpbig;
    if ((rc = upload_fb(c, m2.limbs(sb, LB), &dm)) ||
        (rc = upload_fb(c, mul_pow2_mod(HBig(1), 2 * RB, m2).limbs(sb, LB), &dR2)) ||
        (rc = upload_fb(c, mul_pow2_mod(HBig(1), RB, m2).limbs(sb, LB), &done)) || (rc = upload_fb(c, bl, &dbases)) ||
        (rc = upload_fb(c, nm, &dnm)) || (rc = upload_fb(c, mul(m2, pow2(PB)).limbs(sb, LB), &dpbig)))
      return fb_unavailable(c, pai_last_error());
    // lo/hi half-digit tables: build scratch only, released once the table is filled
    if (hipMalloc(&lohi[h], (size_t)K * 2 * FB_LO * lohi_limbs * 4) != hipSuccess) return fb_unavailable(c, "table allocation failed");
    c->fb_mem.push_back(lohi[h]);
    dlohi = (uint32_t*)lohi[h];
    {
      SetupTrace tr_m("  table allocation (one half)");
      if (!(t[h] = TableArena::get().alloc(c->device, ((size_t)K << W) * (fb_table_row_words(c) / 4) * sizeof(uint4))))
        return fb_unavailable(c, "table allocation failed");
    }
    c->fb_tables.push_back(t[h]);
    hv[h] = FbHalf{(const uint4*)t[h], dm, dR2, done, dbases, dlohi, dnm, dpbig, mont_prime(m2, LB)};
    if (pair_ok) {
      // pair constants: (x mod p_h, x div p_h) of Montgomery-form values x = v R mod p_h^2, R = 2^(28 S)
      const HBig& P = primes[h];
      const size_t RS = (size_t)LB * ps;
      auto split = [&](const HBig& v, std::vector<uint32_t>& out) {
        const HBig qt = div_big(v, P), rm = sub(v, mul(qt, P));
        const std::vector<uint32_t> a = rm.limbs(ps, LB), b = qt.limbs(ps, LB);
        out.insert(out.end(), a.begin(), a.end());
        out.insert(out.end(), b.begin(), b.end());
      };
      std::vector<uint32_t> one_p, nm_p;
      const std::vector<uint32_t>& bases_p = hp[h].bases_p;   // B_k R, B_k^(2^LO) R (host prep above)
      split(mul_pow2_mod(HBig(1), RS, m2), one_p);
      const HBig other = primes[1 - h];
      std::vector<uint32_t> nmr_p;   // the same times R (k_fbs: gamma R joins the b sum)
      for (int k = 0; k < FBP_NC; ++k) {
        const std::vector<uint32_t> v = mul_pow2_mod(mod(other, P), (size_t)FBP_CB * k, P).limbs(ps, LB);
        nm_p.insert(nm_p.end(), v.begin(), v.end());
        const std::vector<uint32_t> r = mul_pow2_mod(mod(other, P), (size_t)FBP_CB * k + RS, P).limbs(ps, LB);
        nmr_p.insert(nmr_p.end(), r.begin(), r.end());
      }
      // position 0's lo entries are multiplied by kappa R (FbpHalf::kapR): kappa = q^-2 mod p^2 for the p half, so
      // that the sampler leaves w_p q^-2 for k_fbp_fin; 1 for the q half
      std::vector<uint32_t> kap_p;
      if (h == 0) {
        const HBig kap = inv_mod(sq[1], sq[0]);
        if (kap.is_zero()) return fb_unavailable(c, "q^2 not invertible mod p^2");
        split(mul_pow2_mod(kap, RS, m2), kap_p);
      }
      uint32_t *pp, *pone, *pbases, *pnm, *pnmr, *ppbig, *pkap = nullptr;
      if ((rc = upload_fb(c, P.limbs(ps, LB), &pp)) || (rc = upload_fb(c, one_p, &pone)) ||
          (rc = upload_fb(c, bases_p, &pbases)) || (rc = upload_fb(c, nm_p, &pnm)) || (rc = upload_fb(c, nmr_p, &pnmr)) ||
          (rc = upload_fb(c, mul(P, pow2(FBP_PB)).limbs(ps, LB), &ppbig)) ||
          (h == 0 && (rc = upload_fb(c, kap_p, &pkap))))
        return fb_unavailable(c, pai_last_error());
      if (h != 0) pkap = pone;
      // factored rows (kernels_fbp.hpp): inverse tables of the lo/hi entries' A parts and the batch inversion's
      // scratch -- released with lohi
      void *vinv = nullptr, *vpre = nullptr, *vcv = nullptr;
      const size_t em = (size_t)1 << (W - W / 2);
      if (hipMalloc(&vinv, (size_t)K * 2 * FB_LO * ps * 4) != hipSuccess ||
          (c->fb_mem.push_back(vinv), hipMalloc(&vpre, (size_t)2 * K * em * ps * 4) != hipSuccess) ||
          (c->fb_mem.push_back(vpre), hipMalloc(&vcv, (size_t)2 * K * ps * 4) != hipSuccess))
        return fb_unavailable(c, "table allocation failed");
      c->fb_mem.push_back(vcv);
      for (void* q : {vinv, vpre, vcv}) fb_scratch.push_back(q);
      pcval[h] = (uint32_t*)vcv;
      pv[h] = FbpHalf{(const uint4*)t[h], pp, pone, pbases, dlohi, pnm, ppbig, mont_prime(P, LB),
                      (uint32_t*)vinv, (uint32_t*)vpre, (uint32_t*)vcv, pkap, pnmr};
      if (shoup) {
        const HBig R2 = pow2(2 * RS);
        const HBig mu = div_big(R2, P);
        if (mu.bits() > (size_t)LB * (ps + 1)) return fb_unavailable(c, "Shoup rows: mu exceeds S + 1 limbs");
        fcst_host[h] = mu.limbs(ps + 2, LB);
        const std::vector<uint32_t> r2 = mod(R2, P).limbs(ps, LB);
        fcst_host[h].insert(fcst_host[h].end(), r2.begin(), r2.end());
      }
    }
    if (gpair_ok) {
      // pair-group constants: S = 76 limbs of p_h, R = 2^(28 S); pairs as [A: S][B: S]
      const HBig& P = primes[h];
      const size_t RS = (size_t)LB * FBGP_S;
      auto split = [&](const HBig& v, std::vector<uint32_t>& out) {
        const HBig qt = div_big(v, P), rm = sub(v, mul(qt, P));
        const std::vector<uint32_t> a = rm.limbs(FBGP_S, LB), b = qt.limbs(FBGP_S, LB);
        out.insert(out.end(), a.begin(), a.end());
        out.insert(out.end(), b.begin(), b.end());
      };
      std::vector<uint32_t> one_p, nm_p;
      const std::vector<uint32_t>& bases_p = hp[h].bases_p;
      split(mul_pow2_mod(HBig(1), RS, m2), one_p);
      for (int k = 0; k < 4; ++k) {
        const std::vector<uint32_t> v = mul_pow2_mod(mod(primes[1 - h], P), (size_t)16 * k, P).limbs(FBGP_S, LB);
        nm_p.insert(nm_p.end(), v.begin(), v.end());
      }
      const HBig r = mul_pow2_mod(HBig(1), RS, P);
      const HBig X = mod(sub(add(P, HBig(1)), r), P);   // (1 - R) mod p_h
      uint32_t *gp, *gx, *gone, *gbases, *gnm, *gpbig, *gp2, *gpr2;
      if ((rc = upload_fb(c, P.limbs(FBGP_S, LB), &gp)) || (rc = upload_fb(c, X.limbs(FBGP_S, LB), &gx)) ||
          (rc = upload_fb(c, one_p, &gone)) || (rc = upload_fb(c, bases_p, &gbases)) || (rc = upload_fb(c, nm_p, &gnm)) ||
          (rc = upload_fb(c, mul(P, pow2(20)).limbs(FBGP_S, LB), &gpbig)) || (rc = upload_fb(c, m2.limbs(sb, LB), &gp2)) ||
          (rc = upload_fb(c, mul_pow2_mod(P, RB, m2).limbs(sb, LB), &gpr2)))
        return fb_unavailable(c, pai_last_error());
      // factored rows (kernels_grp_pair.hpp): inverse tables of the lo/hi entries and the inversion's prefix
      // products -- build scratch, released with lohi
      void *vinv = nullptr, *vpre = nullptr, *vcv = nullptr;
      const size_t em = (size_t)1 << (W - W / 2);
      if (hipMalloc(&vinv, (size_t)K * 2 * FB_LO * FBGP_S * 4) != hipSuccess ||
          (c->fb_mem.push_back(vinv), hipMalloc(&vpre, (size_t)2 * K * em * FBGP_S * 4) != hipSuccess) ||
          (c->fb_mem.push_back(vpre), hipMalloc(&vcv, (size_t)2 * K * FBGP_S * 4) != hipSuccess))
        return fb_unavailable(c, "table allocation failed");
      c->fb_mem.push_back(vcv);
      for (void* q : {vinv, vpre, vcv}) fb_scratch.push_back(q);
      gcval[h] = (uint32_t*)vcv;
      gv[h] = FbgpHalf{(const uint32_t*)t[h], gp, gx, gone, gbases, dlohi, gnm, gpbig, gp2, gpr2, mont_prime(P, LB),
                       mont_prime(m2, LB), (uint32_t*)vinv, (uint32_t*)vpre, (uint32_t*)vcv};
      if (sgp_enabled() &&
          (rc = sgp_make_half(P, primes[1 - h], K, t[h],
                              [&](const std::vector<uint32_t>& v, uint32_t** o) { return upload_fb(c, v, o); }, &sv[h])))
        return fb_unavailable(c, pai_last_error());
    }
    if (h == 0) {
      c->d_fb_m0 = dm;
      c->fb_mprime0 = mont_prime(m2, LB);
    }
    // exponent reduction mod D_h = p_h - 1
    const HBig D = sub(primes[h], HBig(1));
    const HBig mu = div_big(pow2((size_t)raw_bits), D);
    const std::vector<uint32_t> dw = D.words((D.bits() + 31) / 32), muw = mu.words(4);
    std::copy(dw.begin(), dw.end(), red[h].D);
    std::copy(muw.begin(), muw.end(), red[h].mu);
    red[h].dwords = (int)dw.size();
    red[h].kbits = (int)D.bits();
  }
  // Garner constants (mod p^2): 8 p^2, (q^2)^-1 R, q^2
  const HBig coef = inv_mod(sq[1], sq[0]);
  if (coef.is_zero()) return fb_unavailable(c, "q^2 not invertible mod p^2");
  std::vector<FbHalf> v(hv, hv + 2);
  std::vector<FbRed> vr(red, red + 2);
  if ((rc = upload_fb(c, v, &c->d_fb_halves)) || (rc = upload_fb(c, vr, &c->d_fb_red)) ||
      (rc = upload_fb(c, mul(sq[0], HBig(8)).limbs(sb, LB), &c->d_fb_m8)) ||
      (rc = upload_fb(c, mul_pow2_mod(coef, RB, sq[0]).limbs(sb, LB), &c->d_fb_coefR)) ||
      (rc = upload_fb(c, sq[1].limbs(sb, LB), &c->d_fb_q2)) ||
      (grp && (rc = upload_fb(c, mul_pow2_mod(sq[1], (size_t)LB * c->S_e, c->N).limbs(c->S_e, LB), &c->d_fb_q2Rn))))
    return fb_unavailable(c, pai_last_error());
  const auto t1 = std::chrono::steady_clock::now();
  if (pair_ok) {
    std::vector<FbpHalf> pvv(pv, pv + 2);
    if ((rc = upload_fb(c, pvv, &c->d_fbp_halves))) return fb_unavailable(c, pai_last_error());
    if (shoup) {
      FbsConst fc[2];
      for (int h = 0; h < 2; ++h) {
        uint32_t* d;
        if ((rc = upload_fb(c, fcst_host[h], &d))) return fb_unavailable(c, pai_last_error());
        fc[h] = FbsConst{d, d + ps + 2};
      }
      std::vector<FbsConst> fcv(fc, fc + 2);
      if ((rc = upload_fb(c, fcv, &c->d_fbs_cst))) return fb_unavailable(c, pai_last_error());
    }
    // k_fbp_fin (kernels_fbp.hpp): (q^-1 R)^, (q^-2 R)^ as pairs over p, then q, q^2, p q^2, 2p, 3p
    const HBig &P = primes[0], &Q = primes[1];
    const size_t RS = (size_t)LB * ps;
    std::vector<uint32_t> cs;
    auto put = [&](const HBig& v, int limbs) {
      const std::vector<uint32_t> l = v.limbs(limbs, LB);
      cs.insert(cs.end(), l.begin(), l.end());
    };
    auto put_pair = [&](const HBig& v) {   // v mod p^2 -> (v mod p, v div p)
      const HBig qt = div_big(v, P);
      put(sub(v, mul(qt, P)), ps);
      put(qt, ps);
    };
    const HBig qinv = inv_mod(mod(Q, sq[0]), sq[0]);
    if (qinv.is_zero()) return fb_unavailable(c, "q not invertible mod p^2");
    put_pair(mul_pow2_mod(qinv, RS, sq[0]));
    put_pair(mul_pow2_mod(coef, RS, sq[0]));
    put(Q, ps);
    put(sq[1], 2 * ps);
    put(mul(P, sq[1]), 3 * ps);
    put(mul(P, HBig(2)), ps);
    put(mul(P, HBig(3)), ps);
    if ((rc = upload_fb(c, cs, &c->d_fbp_fin_cs))) return fb_unavailable(c, pai_last_error());
    c->d_fbp_fin_p = const_cast<uint32_t*>(pv[0].p);
    c->fbp_fin_mprime = pv[0].mprime;
  }
  if (gpair_ok) {
    std::vector<FbgpHalf> gvv(gv, gv + 2);
    if ((rc = upload_fb(c, gvv, &c->d_fbgp_halves))) return fb_unavailable(c, pai_last_error());
    if (sgp_enabled()) {
      std::vector<SgpHalf> svv(sv, sv + 2);
      if ((rc = upload_fb(c, svv, &c->d_sgp_fb))) return fb_unavailable(c, pai_last_error());
      c->d_sgp_q = sv[1].p;
    }
  }
  trace_uploads("  fb uploads");
  if (gpair_ok || pair_ok) {   // factored rows: the chain products are inverted on the host between the two phases
    SetupTrace tr_1("  phase 1 (lohi, inv_fwd) + host invert");
    const hipError_t e1 = gpair_ok ? fbgp_build_phase1(c->d_fbgp_halves, K, W, nullptr)
                                   : fbp_build_phase1(ps, c->d_fbp_halves, K, W, nullptr);
    if (e1 != hipSuccess || hipDeviceSynchronize() != hipSuccess) return fb_unavailable(c, "table construction failed");
    for (int h = 0; h < 2; ++h)
      if (pair_host_invert(primes[h], gpair_ok ? gcval[h] : pcval[h], 2 * K, gpair_ok ? FBGP_S : ps))
        return fb_unavailable(c, pai_last_error());
  }
  SetupTrace tr_2("  phase 2 (inv_bwd, fill) + frees");
#if FLEXPAI_XCHECK
  const hipError_t be = gpair_ok ? fbgp_build_phase2(c->d_fbgp_halves, (uint32_t*)t[0], (uint32_t*)t[1], K, W, nullptr)
                        : shoup  ? fbs_build_phase2(ps, c->d_fbp_halves, c->d_fbs_cst, (uint4*)t[0], (uint4*)t[1], K, W, nullptr,
                                                    guard_args(c, (unsigned long long)K << W, 0, 0, 0))
                                 : fbp_build_phase2(ps, c->d_fbp_halves, (uint4*)t[0], (uint4*)t[1], K, W, nullptr);
#else
  const hipError_t be = gpair_ok ? fbgp_build_phase2(c->d_fbgp_halves, (uint32_t*)t[0], (uint32_t*)t[1], K, W, nullptr)
                                 : fbs_build_phase2(ps, c->d_fbp_halves, c->d_fbs_cst, (uint4*)t[0], (uint4*)t[1], K, W, nullptr,
                                                    guard_args(c, (unsigned long long)K << W, 0, 0, 0));
#endif
  if (be != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fb_unavailable(c, "table construction failed");
  if (guard_collect(c, nullptr)) return fb_unavailable(c, pai_last_error());
  for (void* p : lohi) fb_scratch.push_back(p);
  SetupTrace tr_f("  scratch frees");
  for (void* p : fb_scratch) {
    c->fb_mem.erase(std::find(c->fb_mem.begin(), c->fb_mem.end(), p));
    (void)hipFree(p);
  }
  if (sgs && !(gpair_ok && sgp_enabled())) {   // (a test build's $FLEXPAI_SGP=0 context)
    for (uint4*& r : sgs_rows) {
      c->fb_tables.erase(std::find(c->fb_tables.begin(), c->fb_tables.end(), (void*)r));
      TableArena::get().free(r);
      r = nullptr;
    }
  }
  if (gpair_ok && sgp_enabled() && sgs) {
    SetupTrace tr_s("  Shoup rows (k_sgs_conv)");
    if ((rc = sgs_build(c, primes, K, W, t, sv, sgs_rows))) {
      // the factored rows are complete: k_sgp runs on them (split_sampler bit 3 stays clear)
      if (setup_trace_on()) fprintf(stderr, "flexpai-trace Shoup rows failed (%s): k_sgp at W = %d\n", pai_last_error(), W);
      for (uint4*& r : sgs_rows) {
        c->fb_tables.erase(std::find(c->fb_tables.begin(), c->fb_tables.end(), (void*)r));
        TableArena::get().free(r);
        r = nullptr;
      }
    }
  }
  const auto t2 = std::chrono::steady_clock::now();
  c->fb_host_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
  c->fb_dev_ms = std::chrono::duration<float, std::milli>(t2 - t1).count();
  c->fb_table_bytes = fb_bytes(c, W, c->d_sgs_fb != nullptr);
  c->fb_K = K;
  c->fb_pair_s = pair_ok ? ps : 0;
  c->fb_shoup = shoup;
  c->fb_gpair = gpair_ok;
  c->fb_W_used = W;
  c->fb_raw_bits = raw_bits;
  c->fb_state = pai_ctx::FB_READY;
  return 1;
}

// 4096-bit keys (p^2 of 148 limbs): no lane CRT; the fixed-base sampler runs on the group engine
// (kernels_grp.hpp) and k_crt_fin<8> recombines, so only its constants are set up here. Without resident
// tables, encryption takes the public-key path.
static int setup_fbg(pai_ctx* c, const HBig& p, const HBig& q) {
  constexpr int SBG = GRP_TPI * L;
  const size_t pb = std::max(p.bits(), q.bits());
  if ((size_t)LB * SBG < 2 * pb + 4 || c->tpi_e != 8) return 0;
  const size_t RE = (size_t)LB * c->S_e;
  int rc;
  if ((rc = upload(c, mul_pow2_mod(mul(q, q), 2 * RE, c->N).limbs(c->S_e, LB), &c->d_kq)) ||
      (rc = upload(c, mul_pow2_mod(mul(p, p), 2 * RE, c->N).limbs(c->S_e, LB), &c->d_kp)))
    return rc;
  c->crt_sa = 0;
  c->crt_sb = SBG;
  c->fb_p = p;
  c->fb_q = q;
  c->fbg_ok = true;
  // split-pair decryption (kernels_dec4.hpp): p_h of at most 28 * 74 - 24 bits (R >= 2^24 p_h), the ciphertext
  // in at most 4 chunks of 74 limbs; $FLEXPAI_PAIR=0 keeps the group engine's k_decrypt
  bool pair = true;
  if (const char* e = xcheck_env("FLEXPAI_PAIR")) pair = atoi(e) != 0;
  const size_t RS = (size_t)LB * D4_S;
  const int kp = (int)((32 * (size_t)c->ct_words + RS - 1) / RS);
  if (pair && pb + 24 <= RS && kp <= 4 && c->tpi_d == 4) {
    const HBig primes[2] = {p, q};
    Dec4Half dh[2];
    for (int h = 0; h < 2; ++h) {
      const HBig& ph = primes[h];
      const HBig m2 = mul(ph, ph);
      auto split = [&](const HBig& v) {
        const HBig qt = div_big(v, ph), rm = sub(v, mul(qt, ph));
        std::vector<uint32_t> out = rm.limbs(D4_S, LB), b = qt.limbs(D4_S, LB);
        out.insert(out.end(), b.begin(), b.end());
        return out;
      };
      auto one_minus = [&](const HBig& r) {   // (1 - r) mod p_h for 0 < r < p_h
        return mod(sub(add(ph, HBig(1)), r), ph);
      };
      std::vector<uint32_t> pd, kf;
      if (!build_dec4f_program(ph, RS, pd, kf)) return 0;
      HBig oi = inv_mod(mod(primes[1 - h], ph), ph);
      if (oi.is_zero()) return 0;
      const HBig hh = sub(ph, oi);
      uint32_t *dp, *dx1, *dxk, *dck, *dhr, *dprog, *dkf;
      if ((rc = upload(c, ph.limbs(D4_S, LB), &dp)) ||
          (rc = upload(c, one_minus(mul_pow2_mod(HBig(1), RS, ph)).limbs(D4_S, LB), &dx1)) ||
          (rc = upload(c, one_minus(mul_pow2_mod(HBig(1), RS * kp, ph)).limbs(D4_S, LB), &dxk)) ||
          (rc = upload(c, split(mul_pow2_mod(HBig(1), RS * (kp + 1), m2)), &dck)) ||
          (rc = upload(c, mul_pow2_mod(hh, RS, ph).limbs(D4_S, LB), &dhr)) || (rc = upload(c, pd, &dprog)) ||
          (rc = upload(c, kf, &dkf)))
        return rc;
      dh[h] = Dec4Half{dp, dx1, dxk, dck, dhr, dprog, (int)pd.size(), mont_prime(ph, LB), dkf};
    }
    std::vector<Dec4Half> dv(dh, dh + 2);
    if ((rc = upload(c, dv, &c->d_dec4_halves))) return rc;
    c->dec4_kchunks = kp;
    c->dec4_ok = true;
  }
  return 0;
}

// A 4096-bit key's constants for the row kernels (kernels_crtw.hpp; the lane CRT kernels stop at 2048 bits): per
// half, stage A over the 74 limbs of p_h (R^(K+1) mod p_h, the op list over q_h mod (p_h - 1)), stage B over the 148
// limbs of p_h^2 (R^2, coef, the op list over p_h) and decryption (R^(K+1) mod p_h^2, the op list over p_h - 1); the
// finish reuses setup_fbg's q^2 R^2 / p^2 R^2 mod n^2 and the k_dec4 halves. Soft: an unusable key leaves rows_sa = 0.
static int setup_rows4096(pai_ctx* c, const HBig& p, const HBig& q) {
  constexpr int SA = 74, SB = 148;
  c->rows_sa = 0;
  if (c->tpi_e != 8 || !c->d_kq || std::max(p.bits(), q.bits()) + 2 > (size_t)LB * SA) return 0;
  const size_t RA = (size_t)LB * SA, RB = (size_t)LB * SB;
  const int kd = (int)((32 * (size_t)c->ct_words + RB - 1) / RB);
  if (kd > KMAX_CHUNKS) return 0;
  SetupTrace tr("    rows 4096 consts");
  const HBig primes[2] = {p, q};
  const HBig sq[2] = {mul(p, p), mul(q, q)};
  CrtHalf ha[2], hb[2], hd[2];
  int rc;
  for (int h = 0; h < 2; ++h) {
    const HBig& ph = primes[h];
    const HBig& m2 = sq[h];
    std::vector<uint32_t> pa, pb, pd;
    if (!build_lane_program(mod(primes[1 - h], sub(ph, HBig(1))), pa) || !build_lane_program(ph, pb) ||
        !build_lane_program(sub(ph, HBig(1)), pd))
      return 0;
    const HBig coef = inv_mod(sq[1 - h], m2);
    if (coef.is_zero()) return 0;
    std::vector<uint32_t> ck;
    for (int K = 1; K <= KMAX_CHUNKS; ++K) {
      std::vector<uint32_t> v = mul_pow2_mod(HBig(1), RA * (K + 1), ph).limbs(SA, LB);
      ck.insert(ck.end(), v.begin(), v.end());
    }
    std::vector<uint32_t> oneA(SA, 0), oneB(SB, 0);
    oneA[0] = oneB[0] = 1;
    uint32_t *dm, *dck, *done, *dpa, *dm2, *dr2, *dcoef, *dpb, *dck2, *done2, *dpd;
    if ((rc = upload(c, ph.limbs(SA, LB), &dm)) || (rc = upload(c, ck, &dck)) || (rc = upload(c, oneA, &done)) ||
        (rc = upload(c, pa, &dpa)) || (rc = upload(c, m2.limbs(SB, LB), &dm2)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), 2 * RB, m2).limbs(SB, LB), &dr2)) ||
        (rc = upload(c, coef.limbs(SB, LB), &dcoef)) || (rc = upload(c, pb, &dpb)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), RB * (kd + 1), m2).limbs(SB, LB), &dck2)) ||
        (rc = upload(c, oneB, &done2)) || (rc = upload(c, pd, &dpd)))
      return rc;
    ha[h] = CrtHalf{dm, dck, done, dpa, (int)pa.size(), mont_prime(ph, LB)};
    hb[h] = CrtHalf{dm2, dr2, dcoef, dpb, (int)pb.size(), mont_prime(m2, LB)};
    hd[h] = CrtHalf{dm2, dck2, done2, dpd, (int)pd.size(), mont_prime(m2, LB)};
  }
  std::vector<CrtHalf> va(ha, ha + 2), vb(hb, hb + 2), vd(hd, hd + 2);
  if ((rc = upload(c, va, &c->d_crt_a)) || (rc = upload(c, vb, &c->d_crt_b)) || (rc = upload(c, vd, &c->d_decw)))
    return rc;
  c->decw_kchunks = kd;
  c->rows_sa = SA;
  return 0;
}

// CRT encryption constants (kernels_crt.hpp). p < q here (sorted like keypair.py:57-62).
static int setup_crt(pai_ctx* c, const HBig& p, const HBig& q) {
  c->crt_ok = c->fbg_ok = c->dec_pair_ok = c->crt_pair_ok = c->dec4_ok = false;
  const size_t pb = std::max(p.bits(), q.bits());
  int sa = 0, sb = 0;
  for (auto cand : {std::pair<int, int>{19, 37}, std::pair<int, int>{37, 74}}) {
    if ((size_t)LB * cand.first >= pb + 2 && (size_t)LB * cand.second >= 2 * pb + 2) {
      sa = cand.first;
      sb = cand.second;
      break;
    }
  }
  if (!sa) {   // too large for the lane engine: fixed-base on the group engine, protocol-sized calls on rows
    int rc0 = setup_fbg(c, p, q);
    return rc0 ? rc0 : setup_rows4096(c, p, q);
  }
  const size_t RA = (size_t)LB * sa, RB = (size_t)LB * sb, RE = (size_t)LB * c->S_e;
  const HBig primes[2] = {p, q};
  const HBig sq[2] = {mul(p, p), mul(q, q)};
  CrtHalf ha[2], hb[2], hd[2];
  int rc;
  SetupTrace tr_ab("    crt stage A/B consts");
  for (int h = 0; h < 2; ++h) {
    const HBig& ph = primes[h];
    const HBig& other = primes[1 - h];
    // stage A: (r mod p_h)^(other mod (p_h - 1)) mod p_h
    HBig ea = mod(other, sub(ph, HBig(1)));
    std::vector<uint32_t> pa, pbp;
    if (!build_lane_program(ea, pa) || !build_lane_program(ph, pbp)) return 0;
    std::vector<uint32_t> ck;
    for (int K = 1; K <= KMAX_CHUNKS; ++K) {
      std::vector<uint32_t> v = mul_pow2_mod(HBig(1), RA * (K + 1), ph).limbs(sa, LB);
      ck.insert(ck.end(), v.begin(), v.end());
    }
    std::vector<uint32_t> one(sa, 0);
    one[0] = 1;
    uint32_t *dm, *dck, *done, *dpa;
    if ((rc = upload(c, ph.limbs(sa, LB), &dm)) || (rc = upload(c, ck, &dck)) || (rc = upload(c, one, &done)) ||
        (rc = upload(c, pa, &dpa)))
      return rc;
    ha[h] = CrtHalf{dm, dck, done, dpa, (int)pa.size(), mont_prime(ph, LB)};
    // stage B: y^(p_h) mod p_h^2, times (other^2)^-1 mod p_h^2
    const HBig& m2 = sq[h];
    HBig coef = inv_mod(sq[1 - h], m2);
    if (coef.is_zero()) return 0;
    uint32_t *dm2, *dr2, *dcoef, *dpb;
    if ((rc = upload(c, m2.limbs(sb, LB), &dm2)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), 2 * RB, m2).limbs(sb, LB), &dr2)) ||
        (rc = upload(c, coef.limbs(sb, LB), &dcoef)) || (rc = upload(c, pbp, &dpb)))
      return rc;
    hb[h] = CrtHalf{dm2, dr2, dcoef, dpb, (int)pbp.size(), mont_prime(m2, LB)};
    // decryption on 16-lane rows (k_dec_w): c R mod p_h^2 by kd passes, then the op list over p_h - 1
    const int kd = (int)((32 * (size_t)c->ct_words + RB - 1) / RB);
    std::vector<uint32_t> pdw, oneb(sb, 0);
    oneb[0] = 1;
    if (kd <= KMAX_CHUNKS && build_lane_program(sub(ph, HBig(1)), pdw)) {
      uint32_t *dck2, *done2, *dpdw;
      if ((rc = upload(c, mul_pow2_mod(HBig(1), RB * (kd + 1), m2).limbs(sb, LB), &dck2)) || (rc = upload(c, oneb, &done2)) ||
          (rc = upload(c, pdw, &dpdw)))
        return rc;
      hd[h] = CrtHalf{dm2, dck2, done2, dpdw, (int)pdw.size(), mont_prime(m2, LB)};
      c->decw_kchunks = kd;
    } else {
      c->decw_kchunks = 0;
    }
  }
  std::vector<CrtHalf> va(ha, ha + 2), vb(hb, hb + 2), vd(hd, hd + 2);
  if ((rc = upload(c, va, &c->d_crt_a)) || (rc = upload(c, vb, &c->d_crt_b))) return rc;
  if (c->decw_kchunks && (rc = upload(c, vd, &c->d_decw))) return rc;
  // finish: q^2 R^2 mod n^2 and p^2 R^2 mod n^2 (group layout)
  if ((rc = upload(c, mul_pow2_mod(sq[1], 2 * RE, c->N).limbs(c->S_e, LB), &c->d_kq)) ||
      (rc = upload(c, mul_pow2_mod(sq[0], 2 * RE, c->N).limbs(c->S_e, LB), &c->d_kp)))
    return rc;
  c->crt_sa = sa;
  c->crt_sb = sb;
  c->crt_ok = true;
  c->fb_p = p;   // the fixed-base tables are built lazily (ensure_fb)
  c->fb_q = q;
  // lane decryption's CRT constants (p, q, q^-1 R mod p), shared by the pair kernels' k_dec_fin_pair
  {
    SetupTrace tr_d("    lane decrypt consts");
    if ((int)((32 * (size_t)c->ct_words + RB - 1) / RB) > KMAX_CHUNKS) return 0;
    HBig qinv = inv_mod(mod(q, p), p);
    if ((rc = upload(c, p.limbs(sa, LB), &c->d_dec_p)) || (rc = upload(c, q.limbs(sa, LB), &c->d_dec_q)) ||
        (rc = upload(c, mul_pow2_mod(qinv, RA, p).limbs(sa, LB), &c->d_dec_qinvR)))
      return rc;
    c->dec_pprime = mont_prime(p, LB);
    c->dec_lane_ok = true;
  }
  // pair kernels: residues mod p_h^2 as (A, B) over the sa limbs of p_h, R = 2^(28 sa) >= 2^12 p_h
  bool pair = true;
  if (const char* e = xcheck_env("FLEXPAI_PAIR")) pair = atoi(e) != 0;
  if (pair && (size_t)LB * sa >= pb + 12) {
    SetupTrace tr_p("    pair consts");
    const int S2 = 2 * sa;
    auto split = [&](const HBig& v, const HBig& P) {   // canonical pair of v < P^2
      const HBig qt = div_big(v, P), rm = sub(v, mul(qt, P));
      std::vector<uint32_t> out = rm.limbs(sa, LB), b = qt.limbs(sa, LB);
      out.insert(out.end(), b.begin(), b.end());
      return out;
    };
    const int kp = (int)((32 * (size_t)c->ct_words + RA - 1) / RA);
    std::vector<uint32_t> one(S2, 0);
    one[0] = 1;
    DecPairHalf dp[2];
    CrtHalf pw[2], pbh[2];
    for (int h = 0; h < 2; ++h) {
      const HBig& ph = primes[h];
      const HBig& other = primes[1 - h];
      const HBig& m2 = sq[h];
      std::vector<uint32_t> pd, pe, kf;
      const bool decf = !(xcheck_env("FLEXPAI_DECF") && atoi(xcheck_env("FLEXPAI_DECF")) == 0);
      if (!(decf ? build_decf_lane_program(ph, RA, sa, pd, kf) : build_lane_program(sub(ph, HBig(1)), pd)) ||
          !build_lane_program(ph, pe))
        return 0;
      c->decf = decf;
      HBig oi = inv_mod(mod(other, ph), ph);
      HBig coef = inv_mod(sq[1 - h], m2);
      if (oi.is_zero() || coef.is_zero()) return 0;
      const uint32_t mp1 = mont_prime(ph, LB);
      uint32_t *dph, *dck, *dhR, *dpm1, *done, *dprog, *dr2, *dcoef, *dpe, *dkf = nullptr;
      if ((rc = upload(c, ph.limbs(sa, LB), &dph)) ||
          (rc = upload(c, split(mul_pow2_mod(HBig(1), RA * (kp + 1), m2), ph), &dck)) ||
          (rc = upload(c, mul_pow2_mod(sub(ph, oi), RA, ph).limbs(sa, LB), &dhR)) ||
          (rc = upload(c, sub(ph, HBig(1)).limbs(sa, LB), &dpm1)) || (rc = upload(c, one, &done)) ||
          (rc = upload(c, pd, &dprog)) || (rc = upload(c, split(mul_pow2_mod(HBig(1), 2 * RA, m2), ph), &dr2)) ||
          (rc = upload(c, split(coef, ph), &dcoef)) || (rc = upload(c, pe, &dpe)) ||
          (!kf.empty() && (rc = upload(c, kf, &dkf))))
        return rc;
      dp[h] = DecPairHalf{dph, dck, dhR, dpm1, mp1, 0u};
      pw[h] = CrtHalf{dph, dkf, done, dprog, (int)pd.size(), mp1};
      pbh[h] = CrtHalf{dph, dr2, dcoef, dpe, (int)pe.size(), mp1};
    }
    std::vector<DecPairHalf> dpv(dp, dp + 2);
    std::vector<CrtHalf> pwv(pw, pw + 2), pbv(pbh, pbh + 2);
    HBig maxint = sub(div_small(c->n, 3), HBig(1));
    if ((rc = upload(c, dpv, &c->d_decp_halves)) || (rc = upload(c, pwv, &c->d_decp_pow)) ||
        (rc = upload(c, pbv, &c->d_crtp_b)) || (rc = upload(c, c->n.limbs(S2, LB), &c->d_decp_nl)) ||
        (rc = upload(c, maxint.limbs(S2, LB), &c->d_decp_maxint)))
      return rc;
    c->decp_kchunks = kp;
    c->dec_pair_ok = c->dec_lane_ok;   // shares the lane decrypt's p, q, q^-1 R constants
    c->crt_pair_ok = true;
  }
  return 0;
}

static int set_private_impl(pai_ctx* c, HBig p, HBig q);

// Transactional: on any failure every private-key allocation of this call is released and the
// context is left exactly as before (public-key operations keep working, a retry starts clean).
// The fixed-base tables are not built here (ensure_fb, on the first device-RNG encryption).
int pai_ctx_set_private(pai_ctx* c, const uint8_t* p_le, const uint8_t* q_le, size_t half_bytes) {
  if (!c || !p_le || !q_le) return fail(PAI_ERR_ARG, "pai_ctx_set_private: null argument");
  CtxLock lk(c);
  HIPCHK(hipSetDevice(c->device));
  HBig p = HBig::from_le_bytes(p_le, half_bytes), q = HBig::from_le_bytes(q_le, half_bytes);
  if (cmp(mul(p, q), c->n) != 0) return fail(PAI_ERR_KEY, "given public key does not match the given p and q");
  if (cmp(p, q) == 0) return fail(PAI_ERR_KEY, "p and q have to be different");
  if (cmp(q, p) < 0) std::swap(p, q);   // keypair.py:57-62
  if (c->has_priv) return 0;            // same key (p q == n): already set
  c->in_priv = true;
  int rc;
  {
    SetupTrace tr("pai_ctx_set_private");
    rc = set_private_impl(c, p, q);
  }
  trace_uploads("  set_private uploads");
  c->in_priv = false;
  if (!rc && !c->holder) {
    c->holder = true;
    ++g_key_holders;
  }
  if (rc) {
    const std::string msg = g_last_error;
    for (void* a : c->priv_allocs) (void)hipFree(a);
    c->priv_allocs.clear();
    (void)hipGetLastError();
    c->has_priv = c->crt_ok = c->fbg_ok = c->dec_lane_ok = c->dec_pair_ok = c->crt_pair_ok = c->dec4_ok = false;
    c->d_decw = nullptr;
    c->decw_kchunks = 0;
    c->rows_sa = 0;
    c->fb_state = pai_ctx::FB_UNTRIED;
    g_last_error = msg;
  }
  return rc;
}

static int set_private_impl(pai_ctx* c, HBig p, HBig q) {
  const int S = c->S_d;
  const size_t Rbits = (size_t)LB * S;
  HBig hp, hq;
  {
    HBig qi = inv_mod(q, p), pi = inv_mod(p, q);
    if (qi.is_zero() || pi.is_zero()) return fail(PAI_ERR_KEY, "p, q not coprime");
    hp = sub(p, qi);   // (-q)^-1 mod p == L(g^(p-1) mod p^2, p)^-1 (keypair.py:81-90, g = n + 1)
    hq = sub(q, pi);
  }
  HBig primes[2] = {p, q}, hs[2] = {hp, hq};
  size_t ebits = std::max(sub(p, HBig(1)).bits(), sub(q, HBig(1)).bits());
  c->nwin = (int)((ebits + 4) / 5);
  DecHalf hh[2];
  int rc;
  for (int h = 0; h < 2; ++h) {
    const HBig& ph = primes[h];
    HBig m = mul(ph, ph);
    HBig e = sub(ph, HBig(1));
    std::vector<uint8_t> dig(c->nwin);
    for (int w = 0; w < c->nwin; ++w) {
      int v = 0;
      for (int b = 4; b >= 0; --b) v = (v << 1) | e.bit((size_t)(c->nwin - 1 - w) * 5 + b);
      dig[w] = (uint8_t)v;
    }
    uint32_t *dm, *dR3, *done, *dpneg, *dph, *dhR;
    uint8_t* ddig;
    HBig pneg = sub(pow2(Rbits), ph);
    if ((rc = upload(c, m.limbs(S, LB), &dm)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), 3 * Rbits, m).limbs(S, LB), &dR3)) ||
        (rc = upload(c, mul_pow2_mod(HBig(1), Rbits, m).limbs(S, LB), &done)) ||
        (rc = upload(c, pneg.limbs(S, LB), &dpneg)) || (rc = upload(c, ph.limbs(S, LB), &dph)) ||
        (rc = upload(c, mul_pow2_mod(hs[h], Rbits, ph).limbs(S, LB), &dhR)) || (rc = upload(c, dig, &ddig)))
      return rc;
    hh[h] = DecHalf{dm, dR3, done, dpneg, dph, dhR, ddig, mont_prime(m, LB), mont_prime(pneg, LB), mont_prime(ph, LB), 0u};
  }
  std::vector<DecHalf> hv(hh, hh + 2);
  if ((rc = upload(c, hv, &c->d_halves))) return rc;
  HBig qinv = inv_mod(q, p);
  HBig maxint = sub(div_small(c->n, 3), HBig(1));   // keypair.py:29
  if ((rc = upload(c, mul_pow2_mod(qinv, Rbits, p).limbs(S, LB), &c->d_qinvR)) ||
      (rc = upload(c, c->n.limbs(S, LB), &c->d_nlimb)) ||
      (rc = upload(c, mul_pow2_mod(mod(q, c->n), Rbits, c->n).limbs(S, LB), &c->d_qRn)) ||
      (rc = upload(c, maxint.limbs(S, LB), &c->d_maxint)))
    return rc;
  c->nprime_d = mont_prime(c->n, LB);
  c->n_limbs = (int)((c->n.bits() + LB - 1) / LB);
  c->has_priv = true;
  SetupTrace tr("  setup_crt");
  if ((rc = setup_crt(c, p, q))) return rc;
  // a key outside the pair kernels' bounds (R = 2^(28 S) >= 2^12 p_h) -- or a test build's $FLEXPAI_PAIR=0 context --
  // encrypts on the public-key kernels and decrypts on the group engine (the 2S-limb lane kernels were retired in
  // round 6)
  if (c->crt_ok && !c->crt_pair_ok) c->crt_ok = false;
  if (c->dec_lane_ok && !c->dec_pair_ok) c->dec_lane_ok = false;
  return 0;
}

void pai_ctx_destroy(pai_ctx* c) { delete c; }

void pai_release_table_cache(void) { TableArena::get().trim(); }

int pai_ctx_set_option(pai_ctx* c, int option, int value) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  switch (option) {
    case PAI_OPT_CRT_ENCRYPT: c->crt_enabled = value != 0; return 0;
    case PAI_OPT_ROWS_MAX:
      if (value < 0) return fail(PAI_ERR_ARG, "PAI_OPT_ROWS_MAX must be >= 0");
      c->crtw_max = value;
      return 0;
    case PAI_OPT_STAGE_TIMING: c->timing = value != 0; stage_reset(c); return 0;
    case PAI_OPT_LANE_DECRYPT: c->dec_lane_enabled = value != 0; return 0;
    case PAI_OPT_FIXED_BASE: c->fb_enabled = value != 0; return 0;
    case PAI_OPT_PUBLIC_FB: c->pfb_enabled = value != 0; return 0;
    case PAI_OPT_PFB_WINDOW:
      if (!pfb_window_ok(value)) return fail(PAI_ERR_ARG, "public fixed-base window must be 12, 16 or 20");
      if (value == c->pfb_W) return 0;
      c->pfb_W = value;
      HIPCHK(hipSetDevice(c->device));
      pfb_release(c);
      c->pfb_state = pai_ctx::FB_UNTRIED;
      return 0;
    case PAI_OPT_FB_WINDOW:
      if (!fb_window_ok(value)) return fail(PAI_ERR_ARG, "fixed-base window must be 8, 12, 16 or 20 .. 24");
      if (value == c->fb_W) return 0;
      c->fb_W = value;
      HIPCHK(hipSetDevice(c->device));
      fb_release(c);                       // rebuilt lazily for the new window
      c->fb_state = pai_ctx::FB_UNTRIED;
      return 0;
  }
  return fail(PAI_ERR_ARG, "pai_ctx_set_option: unknown option");
}

int pai_ctx_get_option(const pai_ctx* c, int option, int* value) {
  if (!c || !value) return fail(PAI_ERR_ARG, "null argument");
  CtxLock lk(c);
  switch (option) {
    case PAI_OPT_CRT_ENCRYPT: *value = c->crt_enabled ? 1 : 0; return 0;
    case PAI_OPT_CRT_AVAILABLE: *value = c->crt_ok ? 1 : 0; return 0;
    case PAI_OPT_ROWS_MAX: *value = (int)std::min<long long>(c->crtw_max, INT32_MAX); return 0;
    case PAI_OPT_STAGE_TIMING: *value = c->timing ? 1 : 0; return 0;
    case PAI_OPT_LANE_DECRYPT: *value = (c->dec_lane_ok && c->dec_lane_enabled) ? 1 : 0; return 0;
    // 1 when device-RNG encryption will use the fixed bases (tables resident, or not yet tried)
    case PAI_OPT_FIXED_BASE:
      *value = ((c->crt_ok || c->fbg_ok) && c->fb_enabled && c->fb_state != pai_ctx::FB_UNAVAILABLE) ? 1 : 0;
      return 0;
    case PAI_OPT_FB_WINDOW: *value = c->fb_W_used ? c->fb_W_used : c->fb_W ? c->fb_W : fb_default_window(); return 0;
    case PAI_OPT_FB_READY: *value = c->fb_state == pai_ctx::FB_READY ? 1 : 0; return 0;
    case PAI_OPT_PUBLIC_FB:
      *value = (pfb_supported(c) && c->pfb_enabled && c->pfb_state != pai_ctx::FB_UNAVAILABLE) ? 1 : 0;
      return 0;
    case PAI_OPT_PFB_READY: *value = c->pfb_state == pai_ctx::FB_READY ? 1 : 0; return 0;
    case PAI_OPT_PFB_WINDOW: *value = c->pfb_W_used ? c->pfb_W_used : c->pfb_W ? c->pfb_W : pfb_default_window(); return 0;
    case PAI_OPT_FB_PAIR:
      *value = c->fb_state == pai_ctx::FB_READY ? (c->fb_gpair ? FBGP_S : c->fb_pair_s) : 0;
      return 0;
    case PAI_OPT_SPLIT_SAMPLER:
      *value = (c->fb_state == pai_ctx::FB_READY && c->d_sgp_fb ? 1 : 0) |
               (c->pfb_state == pai_ctx::FB_READY && c->d_sgp_pfb ? 2 : 0) |
               (c->fb_state == pai_ctx::FB_READY && c->fb_shoup ? 4 : 0) |
               (c->fb_state == pai_ctx::FB_READY && c->d_sgs_fb ? 8 : 0);
      return 0;
    case PAI_OPT_PAIR:
      *value = ((c->dec_pair_ok || c->dec4_ok) && c->dec_lane_enabled ? 1 : 0) | (c->crt_pair_ok ? 2 : 0) |
               (c->pe_ok || c->pe1_ok ? 4 : 0);
      return 0;
  }
  return fail(PAI_ERR_ARG, "pai_ctx_get_option: unknown option");
}

int pai_ctx_stage_times(pai_ctx* c, float* ms_out, int max_out, int* count) {
  if (!c || !count) return fail(PAI_ERR_ARG, "null argument");
  CtxLock lk(c);
  *count = 0;
  if (c->nev < 2) return 0;
  HIPCHK(hipSetDevice(c->device));
  if (c->nchunk_ev > 0) HIPCHK(hipEventSynchronize(c->ev[c->nchunk_ev - 1][c->nev - 1]));
  const int k = std::min(c->nev - 1, max_out);
  for (int i = 0; i < k; ++i) {
    ms_out[i] = 0.f;
    for (int ch = 0; ch < c->nchunk_ev; ++ch) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, c->ev[ch][i], c->ev[ch][i + 1]));
      ms_out[i] += t;
    }
  }
  *count = k;
  return 0;
}

int pai_ctx_fixed_base_info(pai_ctx* c, uint32_t* g_p, uint32_t* g_q, int* digits, int* window) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (!c->crt_ok && !c->fbg_ok)
    return fail(PAI_ERR_NOPRIV, "fixed-base obfuscation not available (needs the private key)");
  HIPCHK(hipSetDevice(c->device));
  if (!ensure_fb((pai_ctx*)c)) return fail(PAI_ERR_KEY, "fixed-base obfuscation not available: " + c->fb_reason);
  if (g_p) *g_p = c->fb_g[0];
  if (g_q) *g_q = c->fb_g[1];
  if (digits) *digits = c->fb_K;
  if (window) *window = c->fb_W_used;
  return 0;
}

int pai_ctx_fixed_base_prepare(pai_ctx* c) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (!c->crt_ok && !c->fbg_ok)
    return fail(PAI_ERR_NOPRIV, "fixed-base obfuscation not available (needs the private key)");
  HIPCHK(hipSetDevice(c->device));
  if (!ensure_fb(c)) return fail(PAI_ERR_KEY, "fixed-base obfuscation not available: " + c->fb_reason);
  return 0;
}

// The window ensure_fb would choose and its break-even element count (0 when the tables are resident or
// the path is unavailable: nothing left to decide).
static long long fb_threshold(pai_ctx* c) {
  if (c->fb_state != pai_ctx::FB_UNTRIED || (!c->crt_ok && !c->fbg_ok)) return 0;
  const int TW = fb_row_words(c);
  if (!TW) return 0;
  if (!c->fb_W) c->fb_W = fb_default_window();
  bool sgs = false;
  const int w = fb_choose(c, fb_budget(c), &sgs);
  return w ? fb_break_even(c, w, fb_digit_count(c, w), 4 * fb_table_row_words(c) + (sgs ? 16 * SGS_ROW_Q : 0)) : 0;
}

static bool fb_wanted(pai_ctx* c, long long n) {
  if (c->fb_state != pai_ctx::FB_UNTRIED) return true;   // resident, or known unavailable (ensure_fb says)
  if (c->fb_call) return c->fb_call > 0;                 // a host-buffer call decided once for all chunks
  c->fb_seen += n;
  return c->fb_seen >= fb_threshold(c);
}

int pai_ctx_fixed_base_policy(pai_ctx* c, long long* seen, long long* threshold) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (seen) *seen = c->fb_seen;
  if (threshold) *threshold = fb_threshold(c);
  return 0;
}

int pai_ctx_fixed_base_setup(const pai_ctx* c, float* host_ms, float* device_ms, uint64_t* table_bytes) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (c->fb_state != pai_ctx::FB_READY) return fail(PAI_ERR_KEY, "fixed-base tables are not resident");
  if (host_ms) *host_ms = c->fb_host_ms;
  if (device_ms) *device_ms = c->fb_dev_ms;
  if (table_bytes) *table_bytes = c->fb_table_bytes;
  return 0;
}

int pai_ctx_info(const pai_ctx* c, int* key_bits, int* ct_words, int* pt_words) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (key_bits) *key_bits = c->nb;
  if (ct_words) *ct_words = c->ct_words;
  if (pt_words) *pt_words = c->pt_words;
  return 0;
}

// ------------------------------------------------------------------ device entry points
template <int TPI>
static int launch_encrypt(pai_ctx* c, EncParams& p, hipStream_t st) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  const size_t lds = (size_t)GPB * S * 4;
  const int grid = grid_for(c, k_encrypt<TPI>, lds, p.n, GPB);
  int rc = ensure_scratch(c, (size_t)grid * BLOCK * TILE_WORDS_PER_LANE * 4);
  if (rc) return rc;
  p.scratch = (uint32_t*)c->d_scratch;
  stage_mark(c, 0, st);
  hipLaunchKernelGGL(k_encrypt<TPI>, dim3(grid), dim3(BLOCK), lds, st, p);
  HIPCHK(hipGetLastError());
  stage_mark(c, 1, st);
  return 0;
}

// CRT encryption (kernels_crt.hpp) in chunks of CRT_CHUNK elements: stage A (mod p, q), stage B
// (mod p^2, q^2), finish (mod n^2), all asynchronous on `st`.
constexpr long long CRT_CHUNK = 1ll << 22;

template <int TPI>
static int launch_crt_fin(pai_ctx* c, CrtFinParams& f, hipStream_t st) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  const size_t lds = (size_t)GPB * S * 4;
  const int grid = grid_for(c, k_crt_fin<TPI>, lds, f.n, GPB);
  hipLaunchKernelGGL(k_crt_fin<TPI>, dim3(grid), dim3(BLOCK), lds, st, f);
  HIPCHK(hipGetLastError());
  return 0;
}

// Fixed-base encryption (kernels_fb.hpp), chunks of CRT_CHUNK elements: exponent digits, the per-half
// table products with c0 folded in, Garner recombination into the ciphertext words.
static int launch_fb(pai_ctx* c, const EncParams& e, hipStream_t st) {
  const int SB = c->crt_sb;
  const bool grp = SB == GRP_TPI * L;
  const long long N = e.n;
  const long long chunk = std::min(N, CRT_CHUNK);
  int occF = 1, occG = 1;
#if FLEXPAI_XCHECK
  if (grp && !c->fb_gpair) return fail(PAI_ERR_KEY, "fixed-base encrypt: no pair tables");
  if (grp && !c->d_sgp_fb) fbgp_occupancy(&occF);
  if (!grp && !c->fb_pair_s) return fail(PAI_ERR_KEY, "fixed-base encrypt: no pair tables");
#else
  if (grp && !(c->fb_gpair && c->d_sgp_fb)) return fail(PAI_ERR_KEY, "fixed-base encrypt: no split-pair tables");
  if (!grp && !c->fb_shoup) return fail(PAI_ERR_KEY, "fixed-base encrypt: no Shoup tables");
#endif
#if FLEXPAI_XCHECK
  if (c->fb_pair_s && !c->fb_shoup && fbp_occupancy(c->fb_pair_s, &occF)) return fail(PAI_ERR_KEY, "fixed-base encrypt: unsupported size");
#endif
  if (c->fb_shoup && fbs_occupancy(c->fb_pair_s, &occF)) return fail(PAI_ERR_KEY, "fixed-base encrypt: unsupported size");
  // elements per block: one per lane, one per lane pair (k_fbs), or one per lane group (grp)
  const int EPB = grp ? BLOCK / GRP_TPI : c->fb_shoup ? LANE_BLOCK / 2 : LANE_BLOCK;
  const long long lane_blocks = (chunk + EPB - 1) / EPB;
  const int gxF = (int)std::max<long long>(1, std::min<long long>(lane_blocks, (long long)occF * c->cus / 2));
  const int gxG = (int)std::max<long long>(1, std::min<long long>(lane_blocks, (long long)occG * c->cus));
  const size_t dbytes = (size_t)2 * c->fb_K * 4, wbytes = (size_t)2 * std::max(SB, 2 * c->fb_pair_s) * 4;   // per element
  int rc;
  const size_t sbytes = c->d_sgs_fb ? (size_t)2 * (16 * sizeof(uint4) + 2 * 4) : 0;   // k_sgs's b sums
  if ((rc = ensure_work(c, dbytes * chunk + wbytes * (size_t)fbp_npad(chunk) + sbytes * chunk))) return rc;   // pairs: 64-element tiles
  uint32_t* digits = (uint32_t*)c->d_work;
  uint32_t* w = (uint32_t*)((char*)c->d_work + dbytes * chunk);
  uint4* sgs_bsum = (uint4*)((char*)w + wbytes * (size_t)fbp_npad(chunk));
  int dbg_stage = 0;   // test build: $FLEXPAI_DEBUG_SGS_STAGE = 1 stops after k_sgs, 2 after the b sums (or k_sgp)
#if FLEXPAI_XCHECK
  if (const char* ds = getenv("FLEXPAI_DEBUG_SGS_STAGE")) dbg_stage = atoi(ds);
#endif
  uint32_t* sgs_bcc = (uint32_t*)(sgs_bsum + (size_t)2 * 16 * chunk);
  const size_t esz = e.dtype == PAI_F32 ? 4 : 8;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    FbDigitParams pd{};
    pd.n = n;
    std::memcpy(pd.rng_key, e.rng_key, sizeof(pd.rng_key));
    pd.index_base = e.index_base + (unsigned long long)off;
    pd.K = c->fb_K;
    pd.W = c->fb_W_used;
    pd.raw_bits = c->fb_raw_bits;
    pd.red = c->d_fb_red;
    pd.digits = digits;
    const unsigned long long dig_words = (unsigned long long)2 * c->fb_K * chunk, w_words = wbytes * (size_t)fbp_npad(chunk) / 4;
    pd.g = guard_args(c, 0, dig_words, 0, 0);
    const int gD = (int)std::min<long long>((long long)8 * c->cus, (n + FB_DIG_BLOCK - 1) / FB_DIG_BLOCK);
    stage_mark(c, 0, st);
#if defined(FBS_AB) && (FBS_AB & 4)
    if (!c->fb_shoup) HIPCHK(fb_launch_digits(pd, gD, st));   // (k_fbs draws its own)
#else
    HIPCHK(fb_launch_digits(pd, gD, st));
#endif
    stage_mark(c, 1, st);
    FbParams pf{};
    pf.halves = c->d_fb_halves;
    pf.n = n;
    pf.K = c->fb_K;
    pf.W = c->fb_W_used;
    pf.digits = digits;
    pf.out = w;
    pf.x = (const char*)e.x + (size_t)off * esz;
    pf.dtype = e.dtype;
    pf.exp_mode = e.exp_mode;
    pf.fexp = e.fexp;
    pf.exp = e.exp + off;
    pf.status = e.status ? e.status + off : nullptr;
    const int gF = (int)std::min<long long>(gxF, (n + EPB - 1) / EPB);
    if (c->fb_pair_s) {
      FbpParams pp{c->d_fbp_halves, n, pf.K, pf.W, digits, w, pf.x, pf.dtype, pf.exp_mode, pf.fexp, pf.exp, pf.status};
      pp.g = guard_args(c, (unsigned long long)pf.K << pf.W, dig_words, w_words, 0);
#if defined(FBS_AB) && (FBS_AB & 4)
      if (!c->d_abdig && hipMalloc((void**)&c->d_abdig, sizeof(FbDigitParams)) != hipSuccess) return fail(PAI_ERR_HIP, "abD");
      HIPCHK(hipMemcpyAsync(c->d_abdig, &pd, sizeof(pd), hipMemcpyHostToDevice, st));
      pp.dig = c->d_abdig;
#endif
#if FLEXPAI_XCHECK
      if (!c->fb_shoup) HIPCHK(fbp_launch(c->fb_pair_s, pp, gF, st));
#endif
      if (c->fb_shoup) HIPCHK(fbs_launch(c->fb_pair_s, pp, gF, st));
    } else if (grp && c->fb_gpair) {
      const FbgpParams pg{c->d_fbgp_halves, n, pf.K, pf.W, digits, w, pf.x, pf.dtype, pf.exp_mode, pf.fexp, pf.exp, pf.status};
      if (c->d_sgs_fb) {   // split pairs on Shoup rows (kernels_sgs.hpp), then the b sums applied
        int occS = 1;
        sgs_occupancy(&occS);
        SgsParams sp{c->d_sgs_fb, n, pf.K, pf.W, digits, w, sgs_bsum, sgs_bcc};
        sp.g = guard_args(c, (unsigned long long)pf.K << pf.W, dig_words, w_words, 0);
        const long long nb = (n + SGP_PAIRS - 1) / SGP_PAIRS;
        HIPCHK(sgs_launch(sp, (int)std::max<long long>(1, std::min<long long>(nb, (long long)occS * c->cus / 2)), 2, st));
        const SgsFinParams sf{c->d_sgs_fb, n, w, sgs_bsum, sgs_bcc, pf.x, pf.dtype, pf.exp_mode, pf.fexp, pf.exp, pf.status,
                              dbg_stage};
        if (dbg_stage != 1) HIPCHK(sgs_launch_bfin(sf, 2, c->cus, st));
      } else if (c->d_sgp_fb) {   // split pairs (kernels_sgp.hpp): SGP_PAIRS elements per block, grid (gx, 2)
        int occS = 1;
        sgp_occupancy(&occS);
        SgpParams sp{c->d_sgp_fb, n, pf.K, pf.W, digits, w, pf.x, pf.dtype, pf.exp_mode, pf.fexp, pf.exp, pf.status};
        sp.g = guard_args(c, (unsigned long long)pf.K << pf.W, dig_words, w_words, 0);
        const long long nb = (n + SGP_PAIRS - 1) / SGP_PAIRS;
        HIPCHK(sgp_launch(sp, (int)std::max<long long>(1, std::min<long long>(nb, (long long)occS * c->cus / 2)), 2, st));
      } else {
#if FLEXPAI_XCHECK
        HIPCHK(fbgp_launch(pg, gF, st));
#endif
      }
    }
    stage_mark(c, 2, st);
    c->fb_last_w = w;
    c->fb_last_n = n;
    if (dbg_stage) continue;
    if (grp) {   // w_h = c0 G_h^(a_h) mod p_h^2 -> Garner: h mod p^2 (S = 148), c = w_q + q^2 h mod n^2 (S = 296)
      int occH = 1, occC = 1;
      grp_fin_occupancy(&occH, &occC);
      if (c->fb_gpair && c->d_sgp_fb) {   // the pairs -> w_h = A + p_h B mod p_h^2 (timed with the fin stage)
        SgpParams sw{};
        sw.halves = c->d_sgp_fb;
        sw.n = n;
        sw.out = w;
        HIPCHK(sgp_launch_w(sw, 2, c->cus, st));
      } else if (c->fb_gpair) {
        const FbgpParams pg{c->d_fbgp_halves, n, pf.K, pf.W, digits, w, pf.x, pf.dtype, pf.exp_mode, pf.fexp, pf.exp, pf.status};
        const long long gb4 = (n + BLOCK / 4 - 1) / (BLOCK / 4);
        HIPCHK(fbgp_launch_w(pg, (int)std::max<long long>(1, std::min<long long>(gb4, (long long)occH * c->cus / 2)), st));
      }
      const long long gb4 = (n + BLOCK / GRP_TPI - 1) / (BLOCK / GRP_TPI), gb8 = (n + BLOCK / 8 - 1) / (BLOCK / 8);
      FbgGarnerParams gh{w, n, c->d_fb_m0, c->d_fb_m8, c->d_fb_coefR, c->fb_mprime0};
      HIPCHK(grp_launch_garner(gh, (int)std::max<long long>(1, std::min<long long>(gb4, (long long)occH * c->cus)), st));
      // c = w_q + q^2 h on lanes (kernels_sgp.hpp k_sgp_fin): its intermediates' top 2S rows go to the digit buffer
      // (2K rows, dead by now; K >= S at every window the ladder has)
      if (c->d_sgp_q && c->ct_words == SGPF_CT_WORDS && pf.K >= SGP_S && sgp_fin_enabled()) {
        const SgpFinParams sf{w, digits, n, c->d_sgp_q, e.ct + (size_t)off * c->ct_words, c->ct_words};
        HIPCHK(sgp_launch_fin(sf, c->cus, st));
      } else {
        FbgFinParams gf{w, SB, n, c->d_N, c->d_fb_q2Rn, c->mprime_N, e.ct + (size_t)off * c->ct_words, c->ct_words};
        HIPCHK(grp_launch_fin(gf, (int)std::max<long long>(1, std::min<long long>(gb8, (long long)occC * c->cus)), st));
      }
      stage_mark(c, 3, st);
      continue;
    }
    if (c->fb_pair_s) {   // Garner on pairs (kernels_fbp.hpp)
      int occP = 1;
      fbp_fin_occupancy(c->fb_pair_s, &occP);
      FbpFinParams pp{w, n, c->d_fbp_fin_p, c->d_fbp_fin_cs, c->fbp_fin_mprime, e.ct + (size_t)off * c->ct_words,
                      c->ct_words};
      pp.g = guard_args(c, 0, 0, (unsigned long long)n * c->ct_words, w_words);
      const long long nb = (n + LANE_BLOCK - 1) / LANE_BLOCK;
      HIPCHK(fbp_launch_fin(c->fb_pair_s, pp, (int)std::max<long long>(1, std::min<long long>(nb, (long long)occP * c->cus)), st));
      stage_mark(c, 3, st);
      continue;
    }
    (void)gxG;
  }
  return 0;
}

// ------------------------------------------------------------------ public-key fixed bases (kernels_pfb.hpp)
// A party without the private key samples r = g_0^e_0 g_1^e_1 ... g_32^e_32 mod n from 33 bases it drew itself
// (g_0 with Jacobi symbol -1) and exponents from the element's ChaCha20 stream (e_0: nb + 64 bits, e_j: 96 bits),
// and gets r^n mod n^2 as a product of table rows (distribution argument, break-even).
static bool pfb_supported(const pai_ctx* c) {
  return c->pe_ok && c->ct_words == 2 * PFB_PW && (size_t)c->nb + 24 <= (size_t)LB * PFB_S;
}

static void pfb_digit_counts(const pai_ctx* c, int W, int* K0, int* KS) {
  *K0 = (c->nb + PFB_E0_EXTRA + W - 1) / W;
  *KS = (PFB_TBITS + W - 1) / W;
}

static uint64_t pfb_bytes(const pai_ctx* c, int W) {
  int K0, KS;
  pfb_digit_counts(c, W, &K0, &KS);
  return (uint64_t)(K0 + PFB_SHORT * KS) * (1ull << W) * PFB_ROW4 * 16ull;
}

static int pfb_choose_window(pai_ctx* c) {
  if (!c->pfb_W) c->pfb_W = pfb_default_window();
  const uint64_t budget = fb_budget(c);
  for (int w : {20, 16, 12})
    if (w <= c->pfb_W && pfb_bytes(c, w) <= budget) return w;
  return 0;
}

static void pfb_release(pai_ctx* c) {
  for (void* q : c->pfb_mem) (void)hipFree(q);
  c->pfb_mem.clear();
  for (void* q : c->pfb_tables) TableArena::get().free(q);
  c->pfb_tables.clear();
  c->d_pfb = nullptr;
  c->d_sgp_pfb = nullptr;
}

static int pfb_unavailable(pai_ctx* c, const std::string& why) {
  pfb_release(c);
  (void)hipGetLastError();
  c->pfb_state = pai_ctx::FB_UNAVAILABLE;
  c->pfb_reason = why;
  return 0;
}

template <typename T>
static int upload_pfb(pai_ctx* c, const std::vector<T>& v, T** out) {
  void* q = nullptr;
  HIPCHK(hipMalloc(&q, std::max<size_t>(v.size(), 1) * sizeof(T)));
  c->pfb_mem.push_back(q);
  if (!v.empty()) HIPCHK(hipMemcpy(q, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (T*)q;
  return 0;
}

// Jacobi symbol (a | n) for odd n > 0: halvings (second supplement), swaps (reciprocity), subtractions
static int jacobi(HBig a, HBig n) {
  if (cmp(a, n) >= 0) a = mod(a, n);
  int t = 1;
  while (!a.is_zero()) {
    while (!a.is_odd()) {
      a = shr1(a);
      const uint32_t r = n.w[0] & 7u;
      if (r == 3 || r == 5) t = -t;
    }
    if (cmp(a, n) < 0) {
      std::swap(a, n);
      if ((a.w[0] & 3u) == 3u && (n.w[0] & 3u) == 3u) t = -t;
    }
    a = sub(a, n);
  }
  return (n.w.size() == 1 && n.w[0] == 1u) ? t : 0;
}

// uniform in [2, n) from the OS CSPRNG (rejection sampling on bits(n) bits)
static bool random_below(const HBig& n, HBig* out) {
  const size_t nw = n.w.size();
  const int top = (int)(n.bits() - 32 * (nw - 1));
  for (int tries = 0; tries < 1000; ++tries) {
    HBig r;
    r.w.assign(nw, 0);
    size_t got = 0;
    while (got < nw * 4) {
      const ssize_t k = getrandom((char*)r.w.data() + got, nw * 4 - got, 0);
      if (k <= 0) return false;
      got += (size_t)k;
    }
    if (top < 32) r.w[nw - 1] &= (1u << top) - 1u;
    r.trim();
    if (cmp(r, n) < 0 && r.bits() > 1) {
      *out = r;
      return true;
    }
  }
  return false;
}

static int ensure_pfb(pai_ctx* c) {
  if (c->pfb_state == pai_ctx::FB_READY) return 1;
  if (c->pfb_state == pai_ctx::FB_UNAVAILABLE) return 0;
  if (!pfb_supported(c)) return pfb_unavailable(c, "the public fixed-base kernels need a 1537..2048-bit n");
  const int W = pfb_choose_window(c);
  if (!W) return pfb_unavailable(c, "tables do not fit the device memory budget");
  SetupTrace tr_all("ensure_pfb");
  const auto t0 = std::chrono::steady_clock::now();
  int K0, KS;
  pfb_digit_counts(c, W, &K0, &KS);
  const int K = K0 + PFB_SHORT * KS;
  const HBig& n = c->n;
  std::optional<SetupTrace> tr_h(std::in_place, "  pfb host prep (bases, constants)");
  if (c->pfb_bases.empty()) {
    HBig g;
    do {
      if (!random_below(n, &g)) return pfb_unavailable(c, "no randomness for the bases");
    } while (jacobi(g, n) != -1);   // g_0: Jacobi symbol -1, so the publicly visible symbol of c mod n is uniform
    c->pfb_bases.push_back(g);
    for (int j = 0; j < PFB_SHORT; ++j) {
      if (!random_below(n, &g)) return pfb_unavailable(c, "no randomness for the bases");
      c->pfb_bases.push_back(g);
    }
  }
  const HBig& n2 = c->N;
  const size_t RS = (size_t)LB * PFB_S;
  auto split = [&](const HBig& v) {   // v < n^2 -> [v mod n: S limbs][v div n: S limbs]
    const HBig qt = div_big(v, n), rm = sub(v, mul(qt, n));
    std::vector<uint32_t> out = rm.limbs(PFB_S, LB), b = qt.limbs(PFB_S, LB);
    out.insert(out.end(), b.begin(), b.end());
    return out;
  };
  const HBig oneR = mul_pow2_mod(HBig(1), RS, n2);
  const HBig R2 = mul_pow2_mod(oneR, RS, n2);
  const HBig X = mod(sub(add(n, HBig(1)), mul_pow2_mod(HBig(1), RS, n)), n);   // (1 - R) mod n
  std::vector<uint32_t> gl;
  for (const HBig& g : c->pfb_bases) {
    const std::vector<uint32_t> v = g.limbs(PFB_S, LB);
    gl.insert(gl.end(), v.begin(), v.end());
  }
  tr_h.reset();
  pfb_release(c);
  std::optional<SetupTrace> tr_m(std::in_place, "  pfb uploads + hipMalloc");
  uint32_t *dn, *dx, *done, *dr2, *dgl, *dnw, *dbases, *dlohi;
  uint4* dtab;
  int rc;
  if ((rc = upload_pfb(c, n.limbs(PFB_S, LB), &dn)) || (rc = upload_pfb(c, X.limbs(PFB_S, LB), &dx)) ||
      (rc = upload_pfb(c, split(oneR), &done)) || (rc = upload_pfb(c, split(R2), &dr2)) ||
      (rc = upload_pfb(c, gl, &dgl)) || (rc = upload_pfb(c, n.words(PFB_PW), &dnw)))
    return pfb_unavailable(c, pai_last_error());
  void *vb = nullptr, *vl = nullptr, *vt = nullptr, *vinv = nullptr, *vpre = nullptr;
  void* vcv = nullptr;
  if (hipMalloc(&vcv, (size_t)2 * K * PFB_S * 4) != hipSuccess) return pfb_unavailable(c, "table allocation failed");
  c->pfb_mem.push_back(vcv);
  if (hipMalloc(&vinv, (size_t)K * 2 * FB_LO * PFB_S * 4) != hipSuccess) return pfb_unavailable(c, "table allocation failed");
  c->pfb_mem.push_back(vinv);
  if (hipMalloc(&vpre, (size_t)2 * K * ((size_t)1 << (W - W / 2)) * PFB_S * 4) != hipSuccess)
    return pfb_unavailable(c, "table allocation failed");
  c->pfb_mem.push_back(vpre);
  if (hipMalloc(&vb, (size_t)K * 2 * 2 * PFB_S * 4) != hipSuccess) return pfb_unavailable(c, "table allocation failed");
  c->pfb_mem.push_back(vb);
  if (hipMalloc(&vl, (size_t)K * 2 * FB_LO * 2 * PFB_S * 4) != hipSuccess) return pfb_unavailable(c, "table allocation failed");
  c->pfb_mem.push_back(vl);
  if (!(vt = TableArena::get().alloc(c->device, ((size_t)K << W) * PFB_ROW4 * sizeof(uint4))))
    return pfb_unavailable(c, "table allocation failed");
  c->pfb_tables.push_back(vt);
  dbases = (uint32_t*)vb;
  dlohi = (uint32_t*)vl;
  dtab = (uint4*)vt;
  PfbConst pc{};
  pc.g = FbgpHalf{(const uint32_t*)dtab, dn, dx, done, dbases, dlohi, nullptr, nullptr, nullptr, nullptr,
                  mont_prime(n, LB), 0u, (uint32_t*)vinv, (uint32_t*)vpre, (uint32_t*)vcv};
  pc.table = dtab;
  pc.gl = dgl;
  pc.r2 = dr2;
  pc.nw = dnw;
  pc.nbits = (int)n.bits();
  pc.nbases = (int)c->pfb_bases.size();
  pc.K = K;
  pc.W = W;
  pc.K0 = K0;
  pc.KS = KS;
  std::vector<PfbConst> pv{pc};
  PfbConst* dpc = nullptr;
  if ((rc = upload_pfb(c, pv, &dpc))) return pfb_unavailable(c, pai_last_error());
  SgpHalf* dsgp = nullptr;
  if (sgp_enabled()) {
    SgpHalf sh{};
    if ((rc = sgp_make_half(n, HBig(1), K, dtab,
                            [&](const std::vector<uint32_t>& v, uint32_t** o) { return upload_pfb(c, v, o); }, &sh)))
      return pfb_unavailable(c, pai_last_error());
    std::vector<SgpHalf> shv{sh};
    if ((rc = upload_pfb(c, shv, &dsgp))) return pfb_unavailable(c, pai_last_error());
  }
  tr_m.reset();
  const auto t1 = std::chrono::steady_clock::now();
  {
    SetupTrace tr_1("  pfb phase 1 (chains, lohi, inv_fwd)");
    if (pfb_build_phase1(dpc, pc.nbases, K, W, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return pfb_unavailable(c, "table construction failed");
  }
  {
    SetupTrace tr_i("  pfb host invert");
    if (pair_host_invert(n, (uint32_t*)vcv, 2 * K, PFB_S)) return pfb_unavailable(c, pai_last_error());
  }
  {
    SetupTrace tr_2("  pfb phase 2 (inv_bwd, fill)");
    if (pfb_build_phase2(dpc, K, W, dtab, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return pfb_unavailable(c, "table construction failed");
  }
  SetupTrace tr_f("  pfb scratch frees");
  for (void* q : {vb, vl, vinv, vpre, vcv}) {   // build scratch
    c->pfb_mem.erase(std::find(c->pfb_mem.begin(), c->pfb_mem.end(), q));
    (void)hipFree(q);
  }
  const auto t2 = std::chrono::steady_clock::now();
  c->d_pfb = dpc;
  c->d_sgp_pfb = dsgp;
  c->pfb_host_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
  c->pfb_dev_ms = std::chrono::duration<float, std::milli>(t2 - t1).count();
  c->pfb_table_bytes = pfb_bytes(c, W);
  c->pfb_K = K;
  c->pfb_K0 = K0;
  c->pfb_KS = KS;
  c->pfb_W_used = W;
  c->pfb_state = pai_ctx::FB_READY;
  return 1;
}

// Break-even of the public tables, from measurements on one MI355X (tools/pfb_breakeven.py): the build takes 0.114 s +
// 1.91 ns per row on memory the process has not released before (0.117 / 0.155 / 0.648 s at W = 12 / 16 / 20, round 5,
// profiles/r05_pfb_breakeven_before.json; round 6: 0.094 / 0.137 s at W = 12 / 16), and each element then costs
// 1 / rate(W) on k_sgp (round 6, the final library: 3.00 M / 3.93 M / 4.78 M enc/s, profiles/r06e_pfb_breakeven.json)
// instead of 1 / 552 k on the factored k_pe_* chain (round 5's 503 k predated that chain) -- 1.81 us -- so the
// break-even is ~100 k elements at the default W = 16
static long long pfb_threshold(pai_ctx* c) {
  if (c->pfb_state != pai_ctx::FB_UNTRIED || !pfb_supported(c)) return 0;
  if (const char* e = getenv("FLEXPAI_PFB_MIN_ELEMS")) return atoll(e);
  const int W = pfb_choose_window(c);
  if (!W) return 0;
  int K0, KS;
  pfb_digit_counts(c, W, &K0, &KS);
  const double build_s = 0.114 + (double)(K0 + PFB_SHORT * KS) * (double)(1ull << W) * 1.91e-9;
  const double rate = W >= 20 ? 4.78e6 : W >= 16 ? 3.93e6 : 3.00e6;
  const double save_s = 1.0 / 5.52e5 - 1.0 / rate;
  return (long long)(build_s / save_s) + 1;
}

static bool pfb_wanted(pai_ctx* c, long long n) {
  if (c->pfb_state != pai_ctx::FB_UNTRIED) return true;
  if (c->pfb_call) return c->pfb_call > 0;
  c->pfb_seen += n;
  return c->pfb_seen >= pfb_threshold(c);
}

// digits, k_pfb, k_pe_fin per chunk of CRT_CHUNK elements
static int launch_pfb(pai_ctx* c, const EncParams& e, hipStream_t st) {
  const long long N = e.n;
  const long long chunk = std::min(N, CRT_CHUNK);
#if FLEXPAI_XCHECK
  int occ = 1;
  pfb_occupancy(&occ);
  constexpr int GPB = BLOCK / PFB_TPI;
  const int gx = (int)std::max<long long>(1, std::min<long long>((chunk + GPB - 1) / GPB, (long long)occ * c->cus));
#else
  if (!c->d_sgp_pfb) return fail(PAI_ERR_KEY, "public fixed-base encrypt: no split-pair tables");
#endif
  const size_t dbytes = (size_t)c->pfb_K * 4, xbytes = (size_t)2 * PFB_SP * 4;
  int rc;
  if ((rc = ensure_work(c, (dbytes + xbytes) * chunk))) return rc;
  uint32_t* digits = (uint32_t*)c->d_work;
  uint32_t* xw = (uint32_t*)((char*)c->d_work + dbytes * chunk);
  const size_t esz = e.dtype == PAI_F32 ? 4 : 8;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    PfbDigitParams pd{};
    pd.n = n;
    std::memcpy(pd.rng_key, e.rng_key, sizeof(pd.rng_key));
    pd.index_base = e.index_base + (unsigned long long)off;
    pd.K = c->pfb_K;
    pd.W = c->pfb_W_used;
    pd.digits = digits;
    const int gD = (int)std::max<long long>(1, std::min<long long>((long long)8 * c->cus, (n + PFB_DIG_BLOCK - 1) / PFB_DIG_BLOCK));
    stage_mark(c, 0, st);
    HIPCHK(pfb_launch_digits(pd, gD, st));
    stage_mark(c, 1, st);
    const PfbParams pp{c->d_pfb, n, digits, (const char*)e.x + (size_t)off * esz, e.dtype, e.exp_mode, e.fexp,
                       e.exp + off, e.status ? e.status + off : nullptr, xw};
    if (c->d_sgp_pfb) {   // split pairs (kernels_sgp.hpp)
      int occS = 1;
      sgp_occupancy(&occS);
      SgpParams sp{c->d_sgp_pfb, n, c->pfb_K, c->pfb_W_used, digits, xw, pp.x, pp.dtype, pp.exp_mode, pp.fexp, pp.exp,
                   pp.status};
      sp.g = guard_args(c, (unsigned long long)c->pfb_K << c->pfb_W_used, (unsigned long long)c->pfb_K * chunk,
                        (unsigned long long)2 * PFB_SP * chunk, 0);
      const long long nb = (n + SGP_PAIRS - 1) / SGP_PAIRS;
      HIPCHK(sgp_launch(sp, (int)std::max<long long>(1, std::min<long long>(nb, (long long)occS * c->cus)), 1, st));
    } else {
#if FLEXPAI_XCHECK
      HIPCHK(pfb_launch(pp, (int)std::min<long long>(gx, (n + GPB - 1) / GPB), st));
#endif
    }
    stage_mark(c, 2, st);
    PeParams pf{};
    pf.k = c->d_pe;
    pf.n = n;
    pf.xw = xw;
    pf.ct = e.ct + (size_t)off * c->ct_words;
    pf.ct_words = c->ct_words;
    HIPCHK(pe_launch_fin(pf, c->cus, st));
    stage_mark(c, 3, st);
  }
  return 0;
}

int pai_ctx_public_fb_prepare(pai_ctx* c) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  HIPCHK(hipSetDevice(c->device));
  if (!ensure_pfb(c)) return fail(PAI_ERR_KEY, "public fixed-base obfuscation not available: " + c->pfb_reason);
  return 0;
}

int pai_ctx_public_fb_set_bases(pai_ctx* c, const uint8_t* bases_le, size_t base_bytes, int nbases) {
  if (!c || !bases_le || base_bytes == 0) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: null argument");
  CtxLock lk(c);
  if (nbases != PFB_NBASES) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: wrong number of bases");
  std::vector<HBig> bs;
  for (int j = 0; j < nbases; ++j) {
    HBig g = HBig::from_le_bytes(bases_le + (size_t)j * base_bytes, base_bytes);
    if (g.bits() < 2 || cmp(g, c->n) >= 0) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: need 1 < g < n");
    // the distribution argument needs units, g_0 with Jacobi symbol -1 (so that (c mod n | n) is
    // uniform) and distinct bases: reject anything weaker rather than sample a visibly biased r
    if (inv_mod(g, c->n).is_zero()) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: a base is not a unit mod n");
    for (const HBig& h : bs)
      if (cmp(h, g) == 0) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: repeated base");
    if (j == 0 && jacobi(g, c->n) != -1)
      return fail(PAI_ERR_ARG, "pai_ctx_public_fb_set_bases: g_0 must have Jacobi symbol -1 mod n");
    bs.push_back(g);
  }
  HIPCHK(hipSetDevice(c->device));
  pfb_release(c);
  c->pfb_bases = bs;
  c->pfb_state = pai_ctx::FB_UNTRIED;
  return 0;
}

int pai_ctx_public_fb_info(pai_ctx* c, uint8_t* bases_le, size_t base_bytes, int* nbases, int* digits, int* window,
                           int* e0_digits) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (c->pfb_state != pai_ctx::FB_READY) return fail(PAI_ERR_KEY, "public fixed-base tables are not resident");
  if (bases_le) {
    for (size_t j = 0; j < c->pfb_bases.size(); ++j) {
      const std::vector<uint32_t> w = c->pfb_bases[j].words((base_bytes + 3) / 4);
      if (c->pfb_bases[j].bits() > 8 * base_bytes) return fail(PAI_ERR_ARG, "pai_ctx_public_fb_info: base_bytes too small");
      std::memcpy(bases_le + j * base_bytes, w.data(), base_bytes);
    }
  }
  if (nbases) *nbases = (int)c->pfb_bases.size();
  if (digits) *digits = c->pfb_K;
  if (window) *window = c->pfb_W_used;
  if (e0_digits) *e0_digits = c->pfb_K0;
  return 0;
}

int pai_ctx_public_fb_policy(pai_ctx* c, long long* seen, long long* threshold) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (seen) *seen = c->pfb_seen;
  if (threshold) *threshold = pfb_threshold(c);
  return 0;
}

// public-key encryption on split pairs (kernels_pe.hpp, engine_pe.hip), in chunks of CRT_CHUNK elements
// the modulus of a batch inversion on the group engine: n^2 (ciphertexts, TPI = tpi_e) or n (the public-key chain's
// bases, TPI = 2)
struct InvMod {
  int tpi, W, S;             // group size, words per value, limbs (TPI L)
  const uint32_t *N, *R2, *oneR;
  uint32_t mprime;
  const HBig* mod;
};
static int batch_invert(pai_ctx* c, uint32_t* x, const uint8_t* flag, long long n, hipStream_t st, const InvMod& md);
static int batch_invert(pai_ctx* c, uint32_t* x, const uint8_t* flag, long long n, hipStream_t st);
static int batch_invert_async(pai_ctx* c, uint32_t* x, long long n, hipStream_t st, const InvMod& md, uint32_t** d_noinv);

// Chunks below this many elements take the general chain: the factored one saves ~0.2 us per element (k_pe_pow_f
// against k_pe_pow) and costs the batch inversion's fixed ~1-2 ms of short dependent launches. $FLEXPAI_PEF_MIN
// overrides (the parity tests force both chains on the same inputs).
static long long pef_min_elems() {
  if (const char* e = getenv("FLEXPAI_PEF_MIN")) return atoll(e);
  return 16384;
}

// public-key encryption for n <= 1024 bits on pairs (kernels_pe1.hpp, engine_pe1.hip), in chunks of CRT_CHUNK elements;
// stage times: the obfuscator words + k_dec_pre_pair, k_pe1_pow, k_pe1_fin
static int launch_pe1(pai_ctx* c, const EncParams& e, hipStream_t st) {
  const long long N = e.n;
  const long long chunk = std::min(N, CRT_CHUNK);
  const int RW = e.obf == PAI_OBF_GIVEN ? e.r_words : e.rng_words;
  const int kchunks = 2;   // r's digits in two chunks of S (zeros past its words): the constant is the pair of R^3
  if (RW <= 0 || 32 * RW > kchunks * LB * PE1_S) return fail(PAI_ERR_ARG, "1024-bit pair encrypt: obfuscator too wide");
  int occ = 1;
  pe1_occupancy(&occ);
  const long long lb = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  const int gx = (int)std::max<long long>(1, std::min<long long>(lb, (long long)occ * c->cus));
  int rc = ensure_scratch(c, (size_t)gx * LANE_BLOCK * lane_scratch_words<2 * PE1_S>() * 4);
  if (rc) return rc;
  const size_t rwb = (size_t)RW * 4, xwb = (size_t)2 * PE1_S * 4;   // per element
  if ((rc = ensure_work(c, (rwb + xwb) * chunk))) return rc;
  const size_t esz = e.dtype == PAI_F32 ? 4 : 8;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    hipEvent_t* ev = stage_chunk(c);
    if (ev) c->nev = 4;
    Pe1Params p{};
    p.x = (const char*)e.x + (size_t)off * esz;
    p.dtype = e.dtype;
    p.exp_mode = e.exp_mode;
    p.fexp = e.fexp;
    p.obf = e.obf;
    p.r = e.r ? e.r + (size_t)off * e.r_stride : nullptr;
    p.r_stride = e.r_stride;
    p.r_words = e.r_words;
    p.rng_words = e.rng_words;
    std::memcpy(p.rng_key, e.rng_key, sizeof(p.rng_key));
    p.index_base = e.index_base + (unsigned long long)off;
    p.n = n;
    p.nl = c->d_pe1_n;
    p.one = c->d_pe1_one;
    p.prog = c->d_pe1_prog;
    p.nprog = c->pe1_nprog;
    p.r2n = c->d_pe1_r2n;
    p.mprime = c->pe1_mprime;
    p.rw = (uint32_t*)c->d_work;
    p.rw_words = RW;
    p.xw = (uint32_t*)((char*)c->d_work + rwb * chunk);
    p.scratch = (uint32_t*)c->d_scratch;
    p.ct = e.ct + (size_t)off * c->ct_words;
    p.exp = e.exp + off;
    p.status = e.status ? e.status + off : nullptr;
    p.ct_words = c->ct_words;
    const DecPairPreParams pre{c->d_pe1_half, n, p.rw, RW, kchunks, p.xw};
    HIPCHK(pe1_launch(p, pre, gx, c->cus, st, ev));
  }
  return 0;
}

static int launch_pe(pai_ctx* c, const EncParams& e, hipStream_t st) {
  const long long N = e.n;
  const long long chunk = std::min(N, CRT_CHUNK);
  Dec4Geom g;
  pe_geometry(c->cus, chunk, &g);
  int rc = ensure_scratch(c, g.scratch_bytes);
  if (rc) return rc;
  const size_t xbytes = (size_t)2 * D4_S * 4;   // per element, + 8 for M
  const size_t awbytes = c->pef_ok ? (size_t)c->pt_words * 4 : 0, iobytes = c->pef_ok ? (size_t)D4_S * 4 : 0;
  if ((rc = ensure_work(c, (xbytes + 8 + awbytes + iobytes) * chunk))) return rc;
  const size_t esz = e.dtype == PAI_F32 ? 4 : 8;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    hipEvent_t* ev = stage_chunk(c);
    if (ev) c->nev = 4;
    PeParams p{};
    p.k = c->d_pe;
    p.x = (const char*)e.x + (size_t)off * esz;
    p.dtype = e.dtype;
    p.exp_mode = e.exp_mode;
    p.fexp = e.fexp;
    p.obf = e.obf;
    p.r = e.r ? e.r + (size_t)off * e.r_stride : nullptr;
    p.r_stride = e.r_stride;
    p.r_words = e.r_words;
    p.rng_words = e.rng_words;
    std::memcpy(p.rng_key, e.rng_key, sizeof(p.rng_key));
    p.index_base = e.index_base + (unsigned long long)off;
    p.n = n;
    p.xw = (uint32_t*)c->d_work;
    p.M = (int64_t*)((char*)c->d_work + xbytes * chunk);
    p.scratch = (uint32_t*)c->d_scratch;
    p.ct = e.ct + (size_t)off * c->ct_words;
    p.ct_words = c->ct_words;
    p.exp = e.exp + off;
    p.status = e.status ? e.status + off : nullptr;
    if (!c->pef_ok || n < pef_min_elems()) {
      HIPCHK(pe_launch(p, g, st, ev));
      continue;
    }
    // the factored chain: A_r's batch inversion mod n (one host inversion per chunk), iota, k_pe_pow_f
    p.aw = (uint32_t*)((char*)c->d_work + (xbytes + 8) * chunk);
    p.aw_words = c->pt_words;
    p.iota = (uint32_t*)((char*)p.aw + awbytes * chunk);
    HIPCHK(pe_launch_pre_aw(p, g, st, ev));
    uint32_t* noinv = nullptr;
    rc = batch_invert_async(c, p.aw, n, st,
                            InvMod{2, c->pt_words, 2 * L, c->d_pe_n, c->d_pe_r2, c->d_pe_oneR, c->pe_mprime, &c->n}, &noinv);
    if (rc) return rc;
    // an A_r that shares a factor with n (no inverse): the device flag sends this chunk down the general chain
    p.noinv = noinv;
    HIPCHK(pe_launch_iota_pow_f(p, g, st, ev));
  }
  return 0;
}

// k_crt_fin over elements [off, off + n) of the call: c = (u_p q^2 + u_q p^2) c0 mod n^2 from u [2][sb][n]
static int crt_finish(pai_ctx* c, const EncParams& e, const uint32_t* u, int sb, long long off, long long n,
                      hipStream_t st) {
  const size_t esz = e.dtype == PAI_F32 ? 4 : 8;
  CrtFinParams f{};
  f.x = (const char*)e.x + (size_t)off * esz;
  f.dtype = e.dtype;
  f.exp_mode = e.exp_mode;
  f.fexp = e.fexp;
  f.u = u;
  f.sb = sb;
  f.n = n;
  f.N = c->d_N;
  f.nl = c->d_nl;
  f.kq = c->d_kq;
  f.kp = c->d_kp;
  f.mprime = c->mprime_N;
  f.ct = e.ct + (size_t)off * c->ct_words;
  f.exp = e.exp + off;
  f.status = e.status ? e.status + off : nullptr;
  f.ct_words = c->ct_words;
  switch (c->tpi_e) {
    case 2: return launch_crt_fin<2>(c, f, st);
    case 4: return launch_crt_fin<4>(c, f, st);
    case 8: return launch_crt_fin<8>(c, f, st);
  }
  return fail(PAI_ERR_KEY, "CRT finish: unsupported group size");
}

// A call of at most crtw_max elements: both exponentiations on 16-lane rows (k_crt_w, kernels_crtw.hpp), then
// k_crt_fin. Same constants, op lists and output as k_crt_a + k_crt_b_pair; stage times: k_crt_w, k_crt_fin.
static int launch_crtw(pai_ctx* c, const EncParams& e, int sa, int sb, int r_words, int kchunks, hipStream_t st) {
  const long long N = e.n;
  int rc = ensure_work(c, (size_t)2 * sb * 4 * N);
  if (rc) return rc;
  uint32_t* u = (uint32_t*)c->d_work;
  crtw::Params p{};
  p.ha = c->d_crt_a;
  p.hb = c->d_crt_b;
  p.n = N;
  p.obf = e.obf;
  p.r = e.r;
  p.r_stride = e.r_stride;
  p.r_words = r_words;
  std::memcpy(p.rng_key, e.rng_key, sizeof(p.rng_key));
  p.index_base = e.index_base;
  p.kchunks = kchunks;
  p.out = u;
  stage_mark(c, 0, st);
  HIPCHK(crtw_launch(sa, p, st));
  stage_mark(c, 1, st);
  if ((rc = crt_finish(c, e, u, sb, 0, N, st))) return rc;
  stage_mark(c, 2, st);
  return 0;
}

template <int SA, int SB>
static int launch_crt(pai_ctx* c, const EncParams& e, hipStream_t st) {
  static_assert(SB == 2 * SA || SB == 2 * SA - 1, "stage sizes");
  if (e.obf == PAI_OBF_RNG && c->fb_enabled && fb_wanted(c, e.n) && ensure_fb(c)) {
    const int rc = launch_fb(c, e, st);
    return rc ? rc : guard_collect(c, st);
  }
  const long long N = e.n;
  const int r_words = e.obf == PAI_OBF_GIVEN ? e.r_words : e.rng_words;
  const int kchunks = (32 * r_words + LB * SA - 1) / (LB * SA);
  if (kchunks > KMAX_CHUNKS || (e.obf == PAI_OBF_RNG && r_words > RBUF_WORDS))
    return fail(PAI_ERR_ARG, "CRT encrypt: obfuscator too wide");
  if (N <= c->crtw_max) return launch_crtw(c, e, SA, SB, r_words, kchunks, st);
  const long long chunk = std::min(N, CRT_CHUNK);
  int occA = 1, occB = 1;
  if (crt_lane_occupancy(SA, &occA, &occB)) return fail(PAI_ERR_KEY, "CRT encrypt: unsupported size");
  const bool bpair = c->crt_pair_ok;   // stage B on pairs (kernels_pair.hpp)
#if !FLEXPAI_XCHECK
  if (!bpair) return fail(PAI_ERR_KEY, "CRT encrypt: no pair constants");
#endif
  if (bpair && crt_b_pair_occupancy(SA, &occB)) return fail(PAI_ERR_KEY, "CRT encrypt: unsupported size");
  const long long lanes_blocks = (chunk + LANE_BLOCK - 1) / LANE_BLOCK;
  const int gxA = (int)std::max<long long>(1, std::min<long long>(lanes_blocks, (long long)occA * c->cus / 2));
  const int gxB = (int)std::max<long long>(1, std::min<long long>(lanes_blocks, (long long)occB * c->cus / 2));
  const size_t scrA = (size_t)2 * gxA * LANE_BLOCK * lane_scratch_words<SA>() * 4;
  const size_t scrB = (size_t)2 * gxB * LANE_BLOCK * lane_scratch_words<SB>() * 4;
  int rc = ensure_scratch(c, std::max(scrA, scrB));
  if (rc) return rc;
  const size_t ybytes = (size_t)2 * SA * 4;   // per element
  if ((rc = ensure_work(c, (ybytes + (size_t)2 * SB * 4) * chunk))) return rc;
  uint32_t* y = (uint32_t*)c->d_work;
  uint32_t* u = (uint32_t*)((char*)c->d_work + ybytes * chunk);
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    CrtParams pa{};
    pa.halves = c->d_crt_a;
    pa.n = n;
    pa.obf = e.obf;
    pa.r = e.r ? e.r + (size_t)off * e.r_stride : nullptr;
    pa.r_stride = e.r_stride;
    pa.r_words = r_words;
    std::memcpy(pa.rng_key, e.rng_key, sizeof(pa.rng_key));
    pa.index_base = e.index_base + (unsigned long long)off;
    pa.kchunks = kchunks;
    pa.out = y;
    pa.scratch = (uint32_t*)c->d_scratch;
    const int gA = (int)std::min<long long>(gxA, (n + LANE_BLOCK - 1) / LANE_BLOCK);
    stage_mark(c, 0, st);
    HIPCHK(crt_launch_a(SA, pa, gA, st));
    stage_mark(c, 1, st);
    HIPCHK(hipGetLastError());
    CrtParams pb{};
    pb.halves = bpair ? c->d_crtp_b : c->d_crt_b;
    pb.n = n;
    pb.yin = y;
    pb.out = u;
    pb.scratch = (uint32_t*)c->d_scratch;
    const int gB = (int)std::min<long long>(gxB, (n + LANE_BLOCK - 1) / LANE_BLOCK);
    HIPCHK(crt_b_pair_launch(SA, pb, gB, st));
    HIPCHK(hipGetLastError());
    stage_mark(c, 2, st);
    if ((rc = crt_finish(c, e, u, SB, off, n, st))) return rc;
    stage_mark(c, 3, st);
  }
  return 0;
}

int pai_encrypt_dev(pai_ctx* c, int dtype, const void* d_x, size_t N, int exp_mode, int32_t fixed_exp, int obf_mode,
                    const uint32_t* d_r_words, size_t r_stride_words, size_t r_words, const uint8_t* rng_key32,
                    uint64_t index_base, uint32_t* d_ct, int32_t* d_exp, int32_t* d_status, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (N == 0) return 0;
  if (dtype < 0 || dtype > 2 || !d_x || !d_ct || !d_exp) return fail(PAI_ERR_ARG, "pai_encrypt_dev: bad arguments");
  if (obf_mode == PAI_OBF_GIVEN && (!d_r_words || r_words == 0 || r_words > (size_t)c->ct_words))
    return fail(PAI_ERR_ARG, "pai_encrypt_dev: r must be given with 0 < r_words <= ct_words");
  if (obf_mode == PAI_OBF_RNG && !rng_key32) return fail(PAI_ERR_ARG, "pai_encrypt_dev: rng key required");
  if (obf_mode < 0 || obf_mode > 2) return fail(PAI_ERR_ARG, "pai_encrypt_dev: bad obf_mode");
  HIPCHK(hipSetDevice(c->device));
  stage_reset(c);
  EncParams p{};
  p.x = d_x;
  p.dtype = dtype;
  p.exp_mode = exp_mode;
  p.fexp = fixed_exp;
  p.obf = obf_mode;
  p.r = d_r_words;
  p.r_stride = (long long)r_stride_words;
  p.r_words = (int)r_words;
  p.rng_words = (c->nb + 64 + 31) / 32;
  if (rng_key32)
    for (int i = 0; i < 8; ++i) std::memcpy(&p.rng_key[i], rng_key32 + 4 * i, 4);
  p.index_base = index_base;
  p.ct = d_ct;
  p.exp = d_exp;
  p.status = d_status;
  p.n = (long long)N;
  p.N = c->d_N;
  p.R2 = c->d_R2;
  p.nl = c->d_nl;
  p.mprime = c->mprime_N;
  p.prog = c->d_prog;
  p.nprog = c->nprog;
  p.ct_words = c->ct_words;
  hipStream_t st = (hipStream_t)stream;
  if (obf_mode == PAI_OBF_RNG && c->fbg_ok && c->crt_enabled && c->fb_enabled && fb_wanted(c, p.n) && ensure_fb(c)) {
    const int rc = launch_fb(c, p, st);
    return rc ? rc : guard_collect(c, st);
  }
  if (obf_mode != PAI_OBF_NONE && c->rows_sa && c->crt_enabled && p.n <= c->crtw_max) {   // 4096 bits, protocol-sized
    const int r_words = obf_mode == PAI_OBF_GIVEN ? p.r_words : p.rng_words;
    const int kchunks = (32 * r_words + LB * c->rows_sa - 1) / (LB * c->rows_sa);
    if (kchunks <= KMAX_CHUNKS && r_words <= crtw::RW_WORDS)
      return launch_crtw(c, p, c->rows_sa, 2 * c->rows_sa, r_words, kchunks, st);
  }
  if (obf_mode != PAI_OBF_NONE && c->crt_ok && c->crt_enabled) {
    if (c->crt_sa == 19) return launch_crt<19, 37>(c, p, st);
    if (c->crt_sa == 37) return launch_crt<37, 74>(c, p, st);
  }
  if (obf_mode == PAI_OBF_RNG && c->pfb_enabled && pfb_supported(c) && pfb_wanted(c, p.n) && ensure_pfb(c)) {
    const int rc = launch_pfb(c, p, st);
    return rc ? rc : guard_collect(c, st);
  }
  if (obf_mode != PAI_OBF_NONE && p.n <= c->crtw_max && c->d_pew_prog) {   // protocol-sized: k_pe_w on rows
    stage_mark(c, 0, st);
    HIPCHK(pew_launch(c->S_e, p, c->d_pew_prog, c->pew_nprog, st));
    stage_mark(c, 1, st);
    return 0;
  }
  if (obf_mode != PAI_OBF_NONE && c->pe_ok && c->ct_words == 2 * 64) return launch_pe(c, p, st);
  if (obf_mode != PAI_OBF_NONE && c->pe1_ok) return launch_pe1(c, p, st);
  switch (c->tpi_e) {
    case 2: return launch_encrypt<2>(c, p, st);
    case 4: return launch_encrypt<4>(c, p, st);
    case 8: return launch_encrypt<8>(c, p, st);
  }
  return fail(PAI_ERR_KEY, "unsupported group size");
}

template <int TPI>
static int launch_add(pai_ctx* c, AddParams& p, hipStream_t st) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  const size_t lds = (size_t)GPB * S * 4;
  const int grid = grid_for(c, k_add<TPI>, lds, p.n, GPB);
  hipLaunchKernelGGL(k_add<TPI>, dim3(grid), dim3(BLOCK), lds, st, p);
  HIPCHK(hipGetLastError());
  return 0;
}

// k-way add of p.k <= ADD_KMAX operands per instance: schedule sort (k_add_plan, k_add_scan,
// k_add_scatter) then the Horner product k_add (kernels.hpp).
static int run_add(pai_ctx* c, AddParams p, hipStream_t st) {
  if (p.n <= 0) return 0;
  const size_t nb_bucket = align16((size_t)p.n * 2), nb_perm = align16((size_t)p.n * 4);
  int rc = ensure_buf(&c->d_addplan, &c->addplan_bytes, nb_bucket + nb_perm + ADD_TMAX * 4);
  if (rc) return rc;
  uint16_t* bucket = (uint16_t*)c->d_addplan;
  int* perm = (int*)((char*)c->d_addplan + nb_bucket);
  unsigned* hist = (unsigned*)((char*)c->d_addplan + nb_bucket + nb_perm);
  p.N = c->d_N;
  p.RS = c->d_RS;
  p.mprime = c->mprime_N;
  p.ct_words = c->ct_words;
  p.perm = nullptr;
  const int g = (int)std::max<long long>(1, std::min<long long>((p.n + 255) / 256, 8ll * c->cus));
  HIPCHK(hipMemsetAsync(hist, 0, ADD_TMAX * 4, st));
  hipLaunchKernelGGL(k_add_plan<0>, dim3(g), dim3(256), 0, st, p, bucket, hist);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_add_scan<0>, dim3(1), dim3(ADD_TMAX), 0, st, hist);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_add_scatter<0>, dim3(g), dim3(256), 0, st, (long long)p.n, (const uint16_t*)bucket, hist, perm);
  HIPCHK(hipGetLastError());
  p.perm = perm;
  switch (c->tpi_e) {
    case 2: return launch_add<2>(c, p, st);
    case 4: return launch_add<4>(c, p, st);
    case 8: return launch_add<8>(c, p, st);
  }
  return fail(PAI_ERR_KEY, "unsupported group size");
}

static AddParams add_params(const uint32_t* cts, const int32_t* exps, int k, long long N, uint32_t* out, int32_t* out_exp,
                            const long long* gidx = nullptr) {
  AddParams p{};
  p.cts = cts;
  p.exps = exps;
  p.k = k;
  p.out = out;
  p.out_exp = out_exp;
  p.n = N;
  p.gidx = gidx;
  return p;
}

static int add_dev(pai_ctx* c, const uint32_t* cts, const int32_t* exps, int k, long long N, uint32_t* out,
                   int32_t* out_exp, hipStream_t st);

int pai_add_dev(pai_ctx* c, const uint32_t* d_cts, const int32_t* d_exps, int k, size_t N, uint32_t* d_out,
                int32_t* d_exp_out, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (N == 0) return 0;
  if (k < 1 || !d_cts || !d_exps || !d_out || !d_exp_out) return fail(PAI_ERR_ARG, "pai_add_dev: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  return add_dev(c, d_cts, d_exps, k, (long long)N, d_out, d_exp_out, (hipStream_t)stream);
}

template <int TPI>
static int launch_decrypt(pai_ctx* c, DecParams& p, hipStream_t st) {
  constexpr int S = TPI * L;
  constexpr int EPB = BLOCK / (2 * TPI);
  const size_t lds = (size_t)EPB * 4 * S * 4;
  const int grid = grid_for(c, k_decrypt<TPI>, lds, p.n, EPB);
  int rc = ensure_scratch(c, (size_t)grid * EPB * 2 * TABLE_FIX * S * 4);
  if (rc) return rc;
  p.scratch = (uint32_t*)c->d_scratch;
  hipLaunchKernelGGL(k_decrypt<TPI>, dim3(grid), dim3(BLOCK), lds, st, p);
  HIPCHK(hipGetLastError());
  return 0;
}

// pair decryption (kernels_pair.hpp, engine_pair.hip), in chunks of CRT_CHUNK elements
// The pair kernels' final stage over elements [off, off + n) from the pairs in xw ([2][2S][n])
static DecPairFinParams dec_pair_fin_params(pai_ctx* c, const DecParams& d, uint32_t* xw, long long off, long long n) {
  DecPairFinParams f{};
  f.halves = c->d_decp_halves;
  f.n = n;
  f.xh = xw;
  f.exp = d.exp + off;
  f.p = c->d_dec_p;
  f.q = c->d_dec_q;
  f.qinvR = c->d_dec_qinvR;
  f.pprime = c->dec_pprime;
  f.nlimb = c->d_decp_nl;
  f.maxint = c->d_decp_maxint;
  f.val = d.val + off;
  f.mant = d.mant ? d.mant + off : nullptr;
  f.status = d.status + off;
  f.raw = d.raw ? d.raw + (size_t)off * c->pt_words : nullptr;
  f.pt_words = c->pt_words;
  return f;
}

// A call of at most crtw_max ciphertexts: c^(p_h - 1) mod p_h^2 on 16-lane rows (k_dec_w, kernels_crtw.hpp) into
// the pairs k_dec_fin_pair takes; stage times: k_dec_w, k_dec_fin_pair.
static int launch_decw(pai_ctx* c, const DecParams& d, hipStream_t st) {
  const long long N = d.n;
  const int S = c->crt_sa;
  int rc = ensure_work(c, (size_t)4 * S * N * 4);
  if (rc) return rc;
  uint32_t* xw = (uint32_t*)c->d_work;
  crtw::DecParams p{c->d_decw, c->d_crt_a, N, d.ct, c->ct_words, c->decw_kchunks, xw};
  stage_mark(c, 0, st);
  HIPCHK(decw_launch(S, p, st));
  stage_mark(c, 1, st);
  const DecPairFinParams f = dec_pair_fin_params(c, d, xw, 0, N);
  HIPCHK(dec_pair_launch_fin(S, f, (int)std::min<long long>((N + LANE_BLOCK - 1) / LANE_BLOCK, 4ll * c->cus), st));
  stage_mark(c, 2, st);
  return 0;
}

static int launch_dec_pair(pai_ctx* c, const DecParams& d, hipStream_t st) {
  const long long N = d.n;
  if (N <= c->crtw_max && c->d_decw) return launch_decw(c, d, st);
  const long long chunk = std::min(N, CRT_CHUNK);
  const int S = c->crt_sa;
  DecLaneGeom g;
  if (dec_pair_geometry(S, c->cus, chunk, &g, c->decf)) return fail(PAI_ERR_KEY, "pair decrypt: unsupported size");
  int rc = ensure_scratch(c, g.scratch_bytes);
  if (rc) return rc;
  if ((rc = ensure_work(c, (size_t)4 * S * chunk * 4))) return rc;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    hipEvent_t* ev = stage_chunk(c);
    if (ev) c->nev = 4;
    uint32_t* xw = (uint32_t*)c->d_work;   // [2][2S][n]: c~, then x_h in place
    DecPairPreParams pre{c->d_decp_halves, n, d.ct + (size_t)off * c->ct_words, c->ct_words, c->decp_kchunks, xw};
    CrtParams pw{};
    pw.halves = c->d_decp_pow;
    pw.n = n;
    pw.yin = xw;
    pw.out = xw;
    pw.scratch = (uint32_t*)c->d_scratch;
    const DecPairFinParams f = dec_pair_fin_params(c, d, xw, off, n);
    HIPCHK(dec_pair_launch(S, pre, pw, f, g, st, ev, c->decf));
  }
  return 0;
}

// 4096-bit split-pair decryption (kernels_dec4.hpp, engine_dec4.hip), in chunks of CRT_CHUNK elements
// A 4096-bit call of at most crtw_max ciphertexts: c^(p_h - 1) mod p_h^2 on rows (k_dec_w<74, 148>) into the pairs
// k_dec4_L takes, then k_dec4_L and k_dec4_fin; stage times: k_dec_w, k_dec4_L + k_dec4_fin.
static int launch_decw4(pai_ctx* c, const DecParams& d, hipStream_t st) {
  const long long N = d.n;
  Dec4Geom g;
  dec4_geometry(c->cus, N, &g);
  const size_t xbytes = (size_t)2 * 2 * D4_S * 4, mbytes = (size_t)2 * D4_S * 4;   // per element
  int rc = ensure_work(c, (xbytes + mbytes) * N);
  if (rc) return rc;
  Dec4Params p{};
  p.halves = c->d_dec4_halves;
  p.n = N;
  p.ct = d.ct;
  p.ct_words = c->ct_words;
  p.kchunks = c->dec4_kchunks;
  p.x = (uint32_t*)c->d_work;
  p.mh = (uint32_t*)((char*)c->d_work + xbytes * N);
  p.scratch = (uint32_t*)c->d_scratch;
  crtw::DecParams w{c->d_decw, c->d_crt_a, N, d.ct, c->ct_words, c->decw_kchunks, p.x};
  stage_mark(c, 0, st);
  HIPCHK(decw_launch(c->rows_sa, w, st));
  stage_mark(c, 1, st);
  HIPCHK(dec4_launch_tail(p, d, g, st));
  stage_mark(c, 2, st);
  return 0;
}

static int launch_dec4(pai_ctx* c, const DecParams& d, hipStream_t st) {
  const long long N = d.n;
  if (N <= c->crtw_max && c->rows_sa && c->d_decw) return launch_decw4(c, d, st);
  const long long chunk = std::min(N, CRT_CHUNK);
  Dec4Geom g;
  dec4_geometry(c->cus, chunk, &g);
  int rc = ensure_scratch(c, g.scratch_bytes);
  if (rc) return rc;
  const size_t xbytes = (size_t)2 * 2 * D4_S * 4, mbytes = (size_t)2 * D4_S * 4;   // per element
  if ((rc = ensure_work(c, (xbytes + mbytes) * chunk))) return rc;
  for (long long off = 0; off < N; off += chunk) {
    const long long n = std::min(chunk, N - off);
    hipEvent_t* ev = stage_chunk(c);
    if (ev) c->nev = 4;
    Dec4Params p{};
    p.halves = c->d_dec4_halves;
    p.n = n;
    p.ct = d.ct + (size_t)off * c->ct_words;
    p.ct_words = c->ct_words;
    p.kchunks = c->dec4_kchunks;
    p.x = (uint32_t*)c->d_work;
    p.mh = (uint32_t*)((char*)c->d_work + xbytes * chunk);
    p.scratch = (uint32_t*)c->d_scratch;
    DecParams f = d;
    f.ct += (size_t)off * c->ct_words;
    f.exp += off;
    f.n = n;
    f.val += off;
    if (f.mant) f.mant += off;
    f.status += off;
    if (f.raw) f.raw += (size_t)off * c->pt_words;
    HIPCHK(dec4_launch(p, f, g, st, ev));
  }
  return 0;
}

int pai_decrypt_dev(pai_ctx* c, const uint32_t* d_ct, const int32_t* d_exp, size_t N, double* d_val, int64_t* d_mant,
                    int32_t* d_status, uint32_t* d_raw, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (!c->has_priv) return fail(PAI_ERR_NOPRIV, "pai_decrypt: context has no private key");
  if (N == 0) return 0;
  if (!d_ct || !d_exp || !d_val || !d_status) return fail(PAI_ERR_ARG, "pai_decrypt_dev: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  stage_reset(c);
  DecParams p{};
  p.ct = d_ct;
  p.exp = d_exp;
  p.n = (long long)N;
  p.val = d_val;
  p.mant = d_mant;
  p.status = d_status;
  p.raw = d_raw;
  p.halves = c->d_halves;
  p.qinvR = c->d_qinvR;
  p.nlimb = c->d_nlimb;
  p.qRn = c->d_qRn;
  p.maxint = c->d_maxint;
  p.nprime = c->nprime_d;
  p.nwin = c->nwin;
  p.ct_words = c->ct_words;
  p.pt_words = c->pt_words;
  p.n_limbs = c->n_limbs;
  hipStream_t st = (hipStream_t)stream;
  if (c->dec_pair_ok && c->dec_lane_enabled) return launch_dec_pair(c, p, st);
  if (c->dec4_ok && c->dec_lane_enabled) return launch_dec4(c, p, st);
  switch (c->tpi_d) {
    case 1: return launch_decrypt<1>(c, p, st);
    case 2: return launch_decrypt<2>(c, p, st);
    case 4: return launch_decrypt<4>(c, p, st);
  }
  return fail(PAI_ERR_KEY, "unsupported group size");
}

// ------------------------------------------------------------------ host-buffer entry points
struct DevScope {
  std::vector<void*> ptrs;
  ~DevScope() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return (T*)p;
  }
};

// ------------------------------------------------------------------ ciphertext x plaintext

static int inv_grid(pai_ctx* c, int tpi, long long nseg) {
  int occ = 1;
  if (mul_occupancy(tpi, &occ)) occ = 1;
  const int gpb = BLOCK / tpi;
  return (int)std::max<long long>(1, std::min<long long>((nseg + gpb - 1) / gpb, (long long)occ * c->cus));
}

// Batch inversion (Montgomery's trick, kernels_mul.hpp) of the flagged values of x [n][W] in place,
// on `st`. Segment products are reduced level by level to ONE value, inverted on the host (the only
// modular inversion mod n^2; gmpy_math.invert, gmpy_math.py:66-74), and expanded back down. The
// host step synchronises `st` once. Not invertible -> PAI_ERR_NOINV ("no inverse exists").
static int batch_invert(pai_ctx* c, uint32_t* x, const uint8_t* flag, long long n, hipStream_t st) {
  return batch_invert(c, x, flag, n, st, InvMod{c->tpi_e, c->ct_words, c->S_e, c->d_N, c->d_R2, c->d_oneR, c->mprime_N, &c->N});
}
static int batch_invert(pai_ctx* c, uint32_t* x, const uint8_t* flag, long long n, hipStream_t st, const InvMod& md) {
  const int S = md.S, W = md.W;
  // segment length per level: INV_SEG where there are values enough to fill the chip with segments, down to 4 on the
  // upper levels, whose few groups would otherwise walk chains of 64 dependent products (round 5: the 1M-value
  // inversion's levels above the first took ~22 of its 37 ms as 64-long chains over 16 k, 256 and 4 values)
  std::vector<long long> ns{n};
  std::vector<int> seg;
  do {
    seg.push_back((int)std::max<long long>(4, std::min<long long>(INV_SEG, ns.back() / 4096)));
    ns.push_back((ns.back() + seg.back() - 1) / seg.back());
  } while (ns.back() > 1);
  const int levels = (int)ns.size() - 1;
  std::vector<size_t> pre_off(levels), seg_off(levels);
  size_t off = 0;
  for (int l = 0; l < levels; ++l) {
    pre_off[l] = off;
    off = align16(off + (size_t)ns[l] * S * 4);
    seg_off[l] = off;
    off = align16(off + (size_t)ns[l + 1] * W * 4);
  }
  int rc = ensure_buf(&c->d_inv, &c->inv_bytes, off);
  if (rc) return rc;
  char* base = (char*)c->d_inv;
  auto params = [&](int l) {
    InvParams p{};
    p.x = l == 0 ? x : (uint32_t*)(base + seg_off[l - 1]);
    p.flag = l == 0 ? flag : nullptr;
    p.n = ns[l];
    p.pre = (uint32_t*)(base + pre_off[l]);
    p.seg = (uint32_t*)(base + seg_off[l]);
    p.N = md.N;
    p.R2 = md.R2;
    p.oneR = md.oneR;
    p.mprime = md.mprime;
    p.ct_words = W;
    p.seg_len = seg[l];
    return p;
  };
  for (int l = 0; l < levels; ++l) HIPCHK(inv_launch(md.tpi, true, params(l), inv_grid(c, md.tpi, ns[l + 1]), st));
  uint32_t* top = (uint32_t*)(base + seg_off[levels - 1]);
  c->inv_host.assign(W, 0);
  HIPCHK(hipMemcpyAsync(c->inv_host.data(), top, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  HBig v;
  v.w = c->inv_host;
  v.trim();
  HBig inv = inv_mod(v, *md.mod);
  if (inv.is_zero()) return fail(PAI_ERR_NOINV, "invert() no inverse exists");
  c->inv_host = inv.words(W);
  HIPCHK(hipMemcpyAsync(top, c->inv_host.data(), (size_t)W * 4, hipMemcpyHostToDevice, st));
  for (int l = levels - 1; l >= 0; --l) HIPCHK(inv_launch(md.tpi, false, params(l), inv_grid(c, md.tpi, ns[l + 1]), st));
  return 0;
}

// The public-key encryption's batch inversion (launch_pe) without blocking the caller: batch_invert's levels, but the top
// value is inverted by a host function queued on `st` (hipLaunchHostFunc: it runs when the stream reaches it, on the
// runtime's thread, touching only the pinned words) instead of after a hipStreamSynchronize, so pai_encrypt_dev stays
// asynchronous and capturable. An A_r that shares a factor with n (no inverse, probability ~2^-1023 for
// random r; r = 0, n, 5p given explicitly) sets *d_noinv = 1, and the kernels choose the chain on the device:
// k_pe_iota / k_pe_pow_f exit, the general k_pe_pow runs (kernels_pe.hpp, PeParams::noinv).
static void inv_top_host(void* u) {
  auto* a = (pai_ctx::AsyncInv*)u;
  try {
    HBig v;
    v.w.assign(a->pin, a->pin + a->W);
    v.trim();
    const HBig inv = inv_mod(v, a->mod);
    if (inv.is_zero()) {
      a->pin[a->W] = 1u;
      return;
    }
    const std::vector<uint32_t> w = inv.words(a->W);
    std::memcpy(a->pin, w.data(), (size_t)a->W * 4);
    a->pin[a->W] = 0u;
  } catch (...) {
    a->pin[a->W] = 1u;   // the general chain, same ciphertexts
  }
}

static int batch_invert_async(pai_ctx* c, uint32_t* x, long long n, hipStream_t st, const InvMod& md, uint32_t** d_noinv) {
  const int S = md.S, W = md.W;
  std::vector<long long> ns{n};
  std::vector<int> seg;
  do {
    seg.push_back((int)std::max<long long>(4, std::min<long long>(INV_SEG, ns.back() / 4096)));
    ns.push_back((ns.back() + seg.back() - 1) / seg.back());
  } while (ns.back() > 1);
  const int levels = (int)ns.size() - 1;
  std::vector<size_t> pre_off(levels), seg_off(levels);
  size_t off = 0;
  for (int l = 0; l < levels; ++l) {
    pre_off[l] = off;
    off = align16(off + (size_t)ns[l] * S * 4);
    seg_off[l] = off;
    off = align16(off + (size_t)ns[l + 1] * W * 4);
  }
  const size_t flag_off = off;
  off += 16;
  int rc = ensure_buf(&c->d_inv, &c->inv_bytes, off);
  if (rc) return rc;
  if (!c->inv_async || c->inv_async->W != W || !(c->inv_async->mod.w == md.mod->w)) {
    if (!c->inv_async) c->inv_async = new pai_ctx::AsyncInv;
    if (c->inv_async->pin && c->inv_async->W < W) {
      HIPCHK(hipStreamSynchronize(st));   // (once per context: a previous call's host function may still read it)
      (void)hipHostFree(c->inv_async->pin);
      c->inv_async->pin = nullptr;
    }
    if (!c->inv_async->pin) HIPCHK(hipHostMalloc((void**)&c->inv_async->pin, (size_t)(W + 4) * 4, hipHostMallocDefault));
    c->inv_async->W = W;
    c->inv_async->mod = *md.mod;
  }
  char* base = (char*)c->d_inv;
  auto params = [&](int l) {
    InvParams p{};
    p.x = l == 0 ? x : (uint32_t*)(base + seg_off[l - 1]);
    p.flag = nullptr;
    p.n = ns[l];
    p.pre = (uint32_t*)(base + pre_off[l]);
    p.seg = (uint32_t*)(base + seg_off[l]);
    p.N = md.N;
    p.R2 = md.R2;
    p.oneR = md.oneR;
    p.mprime = md.mprime;
    p.ct_words = W;
    p.seg_len = seg[l];
    return p;
  };
  for (int l = 0; l < levels; ++l) HIPCHK(inv_launch(md.tpi, true, params(l), inv_grid(c, md.tpi, ns[l + 1]), st));
  uint32_t* top = (uint32_t*)(base + seg_off[levels - 1]);
  uint32_t* flag = (uint32_t*)(base + flag_off);
  uint32_t* pin = c->inv_async->pin;
  HIPCHK(hipMemcpyAsync(pin, top, (size_t)W * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipLaunchHostFunc(st, inv_top_host, c->inv_async));
  HIPCHK(hipMemcpyAsync(top, pin, (size_t)W * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(flag, pin + W, 4, hipMemcpyHostToDevice, st));
  // (with no inverse the words copied back are the top value itself: the levels below produce values nobody reads)
  for (int l = levels - 1; l >= 0; --l) HIPCHK(inv_launch(md.tpi, false, params(l), inv_grid(c, md.tpi, ns[l + 1]), st));
  *d_noinv = flag;
  return 0;
}

// k_mul over n terms (p: index maps, scalars; outputs set by the caller)
static int launch_mul(pai_ctx* c, MulParams& p, hipStream_t st) {
  int occ = 1;
  if (mul_occupancy(c->tpi_e, &occ)) return fail(PAI_ERR_KEY, "unsupported group size");
  const int gpb = BLOCK / c->tpi_e;
  const int grid = (int)std::max<long long>(1, std::min<long long>((p.n + gpb - 1) / gpb, (long long)occ * c->cus));
  int rc = ensure_scratch(c, (size_t)grid * BLOCK * TILE_WORDS_PER_LANE * 4);
  if (rc) return rc;
  p.N = c->d_N;
  p.R2 = c->d_R2;
  p.oneR = c->d_oneR;
  p.mprime = c->mprime_N;
  p.ct_words = c->ct_words;
  p.scratch = (uint32_t*)c->d_scratch;
  HIPCHK(mul_launch(c->tpi_e, p, grid, st));
  return 0;
}

// k consecutive [N][W] operand arrays; more than ADD_KMAX operands are summed in chunks of ADD_KMAX
// (the partial sums are exact ciphertexts, so the result is the same integer)
static int add_dev(pai_ctx* c, const uint32_t* cts, const int32_t* exps, int k, long long N, uint32_t* out,
                   int32_t* out_exp, hipStream_t st) {
  if (k <= ADD_KMAX) return run_add(c, add_params(cts, exps, k, N, out, out_exp), st);
  const int parts = (k + ADD_KMAX - 1) / ADD_KMAX;
  const size_t W = c->ct_words;
  uint32_t* pc = nullptr;
  int32_t* pe = nullptr;
  HIPCHK(hipMallocAsync((void**)&pc, (size_t)parts * N * W * 4, st));
  HIPCHK(hipMallocAsync((void**)&pe, (size_t)parts * N * 4, st));
  int rc = 0;
  for (int q = 0; q < parts && !rc; ++q) {
    const int kq = std::min(ADD_KMAX, k - q * ADD_KMAX);
    rc = run_add(c, add_params(cts + (size_t)q * ADD_KMAX * N * W, exps + (size_t)q * ADD_KMAX * N, kq, N,
                               pc + (size_t)q * N * W, pe + (size_t)q * N), st);
  }
  if (!rc) rc = add_dev(c, pc, pe, parts, N, out, out_exp, st);
  (void)hipFreeAsync(pc, st);
  (void)hipFreeAsync(pe, st);
  return rc;
}

int pai_mul_dev(pai_ctx* c, const uint32_t* d_ct, const int32_t* d_exp, size_t N, int dtype, const void* d_x,
                size_t x_stride, uint32_t* d_out, int32_t* d_exp_out, int32_t* d_status, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (N == 0) return 0;
  if (!d_ct || !d_exp || !d_x || !d_out || !d_exp_out || dtype < 0 || dtype > 2 || x_stride > 1)
    return fail(PAI_ERR_ARG, "pai_mul_dev: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = ensure_buf(&c->d_mul, &c->mul_bytes, N);
  if (rc) return rc;
  MulParams p{};
  p.ct = d_ct;
  p.exp = d_exp;
  p.m = (long long)N;
  p.d = 1;
  p.cs_i = 1;
  p.xs_i = (long long)x_stride;
  p.x = d_x;
  p.dtype = dtype;
  p.n = (long long)N;
  p.out = d_out;
  p.out_exp = d_exp_out;
  p.status = d_status;
  p.neg = (uint8_t*)c->d_mul;
  if ((rc = launch_mul(c, p, st))) return rc;
  return batch_invert(c, d_out, (const uint8_t*)c->d_mul, (long long)N, st);
}

// E(x) + y over arrays (encrypted_number.py:139-164): k_plain encodes y_i with max_exponent e_i into
// c0_i = 1 + n M_i (r = 1) and E_i, then ONE 2-way k_add aligns E(x_i) to E_i and multiplies.
int pai_add_plain_dev(pai_ctx* c, const uint32_t* d_ct, const int32_t* d_exp, size_t N, int dtype, const void* d_x,
                      size_t x_stride, uint32_t* d_out, int32_t* d_exp_out, int32_t* d_status, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (N == 0) return 0;
  if (!d_ct || !d_exp || !d_x || !d_out || !d_exp_out || dtype < 0 || dtype > 2 || x_stride > 1)
    return fail(PAI_ERR_ARG, "pai_add_plain_dev: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t W = c->ct_words, cbytes = align16(2 * N * W * 4);
  int rc = ensure_buf(&c->d_plain, &c->plain_bytes, cbytes + 2 * N * 4);
  if (rc) return rc;
  uint32_t* ops = (uint32_t*)c->d_plain;
  int32_t* oexp = (int32_t*)((char*)c->d_plain + cbytes);
  HIPCHK(hipMemcpyAsync(ops, d_ct, N * W * 4, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(oexp, d_exp, N * 4, hipMemcpyDeviceToDevice, st));
  PlainParams p{};
  p.exp = d_exp;
  p.x = d_x;
  p.dtype = dtype;
  p.xs = (long long)x_stride;
  p.n = (long long)N;
  p.c0 = ops + N * W;
  p.e0 = oexp + N;
  p.status = d_status;
  p.N = c->d_N;
  p.nl = c->d_nl;
  p.ct_words = c->ct_words;
  p.max_bits = c->nb - 3;
  HIPCHK(plain_launch(c->tpi_e, p, (long long)N, c->cus, st));
  return add_dev(c, ops, oexp, 2, (long long)N, d_out, d_exp_out, st);
}

// Segmented k-way add (per-bin sums of IV_FFS, hetero_bin.py:28-36): a reduction tree of
// 16-operand k_add passes whose operands are gathered through a row index (AddParams.gidx), so segments of
// any length share one launch per level. Segment metadata (index, offsets) is host memory.
constexpr int SEG_CHUNK = 16;

int pai_segment_add_dev(pai_ctx* c, const uint32_t* d_ct, const int32_t* d_exp, size_t N, const int64_t* index,
                        const int64_t* seg_off, size_t nseg, uint32_t* d_out, int32_t* d_exp_out, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (nseg == 0) return 0;
  if (!d_ct || !d_exp || !seg_off || !d_out || !d_exp_out) return fail(PAI_ERR_ARG, "pai_segment_add_dev: bad arguments");
  if (seg_off[0] != 0) return fail(PAI_ERR_ARG, "pai_segment_add_dev: seg_off[0] must be 0");
  for (size_t s = 0; s < nseg; ++s)
    if (seg_off[s + 1] < seg_off[s]) return fail(PAI_ERR_ARG, "pai_segment_add_dev: offsets must not decrease");
  const long long total = seg_off[nseg];
  if (total > 0 && !index) return fail(PAI_ERR_ARG, "pai_segment_add_dev: index required");
  for (long long t = 0; t < total; ++t)
    if (index[t] < 0 || (size_t)index[t] >= N) return fail(PAI_ERR_ARG, "pai_segment_add_dev: index out of range");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t W = c->ct_words;
  const int C = SEG_CHUNK;
  // members of every segment as source rows; each level maps them to ceil(len / C) partial sums
  std::vector<long long> len(nseg), src(total);
  for (size_t s = 0; s < nseg; ++s) len[s] = seg_off[s + 1] - seg_off[s];
  for (long long t = 0; t < total; ++t) src[t] = index[t];
  long long max_parts = 0;
  for (size_t s = 0; s < nseg; ++s) max_parts += (len[s] + C - 1) / C;
  const size_t o_a = 0, o_b = align16(o_a + (size_t)max_parts * W * 4), o_ea = align16(o_b + (size_t)max_parts * W * 4),
               o_eb = align16(o_ea + (size_t)max_parts * 4), o_g = align16(o_eb + (size_t)max_parts * 4),
               need = align16(o_g + (size_t)std::max<long long>(max_parts, (long long)nseg) * C * 8);
  int rc = ensure_buf(&c->d_seg, &c->seg_bytes, need);
  if (rc) return rc;
  char* b = (char*)c->d_seg;
  uint32_t* part[2] = {(uint32_t*)(b + o_a), (uint32_t*)(b + o_b)};
  int32_t* pexp[2] = {(int32_t*)(b + o_ea), (int32_t*)(b + o_eb)};
  long long* d_g = (long long*)(b + o_g);
  const uint32_t* in = d_ct;
  const int32_t* in_e = d_exp;
  int side = 0;
  std::vector<long long> g;
  for (;;) {
    long long maxlen = 0;
    for (size_t s = 0; s < nseg; ++s) maxlen = std::max(maxlen, len[s]);
    const bool last = maxlen <= C;
    // one gather row of C sources per output (padding -1); the last level has one output per segment
    g.clear();
    std::vector<long long> nlen(nseg), nsrc;
    long long pos = 0;
    for (size_t s = 0; s < nseg; ++s) {
      const long long parts = last ? 1 : (len[s] + C - 1) / C;
      for (long long q = 0; q < parts; ++q) {
        for (int j = 0; j < C; ++j) {
          const long long t = q * C + j;
          g.push_back(t < len[s] ? src[pos + t] : -1);
        }
        nsrc.push_back((long long)nsrc.size());
      }
      pos += len[s];
      nlen[s] = parts;
    }
    const long long outs = (long long)nsrc.size();
    HIPCHK(hipMemcpyAsync(d_g, g.data(), g.size() * 8, hipMemcpyHostToDevice, st));
    uint32_t* o = last ? d_out : part[side];
    int32_t* oe = last ? d_exp_out : pexp[side];
    if ((rc = run_add(c, add_params(in, in_e, C, outs, o, oe, d_g), st))) return rc;
    HIPCHK(hipStreamSynchronize(st));   // the gather rows (host vector) are reused by the next level
    if (last) return 0;
    in = o;
    in_e = oe;
    side ^= 1;
    len.swap(nlen);
    src.swap(nsrc);
  }
}

constexpr int MATMUL_CHUNK = 16;   // operands per k_add pass of the reduction tree

int pai_matmul_dev(pai_ctx* c, const uint32_t* d_ct, const int32_t* d_exp, size_t m, size_t K, int dtype,
                   const void* d_x, size_t d, uint32_t* d_out, int32_t* d_exp_out, void* stream) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c, (hipStream_t)stream);
  if (m == 0 || d == 0) return 0;
  if (K == 0 || !d_ct || !d_exp || !d_x || !d_out || !d_exp_out || dtype < 0 || dtype > 2)
    return fail(PAI_ERR_ARG, "pai_matmul_dev: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t W = c->ct_words, Np = m * d, T = K * Np;
  const int C = MATMUL_CHUNK;
  const size_t Kp = K > (size_t)C ? (K + C - 1) / C * C : K;          // rows of the term buffer
  const size_t Pr = (Kp + C - 1) / C + C;                              // rows of the partial buffer
  const size_t o_terms = 0, o_texp = align16(o_terms + Kp * Np * W * 4), o_flag = align16(o_texp + Kp * Np * 4),
               o_part = align16(o_flag + T), o_pexp = align16(o_part + Pr * Np * W * 4), total = align16(o_pexp + Pr * Np * 4);
  int rc = ensure_buf(&c->d_mul, &c->mul_bytes, total);
  if (rc) return rc;
  char* b = (char*)c->d_mul;
  uint32_t* terms = (uint32_t*)(b + o_terms);
  int32_t* texp = (int32_t*)(b + o_texp);
  uint8_t* flag = (uint8_t*)(b + o_flag);
  uint32_t* part = (uint32_t*)(b + o_part);
  int32_t* pexp = (int32_t*)(b + o_pexp);
  // terms (k, i, j) = c[i][k] (x) x[k][j], k-major: the k_add layout of K operands over m d outputs
  MulParams p{};
  p.ct = d_ct;
  p.exp = d_exp;
  p.m = (long long)m;
  p.d = (long long)d;
  p.cs_i = (long long)K;
  p.cs_k = 1;
  p.xs_k = (long long)d;
  p.xs_j = 1;
  p.x = d_x;
  p.dtype = dtype;
  p.n = (long long)T;
  p.out = terms;
  p.out_exp = texp;
  p.neg = flag;
  if ((rc = launch_mul(c, p, st))) return rc;
  if ((rc = batch_invert(c, terms, flag, (long long)T, st))) return rc;
  // reduction over k: passes of C operands (padding operands: exponent PAD_EXP), then the rest
  uint32_t* cur = terms;
  int32_t* cur_e = texp;
  size_t Kc = K;
  bool in_terms = true;
  while (Kc > (size_t)C) {
    const size_t Kn = (Kc + C - 1) / C;
    if (Kn * C > Kc) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(cur_e + Kc * Np), PAD_EXP, (Kn * C - Kc) * Np, st));
    uint32_t* nxt = in_terms ? part : terms;
    int32_t* nxt_e = in_terms ? pexp : texp;
    if ((rc = add_dev(c, cur, cur_e, C, (long long)(Kn * Np), nxt, nxt_e, st))) return rc;
    cur = nxt;
    cur_e = nxt_e;
    Kc = Kn;
    in_terms = !in_terms;
  }
  return add_dev(c, cur, cur_e, (int)Kc, (long long)Np, d_out, d_exp_out, st);
}

int pai_mul(pai_ctx* c, const uint32_t* ct, const int32_t* exp, size_t N, int dtype, const void* x, size_t x_stride,
            uint32_t* ct_out, int32_t* exp_out, int32_t* status_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (N == 0) return 0;
  if (!ct || !exp || !x || !ct_out || !exp_out || x_stride > 1) return fail(PAI_ERR_ARG, "pai_mul: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words, esz = dtype == PAI_F32 ? 4 : 8, nx = x_stride ? N : 1;
  DevScope ds;
  uint32_t* dct = ds.alloc<uint32_t>(N * W);
  int32_t* dexp = ds.alloc<int32_t>(N);
  void* dx = ds.alloc<uint8_t>(nx * esz);
  uint32_t* dout = ds.alloc<uint32_t>(N * W);
  int32_t* dexo = ds.alloc<int32_t>(N);
  int32_t* dst = ds.alloc<int32_t>(N);
  if (!dct || !dexp || !dx || !dout || !dexo || !dst) return fail(PAI_ERR_HIP, "pai_mul: device allocation failed");
  HIPCHK(hipMemcpy(dct, ct, N * W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dexp, exp, N * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx, x, nx * esz, hipMemcpyHostToDevice));
  int rc = pai_mul_dev(c, dct, dexp, N, dtype, dx, x_stride, dout, dexo, dst, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(ct_out, dout, N * W * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(exp_out, dexo, N * 4, hipMemcpyDeviceToHost));
  if (status_out) HIPCHK(hipMemcpy(status_out, dst, N * 4, hipMemcpyDeviceToHost));
  return 0;
}

int pai_add_plain(pai_ctx* c, const uint32_t* ct, const int32_t* exp, size_t N, int dtype, const void* x,
                  size_t x_stride, uint32_t* ct_out, int32_t* exp_out, int32_t* status_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (N == 0) return 0;
  if (!ct || !exp || !x || !ct_out || !exp_out || x_stride > 1) return fail(PAI_ERR_ARG, "pai_add_plain: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words, esz = dtype == PAI_F32 ? 4 : 8, nx = x_stride ? N : 1;
  DevScope ds;
  uint32_t* dct = ds.alloc<uint32_t>(N * W);
  int32_t* dexp = ds.alloc<int32_t>(N);
  void* dx = ds.alloc<uint8_t>(nx * esz);
  uint32_t* dout = ds.alloc<uint32_t>(N * W);
  int32_t* dexo = ds.alloc<int32_t>(N);
  int32_t* dst = ds.alloc<int32_t>(N);
  if (!dct || !dexp || !dx || !dout || !dexo || !dst) return fail(PAI_ERR_HIP, "pai_add_plain: device allocation failed");
  HIPCHK(hipMemcpy(dct, ct, N * W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dexp, exp, N * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx, x, nx * esz, hipMemcpyHostToDevice));
  int rc = pai_add_plain_dev(c, dct, dexp, N, dtype, dx, x_stride, dout, dexo, dst, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(ct_out, dout, N * W * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(exp_out, dexo, N * 4, hipMemcpyDeviceToHost));
  if (status_out) HIPCHK(hipMemcpy(status_out, dst, N * 4, hipMemcpyDeviceToHost));
  return 0;
}

int pai_segment_add(pai_ctx* c, const uint32_t* ct, const int32_t* exp, size_t N, const int64_t* index,
                    const int64_t* seg_off, size_t nseg, uint32_t* ct_out, int32_t* exp_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (nseg == 0) return 0;
  if ((N && (!ct || !exp)) || !seg_off || !ct_out || !exp_out) return fail(PAI_ERR_ARG, "pai_segment_add: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words;
  DevScope ds;
  uint32_t* dct = ds.alloc<uint32_t>(N * W);
  int32_t* dexp = ds.alloc<int32_t>(N);
  uint32_t* dout = ds.alloc<uint32_t>(nseg * W);
  int32_t* dexo = ds.alloc<int32_t>(nseg);
  if (!dct || !dexp || !dout || !dexo) return fail(PAI_ERR_HIP, "pai_segment_add: device allocation failed");
  if (N) {
    HIPCHK(hipMemcpy(dct, ct, N * W * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dexp, exp, N * 4, hipMemcpyHostToDevice));
  }
  int rc = pai_segment_add_dev(c, dct, dexp, N, index, seg_off, nseg, dout, dexo, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(ct_out, dout, nseg * W * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(exp_out, dexo, nseg * 4, hipMemcpyDeviceToHost));
  return 0;
}

int pai_matmul(pai_ctx* c, const uint32_t* ct, const int32_t* exp, size_t m, size_t K, int dtype, const void* x,
               size_t d, uint32_t* ct_out, int32_t* exp_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (m == 0 || d == 0) return 0;
  if (K == 0 || !ct || !exp || !x || !ct_out || !exp_out) return fail(PAI_ERR_ARG, "pai_matmul: bad arguments");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words, esz = dtype == PAI_F32 ? 4 : 8;
  DevScope ds;
  uint32_t* dct = ds.alloc<uint32_t>(m * K * W);
  int32_t* dexp = ds.alloc<int32_t>(m * K);
  void* dx = ds.alloc<uint8_t>(K * d * esz);
  uint32_t* dout = ds.alloc<uint32_t>(m * d * W);
  int32_t* dexo = ds.alloc<int32_t>(m * d);
  if (!dct || !dexp || !dx || !dout || !dexo) return fail(PAI_ERR_HIP, "pai_matmul: device allocation failed");
  HIPCHK(hipMemcpy(dct, ct, m * K * W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dexp, exp, m * K * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dx, x, K * d * esz, hipMemcpyHostToDevice));
  int rc = pai_matmul_dev(c, dct, dexp, m, K, dtype, dx, d, dout, dexo, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(ct_out, dout, m * d * W * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(exp_out, dexo, m * d * 4, hipMemcpyDeviceToHost));
  return 0;
}

// ------------------------------------------------------------------ host-buffer entry points
// The operands cross PCIe in chunks that overlap the kernels: outputs of chunk i are copied to the
// caller while chunk i+1 computes (encrypt), inputs of chunk i+1 are copied while chunk i computes
// (decrypt, add). Ciphertexts do not depend on the chunking (the device RNG is keyed by the global
// element index). Device copies live in one buffer kept by the context (grown on demand).
constexpr size_t HOST_CHUNK_MIN = (size_t)1 << 17;   // elements: large enough to fill the chip per chunk
constexpr int HOST_CHUNKS_MAX = 16;
constexpr size_t PIN_SLOT_MAX = (size_t)64 << 20;     // bytes per pinned staging slot (two slots)

// Chunking for N elements moving stage_per_elem bytes each through the pinned slots; grows the
// context's device buffer to dev_bytes, the pinned slots and the per-chunk events.
static int host_pipe(pai_ctx* c, size_t N, size_t dev_bytes, size_t stage_per_elem, size_t* chunk, int* nch) {
  if (!c->s_comp) HIPCHK(hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking));
  if (!c->s_copy) HIPCHK(hipStreamCreateWithFlags(&c->s_copy, hipStreamNonBlocking));
  size_t k = std::max<size_t>(1, std::min<size_t>(HOST_CHUNKS_MAX, N / HOST_CHUNK_MIN));
  k = std::max(k, (N * stage_per_elem + PIN_SLOT_MAX - 1) / PIN_SLOT_MAX);
  *chunk = (N + k - 1) / k;
  *nch = (int)((N + *chunk - 1) / *chunk);
  for (auto* v : {&c->hev, &c->pev})
    while (v->size() < (size_t)*nch) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      v->push_back(e);
    }
  const size_t slot = *chunk * stage_per_elem;
  if (slot > c->pin_bytes) {
    for (void*& p : c->h_pin) {
      if (p) HIPCHK(hipHostFree(p));
      p = nullptr;
    }
    c->pin_bytes = 0;
    for (void*& p : c->h_pin) HIPCHK(hipHostMalloc(&p, slot, hipHostMallocDefault));
    c->pin_bytes = slot;
  }
  return ensure_buf(&c->d_hostio, &c->hostio_bytes, dev_bytes);
}

// memcpy between the pinned slots and caller memory on several host threads (a single thread moves
// ~10 GB/s, below the PCIe rate).
static void par_copy(void* dst, const void* src, size_t bytes) {
  const size_t hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t T = bytes < ((size_t)4 << 20) ? 1 : std::min<size_t>(16, hw);
  if (T == 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t part = ((bytes + T - 1) / T + 4095) & ~(size_t)4095;
  std::vector<std::thread> th;
  for (size_t t = 0; t < T && t * part < bytes; ++t)
    th.emplace_back([=] { std::memcpy((char*)dst + t * part, (const char*)src + t * part, std::min(part, bytes - t * part)); });
  for (auto& x : th) x.join();
}

// Carves typed regions out of the context's host-io buffer (256-byte aligned).
struct Carve {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t n) {
    T* p = (T*)(base + off);
    off = (off + std::max<size_t>(n, 1) * sizeof(T) + 255) & ~(size_t)255;
    return p;
  }
};
static size_t carve_bytes(std::initializer_list<size_t> sizes) {
  size_t t = 0;
  for (size_t b : sizes) t += (std::max<size_t>(b, 1) + 255) & ~(size_t)255;
  return t;
}

// Scope of one host-buffer call (pai_encrypt / pai_add / pai_decrypt): the stage timing is reset once and
// then spans every chunk's *_dev call; the fixed-base decision of the call is dropped at exit.
struct HostCall {
  pai_ctx* c;
  explicit HostCall(pai_ctx* ctx) : c(ctx) {
    stage_reset(c);
    c->stage_keep = true;
  }
  ~HostCall() {
    c->stage_keep = false;
    c->fb_call = 0;
    c->pfb_call = 0;
  }
};

int pai_encrypt(pai_ctx* c, int dtype, const void* x, size_t N, int exp_mode, int32_t fixed_exp, int obf_mode,
                const uint8_t* r_le, size_t r_stride_bytes, size_t r_bytes, const uint8_t* rng_key32,
                uint64_t index_base, uint32_t* ct_out, int32_t* exp_out, int32_t* status_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (N == 0) return 0;
  if (!x || !ct_out || !exp_out) return fail(PAI_ERR_ARG, "pai_encrypt: null buffer");
  if (obf_mode == PAI_OBF_GIVEN && (!r_le || r_bytes == 0)) return fail(PAI_ERR_ARG, "pai_encrypt: r required");
  HIPCHK(hipSetDevice(c->device));
  const size_t esz = dtype == PAI_F32 ? 4 : 8, W = c->ct_words;
  const size_t r_words = obf_mode == PAI_OBF_GIVEN ? (r_bytes + 3) / 4 : 0;
  const size_t r_cnt = obf_mode == PAI_OBF_GIVEN ? (r_stride_bytes ? N : 1) : 0;
  size_t CH;
  int nch, rc;
  if ((rc = host_pipe(c, N, carve_bytes({N * esz, N * W * 4, N * 4, N * 4, r_cnt * r_words * 4}), W * 4, &CH, &nch)))
    return rc;
  Carve cv{(char*)c->d_hostio};
  void* dx = cv.take<uint8_t>(N * esz);
  uint32_t* dct = cv.take<uint32_t>(N * W);
  int32_t* dexp = cv.take<int32_t>(N);
  int32_t* dst = cv.take<int32_t>(N);
  uint32_t* dr = cv.take<uint32_t>(r_cnt * r_words);
  hipStream_t sc = c->s_comp, sy = c->s_copy;
  HIPCHK(hipMemcpyAsync(dx, x, N * esz, hipMemcpyHostToDevice, sc));
  if (r_cnt) {
    std::vector<uint32_t> hr(r_cnt * r_words, 0);
    for (size_t i = 0; i < r_cnt; ++i) std::memcpy(&hr[i * r_words], r_le + i * r_stride_bytes, r_bytes);
    HIPCHK(hipMemcpyAsync(dr, hr.data(), hr.size() * 4, hipMemcpyHostToDevice, sc));
    HIPCHK(hipStreamSynchronize(sc));   // hr is released at the end of this scope
  }
  const size_t r_stride_words = r_stride_bytes ? r_words : 0;
  // one fixed-base decision and one stage-timing record for the whole call: the ciphertexts of a call do
  // not depend on how it is chunked
  HostCall hc(c);
  if (obf_mode == PAI_OBF_RNG) {
    if ((c->crt_ok || c->fbg_ok) && c->crt_enabled) c->fb_call = fb_wanted(c, (long long)N) ? 1 : -1;
    else if (c->pfb_enabled && pfb_supported(c)) c->pfb_call = pfb_wanted(c, (long long)N) ? 1 : -1;
  }
  // every chunk's kernels are queued first; the copy stream then drains chunk i while i+1.. compute
  for (int i = 0; i < nch; ++i) {
    const size_t off = (size_t)i * CH, n = std::min(CH, N - off);
    rc = pai_encrypt_dev(c, dtype, (const char*)dx + off * esz, n, exp_mode, fixed_exp, obf_mode,
                         dr ? dr + off * r_stride_words : nullptr, r_stride_words, r_words, rng_key32,
                         index_base + off, dct + off * W, dexp + off, dst + off, sc);
    if (rc) {
      (void)hipStreamSynchronize(sc);
      return rc;
    }
    HIPCHK(hipEventRecord(c->hev[i], sc));
  }
  // ciphertext words: device -> pinned slot (i & 1) on the copy stream, then the host threads move the
  // slot into the caller's buffer while chunk i+1 crosses PCIe and later chunks compute
  auto d2h = [&](int i) -> int {
    const size_t off = (size_t)i * CH, n = std::min(CH, N - off);
    HIPCHK(hipStreamWaitEvent(sy, c->hev[i], 0));
    HIPCHK(hipMemcpyAsync(c->h_pin[i & 1], dct + off * W, n * W * 4, hipMemcpyDeviceToHost, sy));
    HIPCHK(hipEventRecord(c->pev[i], sy));
    return 0;
  };
  if ((rc = d2h(0))) return rc;
  for (int i = 0; i < nch; ++i) {
    if (i + 1 < nch && (rc = d2h(i + 1))) return rc;   // its slot's previous chunk (i - 1) is consumed
    const size_t off = (size_t)i * CH, n = std::min(CH, N - off);
    HIPCHK(hipEventSynchronize(c->pev[i]));
    par_copy(ct_out + off * W, c->h_pin[i & 1], n * W * 4);
  }
  HIPCHK(hipMemcpyAsync(exp_out, dexp, N * 4, hipMemcpyDeviceToHost, sc));
  if (status_out) HIPCHK(hipMemcpyAsync(status_out, dst, N * 4, hipMemcpyDeviceToHost, sc));
  HIPCHK(hipStreamSynchronize(sc));
  HIPCHK(hipStreamSynchronize(sy));
  return 0;
}

int pai_add(pai_ctx* c, const uint32_t* const* cts, const int32_t* const* exps, int k, size_t N, uint32_t* ct_out,
            int32_t* exp_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (N == 0) return 0;
  if (k < 1 || !cts || !exps || !ct_out || !exp_out) return fail(PAI_ERR_ARG, "pai_add: bad arguments");
  for (int j = 0; j < k; ++j)
    if (!cts[j] || !exps[j]) return fail(PAI_ERR_ARG, "pai_add: null operand");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words;
  size_t CH;
  int nch, rc;
  if ((rc = host_pipe(c, N, carve_bytes({(size_t)k * N * W * 4, (size_t)k * N * 4, N * W * 4, N * 4}),
                     (size_t)k * W * 4, &CH, &nch)))
    return rc;
  Carve cv{(char*)c->d_hostio};
  // chunk i's operands are contiguous [k][n_i][W] at offset k off (the k_add layout of that chunk)
  uint32_t* dcts = cv.take<uint32_t>((size_t)k * N * W);
  int32_t* dexps = cv.take<int32_t>((size_t)k * N);
  uint32_t* dout = cv.take<uint32_t>(N * W);
  int32_t* dexp = cv.take<int32_t>(N);
  hipStream_t sc = c->s_comp, sy = c->s_copy;
  HostCall hc(c);
  for (int i = 0; i < nch; ++i) {
    const size_t off = (size_t)i * CH, n = std::min(CH, N - off);
    uint32_t* cc = dcts + (size_t)k * off * W;
    int32_t* ce = dexps + (size_t)k * off;
    // inputs of chunk i: caller -> pinned slot (host threads, while chunk i-1 computes) -> device
    if (i >= 2) HIPCHK(hipEventSynchronize(c->hev[i - 2]));   // the slot's previous upload is done
    uint32_t* slot = (uint32_t*)c->h_pin[i & 1];
    for (int j = 0; j < k; ++j) par_copy(slot + (size_t)j * n * W, cts[j] + off * W, n * W * 4);
    HIPCHK(hipMemcpyAsync(cc, slot, (size_t)k * n * W * 4, hipMemcpyHostToDevice, sy));
    for (int j = 0; j < k; ++j)
      HIPCHK(hipMemcpyAsync(ce + (size_t)j * n, exps[j] + off, n * 4, hipMemcpyHostToDevice, sy));
    HIPCHK(hipEventRecord(c->hev[i], sy));
    HIPCHK(hipStreamWaitEvent(sc, c->hev[i], 0));
    if ((rc = pai_add_dev(c, cc, ce, k, n, dout + off * W, dexp + off, sc))) {
      (void)hipStreamSynchronize(sc);
      return rc;
    }
  }
  HIPCHK(hipMemcpyAsync(ct_out, dout, N * W * 4, hipMemcpyDeviceToHost, sc));
  HIPCHK(hipMemcpyAsync(exp_out, dexp, N * 4, hipMemcpyDeviceToHost, sc));
  HIPCHK(hipStreamSynchronize(sc));
  return 0;
}

int pai_decrypt(pai_ctx* c, const uint32_t* ct, const int32_t* exp, size_t N, double* val_out, int64_t* mant_out,
                int32_t* status_out, uint32_t* raw_out) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (!c->has_priv) return fail(PAI_ERR_NOPRIV, "pai_decrypt: context has no private key");
  if (N == 0) return 0;
  if (!ct || !exp || !val_out || !status_out) return fail(PAI_ERR_ARG, "pai_decrypt: null buffer");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = c->ct_words, P = raw_out ? c->pt_words : 0;
  size_t CH;
  int nch, rc;
  if ((rc = host_pipe(c, N, carve_bytes({N * W * 4, N * 4, N * 8, N * 8, N * 4, N * P * 4}), W * 4, &CH, &nch)))
    return rc;
  Carve cv{(char*)c->d_hostio};
  uint32_t* dct = cv.take<uint32_t>(N * W);
  int32_t* dexp = cv.take<int32_t>(N);
  double* dval = cv.take<double>(N);
  int64_t* dmant = cv.take<int64_t>(N);
  int32_t* dst = cv.take<int32_t>(N);
  uint32_t* draw = cv.take<uint32_t>(N * P);
  hipStream_t sc = c->s_comp, sy = c->s_copy;
  HostCall hc(c);
  for (int i = 0; i < nch; ++i) {
    const size_t off = (size_t)i * CH, n = std::min(CH, N - off);
    if (i >= 2) HIPCHK(hipEventSynchronize(c->hev[i - 2]));   // the slot's previous upload is done
    par_copy(c->h_pin[i & 1], ct + off * W, n * W * 4);
    HIPCHK(hipMemcpyAsync(dct + off * W, c->h_pin[i & 1], n * W * 4, hipMemcpyHostToDevice, sy));
    HIPCHK(hipMemcpyAsync(dexp + off, exp + off, n * 4, hipMemcpyHostToDevice, sy));
    HIPCHK(hipEventRecord(c->hev[i], sy));
    HIPCHK(hipStreamWaitEvent(sc, c->hev[i], 0));
    if ((rc = pai_decrypt_dev(c, dct + off * W, dexp + off, n, dval + off, dmant + off, dst + off,
                              raw_out ? draw + off * P : nullptr, sc))) {
      (void)hipStreamSynchronize(sc);
      return rc;
    }
  }
  HIPCHK(hipMemcpyAsync(val_out, dval, N * 8, hipMemcpyDeviceToHost, sc));
  if (mant_out) HIPCHK(hipMemcpyAsync(mant_out, dmant, N * 8, hipMemcpyDeviceToHost, sc));
  HIPCHK(hipMemcpyAsync(status_out, dst, N * 4, hipMemcpyDeviceToHost, sc));
  if (raw_out) HIPCHK(hipMemcpyAsync(raw_out, draw, N * P * 4, hipMemcpyDeviceToHost, sc));
  HIPCHK(hipStreamSynchronize(sc));
  return 0;
}

// ------------------------------------------------------------------ debugging hook (tests / tools only)
// Copies the per-half sampler outputs (c0 G_h^a_h mod h^2) of the last fixed-base chunk: limbs [2][SB][n] (k_fb,
// k_fbg), or canonical pairs [2][2S][n] with *sb = 2S for the pair tables (k_fbs/k_fbp; the p half times q^-2).
extern "C" int pai_debug_fb_w(pai_ctx* c, uint32_t* out, size_t max_words, long long* n, int* sb) {
  if (!c) return fail(PAI_ERR_ARG, "null ctx");
  CtxLock lk(c);
  if (!c->fb_last_w) return fail(PAI_ERR_ARG, "no fixed-base output");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());
  const int rows = c->fb_pair_s ? 2 * c->fb_pair_s : c->crt_sb;
  const long long ne = c->fb_last_n;
  const size_t words = (size_t)2 * rows * ne;
  if (words > max_words) return fail(PAI_ERR_ARG, "buffer too small");
  if (c->fb_pair_s) {   // 64-element tiles (kernels_fbp.hpp fbp_pair_index) -> [2][2S][n]
    const long long np = fbp_npad(ne);
    std::vector<uint32_t> t((size_t)2 * rows * np);
    HIPCHK(hipMemcpy(t.data(), c->fb_last_w, t.size() * 4, hipMemcpyDeviceToHost));
    for (int h = 0; h < 2; ++h)
      for (int j = 0; j < rows; ++j)
        for (long long i = 0; i < ne; ++i)
          out[((size_t)h * rows + j) * ne + i] = t[(size_t)h * rows * np + (size_t)(i >> 6) * rows * 64 + (size_t)j * 64 + (i & 63)];
  } else {
    HIPCHK(hipMemcpy(out, c->fb_last_w, words * 4, hipMemcpyDeviceToHost));
  }
  *n = c->fb_last_n;
  *sb = rows;
  return 0;
}

// ------------------------------------------------------------------ engine unit-test hook (test build only)
#if FLEXPAI_XCHECK
template <int TPI>
static int launch_debug(pai_ctx* c, DbgParams& p) {
  constexpr int S = TPI * L;
  constexpr int GPB = BLOCK / TPI;
  const size_t lds = (size_t)GPB * S * 4;
  const int grid = (int)((p.n + GPB - 1) / GPB);
  int rc = ensure_scratch(c, (size_t)grid * BLOCK * TILE_WORDS_PER_LANE * 4);
  if (rc) return rc;
  p.scratch = (uint32_t*)c->d_scratch;
  hipLaunchKernelGGL(k_debug<TPI>, dim3(grid), dim3(BLOCK), lds, (hipStream_t)0, p);
  HIPCHK(hipGetLastError());
  return 0;
}

#endif

extern "C" int pai_debug_engine(pai_ctx* c, int op, const uint32_t* a, const uint32_t* b, size_t N, uint32_t* out,
                                int32_t* flag) {
#if !FLEXPAI_XCHECK
  (void)c, (void)op, (void)a, (void)b, (void)N, (void)out, (void)flag;
  return fail(PAI_ERR_ARG, "pai_debug_engine: in the test build (libflexpai_xcheck.so) only");
#else
  if (!c || N == 0) return fail(PAI_ERR_ARG, "pai_debug_engine: bad args");
  CtxLock lk(c);
  HIPCHK(hipSetDevice(c->device));
  DevScope ds;
  const size_t W = c->ct_words;
  uint32_t* da = ds.alloc<uint32_t>(N * W);
  uint32_t* db = ds.alloc<uint32_t>(N * W);
  uint32_t* dout = ds.alloc<uint32_t>(N * W);
  int32_t* dflag = ds.alloc<int32_t>(N);
  HIPCHK(hipMemcpy(da, a, N * W * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db, b, N * W * 4, hipMemcpyHostToDevice));
  DbgParams p{op, da, db, dout, dflag, (long long)N, (int)W, c->d_N, c->d_R2, c->d_nl, c->mprime_N,
              c->d_prog, c->nprog, nullptr};
  int rc = 0;
  switch (c->tpi_e) {
    case 2: rc = launch_debug<2>(c, p); break;
    case 4: rc = launch_debug<4>(c, p); break;
    case 8: rc = launch_debug<8>(c, p); break;
  }
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, dout, N * W * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(flag, dflag, N * 4, hipMemcpyDeviceToHost));
  return 0;
#endif
}
