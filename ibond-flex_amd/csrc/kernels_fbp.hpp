// Fixed-base obfuscation on p-adic pairs (bn_pair.hpp): the sampler of kernels_fb.hpp with every
// product mod p_h^2 done over the S limbs of p_h instead of a Montgomery product over the 2S limbs of
// p_h^2 (8 S^2 MACs). Same distribution, same ciphertext bits.
//
// Factored rows. A table entry T' = T_k[d] R mod p_h^2 (R = 2^(28 S)) is stored as T' = a (1 + p_h b) with
// a = T' mod p_h and b = (T' div p_h) a^-1 mod p_h: PW 32-bit words of a, then PW words of b R mod p_h -- 256 B
// for a 2048-bit key. The product of the K entries an element selects is
//   prod_k T'_k = (prod_k a_k) (1 + p_h sum_k b_k)   (mod p_h^2)
// so the loop multiplies the pair by (a_k, 0) -- 4 S^2 MACs instead of the 5 S^2 of a general pair product
// (bn_pair.hpp mont_mul_a0) -- while the b R words go into a running sum (PW words + a carry word, in VGPRs),
// and one product mod p_h at the end applies the factor: (A + p B)(1 + p bs) = A + p (B + A bs). The
// accumulator starts at c0 = 1 + n M = 1 + p_h (n / p_h) M, i.e. the pair (1, (n / p_h) M mod p_h), with the
// second component an unreduced sum of 8-bit chunks of |M| (< 2^PB p_h; the first product keeps B < 2 p_h
// while R >= 2^(PB+1) p_h). Every product multiplies a plain pair by a Montgomery-form row, so the result stays
// plain: after the K products and the correction the pair is c0 G_h^(a_h) mod p_h^2, written as its canonical
// pair for k_fbp_fin's Garner recombination (below).
#pragma once
#include "bn_pair.hpp"
#include "kernels_fb.hpp"

namespace fpai {

template <int S>
struct FbpGeom;
template <>
struct FbpGeom<19> {   // 1024-bit keys: p_h < 2^512
  static constexpr int SB = 37, PW = 16;
};
template <>
struct FbpGeom<37> {   // 2048-bit keys: p_h < 2^1024
  static constexpr int SB = 74, PW = 32;
};
constexpr int FBP_CB = 8, FBP_NC = 8, FBP_PB = 11;    // c0 chunks: 8 x 8 bits of |M| (sum < 2^11 p_h); offset 2^11 p_h

struct FbpHalf {
  const uint4* table;      // [K][2^W][2 PW / 4] quads: words of a, then of b R mod p_h, of T_k[d] R mod p_h^2 (header)
  const uint32_t* p;       // p_h, S limbs
  const uint32_t* oneR;    // pair of R mod p_h^2 (2S limbs: A then B)
  const uint32_t* bases;   // [K][2][2S] pairs of B_k R and B_k^(2^LO) R mod p_h^2 (table construction)
  uint32_t* lohi;          // [K][2][FB_LO][2S] scratch of the table construction
  const uint32_t* nm;      // [NC][S] (n / p_h) 2^(CB c) mod p_h
  const uint32_t* pbig;    // [S] 2^PB p_h
  uint32_t mprime;         // -p_h^-1 mod 2^28
  // factored rows: inverses of the lo/hi entries' A parts, and the batch inversion's scratch (k_fbp_inv_*)
  uint32_t* inv;           // [K][2][FB_LO][S]: (A of lo/hi entry)^-1 R mod p_h
  uint32_t* pre;           // [2K][2^max(LO,HI)][S] prefix products
  uint32_t* cval;          // [2K][S]: each chain's product, then its inverse R^2 (host)
  // pair of kappa R mod p_h^2, multiplied into position 0's lo entries (k_fbp_lohi): kappa = q^-2 mod p^2 for the p
  // half, so that every row of position 0 carries it and k_fbp_fin receives w_p q^-2; kappa = 1 (oneR) for the q half
  const uint32_t* kapR;
  const uint32_t* nmR;     // [NC][S] (n / p_h) 2^(CB c) R mod p_h: k_fbs's start gamma R in the b sum (kernels_fbs.hpp)
};

// The canonical pairs k_fbp leaves for k_fbp_fin, in tiles of 64 elements: [half][i / 64][2S limbs][i % 64] (n
// rounded up to 64): a wave's limb j is one 256-B line and every limb of an element sits at a compile-time offset
// from one address.
__host__ __device__ constexpr long long fbp_npad(long long n) { return (n + 63) & ~63ll; }
template <int S>
__device__ __forceinline__ size_t fbp_pair_index(long long i, int half, long long n) {
  return (size_t)half * 2 * S * fbp_npad(n) + (size_t)(i >> 6) * 2 * S * 64 + (size_t)(i & 63);
}

struct FbpParams {
  const FbpHalf* halves;   // [2]
  long long n;
  int K, W;
  const uint32_t* digits;  // [2][K][n]
  uint32_t* out;           // canonical pairs (A limbs, then B) for k_fbp_fin in 64-element tiles (fbp_pair_index)
  const void* x;
  int dtype, exp_mode, fexp;
  int32_t* exp;
  int32_t* status;
  GuardArgs g;             // test build (guard.hpp): rows = K 2^W, digits = 2 K n, out = the pair tiles' words
#if defined(FBS_AB) && (FBS_AB & 4)
  const FbDigitParams* dig;   // measurement build (kernels_fbs.hpp FBS_AB & 4): k_fbs draws its own digits
#endif
};

// LDS words at a byte offset from this lane's row base (offsets past the 16-bit immediate take a second base)
template <int OFF>
__device__ __forceinline__ uint32_t lds_word_rd(uint32_t addr) {
  if constexpr (OFF < 65536) return lds_read_word<OFF>(addr);
  else return lds_read_word<OFF - 65536>(addr + 65536u);
}
template <int OFF>
__device__ __forceinline__ void lds_word_wr(uint32_t addr, uint32_t v) {
  if constexpr (OFF < 65536) asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF) : "memory");
  else asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(addr + 65536u), "v"(v), "i"(OFF - 65536) : "memory");
}

// Per product with a factored row, in LDS ([quad][lane] layout, quads of LANE_BLOCK x 16 B): the a words in quads
// 0 .. PW/4 - 1, the b R words in quads PW/4 .. PW/2 - 1 (summed first, then dead), and the first pass's reduction
// digits q1_j in word slots j of quads PW/4 + j/4 (the dead b R quads, then FBP_XQ extra quads).
template <int S, int PW>
struct FbpLds {
  static constexpr int TQ = PW / 2;                                       // quads of a DMA'd row
  static constexpr int NQ = PW / 4 + (S + 3) / 4 > TQ ? PW / 4 + (S + 3) / 4 : TQ;   // quads per lane
  static constexpr int a_off(int w) { return (w / 4) * LANE_BLOCK * 16 + (w % 4) * 4; }
  static constexpr int q_off(int j) { return (PW / 4 + j / 4) * LANE_BLOCK * 16 + (j % 4) * 4; }
};

// The multiplier's digits a_J from the a words, read D words ahead: digit J needs words (28 J) / 32 and
// (28 J + 27) / 32. Pass 1 of mont_mul_a0 (FbpAReader): the LDS operations in flight are the word reads, issued at
// the digits, and one q1 write after each digit (FbpQPut), and every wait names the exact count of operations
// issued after the words it needs. Pass 2 (FbpAQReader): the word reads and the q1 reads, q1_j read QD digits ahead.
template <int S, int PW, int D>
struct FbpWordSched {
  static constexpr int lo(int J) { return (28 * J) >> 5; }
  static constexpr int hi(int J) { return (28 * J + 27) >> 5 < PW - 1 ? (28 * J + 27) >> 5 : PW - 1; }
  static constexpr int issued(int J) { return J < 0 ? -1 : (hi(J) + D < PW - 1 ? hi(J) + D : PW - 1); }
  static constexpr int nA(int J) { return issued(J) - issued(J - 1); }
  static constexpr int batch_of(int w) {   // the digit whose issue phase reads word w
    int j = 0;
    while (issued(j) < w) ++j;
    return j;
  }
  __device__ static __forceinline__ uint32_t digit(int, uint32_t) { return 0; }
};

template <int S, int PW, int D>
struct FbpAReader {
  using Sc = FbpWordSched<S, PW, D>;
  uint32_t addr;
  uint32_t wa[PW];
  // operations issued before digit J's issue phase: the words of digits < J and their q1 writes
  static constexpr int before(int J) { return Sc::issued(J - 1) + 1 + J; }
  static constexpr int pos(int w) { return before(Sc::batch_of(w)) + (w - Sc::issued(Sc::batch_of(w) - 1) - 1); }
  template <int W0, int... Ws>
  __device__ __forceinline__ void issue(std::integer_sequence<int, Ws...>) {
    ((wa[W0 + Ws] = lds_word_rd<FbpLds<S, PW>::a_off(W0 + Ws)>(addr)), ...);
  }
  template <int J>
  __device__ __forceinline__ uint32_t operator()(std::integral_constant<int, J>) {
    constexpr int from = Sc::issued(J - 1) + 1, to = Sc::issued(J);
    issue<from>(std::make_integer_sequence<int, (to >= from ? to - from + 1 : 0)>{});
    constexpr int l = Sc::lo(J), h = Sc::hi(J);
    constexpr int pending = before(J) + Sc::nA(J) - 1 - pos(h);
    static_assert(pending >= 0 && pending <= 15, "lgkmcnt range");
    if constexpr (l == h) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(wa[l]) : "i"(pending));
    else asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(wa[l]), "+v"(wa[h]) : "i"(pending));
    constexpr int sh = (28 * J) & 31;
    if constexpr (sh + 28 <= 32) return (wa[l] >> sh) & lane::LMASK;
    else if constexpr (l + 1 < PW) return __builtin_amdgcn_alignbit(wa[l + 1], wa[l], sh) & lane::LMASK;
    else return wa[l] >> sh;
  }
};

template <int S, int PW>
struct FbpQPut {
  uint32_t addr;
  template <int J>
  __device__ __forceinline__ void operator()(std::integral_constant<int, J>, uint32_t q) {
    lds_word_wr<FbpLds<S, PW>::q_off(J)>(addr, q);
  }
};

template <int S, int PW, int D, int QD>
struct FbpAQReader {
  using Sc = FbpWordSched<S, PW, D>;
  static_assert(QD >= 1 && QD < S, "q1 read-ahead");
  uint32_t addr;
  uint32_t wa[PW], wq[S];
  // issue phase of digit J: (J = 0: q1_0 .. q1_(QD-1)), the words of batch J, then q1_(J+QD) if it exists
  static constexpr int nq(int J) { return (J == 0 ? QD : 0) + (J + QD < S ? 1 : 0); }
  static constexpr int before(int J) {
    int s = 0;
    for (int t = 0; t < J; ++t) s += Sc::nA(t) + nq(t);
    return s;
  }
  static constexpr int pos_a(int w) {
    const int jb = Sc::batch_of(w);
    return before(jb) + (jb == 0 ? QD : 0) + (w - Sc::issued(jb - 1) - 1);
  }
  static constexpr int pos_q(int i) { return i < QD ? i : before(i - QD) + (i == QD ? QD : 0) + Sc::nA(i - QD); }
  template <int W0, int... Ws>
  __device__ __forceinline__ void issue(std::integer_sequence<int, Ws...>) {
    ((wa[W0 + Ws] = lds_word_rd<FbpLds<S, PW>::a_off(W0 + Ws)>(addr)), ...);
  }
  template <int... Is>
  __device__ __forceinline__ void issue_q(std::integer_sequence<int, Is...>) {
    ((wq[Is] = lds_word_rd<FbpLds<S, PW>::q_off(Is)>(addr)), ...);
  }
  template <int J>
  __device__ __forceinline__ uint2 operator()(std::integral_constant<int, J>) {
    if constexpr (J == 0) issue_q(std::make_integer_sequence<int, QD>{});
    constexpr int from = Sc::issued(J - 1) + 1, to = Sc::issued(J);
    issue<from>(std::make_integer_sequence<int, (to >= from ? to - from + 1 : 0)>{});
    if constexpr (J + QD < S) wq[J + QD] = lds_word_rd<FbpLds<S, PW>::q_off(J + QD)>(addr);
    constexpr int l = Sc::lo(J), h = Sc::hi(J);
    constexpr int need = pos_a(h) > pos_q(J) ? pos_a(h) : pos_q(J);
    constexpr int pending = before(J) + Sc::nA(J) + nq(J) - 1 - need;
    static_assert(pending >= 0 && pending <= 15, "lgkmcnt range");
    if constexpr (l == h) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(wa[l]), "+v"(wq[J]) : "i"(pending));
    else asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(wa[l]), "+v"(wa[h]), "+v"(wq[J]) : "i"(pending));
    constexpr int sh = (28 * J) & 31;
    uint32_t x;
    if constexpr (sh + 28 <= 32) x = (wa[l] >> sh) & lane::LMASK;
    else if constexpr (l + 1 < PW) x = __builtin_amdgcn_alignbit(wa[l + 1], wa[l], sh) & lane::LMASK;
    else x = wa[l] >> sh;
    return make_uint2(x, wq[J]);
  }
};

// ---- the same two readers on 16-byte LDS reads (ds_read_b128: four words, or four q1 digits, per read)
typedef uint32_t fbp_u32x4 __attribute__((ext_vector_type(4)));
template <int OFF>
__device__ __forceinline__ fbp_u32x4 lds_quad_rd(uint32_t addr) {
  fbp_u32x4 v;
  if constexpr (OFF < 65536) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  else asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr + 65536u), "i"(OFF - 65536) : "memory");
  return v;
}
template <int C>
__device__ __forceinline__ uint32_t quad_word(const fbp_u32x4& v) {
  if constexpr (C == 0) return v.x;
  else if constexpr (C == 1) return v.y;
  else if constexpr (C == 2) return v.z;
  else return v.w;
}
// 28-bit digit J of the words held in quads qa (digit J needs words lo(J), hi(J))
template <int PW, int J>
__device__ __forceinline__ uint32_t fbp_quad_digit(const fbp_u32x4 (&qa)[PW / 4]) {
  constexpr int l = (28 * J) >> 5, sh = (28 * J) & 31;
  const uint32_t wl = quad_word<l % 4>(qa[l / 4]);
  if constexpr (sh + 28 <= 32) return (wl >> sh) & lane::LMASK;
  else if constexpr (l + 1 < PW) return __builtin_amdgcn_alignbit(quad_word<(l + 1) % 4>(qa[(l + 1) / 4]), wl, sh) & lane::LMASK;
  else return wl >> sh;
}

template <int S, int PW, int DQ>
struct FbpQuadSched {
  static constexpr int NQA = PW / 4;   // quads of a
  static constexpr int NQQ = (S + 3) / 4;   // quads of the q1 record
  static constexpr int hi(int J) { return (28 * J + 27) >> 5 < PW - 1 ? (28 * J + 27) >> 5 : PW - 1; }
  static constexpr int need(int J) { return hi(J) / 4; }
  static constexpr int issued(int J) { return J < 0 ? -1 : (need(J) + DQ < NQA - 1 ? need(J) + DQ : NQA - 1); }
  static constexpr int nA(int J) { return issued(J) - issued(J - 1); }
  static constexpr int batch_of(int g) {
    int j = 0;
    while (issued(j) < g) ++j;
    return j;
  }
};

// pass 1: a quads issued DQ quads ahead; one q1 write per digit (FbpQPut) follows each digit's wait
template <int S, int PW, int DQ>
struct FbpAQuadReader {
  using Sc = FbpQuadSched<S, PW, DQ>;
  uint32_t addr;
  fbp_u32x4 qa[PW / 4];
  static constexpr int before(int J) { return Sc::issued(J - 1) + 1 + J; }
  static constexpr int pos(int g) { return before(Sc::batch_of(g)) + (g - Sc::issued(Sc::batch_of(g) - 1) - 1); }
  template <int G0, int... Gs>
  __device__ __forceinline__ void issue(std::integer_sequence<int, Gs...>) {
    ((qa[G0 + Gs] = lds_quad_rd<(G0 + Gs) * LANE_BLOCK * 16>(addr)), ...);
  }
  template <int J>
  __device__ __forceinline__ uint32_t operator()(std::integral_constant<int, J>) {
    constexpr int from = Sc::issued(J - 1) + 1, to = Sc::issued(J);
    issue<from>(std::make_integer_sequence<int, (to >= from ? to - from + 1 : 0)>{});
    constexpr int gl = ((28 * J) >> 5) / 4, gh = Sc::need(J);
    constexpr int pending = before(J) + Sc::nA(J) - 1 - pos(gh);
    static_assert(pending >= 0 && pending <= 15, "lgkmcnt range");
    if constexpr (J == 0 || gh > Sc::need(J - 1)) {   // a quad not waited for yet (quads land in order)
      if constexpr (gl == gh) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(qa[gl]) : "i"(pending));
      else asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(qa[gl]), "+v"(qa[gh]) : "i"(pending));
    }
    return fbp_quad_digit<PW, J>(qa);
  }
};

// pass 2: the a quads as in pass 1, and the q1 record by quads (quad 0 first, quad Q + 1 at digit 4 Q)
template <int S, int PW, int DQ>
struct FbpAQQuadReader {
  using Sc = FbpQuadSched<S, PW, DQ>;
  uint32_t addr;
  fbp_u32x4 qa[PW / 4], qq[Sc::NQQ];
  static constexpr int nq(int J) { return (J == 0 ? 1 : 0) + ((J % 4 == 0 && J / 4 + 1 < Sc::NQQ) ? 1 : 0); }
  static constexpr int before(int J) {
    int s = 0;
    for (int t = 0; t < J; ++t) s += Sc::nA(t) + nq(t);
    return s;
  }
  static constexpr int pos_a(int g) {
    const int jb = Sc::batch_of(g);
    return before(jb) + (jb == 0 ? 1 : 0) + (g - Sc::issued(jb - 1) - 1);
  }
  static constexpr int pos_q(int Q) { return Q == 0 ? 0 : before(4 * (Q - 1)) + (Q == 1 ? 1 : 0) + Sc::nA(4 * (Q - 1)); }
  template <int G0, int... Gs>
  __device__ __forceinline__ void issue(std::integer_sequence<int, Gs...>) {
    ((qa[G0 + Gs] = lds_quad_rd<(G0 + Gs) * LANE_BLOCK * 16>(addr)), ...);
  }
  template <int J>
  __device__ __forceinline__ uint2 operator()(std::integral_constant<int, J>) {
    if constexpr (J == 0) qq[0] = lds_quad_rd<FbpLds<S, PW>::q_off(0)>(addr);
    constexpr int from = Sc::issued(J - 1) + 1, to = Sc::issued(J);
    issue<from>(std::make_integer_sequence<int, (to >= from ? to - from + 1 : 0)>{});
    if constexpr (J % 4 == 0 && J / 4 + 1 < Sc::NQQ) qq[J / 4 + 1] = lds_quad_rd<FbpLds<S, PW>::q_off(J + 4)>(addr);
    constexpr int gl = ((28 * J) >> 5) / 4, gh = Sc::need(J), Q = J / 4;
    constexpr int need = pos_a(gh) > pos_q(Q) ? pos_a(gh) : pos_q(Q);
    constexpr int pending = before(J) + Sc::nA(J) + nq(J) - 1 - need;
    static_assert(pending >= 0 && pending <= 15, "lgkmcnt range");
    if constexpr (J == 0 || gh > Sc::need(J - 1) || J % 4 == 0) {   // a new a quad or a new q1 quad
      if constexpr (gl == gh) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(qa[gl]), "+v"(qq[Q]) : "i"(pending));
      else asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(qa[gl]), "+v"(qa[gh]), "+v"(qq[Q]) : "i"(pending));
    }
    return make_uint2(fbp_quad_digit<PW, J>(qa), quad_word<J % 4>(qq[Q]));
  }
};

// the b R words of this lane's row in LDS (quads PW/4 .. PW/2 - 1) into the running sum bs (PW words) + bc
template <int PW>
__device__ __forceinline__ void fbp_bsum_add(uint32_t (&bs)[PW], uint32_t& bc, const uint4* lrow) {
  unsigned int c = 0;
#pragma unroll
  for (int q = 0; q < PW / 4; ++q) {
    const uint4 v = lrow[(PW / 4 + q) * LANE_BLOCK];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) bs[4 * q + t] = __builtin_addc(bs[4 * q + t], w[t], c, &c);   // 32-bit add-with-carry chain
  }
  bc += c;
  // the sum is complete here: otherwise LLVM sinks the adds past the product (the sum is not read there) and keeps
  // the row words it loaded live across it
#pragma unroll
  for (int j = 0; j < PW; ++j) asm volatile("" : "+v"(bs[j]));
  asm volatile("" : "+v"(bc));
  __builtin_amdgcn_sched_barrier(0);
}

// (A, B) <- (A, B)(1 + p bs) = (A, B + REDC(A (bs R))), bs R = the words bs + bc 2^(32 PW) (< 2^(32 PW + 7), i.e.
// S canonical limbs); REDC(A bs R) < p + 2^8 p^2 / R < 2p, so B < 4p on exit
template <int S, int PW>
__device__ __forceinline__ void fbp_apply_bsum(uint32_t (&A)[S], uint32_t (&B)[S], const uint32_t (&bs)[PW], uint32_t bc,
                                               const uint32_t (&m)[S], uint32_t mprime) {
  static_assert(28 * S >= 32 * PW + 7, "the sum fits S limbs");
  uint32_t bl[S], U[S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    bl[j] = lane::limb_from_words([&](int w) { return w < PW ? bs[w] : bc; }, PW + 1, j);
    U[j] = A[j];
  }
  lane::mont_mul<S>(U, bl, m, mprime);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const uint32_t v = B[j] + U[j] + c;
    B[j] = v & lane::LMASK;
    c = v >> lane::LB;
  }
}

// c0 = 1 + n M as the pair (1, (n / p_h) M mod p_h), second component partially reduced (header)
template <int S>
__device__ __forceinline__ void fbp_c0(int64_t M, const FbpHalf* __restrict__ H, uint32_t (&A)[S], uint32_t (&B)[S]) {
  const bool neg = M < 0;
  const uint64_t mag = neg ? (uint64_t)0 - (uint64_t)M : (uint64_t)M;
  uint32_t mc[FBP_NC];
#pragma unroll
  for (int c = 0; c < FBP_NC; ++c) mc[c] = (uint32_t)((mag >> (FBP_CB * c)) & ((1ull << FBP_CB) - 1ull));
  const uint32_t* nm = opaque_uniform(H->nm);
  const uint32_t* pb = opaque_uniform(H->pbig);
  int64_t carry = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < FBP_NC; ++c) s += (uint64_t)nm[c * S + j] * mc[c];
    const int64_t v = carry + (neg ? (int64_t)pb[j] - (int64_t)s : (int64_t)s);
    B[j] = (uint32_t)v & lane::LMASK;
    carry = v >> lane::LB;
    A[j] = j == 0 ? 1u : 0u;
    __builtin_amdgcn_sched_barrier(0);
  }
}

// limb K of w = A + p B (product scanning; p in SGPRs)
template <int S, int K>
__device__ __forceinline__ uint64_t fbp_col(const uint32_t (&A)[S], const uint32_t (&B)[S], const uint32_t (&m)[S]) {
  uint64_t s = K < S ? (uint64_t)A[K] : 0ull;
  constexpr int lo = K < S ? 0 : K - S + 1, hi = K < S ? K : S - 1;
#pragma unroll
  for (int i = lo; i <= hi; ++i) s += (uint64_t)B[i] * m[K - i];
  return s;
}
template <int S, int SB, int... Ks>
__device__ __forceinline__ void fbp_store_w(const uint32_t (&A)[S], const uint32_t (&B)[S], const uint32_t (&m)[S], uint32_t* out,
                                            long long n, std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0;
  ((acc += fbp_col<S, Ks>(A, B, m), out[(size_t)Ks * n] = (uint32_t)acc & lane::LMASK, acc >>= lane::LB), ...);
}

// Per element and half: c0 prod_k T_k[d_k] mod p_h^2 by products with factored rows (header); row k in LDS
// (DMA one digit ahead, one buffer per wave, two waves per SIMD), as k_fb.
#ifndef FBP_RD
#define FBP_RD 3   // words read ahead of the digit that needs them
#endif
#ifndef FBP_QD
#define FBP_QD 2   // q1 digits read ahead in the second pass
#endif
#ifndef FBP_QUADS
#define FBP_QUADS 1   // row words and q1 digits by 16-byte reads (FbpAQuadReader), or one word per read
#endif
#ifndef FBP_DQ
#define FBP_DQ 1   // quads read ahead of the quad a digit needs
#endif
template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_fbp(FbpParams p) {
  using G = FbpGeom<S>;
  constexpr int SB = G::SB, PW = G::PW, TQ = 2 * PW / 4;
  __shared__ uint4 lbuf[FbpLds<S, PW>::NQ * LANE_BLOCK];
  const int half = blockIdx.y;
  const FbpHalf* H = p.halves + half;
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = H->p[j];
  const uint32_t mprime = H->mprime;
  const uint4* table = H->table;
  const int K = p.K, W = p.W;
  uint4* brow = lbuf + (threadIdx.x & ~63u);
  typedef __attribute__((address_space(3))) uint4 lds_uint4;
  const uint32_t addr0 = (uint32_t)(size_t)(lds_uint4*)(lbuf + threadIdx.x);
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const long long ii = i < p.n ? i : p.n - 1;
    const uint32_t* dg = p.digits + (size_t)half * K * p.n + ii;
    uint32_t d0 = dg[0];
    uint32_t dn = K > 1 ? dg[p.n] : 0u;
    double xv;
    int64_t xi = 0;
    if (p.dtype == 0) xv = (double)((const float*)p.x)[ii];
    else if (p.dtype == 1) xv = ((const double*)p.x)[ii];
    else { xi = ((const int64_t*)p.x)[ii]; xv = 0.0; }
    asm volatile("" : "+v"(d0), "+v"(dn), "+v"(xv), "+v"(xi));
    fb_row_to_lds<TQ>(table, d0, brow);
    int64_t M = 0;
    int e = 0, st;
    const bool fixed = p.exp_mode != 0;
    if (p.dtype == 2) st = encode_int(xi, fixed, p.fexp, M, e);
    else st = encode_float(xv, fixed, p.fexp, M, e);
    if (half == 0 && i < p.n) {
      p.exp[i] = e;
      if (p.status) p.status[i] = st;
    }
    uint32_t A[S], B[S];
    fbp_c0<S>(M, H, A, B);
    uint32_t bs[PW], bc = 0;
#pragma unroll
    for (int j = 0; j < PW; ++j) bs[j] = 0;
    uint32_t dn2 = K > 2 ? dg[2 * p.n] : 0u;
    for (int k = 0; k < K; ++k) {
      lds_dma_wait();                                     // row k landed, digit k+2 loaded
      fbp_bsum_add<PW>(bs, bc, lbuf + threadIdx.x);
#if FBP_QUADS
      pair::mont_mul_a0<S>(A, B, FbpAQuadReader<S, PW, FBP_DQ>{addr0}, FbpQPut<S, PW>{addr0},
                           FbpAQQuadReader<S, PW, FBP_DQ>{addr0}, m, mprime);
#else
      pair::mont_mul_a0<S>(A, B, FbpAReader<S, PW, FBP_RD>{addr0}, FbpQPut<S, PW>{addr0},
                           FbpAQReader<S, PW, FBP_RD, FBP_QD>{addr0}, m, mprime);
#endif
      if (k + 1 < K) {                                    // (every read of the row completed inside)
        const uint32_t dk1 = dn;
        dn = dn2;
        if (k + 3 < K) dn2 = dg[(size_t)(k + 3) * p.n];
        fb_row_to_lds<TQ>(table, ((size_t)(k + 1) << W) + dk1, brow);
      }
    }
    if (i < p.n) {
      fbp_apply_bsum<S, PW>(A, B, bs, bc, m, mprime);
      lane::cond_sub<S>(B, m);                            // B < 4p -> < 2p
      lane::cond_sub<S>(B, m);
      pair::canon<S>(A, B, m);
      uint32_t* o = p.out + fbp_pair_index<S>(i, half, p.n);
#pragma unroll
      for (int j = 0; j < 2 * S; ++j) o[j * 64] = j < S ? A[j] : B[j - S];
    }
  }
}

// ---------------------------------------------------------------- Garner on pairs -> ciphertext words
// c = w_q + q^2 h, h = (w_p - w_q) q^-2 mod p^2 (k_fb_fin's recombination) from the canonical pairs
// (A_p, B_p), (A_q, B_q) that k_fbp leaves (w_h = A_h + h B_h), with every product mod p^2 a pair product
// over the S limbs of p (bn_pair.hpp) and so in half the registers of k_fb_fin's 2S-limb products:
//   X = (B_q, 0) (q R)^ R^-1            = q B_q mod p^2                          4 S^2 MACs (B row zero)
//   D = (A_p + 4p - A_q - X_A,  B_p + 3p - X_B - 4)    == w_p - w_q, A < 5p, B < 4p (needs q < 2p)
//   H = D (q^-2 R)^ R^-1, canonical     = h = H_A + p H_B < p^2                  5 S^2
//   c = A_q + q B_q + q^2 H_A + p q^2 H_B (product scanning, words out)          6 S^2
// (u^ = the pair of u mod p^2.) Bounds: an operand below 5p (4p) keeps REDC's outputs below 2p while
// R > 10 p^2 / p; every column of the last sum takes at most 3S products < 2^56.
struct FbpFinParams {
  const uint32_t* pr;      // canonical pairs from k_fbp in 64-element tiles (fbp_pair_index; half 0: p, half 1: q)
  long long n;
  const uint32_t* p;       // S limbs of p
  const uint32_t* cs;      // 12 S words: (q^-1 R)^ [2S], (q^-2 R)^ [2S], q [S], q^2 [2S], p q^2 [3S], 2p [S], 3p [S]
  uint32_t mprime;         // -p^-1 mod 2^28
  uint32_t* ct;
  int ct_words;
  GuardArgs g;             // test build (guard.hpp): in = the pair tiles' words, out = n ct_words
};

template <int S>
struct FbpFin2Digits {   // digits (c1a, c1b, c2a, c2b) of C1 = (q^-2 R)^ at d + 2S and C2 = (q^-1 R)^ at d, one digit ahead
  const uint32_t* d;
  uint4 nx = make_uint4(0u, 0u, 0u, 0u);
  template <int J>
  __device__ __forceinline__ uint4 operator()(std::integral_constant<int, J>) {
    const uint4 r = J == 0 ? make_uint4(d[2 * S], d[3 * S], d[0], d[S]) : nx;
    if constexpr (J + 1 < S) nx = make_uint4(d[2 * S + J + 1], d[3 * S + J + 1], d[J + 1], d[S + J + 1]);
    return r;
  }
};

// the pair (A, B), A < 3p, B < 4p (B + 2 < 4p once A's multiples of p moved in) -> canonical A, B < p
template <int S>
__device__ __forceinline__ void fbpf_canon3(uint32_t (&A)[S], uint32_t (&B)[S], const uint32_t (&m)[S]) {
#pragma unroll 1
  for (int r = 0; r < 2; ++r) {
    uint32_t d[S];
    const bool lt = lane::sub<S>(A, m, d);
    uint32_t c = lt ? 0u : 1u;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      A[i] = lt ? A[i] : d[i];
      const uint32_t v = B[i] + c;
      B[i] = v & lane::LMASK;
      c = v >> lane::LB;
    }
  }
#pragma unroll 1
  for (int r = 0; r < 3; ++r) lane::cond_sub<S>(B, m);
}

// limb K of A_q + q B_q + q^2 H_A + p q^2 H_B (constants q, q^2, p q^2 at cq, cq + S, cq + 3S in LDS)
template <int S, int K>
__device__ __forceinline__ uint64_t fbpf_col(const uint32_t (&a1)[S], const uint32_t (&b1)[S], const uint32_t (&ha)[S],
                                             const uint32_t (&hb)[S], const uint32_t* __restrict__ cq) {
  uint64_t s = K < S ? (uint64_t)a1[K] : 0ull;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (K - i >= 0 && K - i < S) s += (uint64_t)b1[i] * cq[K - i];
    if (K - i >= 0 && K - i < 2 * S) s += (uint64_t)ha[i] * cq[S + K - i];
    if (K - i >= 0 && K - i < 3 * S) s += (uint64_t)hb[i] * cq[3 * S + K - i];
  }
  return s;
}
// The ciphertext words leave through the wave's LDS tile (dead once w_q is in registers), HW words of each ciphertext
// at a time (64 at nb = 2048, 32 at 1024: what a lane's share of the tile holds): each lane writes its words to its
// own row (stride HW + 4 words, padded against bank conflicts), then the wave stores the 64 rows as instructions of
// 1 KB, each whole HW-word pieces of 1024 / (4 HW) ciphertexts -- full lines, where per-lane 16-B stores 512 B apart
// left L2 to write back partial lines (1.8x the output bytes, profiles/pmc_k_fbp_fin_latest.json of round 3).
template <int CW>
struct FbpfHW {   // words per piece: 64 of a 2048-bit key's 128, 32 of a 1024-bit key's 64
  static constexpr int value = CW >= 128 ? 64 : 32;
};
template <int HW>
struct FbpfOut {
  static constexpr int OST = HW + 4, LPE = HW / 4, EPI = 64 / LPE;   // row stride; lanes per piece; pieces per store
  uint32_t lrow;       // this lane's row in the tile (LDS byte address)
  uint32_t tile;       // the tile (wave-uniform LDS byte address)
  uint32_t* ct;        // the wave's first ciphertext
  int ct_words, nvalid;   // words per ciphertext; valid elements of the wave (<= 64)
  int lane;
  __device__ __forceinline__ void put(int w, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {   // words w .. w+3
    const fbp_u32x4 v = {a, b, c, d};
    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(lrow), "v"(v), "i"(0) : "memory");
    lrow += 16;
    (void)w;
  }
  __device__ __forceinline__ void flush(int half) {   // rows -> words [64 half, 64 half + 64) of each ciphertext
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int sub = lane % LPE, el = lane / LPE;
#pragma unroll
    for (int g = 0; g < 64 / EPI; ++g) {
      const int e = EPI * g + el;
      fbp_u32x4 v;
      const uint32_t a = tile + (uint32_t)((e * OST + 4 * sub) * 4);
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) :: "memory");
      if (e < nvalid) *reinterpret_cast<fbp_u32x4*>(ct + (size_t)e * ct_words + HW * half + 4 * sub) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the rows are rewritten by the next piece)
    lrow -= HW * 4;
  }
};
template <int S, int CW, int K>
__device__ __forceinline__ void fbpf_out_step(uint64_t& acc, uint64_t& buf, uint32_t (&o4)[4], const uint32_t (&a1)[S],
                                              const uint32_t (&b1)[S], const uint32_t (&ha)[S], const uint32_t (&hb)[S],
                                              const uint32_t* __restrict__ cq, FbpfOut<FbpfHW<CW>::value>& out) {
  acc += fbpf_col<S, K>(a1, b1, ha, hb, cq);
  const uint32_t limb = (uint32_t)acc & lane::LMASK;
  acc >>= lane::LB;
  constexpr int NB = (28 * K) % 32;           // bits held in buf before this limb
  buf |= (uint64_t)limb << NB;
  if constexpr (NB + 28 >= 32) {
    constexpr int w = (28 * K) / 32;          // word completed by this limb
    o4[w % 4] = (uint32_t)buf;
    buf >>= 32;
    if constexpr (w % 4 == 3 && w < CW) {
      constexpr int HW = FbpfHW<CW>::value;
      out.put(w - 3, o4[0], o4[1], o4[2], o4[3]);
      if constexpr (w % HW == HW - 1) out.flush(w / HW);
    }
  }
}
template <int S, int CW, int... Ks>
__device__ __forceinline__ void fbpf_out_all(const uint32_t (&a1)[S], const uint32_t (&b1)[S], const uint32_t (&ha)[S],
                                             const uint32_t (&hb)[S], const uint32_t* __restrict__ cq, FbpfOut<FbpfHW<CW>::value>& out,
                                             std::integer_sequence<int, Ks...>) {
  static_assert(CW % FbpfHW<CW>::value == 0, "whole pieces");
  uint64_t acc = 0, buf = 0;
  uint32_t o4[4] = {0u, 0u, 0u, 0u};
  (fbpf_out_step<S, CW, Ks>(acc, buf, o4, a1, b1, ha, hb, cq, out), ...);
}

// The final sum as c = A_q + q (B_q + q h), h = H_A + p H_B < p^2 (2S limbs): three product-scanning passes whose
// multiplier limbs are p (SGPRs) and q (VGPRs, the same value in every lane), S^2 + 2 S^2 + 3 S^2 MACs -- the count of
// the direct sum over the constants q, q^2 and p q^2, but without an LDS read per MAC for the constant's limb.
template <int S, int K>
__device__ __forceinline__ uint64_t fbpf_hcol(const uint32_t (&ha)[S], const uint32_t (&hb)[S], const uint32_t (&m)[S]) {
  uint64_t s = K < S ? (uint64_t)ha[K] : 0ull;
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (K - i >= 0 && K - i < S) s += (uint64_t)hb[i] * m[K - i];
  return s;
}
template <int S, int... Ks>
__device__ __forceinline__ void fbpf_h(const uint32_t (&ha)[S], const uint32_t (&hb)[S], const uint32_t (&m)[S],
                                       uint32_t (&h)[2 * S], std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0;
  ((acc += fbpf_hcol<S, Ks>(ha, hb, m), h[Ks] = lane::limb32(acc), acc >>= lane::LB), ...);
}
template <int S, int K>
__device__ __forceinline__ uint64_t fbpf_tcol(const uint32_t (&h)[2 * S], const uint32_t (&qv)[S], const uint32_t* wq) {
  uint64_t s = K < S ? (uint64_t)wq[(S + K) * 64] : 0ull;   // B_q from the w_q tile
#pragma unroll
  for (int i = 0; i < 2 * S; ++i)
    if (K - i >= 0 && K - i < S) s += (uint64_t)h[i] * qv[K - i];
  return s;
}
template <int S, int... Ks>
__device__ __forceinline__ void fbpf_t(const uint32_t (&h)[2 * S], const uint32_t (&qv)[S], const uint32_t* wq,
                                       uint32_t (&t)[3 * S], std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0;
  ((acc += fbpf_tcol<S, Ks>(h, qv, wq), t[Ks] = lane::limb32(acc), acc >>= lane::LB), ...);
}
template <int S, int CW, int K>
__device__ __forceinline__ void fbpf_cstep(uint64_t& acc, uint64_t& buf, uint32_t (&o4)[4], const uint32_t (&t)[3 * S],
                                           const uint32_t (&qv)[S], const uint32_t (&a1)[S], FbpfOut<FbpfHW<CW>::value>& out) {
  uint64_t s = K < S ? (uint64_t)a1[K] : 0ull;
#pragma unroll
  for (int i = 0; i < 3 * S; ++i)
    if (K - i >= 0 && K - i < S) s += (uint64_t)t[i] * qv[K - i];
  acc += s;
  const uint32_t limb = (uint32_t)acc & lane::LMASK;
  acc >>= lane::LB;
  constexpr int NB = (28 * K) % 32;
  buf |= (uint64_t)limb << NB;
  if constexpr (NB + 28 >= 32) {
    constexpr int w = (28 * K) / 32;
    o4[w % 4] = (uint32_t)buf;
    buf >>= 32;
    if constexpr (w % 4 == 3 && w < CW) {
      constexpr int HW = FbpfHW<CW>::value;
      out.put(w - 3, o4[0], o4[1], o4[2], o4[3]);
      if constexpr (w % HW == HW - 1) out.flush(w / HW);
    }
  }
}
template <int S, int CW, int... Ks>
__device__ __forceinline__ void fbpf_c(const uint32_t (&t)[3 * S], const uint32_t (&qv)[S], const uint32_t (&a1)[S],
                                       FbpfOut<FbpfHW<CW>::value>& out, std::integer_sequence<int, Ks...>) {
  uint64_t acc = 0, buf = 0;
  uint32_t o4[4] = {0u, 0u, 0u, 0u};
  (fbpf_cstep<S, CW, Ks>(acc, buf, o4, t, qv, a1, out), ...);
}

// the wave's 64-element tile of half h's pairs (2S limbs x 64 elements, contiguous, 256-B aligned; tiles are padded
// to 64 elements) -> the wave's LDS tile at lb, 1 KB per DMA
template <int S>
__device__ __forceinline__ void fbpf_tile_dma(const uint32_t* pr, long long e0, int h, long long n, uint32_t lb, int lane,
                                              GuardArgs gd) {
  const size_t t0 = fbp_pair_index<S>(e0, h, n);
  uint64_t src = (uint64_t)(reinterpret_cast<const uint4*>(pr + (FPAI_GUARD_OK(gd, GS_FIN_TILE, t0 + 2 * S * 64 - 1, gd.in, e0) ? t0 : 0)) + lane);
  constexpr int NI = (32 * S + 63) / 64, REM = (32 * S) % 64;
#pragma unroll
  for (int g = 0; g < NI; ++g) {
    uint32_t dst = lb + (uint32_t)(g * 1024);
    asm volatile("" : "+s"(dst));
    if (REM == 0 || g + 1 < NI || lane < REM)
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(size_t)dst, 16, 0, 0);
    src += 1024;
    asm volatile("" : "+v"(src));   // one address register, advanced per DMA (not 19 precomputed)
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int S>
__global__ __launch_bounds__(LANE_BLOCK, 2) void k_fbp_fin(FbpFinParams p) {
  constexpr int CW = 2 * FbGeom<FbpGeom<S>::SB>::TW;   // ciphertext words
  constexpr int NL = (32 * CW + 27) / 28;             // limbs that cover them
  static_assert(NL <= 4 * S, "c < n^2 fits 4 S limbs");
  __shared__ uint32_t cs[12 * S];
  // the waves' 64-element tiles of w_p pairs (2S limbs x 64 elements each), streamed in by DMA during X's product; then
  // w_q's tile for the final sum, then the ciphertext rows on the way out
  __shared__ __attribute__((aligned(16))) uint32_t wpl[(LANE_BLOCK / 64) * 2 * S * 64];
  for (int j = threadIdx.x; j < 12 * S; j += blockDim.x) cs[j] = p.cs[j];
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = p.p[j];
  const uint32_t mprime = p.mprime;
  const uint32_t* p2 = cs + 10 * S;
  const uint32_t* p3 = cs + 11 * S;
  const int lane = threadIdx.x & 63;
  uint32_t* wpp = wpl + (threadIdx.x >> 6) * 2 * S * 64;   // limb j of this lane's w_p at wpp[64 j + lane]
  for (long long base = (long long)blockIdx.x * LANE_BLOCK; base < p.n; base += (long long)gridDim.x * LANE_BLOCK) {
    const long long i = base + threadIdx.x;
    const bool valid = i < p.n;
    const long long ii = valid ? i : p.n - 1;
    const size_t iq = fbp_pair_index<S>(ii, 1, p.n);
    const uint32_t* pq = p.pr + (FPAI_GUARD_OK(p.g, GS_FIN_TILE, iq + (2 * S - 1) * 64, p.g.in, ii) ? iq : 0);
    // the wave's first element (wave-uniform: in SGPRs, so it costs no VGPRs across the products)
    long long e0 = base + (long long)(uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
    const bool wave_live = e0 < p.n;   // (a wave past the end computes the last element; it must not store)
    if (!wave_live) e0 = (p.n - 1) & ~63ll;
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    {   // the wave's w_p tile -> LDS
      const uint32_t lb = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_u32*)wpp);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous element's reads of the tile are done
      fbpf_tile_dma<S>(p.pr, e0, 0, p.n, lb, lane, p.g);
    }
    // Y = w_q q^-2 mod p^2 = A_q q^-2 + B_q q^-1: one lock-step pass over the two B-free operands (bn_pair.hpp
    // mont_mul2_a0), 6 S^2 MACs
    uint32_t xa[S], xb[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      xa[j] = pq[j * 64];
      xb[j] = pq[(S + j) * 64];
    }
    pair::mont_mul2_a0<S>(xa, xb, FbpFin2Digits<S>{cs}, m, mprime);
    // h = w_p q^-2 - Y (the p half's position-0 rows carry q^-2, FbpHalf::kapR), as the pair
    // D = (W_A + 2p - Y_A, W_B + 3p - Y_B - 2): parts in (0, 3p) and (p - 2, 4p), then canonical
    {
      lds_dma_wait();   // the w_p tile landed
      int tx = threadIdx.x;
      asm volatile("" : "+v"(tx));   // (the tile address is rebuilt here, not held across the products)
      const uint32_t* wq = wpl + (tx >> 6) * 2 * S * 64 + (tx & 63);
      int64_t ca = 0, cb = 0;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const int64_t va = (int64_t)wq[j * 64] + (int64_t)p2[j] - (int64_t)xa[j] + ca;
        const int64_t vb = (int64_t)wq[(S + j) * 64] + (int64_t)p3[j] - (int64_t)xb[j] - (j == 0 ? 2 : 0) + cb;
        xa[j] = (uint32_t)va & lane::LMASK;
        xb[j] = (uint32_t)vb & lane::LMASK;
        ca = va >> lane::LB;
        cb = vb >> lane::LB;
      }
    }
    fbpf_canon3<S>(xa, xb, m);
    {   // w_p is consumed: the wave's w_q tile -> the same LDS tile, read by the final sum (instead of w_q from HBM a
        // second time); issued after h's product, which holds every register
      const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t lb = (uint32_t)(size_t)(lds_u32*)(wpl + wv * 2 * S * 64);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every lane's reads of w_p are done
      int ln = threadIdx.x & 63;
      asm volatile("" : "+v"(ln));
      fbpf_tile_dma<S>(p.pr, e0, 1, p.n, lb, ln, p.g);
    }
    // c = w_q + q^2 h = A_q + q (B_q + q h), h = H_A + p H_B (fbpf_h / fbpf_t / fbpf_c)
    uint32_t t[3 * S];
    {
      uint32_t h[2 * S];
      fbpf_h<S>(xa, xb, m, h, std::make_integer_sequence<int, 2 * S>{});
      uint32_t qv[S];
#pragma unroll
      for (int j = 0; j < S; ++j) qv[j] = cs[4 * S + j];
      lds_dma_wait();   // the w_q tile landed
      int tx = threadIdx.x;
      asm volatile("" : "+v"(tx));
      const uint32_t* wq = wpl + (tx >> 6) * 2 * S * 64 + (tx & 63);
      fbpf_t<S>(h, qv, wq, t, std::make_integer_sequence<int, 3 * S>{});
    }
    {
      uint32_t a1[S], qv[S];
      int tx = threadIdx.x;
      asm volatile("" : "+v"(tx));
      const uint32_t* wq = wpl + (tx >> 6) * 2 * S * 64 + (tx & 63);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        a1[j] = wq[j * 64];
        qv[j] = cs[4 * S + j];
      }
      using Out = FbpfOut<FbpfHW<CW>::value>;
      static_assert(64 * Out::OST <= 2 * S * 64, "the output rows fit the tile");
      const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t tile = (uint32_t)(size_t)(lds_u32*)(wpl + wv * 2 * S * 64);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every lane's reads of w_q are done (a1 in registers)
      const long long left = p.n - e0;
      const uint64_t cta = (uint64_t)(p.ct + (size_t)e0 * p.ct_words);   // wave-uniform: SGPRs
      // (readfirstlane returns int: through uint32_t, or an address half >= 2^31 sign-extends)
      uint32_t* ctw = (uint32_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cta >> 32)) << 32) |
                                  (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cta));
      int ln = threadIdx.x & 63;
      asm volatile("" : "+v"(ln));
      int nv = wave_live ? (int)__builtin_amdgcn_readfirstlane((uint32_t)(left < 64 ? left : 64)) : 0;
      if (nv > 0 && !FPAI_GUARD_OK(p.g, GS_FIN_CT, (size_t)(e0 + nv) * p.ct_words - 1, p.g.out, e0)) nv = 0;
      Out out{tile + (uint32_t)(ln * Out::OST * 4), tile, ctw, p.ct_words, nv, ln};
      fbpf_c<S, CW>(t, qv, a1, out, std::make_integer_sequence<int, NL>{});
    }
  }
}

// ---------------------------------------------------------------- per-key table in pair form
// k_fbp_lohi: per position k, lo[j] = B_k^j R (j < 2^LO) and hi[j] = B_k^(2^LO j) R (j < 2^(W-LO)) by
// square-and-multiply from R (the pair of one; position 0's lo entries times kappa R, FbpHalf::kapR, so that
// T_0[d] = kappa B_0^d); k_fbp_inv_*: the inverses of their A parts mod p_h; k_fbp_fill:
// T_k[d] R = lo[d & (2^LO - 1)] hi[d >> LO] R^-1, one pair product per entry, factored (header) and stored as words.
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_fbp_lohi(const FbpHalf* halves, int K, int W) {
  const int k = blockIdx.x, half = blockIdx.y;
  const FbpHalf* H = halves + half;
  const int LO = W / 2, HI = W - LO;
  uint32_t m[S], A[S], B[S];
#pragma unroll
  for (int i = 0; i < S; ++i) m[i] = H->p[i];
  for (int s = 0; s < 2; ++s) {
    const int bits = s ? HI : LO;
    const uint32_t* x = H->bases + ((size_t)k * 2 + s) * 2 * S;
    for (uint32_t j = threadIdx.x; j < (1u << bits); j += blockDim.x) {
#pragma unroll
      for (int i = 0; i < S; ++i) {
        A[i] = H->oneR[i];
        B[i] = H->oneR[S + i];
      }
      for (int b = bits - 1; b >= 0; --b) {
        pair::mont_sqr<S>(A, B, m, H->mprime);
        if ((j >> b) & 1u)
          pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(x[decltype(J)::value], x[S + decltype(J)::value]); }, m,
                            H->mprime);
      }
      if (k == 0 && s == 0) {   // position 0's lo entries carry kappa
        const uint32_t* kr = H->kapR;
        pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(kr[decltype(J)::value], kr[S + decltype(J)::value]); }, m,
                          H->mprime);
      }
      uint32_t* o = H->lohi + (((size_t)k * 2 + s) * FB_LO + j) * 2 * S;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        o[i] = A[i];
        o[S + i] = B[i];
      }
    }
  }
}

template <int S, int... Gs>
__device__ __forceinline__ void fbp_store_row(uint4* __restrict__ dst, const uint32_t (&A)[S], const uint32_t (&B)[S],
                                              std::integer_sequence<int, Gs...>) {
  ((dst[Gs] = make_uint4(fb_word<S, 4 * Gs>(A), fb_word<S, 4 * Gs + 1>(A), fb_word<S, 4 * Gs + 2>(A), fb_word<S, 4 * Gs + 3>(A))), ...);
  ((dst[sizeof...(Gs) + Gs] =
        make_uint4(fb_word<S, 4 * Gs>(B), fb_word<S, 4 * Gs + 1>(B), fb_word<S, 4 * Gs + 2>(B), fb_word<S, 4 * Gs + 3>(B))),
   ...);
}

// Batch inversion of the lo/hi entries' A parts (Montgomery's trick; kernels_grp_pair.hpp's k_pair_inv_* on the lane
// engine), one lane per chain c = (k, lo|hi) of a half, R-forms throughout: k_fbp_inv_fwd writes the prefix products
// P_j = (L_0 .. L_j) R and the chain's product; the host (pair_host_invert) turns each chain product into its inverse
// I = (L_0 .. L_(E-1))^-1 R; k_fbp_inv_bwd: inv_j = I_j P_(j-1) = L_j^-1 R, I_(j-1) = I_j L_j.
template <int S>
struct FbpInvChain {
  int E;
  bool valid;
  const uint32_t* lh;   // entry j's A part at lh + 2 S j
  uint32_t* pre;        // prefix product j at pre + S j
  uint32_t* inv;        // inverse j at inv + S j
  uint32_t* cval;
  __device__ FbpInvChain(const FbpHalf* H, int K, int W) {
    const int c0 = blockIdx.x * blockDim.x + threadIdx.x;
    valid = c0 < 2 * K;
    const int c = valid ? c0 : 0, k = c >> 1, sp = c & 1;
    const int LO = W / 2, HI = W - LO, EM = 1 << (HI > LO ? HI : LO);
    E = 1 << (sp ? HI : LO);
    lh = H->lohi + ((size_t)k * 2 + sp) * FB_LO * 2 * S;
    pre = H->pre + (size_t)c * EM * S;
    inv = H->inv + ((size_t)k * 2 + sp) * FB_LO * S;
    cval = H->cval + (size_t)c * S;
  }
};

template <int S>
__global__ __launch_bounds__(64) void k_fbp_inv_fwd(const FbpHalf* halves, int K, int W) {
  const FbpHalf* H = halves + blockIdx.y;
  const FbpInvChain<S> ch(H, K, W);
  if (!ch.valid) return;
  uint32_t m[S], acc[S], x[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    m[i] = H->p[i];
    acc[i] = ch.lh[i];
    ch.pre[i] = acc[i];
  }
  for (int j = 1; j < ch.E; ++j) {
#pragma unroll
    for (int i = 0; i < S; ++i) x[i] = ch.lh[(size_t)j * 2 * S + i];
    lane::mont_mul<S>(acc, x, m, H->mprime);
#pragma unroll
    for (int i = 0; i < S; ++i) ch.pre[(size_t)j * S + i] = acc[i];
  }
  lane::cond_sub<S>(acc, m);
#pragma unroll
  for (int i = 0; i < S; ++i) ch.cval[i] = acc[i];
}

template <int S>
__global__ __launch_bounds__(64) void k_fbp_inv_bwd(const FbpHalf* halves, int K, int W) {
  const FbpHalf* H = halves + blockIdx.y;
  const FbpInvChain<S> ch(H, K, W);
  if (!ch.valid) return;
  uint32_t m[S], I[S], x[S], t[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    m[i] = H->p[i];
    I[i] = ch.cval[i];
  }
  for (int j = ch.E - 1; j >= 1; --j) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      t[i] = I[i];
      x[i] = ch.pre[(size_t)(j - 1) * S + i];
    }
    lane::mont_mul<S>(t, x, m, H->mprime);
    lane::cond_sub<S>(t, m);
#pragma unroll
    for (int i = 0; i < S; ++i) {
      ch.inv[(size_t)j * S + i] = t[i];
      x[i] = ch.lh[(size_t)j * 2 * S + i];
    }
    lane::mont_mul<S>(I, x, m, H->mprime);
  }
  lane::cond_sub<S>(I, m);
#pragma unroll
  for (int i = 0; i < S; ++i) ch.inv[i] = I[i];
}

// T' = lo hi R^-1 = L H R as its canonical pair (A, B), then the factored row (header): a = A, b R = B (L H)^-1 =
// REDC(B X) with X = REDC(inv_lo inv_hi) = (L H)^-1 R
template <int S>
__global__ __launch_bounds__(LANE_BLOCK) void k_fbp_fill(const FbpHalf* halves, int K, int W, uint4* table0, uint4* table1) {
  constexpr int PW = FbpGeom<S>::PW, TQ = 2 * PW / 4;
  const int ent = 1 << W;
  const int per = (ent + LANE_BLOCK - 1) / LANE_BLOCK;
  const int k = blockIdx.x / per;
  const int d = (blockIdx.x % per) * LANE_BLOCK + threadIdx.x;
  if (d >= ent) return;
  const int half = blockIdx.y;
  const FbpHalf* H = halves + half;
  uint4* table = half ? table1 : table0;
  const int LO = W / 2;
  const int dl = d & ((1 << LO) - 1), dh = d >> LO;
  const uint32_t* lo = H->lohi + (((size_t)k * 2 + 0) * FB_LO + dl) * 2 * S;
  const uint32_t* hi = H->lohi + (((size_t)k * 2 + 1) * FB_LO + dh) * 2 * S;
  uint32_t m[S], A[S], B[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    m[i] = H->p[i];
    A[i] = lo[i];
    B[i] = lo[S + i];
  }
  pair::mont_mul<S>(A, B, [&](auto J) { return make_uint2(hi[decltype(J)::value], hi[S + decltype(J)::value]); }, m, H->mprime);
  pair::canon<S>(A, B, m);
  {
    const uint32_t* il = H->inv + (((size_t)k * 2 + 0) * FB_LO + dl) * S;
    const uint32_t* ih = H->inv + (((size_t)k * 2 + 1) * FB_LO + dh) * S;
    uint32_t X[S], Y[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      X[i] = il[i];
      Y[i] = ih[i];
    }
    lane::mont_mul<S>(X, Y, m, H->mprime);
    lane::mont_mul<S>(B, X, m, H->mprime);
    lane::cond_sub<S>(B, m);
  }
  fbp_store_row<S>(table + ((size_t)k * ent + d) * TQ, A, B, std::make_integer_sequence<int, PW / 4>{});
}

}  // namespace fpai
