// Lane-group big-number engine for gfx950 (CDNA4): one Paillier operand per group of TPI
// lanes inside a 64-lane wavefront, L = 37 limbs of LB = 28 bits per lane.
//
// Why 28-bit limbs: on gfx950 `v_mad_u64_u32` issues at ~0.85 of the full VALU rate
// (profiles/r01_step0_int_throughput.txt), so the cheapest 32x32->64 MAC is ONE mad into a
// 64-bit accumulator. In the rotating CIOS loop below a physical accumulator lives for L
// iterations and receives at most 2 products (< 2^56) per iteration plus one carry (< 2^36):
// 74 * 2^56 + 2^36 < 2^62.3, so no carry handling is needed inside the loop ("lazy"
// accumulators). Carries are resolved once per product (normalize) with an in-lane pass, a DPP
// lane shift and a ballot carry-lookahead. L = 37 keeps the per-iteration overhead (digit
// broadcast, one-limb shift) at ~9% of the 2L MACs; TPI = 4 covers n^2 of a 2048-bit key
// (4 * 37 * 28 = 4144 bits), TPI = 2 covers p^2.
//
// Layout: lane t of a group owns limbs [Lt, Lt+L) of every operand (lane-major), so the
// per-iteration Montgomery shift moves only ONE 27-bit value across lanes (DPP row_shl:1),
// and the reduction digit q is broadcast from the group's lane 0 with DPP (no LDS).
// The multiplicand B of every product is read limb by limb from the group's LDS slot as a
// same-address broadcast.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace fpai {

constexpr int LB = 28;                        // limb bits
constexpr uint32_t LMASK = (1u << LB) - 1u;
constexpr int L = 37;                         // limbs per lane

// ---------------------------------------------------------------- cross-lane primitives
// lane i <- lane i+1 within a 16-lane DPP row; lanes whose source is outside the row get 0.
__device__ __forceinline__ uint32_t dpp_from_next(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x101, 0xF, 0xF, true);
}
// lane i <- lane i-1 within a row; row lane 0 gets 0.
__device__ __forceinline__ uint32_t dpp_from_prev(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);
}

// Broadcast the value held by the group's first lane to all TPI lanes of the group.
template <int TPI>
__device__ __forceinline__ uint32_t bcast0(uint32_t v) {
  static_assert(TPI == 1 || TPI == 2 || TPI == 4 || TPI == 8 || TPI == 16, "TPI");
  if constexpr (TPI == 1) {
    return v;
  } else if constexpr (TPI == 2) {   // every lane is written: no old value (saves a v_mov per broadcast)
    return __builtin_amdgcn_mov_dpp(v, 0xA0, 0xF, 0xF, false);          // quad_perm [0,0,2,2]
  } else if constexpr (TPI == 4) {
    return __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, false);          // quad_perm [0,0,0,0]
  } else if constexpr (TPI == 8) {
    uint32_t t = __builtin_amdgcn_update_dpp(0u, v, 0x00, 0xF, 0xF, false);
    return __builtin_amdgcn_update_dpp(t, t, 0x114, 0xF, 0xA, false);   // row_shr:4 into banks 1,3
  } else {
    return __builtin_amdgcn_update_dpp(0u, v, 0x150, 0xF, 0xF, false);  // row_newbcast:0
  }
}

// bit mask of the top lane of every group within the 64-lane wave
template <int TPI>
__device__ __forceinline__ uint64_t top_lanes_mask() {
  uint64_t m = 0;
#pragma unroll
  for (int g = TPI - 1; g < 64; g += TPI) m |= 1ull << g;
  return m;
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Given per-lane "generate" and "propagate" predicates of a carry (or borrow) chain running
// from lane 0 upwards inside each group, return the carry INTO this lane. Propagation is cut at
// group boundaries.
template <int TPI>
__device__ __forceinline__ uint32_t lookahead_carry_in(bool g, bool p, int lane) {
  // The top lane of each group neither generates nor propagates here (its carry OUT is the
  // group's overflow/sign and is derived by the caller), so nothing leaks into the next group.
  const uint64_t keep = ~top_lanes_mask<TPI>();
  const uint64_t G = ballot(g) & keep;
  const uint64_t X = G | (ballot(p) & keep);
  const uint64_t S = X + G;
  const uint64_t cin = S ^ X ^ G;
  return (uint32_t)((cin >> lane) & 1ull);
}

// ---------------------------------------------------------------- normalisation
// P holds the value sum_i P[i] * 2^(LB*(Lt+i)) (unsigned 64-bit accumulators, < 2^63).
// Produce canonical LB-bit limbs r. The total must be < 2^(LB*L*TPI).
template <int TPI>
__device__ __forceinline__ void normalize(const uint64_t (&P)[L], uint32_t (&r)[L], int lane, int tig) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint64_t v = P[i] + c;
    r[i] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  uint32_t inlo = dpp_from_prev((uint32_t)c);
  uint32_t inhi = dpp_from_prev((uint32_t)(c >> 32));
  if (tig == 0) { inlo = 0; inhi = 0; }
  c = ((uint64_t)inhi << 32) | inlo;
  {
    const uint64_t v = (uint64_t)r[0] + c;
    r[0] = (uint32_t)v & LMASK;
    c = v >> LB;
  }
  uint32_t c32 = (uint32_t)c;
#pragma unroll
  for (int i = 1; i < L; ++i) {
    const uint32_t v = r[i] + c32;
    r[i] = v & LMASK;
    c32 = v >> LB;
  }
  // c32 in {0,1}: resolve lane-to-lane ripple (almost never needed)
  if (ballot(c32 != 0) != 0ull) {
    bool all_ones = true;
#pragma unroll
    for (int i = 0; i < L; ++i) all_ones &= (r[i] == LMASK);
    uint32_t ci = lookahead_carry_in<TPI>(c32 != 0, all_ones, lane);
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint32_t v = r[i] + ci;
      r[i] = v & LMASK;
      ci = v >> LB;
    }
  }
}

// d = a - b for canonical limb vectors. Returns true (group-uniform) when a < b; d is then
// the two's-complement wrap and must be discarded by the caller.
template <int TPI>
__device__ __forceinline__ bool sub_limbs(const uint32_t (&a)[L], const uint32_t (&b)[L], uint32_t (&d)[L],
                                          int lane, int tig) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t v = (int32_t)a[i] - (int32_t)b[i] + c;
    d[i] = (uint32_t)v & LMASK;
    c = v >> LB;            // arithmetic: -1 or 0
  }
  const int32_t b1 = c;     // pass-1 borrow out of this lane
  int32_t bin = (int32_t)dpp_from_prev((uint32_t)c);
  if (tig == 0) bin = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t v = (int32_t)d[i] + bin;
    d[i] = (uint32_t)v & LMASK;
    bin = v >> LB;
  }
  // bin in {-1,0}: borrow out of this lane. Lookahead for lanes whose limbs are all zero.
  bool all_zero = true;
#pragma unroll
  for (int i = 0; i < L; ++i) all_zero &= (d[i] == 0u);
  const bool gen = (bin != 0);
  const uint32_t bi = lookahead_carry_in<TPI>(gen, all_zero, lane);
  if (ballot(bi != 0) != 0ull) {
    int32_t b2 = -(int32_t)bi;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int32_t v = (int32_t)d[i] + b2;
      d[i] = (uint32_t)v & LMASK;
      b2 = v >> LB;
    }
  }
  // borrow out of the top lane of the group = sign (at most one of the three can be set there,
  // since |a - b| < 2^(LB*L*TPI))
  const bool neg_here = (tig == TPI - 1) && (b1 != 0 || gen || (all_zero && bi));
  const uint64_t NB = ballot(neg_here);
  const int gbase = lane - tig;
  return ((NB >> (gbase + TPI - 1)) & 1ull) != 0ull;
}

// r <- r - m if r >= m (r < 2m on entry); canonical result.
template <int TPI>
__device__ __forceinline__ void cond_sub(uint32_t (&r)[L], const uint32_t (&m)[L], int lane, int tig) {
  uint32_t d[L];
  const bool neg = sub_limbs<TPI>(r, m, d, lane, tig);
  if (!neg) {
#pragma unroll
    for (int i = 0; i < L; ++i) r[i] = d[i];
  }
}

// ---------------------------------------------------------------- CIOS Montgomery loop
// Runs nouter*L iterations j of
//     T += a * B[j]           (if AB)
//     q  = (T_0 * mprime) mod 2^LB, broadcast from group lane 0
//     T += q * m ; T >>= LB   (lazy: only T_0's carry is moved, to T_1)
// with B read from the group's LDS slot. If COLLECT, digit q of iteration j is stored in
// out[j % L] of group lane j / L (used for exact division).
// After a multiple of L iterations the rotating register mapping is the identity again.
// The one-limb shift moves each lane's lowest limb to the previous lane's top slot; a group's
// top lane receives the next group's lowest limb, which is 0 mod 2^LB after the reduction step.
// One CIOS iteration with a compile-time rotation S_ (the L iterations of an outer step are
// expanded by an index_sequence, so the accumulator indices are constants and P stays in VGPRs;
// a plain `#pragma unroll` is not honoured at L = 37).
template <int TPI, bool AB, bool COLLECT, int S_>
__device__ __forceinline__ void cios_step(uint64_t (&P)[L], const uint32_t (&a)[L], const uint32_t* __restrict__ Bo,
                                          uint32_t& bcur, const uint32_t (&m)[L], uint32_t mprime, bool collect_here,
                                          uint32_t (&out)[L]) {
  if constexpr (AB) {
    const uint32_t bj = bcur;
    // B digit of the next iteration, read one iteration ahead (the LDS latency hides behind
    // this iteration's 2L MACs; the scheduler is fenced per iteration below)
    if constexpr (S_ + 1 < L) bcur = Bo[S_ + 1];
#pragma unroll
    for (int i = 0; i < L; ++i) P[(i + S_) % L] += (uint64_t)a[i] * bj;
  }
  const uint32_t q = bcast0<TPI>(((uint32_t)P[S_] * mprime) & LMASK);
  if constexpr (COLLECT) out[S_] = collect_here ? q : out[S_];
#pragma unroll
  for (int i = 0; i < L; ++i) P[(i + S_) % L] += (uint64_t)q * m[i];
  const uint64_t v0 = P[S_];
  P[(S_ + 1) % L] += v0 >> LB;
  P[S_] = (uint64_t)dpp_from_next((uint32_t)v0 & LMASK);
  // Pin every accumulator at the iteration boundary: without this, the fully unrolled chain of
  // adds is re-associated into per-column dependent MAC chains (product scanning), which is
  // latency-bound. With it, each iteration is 2L independent MACs.
#pragma unroll
  for (int i = 0; i < L; ++i) asm volatile("" : "+v"(P[i]));
  // keep the scheduler from interleaving whole iterations (it hoists the B loads and the next
  // products and runs out of VGPRs); one iteration alone has 2L independent MACs of ILP
  __builtin_amdgcn_sched_barrier(0);
}

template <int TPI, bool AB, bool COLLECT, int... Ss>
__device__ __forceinline__ void cios_outer(uint64_t (&P)[L], const uint32_t (&a)[L], const uint32_t* __restrict__ Bo,
                                           const uint32_t (&m)[L], uint32_t mprime, bool collect_here,
                                           uint32_t (&out)[L], std::integer_sequence<int, Ss...>) {
  uint32_t bcur = 0;
  if constexpr (AB) bcur = Bo[0];
  (cios_step<TPI, AB, COLLECT, Ss>(P, a, Bo, bcur, m, mprime, collect_here, out), ...);
}

template <int TPI, bool AB, bool COLLECT>
__device__ __forceinline__ void cios(uint64_t (&P)[L], const uint32_t (&a)[L], const uint32_t* __restrict__ Bsh,
                                     int nouter, const uint32_t (&m)[L], uint32_t mprime, int tig,
                                     uint32_t (&out)[L]) {
  for (int o = 0; o < nouter; ++o) {
    cios_outer<TPI, AB, COLLECT>(P, a, AB ? Bsh + o * L : nullptr, m, mprime, tig == o, out,
                                 std::make_integer_sequence<int, L>{});
  }
}

// Compiler-level ordering for LDS traffic inside one wavefront (LDS executes a wave's DS
// instructions in order, so program order is all that is needed between lanes of a group).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int TPI>
__device__ __forceinline__ void write_limbs_lds(uint32_t* Bsh, const uint32_t (&x)[L], int tig) {
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < L; ++i) Bsh[tig * L + i] = x[i];
  wave_lds_fence();
}

// r = a * B * 2^(-LB*L*TPI*k) mod m, where B (L*TPI*k limbs) is in the LDS slot, k = nouter/TPI.
// Inputs a < 2m (or < 4m when R > 8m), B < 2m  ->  r < 2m, canonical limbs.
template <int TPI>
__device__ __forceinline__ void montmul(uint32_t (&r)[L], const uint32_t (&a)[L], const uint32_t* Bsh, int nouter,
                                        const uint32_t (&m)[L], uint32_t mprime, int lane, int tig) {
  uint64_t P[L];
#pragma unroll
  for (int i = 0; i < L; ++i) P[i] = 0;
  uint32_t dummy[L];
  cios<TPI, true, false>(P, a, Bsh, nouter, m, mprime, tig, dummy);
  normalize<TPI>(P, r, lane, tig);
}

// ---------------------------------------------------------------- limb <-> word packing
// words: little-endian 32-bit words of an integer (nwords of them). Lane tig extracts its
// L limbs of LB bits.
template <typename Ptr>
__device__ __forceinline__ void words_to_limbs(Ptr words, int nwords, uint32_t (&x)[L], int tig) {
  // opaque copy: stops LICM from hoisting the L per-limb (word index, shift, bound) triples out
  // of the caller's element loop, which would pin ~3L VGPRs for the whole kernel
  int t = tig;
  asm volatile("" : "+v"(t));
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = (t * L + i) * LB;
    const int wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = (wi < nwords) ? (uint64_t)words[wi] : 0ull;
    const uint64_t hi = (wi + 1 < nwords) ? (uint64_t)words[wi + 1] : 0ull;
    x[i] = (uint32_t)(((hi << 32) | lo) >> sh) & LMASK;
  }
}

// Produce 32-bit word j (bits [32j, 32j+32)) from canonical limbs held in an LDS slot of
// `nlimbs` limbs.
__device__ __forceinline__ uint32_t limbs_word(const uint32_t* limbs, int nlimbs, int j) {
  const int bit = 32 * j;
  const int k = bit / LB, sh = bit - k * LB;
  uint64_t v = (uint64_t)limbs[k] >> sh;
  if (k + 1 < nlimbs) v |= (uint64_t)limbs[k + 1] << (LB - sh);
  if (k + 2 < nlimbs && 2 * LB - sh < 32) v |= (uint64_t)limbs[k + 2] << (2 * LB - sh);
  return (uint32_t)v;
}

}  // namespace fpai
