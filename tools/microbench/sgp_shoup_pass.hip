// Feasibility measurement for Shoup rows in k_sgp: the arithmetic of one
// table-row product on split pairs at S = 74 (even lane A, odd lane B), rows already in LDS (no row stream), as
//   mont<W>   : k_sgp's Montgomery split pass (kernels_sgp.hpp sgp_pass, 2 S^2 lane-MACs), W waves per SIMD;
//   shoup<W,L>: the Shoup product of kernels_fbs.hpp at S = 74 (S (S + 1) / 2 + S (S + 1) lane-MACs): step 1 the
//               quotient from the columns >= S - 1 of X a' (75 accumulators), step 2 the columns 0 .. S - 1 of
//               X a + Q (R - p) in two sweeps of 37 columns (X, Q and 37 accumulators: 222 VGPRs), the first
//               sweep's limbs stashed -- in AGPRs (L = 0) or in LDS (L = 1) -- while the second runs.
// Each lane pair runs K dependent products (row k & 1 for product k); the first 64 pairs' results are written and
// checked against Python's big integers (tools/microbench/sgp_shoup_vec.py). Reported: pair-products per second.
//   python tools/microbench/sgp_shoup_vec.py gen /tmp/v.bin
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ibond-flex_amd/csrc tools/microbench/sgp_shoup_pass.hip -o ssp
//   ./ssp v.bin K out_prefix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "kernels_sgp.hpp"

using namespace fpai;

constexpr int S = SGP_S, NQ = (S + 3) / 4, SA = 37, SB = S - SA, PAIRS = 64;
constexpr int VEC_WORDS = S + 1 + 4 * S + 128 + PAIRS * 2 * S;

struct Vec {
  const uint32_t *m, *a, *ap, *aw, *x;
  uint32_t mprime;
};

template <int J>
__device__ __forceinline__ uint32_t qword(const uint4& v) {
  return J == 0 ? v.x : J == 1 ? v.y : J == 2 ? v.z : v.w;
}

// ---------------------------------------------------------------- Shoup
// LDS rows, [buffer][number: a, a'][quad][pair of the wave] 16 B each: both lanes of a pair read one address (one
// copy per block, read by its four waves: the same banks as four copies, a quarter of the LDS)
constexpr int SH_WAVE_Q = 2 * 2 * NQ * 32;   // uint4 (2 buffers)
__device__ __forceinline__ const uint4* sh_num(const uint4* wave, int buf, int num, int pw) {
  return wave + (buf * 2 + num) * NQ * 32 + pw;
}

// step 1, consumption index T (J = S - 1 - T, quads descending)
template <int T>
__device__ __forceinline__ void s1_digit(uint64_t (&P)[S + 1], const uint32_t (&X)[S], const uint4* q, uint4& cur, uint4& nxt) {
  constexpr int J = S - 1 - T;
  if constexpr (T > 0 && J % 4 == 3) cur = nxt;
  if constexpr ((T == 0 || J % 4 == 3) && J / 4 > 0) nxt = q[(J / 4 - 1) * 32];
  const uint32_t d = qword<J % 4>(cur);
#pragma unroll
  for (int i = S - 1 - J; i < S; ++i) P[i + J - (S - 1)] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = 0; i <= S; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int... Ts>
__device__ __forceinline__ void s1_all(uint64_t (&P)[S + 1], const uint32_t (&X)[S], const uint4* q, std::integer_sequence<int, Ts...>) {
  uint4 cur = q[(NQ - 1) * 32], nxt;
  (s1_digit<Ts>(P, X, q, cur, nxt), ...);
}

// step 2, digit J (ascending) restricted to the columns [C0, C0 + NC)
template <int C0, int NC, int NJ, int J>
__device__ __forceinline__ void s2_digit(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                         const uint4* a, uint4& cur, uint4& nxt) {
  if constexpr (J % 4 == 0) {
    if constexpr (J > 0) cur = nxt;
    if constexpr (J / 4 + 1 < (NJ + 3) / 4) nxt = a[(J / 4 + 1) * 32];
  }
  const uint32_t d = qword<J % 4>(cur);
  const uint32_t pb = J == 0 ? (lane::LMASK + 1u) - m[0] : lane::LMASK - m[J];
  constexpr int lo = C0 - J > 0 ? C0 - J : 0, hi = C0 + NC - 1 - J;   // i range
#pragma unroll
  for (int i = lo; i <= hi && i < S; ++i) P[i + J - C0] += (uint64_t)X[i] * d;
#pragma unroll
  for (int i = lo; i <= hi && i < S; ++i) P[i + J - C0] += (uint64_t)Q[i] * pb;
#pragma unroll
  for (int i = 0; i < NC; ++i) asm volatile("" : "+v"(P[i]));
  __builtin_amdgcn_sched_barrier(0);
}
template <int C0, int NC, int NJ, int... Js>
__device__ __forceinline__ void s2_all(uint64_t (&P)[NC], const uint32_t (&X)[S], const uint32_t (&Q)[S], const uint32_t (&m)[S],
                                       const uint4* a, std::integer_sequence<int, Js...>) {
  uint4 cur = a[0], nxt;
  (s2_digit<C0, NC, NJ, Js>(P, X, Q, m, a, cur, nxt), ...);
}

template <int W, int L>
__global__ __launch_bounds__(256, W) void k_shoup(Vec v, int K, uint32_t* out) {
  __shared__ uint4 rows[SH_WAVE_Q];
  __shared__ uint32_t stash[L ? 4 * SA * 64 : 1];
  const int lane = threadIdx.x & 63, tig = threadIdx.x & 1, pw = lane >> 1, wv = threadIdx.x >> 6;
  const bool odd = tig != 0;
  uint4* wrows = rows;
  // rows: lane tig fills buffer tig (a_tig, a'_tig) of its pair
  for (int num = 0; num < 2; ++num) {
    const uint32_t* src = (num ? v.ap : v.a) + tig * S;
    uint4* dst = const_cast<uint4*>(sh_num(wrows, tig, num, pw));
    for (int g = 0; g < NQ; ++g) {
      uint32_t w[4];
      for (int j = 0; j < 4; ++j) w[j] = 4 * g + j < S ? src[4 * g + j] : 0u;
      dst[g * 32] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = v.m[j];
  const long long pair = (long long)blockIdx.x * 128 + (threadIdx.x >> 1);
  uint32_t X[S];
#pragma unroll
  for (int j = 0; j < S; ++j) X[j] = v.x[((pair % PAIRS) * 2 + tig) * S + j];
  uint32_t ob = odd ? 1u : 0u;
  asm volatile("" : "+v"(ob));
  for (int k = 0; k < K; ++k) {
    const int buf = k & 1;
    uint32_t Q[S];
    {
      uint64_t P[S + 1];
#pragma unroll
      for (int i = 0; i <= S; ++i) P[i] = 0;
      s1_all(P, X, sh_num(wrows, buf, 1, pw), std::make_integer_sequence<int, S>{});
      uint64_t c = P[0] >> lane::LB;
#pragma unroll
      for (int i = 1; i <= S; ++i) {
        const uint64_t t = P[i] + c;
        Q[i - 1] = lane::limb32(t);
        c = t >> lane::LB;
      }
    }
    const uint4* ar = sh_num(wrows, buf, 0, pw);
    uint32_t lo[SA];
    uint64_t c = 0;
    {
      uint64_t P[SA];
#pragma unroll
      for (int i = 0; i < SA; ++i) P[i] = 0;
      s2_all<0, SA, SA>(P, X, Q, m, ar, std::make_integer_sequence<int, SA>{});
#pragma unroll
      for (int i = 0; i < SA; ++i) {
        const uint32_t qa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[i], 0xA0, 0xF, 0xF, false);
        const uint64_t t = P[i] + c + (uint64_t)qa * ob;
        const uint32_t l = lane::limb32(t);
        c = t >> lane::LB;
        if constexpr (L) stash[(wv * SA + i) * 64 + lane] = l;
        else asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(lo[i]) : "v"(l));
      }
    }
    {
      uint64_t P[SB];
#pragma unroll
      for (int i = 0; i < SB; ++i) P[i] = 0;
      s2_all<SA, SB, S>(P, X, Q, m, ar, std::make_integer_sequence<int, S>{});
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        const uint32_t qa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Q[SA + i], 0xA0, 0xF, 0xF, false);
        const uint64_t t = P[i] + c + (uint64_t)qa * ob;
        X[SA + i] = lane::limb32(t);
        c = t >> lane::LB;
      }
    }
#pragma unroll
    for (int i = 0; i < SA; ++i) {
      if constexpr (L) X[i] = stash[(wv * SA + i) * 64 + lane];
      else asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(X[i]) : "a"(lo[i]));
    }
  }
  if (pair < PAIRS) {
#pragma unroll
    for (int j = 0; j < S; ++j) out[(pair * 2 + tig) * S + j] = X[j];
  }
}

// ---------------------------------------------------------------- Montgomery (k_sgp's pass)
template <int W>
__global__ __launch_bounds__(256, W) void k_mont(Vec v, int K, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t rows[2 * SGP_WAVE_ROWS];   // (one copy per block, as above)
  const int lane = threadIdx.x & 63, tig = threadIdx.x & 1, pw = lane >> 1, wv = threadIdx.x >> 6;
  const bool odd = tig != 0;
  uint32_t* wrows = rows;
  (void)wv;
  {
    uint32_t* r = wrows + tig * SGP_WAVE_ROWS + (pw >> 2) * SGP_GROUP + 4 * (pw & 3);
    for (int w = 0; w < SGP_AW; ++w) r[sgp_word_off<true>(w)] = v.aw[tig * 64 + w];
  }
  __syncthreads();
  uint32_t m[S];
#pragma unroll
  for (int j = 0; j < S; ++j) m[j] = v.m[j];
  const uint32_t mprime = v.mprime;
  const long long pair = (long long)blockIdx.x * 128 + (threadIdx.x >> 1);
  uint32_t x[S];
#pragma unroll
  for (int j = 0; j < S; ++j) x[j] = v.x[((pair % PAIRS) * 2 + tig) * S + j];
  for (int k = 0; k < K; ++k) {
    const uint32_t* my_row = wrows + (k & 1) * SGP_WAVE_ROWS + (pw >> 2) * SGP_GROUP + 4 * (pw & 3);
    uint64_t P[S];
#pragma unroll
    for (int i = 0; i < S; ++i) P[i] = 0;
    sgp_pass<S, SGP_AW, true>(P, x, my_row, m, mprime, odd, std::make_integer_sequence<int, S>{});
    lane::normalize<S>(P, x);
  }
  if (pair < PAIRS) {
#pragma unroll
    for (int j = 0; j < S; ++j) out[(pair * 2 + tig) * S + j] = x[j];
  }
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s vec.bin K out_prefix\n", argv[0]);
    return 2;
  }
  std::vector<uint32_t> h(VEC_WORDS);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(h.data(), 4, VEC_WORDS, f) != (size_t)VEC_WORDS) {
    fprintf(stderr, "bad vector file\n");
    return 2;
  }
  fclose(f);
  const int K = atoi(argv[2]);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  Vec v;
  v.m = d;
  v.mprime = h[S];
  v.a = d + S + 1;
  v.ap = v.a + 2 * S;
  v.aw = v.ap + 2 * S;
  v.x = v.aw + 128;
  uint32_t* dout;
  CK(hipMalloc(&dout, PAIRS * 2 * S * 4));
  const int blocks = cus * 8;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("device %s CUs %d, %d blocks x 128 pairs x K = %d products\n", prop.gcnArchName, cus, blocks, K);
  auto run = [&](const char* name, const char* file, int lanemacs, auto launch) {
    launch(2);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      launch(K);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double prods = (double)blocks * 128 * K;
    printf("%-14s %9.3f ms  %8.4g pair-products/s  %6.2f ns/product/pair-slot  %6.2f T lane-MAC/s\n", name, best,
           prods / (best * 1e-3), best * 1e6 / (prods / (cus * 128.0)), prods * 2.0 * lanemacs / (best * 1e-3) / 1e12);
    std::vector<uint32_t> o(PAIRS * 2 * S);
    CK(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
    char path[512];
    snprintf(path, sizeof path, "%s_%s.bin", argv[3], file);
    FILE* g = fopen(path, "wb");
    if (g) {
      fwrite(o.data(), 4, o.size(), g);
      fclose(g);
    }
  };
  const int mont_macs = 2 * S * S, shoup_macs = S * (S + 1) / 2 + S * (S + 1);
  run("mont w2", "mont", mont_macs, [&](int k) { k_mont<2><<<blocks, 256>>>(v, k, dout); });
  run("mont w1", "mont_w1", mont_macs, [&](int k) { k_mont<1><<<blocks, 256>>>(v, k, dout); });
  run("shoup w1 agpr", "shoup", shoup_macs, [&](int k) { k_shoup<1, 0><<<blocks, 256>>>(v, k, dout); });
  run("shoup w1 lds", "shoup_w1l", shoup_macs, [&](int k) { k_shoup<1, 1><<<blocks, 256>>>(v, k, dout); });
  run("shoup w2 lds", "shoup_w2l", shoup_macs, [&](int k) { k_shoup<2, 1><<<blocks, 256>>>(v, k, dout); });
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
