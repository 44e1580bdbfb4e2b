// The prototype k_sgs (Shoup rows, tools/microbench/sgs_kernel.hpp) against the library's k_sgp (Montgomery split
// pass, kernels_sgp.hpp) streaming random rows of one table half from HBM -- the measurement for VERDICT r4 item 3
// before the tables and the b-sum kernel are built -- and a small exactness check of k_sgs on real rows.
//   time : ./sgs_stream time <n> <W> <K>      one half, random 28-bit limbs in every row, random digits: k_sgp on a
//                                             table of 512-B factored rows, k_sgs on 640-B Shoup rows with (BS = 1) or
//                                             without (BS = 0) the b sum over the factored table's b halves
//   check: ./sgs_stream check <vec.bin> <out.bin> [2]   rows (k, 0) = (a0, a0', b0), (k, 1) = (a1, a1', b1) of
//                                             tools/microbench/sgp_shoup_vec.py, digit k of element e = (k + e) & 1,
//                                             K = 9, k_sgs BS = 1 (or k_sgs2); the first 64 pairs and b sums written
//                                             for check_sgs
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "sgs_kernel.hpp"

using namespace fpai;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_fill(uint32_t* w, size_t nw, uint32_t seed, uint32_t mask) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed ^ (uint32_t)(i >> 32) * 40503u;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    x *= 3266489917u;
    x ^= x >> 16;
    w[i] = x & mask;
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s time <n> <W> <K> | check <vec.bin> <out.bin>\n", argv[0]);
    return 2;
  }
  constexpr int S = SGP_S;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const bool check = strcmp(argv[1], "check") == 0;
  const long long n = check ? 4096 : atoll(argv[2]);
  const int W = check ? 1 : atoi(argv[3]);
  const int K = check ? 9 : atoi(argv[4]);
  const size_t rows = (size_t)K << W;
  const size_t tab_words = rows * SGS_ROW_Q * 4, ttab_words = rows * FBGP_ROW4 * 4;
  uint32_t *tab, *ttab, *dig, *out, *consts, *bcc;
  uint4* bsum;
  CK(hipMalloc(&tab, tab_words * 4));
  CK(hipMalloc(&ttab, ttab_words * 4));
  CK(hipMalloc(&bsum, (size_t)16 * n * 16));
  CK(hipMalloc(&bcc, (size_t)2 * n * 4));
  CK(hipMalloc(&dig, (size_t)K * n * 4));
  CK(hipMalloc(&out, (size_t)2 * S * n * 4));
  CK(hipMalloc(&consts, 16 * S * 4));
  std::vector<uint32_t> hm(S);
  if (!check) {
    k_fill<<<4096, 256>>>(tab, tab_words, 0x1234567u, lane::LMASK);
    k_fill<<<4096, 256>>>(ttab, ttab_words, 0x7654321u, 0xFFFFFFFFu);
    k_fill<<<4096, 256>>>(dig, (size_t)K * n, 0x89abcdu, (1u << W) - 1u);
    k_fill<<<16, 256>>>(consts, 16 * S, 0x5555u, lane::LMASK);
    CK(hipMemcpy(hm.data(), consts, S * 4, hipMemcpyDeviceToHost));
    hm[S - 1] |= 1u << 27;   // (m > 2^(28 (S - 1)))
    hm[0] |= 1u;
  } else {
    const int VW = S + 1 + 4 * S + 128 + 64 * 2 * S;
    std::vector<uint32_t> v(VW);
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(v.data(), 4, VW, f) != (size_t)VW) {
      fprintf(stderr, "bad vector file\n");
      return 2;
    }
    fclose(f);
    for (int j = 0; j < S; ++j) hm[j] = v[j];
    std::vector<uint32_t> t(tab_words, 0u), tt(ttab_words, 0u);
    for (size_t r = 0; r < rows; ++r) {
      const int d = (int)(r & 1);
      for (int j = 0; j < S; ++j) {
        t[r * SGS_ROW_Q * 4 + j] = v[S + 1 + d * S + j];                      // a_d
        t[r * SGS_ROW_Q * 4 + SGS_NQ * 4 + j] = v[S + 1 + 2 * S + d * S + j];  // a_d'
      }
      for (int j = 0; j < 64; ++j) tt[r * FBGP_ROW4 * 4 + 64 + j] = 0x9E3779B9u * (uint32_t)(2 * j + d + 1) ^ 0xA5A5A5A5u * (uint32_t)d;
    }
    CK(hipMemcpy(tab, t.data(), tab_words * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ttab, tt.data(), ttab_words * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> dg((size_t)K * n);
    for (int k = 0; k < K; ++k)
      for (long long e = 0; e < n; ++e) dg[(size_t)k * n + e] = (uint32_t)((k + e) & 1);
    CK(hipMemcpy(dig, dg.data(), dg.size() * 4, hipMemcpyHostToDevice));
  }
  CK(hipMemcpy(consts, hm.data(), S * 4, hipMemcpyHostToDevice));   // consts[0 .. S): m
  SgsHalf sh{reinterpret_cast<const uint4*>(tab), consts, reinterpret_cast<const uint4*>(ttab) + FBGP_PW / 4, FBGP_ROW4};
  SgsHalf* dsh;
  CK(hipMalloc(&dsh, sizeof sh));
  CK(hipMemcpy(dsh, &sh, sizeof sh, hipMemcpyHostToDevice));
  SgsParams sp{};
  sp.halves = dsh;
  sp.n = n;
  sp.K = K;
  sp.W = W;
  sp.digits = dig;
  sp.out = out;
  sp.bsum = bsum;
  sp.bcc = bcc;
  const int grid = (int)std::min<long long>((n + 127) / 128, (long long)cus * 2);
  if (check) {
    if (argc > 4 && atoi(argv[4]) == 2) k_sgs2<S><<<dim3(grid, 1), LANE_BLOCK>>>(sp);
    else k_sgs<S, 1><<<dim3(grid, 1), LANE_BLOCK>>>(sp);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> o((size_t)2 * S * n), r(64 * 2 * S), bs((size_t)64 * n), cc((size_t)2 * n), rb(64 * 66);
    CK(hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(bs.data(), bsum, bs.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(cc.data(), bcc, cc.size() * 4, hipMemcpyDeviceToHost));
    for (int e = 0; e < 64; ++e) {
      for (int c = 0; c < 2; ++c)
        for (int i = 0; i < S; ++i) r[(e * 2 + c) * S + i] = o[((size_t)c * S + i) * n + e];
      for (int w = 0; w < 64; ++w) rb[e * 66 + w] = bs[((size_t)(w / 4) * n + e) * 4 + w % 4];
      rb[e * 66 + 64] = cc[e];
      rb[e * 66 + 65] = cc[n + e];
    }
    FILE* g = fopen(argv[3], "wb");
    if (!g) return 2;
    fwrite(r.data(), 4, r.size(), g);
    fwrite(rb.data(), 4, rb.size(), g);
    fclose(g);
    printf("k_sgs check run done (K = %d, n = %lld)\n", K, n);
    return 0;
  }
  // k_sgp on the same allocation (512-B rows), constants from the random words
  float* x;
  int32_t* ex;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&ex, n * 4));
  CK(hipMemset(x, 0, n * 4));
  SgpHalf gh{};
  gh.table = reinterpret_cast<const uint4*>(ttab);
  gh.p = consts;
  gh.ca = consts + S;
  gh.cb = consts + 2 * S;
  gh.nmc = consts + 3 * S;
  gh.pbig = consts + 7 * S;
  gh.mprime = 0x0123457u;
  SgpHalf* dgh;
  CK(hipMalloc(&dgh, sizeof gh));
  CK(hipMemcpy(dgh, &gh, sizeof gh, hipMemcpyHostToDevice));
  SgpParams gp{};
  gp.halves = dgh;
  gp.n = n;
  gp.K = K;
  gp.W = W;
  gp.digits = dig;
  gp.out = out;
  gp.x = x;
  gp.dtype = 0;
  gp.exp = ex;
  gp.status = nullptr;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("device %s CUs %d, n %lld, W %d, K %d, grid %d x %d\n", prop.gcnArchName, cus, n, W, K, grid, LANE_BLOCK);
  auto timeit = [&](auto launch) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  auto sgp = [&]() { k_sgp<S><<<dim3(grid, 1), LANE_BLOCK>>>(gp); };
  auto sgs0 = [&]() { k_sgs<S, 0><<<dim3(grid, 1), LANE_BLOCK>>>(sp); };
  auto sgs1 = [&]() { k_sgs<S, 1><<<dim3(grid, 1), LANE_BLOCK>>>(sp); };
  auto sgs2 = [&]() { k_sgs2<S><<<dim3(grid, 1), LANE_BLOCK>>>(sp); };
  timeit(sgp);
  timeit(sgs0);
  timeit(sgs1);
  timeit(sgs2);
  for (int r = 0; r < 3; ++r) {
    const float a = timeit(sgp), b = timeit(sgs0), c = timeit(sgs1), d = timeit(sgs2);
    printf("round %d: k_sgp %.3f ms (K %d products, b sum included)  k_sgs %.3f ms without the b sum (%.3f)  %.3f ms with "
           "it in global memory (%.3f)  k_sgs2 %.3f ms with it in registers (%.3f)\n",
           r, a, K, b, b / a, c, c / a, d, d / a);
    fflush(stdout);
  }
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
