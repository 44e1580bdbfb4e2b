// Step-1 microbenchmark: Montgomery products per second on gfx950 for the engine variants the
// Paillier kernels can be built from (decides the CRT-half / decrypt datapath):
//   group<TPI>   : lane-group CIOS (bn_group.hpp), L = 37 limbs/lane, S = 37*TPI, B via LDS
//   lane<S> sqr  : one number per lane (bn_lane.hpp), triangle squaring
//   lane<S> mul  : one number per lane, general product (b in VGPRs)
// Each thread group runs ITERS dependent products; reported: products/s for the whole chip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ibond-flex_amd/csrc montmul_variants.hip -o mmv
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "bn_group.hpp"
#include "bn_lane.hpp"

using namespace fpai;

template <int TPI>
__global__ __launch_bounds__(256, 2) void k_group(const uint32_t* N, uint32_t* out, int iters, uint32_t mprime) {
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63, tig = threadIdx.x % TPI, gib = threadIdx.x / TPI;
  uint32_t* slot = smem + gib * TPI * L;
  uint32_t m[L], a[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    m[i] = N[tig * L + i];
    a[i] = (N[tig * L + i] ^ (threadIdx.x * 2654435761u)) & LMASK;
  }
  if (tig == TPI - 1) a[L - 1] = 0;
  for (int it = 0; it < iters; ++it) {
    write_limbs_lds<TPI>(slot, a, tig);
    montmul<TPI>(a, a, slot, TPI, m, mprime, lane, tig);
  }
#pragma unroll
  for (int i = 0; i < L; ++i) out[(blockIdx.x * 256 + threadIdx.x) * L + i] = a[i];
}

template <int S, bool SQR, int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_lane(const uint32_t* N, uint32_t* out, int iters, uint32_t mprime) {
  uint32_t m[S], a[S], b[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    m[i] = N[i];
    a[i] = (N[i] ^ (threadIdx.x * 2654435761u + i)) & lane::LMASK;
    b[i] = (N[i] ^ (threadIdx.x * 40503u + blockIdx.x + i)) & lane::LMASK;
  }
  a[S - 1] = 0;
  b[S - 1] = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (SQR) lane::mont_sqr<S>(a, m, mprime);
    else lane::mont_mul<S>(a, b, m, mprime);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) out[(blockIdx.x * 256 + threadIdx.x) * S + i] = a[i];
}

static uint32_t mprime_of(uint32_t m0) {
  uint32_t x = 1;
  for (int i = 0; i < 6; ++i) x *= 2u - m0 * x;
  return (0u - x) & lane::LMASK;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d\n", prop.gcnArchName, cus);
  uint32_t hN[8 * L];
  for (int i = 0; i < 8 * L; ++i) hN[i] = (0x9E3779B9u * (i + 1)) & lane::LMASK;
  hN[0] |= 1;
  uint32_t *dN, *dout;
  (void)hipMalloc(&dN, sizeof(hN));
  (void)hipMemcpy(dN, hN, sizeof(hN), hipMemcpyHostToDevice);
  const int blocks = cus * 8;
  (void)hipMalloc(&dout, (size_t)blocks * 256 * 160 * 4);
  const uint32_t mp = mprime_of(hN[0]);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char* name, int S, int elems_per_block, auto launch) {
    const int iters = 400;
    launch(iters / 4);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0);
      launch(iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double prods = (double)blocks * elems_per_block * iters;
    const double rate = prods / (best * 1e-3);
    const double macs = 2.0 * S * S;   // schoolbook CIOS count, for comparison across variants
    printf("%-22s S=%3d  %9.3f ms  %10.4g prod/s  %7.2f T(2S^2-MAC)/s\n", name, S, best, rate, rate * macs / 1e12);
  };
  const size_t lds2 = 256 / 2 * 2 * L * 4, lds4 = 256 / 4 * 4 * L * 4;
  run("group<2>", 2 * L, 128, [&](int it) { k_group<2><<<blocks, 256, lds2>>>(dN, dout, it, mp); });
  run("group<4>", 4 * L, 64, [&](int it) { k_group<4><<<blocks, 256, lds4>>>(dN, dout, it, mp); });
  run("lane<37> sqr w2", 37, 256, [&](int it) { k_lane<37, true, 2><<<blocks, 256>>>(dN, dout, it, mp); });
  run("lane<37> mul w2", 37, 256, [&](int it) { k_lane<37, false, 2><<<blocks, 256>>>(dN, dout, it, mp); });
  run("lane<74> sqr w1", 74, 256, [&](int it) { k_lane<74, true, 1><<<blocks, 256>>>(dN, dout, it, mp); });
  run("lane<74> sqr w2", 74, 256, [&](int it) { k_lane<74, true, 2><<<blocks, 256>>>(dN, dout, it, mp); });
  run("lane<74> mul w1", 74, 256, [&](int it) { k_lane<74, false, 1><<<blocks, 256>>>(dN, dout, it, mp); });
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
