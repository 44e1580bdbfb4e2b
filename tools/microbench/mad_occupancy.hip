// v_mad_u64_u32 issue rate against waves per SIMD: does a product loop at 2 waves/SIMD (k_fbp, k_dec_pow_pair)
// reach the 8-wave rate int_throughput.hip measures? 256-thread blocks (one wave per SIMD), cus * w blocks
// resident at once for w waves per SIMD; CH independent accumulators per lane, multiplier in a VGPR (V) or an
// SGPR (S, as the modulus limbs of the pair kernels).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 8192

template <int CH, bool SOP>
__global__ __launch_bounds__(256) void k_mad(uint64_t* out, uint32_t s) {
  uint64_t a[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) a[i] = threadIdx.x + i;
  uint32_t x = s + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (SOP) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(x), "s"(s) : "vcc");
      else asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(s) : "vcc");
    }
  }
  uint64_t r = 0;
  for (int i = 0; i < CH; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int CH, bool SOP>
static void run(const char* name, int cus, void* buf, hipEvent_t e0, hipEvent_t e1) {
  for (int w : {1, 2, 3, 4, 8}) {
    const int blocks = cus * w;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0);
      k_mad<CH, SOP><<<blocks, 256>>>((uint64_t*)buf, 12345u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double ops = (double)blocks * 256 * ITERS * CH;
    printf("%-10s CH=%2d waves/SIMD=%d  %8.3f ms  %7.3f T MAC/s\n", name, CH, w, best, ops / (best * 1e-3) / 1e12);
  }
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d\n", prop.gcnArchName, cus);
  void* buf;
  hipMalloc(&buf, (size_t)cus * 8 * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  run<16, false>("vgpr", cus, buf, e0, e1);
  run<32, false>("vgpr", cus, buf, e0, e1);
  run<32, true>("sgpr", cus, buf, e0, e1);
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return 0;
}
