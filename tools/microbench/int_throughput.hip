// Step-0 microbenchmark: per-CU throughput on gfx950 of the
// instructions a big-integer Montgomery product can be built from. Each kernel runs
// 16 independent chains per lane so latency is hidden; rates are reported as lane-ops
// per second and normalised to v_fma_f32 (known full rate: 128 lane-ops/clk/CU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 16384
#define CHAINS 16

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

__global__ void k_fma_f32(float* out, float s) {
  float a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(s), "v"(s));
    REP16(OP)
#undef OP
  }
  float r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma_f64(double* out, double s) {
  double a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(s), "v"(s));
    REP16(OP)
#undef OP
  }
  double r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u64(uint64_t* out, uint32_t s) {
  uint64_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  uint32_t x = s + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(s) : "vcc");
    REP16(OP)
#undef OP
  }
  uint64_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_i64(uint64_t* out, uint32_t s) {
  uint64_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  uint32_t x = s + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(x), "v"(s) : "vcc");
    REP16(OP)
#undef OP
  }
  uint64_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi_u32(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_lo_u32(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad_u24(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_mad_u32_u24 %0, %1, %1, %0" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_lshl_add_u64(uint64_t* out, uint64_t s) {
  uint64_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint64_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_addc_u32(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(s) : "vcc");
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_add3_u32(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_dpp_shr(uint32_t* out, uint32_t s) {
  uint32_t a[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_add_u32_dpp %0, %0, %1 row_shr:1 bound_ctrl:0" : "+v"(a[i]) : "v"(s));
    REP16(OP)
#undef OP
  }
  uint32_t r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_cvt_f64_u32(double* out, uint32_t s) {
  double a[CHAINS];
  uint32_t x = s + threadIdx.x;
#pragma unroll
  for (int i = 0; i < CHAINS; ++i) a[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#define OP(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[i]) : "v"(x + i));
    REP16(OP)
#undef OP
  }
  double r = 0; for (int i = 0; i < CHAINS; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*launcher)(void*, int, int);

int main() {
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  const int threads = 256;
  const int blocks = cus * 8;  // 32 waves/CU
  void* buf; hipMalloc(&buf, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct T { const char* name; int which; } tests[] = {
    {"v_fma_f32", 0}, {"v_fma_f64", 1}, {"v_mad_u64_u32", 2}, {"v_mul_hi_u32", 3},
    {"v_mul_lo_u32", 4}, {"v_mad_u32_u24", 5}, {"v_lshl_add_u64", 6}, {"v_addc_co_u32", 7},
    {"v_add3_u32", 8}, {"v_add_u32_dpp row_shr", 9}, {"v_cvt_f64_u32", 10}, {"v_mad_i64_i32", 11}};
  double fma32_rate = 0;
  for (auto& t : tests) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      switch (t.which) {
        case 0: k_fma_f32<<<blocks, threads>>>((float*)buf, 1.0001f); break;
        case 1: k_fma_f64<<<blocks, threads>>>((double*)buf, 1.0001); break;
        case 2: k_mad_u64<<<blocks, threads>>>((uint64_t*)buf, 12345u); break;
        case 3: k_mul_hi_u32<<<blocks, threads>>>((uint32_t*)buf, 0x9e3779b9u); break;
        case 4: k_mul_lo_u32<<<blocks, threads>>>((uint32_t*)buf, 0x9e3779b9u); break;
        case 5: k_mad_u24<<<blocks, threads>>>((uint32_t*)buf, 12345u); break;
        case 6: k_lshl_add_u64<<<blocks, threads>>>((uint64_t*)buf, 12345ull); break;
        case 7: k_addc_u32<<<blocks, threads>>>((uint32_t*)buf, 12345u); break;
        case 8: k_add3_u32<<<blocks, threads>>>((uint32_t*)buf, 12345u); break;
        case 9: k_dpp_shr<<<blocks, threads>>>((uint32_t*)buf, 12345u); break;
        case 10: k_cvt_f64_u32<<<blocks, threads>>>((double*)buf, 12345u); break;
        case 11: k_mad_i64<<<blocks, threads>>>((uint64_t*)buf, 12345u); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    double ops = (double)blocks * threads * ITERS * CHAINS;
    double rate = ops / (best * 1e-3);
    if (t.which == 0) fma32_rate = rate;
    printf("%-24s %8.3f ms  %10.3f Tlane-op/s  %6.1f lane-op/clk/CU (rel fma_f32=128)\n", t.name, best,
           rate / 1e12, 128.0 * rate / fma32_rate);
  }
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return 0;
}
