// FP64-FMA big-number products against the v_mad_u64_u32 ones (VERDICT r2 "weak" 7): the raw
// schoolbook product of two 1024-bit numbers (the reduction half of a Montgomery product has the same shape), per
// lane, many lanes, timed by HIP events.
//
//   int : 37 x 37 limbs of 28 bits, P[i + j] += a_i b_j by v_mad_u64_u32 (1369 instructions per product): the
//         datapath of every kernel in this repository
//   fp64: 20 x 20 limbs of 52 bits held as doubles; each limb product exactly, in 6 instructions:
//           hr = fma(a, b, 2^104)            the rounded high part in the mantissa (ULP 2^52)
//           lo = fma(a, b, 2^104 - hr)       the exact remainder, |lo| <= 2^51
//           lb = lo + 1.5 2^52               lo in the mantissa (ULP 1)
//           H[i + j + 1] += bits(hr), H[i + j] += bits(lb)   (64-bit integer adds; biases removed at the end)
//         2400 instructions per product. (Accumulating the high parts in doubles instead would need an exponent
//         above the sum of 2n terms, i.e. a ULP of 2^58, and the remainders would no longer be exact.)
// The fp64 product is checked against exact integer arithmetic on the host for a few lanes.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dfma_product tools/microbench/dfma_product.hip && /tmp/dfma_product
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <utility>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int IL = 37, FL = 20, REPS = 64;
constexpr double C104 = 20282409603651670423947251286016.0;   // 2^104
constexpr double BIAS = 6755399441055744.0;                    // 1.5 * 2^52

__device__ __forceinline__ uint64_t bits(double d) { return (uint64_t)__double_as_longlong(d); }

template <int I, int... Js>
__device__ __forceinline__ void int_row(uint64_t (&P)[2 * IL], uint32_t (&a)[IL], const uint32_t (&b)[IL],
                                        std::integer_sequence<int, Js...>) {
  ((P[I + Js] += (uint64_t)a[I] * b[Js]), ...);
  asm volatile("" : "+v"(a[I]));   // one row at a time (no cross-row re-association)
}
template <int... Is>
__device__ __forceinline__ void int_product(uint64_t (&P)[2 * IL], uint32_t (&a)[IL], const uint32_t (&b)[IL],
                                            std::integer_sequence<int, Is...>) {
  (int_row<Is>(P, a, b, std::make_integer_sequence<int, IL>{}), ...);
}

__global__ __launch_bounds__(256) void k_int(uint64_t* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[IL], b[IL];
#pragma unroll
  for (int i = 0; i < IL; ++i) {
    a[i] = (t * 2654435761u + i * 40503u + seed) & 0xFFFFFFFu;
    b[i] = (t * 2246822519u + i * 69069u + seed) & 0xFFFFFFFu;
  }
  uint64_t P[2 * IL];
#pragma unroll
  for (int k = 0; k < 2 * IL; ++k) P[k] = 0;
  for (int r = 0; r < REPS; ++r) {
    int_product(P, a, b, std::make_integer_sequence<int, IL>{});
#pragma unroll
    for (int j = 0; j < IL; ++j) b[j] ^= (uint32_t)P[j] & 1u;
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 2 * IL; ++k) s += P[k];
  out[t] = s;
}

__global__ __launch_bounds__(256) void k_fp64(uint64_t* out, uint64_t* cols, uint32_t seed, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  double a[FL], b[FL];
#pragma unroll
  for (int i = 0; i < FL; ++i) {
    const uint64_t va = ((uint64_t)(t * 2654435761u + i * 40503u + seed) << 20) ^ (uint64_t)(t + i * 977u);
    const uint64_t vb = ((uint64_t)(t * 2246822519u + i * 69069u + seed) << 20) ^ (uint64_t)(t * 31u + i);
    a[i] = (double)(va & ((1ull << 52) - 1));
    b[i] = (double)(vb & ((1ull << 52) - 1));
  }
  uint64_t H[2 * FL + 1];   // one 64-bit column per 52-bit position: the biased bits of high and low parts
#pragma unroll
  for (int k = 0; k < 2 * FL + 1; ++k) H[k] = 0;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int i = 0; i < FL; ++i) {
#pragma unroll
      for (int j = 0; j < FL; ++j) {
        const double hr = __builtin_fma(a[i], b[j], C104);
        const double lo = __builtin_fma(a[i], b[j], C104 - hr);
        const double lb = lo + BIAS;
        H[i + j + 1] += bits(hr);
        H[i + j] += bits(lb);
      }
      asm volatile("" : "+v"(a[i]));
    }
    if (r + 1 < reps) {
#pragma unroll
      for (int j = 0; j < FL; ++j) b[j] += (double)(uint32_t)(H[j + 1] & 1u);
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 2 * FL + 1; ++k) s += H[k];
  out[t] = s;
  if (cols && t < 4) {   // the product's columns and its operands (reps = 1), for the host check
    for (int k = 0; k < 2 * FL + 1; ++k) cols[t * 128 + k] = H[k];
    for (int i = 0; i < FL; ++i) {
      cols[t * 128 + 81 + i] = (uint64_t)a[i];
      cols[t * 128 + 101 + i] = (uint64_t)b[i];
    }
  }
}

// exact check on the host: sum_k (H_k - n_k bits(2^104) - m_k bits(1.5 2^52)) 2^(52 k) == A B (the column values
// are < 2^58 in magnitude, so the wrapped 64-bit differences are exact)
static bool check(const uint64_t* c) {
  uint64_t bh, bl;
  const double c104 = C104, bias = BIAS;
  memcpy(&bh, &c104, 8);
  memcpy(&bl, &bias, 8);
  // columns as signed __int128 values of weight 2^(52 k)
  __int128 col[2 * FL + 2] = {0};
  for (int k = 0; k < 2 * FL + 1; ++k) {
    const uint64_t nh = k == 0 ? 0 : (k - 1 < FL ? k : 2 * FL - k);       // terms with i + j + 1 = k
    const uint64_t nl = k < FL ? k + 1 : k < 2 * FL ? 2 * FL - k - 1 : 0;  // terms with i + j = k
    col[k] = (__int128)(int64_t)(c[k] - nh * bh - nl * bl);
  }
  // expected: A B in 52-bit columns
  __int128 want[2 * FL + 2] = {0};
  for (int i = 0; i < FL; ++i)
    for (int j = 0; j < FL; ++j) {
      const unsigned __int128 p = (unsigned __int128)c[81 + i] * c[101 + j];
      want[i + j] += (__int128)(p & ((((unsigned __int128)1) << 52) - 1));
      want[i + j + 1] += (__int128)(p >> 52);
    }
  // normalise both to 52-bit digits and compare
  auto norm = [](__int128* v) {
    __int128 carry = 0;
    for (int k = 0; k < 2 * FL + 2; ++k) {
      const __int128 x = v[k] + carry;
      __int128 d = x % ((__int128)1 << 52);
      if (d < 0) d += (__int128)1 << 52;
      carry = (x - d) / ((__int128)1 << 52);
      v[k] = d;
    }
    return carry;
  };
  const __int128 c1 = norm(col), c2 = norm(want);
  if (c1 != c2) return false;
  for (int k = 0; k < 2 * FL + 2; ++k)
    if (col[k] != want[k]) return false;
  return true;
}

int main() {
  int dev = 0, cus = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 16, threads = 256;
  const size_t lanes = (size_t)blocks * threads;
  uint64_t *out, *cols;
  CHK(hipMalloc(&out, lanes * 8));
  CHK(hipMalloc(&cols, 4 * 128 * 8));
  // exactness of the fp64 product (one repetition)
  hipLaunchKernelGGL(k_fp64, dim3(1), dim3(64), 0, 0, out, cols, 7u, 1);
  CHK(hipDeviceSynchronize());
  std::vector<uint64_t> hc(4 * 128);
  CHK(hipMemcpy(hc.data(), cols, hc.size() * 8, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int l = 0; l < 4; ++l) ok = ok && check(hc.data() + l * 128);
  printf("fp64 product exact vs host integer arithmetic (4 lanes): %s\n", ok ? "yes" : "NO");
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int pass = 0; pass < 2; ++pass) {   // pass 0 warms up
    float ms_i, ms_f;
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_int, dim3(blocks), dim3(threads), 0, 0, out, 1u);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms_i, e0, e1));
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_fp64, dim3(blocks), dim3(threads), 0, 0, out, (uint64_t*)nullptr, 1u, REPS);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms_f, e0, e1));
    if (pass == 1) {
      const double prods = (double)lanes * REPS;
      printf("lanes %zu, %d products of 1024 x 1024 bits per lane\n", lanes, REPS);
      printf("int  (37 x 37 limbs of 28 bits, v_mad_u64_u32): %8.3f ms  %.3e products/s  %.2f T MAC/s\n", ms_i,
             prods / (ms_i * 1e-3), prods * IL * IL / (ms_i * 1e-3) / 1e12);
      printf("fp64 (20 x 20 limbs of 52 bits, 2 FMA + 2 FADD + 2 int adds): %8.3f ms  %.3e products/s  %.2f T limb-products/s\n",
             ms_f, prods / (ms_f * 1e-3), prods * FL * FL / (ms_f * 1e-3) / 1e12);
      printf("fp64 / int time: %.3f\n", ms_f / ms_i);
    }
  }
  CHK(hipFree(out));
  CHK(hipFree(cols));
  return ok ? 0 : 2;
}
