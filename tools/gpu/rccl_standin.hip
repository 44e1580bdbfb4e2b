// A stand-in for the N = 8 all-gather's copy kernels on ONE MI355X (bench.py extra.allgather_contention_1gpu; VERDICT r5
// next #2): RCCL moves each step's 7 received shards with copy kernels that hold their workgroups (one per channel) for
// as long as xGMI needs, not for as long as HBM would. This kernel copies `bytes` from src to dst with `blocks`
// workgroups of 256 lanes that stay resident for `duration_ns`: block b copies its slice in 64-KiB pieces and, after
// piece k, waits on the 100-MHz wall clock until k + 1 pieces' share of the duration has passed (s_sleep in the loop,
// so the waves hold their CU slots without issuing). Bench-only tooling: not part of libflexpai.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__global__ __launch_bounds__(256) void k_throttled_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        unsigned long long quads, unsigned long long ticks) {
  const unsigned long long per = (quads + gridDim.x - 1) / gridDim.x;
  const unsigned long long lo = per * blockIdx.x;
  const unsigned long long hi = lo + per < quads ? lo + per : quads;
  if (lo >= hi) return;
  constexpr unsigned long long PIECE = 4096;   // quads: 64 KiB per piece
  const unsigned long long pieces = (hi - lo + PIECE - 1) / PIECE;
  const unsigned long long t0 = wall_clock64();
  for (unsigned long long k = 0; k < pieces; ++k) {
    const unsigned long long a = lo + k * PIECE, b = a + PIECE < hi ? a + PIECE : hi;
    for (unsigned long long i = a + threadIdx.x; i < b; i += blockDim.x) dst[i] = src[i];
    const unsigned long long due = t0 + ticks * (k + 1) / pieces;
    while (wall_clock64() < due) __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace

// 0 on success. duration_ns = 0: copy at full speed. Wall clock: 100 MHz on gfx950 (10 ns per tick).
extern "C" int standin_throttled_copy(const void* src, void* dst, unsigned long long bytes, int blocks,
                                      unsigned long long duration_ns, void* stream) {
  if (!src || !dst || blocks < 1 || bytes % 16) return 1;
  hipLaunchKernelGGL(k_throttled_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, (uint4*)dst,
                     bytes / 16, duration_ns / 10);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
