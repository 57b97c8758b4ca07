// ubench_dfa2.hip -- calibrate the v2 DFA step on gfx950: u8 next-state table,
// address = v_perm(state, data, sel) = state*256 + byte (one VALU on the chain),
// event bit shifted into a per-lane mask by one v_alignbit.  Sweeps waves per CU
// (occupancy) and independent chains per lane (ILP).  Reports CU cycles per
// wave-step (64 lane-bytes) at 2.4 GHz and the equivalent byte rate.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_dfa2.hip -o tools/ubench_dfa2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kRows = 48;                 // states (row r at LDS r*256)
constexpr int kTable = kRows * 256;

template <int CHAINS>
__global__ void k(const uint8_t *table, uint32_t *out, int iters, uint32_t seed, uint32_t ascii)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (int i = threadIdx.x; i < kTable; i += blockDim.x) lds[i] = table[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t e[CHAINS], ev[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) { e[c] = (seed * (lane + 1) + c * 5) % kRows; ev[c] = 0; }
  uint32_t data = seed ^ (lane * 0x9E3779B9u) ^ (blockIdx.x << 8);
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int b = 0; b < 4; b++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
          const uint32_t d = ascii ? (((data ^ (c * 0x35353535u)) & 0x3f3f3f3fu) | 0x30303030u) : (data ^ (c * 0x35353535u));
          const uint32_t a = __builtin_amdgcn_perm(e[c], d, 0x0c0c0400u | (uint32_t) b);
          e[c] = *reinterpret_cast<const __attribute__((address_space(3))) uint8_t *>((size_t) a);
          asm("v_alignbit_b32 %0, %1, %0, 1" : "+v"(ev[c]) : "v"(e[c]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      data = data * 1103515245u + 12345u;
    }
#pragma unroll
    for (int c = 0; c < CHAINS; c++) acc += ev[c];
  }
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc += e[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int CHAINS>
void run(const uint8_t *d_table, uint32_t *d_out, int cus, int waves_per_wg, int wg_per_cu, uint32_t ascii = 0)
{
  auto fn = k<CHAINS>;
  size_t lds = 160 * 1024 / wg_per_cu;   // pad LDS so at most wg_per_cu workgroups fit on a CU
  if (lds > 64 * 1024) lds = 64 * 1024;
  CHECK(hipFuncSetAttribute((const void *) fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, waves_per_wg * 64, lds));
  if (per_cu > wg_per_cu) per_cu = wg_per_cu;
  const int grid = cus * per_cu, iters = 1000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves_per_wg * 64), lds, 0, d_table, d_out, 10, 1u, ascii);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves_per_wg * 64), lds, 0, d_table, d_out, iters, 7u, ascii);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double wave_steps = (double) grid * waves_per_wg * iters * 16 * CHAINS;
  const double per_cu_ns = ms * 1e6 / (wave_steps / cus);
  const double gbs = wave_steps * 64 / (ms * 1e-3) / 1e9;
  printf("%s waves/CU %2d (%2d x %d) chains %d: %.2f cyc@2.4GHz per wave-step per CU, %.0f GB/s\n",
         ascii ? "one-row ascii" : "random      ", waves_per_wg * per_cu, waves_per_wg, per_cu, CHAINS, per_cu_ns * 2.4, gbs);
}

int main()
{
  int dev = 0, cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint8_t *h = (uint8_t *) malloc(kTable);
  for (int r = 0; r < kRows; r++)
    for (int c = 0; c < 256; c++) h[r * 256 + c] = (uint8_t) ((r * 7 + c * 13 + (c >> 3)) % kRows);
  uint8_t *d_table;
  uint32_t *d_out;
  CHECK(hipMalloc(&d_table, kTable));
  CHECK(hipMalloc(&d_out, 1 << 24));
  CHECK(hipMemcpy(d_table, h, kTable, hipMemcpyHostToDevice));
  const int cfg[][2] = {{8, 1}, {16, 1}, {12, 2}, {16, 2}};
  for (auto &w : cfg) {
    run<1>(d_table, d_out, cus, w[0], w[1]);
    run<2>(d_table, d_out, cus, w[0], w[1]);
    run<4>(d_table, d_out, cus, w[0], w[1]);
  }
  /* one-row table: every lane stays in row 5, ASCII bytes -> no bank conflicts */
  for (int r = 0; r < kRows; r++)
    for (int c = 0; c < 256; c++) h[r * 256 + c] = 5;
  CHECK(hipMemcpy(d_table, h, kTable, hipMemcpyHostToDevice));
  for (auto &w : cfg) {
    run<1>(d_table, d_out, cus, w[0], w[1], 1);
    run<2>(d_table, d_out, cus, w[0], w[1], 1);
    run<4>(d_table, d_out, cus, w[0], w[1], 1);
  }
  return 0;
}
