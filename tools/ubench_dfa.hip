// ubench_dfa.hip -- calibrate the DFA step primitive on gfx950.
//
// One "step" per chain: e = LDS[(e & 0xffff) + 4*byte] (dependent table read),
// optionally one ds_write_b16 capture per step; CHAINS independent chains per
// lane (ILP).  Reports CU cycles per wave-step (64 lane-bytes).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_dfa.hip -o tools/ubench_dfa
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define LDS __attribute__((address_space(3)))
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kRows = 32, kRowBytes = 1040, kTable = kRows * kRowBytes;

template <int WAVES, int CHAINS, int CAP, int RING>
__global__ __launch_bounds__(WAVES * 64) void k(const uint32_t *table, uint32_t *out, int iters, uint32_t seed)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (int i = threadIdx.x; i < kTable / 4; i += WAVES * 64) ((uint32_t *) lds)[i] = table[i];
  __syncthreads();
  const uint32_t base = (uint32_t) (size_t) (LDS uint8_t *) lds;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t ring = base + kTable + wave * RING * 64 + 2 * lane;
  uint32_t e[CHAINS], cap[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) { e[c] = (seed * (lane + 1) + c * 5) % kRows * kRowBytes; cap[c] = c * 16; }
  uint32_t pos = 0;
  uint32_t data = seed ^ (lane * 0x9E3779B9u) ^ (blockIdx.x << 8);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < 16; s++) {
      uint32_t b = (data >> ((s & 3) * 8)) & 0xff;
#pragma unroll
      for (int c = 0; c < CHAINS; c++) {
        e[c] = *(const LDS uint32_t *) (size_t) (base + (e[c] & 0xffff) + ((b ^ (c * 0x35)) & 0xff) * 4);
        if (CAP == 1) {
          cap[c] += e[c] >> 24;
          *(LDS uint16_t *) (size_t) (ring + (((cap[c] + (e[c] >> 16)) & (RING - 2)) << 6)) = (uint16_t) pos;
        } else if (CAP == 2) {
          if (((e[c] >> 16) & 0xe) == 0) {
            cap[c] += 2;
            *(LDS uint16_t *) (size_t) (ring + ((cap[c] & (RING - 2)) << 6)) = (uint16_t) pos;
          }
        } else if (CAP == 3) {
          cap[c] |= ((e[c] >> 17) & 1) << s;
        }
      }
      pos++;
      if ((s & 3) == 3) data = data * 1103515245u + 12345u;
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc += e[c] + cap[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int WAVES, int CHAINS, int CAP, int RING = 64>
void run(const uint32_t *d_table, uint32_t *d_out, int cus)
{
  auto fn = k<WAVES, CHAINS, CAP, RING>;
  const size_t lds = kTable + WAVES * RING * 64;
  CHECK(hipFuncSetAttribute((const void *) fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, WAVES * 64, lds));
  const int grid = cus * per_cu, iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(WAVES * 64), lds, 0, d_table, d_out, 10, 1u);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(WAVES * 64), lds, 0, d_table, d_out, iters, 7u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double wave_steps = (double) grid * WAVES * iters * 16 * CHAINS;
  const double per_cu_ns = ms * 1e6 / (wave_steps / cus);
  const double gbs = wave_steps * 64 / (ms * 1e-3) / 1e9;   // 64 B per wave-step
  printf("waves/WG %2d x %d WG/CU  chains %d cap %d ring %3d: %.2f cycles@2.4GHz per wave-step per CU, equiv %.0f GB/s\n",
         WAVES, per_cu, CHAINS, CAP, RING, per_cu_ns * 2.4, gbs);
}

// Conflict-free variant: byte -> class through a 256-B class table (ASCII hits
// distinct banks), then (state, class) -> entry in a table replicated 32 times
// so lane l always reads bank l % 32; capture ring laid out one dword column per
// lane (bank = lane % 32).
constexpr int kCls = 16, kStates = 32, kRep = 32;
constexpr int kRepTable = kStates * kCls * kRep * 4;   // 64 KiB
template <int WAVES, int CHAINS, int CAP>
__global__ __launch_bounds__(WAVES * 64) void kcf(const uint32_t *table, uint32_t *out, int iters, uint32_t seed)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (int i = threadIdx.x; i < kRepTable / 4; i += WAVES * 64) {
    const int ent = i / kRep;  // (state, class)
    const uint32_t nxt = (uint32_t) ((ent * 7 + 3) % kStates);
    ((uint32_t *) lds)[i] = (nxt << 11) | ((ent & 7) * 2u << 16) | ((ent % 13 == 0) ? 8u << 24 : 0u);
  }
  for (int i = threadIdx.x; i < 256; i += WAVES * 64) lds[kRepTable + i] = (uint8_t) (((i * 5) % kCls) << 3);  // class << 3 (x16 B... scaled below)
  __syncthreads();
  const uint32_t base = (uint32_t) (size_t) (LDS uint8_t *) lds;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t lane4 = base + (lane & 31) * 4;
  const uint32_t ring = base + kRepTable + 256 + wave * 4096 + 4 * lane;
  uint32_t e[CHAINS], cap[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) { e[c] = ((seed * (lane + 1) + c * 5) % kStates) << 11; cap[c] = c * 16; }
  uint32_t pos = 0;
  uint32_t data = seed ^ (lane * 0x9E3779B9u) ^ (blockIdx.x << 8);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < 16; s++) {
      uint32_t b = (data >> ((s & 3) * 8)) & 0xff;
      const uint32_t cls = *(const LDS uint8_t *) (size_t) (base + kRepTable + b);   // class * 8
#pragma unroll
      for (int c = 0; c < CHAINS; c++) {
        const uint32_t addr = (e[c] & 0xf800u) | (cls << 4) | lane4;   // state*2048 + class*128 + lane*4
        e[c] = *(const LDS uint32_t *) (size_t) addr;
        if (CAP == 1) {
          cap[c] += e[c] >> 24;
          const uint32_t rb = (cap[c] + (e[c] >> 16)) & 62;
          *(LDS uint16_t *) (size_t) (ring + ((rb & 60) << 6) + (rb & 2)) = (uint16_t) pos;
        } else if (CAP == 3) {
          cap[c] |= ((e[c] >> 17) & 1) << s;
        }
      }
      pos++;
      if ((s & 3) == 3) data = data * 1103515245u + 12345u;
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) acc += e[c] + cap[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int WAVES, int CHAINS, int CAP>
void runcf(uint32_t *d_out, int cus)
{
  auto fn = kcf<WAVES, CHAINS, CAP>;
  const size_t lds = kRepTable + 256 + WAVES * 4096;
  CHECK(hipFuncSetAttribute((const void *) fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, WAVES * 64, lds));
  const int grid = cus * per_cu, iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(WAVES * 64), lds, 0, (const uint32_t *) nullptr, d_out, 10, 1u);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(WAVES * 64), lds, 0, (const uint32_t *) nullptr, d_out, iters, 7u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double wave_steps = (double) grid * WAVES * iters * 16 * CHAINS;
  const double per_cu_ns = ms * 1e6 / (wave_steps / cus);
  const double gbs = wave_steps * 64 / (ms * 1e-3) / 1e9;
  printf("CONFLICT-FREE waves/WG %2d x %d WG/CU  chains %d cap %d: %.2f cycles@2.4GHz per wave-step per CU, equiv %.0f GB/s\n",
         WAVES, per_cu, CHAINS, CAP, per_cu_ns * 2.4, gbs);
}

int main()
{
  int dev = 0, cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t *h = (uint32_t *) malloc(kTable);
  for (int r = 0; r < kRows; r++)
    for (int c = 0; c < kRowBytes / 4; c++) {
      uint32_t nxt = (uint32_t) ((r * 7 + c * 13 + (c >> 3)) % kRows);
      h[r * kRowBytes / 4 + c] = nxt * kRowBytes | ((c & 7) * 2u << 16) | ((c % 61 == 0) ? 8u << 24 : 0u);
    }
  uint32_t *d_table, *d_out;
  CHECK(hipMalloc(&d_table, kTable));
  CHECK(hipMalloc(&d_out, 1 << 24));
  CHECK(hipMemcpy(d_table, h, kTable, hipMemcpyHostToDevice));
  run<4, 1, 0>(d_table, d_out, cus);
  run<8, 1, 0>(d_table, d_out, cus);
  run<16, 1, 0>(d_table, d_out, cus);
  run<16, 2, 0>(d_table, d_out, cus);
  run<16, 4, 0>(d_table, d_out, cus);
  run<8, 2, 0>(d_table, d_out, cus);
  run<8, 4, 0>(d_table, d_out, cus);
  run<16, 1, 1>(d_table, d_out, cus);
  run<16, 2, 1>(d_table, d_out, cus);
  run<16, 4, 1, 32>(d_table, d_out, cus);
  run<8, 2, 1>(d_table, d_out, cus);
  run<8, 4, 1>(d_table, d_out, cus);
  run<16, 1, 2>(d_table, d_out, cus);
  run<16, 1, 3>(d_table, d_out, cus);
  run<16, 2, 3>(d_table, d_out, cus);
  runcf<16, 1, 3>(d_out, cus);
  runcf<16, 2, 3>(d_out, cus);
  runcf<16, 1, 0>(d_out, cus);
  runcf<16, 1, 1>(d_out, cus);
  runcf<16, 2, 1>(d_out, cus);
  runcf<8, 1, 1>(d_out, cus);
  runcf<8, 2, 1>(d_out, cus);
  return 0;
}
