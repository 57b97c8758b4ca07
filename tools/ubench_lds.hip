// ubench_lds.hip -- LDS read throughput on gfx950 by access width and address
// pattern (diagnostic for the DFA table format).  Each lane issues independent
// reads (no dependent chain) from addresses in [0, 48 KiB); reports CU cycles per
// wave-instruction at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define LDSP(T, a) (*reinterpret_cast<const __attribute__((address_space(3))) T *>((size_t) (a)))

// PAT 0: random per lane (row r random, byte random)   PAT 1: same row, random byte
// PAT 2: all lanes one address (broadcast)             PAT 3: lane-linear (a = lane*W)
// PAT 5: ds_bpermute_b32 from a random lane (a table held one entry per lane)
template <int W, int PAT>
__global__ void k(uint32_t *out, int iters, uint32_t seed)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (int i = threadIdx.x; i < 48 * 1024 / 4; i += blockDim.x) ((uint32_t *) lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = seed ^ (lane * 0x9E3779B9u) ^ (blockIdx.x << 8) ^ (threadIdx.x << 20);
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      x = x * 1103515245u + 12345u;
      uint32_t r;
      if (PAT == 0) r = ((x >> 8) % 48u) * 256u + (x >> 24);
      else if (PAT == 1) r = 7u * 256u + (x >> 24);
      else if (PAT == 4) r = 7u * 256u + 0x30u + ((x >> 24) & 0x3fu);                            /* one row, ASCII: no conflicts */
      else if (PAT == 2) r = 7u * 256u + (((uint32_t) it * 8u + (uint32_t) j) & 63u) * 4u;   /* all lanes one address */
      else r = (lane * W + ((uint32_t) it * 8u + (uint32_t) j) * 256u) & 0xbfffu;            /* lane-linear, conflict-free */
      a[j] = r & ~(uint32_t) (W - 1);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (PAT == 5) { acc += (uint32_t) __builtin_amdgcn_ds_bpermute((int) (a[j] & 252u), (int) (acc ^ lane)); continue; }
      if (W == 1) acc += LDSP(uint8_t, a[j]);
      else if (W == 2) acc += LDSP(uint16_t, a[j]);
      else if (W == 4) acc += LDSP(uint32_t, a[j]);
      else { uint64_t v = LDSP(uint64_t, a[j]); acc += (uint32_t) v ^ (uint32_t) (v >> 32); }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int W, int PAT>
void run(uint32_t *d_out, int cus, const char *name)
{
  auto fn = k<W, PAT>;
  const size_t lds = 64 * 1024;
  CHECK(hipFuncSetAttribute((const void *) fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
  const int waves = 16, per_cu = 2, grid = cus * per_cu, iters = 2000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves * 64), lds, 0, d_out, 10, 1u);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves * 64), lds, 0, d_out, iters, 7u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double instrs = (double) grid * waves * iters * 8;
  printf("%-28s width %d: %.2f cyc@2.4GHz per wave-instruction per CU\n", name, W, ms * 1e6 / (instrs / cus) * 2.4);
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *d_out;
  CHECK(hipMalloc(&d_out, 1 << 24));
  run<1, 0>(d_out, cus, "random row, random byte");
  run<1, 1>(d_out, cus, "one row, random byte");
  run<1, 2>(d_out, cus, "broadcast");
  run<1, 3>(d_out, cus, "lane-linear");
  run<2, 0>(d_out, cus, "random row, random byte");
  run<2, 1>(d_out, cus, "one row, random byte");
  run<2, 2>(d_out, cus, "broadcast");
  run<4, 0>(d_out, cus, "random row, random byte");
  run<4, 1>(d_out, cus, "one row, random byte");
  run<4, 2>(d_out, cus, "broadcast");
  run<4, 3>(d_out, cus, "lane-linear");
  run<8, 0>(d_out, cus, "random row, random byte");
  run<8, 3>(d_out, cus, "lane-linear");
  run<1, 4>(d_out, cus, "one row, ascii byte");
  run<4, 5>(d_out, cus, "ds_bpermute random lane");
  run<4, 4>(d_out, cus, "one row, ascii byte");
  return 0;
}
