// ubench_lds2.hip -- LDS ds_read_u8 cost vs address pattern on gfx950: random byte
// among N distinct dwords of one row, a random permutation of 64 dwords, and
// lane-linear.  Independent reads, 16 waves per CU; cycles per wave-instruction
// per CU at 2.4 GHz.   hipcc --offload-arch=gfx950 -O3 tools/ubench_lds2.hip -o tools/ubench_lds2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define LDSP(T, a) (*reinterpret_cast<const __attribute__((address_space(3))) T *>((size_t) (a)))

// MODE 0: random byte in N distinct dwords (dword = rand % N, spread over the row by stride S)
// MODE 1: lane l reads dword perm(l) (a fixed xor-permutation), byte 0
// MODE 2: lane l reads dword l (lane-linear)
// MODE 3: lane l reads dword (l * 17) & 63 (a stride permutation)
template <int MODE>
__global__ void k(uint32_t *out, int iters, uint32_t n, uint32_t stride)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  for (int i = threadIdx.x; i < 16 * 1024 / 4; i += blockDim.x) ((uint32_t *) lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = (lane * 0x9E3779B9u) ^ (blockIdx.x << 8) ^ (threadIdx.x << 20);
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      x = x * 1103515245u + 12345u;
      uint32_t r;
      if (MODE == 0) r = 4u * ((((x >> 8) & (n - 1u)) * stride) & 63u) + ((x >> 24) & 3u);
      else if (MODE == 1) r = 4u * (lane ^ (((uint32_t) it * 8u + (uint32_t) j) & 63u));
      else if (MODE == 2) r = 4u * lane + 256u * ((x >> 20) & 7u);
      else r = 4u * ((lane * 17u + (uint32_t) it + (uint32_t) j) & 63u);
      a[j] = 1024u + r + (MODE == 0 ? 256u * ((x >> 4) & 7u) * 0u : 0u);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) acc += LDSP(uint8_t, a[j]);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
void run(uint32_t *d_out, int cus, uint32_t n, uint32_t stride, const char *name)
{
  auto fn = k<MODE>;
  const int waves = 16, grid = cus, iters = 4000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves * 64), 16 * 1024, 0, d_out, 10, n, stride);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(waves * 64), 16 * 1024, 0, d_out, iters, n, stride);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double instrs = (double) grid * waves * iters * 8;
  printf("%-40s n=%2u stride=%2u: %.2f cyc@2.4GHz per wave-instruction per CU\n", name, n, stride, ms * 1e6 / (instrs / cus) * 2.4);
}

int main()
{
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *d_out;
  CHECK(hipMalloc(&d_out, 1 << 24));
  for (uint32_t n : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) run<0>(d_out, cus, n, 1, "random byte in n consecutive dwords");
  for (uint32_t n : {8u, 16u, 32u}) run<0>(d_out, cus, n, 2, "random byte in n dwords, stride 2");
  run<1>(d_out, cus, 64, 1, "xor permutation of 64 dwords");
  run<2>(d_out, cus, 64, 1, "lane-linear");
  run<3>(d_out, cus, 64, 17, "stride-17 permutation");
  return 0;
}
