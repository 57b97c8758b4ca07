// ubench_stream.hip -- HBM read ceilings of the access patterns a lane-per-request
// parser can use on gfx950 (MI355X), over a 2 GiB buffer (>> 256 MiB MALL):
//   coal    wave reads 1 KiB contiguous per global_load_dwordx4 (16 B per lane)
//   win     each lane reads its own 128-B window (8 x global_load_dwordx4, imm offsets),
//           the wave's windows 256 B apart (config 2's request stride), 2 windows in a row
//   dma1    LDS-DMA, 8 whole 128-B lines per instruction, 1 window per lane in flight (r01 kernel)
//   dma2    as dma1 with 2 windows per lane in flight (double-buffered staging)
// Each read is consumed (xor into a register).  Reports GB/s and the in-kernel
// shader clock (s_memtime / s_memrealtime at 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o tools/ubench_stream
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gq;

__device__ unsigned long long g_clk[2];

__device__ __forceinline__ void clk_begin(unsigned long long &t, unsigned long long &r)
{
  t = __builtin_amdgcn_s_memtime();
  r = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void clk_end(unsigned long long t, unsigned long long r)
{
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    g_clk[0] = t1 - t;
    g_clk[1] = r1 - r;
  }
}

template <int NT, int UNROLL>
__global__ void coal(const uint8_t *buf, uint64_t bytes, uint32_t *out)
{
  unsigned long long t, r;
  clk_begin(t, r);
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x * 16 * UNROLL;
  uint32_t acc = 0;
  for (uint64_t at = ((uint64_t) blockIdx.x * blockDim.x * UNROLL + threadIdx.x) * 16; at < bytes; at += stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      gq *p = (gq *) (uintptr_t) (buf + at + (uint64_t) u * blockDim.x * 16);
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  clk_end(t, r);
}

// lane-per-window: each lane reads WIN windows of 128 B (consecutive) of "its request" per round
template <int NT, int WIN>
__global__ void win(const uint8_t *buf, uint64_t bytes, uint32_t *out)
{
  unsigned long long t, r;
  clk_begin(t, r);
  const uint64_t per_round = (uint64_t) gridDim.x * blockDim.x * 128 * WIN;
  uint32_t acc = 0;
  for (uint64_t base = (uint64_t) (blockIdx.x * blockDim.x + threadIdx.x) * 128 * WIN; base < bytes; base += per_round) {
    u32x4 v[8 * WIN];
#pragma unroll
    for (int q = 0; q < 8 * WIN; q++) {
      gq *p = (gq *) (uintptr_t) (buf + base + 16 * q);
      v[q] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int q = 0; q < 8 * WIN; q++) acc ^= v[q][0] ^ v[q][1] ^ v[q][2] ^ v[q][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  clk_end(t, r);
}

// config 2's 64-B window progression: lane l owns request r (256 B); round k
// reads bytes [64k, 64k + 64) of it (4 x dwordx4), 4 rounds per request, then
// the lane moves on by the grid's lane count
template <int NT>
__global__ void win64(const uint8_t *buf, uint64_t bytes, uint32_t *out)
{
  unsigned long long t, r;
  clk_begin(t, r);
  const uint64_t lanes = (uint64_t) gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t req = blockIdx.x * blockDim.x + threadIdx.x; req * 256 < bytes; req += lanes) {
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
      u32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        gq *p = (gq *) (uintptr_t) (buf + req * 256 + 64 * k + 16 * q);
        v[q] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int q = 0; q < 4; q++) acc ^= v[q][0] ^ v[q][1] ^ v[q][2] ^ v[q][3];
      acc = __builtin_amdgcn_readfirstlane(acc) ^ acc;   /* keep the rounds apart */
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  clk_end(t, r);
}

// config 5's access: lane l owns request r (STRIDE bytes apart) and reads its
// first BYTES (whole 16-B pieces) once; reported GB/s counts the bytes read
template <int BYTES, int STRIDE>
__global__ void sparse(const uint8_t *buf, uint64_t bytes, uint32_t *out)
{
  unsigned long long t, r;
  clk_begin(t, r);
  const uint64_t lanes = (uint64_t) gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t req = blockIdx.x * blockDim.x + threadIdx.x; req * STRIDE < bytes; req += lanes) {
    u32x4 v[BYTES / 16];
#pragma unroll
    for (int q = 0; q < BYTES / 16; q++) v[q] = *(gq *) (uintptr_t) (buf + req * STRIDE + 16 * q);
#pragma unroll
    for (int q = 0; q < BYTES / 16; q++) acc ^= v[q][0] ^ v[q][1] ^ v[q][2] ^ v[q][3];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  clk_end(t, r);
}

// LDS-DMA: per wave, a staging slot of 64 windows x 128 B; instruction i fetches
// 8 whole lines (windows 8i..8i+7); SLOTS slots in flight, consumed in order
template <int NT, int SLOTS, int OFF = 0>
__global__ void dma(const uint8_t *buf, uint64_t bytes, uint32_t *out)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  unsigned long long t, r;
  clk_begin(t, r);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const uint32_t slot_bytes = 64 * 128;
  uint8_t *mine = lds + (size_t) wave * SLOTS * slot_bytes;
  const uint64_t per_round = (uint64_t) gridDim.x * waves * slot_bytes;
  uint64_t src = ((uint64_t) blockIdx.x * waves + wave) * slot_bytes;
  uint32_t acc = 0;
  auto issue = [&](uint64_t s, int slot) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const void *g = buf + OFF + (s < bytes ? s : 0) + 1024u * i + 16u * lane;
      __attribute__((address_space(3))) void *l =
          (__attribute__((address_space(3))) void *) (mine + slot * slot_bytes + 1024u * i);
      if (NT) __builtin_amdgcn_global_load_lds(g, l, 16, 0, 2);
      else __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
    }
  };
#pragma unroll
  for (int k = 0; k < SLOTS; k++) issue(src + (uint64_t) k * per_round, k);
  int slot = 0;
  for (uint64_t s = src; s < bytes; s += per_round) {
    if (SLOTS == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    const u32x4 *w = reinterpret_cast<const u32x4 *>(mine + slot * slot_bytes + 128 * lane);
    u32x4 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = w[q];
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= v[q][0] ^ v[q][1] ^ v[q][2] ^ v[q][3];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue(s + (uint64_t) SLOTS * per_round, slot);
    slot = SLOTS == 1 ? 0 : slot ^ 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  clk_end(t, r);
}

// record writes: each lane owns a 128-B line (a request's max_headers = 16
// record slots) and writes the first BYTES of it with STORE-byte stores
template <int BYTES, int STORE>
__global__ void wrec(uint8_t *dst, uint64_t lines, uint32_t *out)
{
  const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lines) return;
  uint8_t *l = dst + i * 128;
  if (STORE == 16) {
#pragma unroll
    for (int q = 0; q < BYTES / 16; q++)
      *reinterpret_cast<__attribute__((address_space(1))) u32x4 *>((uintptr_t) (l + 16 * q)) = u32x4{(uint32_t) i, 1, 2, 3};
  } else {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int q = 0; q < BYTES / 8; q++)
      *reinterpret_cast<__attribute__((address_space(1))) u32x2 *>((uintptr_t) (l + 8 * q)) = u32x2{(uint32_t) i, 1};
  }
}

template <class F>
void run_w(const char *name, F fn, uint8_t *dst, uint64_t lines, uint32_t *out)
{
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int block = 256;
  const int grid = (int) ((lines + block - 1) / block);
  float best = 1e9;
  for (int rep = 0; rep < 6; rep++) {
    CHECK(hipMemset(dst, 0, lines * 128));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(block), 0, 0, dst, lines, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (rep && ms < best) best = ms;
  }
  printf("%-34s %8.1f us for %llu lines\n", name, best * 1e3, (unsigned long long) lines);
  fflush(stdout);
}

template <class F>
void run(const char *name, F fn, int grid, int block, size_t lds, const uint8_t *buf, uint64_t bytes, uint32_t *out,
         double useful = 1.0)
{
  if (lds) CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(block), lds, 0, buf, bytes, out);
  CHECK(hipDeviceSynchronize());
  float best = 1e9;
  double mhz = 0;
  for (int rep = 0; rep < 5; rep++) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(block), lds, 0, buf, bytes, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) {
      best = ms;
      unsigned long long c[2];
      CHECK(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_clk), sizeof c, 0, hipMemcpyDeviceToHost));
      mhz = c[1] ? (double) c[0] / (double) c[1] * 100.0 : 0;
    }
  }
  printf("%-34s grid %5d x %4d  %8.1f GB/s  %.3f ms  clock %.0f MHz\n", name, grid, block, bytes * useful / (best * 1e-3) / 1e9, best, mhz);
  fflush(stdout);
}

int main(int argc, char **argv)
{
  const char *only = argc > 1 ? argv[1] : "";   /* "pmc": the FETCH_SIZE calibration pair only */
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 2ull << 30;
  uint8_t *buf;
  uint32_t *out;
  CHECK(hipMalloc(&buf, bytes + 65536));
  CHECK(hipMemset(buf, 0x41, bytes + 65536));
  CHECK(hipMalloc(&out, 64u << 20));
  if (only[0] == 'w') {   /* record-write patterns, 1M lines (config 2's hdrs array) */
    const uint64_t lines = 1u << 20;
    uint8_t *dst = buf + (1ull << 30);
    run_w("write 32 B of 128 (2 x 16 B)", wrec<32, 16>, dst, lines, out);
    run_w("write 32 B of 128 (4 x 8 B)", wrec<32, 8>, dst, lines, out);
    run_w("write 64 B of 128 (4 x 16 B)", wrec<64, 16>, dst, lines, out);
    run_w("write 128 B of 128 (8 x 16 B)", wrec<128, 16>, dst, lines, out);
    run_w("write 16 B of 128 (1 x 16 B)", wrec<16, 16>, dst, lines, out);
    return 0;
  }
  if (only[0] == 's') {   /* sparse reads: header bytes of 1 KiB requests; GB/s of bytes read */
    for (int wpc : {16, 32}) {
      const int block = 256, grid = cus * wpc / 4;
      char name[64];
      snprintf(name, sizeof name, "sparse 128/1024 waves/CU %d", wpc); run(name, sparse<128, 1024>, grid, block, 0, buf, bytes, out, 1.0 / 8);
      snprintf(name, sizeof name, "sparse 192/1024 waves/CU %d", wpc); run(name, sparse<192, 1024>, grid, block, 0, buf, bytes, out, 3.0 / 16);
      snprintf(name, sizeof name, "sparse 256/1024 waves/CU %d", wpc); run(name, sparse<256, 1024>, grid, block, 0, buf, bytes, out, 1.0 / 4);
      snprintf(name, sizeof name, "sparse 384/1024 waves/CU %d", wpc); run(name, sparse<384, 1024>, grid, block, 0, buf, bytes, out, 3.0 / 8);
      snprintf(name, sizeof name, "dense 256/256 waves/CU %d", wpc); run(name, sparse<256, 256>, grid, block, 0, buf, bytes, out);
    }
    return 0;
  }
  if (only[0]) {
    /* FETCH_SIZE calibration: 2 GiB read by whole-line LDS-DMA windows, then by
     * the same windows 36 B off line alignment (every window straddles two lines) */
    run("dma1 nt aligned (calibration)", dma<1, 1, 0>, cus, 1024, 16 * 8192, buf, bytes, out);
    run("dma1 unaligned +36 (calibration)", dma<0, 1, 36>, cus, 1024, 16 * 8192, buf, bytes, out);
    run("win 1x128B unaligned +36", win<0, 1>, cus * 4, 256, 0, buf + 36, bytes, out);
    return 0;
  }
  for (int wpc : {8, 16, 32}) {
    const int block = 256, grid = cus * wpc / 4;
    char name[64];
    snprintf(name, sizeof name, "coal x4 waves/CU %d", wpc); run(name, coal<0, 4>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "coal x4 nt waves/CU %d", wpc); run(name, coal<1, 4>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "coal x8 waves/CU %d", wpc); run(name, coal<0, 8>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "win 1x128B waves/CU %d", wpc); run(name, win<0, 1>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "win 1x128B nt waves/CU %d", wpc); run(name, win<1, 1>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "win 2x128B waves/CU %d", wpc); run(name, win<0, 2>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "win64 progression waves/CU %d", wpc); run(name, win64<0>, grid, block, 0, buf, bytes, out);
    snprintf(name, sizeof name, "win64 progression nt waves/CU %d", wpc); run(name, win64<1>, grid, block, 0, buf, bytes, out);
  }
  for (int wpc : {8, 16}) {
    const int block = wpc * 64, grid = cus;
    char name[64];
    snprintf(name, sizeof name, "dma1 waves/CU %d", wpc); run(name, dma<0, 1>, grid, block, (size_t) wpc * 8192, buf, bytes, out);
    snprintf(name, sizeof name, "dma1 nt waves/CU %d", wpc); run(name, dma<1, 1>, grid, block, (size_t) wpc * 8192, buf, bytes, out);
    snprintf(name, sizeof name, "dma1 +36 waves/CU %d", wpc); run(name, dma<0, 1, 36>, grid, block, (size_t) wpc * 8192, buf, bytes, out);
    if (wpc <= 8) {
      snprintf(name, sizeof name, "dma2 waves/CU %d", wpc); run(name, dma<0, 2>, grid, block, (size_t) wpc * 16384, buf, bytes, out);
      snprintf(name, sizeof name, "dma2 nt waves/CU %d", wpc); run(name, dma<1, 2>, grid, block, (size_t) wpc * 16384, buf, bytes, out);
    }
  }
  return 0;
}
