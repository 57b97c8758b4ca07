// ubench_lines.hip -- does config 2's window order cost HBM bandwidth?
//
// rhp_dfa_kernel walks one 128-B window per lane per iteration; with 256-B
// requests a wave's 64 windows of one iteration are the FIRST lines of 64
// consecutive requests (every other 128-B line of a 16 KiB run), the next
// iteration their SECOND lines.  This streams config 2's 268 MB over 4 rotated
// copies with the kernel's LDS-DMA loads (8 x 1 KiB per wave per iteration,
// 8 whole lines per instruction, 16 waves per CU, one iteration in flight per
// wave) and writes 32 B of compact records per request (write-through), in
// two line orders:
//   alt     iteration 2k: lines 0, 2, 4 .. 126 of the group, 2k+1: 1, 3 .. 127  (the kernel's)
//   contig  iteration 2k: lines 0 .. 63, 2k+1: lines 64 .. 127
// No parsing: the read back from LDS is xor-folded.  Prints us per launch.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lines.hip -o tools/ubench_lines
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kBytes = 268435456ull;   /* 1M x 256 B */
constexpr uint32_t kReqs = (uint32_t) (kBytes / 256);
constexpr int kWaves = 16;

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

/* line (0..127) of the wave's 16 KiB group that lane w's window takes at iteration parity it */
template <int ORDER>
__device__ __forceinline__ uint32_t line_of(uint32_t w, uint32_t it)
{
  if (ORDER == 0) return 2u * w + it;   /* alt */
  return 64u * it + w;                  /* contig */
}

template <int ORDER, int WT>
__global__ __launch_bounds__(kWaves * 64, 1) void lines(const uint8_t *buf, uint32_t *lens, uint32_t *out)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t stage = __builtin_amdgcn_readfirstlane(wave * 8192u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf), 0, -1, 0x00020000);
  /* the wave's groups of 64 requests: a contiguous range per workgroup, waves interleaved */
  const uint32_t groups = kReqs / 64u, per_wg = groups / gridDim.x;
  const uint32_t g0 = blockIdx.x * per_wg;
  uint32_t acc = 0;
  uint32_t it_total = 2u * (per_wg / kWaves);
  auto issue = [&](uint32_t k) {
    const uint32_t g = g0 + wave + kWaves * (k >> 1), it = k & 1u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      /* instruction i: windows 8i .. 8i+7, lane j a 16-B part of window 8i + (j >> 3) */
      const uint32_t w = 8u * i + (lane >> 3), part = lane & 7u;
      const uint32_t off = g * 16384u + 128u * line_of<ORDER>(w, it) + 16u * part;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *) (lds + stage + 1024u * i), 16,
                                               off, 0, 0, 2);
    }
  };
  issue(0);
  for (uint32_t k = 0; k < it_total; k++) {
    wait_vm0();
    u32x4 W[8];
#pragma unroll
    for (int q = 0; q < 8; q++)
      W[q] = *reinterpret_cast<const u32x4 *>(lds + stage + (lane >> 3) * 1024u + (lane & 7u) * 128u + 16u * q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (k + 1 < it_total) issue(k + 1);
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= W[q][0] ^ W[q][1] ^ W[q][2] ^ W[q][3];
    if (k & 1u) {   /* the group's records: 16 B request + 4 x 4 B lengths, header-major */
      const uint32_t g = g0 + wave + kWaves * (k >> 1), i = 64u * g + lane;
      uint32_t *r = lens + 4u * i;
      if (WT) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(r), "v"(u32x4{acc, 1, 2, 3}) : "memory");
      else *reinterpret_cast<u32x4 *>(r) = u32x4{acc, 1, 2, 3};
#pragma unroll
      for (int h = 0; h < 4; h++) {
        uint32_t *q = lens + 4u * kReqs + (uint32_t) h * kReqs + i;
        if (WT) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(q), "v"(acc + h) : "memory");
        else *q = acc + h;
      }
    }
  }
  out[blockIdx.x * blockDim.x + tid] = acc;
}

/* config 5's shape (round 6): 1M requests 1 KiB apart, of
 * each only the header section's two 128-B lines read (iterations 2k, 2k+1:
 * line 0 then line 1 of the wave's 64 requests, LDS-DMA as the kernel), and
 * RB bytes of records written per request: the request record (16 B or dense
 * 8 B), the compact http record (8 B) and four header lengths (4 B or dense
 * 2 B), header-major, written through. */
constexpr uint64_t kPostStride = 1024;
template <int DENSE>
__global__ __launch_bounds__(kWaves * 64, 1) void post5(const uint8_t *buf, uint32_t *lens, uint32_t *out)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t stage = __builtin_amdgcn_readfirstlane(wave * 8192u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf), 0, -1, 0x00020000);
  const uint32_t groups = kReqs / 64u, per_wg = groups / gridDim.x;
  const uint32_t g0 = blockIdx.x * per_wg;
  uint32_t acc = 0;
  const uint32_t it_total = 2u * (per_wg / kWaves);
  auto issue = [&](uint32_t k) {
    const uint32_t g = g0 + wave + kWaves * (k >> 1), it = k & 1u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t w = 8u * i + (lane >> 3), part = lane & 7u;
      const uint32_t off = (uint32_t) ((64u * g + w) * kPostStride) + 128u * it + 16u * part;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *) (lds + stage + 1024u * i), 16,
                                               off, 0, 0, 2);
    }
  };
  issue(0);
  for (uint32_t k = 0; k < it_total; k++) {
    wait_vm0();
    u32x4 W[8];
#pragma unroll
    for (int q = 0; q < 8; q++)
      W[q] = *reinterpret_cast<const u32x4 *>(lds + stage + (lane >> 3) * 1024u + (lane & 7u) * 128u + 16u * q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (k + 1 < it_total) issue(k + 1);
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= W[q][0] ^ W[q][1] ^ W[q][2] ^ W[q][3];
    if (k & 1u) {
      const uint32_t g = g0 + wave + kWaves * (k >> 1), i = 64u * g + lane;
      uint8_t *base = reinterpret_cast<uint8_t *>(lens);
      if (DENSE) {
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(base + 8ull * i), "v"(u32x2{acc, 1}) : "memory");
      } else {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(base + 16ull * i), "v"(u32x4{acc, 1, 2, 3}) : "memory");
      }
      asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(base + 16ull * kReqs + 8ull * i), "v"(u32x2{acc, 7}) : "memory");
#pragma unroll
      for (int h = 0; h < 4; h++) {
        uint8_t *q = base + 24ull * kReqs + (DENSE ? 2ull : 4ull) * ((uint64_t) h * kReqs + i);
        if (DENSE) asm volatile("global_store_short %0, %1, off sc1" ::"v"(q), "v"(acc + h) : "memory");
        else asm volatile("global_store_dword %0, %1, off sc1" ::"v"(q), "v"(acc + h) : "memory");
      }
    }
  }
  out[blockIdx.x * blockDim.x + tid] = acc;
}

template <class L>
void run(const char *name, L launch, uint8_t **in, uint64_t bytes = kBytes)
{
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int steps = 50;
  for (int k = 0; k < 8; k++) launch(in[k % 4]);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int k = 0; k < steps; k++) launch(in[k % 4]);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / steps;
  printf("%-44s %7.1f us  %6.0f GB/s read  frac %.3f\n", name, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
  fflush(stdout);
}

int main()
{
  uint8_t *in[4];
  for (int k = 0; k < 4; k++) {
    CHECK(hipMalloc(&in[k], kBytes + 4096));
    CHECK(hipMemset(in[k], k + 1, kBytes + 4096));
  }
  uint32_t *lens, *out;
  CHECK(hipMalloc(&lens, 32ull * kReqs + 65536));
  CHECK(hipMalloc(&out, 4 << 20));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t lds = kWaves * 8192;
#define RUN(ORDER, WT, NAME)                                                                                       \
  do {                                                                                                             \
    CHECK(hipFuncSetAttribute((const void *) lines<ORDER, WT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds)); \
    run(NAME, [&](uint8_t *b) { hipLaunchKernelGGL((lines<ORDER, WT>), dim3(cus), dim3(kWaves * 64), lds, 0, b, lens, out); }, in); \
  } while (0)
  printf("CUs %d, %llu B per launch, 4 rotated copies, LDS-DMA windows, 16 waves per CU\n", cus, (unsigned long long) kBytes);
  if (getenv("POST5")) {   /* config 5's shape: 1 GiB copies, two lines read per 1 KiB request */
    uint8_t *pin[4];
    for (int k = 0; k < 4; k++) {
      CHECK(hipMalloc(&pin[k], kReqs * kPostStride + 4096));
      CHECK(hipMemset(pin[k], k + 1, kReqs * kPostStride + 4096));
    }
    uint32_t *plens;
    CHECK(hipMalloc(&plens, 40ull * kReqs + 65536));
    /* "read" rate over the header sections' algorithmic bytes (133.3 B mean per request in config 5) */
    const uint64_t alg = 139767435ull;
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipFuncSetAttribute((const void *) post5<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
      run("post5: 2 lines per 1 KiB request, 40 B records wt", [&](uint8_t *b) { hipLaunchKernelGGL((post5<0>), dim3(cus), dim3(kWaves * 64), lds, 0, b, plens, out); }, pin, alg);
      CHECK(hipFuncSetAttribute((const void *) post5<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
      run("post5: 2 lines per 1 KiB request, 24 B records wt", [&](uint8_t *b) { hipLaunchKernelGGL((post5<1>), dim3(cus), dim3(kWaves * 64), lds, 0, b, plens, out); }, pin, alg);
    }
    return 0;
  }
  for (int rep = 0; rep < 3; rep++) {
    RUN(0, 1, "alt (kernel order) + 32 B wt records");
    RUN(1, 1, "contig + 32 B wt records");
    RUN(0, 0, "alt (kernel order), plain records");
    RUN(1, 0, "contig, plain records");
  }
  return 0;
}
