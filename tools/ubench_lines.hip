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

/* Depth and records (round 6, second session): the alt order with NW waves per
 * CU, each with DEPTH window sets in flight (DEPTH x 8 KiB of staging per
 * wave), and REC bytes of records per request: 0 none, 1 compact (16 B request
 * record + 4 x 4 B header-major lengths), 2 dense (8 B + 4 x 2 B), written
 * through.  Same bytes read as lines<0, 1>. */
template <int NW, int DEPTH, int REC>
__global__ __launch_bounds__(NW * 64, 1) void lines2(const uint8_t *buf, uint32_t *lens, uint32_t *out)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t stage0 = __builtin_amdgcn_readfirstlane(wave * 8192u * DEPTH);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf), 0, -1, 0x00020000);
  const uint32_t groups = kReqs / 64u, per_wg = groups / gridDim.x;
  const uint32_t g0 = blockIdx.x * per_wg;
  uint32_t acc = 0;
  const uint32_t it_total = 2u * (per_wg / NW);
  auto issue = [&](uint32_t k) {
    const uint32_t g = g0 + wave + NW * (k >> 1), it = k & 1u;
    const uint32_t stage = stage0 + 8192u * (k % DEPTH);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t w = 8u * i + (lane >> 3), part = lane & 7u;
      const uint32_t off = g * 16384u + 128u * line_of<0>(w, it) + 16u * part;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *) (lds + stage + 1024u * i), 16,
                                               off, 0, 0, 2);
    }
  };
#pragma unroll
  for (uint32_t d = 0; d < (uint32_t) DEPTH; d++)
    if (d < it_total) issue(d);
  for (uint32_t k = 0; k < it_total; k++) {
    /* window k landed; the 8 loads of k + 1 (and the 5 record stores of iteration k - 1, issued after
     * them) may still fly: vmcnt counts in issue order */
    if (DEPTH == 2 && k + 1 < it_total) {
      if (REC && k > 0 && !(k & 1u)) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      wait_vm0();
    }
    const uint32_t stage = stage0 + 8192u * (k % DEPTH);
    u32x4 W[8];
#pragma unroll
    for (int q = 0; q < 8; q++)
      W[q] = *reinterpret_cast<const u32x4 *>(lds + stage + (lane >> 3) * 1024u + (lane & 7u) * 128u + 16u * q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (k + DEPTH < it_total) issue(k + DEPTH);
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= W[q][0] ^ W[q][1] ^ W[q][2] ^ W[q][3];
    if (REC && (k & 1u)) {
      const uint32_t g = g0 + wave + NW * (k >> 1), i = 64u * g + lane;
      uint8_t *base = reinterpret_cast<uint8_t *>(lens);
      if (REC == 3) {   /* the 16 B as ONE request-major record, one 16-byte write-through store */
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(base + 16ull * i), "v"(u32x4{acc, 1, 2, 3}) : "memory");
      } else if (REC == 4) {   /* dense header-major, plain stores */
        *reinterpret_cast<u32x2 *>(base + 8ull * i) = u32x2{acc, 1};
#pragma unroll
        for (int h = 0; h < 4; h++) *reinterpret_cast<uint16_t *>(base + 16ull * kReqs + 2ull * ((uint64_t) h * kReqs + i)) = (uint16_t) (acc + h);
      } else if (REC == 5) {   /* one request-major 16 B record, plain store */
        *reinterpret_cast<u32x4 *>(base + 16ull * i) = u32x4{acc, 1, 2, 3};
      }
      if (REC == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(base + 16ull * i), "v"(u32x4{acc, 1, 2, 3}) : "memory");
      else if (REC == 2) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(base + 8ull * i), "v"(u32x2{acc, 1}) : "memory");
#pragma unroll
      for (int h = 0; h < 4 && REC <= 2; h++) {
        uint8_t *q = base + 16ull * kReqs + (REC == 1 ? 4ull : 2ull) * ((uint64_t) h * kReqs + i);
        if (REC == 1) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(q), "v"(acc + h) : "memory");
        else asm volatile("global_store_short %0, %1, off sc1" ::"v"(q), "v"(acc + h) : "memory");
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
void run(const char *name, L launch, uint8_t **in, uint64_t bytes = kBytes, bool two_streams = false)
{
  static hipStream_t st[2] = {nullptr, nullptr};
  if (two_streams && !st[0]) {
    CHECK(hipStreamCreate(&st[0]));
    CHECK(hipStreamCreate(&st[1]));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int steps = 50;
  for (int k = 0; k < 8; k++) launch(in[k % 4], two_streams ? st[k & 1] : (hipStream_t) 0);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int k = 0; k < steps; k++) launch(in[k % 4], two_streams ? st[k & 1] : (hipStream_t) 0);
  CHECK(hipDeviceSynchronize());
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
    run(NAME, [&](uint8_t *b, hipStream_t s) { hipLaunchKernelGGL((lines<ORDER, WT>), dim3(cus), dim3(kWaves * 64), lds, s, b, lens, out); }, in); \
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
      run("post5: 2 lines per 1 KiB request, 40 B records wt", [&](uint8_t *b, hipStream_t s) { hipLaunchKernelGGL((post5<0>), dim3(cus), dim3(kWaves * 64), lds, s, b, plens, out); }, pin, alg);
      CHECK(hipFuncSetAttribute((const void *) post5<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
      run("post5: 2 lines per 1 KiB request, 24 B records wt", [&](uint8_t *b, hipStream_t s) { hipLaunchKernelGGL((post5<1>), dim3(cus), dim3(kWaves * 64), lds, s, b, plens, out); }, pin, alg);
    }
    return 0;
  }
  if (getenv("LINES2")) {   /* depth, wave count and record bytes of the alt order */
#define RUN2G(NW, DEPTH, REC, TWO, G, EXTRA, NAME)                                                                  \
  do {                                                                                                             \
    const size_t l2 = (size_t) NW * DEPTH * 8192 + (EXTRA);                                                        \
    CHECK(hipFuncSetAttribute((const void *) lines2<NW, DEPTH, REC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) l2)); \
    run(NAME, [&](uint8_t *b, hipStream_t s) { hipLaunchKernelGGL((lines2<NW, DEPTH, REC>), dim3(cus * (G)), dim3(NW * 64), l2, s, b, lens, out); }, in, kBytes, TWO); \
  } while (0)
#define RUN2(NW, DEPTH, REC, TWO, NAME) RUN2G(NW, DEPTH, REC, TWO, 1, 0, NAME)
    if (getenv("LINES2_WG")) {   /* one 16-wave workgroup per CU against two 8-wave ones (80 KB of LDS each) */
      for (int rep = 0; rep < 3; rep++) {
        RUN2G(16, 1, 2, false, 1, 27 * 1024, "1 x 16 waves per CU, 16 B dense, one stream");
        RUN2G(16, 1, 2, true, 1, 27 * 1024, "1 x 16 waves per CU, 16 B dense, two streams");
        RUN2G(8, 1, 2, false, 2, 15 * 1024, "2 x 8 waves per CU, 16 B dense, one stream");
        RUN2G(8, 1, 2, true, 2, 15 * 1024, "2 x 8 waves per CU, 16 B dense, two streams");
      }
      return 0;
    }
    for (int rep = 0; rep < 2; rep++) {
      RUN2(16, 1, 3, false, "16 waves x 1 deep, 16 B one dwordx4 wt");
      RUN2(16, 1, 5, false, "16 waves x 1 deep, 16 B one dwordx4 plain");
      RUN2(16, 1, 4, false, "16 waves x 1 deep, 16 B dense plain");
      RUN2(12, 1, 3, false, "12 waves x 1 deep, 16 B one dwordx4 wt");
      RUN2(16, 1, 0, false, "16 waves x 1 deep, no records");
      RUN2(16, 1, 1, false, "16 waves x 1 deep, 32 B wt records");
      RUN2(16, 1, 2, false, "16 waves x 1 deep, 16 B wt dense records");
      RUN2(16, 1, 2, true, "16 waves x 1 deep, 16 B dense, two streams");
      RUN2(8, 2, 0, false, "8 waves x 2 deep, no records");
      RUN2(8, 2, 2, false, "8 waves x 2 deep, 16 B wt dense records");
      RUN2(8, 2, 2, true, "8 waves x 2 deep, 16 B dense, two streams");
      RUN2(8, 1, 2, false, "8 waves x 1 deep, 16 B wt dense records");
      RUN2(12, 1, 2, false, "12 waves x 1 deep, 16 B wt dense records");
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
