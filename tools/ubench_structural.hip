// ubench_structural.hip -- what north_star's "wavefront ballot/prefix" structural
// pass costs on gfx950 (MI355X) before it has produced a single record: every
// byte of config 2's 268 MB (4 rotated copies, 1 GiB, as bench.py) is read with
// coalesced global_load_dwordx4 (16 B per lane, a wave streams 1 KiB per load),
// classified into the byte classes the grammar needs (LF, CR, ':', SP, CTL/DEL),
// each class packed into a 16-bit per-lane mask (natural byte order), and the
// line ends prefix-counted across the wave (the line index every LF's record
// would need).  Nothing is validated beyond the classes and no record is
// written, so the time is a LOWER bound for a kernel built that way; compare
// with the read-only ceiling (tools/ubench_ceiling.hip, 42 us) and the pair-DFA
// kernel's whole parse (68 us, records included).
//   CLASSES = 1 (LF only) .. 5 (LF, CR, ':', SP, CTL/DEL)
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_structural.hip -o tools/ubench_structural
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gq;

constexpr uint64_t kBytes = 268435456ull;   /* 1M x 256 B */

/* bit 7 of each byte of the result is set where the byte of v equals c:
 * (w ^ C) + 0x7f7f7f7f carries into bit 7 unless the low 7 bits match, and
 * bit 7 of v itself must be clear */
__device__ __forceinline__ uint32_t eq_mask(uint32_t v, uint32_t w, uint32_t c)
{
  return ~(((w ^ (c * 0x01010101u)) + 0x7f7f7f7fu) | v) & 0x80808080u;
}
/* bytes < 0x20 or == 0x7f */
__device__ __forceinline__ uint32_t ctl_mask(uint32_t v, uint32_t w)
{
  const uint32_t lt20 = ~((w + 0x60606060u) | v) & 0x80808080u;
  return lt20 | eq_mask(v, w, 0x7fu);
}
/* four dwords' bit-7 flags -> 16 bits in byte order (byte 4d + b at bit 4d + b) */
__device__ __forceinline__ uint32_t pack16(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3)
{
  auto nib = [](uint32_t m) { return (((m >> 7) & 0x01010101u) * 0x01020408u) >> 24; };
  return nib(m0) | nib(m1) << 4 | nib(m2) << 8 | nib(m3) << 12;
}

template <int CLASSES, int U>
__global__ __launch_bounds__(1024) void structural(const uint8_t *buf, uint32_t *out)
{
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t) gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0, lines = 0;
  for (uint64_t c = (uint64_t) blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c * 1024 * U < kBytes; c += waves) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      v[u] = __builtin_nontemporal_load((gq *) (uintptr_t) (buf + (c * U + u) * 1024 + 16 * lane));
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t w[4], lf[4], cr[4], co[4], sp[4], ct[4];
#pragma unroll
      for (int d = 0; d < 4; d++) {
        w[d] = v[u][d] & 0x7f7f7f7fu;
        lf[d] = eq_mask(v[u][d], w[d], '\n');
        if (CLASSES >= 2) cr[d] = eq_mask(v[u][d], w[d], '\r');
        if (CLASSES >= 3) co[d] = eq_mask(v[u][d], w[d], ':');
        if (CLASSES >= 4) sp[d] = eq_mask(v[u][d], w[d], ' ');
        if (CLASSES >= 5) ct[d] = ctl_mask(v[u][d], w[d]);
      }
      const uint32_t mlf = pack16(lf[0], lf[1], lf[2], lf[3]);
      uint32_t mix = mlf;
      if (CLASSES >= 2) mix ^= pack16(cr[0], cr[1], cr[2], cr[3]) << 1;
      if (CLASSES >= 3) mix ^= pack16(co[0], co[1], co[2], co[3]) << 2;
      if (CLASSES >= 4) mix ^= pack16(sp[0], sp[1], sp[2], sp[3]) << 3;
      if (CLASSES >= 5) mix ^= pack16(ct[0], ct[1], ct[2], ct[3]) << 4;
      /* the wave's line ends: each lane's first line index (exclusive prefix of
       * the LF counts over the lanes below it) */
      uint32_t x = (uint32_t) __builtin_popcount(mlf);
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t) __shfl_up((int) x, d);
        x += lane >= (uint32_t) d ? y : 0u;
      }
      lines += x;
      acc ^= mix;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ lines;
}

template <class L>
void run(const char *name, L launch, uint8_t **in)
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
  printf("%-44s %7.1f us  %6.0f GB/s  frac %.3f\n", name, us, kBytes / us / 1e3, kBytes / us / 1e3 / 8000.0);
  fflush(stdout);
}

int main()
{
  uint8_t *in[4];
  for (int k = 0; k < 4; k++) {
    CHECK(hipMalloc(&in[k], kBytes + 4096));
    /* request-like bytes: a 256-B line pattern with LFs, CRs, colons and spaces */
    CHECK(hipMemset(in[k], 'a', kBytes + 4096));
  }
  {
    static const char pat[] = "GET /abc HTTP/1.1\r\nHost: tfb-server:8080\r\nAccept: text/plain\r\n\r\n";
    uint8_t *h = (uint8_t *) malloc(1 << 20);
    for (int i = 0; i < (1 << 20); i++) h[i] = (uint8_t) pat[i % (sizeof pat - 1)];
    for (int k = 0; k < 4; k++)
      for (uint64_t o = 0; o < kBytes; o += 1 << 20) CHECK(hipMemcpy(in[k] + o, h, 1 << 20, hipMemcpyHostToDevice));
    free(h);
  }
  uint32_t *out;
  CHECK(hipMalloc(&out, 4 << 20));
  printf("CUs 256 x 1024 threads, 268435456 B per launch, 4 rotated copies\n");
#define RUN(C, U)                                                                                         \
  run("classes " #C " (LF..), " #U " loads in flight", [&](uint8_t *b) {                                  \
    hipLaunchKernelGGL((structural<C, U>), dim3(256), dim3(1024), 0, 0, b, out); }, in)
  for (int rep = 0; rep < 2; rep++) {
    RUN(1, 4);
    RUN(3, 4);
    RUN(5, 4);
    RUN(5, 8);
  }
  return 0;
}
