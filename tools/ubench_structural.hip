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
#include <initializer_list>

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

/* ---- round 4: one class byte per input byte from a v_perm_b32 nibble LUT ----
 * class(x) = LO[x & 15] & HI[x >> 4], each class bit a rectangle (a set of low
 * nibbles x a set of high nibbles), the usual byte-class split of a
 * SIMD parser.  The bits, exact for these byte sets:
 *   0 LF 0x0a    1 CR 0x0d    2 ':' 0x3a    3 SP 0x20
 *   4 CTL 0x10-0x1f      6 CTL 0x00-0x0f but HT      7 DEL 0x7f
 *   5 one rectangle of the non-tchar bytes (0x22, 0x28, 0x29, 0x2c, 0x2f and
 *     0x5b-0x5d: hi {2, 5} x lo {2, 8, 9, c, f, b, d}; the rest of the
 *     non-tchar set would take more bits -- the cost is the same)
 * A 16-entry lookup is two v_perm_b32 (entries 0-7 and 8-15, selector & 7)
 * merged per byte on the selector's bit 3 (expanded to a byte mask by a packed
 * 16-bit multiply, no carry between bytes), so LO and HI cost 2 x 5 VALU per
 * dword plus the nibble split.  Per lane and 16-B part, two 16-bit masks are
 * kept -- structural (LF, CR, ':') and invalid (the CTL/DEL bits) -- and the
 * line ends are prefix-counted across the wave with a ballot per byte
 * position.  No record is written. */
struct Lut16 { uint32_t t0, t1, t2, t3; };   /* entries 0-3, 4-7, 8-11, 12-15 */

__host__ __device__ constexpr uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
  return a | b << 8 | c << 16 | d << 24;
}

__device__ __forceinline__ uint32_t lut16(const Lut16 &t, uint32_t sel /* 4 nibbles, one per byte */)
{
  const uint32_t s7 = sel & 0x07070707u;
  const uint32_t a = __builtin_amdgcn_perm(t.t1, t.t0, s7);
  const uint32_t b = __builtin_amdgcn_perm(t.t3, t.t2, s7);
  /* per byte 0xff where the nibble is >= 8: bit 3 moved to bit 0 of each byte
   * (0x01 per byte), times 0xff per 16-bit half (no carry into the next byte) */
  const uint32_t b3 = (sel >> 3) & 0x01010101u;
  typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 mm = __builtin_bit_cast(u16x2, b3) * (u16x2){0xffu, 0xffu};   /* v_pk_mul_lo_u16 */
  const uint32_t m = __builtin_bit_cast(uint32_t, mm);
  return (b & m) | (a & ~m);   /* v_bfi_b32 */
}

/* per-byte bit 7 flags of four dwords -> 16-bit mask in byte order */
__device__ __forceinline__ uint32_t msb16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3)
{
  auto nib = [](uint32_t f) { return ((f & 0x80808080u) * 0x00204081u) >> 28; };   /* bits 7,15,23,31 -> 28..31 */
  return nib(f0) | nib(f1) << 4 | nib(f2) << 8 | nib(f3) << 12;
}

template <int U>
__global__ __launch_bounds__(1024) void structural_lut(const uint8_t *buf, uint32_t *out, Lut16 LO, Lut16 HI)
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
      uint32_t st[4], bad[4];
#pragma unroll
      for (int d = 0; d < 4; d++) {
        const uint32_t x = v[u][d];
        const uint32_t cls = lut16(LO, x & 0x0f0f0f0fu) & lut16(HI, (x >> 4) & 0x0f0f0f0fu);
        /* per byte: bit 7 set where any structural / invalid bit is (no carry
         * between bytes: the masked bytes are <= 0x7f before the add) */
        st[d] = (cls & 0x07070707u) + 0x7f7f7f7fu;
        bad[d] = ((cls & 0x50505050u) + 0x7f7f7f7fu) | cls;
      }
      const uint32_t ms = msb16(st[0], st[1], st[2], st[3]);
      const uint32_t mb = msb16(bad[0], bad[1], bad[2], bad[3]);
      /* line ends for the prefix: LF is the structural byte whose class is 1 */
      uint32_t x = (uint32_t) __builtin_popcount(ms);
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t) __shfl_up((int) x, d);
        x += lane >= (uint32_t) d ? y : 0u;
      }
      lines += x;
      acc ^= ms ^ (mb << 16);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ lines;
}

/* the LUTs for the class bits above */
static void make_luts(Lut16 &LO, Lut16 &HI)
{
  uint8_t lo[16] = {0}, hi[16] = {0};
  auto rect = [&](int bit, std::initializer_list<int> los, std::initializer_list<int> his) {
    for (int l : los) lo[l] |= (uint8_t) (1u << bit);
    for (int h : his) hi[h] |= (uint8_t) (1u << bit);
  };
  rect(0, {0xa}, {0x0});
  rect(1, {0xd}, {0x0});
  rect(2, {0xa}, {0x3});
  rect(3, {0x0}, {0x2});
  rect(4, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {0x1});
  rect(6, {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 14, 15}, {0x0});
  rect(7, {0xf}, {0x7});
  rect(5, {0x2, 0x8, 0x9, 0xc, 0xf, 0xb, 0xd}, {0x2, 0x5});
  auto pk = [](const uint8_t *t) { return Lut16{pack4(t[0], t[1], t[2], t[3]), pack4(t[4], t[5], t[6], t[7]),
                                                pack4(t[8], t[9], t[10], t[11]), pack4(t[12], t[13], t[14], t[15])}; };
  LO = pk(lo);
  HI = pk(hi);
}

/* the classes agree with a byte-wise reference on every byte value */
__global__ void lut_check(Lut16 LO, Lut16 HI, uint32_t *cls)
{
  const uint32_t b = threadIdx.x;   /* 256 threads: byte values */
  const uint32_t x = b * 0x01010101u;
  cls[b] = (lut16(LO, x & 0x0f0f0f0fu) & lut16(HI, (x >> 4) & 0x0f0f0f0fu)) & 0xffu;
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
  {
    Lut16 LO, HI;
    make_luts(LO, HI);
    uint32_t *dc, hc[256];
    CHECK(hipMalloc(&dc, 256 * 4));
    hipLaunchKernelGGL(lut_check, dim3(1), dim3(256), 0, 0, LO, HI, dc);
    CHECK(hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost));
    int bad = 0;
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t want = (b == 0x0a) | (b == 0x0d) << 1 | (b == 0x3a) << 2 | (b == 0x20) << 3 | (b >= 0x10 && b < 0x20) << 4 |
                      (b < 0x10 && b != 0x09) << 6 | (b == 0x7f) << 7;
      const uint32_t h = b >> 4, l = b & 15;
      want |= ((h == 2 || h == 5) && (l == 2 || l == 8 || l == 9 || l == 0xc || l == 0xf || l == 0xb || l == 0xd)) << 5;
      bad += hc[b] != want;
    }
    printf("nibble LUT classes: %s (%d of 256 byte values differ from the byte-wise reference)\n", bad ? "WRONG" : "exact", bad);
    if (getenv("ONLY_LUT")) {
      for (int rep = 0; rep < 2; rep++) {
        run("LUT classes, 2 masks + LF prefix, 4 loads", [&](uint8_t *b) {
          hipLaunchKernelGGL((structural_lut<4>), dim3(256), dim3(1024), 0, 0, b, out, LO, HI); }, in);
        run("LUT classes, 2 masks + LF prefix, 8 loads", [&](uint8_t *b) {
          hipLaunchKernelGGL((structural_lut<8>), dim3(256), dim3(1024), 0, 0, b, out, LO, HI); }, in);
      }
      return 0;
    }
  }
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
