/*
 * rhp_writer.hip -- MI355X (gfx950) batched HTTP/1.1 response serialization.
 *
 * http_write_response (src/reactor/http.c:286-297, with _basic :236-259 and
 * _extended :261-284) for n responses at once, so the reactor's response side can
 * run as one device pass per round like the parse side.
 * Four launches on the caller's stream:
 *
 *   rhp_resp_tile_*_kernel every response's size, exactly the sum the reference
 *                          allocates (http.c:244-246, 270-272; the date is the
 *                          fixed 29 bytes the "37" there assumes), then a
 *                          reduce-then-scan over 4096-size tiles (tile sums in
 *                          the caller's work[], one workgroup scans those, every
 *                          tile is scanned in place): exclusive prefix sum ->
 *                          out_off
 *   rhp_resp_write_kernel  wave per group of 64 consecutive responses: each lane
 *                          assembles its response in the wave's LDS stage in the
 *                          reference's push order (http_push_data /
 *                          http_push_field, http.c:51-69; the Content-Length
 *                          digits as http_u32_sprint, :17-44, prints them), then
 *                          the wave stores the group's contiguous output with
 *                          16-byte stores (the stage is shifted so LDS and HBM
 *                          agree modulo 16; byte stores only at the group's two
 *                          unaligned edges).  A group larger than the stage (big
 *                          bodies) is written response by response, the wave's 64
 *                          lanes copying each segment
 *
 * Byte copies are HBM-bound; the response bytes written are the algorithmic bytes.
 */
#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <string.h>

#include "rhp.h"

namespace {

struct WParams {
  const uint8_t *arena;
  const rhp_resp_t *resps;
  const rhp_resp_field_t *fields;
  uint64_t *out_off;
  uint8_t *out;
  uint64_t out_size;
  uint32_t n;
  uint32_t date[8];   /* the 29 date bytes, little-endian in dwords */
};

/* the constant text between the variable parts of a response (http.c:250-258) */
__constant__ const char kHead[] = "HTTP/1.1 ";                    /* 9 */
__constant__ const char kServerDate[] = "\r\nServer: *\r\nDate: ";  /* 19: status CRLF, Server field, "Date: " */
__constant__ const char kType[] = "\r\nContent-Type: ";            /* 16 */
__constant__ const char kLength[] = "\r\nContent-Length: ";        /* 18 */
__constant__ const uint32_t kPow10[10] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u,
                                          1000000000u};

/* decimal digits of v (http_u32_len, http.c:8-15) */
__device__ __forceinline__ uint32_t u32_len(uint32_t v)
{
  uint32_t l = 1;
  while (l < 10 && v >= kPow10[l]) l++;
  return l;
}

/* every byte of a response except its variable parts:
 * 9 + 2 + 11 + 37 + 16 + 18 + 2 (http.c:244) */
constexpr uint64_t kFixed = 9 + 2 + 11 + 37 + 16 + 18 + 2;

__device__ __forceinline__ uint64_t resp_size(const WParams &p, const rhp_resp_t &r)
{
  uint64_t size = kFixed + r.status.len + r.type.len + u32_len(r.body.len) + r.body.len;
  for (uint32_t f = 0; f < r.fields_count; f++) {
    const rhp_resp_field_t x = p.fields[r.fields_first + f];
    size += (uint64_t) x.name.len + 2 + x.value.len + 2;   /* http.c:272 */
  }
  return size;
}


/* out_off[1..n] sizes -> out_off[0..n] offsets, reduce-then-scan over tiles of
 * kTile sizes: tile sums into work[], one workgroup scans work[] (exclusive),
 * then every tile is scanned in place with its carry.  Loads and stores are
 * coalesced; within a workgroup a thread scans 4 consecutive sizes, a wave its
 * 64 threads through shuffles, the workgroup its 16 waves through LDS. */
constexpr uint32_t kTile = 4096;   /* 1024 threads x 4 */

__device__ __forceinline__ unsigned long long wave_incl_scan(unsigned long long v, uint32_t lane)
{
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(v, o);
    if ((int) lane >= o) v += u;
  }
  return v;
}

/* inclusive scan of one value per thread over a 1024-thread workgroup */
__device__ __forceinline__ unsigned long long block_incl_scan(unsigned long long v, unsigned long long *part)
{
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  v = wave_incl_scan(v, lane);
  if (lane == 63) part[w] = v;
  __syncthreads();
  if (w == 0) {
    unsigned long long x = lane < 16 ? part[lane] : 0;
    x = wave_incl_scan(x, lane);
    if (lane < 16) part[lane] = x;
  }
  __syncthreads();
  return v + (w ? part[w - 1] : 0);
}

/* sizes of a tile's responses into out_off[1..], and the tile's sum */
__global__ __launch_bounds__(1024) void rhp_resp_tile_sum_kernel(WParams p, uint64_t *work)
{
  __shared__ unsigned long long part[16];
  const uint64_t lo = 1 + (uint64_t) blockIdx.x * kTile, hi = min(lo + kTile, (uint64_t) p.n + 1);
  unsigned long long s = 0;
  for (uint64_t k = lo + threadIdx.x; k < hi; k += 1024) {
    const uint64_t z = resp_size(p, p.resps[k - 1]);
    p.out_off[k] = z;
    s += z;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < 16; w++) t += part[w];
    work[blockIdx.x] = t;
  }
}

/* work[0..tiles) -> exclusive offsets (one workgroup, 1024 per round) */
__global__ __launch_bounds__(1024) void rhp_resp_top_scan_kernel(uint64_t *work, uint32_t tiles)
{
  __shared__ unsigned long long part[16];
  unsigned long long carry = 0;
  for (uint32_t b = 0; b < tiles; b += 1024) {
    const uint32_t k = b + threadIdx.x;
    const unsigned long long v = k < tiles ? work[k] : 0;
    const unsigned long long inc = block_incl_scan(v, part);
    if (k < tiles) work[k] = carry + inc - v;
    carry += part[15];   /* the round's total */
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void rhp_resp_tile_scan_kernel(uint64_t *a, uint32_t n, const uint64_t *work)
{
  __shared__ unsigned long long part[16];
  const uint64_t base = 1 + (uint64_t) blockIdx.x * kTile + 4u * threadIdx.x, end = (uint64_t) n + 1;
  unsigned long long x[4], s = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    x[q] = base + q < end ? a[base + q] : 0;
    s += x[q];
    x[q] = s;   /* thread-local inclusive */
  }
  const unsigned long long before = block_incl_scan(s, part) - s + work[blockIdx.x];
#pragma unroll
  for (int q = 0; q < 4; q++)
    if (base + q < end) a[base + q] = before + x[q];
  if (blockIdx.x == 0 && threadIdx.x == 0) a[0] = 0;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

/* one segment of a response: bytes up to the first 16-aligned destination,
 * then 16 bytes per lane (1 KiB per store instruction) from funnel-shifted
 * aligned source dwords, then the tail bytes */
__device__ __forceinline__ void put(uint8_t *dst, uint64_t &o, const uint8_t *src, uint32_t len, uint32_t lane)
{
  uint8_t *d = dst + o;
  const uint32_t head = min(len, (uint32_t) ((16u - ((uintptr_t) d & 15u)) & 15u));
  if (len < 128) {
    for (uint32_t j = lane; j < len; j += 64) d[j] = src[j];
    o += len;
    return;
  }
  if (lane < head) d[lane] = src[lane];
  const uint8_t *s = src + head;
  const uint32_t body = (len - head) & ~15u;
  const uintptr_t sa = (uintptr_t) s;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(sa & ~(uintptr_t) 3);
  const uint32_t sh = (uint32_t) sa & 3u, nd = (sh + (len - head) + 3u) >> 2;
  for (uint32_t j = 16u * lane; j < body; j += 1024u) {
    const uint32_t k = j >> 2;
    const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2], w3 = w[k + 3], w4 = k + 4 < nd ? w[k + 4] : 0u;
    *reinterpret_cast<u32x4 *>(d + head + j) = u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                                     __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
  }
  for (uint32_t j = head + body + lane; j < len; j += 64) d[j] = src[j];
  o += len;
}
__device__ __forceinline__ void put_c(uint8_t *dst, uint64_t &o, const char *src, uint32_t len, uint32_t lane)
{
  if (lane < len) dst[o + lane] = (uint8_t) src[lane];
  o += len;
}

/* one response, wave-cooperatively (the path for groups larger than the stage) */
__device__ void write_one(const WParams &p, uint32_t i, uint32_t lane)
{
  uint8_t *dst = p.out;
  const rhp_resp_t r = p.resps[i];
  uint64_t o = p.out_off[i];
  put_c(dst, o, kHead, 9, lane);
  put(dst, o, p.arena + r.status.off, r.status.len, lane);
  put_c(dst, o, kServerDate, 19, lane);
  if (lane < RHP_DATE_LEN) dst[o + lane] = (uint8_t) (p.date[lane >> 2] >> (8u * (lane & 3u)));
  o += RHP_DATE_LEN;
  put_c(dst, o, kType, 16, lane);
  put(dst, o, p.arena + r.type.off, r.type.len, lane);
  put_c(dst, o, kLength, 18, lane);
  const uint32_t v = r.body.len, L = u32_len(v);   /* http_u32_sprint: most significant first */
  if (lane < L) dst[o + lane] = (uint8_t) ('0' + (v / kPow10[L - 1u - lane]) % 10u);
  o += L;
  put_c(dst, o, kType, 2, lane);   /* CRLF */
  for (uint32_t f = 0; f < r.fields_count; f++) {   /* http_push_field (http.c:61-69) */
    const rhp_resp_field_t x = p.fields[r.fields_first + f];
    put(dst, o, p.arena + x.name.off, x.name.len, lane);
    if (lane < 2) dst[o + lane] = lane ? ' ' : ':';
    o += 2;
    put(dst, o, p.arena + x.value.off, x.value.len, lane);
    put_c(dst, o, kType, 2, lane);
  }
  put_c(dst, o, kType, 2, lane);   /* the empty line */
  put(dst, o, p.arena + r.body.off, r.body.len, lane);
}

/* ---- the lane-per-response stage writers (LDS byte o of the wave's stage) ---- */
typedef __attribute__((address_space(3))) uint8_t lds8;

/* a compile-time constant string */
template <uint32_t N>
__device__ __forceinline__ void st_const(lds8 *L, uint32_t &o, const char (&s)[N])
{
#pragma unroll
  for (uint32_t j = 0; j + 1 < N; j++) L[o + j] = (uint8_t) s[j];
  o += N - 1;
}
/* len bytes from global memory at src: the aligned dwords that hold them (no
 * byte outside [src & ~3, src + len + 3) is read), funnel-shifted */
__device__ __forceinline__ void st_span(lds8 *L, uint32_t &o, const uint8_t *src, uint32_t len)
{
  const uintptr_t a = (uintptr_t) src;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t) 3);
  const uint32_t sh = (uint32_t) a & 3u, nd = (sh + len + 3u) >> 2;
  uint32_t lo = len ? w[0] : 0;
  for (uint32_t j = 0; j < len; j += 4) {
    const uint32_t k = (j >> 2) + 1u;
    const uint32_t hi = k < nd ? w[k] : 0u;
    const uint32_t d = __builtin_amdgcn_alignbyte(hi, lo, sh);
    L[o + j] = (uint8_t) d;
    if (j + 1 < len) L[o + j + 1] = (uint8_t) (d >> 8);
    if (j + 2 < len) L[o + j + 2] = (uint8_t) (d >> 16);
    if (j + 3 < len) L[o + j + 3] = (uint8_t) (d >> 24);
    lo = hi;
  }
  o += len;
}

constexpr uint32_t kStage = 16384;   /* LDS bytes per wave: groups up to 16 KiB - 16 */

__global__ __launch_bounds__(256) void rhp_resp_write_kernel(WParams p)
{
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[4 * kStage];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  if (p.out_off[p.n] > p.out_size) return;   /* does not fit: sizes only (rhp.h) */
  lds8 *L = (lds8 *) (stage_all + wv * kStage);
  const uint32_t groups = (p.n + 63u) / 64u;
  for (uint32_t g = wave; g < groups; g += nwaves) {
    const uint32_t i0 = g * 64u, i1 = min(i0 + 64u, p.n);
    const uint64_t G0 = p.out_off[i0], G1 = p.out_off[i1];
    const uint32_t shift = (uint32_t) (uintptr_t) (p.out + G0) & 15u;   /* LDS and HBM agree modulo 16 */
    if (G1 - G0 + shift > kStage) {   /* big responses: the cooperative path */
      for (uint32_t i = i0; i < i1; i++) write_one(p, i, lane);
      continue;
    }
    const uint32_t i = i0 + lane;
    if (i < i1) {
      const rhp_resp_t r = p.resps[i];
      uint32_t o = shift + (uint32_t) (p.out_off[i] - G0);
      st_const(L, o, "HTTP/1.1 ");
      st_span(L, o, p.arena + r.status.off, r.status.len);
      st_const(L, o, "\r\nServer: *\r\nDate: ");
#pragma unroll
      for (uint32_t j = 0; j < RHP_DATE_LEN; j++) L[o + j] = (uint8_t) (p.date[j >> 2] >> (8u * (j & 3u)));
      o += RHP_DATE_LEN;
      st_const(L, o, "\r\nContent-Type: ");
      st_span(L, o, p.arena + r.type.off, r.type.len);
      st_const(L, o, "\r\nContent-Length: ");
      const uint32_t v = r.body.len, D = u32_len(v);   /* http_u32_sprint: most significant first */
      for (uint32_t j = 0; j < D; j++) L[o + j] = (uint8_t) ('0' + (v / kPow10[D - 1u - j]) % 10u);
      o += D;
      st_const(L, o, "\r\n");
      for (uint32_t f = 0; f < r.fields_count; f++) {   /* http_push_field (http.c:61-69) */
        const rhp_resp_field_t x = p.fields[r.fields_first + f];
        st_span(L, o, p.arena + x.name.off, x.name.len);
        st_const(L, o, ": ");
        st_span(L, o, p.arena + x.value.off, x.value.len);
        st_const(L, o, "\r\n");
      }
      st_const(L, o, "\r\n");   /* the empty line */
      st_span(L, o, p.arena + r.body.off, r.body.len);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);   /* lgkmcnt(0): the stage is written (wave-local) */
    __builtin_amdgcn_wave_barrier();
    /* out[G0, G1) <- stage[shift, shift + G1 - G0): 16-byte stores between the
     * first and the last 16-aligned addresses, byte stores outside */
    const uint64_t A0 = G0 + ((16u - shift) & 15u), A1 = G1 - (((uint32_t) (uintptr_t) (p.out + G1)) & 15u);
    if (A0 < A1) {
      for (uint64_t a = A0 + 16u * lane; a < A1; a += 1024u) {
        const uint32_t so = (uint32_t) (a - G0) + shift;
        const u32x4 d = *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(L + so);
        *reinterpret_cast<u32x4 *>(p.out + a) = d;
      }
      if (lane < A0 - G0) p.out[G0 + lane] = L[shift + lane];
      if (lane < G1 - A1) p.out[A1 + lane] = L[shift + (uint32_t) (A1 - G0) + lane];
    } else {   /* the whole group within one 16-byte line (or two) */
      for (uint32_t j = lane; j < G1 - G0; j += 64) p.out[G0 + j] = L[shift + j];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

/* the CU count per device id (one host thread per GPU may call concurrently) */
constexpr int kWriterMaxDevices = 64;
std::atomic<int> g_writer_cus[kWriterMaxDevices];

}  // namespace

extern "C" int rhp_write_responses(const rhp_resp_batch_t *b, void *stream)
{
  if (!b) return -22;
  if (!b->out_off || !b->date || b->date_len != RHP_DATE_LEN) return -22;
  if (b->n > 0 && (!b->arena || !b->resps)) return -22;
  if (!b->out && b->out_size != 0) return -22;
  if (b->n > 0 && !b->work) return -22;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int dev = 0, cus = 0;
  {
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int) e;
    if (dev < 0 || dev >= kWriterMaxDevices) return -22;
    cus = g_writer_cus[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
      e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (e != hipSuccess) return (int) e;
      g_writer_cus[dev].store(cus, std::memory_order_relaxed);
    }
  }
  WParams p;
  p.arena = b->arena;
  p.resps = b->resps;
  p.fields = b->fields;
  p.out_off = b->out_off;
  p.out = b->out;
  p.out_size = b->out_size;
  p.n = b->n;
  memset(p.date, 0, sizeof p.date);
  memcpy(p.date, b->date, RHP_DATE_LEN);
  if (b->n == 0) return (int) hipMemsetAsync(b->out_off, 0, sizeof(uint64_t), s);
  const uint32_t cap = (uint32_t) cus * 8u;
  const uint32_t tiles = (b->n + kTile - 1u) / kTile;
  hipLaunchKernelGGL(rhp_resp_tile_sum_kernel, dim3(tiles), dim3(1024), 0, s, p, b->work);
  hipLaunchKernelGGL(rhp_resp_top_scan_kernel, dim3(1), dim3(1024), 0, s, b->work, tiles);
  hipLaunchKernelGGL(rhp_resp_tile_scan_kernel, dim3(tiles), dim3(1024), 0, s, b->out_off, b->n,
                     (const uint64_t *) b->work);
  uint32_t g3 = (b->n + 255u) / 256u;   /* 4 waves per workgroup, a wave per 64 responses */
  if (g3 > cap) g3 = cap;
  hipLaunchKernelGGL(rhp_resp_write_kernel, dim3(g3), dim3(256), 0, s, p);
  return (int) hipGetLastError();
}
