/*
 * rhp_writer.hip -- MI355X (gfx950) batched HTTP/1.1 response serialization.
 *
 * http_write_response (src/reactor/http.c:286-297, with _basic :236-259 and
 * _extended :261-284) for n responses at once, so the reactor's response side can
 * run as one device pass per round like the parse side.
 * Three launches on the caller's stream:
 *
 *   rhp_resp_size_kernel   thread per response: its size, exactly the sum the
 *                          reference allocates (http.c:244-246, 270-272; the date
 *                          is the fixed 29 bytes the "37" there assumes)
 *   rhp_resp_tile_*_kernel reduce-then-scan over 4096-size tiles (tile sums in the
 *                          caller's work[], one workgroup scans those, every tile
 *                          is scanned in place): exclusive prefix sum -> out_off
 *   rhp_resp_write_kernel  wave per response: each segment copied 64 bytes per
 *                          store instruction in the reference's push order
 *                          (http_push_data / http_push_field, http.c:51-69); the
 *                          Content-Length digits as http_u32_sprint (:17-44) prints
 *                          them, one lane per digit
 *
 * Byte copies are HBM-bound; the response bytes written are the algorithmic bytes.
 */
#include <hip/hip_runtime.h>
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

__global__ __launch_bounds__(256) void rhp_resp_size_kernel(WParams p)
{
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x)
    p.out_off[i + 1] = resp_size(p, p.resps[i]);
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

__global__ __launch_bounds__(1024) void rhp_resp_tile_sum_kernel(const uint64_t *a, uint32_t n, uint64_t *work)
{
  __shared__ unsigned long long part[16];
  const uint64_t lo = 1 + (uint64_t) blockIdx.x * kTile, hi = min(lo + kTile, (uint64_t) n + 1);
  unsigned long long s = 0;
  for (uint64_t k = lo + threadIdx.x; k < hi; k += 1024) s += a[k];
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

/* one segment of a response, 64 bytes per store instruction */
__device__ __forceinline__ void put(uint8_t *dst, uint64_t &o, const uint8_t *src, uint32_t len, uint32_t lane)
{
  for (uint32_t j = lane; j < len; j += 64) dst[o + j] = src[j];
  o += len;
}
__device__ __forceinline__ void put_c(uint8_t *dst, uint64_t &o, const char *src, uint32_t len, uint32_t lane)
{
  if (lane < len) dst[o + lane] = (uint8_t) src[lane];
  o += len;
}

__global__ __launch_bounds__(256) void rhp_resp_write_kernel(WParams p)
{
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  if (p.out_off[p.n] > p.out_size) return;   /* does not fit: sizes only (rhp.h) */
  uint8_t *dst = p.out;
  for (uint32_t i = wave; i < p.n; i += nwaves) {
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
}

int g_writer_cus = 0;

}  // namespace

extern "C" int rhp_write_responses(const rhp_resp_batch_t *b, void *stream)
{
  if (!b) return -22;
  if (!b->out_off || !b->date || b->date_len != RHP_DATE_LEN) return -22;
  if (b->n > 0 && (!b->arena || !b->resps)) return -22;
  if (!b->out && b->out_size != 0) return -22;
  if (b->n > 0 && !b->work) return -22;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (g_writer_cus == 0) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&g_writer_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int) e;
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
  const uint32_t cap = (uint32_t) g_writer_cus * 8u;
  uint32_t g1 = (b->n + 255u) / 256u;
  if (g1 > cap) g1 = cap;
  hipLaunchKernelGGL(rhp_resp_size_kernel, dim3(g1), dim3(256), 0, s, p);
  const uint32_t tiles = (b->n + kTile - 1u) / kTile;
  hipLaunchKernelGGL(rhp_resp_tile_sum_kernel, dim3(tiles), dim3(1024), 0, s, b->out_off, b->n, b->work);
  hipLaunchKernelGGL(rhp_resp_top_scan_kernel, dim3(1), dim3(1024), 0, s, b->work, tiles);
  hipLaunchKernelGGL(rhp_resp_tile_scan_kernel, dim3(tiles), dim3(1024), 0, s, b->out_off, b->n,
                     (const uint64_t *) b->work);
  uint32_t g3 = (b->n + 3u) / 4u;   /* 4 waves per workgroup, a wave per response */
  if (g3 > cap * 4u) g3 = cap * 4u;
  hipLaunchKernelGGL(rhp_resp_write_kernel, dim3(g3), dim3(256), 0, s, p);
  return (int) hipGetLastError();
}
