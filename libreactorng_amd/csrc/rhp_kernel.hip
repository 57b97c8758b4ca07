/*
 * rhp_kernel.hip -- MI355X (gfx950) batched HTTP/1.1 request parser.
 *
 * Hot path: phr_parse_request (picohttpparser.c:383-409) and the framing of
 * http_read_request (http.c:177-234) over a batch of independent requests in
 * HBM.  Design:
 *
 *  - one request per lane, 64 requests per wave in flight, every lane runs the
 *    byte DFA of rhp_dfa.h in lockstep: per byte one LDS table read and one LDS
 *    u16 capture write, no divergence on the byte path;
 *  - each lane streams its own request through a 64-byte register window
 *    (4 x global_load_dwordx4), unaligned starts handled by SKIP states;
 *  - persistent waves pull chunks of requests from one atomic counter and hand
 *    requests to idle lanes at 64-byte block boundaries (ragged lengths);
 *  - a request whose outcome depends on where the buffer ends, or that takes a
 *    rare path (rhp_dfa.h S_SLOW), is finished by the exact scalar path
 *    (rhp_scalar.h) on the same lane.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rhp.h"
#include "rhp_dfa.h"
#include "rhp_scalar.h"

namespace {

using namespace rhp;

__device__ const Table g_table = make_table();

struct Params {
  const uint8_t *bytes;
  uint8_t *bytes_rw;
  const uint64_t *offsets;
  rhp_req_t *reqs;
  rhp_hdr_t *hdrs;
  rhp_http_t *http;
  uint32_t *work;
  uint32_t n;
  uint32_t max_headers;
  uint32_t mode;
  uint32_t cap_lane;     /* capture bytes per lane (multiple of 16) */
};

enum : uint32_t { kChunk = 256, kFastMaxLen = RHP_MAX_LEN - 256 };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define RHP_LDS __attribute__((address_space(3)))

/* LDS accessors on raw 32-bit LDS byte addresses */
__device__ __forceinline__ uint32_t lds_load_u32(uint32_t addr)
{
  return *(const RHP_LDS uint32_t *) (size_t) addr;
}
__device__ __forceinline__ void lds_store_u16(uint32_t addr, uint32_t v)
{
  *(RHP_LDS uint16_t *) (size_t) addr = (uint16_t) v;
}
__device__ __forceinline__ uint32_t lds_load_u16(uint32_t addr)
{
  return *(const RHP_LDS uint16_t *) (size_t) addr;
}
__device__ __forceinline__ void lds_store_u32x4(uint32_t addr, u32x4 v)
{
  *(RHP_LDS u32x4 *) (size_t) addr = v;
}

/* 16 bytes at a 4-byte aligned global address */
__device__ __forceinline__ u32x4 load_window16(const uint8_t *p)
{
  typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  return *reinterpret_cast<const u32x4a4 *>(p);
}

/* ---- per-request completion ---- */

/* Exact scalar path for one request (phr or http mode). */
__device__ void finish_exact(const Params &p, uint32_t i, uint64_t off, uint64_t len)
{
  rhp_req_t r;
  r.flags = RHP_F_EXACT;
  rhp_hdr_t *h = p.hdrs + (uint64_t) i * p.max_headers;
  if (len > RHP_MAX_LEN) {
    r.ret = RHP_RET_TOOLONG;
    r.method_len = r.path_off = r.path_len = 0;
    r.method_off = 0; r.minor_version = -1; r.num_headers = 0;
    p.reqs[i] = r;
    if (p.mode == RHP_MODE_HTTP) {
      rhp_http_t x = {0, 0, 0, 0};
      p.http[i] = x;
    }
    return;
  }
  if (p.mode == RHP_MODE_HTTP) {
    rhp_http_t x;
    scalar_http(p.bytes_rw + off, len, p.max_headers, &r, h, &x);
    p.http[i] = x;
  } else {
    scalar_phr(p.bytes + off, len, p.max_headers, &r, h);
  }
  p.reqs[i] = r;
}

/* Decode the lane's capture area into records (DFA decided ret > 0). */
__device__ void finish_fast_ok(const Params &p, uint32_t i, uint64_t off, uint64_t len, uint32_t cap0,
                               uint32_t count, int32_t ret)
{
  rhp_req_t r;
  uint32_t ms = lds_load_u16(cap0 + C_MS), me = lds_load_u16(cap0 + C_ME);
  uint32_t ps = lds_load_u16(cap0 + C_PS), pe = lds_load_u16(cap0 + C_PE);
  uint32_t vd = lds_load_u16(cap0 + C_VD);
  r.ret = ret;
  r.method_off = (uint8_t) ms;
  r.method_len = (uint16_t) (me - ms);
  r.path_off = (uint16_t) ps;
  r.path_len = (uint16_t) (pe - ps);
  r.minor_version = (int8_t) (p.bytes[off + vd] - '0');
  r.num_headers = (uint16_t) count;
  r.flags = 0;
  p.reqs[i] = r;
  rhp_hdr_t *h = p.hdrs + (uint64_t) i * p.max_headers;
  for (uint32_t k = 0; k < count; k++) {
    uint32_t rec = cap0 + kRlBytes + kHdrBytes * k;
    uint32_t ls = lds_load_u16(rec + C_LS), co = lds_load_u16(rec + C_CO);
    uint32_t vs = lds_load_u16(rec + C_VS), ve = lds_load_u16(rec + C_VE);
    rhp_hdr_t o;
    o.name_off = (uint16_t) ls;
    o.name_len = (uint16_t) (co - ls);
    o.value_off = (uint16_t) vs;
    o.value_len = (uint16_t) (ve > vs ? ve - vs : 0);
    h[k] = o;
  }
  if (p.mode == RHP_MODE_HTTP)
    http_frame(p.bytes_rw + off, len, r, h, &p.http[i]);
}

__device__ void finish_fast_bad(const Params &p, uint32_t i)
{
  rhp_req_t r;
  r.ret = -1;
  r.method_len = r.path_off = r.path_len = 0;
  r.method_off = 0; r.minor_version = -1; r.num_headers = 0; r.flags = 0;
  p.reqs[i] = r;
  if (p.mode == RHP_MODE_HTTP) {
    rhp_http_t x = {-1, 0, 0, 0};
    p.http[i] = x;
  }
}

/*
 * Finalize the lane's request after the DFA stopped or ran past `len`.
 * Decision table (rhp_dfa.h header): a terminal decided at byte TERM is the
 * reference's answer iff TERM < len; anything else is re-parsed exactly.
 */
__device__ void finalize(const Params &p, uint32_t i, uint64_t off, uint64_t len, uint32_t st,
                         uint32_t cap0, uint32_t cap)
{
  uint32_t row = entry_next(st);
  uint32_t count = cap == cap0 ? 0u : (cap - cap0 - kRlBytes) / kHdrBytes + 1u;
  uint32_t term = lds_load_u16(cap == cap0 ? cap0 + C_TERM_RL : cap + C_TERM_H);
  if (row == row_of(S_DONE) && term < len) {
    if (count > p.max_headers) finish_fast_bad(p, i);
    else finish_fast_ok(p, i, off, len, cap0, count, (int32_t) term + 1);
  } else if ((row == row_of(S_ERR1) && term < len) || row == row_of(S_OVF)) {
    finish_fast_bad(p, i);
  } else {
    finish_exact(p, i, off, len);
  }
}

}  // namespace

/*
 * The DFA kernel.  One workgroup = WAVES waves; dynamic LDS = table + per-lane
 * capture areas.  Persistent: grid = workgroups resident on the device.
 */
template <int WAVES, int FLAGS>
__global__ __launch_bounds__(WAVES * 64) void rhp_dfa_kernel(Params p)
{
  /* FLAGS bit 0: prefetch the next 64-byte window while the current one is parsed
   * FLAGS bit 1: odd-dword capture stride (conflict-free LDS capture writes) */
  constexpr bool kPrefetch = FLAGS & 1;
  constexpr bool kOddStride = FLAGS & 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t wave = tid >> 6;

  /* stage the transition table into LDS (it sits at LDS address 0) */
  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(&g_table);
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds);
    for (uint32_t k = tid; k < kTableBytes / 16; k += WAVES * 64) dst[k] = src[k];
  }
  __syncthreads();

  const uint32_t lds_base = (uint32_t) (size_t) (RHP_LDS uint8_t *) lds;   /* LDS address of lds[0] */
  const uint32_t cap0 = lds_base + kTableBytes + (wave * 64u + lane) * p.cap_lane;
  /* capture pointer value once max_headers records have started */
  const uint32_t cap_limit = p.max_headers ? cap0 + kRlBytes + kHdrBytes * (p.max_headers - 1) : cap0;

  /* lane state */
  uint32_t st = entry(S_DONE, C_NONE_T);
  uint32_t cap = cap0;
  int32_t pos = 0;
  bool has = false;
  uint32_t req = 0;
  uint64_t off = 0, len = 0;
  const uint8_t *win = p.bytes;

  bool fresh = false;                 /* lane got a new request at this boundary */
  u32x4 wn[4] = {u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}};

  /* wave-uniform pool of requests */
  uint32_t pool_next = 0, pool_end = 0;
  bool pool_dry = false;

  for (;;) {
    /* ---- block boundary: finish lanes that are done or past their end ---- */
    if (has) {
      bool term = is_terminal_row(entry_next(st));
      if (term || pos >= (int32_t) len) {
        finalize(p, req, off, len, st, cap0, cap);
        has = false;
      }
    }
    /* ---- hand requests to idle lanes ---- */
    uint64_t idle = __ballot(!has);
    while (idle && !pool_dry) {
      if (pool_next >= pool_end) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&p.work[0], (uint32_t) kChunk);
        base = __builtin_amdgcn_readfirstlane(base);
        if (base >= p.n) { pool_dry = true; break; }
        pool_next = base;
        pool_end = min(base + (uint32_t) kChunk, p.n);
      }
      uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) idle, 0));
      uint32_t avail = pool_end - pool_next;
      if (!has && rank < avail) {
        req = pool_next + rank;
        off = p.offsets[req];
        len = p.offsets[req + 1] - off;
        has = true;
        uint32_t mis = (uint32_t) off & 3u;
        win = p.bytes + (off - mis);
        pos = -(int32_t) mis;
        uint32_t s0 = mis == 0 ? S_START : mis == 1 ? S_SKIP1 : mis == 2 ? S_SKIP2 : S_SKIP3;
        if (len > kFastMaxLen) s0 = S_SLOW;
        st = entry(s0, C_NONE_RL);
        cap = cap0;
        if (kOddStride) {
          /* only the VE slots must start at 0 (rhp_dfa.h) */
          for (uint32_t b = kRlBytes + C_VE; b + 2 <= p.cap_lane; b += kHdrBytes) lds_store_u16(cap0 + b, 0);
        } else {
          for (uint32_t b = 0; b < p.cap_lane; b += 16) lds_store_u32x4(cap0 + b, u32x4{0, 0, 0, 0});
        }
        fresh = true;
      }
      uint32_t k = (uint32_t) __popcll(idle);
      pool_next += min(k, avail);
      idle = __ballot(!has);
    }
    if (!__ballot(has)) break;

    /* ---- one 64-byte block: 4 sub-blocks of 16 steps ---- */
    u32x4 w[4];
    if (kPrefetch) {
#pragma unroll
      for (int q = 0; q < 4; q++) w[q] = fresh ? load_window16(win + 16 * q) : wn[q];
#pragma unroll
      for (int q = 0; q < 4; q++) wn[q] = has ? load_window16(win + 64 + 16 * q) : u32x4{0, 0, 0, 0};
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) w[q] = has ? load_window16(win + 16 * q) : u32x4{0, 0, 0, 0};
    }
    fresh = false;

#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        uint32_t c = (w[q][k >> 2] >> ((k & 3) * 8)) & 0xffu;
        uint32_t e = lds_load_u32(lds_base + entry_next(st) + c * 4u);
        cap += entry_inc(e);
        lds_store_u16(cap + entry_slot(e), (uint32_t) pos);
        pos++;
        st = e;
      }
      /* header records beyond capacity: stop the lane (rhp_dfa.h cap_bytes) */
      if (__ballot(cap > cap_limit && !is_terminal_row(entry_next(st)))) {
        if (cap > cap_limit && !is_terminal_row(entry_next(st)))
          st = entry(pos <= (int32_t) len ? S_OVF : S_SLOW, C_NONE_T);
      }
    }
    win += 64;
  }

  /* the last workgroup out re-arms the work counters for the next launch, so a
   * step is exactly one kernel launch (no memset) */
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    uint32_t done = atomicAdd(&p.work[1], 1u);
    if (done == gridDim.x - 1) {
      atomicExch(&p.work[0], 0u);
      atomicExch(&p.work[1], 0u);
    }
  }
}

/* Exact-path-only kernel: one request per thread, grid-stride (RHP_IMPL_EXACT). */
__global__ __launch_bounds__(256) void rhp_exact_kernel(Params p)
{
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x) {
    uint64_t off = p.offsets[i];
    finish_exact(p, i, off, p.offsets[i + 1] - off);
  }
}

/* ------------------------------- host C-ABI ------------------------------- */

namespace {
int g_impl = RHP_IMPL_DFA;
int g_cus = 0;
int g_flags = -1;   /* RHP_DFA_FLAGS (experiments); default below */

int dfa_flags()
{
  if (g_flags < 0) {
    const char *e = getenv("RHP_DFA_FLAGS");
    g_flags = e ? (atoi(e) & 3) : 3;
  }
  return g_flags;
}

template <int FLAGS>
int launch_waves(int waves, const Params &prm, size_t lds, hipStream_t s)
{
  switch (waves) {
  case 8: return launch_dfa<8, FLAGS>(prm, lds, s);
  case 4: return launch_dfa<4, FLAGS>(prm, lds, s);
  case 2: return launch_dfa<2, FLAGS>(prm, lds, s);
  default: return launch_dfa<1, FLAGS>(prm, lds, s);
  }
}

template <int WAVES, int FLAGS>
int launch_dfa(const Params &prm, size_t lds_bytes, hipStream_t s)
{
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&rhp_dfa_kernel<WAVES, FLAGS>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int) e;
    attr_set = true;
  }
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rhp_dfa_kernel<WAVES, FLAGS>, WAVES * 64,
                                                               lds_bytes);
  if (e != hipSuccess) return (int) e;
  if (per_cu < 1) per_cu = 1;
  uint32_t grid = (uint32_t) (g_cus * per_cu);
  uint32_t need = (prm.n + 64 * WAVES - 1) / (64 * WAVES);
  if (grid > need) grid = need > 0 ? need : 1;
  hipLaunchKernelGGL((rhp_dfa_kernel<WAVES, FLAGS>), dim3(grid), dim3(WAVES * 64), lds_bytes, s, prm);
  return (int) hipGetLastError();
}
}  // namespace

extern "C" {

const char *rhp_version(void) { return "rhp 0.1.0 (gfx950)"; }

const char *rhp_kernel_name(void) { return g_impl == RHP_IMPL_EXACT ? "rhp_exact_kernel" : "rhp_dfa_kernel"; }

int rhp_set_impl(int impl)
{
  if (impl != RHP_IMPL_DFA && impl != RHP_IMPL_EXACT) return -22;
  g_impl = impl;
  return 0;
}

int rhp_parse_batch(const rhp_batch_t *b, void *stream)
{
  if (!b) return -22;
  if (b->n == 0) return 0;                       /* nothing to parse, nothing touched */
  if (!b->bytes || !b->offsets || !b->reqs || !b->work) return -22;
  if (b->max_headers > RHP_MAX_HEADERS) return -22;
  if (b->max_headers > 0 && !b->hdrs) return -22;
  if (b->mode == RHP_MODE_HTTP && (!b->http || !b->bytes_rw)) return -22;
  if (b->mode != RHP_MODE_PHR && b->mode != RHP_MODE_HTTP) return -22;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (g_cus == 0) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int) e;
  }
  Params prm;
  prm.bytes = b->bytes;
  prm.bytes_rw = b->bytes_rw;
  prm.offsets = b->offsets;
  prm.reqs = b->reqs;
  prm.hdrs = b->hdrs;
  prm.http = b->http;
  prm.work = b->work;
  prm.n = b->n;
  prm.max_headers = b->max_headers;
  prm.mode = b->mode;
  const int flags = dfa_flags();
  prm.cap_lane = (cap_bytes(b->max_headers) + 15u) & ~15u;
  if (flags & 2) prm.cap_lane += 4;      /* odd number of dwords: lanes hit distinct banks */

  if (g_impl == RHP_IMPL_EXACT) {
    uint32_t grid = (b->n + 255) / 256;
    if (grid > (uint32_t) g_cus * 8) grid = (uint32_t) g_cus * 8;
    hipLaunchKernelGGL(rhp_exact_kernel, dim3(grid), dim3(256), 0, s, prm);
    return (int) hipGetLastError();
  }
  const size_t budget = 160 * 1024;
  size_t per_wave = 64 * (size_t) prm.cap_lane;
  for (int waves = 8; waves >= 1; waves >>= 1) {
    size_t lds = kTableBytes + waves * per_wave;
    if (lds > budget) continue;
    switch (flags) {
    case 0: return launch_waves<0>(waves, prm, lds, s);
    case 1: return launch_waves<1>(waves, prm, lds, s);
    case 2: return launch_waves<2>(waves, prm, lds, s);
    default: return launch_waves<3>(waves, prm, lds, s);
    }
  }
  return -12;
}

}  // extern "C"
