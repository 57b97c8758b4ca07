/*
 * rhp_kernel.hip -- MI355X (gfx950) batched HTTP/1.1 request parser.
 *
 * Hot path: phr_parse_request (picohttpparser.c:383-409) and the framing of
 * http_read_request (http.c:177-234) over a batch of independent requests in
 * HBM.  Design:
 *
 *  - one request per lane, 64 requests per wave in flight; every lane runs the
 *    pair DFA of rhp_dfa.h in lockstep, two bytes per table read:
 *        k0, k1 = class[b0], class[b1]               two ds_read_u8, a chunk ahead
 *        a      = v_perm(idx, codes, sel)            = idx * 256 + k0 * 16 + k1
 *        idx    = T2[a]                              one dependent ds_read_u8
 *        ev     = v_alignbit(idx, ev, 2)             low index bits = event bits
 *    no LDS write and no divergence on the byte path; the kernel is bound by
 *    LDS issue;
 *  - lanes stream their request in 128-byte windows = whole HBM lines: the
 *    wave fetches its 64 lanes' next windows with eight LDS-DMA loads (8
 *    lines each) a whole block ahead of use, into a single-buffered staging
 *    area (8 KiB per wave, one 16-wave workgroup per CU); every lane also
 *    holds its NEXT request's offsets, so a request switch never waits on a
 *    dependent load;
 *  - once per block the event masks are decoded, straight-line per event
 *    (or per CO+EOL pair), into the request-line and header records (stored
 *    in 16-byte pairs); in http mode the decode also leaves framing hints
 *    (GET, the Content-Length / Transfer-Encoding candidates);
 *  - a request the table cannot decide alone (S_SLOW, a terminal at/after
 *    len, no terminal by the end of its buffer) and http framing are finished
 *    after the loop by the workgroup's replay (rhp_scalar.h exact path through
 *    a 16-byte line cache; framing from the hints).
 *
 * The algorithm is mirrored block for block by rhp_emu.cpp (CPU tests).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <stdlib.h>
#include <string.h>

#include "rhp.h"
#include "rhp_dfa.h"
#include "rhp_scalar.h"

namespace {

using namespace rhp;

#ifndef RHP_PAIR
#define RHP_PAIR 1   /* 1: pair DFA (rhp_dfa.h Table2), 0: byte DFA (Table8) */
#endif
#define RHP_NT_ALIGNED (-1)
#ifndef RHP_LDS_AUX
#define RHP_LDS_AUX RHP_NT_ALIGNED   /* window load cache policy: 0 normal, 2 nt, -1 nt when line-aligned (issue) */
#endif
#ifndef RHP_ST_NT
#define RHP_ST_NT 0     /* 1: record stores non-temporal */
#endif
#if RHP_ST_NT
#define RHP_ST_POLICY " nt"
#else
#define RHP_ST_POLICY ""
#endif
#ifndef RHP_EARLY
#define RHP_EARLY 0     /* issue the next window before the decode (128-B windows); measured no gain, profiles/r01/v9 */
#endif
#ifndef RHP_PEND2
#define RHP_PEND2 0     /* two pending requests per lane (see promote); measured worse, profiles/r01/v9 */
#endif
#ifndef RHP_CODE2
#define RHP_CODE2 1     /* pair codes by two table lookups (rhp_dfa.h code_row) */
#endif
#ifndef RHP_SKIP
#define RHP_SKIP 0   /* pair DFA: skip chunks of run bytes wave-uniformly (rhp_dfa.h runs_exact); measured no gain, profiles/r01/v9 */
#endif
#if RHP_PAIR
__device__ const Table2 g_table = make_table2();
#define kTableBytes kTable2Bytes
__device__ __forceinline__ constexpr uint32_t start_index(uint32_t s) { return idx2(s, 0); }
__device__ __forceinline__ bool t_slow(uint32_t i) { return is_slow2(i); }
__device__ __forceinline__ bool t_done(uint32_t i) { return is_done2(i); }
__device__ __forceinline__ bool t_err(uint32_t i) { return is_err2(i); }
#else
__device__ const Table8 g_table = make_table8();
#define kTableBytes kTable8Bytes
__device__ __forceinline__ constexpr uint32_t start_index(uint32_t s) { return idx8(s); }
__device__ __forceinline__ bool t_slow(uint32_t i) { return is_slow8(i); }
__device__ __forceinline__ bool t_done(uint32_t i) { return is_done8(i); }
__device__ __forceinline__ bool t_err(uint32_t i) { return is_err8(i); }
#endif

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
  uint32_t span;    /* requests per workgroup */
};

#ifndef RHP_WAVES_PER_SIMD
#define RHP_WAVES_PER_SIMD 8
#endif

enum : uint32_t {
  kBlock = RHP_BLOCK,                            /* window bytes per lane per loop iteration (64 or 128) */
  kParts = kBlock / 16,                          /* 16-byte parts per window */
  kEvWords = kBlock / 32,                        /* 32-bit event words per block */
  kLdsTable = (kTableBytes + 1023u) & ~1023u,   /* staging starts 1 KiB aligned */
  kStageWave = 64 * kBlock,                      /* one window per lane, single-buffered */
  kPark = 0,                                     /* the DONE index: idle lanes step here */
  kDeferExact = 0x8000u,                         /* reqs[i].flags while deferred (kernel-internal) */
  kDeferFrame = 0x4000u,
  /* workgroup pool area after the staging buffers: counters, then the long-
   * request bitmap (ranges up to kOrderSpan requests) and list */
  kPoolWords = 8,                                /* counter, replay flag, list length, list cursor */
  kOrderSpan = 8192,
  kListCap = 1536,
  kPoolBytes = 4 * kPoolWords + kOrderSpan / 8 + 2 * kListCap
};
static_assert(kBlock == 64 || kBlock == 128, "64- or 128-byte windows");
static_assert(!RHP_EARLY || kBlock == 128, "early issue needs whole-line windows");
static_assert(!(RHP_EARLY && RHP_PEND2), "the early issue predicts the single-pend switch");
static_assert(idx2(S_DONE, 0) == kPark && idx8(S_DONE) == kPark, "parked lanes sit in DONE");

/* LDS byte address of part q (16 B) of lane w's window inside the staging
 * buffer.  The LDS-DMA loads of a wave write lane-linearly (1 KiB per
 * instruction), so the swizzle lives on the source side, chosen so that each
 * lane's ds_read_b128 of its own window are bank-conflict free:
 *   64-B windows:  instruction i, lane j fetches part ((j & 3) - (j >> 4)) & 3
 *                  of lane 16i + (j >> 2)'s window (16 windows per load);
 *   128-B windows: instruction i, lane j fetches part ((j & 7) - (w >> 1)) & 7
 *                  of lane w = 8i + (j >> 3)'s window (8 whole 128-B lines per
 *                  load, so every HBM line is fetched by one instruction). */
__device__ __forceinline__ uint32_t stage_off(uint32_t w, uint32_t q)
{
  if (kBlock == 64) {
    const uint32_t u = w & 15u;
    return (w >> 4) * 1024u + u * 64u + ((q + (u >> 2)) & 3u) * 16u;
  }
  return (w >> 3) * 1024u + (w & 7u) * 128u + ((q + (w >> 1)) & 7u) * 16u;
}
__device__ __forceinline__ uint32_t dma_window(uint32_t i, uint32_t j)   /* whose window lane j fetches in load i */
{
  return kBlock == 64 ? 16u * i + (j >> 2) : 8u * i + (j >> 3);
}
__device__ __forceinline__ uint32_t dma_part(uint32_t w, uint32_t j)     /* ... and which 16-byte part of it */
{
  return kBlock == 64 ? ((j & 3u) - (j >> 4)) & 3u : ((j & 7u) - (w >> 1)) & 7u;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#ifdef RHP_CLOCK
/* diagnostic build only: shader ticks and 100 MHz real-time ticks from the
 * entry of the first wave to its exit, written by block 0 wave 0 (never read
 * by the kernel); the quotient is the shader clock the kernel ran at */
__device__ unsigned long long g_clock[2];
#endif
#ifdef RHP_STAMPS
/* diagnostic build only: per-wave cycle sums per loop section (never read by the kernel) */
__device__ unsigned long long g_stamps[8192 * 8];
__device__ unsigned long long g_stamps_end[8192];   /* entry -> end of the replay, per wave */
#define RHP_STAMP(t) do { __builtin_amdgcn_sched_barrier(0); \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory"); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define RHP_STAMP(t) do { } while (0)
#endif

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

/* The exact parser's byte reader on the GPU: the aligned 16-byte line holding
 * the last byte read stays in registers, so its sequential scan makes one
 * global load per 16 bytes (the batch buffer is 16-aligned and padded) */
struct LineBytes {
  const uint8_t *b;
  uint64_t line;
  u32x4_t c;
  __device__ uint32_t operator()(uint64_t p)
  {
    const uint64_t a = (uint64_t) (uintptr_t) b + p;
    const uint64_t l = a & ~(uint64_t) 15;
    if (l != line) {
      c = *reinterpret_cast<const __attribute__((address_space(1))) u32x4_t *>((uintptr_t) l);
      line = l;
    }
    const uint32_t q = (uint32_t) (a >> 2) & 3u;
    const uint32_t d = q == 0 ? c[0] : q == 1 ? c[1] : q == 2 ? c[2] : c[3];
    return (d >> (8u * ((uint32_t) a & 3u))) & 0xffu;
  }
};

/* Exact scalar path for one request (phr or http mode).  Only called from the
 * post-loop replay, where inlining it lets it reuse the loop's dead registers. */
__device__ __forceinline__ void finish_exact(const Params &p, uint32_t i, uint64_t off, uint64_t len)
{
  rhp_req_t r;
  r.flags = RHP_F_EXACT;
  rhp_hdr_t *h = p.hdrs + (uint64_t) i * p.max_headers;
  if (p.mode == RHP_MODE_HTTP) {
    rhp_http_t x;
    LineBytes B{p.bytes_rw + off, ~0ull, {0, 0, 0, 0}};
    scalar_http_t(B, p.bytes_rw + off, len, p.max_headers, &r, h, &x);
    p.http[i] = x;
  } else {
    LineBytes B{p.bytes + off, ~0ull, {0, 0, 0, 0}};
    scalar_phr_t(B, len, p.max_headers, &r, h);
  }
  p.reqs[i] = r;
}

/* 28 bytes at b (any alignment) as 7 dwords, from three aligned 16-byte loads:
 * the replay's scattered per-lane reads then cost 3 load instructions instead
 * of one per byte (the batch buffer is 16-aligned and padded) */
__device__ __forceinline__ void load28(const uint8_t *b, uint32_t (&d)[7])
{
  typedef __attribute__((address_space(1))) const u32x4_t gq;
  const uintptr_t a = (uintptr_t) b, l = a & ~(uintptr_t) 15;
  const u32x4_t q0 = *reinterpret_cast<gq *>(l), q1 = *reinterpret_cast<gq *>(l + 16), q2 = *reinterpret_cast<gq *>(l + 32);
  const uint32_t c[12] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3], q2[0], q2[1], q2[2], q2[3]};
  const uint32_t k = (uint32_t) (a >> 2) & 3u, sh = (uint32_t) a & 3u;
  uint32_t w[8];
#pragma unroll
  for (int m = 0; m < 8; m++) w[m] = k == 0 ? c[m] : k == 1 ? c[m + 1] : k == 2 ? c[m + 2] : c[m + 3];
#pragma unroll
  for (int m = 0; m < 7; m++) d[m] = __builtin_amdgcn_alignbyte(w[m + 1], w[m], sh);
}

/* byte j of a dword array (j constant after unrolling) */
#define RHP_BYTE(d, j) (((d)[(j) >> 2] >> (8 * ((j) & 3))) & 0xffu)

/* Case-insensitive compare of a parsed header name with a lower-case literal
 * of n <= 28 bytes: OR 0x20 folds letters; the one non-letter, '-', could only
 * collide with CR, which a parsed name cannot hold (tchar only) */
template <uint32_t N>
__device__ __forceinline__ bool name_is(const uint8_t *b, const rhp_hdr_t &h, const char (&lit)[N])
{
  constexpr uint32_t n = N - 1;
  if (h.name_off == RHP_NAME_NULL || h.name_len != n) return false;
  uint32_t d[7];
  load28(b + h.name_off, d);
  uint32_t diff = 0;
#pragma unroll
  for (uint32_t j = 0; j < n; j++) diff |= (RHP_BYTE(d, j) | 0x20u) ^ (uint32_t) lit[j];
  return diff == 0;
}

/* strtoull10 (rhp_scalar.h) over a 28-byte register window; the byte walk
 * continues past it only for longer inputs */
__device__ __forceinline__ uint64_t strtoull10_gpu(const uint8_t *s)
{
  uint32_t d[7];
  load28(s, d);
  uint32_t st = 0;
  bool neg = false, ovf = false;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < 28; j++) num_step(RHP_BYTE(d, j), st, neg, ovf, v);
  for (const uint8_t *q = s + 28; st != 2; q++) num_step(*q, st, neg, ovf, v);
  return ovf ? ~0ull : neg ? 0 - v : v;
}

/* http_frame (rhp_scalar.h) for the replay's common case, from the decode's
 * hints (cand, crec: see the decode state) -- GET, no candidate header, or one
 * that is Content-Length or neither; anything else takes http_frame.  Reads no
 * header record and no method byte: on batches larger than the caches those
 * re-reads are HBM traffic. */
__device__ __forceinline__ bool http_frame_fast(const uint8_t *b, uint64_t len, const rhp_req_t &r, rhp_http_t *x,
                                                uint32_t cand, uint32_t crec_lo, uint32_t crec_hi)
{
  const int64_t n = r.ret;
  rhp_http_t o = {1, 0, (uint64_t) n, 0};
  const uint32_t hdr = cand & 0x3fffffffu;
  if (!(cand & 0x40000000u) && hdr != 0) {   /* not GET (http.c:198-202), some candidate */
    if ((cand >> 31) || (hdr & (hdr - 1)) != 0) return false;
    rhp_hdr_t hc;
    hc.name_off = (uint16_t) crec_lo; hc.name_len = (uint16_t) (crec_lo >> 16);
    hc.value_off = (uint16_t) crec_hi; hc.value_len = (uint16_t) (crec_hi >> 16);
    if (name_is(b, hc, "transfer-encoding")) return false;   /* chunked framing: the general path */
    if (name_is(b, hc, "content-length") && hc.value_len != 0) {
      const uint64_t size = strtoull10_gpu(b + hc.value_off);
      if (len < (uint64_t) n + size) {
        o.result = 0; o.consumed = 0;
      } else {
        o.body_kind = 1; o.body_len = size; o.consumed = (uint64_t) n + size;
      }
    }
  }
  *x = o;
  return true;
}

/* http_read_request framing of a request the DFA parsed (http mode only) */
__device__ __forceinline__ void finish_http(const Params &p, uint32_t i, uint64_t off, uint64_t len, rhp_req_t r,
                                            uint32_t cand, uint32_t crec_lo, uint32_t crec_hi)
{
  const rhp_hdr_t *h = p.hdrs + (uint64_t) i * p.max_headers;
  if (http_frame_fast(p.bytes_rw + off, len, r, &p.http[i], cand, crec_lo, crec_hi)) return;
  http_frame(p.bytes_rw + off, len, r, h, &p.http[i], (cand >> 31) ? ~0ull : (uint64_t) (cand & 0x3fffffffu));
}

/* Params pointers are generic in the kernel's view (they sit in a struct);
 * the hot stores go through explicit global-address-space pointers so they are
 * global_store (VM counter only), not flat_store (VM + LGKM). */
#define GLOBAL(T, x) ((__attribute__((address_space(1))) T *) (x))

/* ev = (ev >> 2) | (idx << 30): the two event bits of a pair index (b0 ->
 * bit 30, b1 -> bit 31) into the top of the mask.  Written as asm so the
 * compiler cannot sink the shifts of a block's steps into one chain at its
 * end, which would keep every step's index alive in its own VGPR. */
__device__ __forceinline__ void ev_shift2(uint32_t &ev, uint32_t idx)
{
  asm("v_alignbit_b32 %0, %1, %0, 2" : "+v"(ev) : "v"(idx));
}

/* s_waitcnt vmcnt(0) / lgkmcnt(0).  Kept as inline asm: the builtin form
 * (which the compiler's wait insertion sees, removing its own vmcnt(0) in the
 * request switch) measured 2 % slower on config 2 -- the kernel is bound by
 * LDS issue, not by that wait (profiles/r01/v6) */
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

/* one byte of LDS at address a (the table is at LDS address 0) */
__device__ __forceinline__ uint32_t lds_u8(uint32_t a)
{
  return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t *>((size_t) a);
}

/* a 16-byte header-record pair, or a single record, at 4-byte alignment */
__device__ __forceinline__ void store_pair(rhp_hdr_t *dst, u32x4 v)
{
  typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  *GLOBAL(u32x4a4, dst) = v;
}
/* keep the compiler from sinking the computation of x into a branch */
__device__ __forceinline__ void opaque(uint32_t &x) { asm("" : "+v"(x)); }

/* store_pair for the lanes in `mask` (a ballot), as straight-line code: the
 * decode loop then has no branch the compiler would structurize (which costs
 * exec bookkeeping and register copies per event).  exec is restored before
 * the asm ends; the trailing s_nop covers the store-data read hazard. */
__device__ __forceinline__ void store_pair_lanes(uint64_t mask, rhp_hdr_t *dst, u32x4 v)
{
  uint64_t saved;
  asm volatile("s_mov_b64 %0, exec\n\t"
               "s_mov_b64 exec, %1\n\t"
               "global_store_dwordx4 %2, %3, off" RHP_ST_POLICY "\n\t"
               "s_mov_b64 exec, %0\n\t"
               "s_nop 1"
               : "=&s"(saved)
               : "s"(mask), "v"(dst), "v"(v)
               : "memory");
}
__device__ __forceinline__ void store_one(rhp_hdr_t *dst, u32x2 v)
{
  typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
#if RHP_ST_NT
  __builtin_nontemporal_store(v, GLOBAL(u32x2a4, dst));
#else
  *GLOBAL(u32x2a4, dst) = v;
#endif
}
__device__ __forceinline__ void store_req(rhp_req_t *dst, const rhp_req_t &r)
{
  u32x4 v;
  __builtin_memcpy(&v, &r, sizeof r);
#if RHP_ST_NT
  __builtin_nontemporal_store(v, GLOBAL(u32x4, dst));
#else
  *GLOBAL(u32x4, dst) = v;
#endif
}
__device__ __forceinline__ void store_http_bad(rhp_http_t *dst)
{
  /* {result -1, body_kind 0, consumed 0, body_len 0} */
  typedef uint32_t u32x2a8 __attribute__((ext_vector_type(2), aligned(8)));
  __attribute__((address_space(1))) u32x2a8 *q = GLOBAL(u32x2a8, dst);
  q[0] = u32x2a8{0xffffffffu, 0u};
  q[1] = u32x2a8{0u, 0u};
  q[2] = u32x2a8{0u, 0u};
}

}  // namespace

/*
 * The DFA kernel.  One workgroup = WAVES waves sharing one LDS copy of the
 * table.  Persistent: grid = workgroups resident on the device.
 */
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64, RHP_WAVES_PER_SIMD) void rhp_dfa_kernel(Params p)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
#ifdef RHP_CLOCK
  const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef RHP_STAMPS
  const uint32_t wave = tid >> 6;
  unsigned long long t_entry = 0;
  RHP_STAMP(t_entry);
#endif

  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(&g_table);
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds);
    for (uint32_t k = tid; k < kTableBytes / 16; k += WAVES * 64) dst[k] = src[k];
    /* pool counters and the long-request bitmap start at zero */
    for (uint32_t k = tid; k < kPoolWords + kOrderSpan / 32; k += WAVES * 64)
      reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave)[k] = 0;
  }
  __syncthreads();

  const uint32_t maxh = p.max_headers;

  /* ---- request pool ----
   * Workgroup g owns requests [g*span, (g+1)*span) (host: span = n / grid).
   * Lanes that need their next request take it from the workgroup's LDS
   * counter (one atomic per wave and refill, for all of the wave's lanes that
   * need one), so the waves of a workgroup drain one shared range request by
   * request and finish together; no global atomic is ever touched.
   * Window addresses are u32 byte offsets from `base` (the 4-aligned start of
   * the range; the host keeps a batch below 4 GiB). */
  const uint32_t wg_lo = min(blockIdx.x * p.span, p.n), wg_hi = min(wg_lo + p.span, p.n);
  uint32_t *wg_counter = reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave);
  uint32_t *wg_deferred = wg_counter + 1;   /* some request of the range needs the replay */
  /* Long requests first.  With lengths as uneven as config 3's, the requests
   * drawn last decide when a wave finishes; the first iteration (which only
   * waits for the first windows) lists the range's requests longer than twice
   * its mean, and refills hand those out before the rest (simulated: -20 %
   * wave-iterations on config 3).  Ranges above kOrderSpan keep plain order. */
  uint32_t *list_n = wg_counter + 2, *list_next = wg_counter + 3;
  uint32_t *long_bits = wg_counter + kPoolWords;
  uint16_t *long_list = reinterpret_cast<uint16_t *>(long_bits + kOrderSpan / 32);
#ifdef RHP_NO_ORDER   /* experiment: plain range order */
  const bool order_on = false;
#else
  const bool order_on = wg_hi - wg_lo <= kOrderSpan;
#endif
  bool list_dry = !order_on;
  bool first_iter = true;   /* the list is complete only after the scan (before the loop) */
  bool pool_dry = wg_lo >= wg_hi;
  const uint64_t base = pool_dry ? 0 : (p.offsets[wg_lo] & ~(uint64_t) 3);
  const uint8_t *wbytes = p.bytes + base;

  /* ---- lane state ---- */
  uint32_t st = kPark;                 /* table index (rhp_dfa.h idx2 / idx8) */
  int32_t pos = 0;                     /* request-relative position of the next byte to step */
  uint32_t ev[kEvWords];               /* events of the block just stepped (32 bytes per word) */
#pragma unroll
  for (int w = 0; w < (int) kEvWords; w++) ev[w] = 0;
  bool has = false;                    /* cur is being parsed */
  uint32_t cur = 0, cur_len = 0, cur_ptr = 0;   /* cur_ptr: window of the block being stepped */
  /* event decoder state of cur (the records of rhp_dfa.h dec_event, built
   * incrementally: every event at p yields part = A | (p - B) << 16):
   *   kn  = k | minor << 3 | nh << 8   events consumed (0..2 request line:
   *                           ME, PE, RL; then 3,4 = CO, EOL), minor version,
   *                           headers done
   *   A,B the anchors of the next event: at PE (A, B) = (ME, ME + 1), so part
   *       = the request-line record; at CO (line start, line start), so part
   *       = name_off | name_len << 16; at EOL (CO + 2, CO + 3), so part =
   *       value_off | value_len << 16
   *   ovf = 0, or 1 + the line start at which max_headers overflowed
   *   rl  = method_len | path_len << 16
   *   cur_lo: name part of the line in progress; rec_lo/rec_hi: the odd
   *   header record waiting for its pair (16-byte stores) */
  uint32_t kn = 0, A = 0, B = 0, ovf = 0, rl = 0, cur_lo = 0;
  /* http mode, framing hints for the replay: cand bits 0..29 = headers whose
   * name length is 14 or 17 (bit 31: such a header at index >= 30), bit 30 =
   * the method is GET; crec = the first such header's record */
  uint32_t cand = 0, crec_lo = 0, crec_hi = 0;
  uint32_t rec_lo = 0, rec_hi = 0;
  bool pend_ok = false;                /* pend: the lane's next request */
  uint32_t pend = 0;
  uint32_t pend_o0 = 0, pend_o1 = 0;   /* low dwords of offsets[pend], offsets[pend+1] as loaded */
#if RHP_PEND2
  /* a second pending request behind pend: refills fill `back`, and a switch
   * promotes it to pend at once, its offsets loaded an iteration earlier, so a
   * lane whose request fits one window starts the next one's window right away
   * instead of idling an iteration while the new pend's offsets arrive */
  bool back_ok = false;
  uint32_t back = 0, back_o0 = 0, back_o1 = 0;
#define RHP_SLOT_OK back_ok
#else
#define RHP_SLOT_OK pend_ok
#endif
  uint32_t nw = 0;                     /* next window: byte offset from base | kind (0 none, 1
                                          continuation, 2 first window of pend); windows are 4-aligned */
  /* the window in registers: half of a 64-B window (the other half is read
   * midway), or a whole 128-B window */
  constexpr int kWRegs = kBlock == 64 ? 2 : 8;
  u32x4 W[kWRegs];
  const uint32_t stage = kLdsTable + (tid >> 6) * kStageWave;

  /* give every lane without a pending request one from the pool; the offsets
   * loads are only consumed at the top of the next block */
  auto take = [&](uint32_t i) {
    /* only the low dwords: a batch is below 4 GiB, so offsets relative to
     * `base` and lengths are exact modulo 2^32 */
    const uint32_t *o = reinterpret_cast<const uint32_t *>(p.offsets + i);
#if RHP_PEND2
    back = i;
    back_o0 = *GLOBAL(const uint32_t, o);
    back_o1 = *GLOBAL(const uint32_t, o + 2);
    back_ok = true;
#else
    pend = i;
    pend_o0 = *GLOBAL(const uint32_t, o);
    pend_o1 = *GLOBAL(const uint32_t, o + 2);
    pend_ok = true;
#endif
  };
  /* back -> pend (RHP_PEND2); call only after a wait_vm0 that covers back's loads */
  auto promote = [&]() {
#if RHP_PEND2
    if (!pend_ok && back_ok) {
      pend = back;
      pend_o0 = back_o0;
      pend_o1 = back_o1;
      pend_ok = true;
      back_ok = false;
    }
#endif
  };
  auto refill_pend = [&]() {
    uint64_t want = __ballot(!RHP_SLOT_OK);
    if (!want || (pool_dry && list_dry)) return;
    if (!list_dry && !first_iter) {   /* the long list first */
      const uint32_t cnt = (uint32_t) __popcll(want);
      uint32_t b0 = 0;
      if (lane == 0) b0 = atomicAdd(list_next, cnt);
      b0 = __builtin_amdgcn_readfirstlane(b0);
      const uint32_t nl = min(*list_n, (uint32_t) kListCap);
      if (b0 + cnt >= nl) list_dry = true;
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) want, 0));
      if (!RHP_SLOT_OK && b0 + rank < nl) take(wg_lo + long_list[b0 + rank]);
      want = __ballot(!RHP_SLOT_OK);
    }
    /* the range in order, skipping the listed requests (a few rounds at most) */
    while (want && !pool_dry) {
      const uint32_t cnt = (uint32_t) __popcll(want);
      uint32_t b0 = 0;
      if (lane == 0) b0 = atomicAdd(wg_counter, cnt);
      b0 = wg_lo + __builtin_amdgcn_readfirstlane(b0);
      if (b0 + cnt >= wg_hi) pool_dry = true;
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) want, 0));
      const uint32_t i = b0 + rank, k = i - wg_lo;
      if (!RHP_SLOT_OK && i < wg_hi && !(order_on && ((long_bits[k >> 5] >> (k & 31)) & 1u))) take(i);
      want = __ballot(!RHP_SLOT_OK);
    }
  };

  /* the long-request scan (see order_on), once, over the part of the range the
   * first refill did not hand out */
  auto scan_long = [&]() {
    const uint32_t span_n = wg_hi - wg_lo, first_n = min(span_n, (uint32_t) (WAVES * 64));
    if (span_n <= first_n) return;
    /* long: length * count > 2 * the range's bytes (no division) */
    const uint64_t twice = 2u * (p.offsets[wg_hi] - p.offsets[wg_lo]);
    /* a wave scans its slice only if its own first requests (offsets already
     * loaded) include a long one: uniform batches skip the scan */
    if (!__ballot(pend_ok && (uint64_t) (pend_o1 - pend_o0) * span_n > twice)) return;
    for (uint32_t k = first_n + tid; k < span_n; k += WAVES * 64) {
      const uint64_t o0 = p.offsets[wg_lo + k], o1 = p.offsets[wg_lo + k + 1];
      if ((o1 - o0) * span_n > twice) {
        const uint32_t at = atomicAdd(list_n, 1u);
        if (at < kListCap) {
          long_list[at] = (uint16_t) k;
          atomicOr(&long_bits[k >> 5], 1u << (k & 31));
        }
      }
    }
  };

  /* one non-terminal event at request position ep (rhp_dfa.h dec_event), for
   * a lane with an event: straight-line selects, one store branch.  The
   * max_headers check (picohttpparser.c:281-284) fires at the CO of a line
   * that starts while nh == maxh; decoding stops there (m = 0), so nh never
   * exceeds maxh and every completed record is stored. */
  auto event = [&](auto &w, uint32_t base, rhp_hdr_t *hout) {
    /* the lowest event of the mask w (lanes with w == 0 change nothing), and
     * the next one: a header line whose CO and EOL both lie in w is taken in
     * one iteration */
    const bool v = w != 0;
    auto ctz = [](auto x) -> uint32_t {
      return (uint32_t) (sizeof(x) == 8 ? __builtin_ctzll((uint64_t) x) : __builtin_ctz((uint32_t) x));
    };
    const uint32_t ep = base + ctz(w);
    auto w1 = w & (w - 1u);
    const uint32_t ep1 = base + ctz(w1);
    const uint32_t k = v ? kn & 7u : 7u;   /* 7: no event */
    const uint32_t part = A | ((ep - B) << 16);
    /* request line (once per request, so behind a uniform branch) -- ME:
     * (A, B) = (ME, ME + 1);  PE: rl = part, A = B = the first line start
     * (PE + 11);  RL: minor = RL - PE - 9 = ep - B + 2 */
    if (__builtin_amdgcn_ballot_w64(k < 3u)) {
      const bool r0 = k == 0u, r1 = k == 1u, r2 = k == 2u;
      uint32_t a0 = ep + 1u, a1 = ep + 11u, mv = ((ep - B + 2u) & 1u) << 3;
      opaque(a0); opaque(a1); opaque(mv);
      rl = r1 ? part : rl;
      kn += r2 ? mv + 1u : (r0 || r1) ? 1u : 0u;
      A = r0 ? ep : r1 ? a1 : A;
      B = r0 ? a0 : r1 ? a1 : B;
    }
    /* header line: CO (k = 3) -> name part, anchors (CO + 2, CO + 3);
     * EOL (k = 4) -> value part, record complete, anchors = the next line start;
     * pair: CO and EOL of one line (below the max_headers capacity) */
    const bool atmax = (kn >> 8) == maxh;
    const bool pair = k == 3u && w1 != 0 && !atmax;
    const bool co = k == 3u && !pair, eol = k == 4u;
    if (__builtin_amdgcn_ballot_w64(co && atmax)) {   /* max_headers check at the line start: stop */
      const bool ov = co && atmax;
      uint32_t o = A + 1u;
      opaque(o);
      ovf = ov ? o : ovf;
      w1 = ov ? 0 : w1;
    }
    uint32_t c2 = ep + 2u, c3 = ep + 3u, e1 = ep + 1u, p1 = c2 | ((ep1 - c3) << 16), f1 = ep1 + 1u;
    opaque(c2); opaque(c3); opaque(e1); opaque(p1); opaque(f1);
    const bool done = pair || eol;              /* a record completes */
    const uint32_t r_lo = pair ? part : cur_lo, r_hi = pair ? p1 : part;
    cur_lo = co ? part : cur_lo;
    kn += co ? 1u : eol ? 255u : pair ? 256u : 0u;
    A = co ? c2 : eol ? e1 : pair ? f1 : A;
    B = co ? c3 : eol ? e1 : pair ? f1 : B;
    w = pair ? w1 & (w1 - 1u) : w1;
    const bool odd = (kn & 256u) != 0;
    if (p.mode == RHP_MODE_HTTP) {   /* uniform: framing candidates only in http mode */
      const uint32_t nlen = r_lo >> 16, hidx = (kn >> 8) - 1u;
      const bool cnd = done && (nlen == 14u || nlen == 17u);
      const bool first = cnd && (cand & 0xbfffffffu) == 0;
      crec_lo = first ? r_lo : crec_lo;
      crec_hi = first ? r_hi : crec_hi;
      cand |= cnd ? (hidx < 30u ? 1u << hidx : 0x80000000u) : 0u;
    }
    rec_lo = done && odd ? r_lo : rec_lo;
    rec_hi = done && odd ? r_hi : rec_hi;
    const uint64_t st_m = __builtin_amdgcn_ballot_w64(done && !odd);
    if (st_m) store_pair_lanes(st_m, hout + (kn >> 8) - 2u, u32x4{rec_lo, rec_hi, r_lo, r_hi});
  };

  /*
   * Decode the block's events and finalize cur when its outcome is known
   * (decisions mirrored by rhp_emu.cpp):
   *   ok    DONE at term < len
   *   bad   ERR at term < len, or max_headers overflow at a line start < len
   *   exact SLOW, a terminal at/after len, or no terminal by the end of the buffer
   */
  auto decode = [&]() {
    if (!has) return;
    const uint32_t e = st;
    const bool slow = t_slow(e);
    const bool term_ev = t_done(e) || t_err(e);
    const int32_t block_pos = pos - (int32_t) kBlock;
    uint64_t mh[kEvWords / 2];
#pragma unroll
    for (int h = 0; h < (int) kEvWords / 2; h++) mh[h] = slow ? 0ull : (((uint64_t) ev[2 * h + 1] << 32) | ev[2 * h]);
#ifdef RHP_EXP_NODECODE   /* timing experiment: only the terminal is taken from the mask (records left unwritten) */
    if (!term_ev) {
#pragma unroll
      for (int h = 0; h < (int) kEvWords / 2; h++) mh[h] = 0;
    }
#endif
    uint32_t term_pos = 0xffffffffu;
    if (term_ev) {   /* the terminal is the block's last event: take it off the mask */
      bool found = false;
#pragma unroll
      for (int h = (int) kEvWords / 2 - 1; h >= 0; h--) {
        if (!found && mh[h]) {
          const uint32_t bt = 63u - (uint32_t) __builtin_clzll(mh[h]);
          term_pos = (uint32_t) (block_pos + 64 * h + (int32_t) bt);
          mh[h] &= ~(1ull << bt);
          found = true;
        }
      }
    }
    rhp_hdr_t *hout = p.hdrs + (uint64_t) cur * maxh;
#ifdef RHP_EXP_NODECODE
#pragma unroll
    for (int h = 0; h < (int) kEvWords / 2; h++) mh[h] = 0;
#endif
#ifdef RHP_DEC32   /* 32-bit event words (experiment) */
#pragma unroll
    for (int q = 0; q < (int) kEvWords; q++) {
      uint32_t w = ovf ? 0u : (uint32_t) (mh[q >> 1] >> (32 * (q & 1)));
      const uint32_t base = (uint32_t) (block_pos + 32 * q);
      if (__ballot(w != 0)) do event(w, base, hout); while (__ballot(w != 0));
    }
#else              /* 64-bit halves: fewer iterations when events are dense */
#pragma unroll
    for (int h = 0; h < (int) kEvWords / 2; h++) {
      uint64_t w = ovf ? 0ull : mh[h];
      const uint32_t base = (uint32_t) (block_pos + 64 * h);
      if (__ballot(w != 0)) do event(w, base, hout); while (__ballot(w != 0));
    }
#endif
    const uint32_t ovf_at = ovf;
    const bool ovfl = ovf_at != 0;
    const bool fin = ovfl || slow || term_ev || (uint32_t) pos >= cur_len;
    if (!fin) return;
    /* a header section the u16 records cannot hold (ret > RHP_MAX_LEN) is left
     * to the exact path, which answers RHP_RET_TOOLONG */
    const bool ok = !ovfl && t_done(e) && term_pos < cur_len && term_pos < RHP_MAX_LEN;
    const bool bad = ovfl ? ovf_at - 1u < cur_len : (t_err(e) && term_pos < cur_len);
    rhp_req_t r = {};
    r.minor_version = -1;
    if (ok) {
      const uint32_t nh = kn >> 8;
      if (nh & 1u) store_one(hout + nh - 1u, u32x2{rec_lo, rec_hi});
      r.ret = (int32_t) term_pos + 1;
      r.method_len = (uint16_t) rl;
      r.path_off = (uint16_t) (rl + 1u);
      r.path_len = (uint16_t) (rl >> 16);
      r.minor_version = (int8_t) ((kn >> 3) & 1u);
      r.num_headers = (uint16_t) nh;
      r.flags = p.mode == RHP_MODE_HTTP ? (uint16_t) kDeferFrame : (uint16_t) 0;   /* framing: replay */
      if (p.mode == RHP_MODE_HTTP) {
        *wg_deferred = 1u;
        /* framing hints for the replay, in the record it will overwrite */
        typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
        *GLOBAL(u32x4a4, &p.http[cur]) = u32x4a4{cand, 0u, crec_lo, crec_hi};
      }
    } else if (bad) {
      r.ret = -1;
      if (p.mode == RHP_MODE_HTTP) store_http_bad(p.http + cur);
    } else {
      r.flags = (uint16_t) kDeferExact;   /* exact path: replay */
      *wg_deferred = 1u;
    }
    store_req(p.reqs + cur, r);
    has = false;
    st = kPark;
  };

  /* The table sits at LDS address 0, so a v_perm result is the address itself.
   * classes16: the byte classes of a 16-byte chunk (16 independent reads of
   * the class row); codes: pair codes class(b0)*16 + class(b1), two per dword;
   * steps16: 8 chained pair steps, two event bits each shifted into ev. */
  auto classes16 = [&](const u32x4 &chunk, uint32_t (&k)[16]) {
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int b = 0; b < 4; b++)
        k[4 * q + b] = lds_u8(__builtin_amdgcn_perm(kClassRow, chunk[q], 0x0c0c0400u | (uint32_t) b));
  };
  auto codes = [&](const uint32_t (&k)[16], uint32_t (&pc)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++)
      pc[q] = ((k[4 * q] << 4) | k[4 * q + 1]) | (((k[4 * q + 2] << 4) | k[4 * q + 3]) << 8);
  };
  auto steps16 = [&](const uint32_t (&pc)[4], uint32_t &ev) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int j = 0; j < 2; j++) {
        st = lds_u8(__builtin_amdgcn_perm(st, pc[q], 0x0c0c0400u | (uint32_t) j));
        ev_shift2(ev, st);
      }
    }
  };
  /* a window's 16-byte chunks: the class reads of chunk q+1 are issued before
   * the chained steps of chunk q, so their latency hides behind the chain */
#if !RHP_PAIR
  /* byte DFA: 16 chained steps per chunk, one event bit each */
  auto steps_chunks = [&](const u32x4 *Wc, int nchunks, uint32_t *evw) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (q >= nchunks) break;
#pragma unroll
      for (int d = 0; d < 4; d++) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          st = lds_u8(__builtin_amdgcn_perm(st, Wc[q][d], 0x0c0c0400u | (uint32_t) b));
          asm("v_alignbit_b32 %0, %1, %0, 1" : "+v"(evw[q >> 1]) : "v"(st));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
#elif RHP_CODE2
  /* pair codes by two lookups (rhp_dfa.h code_row): A = the row of class(b1),
   * B = class(b0) * 16 + class(b1) from that row; 2 VALU per pair for the codes
   * instead of 2 class addresses + 2 packing ops.  Chunk q+1's A reads are issued
   * before chunk q's chain, its B reads (which wait on A) after half the chain. */
  auto codes_a = [&](const u32x4 &chunk, uint32_t (&r)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      r[j] = lds_u8(__builtin_amdgcn_perm(kClassRowR, chunk[j >> 1], 0x0c0c0400u | (uint32_t) (2 * (j & 1) + 1)));
  };
  auto codes_b = [&](const u32x4 &chunk, const uint32_t (&r)[8], uint32_t (&c)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      c[j] = lds_u8(__builtin_amdgcn_perm(r[j], chunk[j >> 1], 0x0c0c0400u | (uint32_t) (2 * (j & 1))));
  };
  auto steps4 = [&](const uint32_t (&c)[8], int j0, uint32_t &ev) {
#pragma unroll
    for (int j = j0; j < j0 + 4; j++) {
      st = lds_u8(__builtin_amdgcn_perm(st, c[j], 0x0c0c0400u));
      ev_shift2(ev, st);
    }
  };
#if RHP_SKIP
  /* run skipping (see the RHP_SKIP form below) on the two-lookup codes */
  auto run16 = [&](const u32x4 &c) -> bool {
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t x = c[d], y = x ^ 0x7f7f7f7fu;
      acc |= ((x - 0x21212121u) & ~x) | ((y - 0x01010101u) & ~y);
    }
    return (acc & 0x80808080u) == 0;
  };
  auto steps_chunks = [&](const u32x4 *Wc, int nchunks, uint32_t *evw) {
    uint32_t c[8], r[8];
    bool ahead = false;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (q >= nchunks) break;
      const uint32_t s = st & ~1u;
      const bool in_run = s == 4u * S_PATH || s == 4u * S_VALUE || s == 4u * S_VWS;
      if (!__builtin_amdgcn_ballot_w64(!in_run) && !__builtin_amdgcn_ballot_w64(!run16(Wc[q]))) {
        st = s == 4u * S_PATH ? 4u * S_PATH : 4u * S_VALUE;
        evw[q >> 1] >>= 16;
        ahead = false;
        continue;
      }
      if (!ahead) {
        codes_a(Wc[q], r);
        codes_b(Wc[q], r, c);
      }
      uint32_t cn[8];
      if (q + 1 < nchunks) codes_a(Wc[q + 1], r);
      __builtin_amdgcn_sched_barrier(0);
      steps4(c, 0, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < nchunks) codes_b(Wc[q + 1], r, cn);
      __builtin_amdgcn_sched_barrier(0);
      steps4(c, 4, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < nchunks) {
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = cn[j];
      }
      ahead = q + 1 < nchunks;
    }
  };
#else
  auto steps_chunks = [&](const u32x4 *Wc, int nchunks, uint32_t *evw) {
    uint32_t c[8], r[8];
    codes_a(Wc[0], r);
    codes_b(Wc[0], r, c);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (q >= nchunks) break;
      uint32_t cn[8];
      if (q + 1 < nchunks) codes_a(Wc[q + 1], r);
      __builtin_amdgcn_sched_barrier(0);
      steps4(c, 0, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < nchunks) codes_b(Wc[q + 1], r, cn);
      __builtin_amdgcn_sched_barrier(0);
      steps4(c, 4, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < nchunks) {
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = cn[j];
      }
    }
  };
#endif
#elif RHP_SKIP
  /* 16 bytes are all run bytes (rhp_dfa.h c_run: > 0x20 and not DEL).  SWAR,
   * exact as an existence test: (x - 0x21..) & ~x has a byte's top bit set for
   * the lowest byte below 0x21 (bytes >= 0x80 are masked by ~x and borrow
   * nothing), and likewise for the zero bytes of x ^ 0x7f.. (DEL) */
  auto run16 = [&](const u32x4 &c) -> bool {
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t x = c[d], y = x ^ 0x7f7f7f7fu;
      acc |= ((x - 0x21212121u) & ~x) | ((y - 0x01010101u) & ~y);
    }
    return (acc & 0x80808080u) == 0;
  };
  /* Chunks whose bytes keep every busy lane of the wave in a run state
   * (S_PATH, S_VALUE, S_VWS) are skipped (rhp_dfa.h runs_exact): the state
   * becomes the run's plain index and the chunk's 16 event bits are zero.
   * The class reads of chunk q+1 are issued ahead (during chunk q's chain)
   * unless chunk q was skipped: inside a run the next chunk is likely skipped
   * too, and its reads would be wasted. */
  auto steps_chunks = [&](const u32x4 *Wc, int nchunks, uint32_t *evw) {
    uint32_t k[16], pc[4];
    bool ahead = false;   /* k holds the classes of chunk q */
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (q >= nchunks) break;
      const uint32_t s = st & ~1u;   /* plain row (e = 0 or 1) */
      const bool in_run = s == 4u * S_PATH || s == 4u * S_VALUE || s == 4u * S_VWS;
      if (!__builtin_amdgcn_ballot_w64(!in_run) && !__builtin_amdgcn_ballot_w64(!run16(Wc[q]))) {
        st = s == 4u * S_PATH ? 4u * S_PATH : 4u * S_VALUE;
        evw[q >> 1] >>= 16;
        ahead = false;
        continue;
      }
      if (!ahead) classes16(Wc[q], k);
      codes(k, pc);
      if (q + 1 < nchunks) classes16(Wc[q + 1], k);
      ahead = q + 1 < nchunks;
      __builtin_amdgcn_sched_barrier(0);
      steps16(pc, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#else
  auto steps_chunks = [&](const u32x4 *Wc, int nchunks, uint32_t *evw) {
    uint32_t k[16], pc[4];
    classes16(Wc[0], k);
    codes(k, pc);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (q >= nchunks) break;
      if (q + 1 < nchunks) classes16(Wc[q + 1], k);
      __builtin_amdgcn_sched_barrier(0);
      steps16(pc, evw[q >> 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < nchunks) codes(k, pc);
    }
  };
#endif

  /* LDS-DMA of every lane's next window (nw) into the staging buffer:
   * kParts loads of 1 KiB (see stage_off) */
  auto issue = [&]() {
    /* all shuffles first (one LDS round trip for the lot), then the loads; a
     * lane without a next window fetches the range's first bytes instead (its
     * staging slot is not read), so no load needs a branch */
    const uint32_t src = (nw & 3u) ? (nw & ~3u) : 0u;
    uint32_t a[kParts];
#pragma unroll
    for (int i = 0; i < (int) kParts; i++) {
      a[i] = (uint32_t) __shfl((int) src, (int) dma_window((uint32_t) i, lane));
#ifdef RHP_EXP_HOTWIN   /* timing experiment (config 2 only): every request reads its range's first request */
      a[i] &= 255u;
#endif
    }
#if RHP_LDS_AUX == RHP_NT_ALIGNED
    /* Cache policy per wave and window: when every window is one whole HBM
     * line (line-aligned requests), no line is read by two windows and the
     * loads go non-temporal (config 2 +19 %, config 5 +9 %); windows that
     * straddle lines share their edge lines with the neighbouring requests'
     * windows, which then hit in L2 (non-temporal: config 3 -5 %) */
    const bool aligned = !(nw & 3u) || ((uint32_t) (uintptr_t) (wbytes + src) & (kBlock - 1u)) == 0;
    const bool nt = !__builtin_amdgcn_ballot_w64(!aligned);
#else
    constexpr bool nt = RHP_LDS_AUX == 2;
#endif
#pragma unroll
    for (int i = 0; i < (int) kParts; i++) {
      const uint32_t part = dma_part(dma_window((uint32_t) i, lane), lane);
      const void *g = reinterpret_cast<const void *>(wbytes + a[i] + 16u * part);
      __attribute__((address_space(3))) void *l = (__attribute__((address_space(3))) void *) (lds + stage + 1024u * i);
      if (nt) __builtin_amdgcn_global_load_lds(g, l, 16, 0, 2);
      else __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
    }
  };

  refill_pend();
  /* The first iteration, peeled: there is no block to decode or switch yet.
   * Issue the first windows, then (while they land) the long-request scan; the
   * barrier makes the list complete before any wave's next refill. */
  wait_vm0();   /* the pending offsets */
  promote();
  nw = pend_ok ? ((pend_o0 & ~3u) - (uint32_t) base) | 2u : 0u;
  issue();
  if (order_on) scan_long();
  __syncthreads();
  first_iter = false;
#if RHP_PEND2
  refill_pend();   /* back, after the long list is complete */
#endif

#ifdef RHP_STAMPS
  unsigned long long t0 = 0, t1 = 0, acc[6] = {0, 0, 0, 0, 0, 0}, t_loop = 0;
  RHP_STAMP(t_loop);
#endif
  /*
   * One iteration = one 64-byte window per lane.
   * [A] take the loads issued one block earlier (window, pending offsets): the
   * loop's only VMEM wait -> [B] decode + finalize the previous block (its
   * stores are older than any load the next [A] waits for) -> [C] switch to the
   * landed window -> [D] hand out pending requests -> [E] issue the next
   * window's loads into the buffer [A] just read -> 64 DFA steps.
   */
  for (;;) {
    RHP_STAMP(t0);
    /* [A] */
    wait_vm0();   /* the window's LDS-DMA has landed (and the pending offsets) */
    const uint32_t p_o0 = pend_o0, p_o1 = pend_o1;
#pragma unroll
    for (int q = 0; q < kWRegs; q++) W[q] = *reinterpret_cast<const u32x4 *>(lds + stage + stage_off(lane, q));
    const uint32_t nw_in = nw;   /* the window now in W */
#if RHP_EARLY
    /* [E] early: the next window is issued before the decode and the switch,
     * so a wave has loads in flight through them as well as through its walk.
     * The switch and finalize are predicted from what is known already: W is
     * pend's first window (kind 2) -> pend's second window if it has one;
     * otherwise cur continues unless its state is terminal (the decode's
     * max_headers stop is the one outcome not foreseen: that lane loads one
     * unused window) -> else the first window of a pend assigned earlier. */
    {
      const uint32_t k = nw_in & 3u;
      uint32_t nn = 0;
      if (k == 2) {
        const uint32_t mis = p_o0 & 3u;
        if (kBlock - mis < p_o1 - p_o0) nn = ((nw_in & ~3u) + kBlock) | 1u;
      } else {
        const bool live = k == 1 && has && !t_done(st) && !t_err(st) && !t_slow(st);
        if (live && (uint32_t) (pos + (int32_t) kBlock) < cur_len) nn = ((nw_in & ~3u) + kBlock) | 1u;
        else if (pend_ok) nn = ((p_o0 & ~3u) - (uint32_t) base) | 2u;
      }
      nw = nn;
      wait_lgkm0();   /* the reads of the buffer above are done */
      issue();
    }
#endif
#ifdef RHP_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RHP_STAMP(t1); acc[0] += t1 - t0; t0 = t1;
#endif
    /* [B] */
    decode();
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[1] += t1 - t0; t0 = t1;
#endif
    /* [C] */
    const uint32_t nw_kind = nw_in & 3u;
    if (nw_kind == 2) {
      cur = pend;
      cur_len = p_o1 - p_o0;
      pend_ok = false;
      has = true;
      const uint32_t mis = (uint32_t) p_o0 & 3u;
      uint32_t s0 = mis == 0 ? S_METHOD0 : mis == 1 ? S_SKIP1 : mis == 2 ? S_SKIP2 : S_SKIP3;
      st = start_index(s0);
      pos = -(int32_t) mis;
      kn = A = B = ovf = rl = 0;
      /* GET: the request's first four bytes are "GET " (the DFA path parses
       * the method from byte 0), read from the window already in registers */
      const uint32_t head = __builtin_amdgcn_alignbyte(W[0][1], W[0][0], mis);
      cand = head == ('G' | 'E' << 8 | 'T' << 16 | (uint32_t) ' ' << 24) ? 0x40000000u : 0u;
    }
    if (nw_kind) cur_ptr = nw_in & ~3u;
    promote();
    const bool pend_ready = pend_ok;   /* assigned before this block: its offsets are valid */
    const uint32_t r_o0 = RHP_PEND2 ? pend_o0 : p_o0;
    /* [D] */
    refill_pend();
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[2] += t1 - t0; t0 = t1;
#endif
#if !RHP_EARLY
    /* [E] next window: continuation of cur, else the first window of a ready pend */
    nw = 0;
    if (has && (uint32_t) (pos + (int32_t) kBlock) < cur_len) nw = (cur_ptr + kBlock) | 1u;
    else if (pend_ready) nw = ((r_o0 & ~3u) - (uint32_t) base) | 2u;
    if (kBlock == 128) wait_lgkm0();   /* [A]'s reads of the buffer are done */
    if (kBlock == 128) issue();
#else
    (void) pend_ready;
    (void) r_o0;
#endif
    if (!__ballot(has || nw || pend_ok || RHP_SLOT_OK)) break;
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[3] += t1 - t0; t0 = t1;
#endif
    /* [F] 64 steps (idle lanes step in the parked terminal state); the second
     * half of the window is read after the first 32, and only then is the
     * buffer refilled with the next window */
#pragma unroll
    for (int w = 0; w < (int) kEvWords; w++) ev[w] = 0;
    if (kBlock == 64) {
#ifndef RHP_EXP_NOSTEP   /* timing experiment: no DFA steps (requests never finish) */
      steps_chunks(W, 2, ev);
#endif
#pragma unroll
      for (int q = 0; q < 2; q++) W[q] = *reinterpret_cast<const u32x4 *>(lds + stage + stage_off(lane, q + 2));
      wait_lgkm0();   /* the buffer is read: refill it */
      issue();
#ifndef RHP_EXP_NOSTEP
      steps_chunks(W, 2, ev + 1);
#endif
    } else {
#ifndef RHP_EXP_NOSTEP
      /* no lane has a request (the first iteration of every wave, whose
       * windows are still in flight): skip the walk, which would only step
       * parked lanes through the LDS */
#ifdef RHP_WALK_ALL
      if (__builtin_amdgcn_ballot_w64(has)) steps_chunks(W, 8, ev);
#else
      if (has) steps_chunks(W, 8, ev);   /* idle lanes off: their LDS reads are not issued */
#endif
#endif
    }
    pos += (int32_t) kBlock;
#ifdef RHP_STAMPS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RHP_STAMP(t1); acc[4] += t1 - t0; acc[5] += 1;
#endif
  }
#ifdef RHP_STAMPS
  if (lane == 0) {
    const uint32_t w = (blockIdx.x * WAVES + wave) % 8192;
    for (int k = 0; k < 6; k++) g_stamps[w * 8 + k] = acc[k];
    unsigned long long t_exit = 0;
    RHP_STAMP(t_exit);
    g_stamps[w * 8 + 6] = t_loop - t_entry;
    g_stamps[w * 8 + 7] = t_exit - t_entry;
  }
#endif

  /* Replay: the rare paths run here, after the DFA loop, so none of their
   * registers are live in it.  Once every wave of the workgroup is done, the
   * workgroup walks its range, one request per thread, and finishes what
   * finalize deferred: the exact scalar path, and http_read_request framing of
   * DFA-parsed requests in http mode.  Nothing to do -> no pass at all. */
  __syncthreads();
#ifndef RHP_NO_REPLAY   /* register-pressure experiments only: deferred requests stay unfinished */
  if (*wg_deferred) {
    for (uint32_t i = wg_lo + tid; i < wg_hi; i += WAVES * 64) {
      /* everything a request needs first, in one round trip */
      rhp_req_t r;
      const u32x4 rv = *GLOBAL(const u32x4, p.reqs + i);
      __builtin_memcpy(&r, &rv, sizeof r);
      const uint64_t off = p.offsets[i], end = p.offsets[i + 1];
      typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
      const u32x4a4 hint = p.mode == RHP_MODE_HTTP ? *GLOBAL(const u32x4a4, &p.http[i]) : u32x4a4{0u, 0u, 0u, 0u};
      const uint32_t f = r.flags;
      if (!(f & (kDeferExact | kDeferFrame))) continue;
      if (f & kDeferExact) {
#ifndef RHP_EXP_NOEXACT   /* timing experiment: exact-path requests left unfinished */
        finish_exact(p, i, off, end - off);
#endif
      } else {
#ifdef RHP_EXP_NOFRAME    /* timing experiment: framing left undone */
        continue;
#endif
        r.flags = 0;
        finish_http(p, i, off, end - off, r, hint[0], hint[2], hint[3]);
        p.reqs[i].flags = 0;
      }
    }
  }
#endif
#ifdef RHP_CLOCK
  if (blockIdx.x == 0 && tid == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    g_clock[0] = t1 - clk_t0;
    g_clock[1] = r1 - clk_r0;
  }
#endif
#ifdef RHP_STAMPS
  if (lane == 0) {
    unsigned long long t_end = 0;
    RHP_STAMP(t_end);
    g_stamps_end[(blockIdx.x * WAVES + wave) % 8192] = t_end - t_entry;
  }
#endif
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
/* Host state is per device and safe for one host thread per GPU (SURVEY.md
 * §8e): the CU count and the kernel's LDS attribute are cached per device id,
 * the implementation choice (rhp_set_impl, diagnostics) is per thread. */
constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];
std::atomic<uint32_t> g_attr[kMaxDevices];   /* bit w: the LDS attribute of rhp_dfa_kernel<w> is set */
thread_local int t_impl = RHP_IMPL_DFA;

int device_cus(int dev, int *cus)
{
  int c = g_cus[dev].load(std::memory_order_relaxed);
  if (c == 0) {
    hipError_t e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int) e;
    g_cus[dev].store(c, std::memory_order_relaxed);
  }
  *cus = c;
  return 0;
}

template <int WAVES>
int launch_dfa(const Params &prm, hipStream_t s, int dev, int cus)
{
  const size_t lds_bytes = kLdsTable + (size_t) WAVES * kStageWave + kPoolBytes;
  const uint32_t bit = 1u << (WAVES / 4);
  if (!(g_attr[dev].load(std::memory_order_acquire) & bit)) {
    /* idempotent: two threads of one device may both set it */
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&rhp_dfa_kernel<WAVES>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds_bytes);
    if (e != hipSuccess) return (int) e;
    g_attr[dev].fetch_or(bit, std::memory_order_release);
  }
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rhp_dfa_kernel<WAVES>, WAVES * 64, lds_bytes);
  if (e != hipSuccess) return (int) e;
  if (per_cu < 1) per_cu = 1;
  uint32_t grid = (uint32_t) (cus * per_cu);
  uint32_t need = (prm.n + 64 * WAVES - 1) / (64 * WAVES);
  if (grid > need) grid = need > 0 ? need : 1;
  /* each workgroup owns a contiguous n/grid share of the requests */
  Params q = prm;
  q.span = (prm.n + grid - 1) / grid;
  hipLaunchKernelGGL(rhp_dfa_kernel<WAVES>, dim3(grid), dim3(WAVES * 64), lds_bytes, s, q);
  return (int) hipGetLastError();
}

int dfa_waves()   /* RHP_WAVES (experiments): waves per workgroup */
{
  static const int w = [] {
    const char *e = getenv("RHP_WAVES");
    return e ? atoi(e) : 16;
  }();
  return w;
}
}  // namespace

extern "C" {

const char *rhp_version(void) { return "rhp 0.4.0 (gfx950)"; }

#ifdef RHP_STAMPS
/* diagnostic build only: copy the per-wave section cycle sums (8192 x 8 u64) */
int rhp_debug_stamps(unsigned long long *host)
{
  return (int) hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps), 0, hipMemcpyDeviceToHost);
}
/* ... and the per-wave entry -> end-of-replay spans (8192 u64) */
int rhp_debug_stamps_end(unsigned long long *host)
{
  return (int) hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps_end), sizeof(g_stamps_end), 0, hipMemcpyDeviceToHost);
}
#endif

#ifdef RHP_CLOCK
/* diagnostic build only: (shader ticks, 100 MHz ticks) of block 0's last launch */
int rhp_debug_clock(unsigned long long *host)
{
  return (int) hipMemcpyFromSymbol(host, HIP_SYMBOL(g_clock), sizeof(g_clock), 0, hipMemcpyDeviceToHost);
}
#endif

const char *rhp_kernel_name(void) { return t_impl == RHP_IMPL_EXACT ? "rhp_exact_kernel" : "rhp_dfa_kernel"; }

int rhp_set_impl(int impl)
{
  if (impl != RHP_IMPL_DFA && impl != RHP_IMPL_EXACT) return -22;
  t_impl = impl;
  return 0;
}

int rhp_parse_batch(const rhp_batch_t *b, void *stream)
{
  if (!b) return -22;
  if (b->n == 0) return 0;                       /* nothing to parse, nothing touched */
  if (!b->bytes || !b->offsets || !b->reqs) return -22;
  if (((uintptr_t) b->bytes & 15u) != 0) return -22;   /* windows and exact-path lines are aligned loads */
  if (b->max_headers > RHP_MAX_HEADERS) return -22;
  if (b->max_headers > 0 && !b->hdrs) return -22;
  if (b->mode == RHP_MODE_HTTP && (!b->http || !b->bytes_rw)) return -22;
  if (b->mode != RHP_MODE_PHR && b->mode != RHP_MODE_HTTP) return -22;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int dev = 0, cus = 0;
  {
    hipError_t e = hipGetDevice(&dev);   /* the calling thread's current device */
    if (e != hipSuccess) return (int) e;
    if (dev < 0 || dev >= kMaxDevices) return -22;
    const int rc = device_cus(dev, &cus);
    if (rc != 0) return rc;
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
  prm.span = 0;

  /* the DFA kernel addresses windows with u32 offsets from its range start;
   * batches of 4 GiB or more take the exact kernel */
  if (t_impl == RHP_IMPL_EXACT || b->bytes_size >= 0xFFFF0000ull) {
    uint32_t grid = (b->n + 255) / 256;
    if (grid > (uint32_t) cus * 8) grid = (uint32_t) cus * 8;
    hipLaunchKernelGGL(rhp_exact_kernel, dim3(grid), dim3(256), 0, s, prm);
    return (int) hipGetLastError();
  }
  switch (dfa_waves()) {
  case 4: return launch_dfa<4>(prm, s, dev, cus);
  case 8: return launch_dfa<8>(prm, s, dev, cus);
  case 12: return launch_dfa<12>(prm, s, dev, cus);
  default: return launch_dfa<16>(prm, s, dev, cus);
  }
}

}  // extern "C"
