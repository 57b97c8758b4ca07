/*
 * rhp_kernel.hip -- MI355X (gfx950) batched HTTP/1.1 request parser.
 *
 * Hot path: phr_parse_request (picohttpparser.c:383-409) and the framing of
 * http_read_request (http.c:177-234) over a batch of independent requests in
 * HBM.  Design:
 *
 *  - one request per lane, 64 requests per wave in flight; every lane runs the
 *    byte DFA of rhp_dfa.h in lockstep: per byte one ds_read_u16 of the table in
 *    LDS and two VALU ops that OR the entry's event bit into a 64-bit block
 *    mask -- no LDS write and no divergence on the byte path;
 *  - lanes stream their request in 64-byte windows (4 x global_load_dwordx4 at
 *    4-byte alignment; unaligned starts enter through SKIP states), the next
 *    window issued a whole block ahead; every lane also holds its NEXT
 *    request's offsets, so a request switch never waits on a dependent load;
 *  - once per block the event mask is decoded (rhp_dfa.h dec_event) into the
 *    request-line record and header records, which are stored to HBM in
 *    16-byte pairs; finished requests are finalized and new ones handed out
 *    (persistent waves pull 256-request chunks from one atomic counter);
 *  - a request whose outcome depends on where its buffer ends, or that takes a
 *    rare path (S_SLOW), is finished by the exact scalar path (rhp_scalar.h).
 *
 * The algorithm is mirrored block for block by rhp_emu.cpp (CPU tests).
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
  uint32_t pad;
  uint32_t span;    /* requests per workgroup */
};

#ifndef RHP_SINGLE_STAGE
#define RHP_SINGLE_STAGE 0
#endif
#ifndef RHP_MIN_WAVES_PER_SIMD
#define RHP_MIN_WAVES_PER_SIMD 1
#endif
enum : uint32_t {
  kBlock = RHP_BLOCK,                            /* window bytes per lane per loop iteration */
  kHalves = kBlock / 64,                         /* 64-byte halves per window */
  kEvWords = kBlock / 32,
  kLdsTable = (kTableBytes + 1023u) & ~1023u,   /* staging starts 1 KiB aligned */
  kStageBuf = 64 * kBlock,                       /* one window per lane */
  kDoubleStage = kHalves == 1 && !RHP_SINGLE_STAGE,
  kStageWave = kDoubleStage ? 2 * kStageBuf : kStageBuf,   /* double-buffered, or refilled right after it is read */
  kDeferExact = 0x8000u,                         /* reqs[i].flags while deferred (kernel-internal) */
  kDeferFrame = 0x4000u
};

/* LDS byte address of part q (16 B) of lane w's window inside one staging
 * buffer.  The LDS-DMA loads of a wave write lane-linearly (1 KiB per
 * instruction), so the swizzle lives on the source side: instruction i, lane j
 * fetches part ((j & 3) - (j >> 4)) & 3 of lane 16i + (j >> 2)'s window, which
 * makes each lane's four ds_read_b128 of its own window bank-conflict free. */
__device__ __forceinline__ uint32_t stage_off(uint32_t w, uint32_t q)
{
#ifdef RHP_OWN_WINDOW
  return q * 1024u + w * 16u;
#endif
  const uint32_t u = w & 15u;
  return (q >> 2) * 4096u + (w >> 4) * 1024u + u * 64u + ((q + (u >> 2)) & 3u) * 16u;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));


#ifdef RHP_STAMPS
/* diagnostic build only: per-wave cycle sums per loop section (never read by the kernel) */
__device__ unsigned long long g_stamps[8192 * 8];
#define RHP_STAMP(t) do { __builtin_amdgcn_sched_barrier(0); \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory"); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define RHP_STAMP(t) do { } while (0)
#endif

/* 16 bytes at a 4-byte aligned global address */
__device__ __forceinline__ u32x4 load_chunk(const uint8_t *p)
{
  typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  return *reinterpret_cast<const u32x4a4 *>(p);
}

/* Exact scalar path for one request (phr or http mode).  Only called from the
 * post-loop replay, where inlining it lets it reuse the loop's dead registers
 * (a call there costs ~14 VGPRs of calling-convention overhead). */
__device__ __forceinline__ void finish_exact(const Params &p, uint32_t i, uint64_t off, uint64_t len)
{
#ifdef RHP_EXPERIMENT_NO_EXACT
  p.reqs[i].ret = -9;
  return;
#endif
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

/* http_read_request framing of a request the DFA parsed (http mode only) */
__device__ __forceinline__ void finish_http(const Params &p, uint32_t i, uint64_t off, uint64_t len, rhp_req_t r)
{
  http_frame(p.bytes_rw + off, len, r, p.hdrs + (uint64_t) i * p.max_headers, &p.http[i]);
}

/* Params pointers are generic in the kernel's view (they sit in a struct);
 * the hot stores go through explicit global-address-space pointers so they are
 * global_store (VM counter only), not flat_store (VM + LGKM). */
#define GLOBAL(T, x) ((__attribute__((address_space(1))) T *) (x))

/* ev |= event bit of entry st at bit position `bit`.  Written as asm so the
 * compiler cannot reassociate a block's ORs into one tree at its end, which
 * would keep every step's entry alive in its own VGPR. */
__device__ __forceinline__ void ev_or(uint32_t &ev, uint32_t st, uint32_t bit)
{
  uint32_t t;
  asm("v_lshrrev_b32 %1, 14, %2\n\tv_lshl_or_b32 %0, %1, %3, %0" : "+v"(ev), "=&v"(t) : "v"(st), "s"(bit));
}

/* a 16-byte header-record pair, or a single record, at 4-byte alignment */
__device__ __forceinline__ void store_pair(rhp_hdr_t *dst, u32x4 v)
{
  typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  *GLOBAL(u32x4a4, dst) = v;
}
__device__ __forceinline__ void store_one(rhp_hdr_t *dst, u32x2 v)
{
  typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
  *GLOBAL(u32x2a4, dst) = v;
}
__device__ __forceinline__ void store_req(rhp_req_t *dst, const rhp_req_t &r)
{
  u32x4 v;
  __builtin_memcpy(&v, &r, sizeof r);
  *GLOBAL(u32x4, dst) = v;
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
__global__ __launch_bounds__(WAVES * 64, RHP_MIN_WAVES_PER_SIMD) void rhp_dfa_kernel(Params p)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
#ifdef RHP_STAMPS
  const uint32_t wave = tid >> 6;
  unsigned long long t_entry = 0;
  RHP_STAMP(t_entry);
#endif

  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(&g_table);
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds);
    for (uint32_t k = tid; k < kTableBytes / 16; k += WAVES * 64) dst[k] = src[k];
    if (tid < 2) reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave)[tid] = 0;   /* pool counter, replay flag */
  }
  __syncthreads();

  const uint32_t maxh = p.max_headers;
  const uint32_t park = row_of(S_DONE);

  /* ---- lane state ---- */
  uint32_t st = park;                  /* LDS offset of the current state's row (= the last entry) */
  int32_t pos = 0, block_pos = 0;      /* request-relative position of the next byte / of the block */
  uint32_t ev[kEvWords];               /* events of the block just stepped */
#pragma unroll
  for (int w = 0; w < (int) kEvWords; w++) ev[w] = 0;
  bool has = false;                    /* cur is being parsed */
  uint32_t cur = 0, cur_len = 0;
  uint64_t cur_off = 0, cur_ptr = 0;   /* cur_ptr: byte offset of the window in W */
  Dec d;
  dec_reset(d);
  uint32_t rec_lo = 0, rec_hi = 0;     /* header record waiting for its pair */
  bool pend_ok = false;                /* pend: the lane's next request */
  uint32_t pend = 0;
  uint64_t pend_o0 = 0, pend_o1 = 0;   /* offsets[pend], offsets[pend+1] as loaded */
  uint32_t nw_kind = 0;                /* next window: 0 none, 1 continuation, 2 first window of pend */
  uint64_t nw_ptr = 0;
  u32x4 W[4];
#pragma unroll
  for (int q = 0; q < 4; q++) W[q] = u32x4{0, 0, 0, 0};
  const uint32_t stage = kLdsTable + (tid >> 6) * kStageWave;   /* this wave's two buffers */
  uint32_t buf = 0;                    /* buffer the next window lands in */

  /* ---- request pool ----
   * Workgroup g owns requests [g*span, (g+1)*span) (host: span = n / grid).
   * Lanes that need their next request take it from the workgroup's LDS
   * counter (one atomic per wave and refill, for all of the wave's lanes that
   * need one), so the 16 waves of a CU drain one shared range request by
   * request and finish together; no global atomic is ever touched. */
  const uint32_t wg_lo = min(blockIdx.x * p.span, p.n), wg_hi = min(wg_lo + p.span, p.n);
  uint32_t *wg_counter = reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave);
  uint32_t *wg_deferred = wg_counter + 1;   /* some request of the range needs the replay */
  bool pool_dry = wg_lo >= wg_hi;

  /* give every lane without a pending request one from the pool; the offsets
   * loads are only consumed at the top of the next block */
  auto refill_pend = [&]() {
    const uint64_t want = __ballot(!pend_ok);
    if (!want || pool_dry) return;
    const uint32_t cnt = (uint32_t) __popcll(want);
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(wg_counter, cnt);
    base = wg_lo + __builtin_amdgcn_readfirstlane(base);
    if (base + cnt >= wg_hi) pool_dry = true;
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) want, 0));
    if (!pend_ok && base + rank < wg_hi) {
      pend = base + rank;
      typedef uint64_t u64x2a8 __attribute__((ext_vector_type(2), aligned(8)));
      const u64x2a8 o = *GLOBAL(const u64x2a8, p.offsets + pend);   /* offsets[pend], offsets[pend+1] */
      pend_o0 = o[0];
      pend_o1 = o[1];
      pend_ok = true;
    }
  };

  /* one non-terminal event at request position ep, for the lanes with `valid`
   * (rhp_dfa.h dec_event): the history shift and the event counter are
   * straight-line; the request-line record (once per request) and the header
   * record (every second event) are branches taken only by the lanes concerned */
  auto event = [&](bool valid, uint32_t ep, rhp_hdr_t *hout) {
    const uint32_t k = d.k;
    if (valid) {
      d.h23 = (d.h23 << 16) | (d.h01 >> 16);
      d.h01 = (d.h01 << 16) | ep;
      d.k = k == 4 ? 3u : k + 1u;
      /* CO: history = CO, prevLF; the max_headers check of the line start */
      if (k == 3 && d.nh == maxh && d.ovf == 0) d.ovf = (d.h01 >> 16) + 2u;
    }
    if (valid && k == 2) {   /* RL: history = RL, PE, ME */
      const uint32_t pe = d.h01 >> 16, me = d.h23 & 0xffffu;
      d.rl01 = me | ((me + 1u) << 16);
      d.rl23 = (pe - me - 1u) | ((ep - pe - 9u) << 16);
      d.h01 = (d.h01 & 0xffff0000u) | (pe + 10u);
    }
    if (valid && k == 4) {   /* EOL: history = LF, CO, prevLF */
      const uint32_t co = d.h01 >> 16, prev = d.h23 & 0xffffu;
      const uint32_t lo = (prev + 1u) | ((co - prev - 1u) << 16);
      const uint32_t hi = (co + 2u) | ((ep - co - 3u) << 16);
      const uint32_t nh = ++d.nh;
      if (nh <= maxh) {
        if (nh & 1u) { rec_lo = lo; rec_hi = hi; }
        else if (!(p.pad & 2)) store_pair(hout + nh - 2u, u32x4{rec_lo, rec_hi, lo, hi});
      }
    }
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
    const uint32_t row = st;
    const bool slow = row == row_of(S_SLOW);
    const bool term_ev = is_done_row(row) || is_err_row(row);
    uint32_t m[kEvWords];
#pragma unroll
    for (int w = 0; w < (int) kEvWords; w++) m[w] = slow ? 0u : ev[w];
    uint32_t term_pos = 0xffffffffu;
    if (term_ev) {   /* the terminal is the block's last event: take it off the mask */
      bool found = false;
#pragma unroll
      for (int w = (int) kEvWords - 1; w >= 0; w--) {
        if (!found && m[w]) {
          const uint32_t bt = 31u - __builtin_clz(m[w]);
          term_pos = (uint32_t) block_pos + 32u * w + bt;
          m[w] &= ~(1u << bt);
          found = true;
        }
      }
    }
    rhp_hdr_t *hout = p.hdrs + (uint64_t) cur * maxh;
#pragma unroll
    for (int w = 0; w < (int) kEvWords; w++) {
      uint32_t mw = d.ovf ? 0u : m[w];
      while (__ballot(mw != 0)) {
        const bool valid = mw != 0;
        const uint32_t bt = __builtin_ctz(mw | 0x80000000u);
        mw &= mw - 1u;
        event(valid, (uint32_t) block_pos + 32u * w + bt, hout);
        mw = d.ovf ? 0u : mw;
      }
    }
    const bool ovf = d.ovf != 0;
    const bool fin = ovf || slow || term_ev || pos >= (int32_t) cur_len;
    if (!fin) return;
    const bool ok = !ovf && is_done_row(row) && term_pos < cur_len;
    const bool bad = ovf ? d.ovf - 1u < cur_len : (is_err_row(row) && term_pos < cur_len);
    rhp_req_t r = {};
    r.minor_version = -1;
    if (ok) {
      if ((d.nh & 1u) && !(p.pad & 2)) store_one(hout + d.nh - 1u, u32x2{rec_lo, rec_hi});
      r.ret = (int32_t) term_pos + 1;
      r.method_len = (uint16_t) d.rl01;
      r.path_off = (uint16_t) (d.rl01 >> 16);
      r.path_len = (uint16_t) d.rl23;
      r.minor_version = (int8_t) (d.rl23 >> 16);
      r.num_headers = (uint16_t) d.nh;
      r.flags = p.mode == RHP_MODE_HTTP ? (uint16_t) kDeferFrame : (uint16_t) 0;   /* framing: replay */
      if (p.mode == RHP_MODE_HTTP) *wg_deferred = 1u;
    } else if (bad) {
      r.ret = -1;
      if (p.mode == RHP_MODE_HTTP) store_http_bad(p.http + cur);
    } else {
      r.flags = (uint16_t) kDeferExact;   /* exact path: replay */
      *wg_deferred = 1u;
    }
    if (!(p.pad & 2)) store_req(p.reqs + cur, r);
    has = false;
    st = park;
  };

  /* 16 DFA steps over one 16-byte chunk; events -> bits [base, base+16) of ev */
  auto steps = [&](const u32x4 &chunk, uint32_t &ev, const int base) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t c = (chunk[k >> 2] >> ((k & 3) * 8)) & 0xffu;
      st = *reinterpret_cast<const uint16_t *>(lds + st + c * 2u);
      ev_or(ev, st, base + k);
      /* keep the scheduler from hoisting the byte extraction of all 64 steps
       * (it would hold 64 VGPRs of precomputed offsets) */
      if ((k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  };

  /* half h of the lane's window from the staging buffer (zeros for an idle lane) */
  auto read_half = [&](uint32_t kind, int h) {
    const uint8_t *sb = lds + stage + (kDoubleStage ? (buf ^ kStageBuf) : 0u);
#pragma unroll
    for (int q = 0; q < 4; q++)
      W[q] = kind ? *reinterpret_cast<const u32x4 *>(sb + stage_off(lane, 4 * h + q)) : u32x4{0, 0, 0, 0};
  };

  /* LDS-DMA of half h of every lane's next window (nw_ptr / nw_kind) */
  auto issue_half = [&](int h) {
    uint8_t *db = lds + stage + (kDoubleStage ? buf : 4096u * h);
#ifdef RHP_OWN_WINDOW
    /* experiment: every lane fetches its own window (lane-linear) */
    if (nw_kind) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(p.bytes + nw_ptr + 64u * h + 16u * i),
                                         (__attribute__((address_space(3))) void *) (db + 1024u * i), 16, 0, 0);
    }
#else
    /* the wave fetches all 64 windows with 4 LDS-DMA loads, 16 windows of 64 B each */
    const uint64_t src = nw_kind ? nw_ptr + 64u * h : ~(uint64_t) 0;
    const uint32_t slo = (uint32_t) src, shi = (uint32_t) (src >> 32);
    const uint32_t part = ((lane & 3u) - (lane >> 4)) & 3u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t w = 16u * i + (lane >> 2);
      const uint32_t lo = __shfl(slo, (int) w), hi = __shfl(shi, (int) w);
      const uint64_t a = ((uint64_t) hi << 32) | lo;
      if (a != ~(uint64_t) 0)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(p.bytes + a + 16u * part),
                                         (__attribute__((address_space(3))) void *) (db + 1024u * i), 16, 0, 0);
    }
#endif
  };

  refill_pend();

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
   * window's loads -> 64 DFA steps.
   */
  for (;;) {
    RHP_STAMP(t0);
    /* [A] */
    const uint64_t p_o0 = pend_o0, p_o1 = pend_o1;
    const uint32_t nw_kind_prev = nw_kind;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* the window's LDS-DMA has landed */
    read_half(nw_kind_prev, 0);
#ifdef RHP_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    RHP_STAMP(t1); acc[0] += t1 - t0; t0 = t1;
#endif
    /* [B] */
    decode();
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[1] += t1 - t0; t0 = t1;
#endif
    /* [C] */
    if (nw_kind == 2) {
      cur = pend; cur_off = p_o0; cur_len = (uint32_t) min(p_o1 - p_o0, (uint64_t) 0xffffffffu);
      pend_ok = false;
      has = true;
      const uint32_t mis = (uint32_t) cur_off & 3u;
      uint32_t s0 = mis == 0 ? S_METHOD0 : mis == 1 ? S_SKIP1 : mis == 2 ? S_SKIP2 : S_SKIP3;
      if (cur_len > kFastMaxLen) s0 = S_SLOW;
      st = row_of(s0);
      pos = -(int32_t) mis;
      dec_reset(d);
    }
    if (nw_kind) cur_ptr = nw_ptr;
    const bool pend_ready = pend_ok;   /* assigned before this block: p_o0/p_o1 valid */
    /* [D] */
    refill_pend();
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[2] += t1 - t0; t0 = t1;
#endif
    /* [E] next window: continuation of cur, else the first window of a ready pend */
    nw_kind = 0;
    if (has && cur_ptr + kBlock < cur_off + cur_len) {
      nw_ptr = cur_ptr + kBlock;
      nw_kind = 1;
    } else if (pend_ready) {
      nw_ptr = p_o0 & ~(uint64_t) 3;
      nw_kind = 2;
    }
    if (!kDoubleStage) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   /* [A]'s reads of this buffer are done */
    issue_half(0);
    if (kDoubleStage) buf ^= kStageBuf;
    if (!__ballot(has || nw_kind || pend_ok)) break;
#ifdef RHP_STAMPS
    RHP_STAMP(t1); acc[3] += t1 - t0; t0 = t1;
#endif
    /* kBlock steps (idle lanes step in the parked terminal state) */
    block_pos = pos;
#pragma unroll
    for (int w = 0; w < (int) kEvWords; w++) ev[w] = 0;
    steps(W[0], ev[0], 0);
    steps(W[1], ev[0], 16);
    steps(W[2], ev[1], 0);
    steps(W[3], ev[1], 16);
    if (kHalves == 2) {
      /* second half of this window, then refill that half with the next window's */
      __builtin_amdgcn_sched_barrier(0);
      read_half(nw_kind_prev, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue_half(1);
      steps(W[0], ev[kEvWords - 2], 0);
      steps(W[1], ev[kEvWords - 2], 16);
      steps(W[2], ev[kEvWords - 1], 0);
      steps(W[3], ev[kEvWords - 1], 16);
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
#ifndef RHP_NO_REPLAY   /* timing experiment only: deferred requests stay unfinished */
  __syncthreads();
  if (*wg_deferred) {
    for (uint32_t i = wg_lo + tid; i < wg_hi; i += WAVES * 64) {
      const uint32_t f = p.reqs[i].flags;
      if (!(f & (kDeferExact | kDeferFrame))) continue;
      const uint64_t off = p.offsets[i], len = p.offsets[i + 1] - off;
      if (f & kDeferExact) {
        finish_exact(p, i, off, len);
      } else {
        rhp_req_t r = p.reqs[i];
        r.flags = 0;
        finish_http(p, i, off, len, r);
        p.reqs[i].flags = 0;
      }
    }
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
int g_impl = RHP_IMPL_DFA;
int g_cus = 0;

template <int WAVES>
int launch_dfa(const Params &prm, hipStream_t s)
{
  const size_t lds_bytes = kLdsTable + (size_t) WAVES * kStageWave + 16;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&rhp_dfa_kernel<WAVES>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds_bytes);
    if (e != hipSuccess) return (int) e;
    attr_set = true;
  }
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rhp_dfa_kernel<WAVES>, WAVES * 64, lds_bytes);
  if (e != hipSuccess) return (int) e;
  if (per_cu < 1) per_cu = 1;
  uint32_t grid = (uint32_t) (g_cus * per_cu);
  uint32_t need = (prm.n + 64 * WAVES - 1) / (64 * WAVES);
  if (grid > need) grid = need > 0 ? need : 1;
  /* each workgroup owns a contiguous n/grid share of the requests */
  Params q = prm;
  q.span = (prm.n + grid - 1) / grid;
  hipLaunchKernelGGL(rhp_dfa_kernel<WAVES>, dim3(grid), dim3(WAVES * 64), lds_bytes, s, q);
  return (int) hipGetLastError();
}

int g_waves = -1;   /* RHP_WAVES (experiments): waves per workgroup */

int dfa_waves()
{
  if (g_waves < 0) {
    const char *e = getenv("RHP_WAVES");
    g_waves = e ? atoi(e) : 16;
  }
  return g_waves;
}
}  // namespace

extern "C" {

const char *rhp_version(void) { return "rhp 0.3.0 (gfx950)"; }

#ifdef RHP_STAMPS
/* diagnostic build only: copy the per-wave section cycle sums (8192 x 8 u64) */
int rhp_debug_stamps(unsigned long long *host)
{
  return (int) hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps), 0, hipMemcpyDeviceToHost);
}
#endif

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
  prm.span = 0;
  {
    const char *e = getenv("RHP_EXPERIMENT");   /* timing experiments only: breaks results */
    prm.pad = e ? (uint32_t) atoi(e) : 0u;
  }

  if (g_impl == RHP_IMPL_EXACT) {
    uint32_t grid = (b->n + 255) / 256;
    if (grid > (uint32_t) g_cus * 8) grid = (uint32_t) g_cus * 8;
    hipLaunchKernelGGL(rhp_exact_kernel, dim3(grid), dim3(256), 0, s, prm);
    return (int) hipGetLastError();
  }
  switch (dfa_waves()) {
  case 4: return launch_dfa<4>(prm, s);
  case 8: return launch_dfa<8>(prm, s);
  case 11: return launch_dfa<11>(prm, s);
  case 10: return launch_dfa<10>(prm, s);
  case 12: return launch_dfa<12>(prm, s);
  default: return launch_dfa<16>(prm, s);
  }
}

}  // extern "C"
