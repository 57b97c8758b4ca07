/*
 * rhp_kernel.hip -- MI355X (gfx950) batched HTTP/1.1 request parser.
 *
 * Hot path: phr_parse_request (picohttpparser.c:383-409) and the framing of
 * http_read_request (http.c:177-234) over a batch of independent requests in
 * HBM.  Design:
 *
 *  - one request per lane, 64 requests per wave in flight; every lane runs the
 *    pair DFA of rhp_dfa.h in lockstep, two bytes per table read:
 *        r      = class-row(b1)                      ds_read_u8 (independent)
 *        code   = T[r * 256 + b0]                    ds_read_u8 (independent)
 *        idx    = T[v_perm(idx, code)]               one dependent ds_read_u8
 *        ev     = v_alignbit(idx, ev, 2)             low index bits = event bits
 *  - lanes stream their request in 128-byte windows (4-aligned): the wave
 *    fetches its 64 lanes' next windows with eight LDS-DMA loads (8 windows
 *    each) one iteration ahead of use, and every lane holds its NEXT request's
 *    offsets, so neither a window nor a request switch waits on a dependent
 *    load (lane-per-window loads straight into registers, interleaved with the
 *    walk, took 43 % longer: profiles/r02/c/ab_direct.txt);
 *  - the events of a window are decoded into records (prefix-XOR split of the
 *    alternating colon / line-end events, one loop trip per header) one
 *    iteration behind the walk, into the issue slots its dependent LDS reads
 *    leave free;
 *  - a request the table cannot decide alone (S_SLOW, a terminal at/after
 *    len, no terminal by the end of its buffer) and http framing are finished
 *    after the loop by the workgroup's replay (rhp_scalar.h exact path through
 *    a 16-byte line cache; framing from the decode's hints).
 *
 * The per-request decisions (fast ok / fast -1 / exact) are mirrored by
 * rhp_emu.cpp (CPU tests).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <type_traits>

#include "rhp.h"
#include "rhp_dfa.h"
#include "rhp_scalar.h"

namespace {

using namespace rhp;

static_assert(RHP_BLOCK == 128, "the kernel walks 128-byte windows (whole HBM lines)");

__device__ const Table2 g_table = make_table2();

struct Params {
  const uint8_t *bytes;
  uint8_t *bytes_rw;
  const uint64_t *offsets;
  rhp_req_t *reqs;
  rhp_hdr_t *hdrs;
  rhp_http_t *http;
  const uint64_t *last_len;   /* phr mode, may be NULL: is_complete first where != 0 */
  bool compact;               /* http mode: de-frame chunked bodies in place (not speculative) */
  uint32_t n;
  uint32_t max_headers;
  uint32_t mode;
  uint32_t span;    /* requests per workgroup */
  uint32_t hs_req;  /* stride of the exact path's rhp_hdr_t records between requests (rhp_layout) */
  uint32_t hs_hdr;  /* ... between the records of one request */
  /* the records the DFA writes: rhp_hdr_t at hdrs, or (RHP_LAYOUT_COMPACT) u32
   * lengths at lens, header-major, the exact path's records then in the wide
   * area at hdrs */
  uint32_t *lens;
  uint32_t rec_req, rec_hdr;
  bool wt_records;   /* records header-major or compact in phr mode: write-through where a range is even */
  /* RHP_LAYOUT_COMPACT in http mode: the 8-byte http records (rhp.h
   * rhp_http_compact_t); `http` then points at their wide area, which also
   * holds the replay's hints */
  uint2 *hc;
  /* RHP_LAYOUT_DENSE (phr mode): the 8-byte request records (rhp_req_dense_t)
   * and the 2-byte header lengths (header-major); `reqs` and `hdrs` then point
   * at their wide areas */
  uint2 *dreq;
  uint16_t *lens16;
  uint32_t *ovf32;   /* ... and the u32 lengths of the headers the u16 cannot hold */
};

/* http records (RHP_MODE_HTTP).  With compact records (p.hc) a record whose
 * consumed follows from ret (rhp.h) is stored compact; the wide ones (the exact
 * path, chunked bodies) go to the wide area and the compact record says so. */
__device__ __forceinline__ void store_hc(const Params &p, uint32_t i, uint32_t w0, uint32_t w1)
{
  typedef uint32_t u32x2a8 __attribute__((ext_vector_type(2), aligned(8)));
  *((__attribute__((address_space(1))) u32x2a8 *) (p.hc + i)) = u32x2a8{w0, w1};
}
__device__ __forceinline__ void mark_wide(const Params &p, uint32_t i)
{
  if (p.hc) store_hc(p, i, RHP_HTTP_WIDE << 16, 0u);
}
/* a final record whose consumed is ret (+ body_len for a Content-Length body,
 * mod 2^64 as http.c:216), or 0; a body_len past 32 bits (a Content-Length
 * whose ret + size wrapped, or a body beyond 4 GiB) keeps the wide record */
__device__ __forceinline__ void put_http(const Params &p, uint32_t i, const rhp_http_t &o)
{
  if (p.hc && !(o.body_len >> 32)) {
    store_hc(p, i, ((uint32_t) o.result & 0xffu) | o.body_kind << 8, (uint32_t) o.body_len);
  } else {
    p.http[i] = o;
    mark_wide(p, i);
  }
}

#ifndef RHP_WAVES_PER_SIMD
#define RHP_WAVES_PER_SIMD 4
#endif

enum : uint32_t {
  kSecDecodeStamp = 6,                           /* Diag section slots of the late form's decode / framing; */
  kSecFrameStamp = 7,                            /* the early form's window reads + [C] / shuffles + [D] */
  kBlock = 128,                                  /* window bytes per lane per loop iteration (early form) */
  kParts = kBlock / 16,                          /* 16-byte parts per window */
  kEvWords = kBlock / 32,                        /* 32-bit event words per window */
  kLdsTable = (kTable2Bytes + 1023u) & ~1023u,   /* staging starts 1 KiB aligned */
  kStageWave = 64 * kBlock,                      /* one window per lane */
  kPark = 0,                                     /* the DONE index: idle lanes step here */
  kDeferExact = 0x8000u,                         /* reqs[i].flags while deferred (kernel-internal) */
  kDeferDense = 0x80u,                           /* ... rhp_req_dense_t flags (RHP_LAYOUT_DENSE) */
  /* http mode: the replay's instructions, in the body_kind word of the hint
   * finalize leaves in http[i] (ret in the low 16 bits) */
  kHintExact = 0x40000000u,
  kHintFrame = 0x80000000u,
  kHintChunked = 0x20000000u,   /* with kHintFrame: the only candidate is a Transfer-Encoding: chunked */
  /* fr: the first framing candidate's evaluation (late-issue kernel) */
  kFrCarry = 1u,      /* its name is Content-Length, its value is being read (digits in fv) */
  kFrTeName = 2u,     /* its name is Transfer-Encoding, its record not complete yet */
  kFrCl = 4u,         /* a Content-Length with a value: fv = strtoull(value) */
  kFrTe = 8u,         /* a Transfer-Encoding with a value */
  kFrDefer = 16u,     /* not evaluated here: the replay frames the request */
  kFrDigits = 32u,    /* the number has started (a sign or a digit was read) */
  kFrNeg = 64u,       /* ... with a '-' */
  kFrStop = 128u,     /* ... and ended (a non-digit was read) */
  kFrCountSh = 8u,    /* bits 8..15: value bytes read */
  kFrMaxValue = 19u,  /* longer values are left to the replay (19 digits cannot overflow) */
  kFrNeither = 1u << 16,   /* its name, read while its line was open, is neither */
  kFrChunked = 1u << 17,   /* a Transfer-Encoding whose value is "chunked" (any case) */
  /* workgroup pool area after the staging buffers: counters, then the replay's
   * list; an uneven range's longest-first order (ranges up to kOrderSpan
   * requests) and its histogram live in the staging buffers of the waves such a
   * range leaves idle */
  kPoolWords = 8,                                /* counter, replay flag, -, -, slow-list length,
                                                    defer-list length */
  kOrderSpan = 8192,
  kOrderBuckets = 64,                            /* window counts 1..63 (63: 63 or more) */
  kDeferCap = 480,                               /* the replay's list (defer) */
  kPoolBytes = 4 * kPoolWords + 2 * kDeferCap,
  kOrderWaves = 2                                /* idle waves whose staging holds an uneven range's order */
};
static_assert(idx2(S_DONE, 0) == kPark, "parked lanes sit in DONE");

/* http mode's window extension (16-byte parts past the 128-byte window, see
 * the kernel's window geometry) and the waves its staging leaves room for */
constexpr uint32_t kHttpXParts = RHP_HTTP_XPARTS;   /* rhp_dfa.h: the emulator walks the same windows */
constexpr int kHttpWaves = kHttpXParts == 0 ? 16 : kHttpXParts <= 2 ? 12 : 8;
#ifndef RHP_CODE_FORM
#define RHP_CODE_FORM 1
#endif
constexpr int kCodeForm = RHP_CODE_FORM;   /* how a pair's code is looked up (the walk's look_a / look_b) */
/* the lowest pair index of a state that is not terminal (DONE, ERR, SLOW and
 * their event forms are the indices below it) */
constexpr uint32_t kLiveIdx = idx2(S_SLOW, 1) + 1u;
static_assert(idx2(S_DONE, 0) < kLiveIdx && idx2(S_ERR, 1) < kLiveIdx && idx2(S_DONE_E, 3) < kLiveIdx &&
              idx2(S_ERR_E, 3) < kLiveIdx && idx2(S_PRE, 0) >= kLiveIdx && idx2(S_SP1_E, 2) >= kLiveIdx,
              "terminal indices lie below every live one");
#ifndef RHP_PHASE_LOCK
#define RHP_PHASE_LOCK 1
#endif

/* LDS byte address of part q (16 B) of lane w's window inside the staging
 * buffer.  The LDS-DMA loads of a wave write lane-linearly (1 KiB per
 * instruction), so the swizzle lives on the source side, chosen so that each
 * lane's ds_read_b128 of its own window are bank-conflict free: instruction i,
 * lane j fetches part ((j & 7) - (w >> 1)) & 7 of lane w = 8i + (j >> 3)'s
 * window (8 whole 128-B lines per load, so every HBM line is fetched by one
 * instruction). */
__device__ __forceinline__ uint32_t stage_off(uint32_t w, uint32_t q)
{
  return (w >> 3) * 1024u + (w & 7u) * 128u + ((q + (w >> 1)) & 7u) * 16u;
}
__device__ __forceinline__ uint32_t dma_window(uint32_t i, uint32_t j) { return 8u * i + (j >> 3); }
__device__ __forceinline__ uint32_t dma_part(uint32_t w, uint32_t j) { return ((j & 7u) - (w >> 1)) & 7u; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

/* s_waitcnt vmcnt(0) / lgkmcnt(0), as inline asm (invisible to the compiler's
 * wait insertion, which would otherwise add waits of its own around them) */
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

/* Diagnostics.  The kernel calls the methods of one `Diag` object at its
 * section boundaries; in product builds every method is empty and the object
 * has no state, so the hot loop compiles as if the calls were not there.
 *
 * RHP_STAMPS (diagnostic build, tools/stamps2.py): per-wave shader-cycle sums
 * per loop section and realtime (100 MHz) marks, stored by each wave's lane 0
 * into a buffer of its own (never read by the kernel): slots 0-4 section
 * cycles, 5 iterations, 6 entry, 7 loop start, 8 loop end, 9 exit, 10
 * lane-windows walked, 11 lane-iterations without a window to walk, 12 of them
 * while the pool still had requests, 13 iterations after the pool ran dry, 14
 * the replay's start (after the workgroup barrier), 15 / 16 the wave's shader
 * cycles in the replay's pass 2 (listed scalar paths) / pass 1, 17 requests it
 * ran in pass 2, 18 requests it framed in pass 1, 19 the prologue's loads
 * landed, 20 / 21 late form: decode_window / frame_window cycles (inside
 * section 2), 22 / 23 pass 2's validation and serial paths / staged moves.  A section that ends with a wait (`sync`) waits for its LDS reads
 * (and, where named, its memory) first, so its cycles include their latency.
 * RHP_CLOCK (diagnostic build, tools/kclock.py): shader ticks and 100 MHz
 * ticks from the entry of block 0 wave 0 to its loop's end. */
#ifdef RHP_STAMPS
enum : uint32_t { kStampSlots = 24 };
__device__ unsigned long long g_stamps[8192 * kStampSlots];
#endif
#ifdef RHP_CLOCK
__device__ unsigned long long g_clock[2];
#endif
struct Diag {
#ifdef RHP_STAMPS
  unsigned long long t0 = 0, t1 = 0, c0 = 0, c1 = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, rp[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long rt_entry = 0, rt_loads = 0, rt_loop = 0, n_walk = 0, n_idle = 0, n_idle_live = 0, n_dry = 0;
  __device__ __forceinline__ static unsigned long long now()
  {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
  }
  __device__ __forceinline__ unsigned long long *slots(uint32_t waves) const
  {
    return g_stamps + ((blockIdx.x * waves + (threadIdx.x >> 6)) % 8192u) * kStampSlots;
  }
  __device__ __forceinline__ void entry() { rt_entry = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void loads_landed() { rt_loads = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void loop_start() { rt_loop = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void mark() { t0 = now(); }
  /* the section that began at the last mark ends here: its cycles into acc[k] */
  __device__ __forceinline__ void section(uint32_t k, bool lgkm = false, bool vm = false)
  {
    if (vm) wait_vm0();
    if (lgkm) wait_lgkm0();
    t1 = now();
    acc[k] += t1 - t0;
    t0 = t1;
  }
  __device__ __forceinline__ void lanes(bool walking, bool pool_dry)
  {
    n_walk += __popcll(__builtin_amdgcn_ballot_w64(walking));
    n_idle += __popcll(__builtin_amdgcn_ballot_w64(!walking));
    if (!pool_dry) n_idle_live += __popcll(__builtin_amdgcn_ballot_w64(!walking));
    else n_dry++;
  }
  __device__ __forceinline__ void iteration_end() { section(4); acc[5] += 1; }
  __device__ __forceinline__ void loop_end(uint32_t waves)
  {
    if ((threadIdx.x & 63u) != 0) return;
    unsigned long long *g = slots(waves);
    for (int k = 0; k < 6; k++) g[k] = acc[k];
    g[6] = rt_entry; g[7] = rt_loop; g[8] = __builtin_amdgcn_s_memrealtime();
    g[10] = n_walk; g[11] = n_idle; g[12] = n_idle_live; g[13] = n_dry; g[19] = rt_loads;
    g[20] = acc[kSecDecodeStamp]; g[21] = acc[kSecFrameStamp];
  }
  __device__ __forceinline__ void replay_start(uint32_t waves)
  {
    if ((threadIdx.x & 63u) == 0) slots(waves)[14] = __builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ void pass_begin() { c0 = now(); }
  __device__ __forceinline__ void pass_end(uint32_t k) { rp[k] += now() - c0; }   /* 0: pass 2, 1: pass 1 */
  __device__ __forceinline__ void framed(bool done) { rp[3] += __popcll(__builtin_amdgcn_ballot_w64(done)); }
  __device__ __forceinline__ void slow_path() { rp[2] += __popcll(__builtin_amdgcn_ballot_w64(true)); }
  /* pass 2's parts: 4 the lanes' validation / serial paths, 5 the wave's staged moves */
  __device__ __forceinline__ void part_begin() { c1 = now(); }
  __device__ __forceinline__ void part_end(uint32_t k) { rp[k] += now() - c1; }
  __device__ __forceinline__ void exit(uint32_t waves)
  {
    if ((threadIdx.x & 63u) != 0) return;
    unsigned long long *g = slots(waves);
    g[9] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 4; k++) g[15 + k] = rp[k];
    g[22] = rp[4]; g[23] = rp[5];
  }
#else
  __device__ void entry() {}
  __device__ void loads_landed() {}
  __device__ void loop_start() {}
  __device__ void mark() {}
  __device__ void section(uint32_t, bool = false, bool = false) {}
  __device__ void lanes(bool, bool) {}
  __device__ void iteration_end() {}
  __device__ void loop_end(uint32_t) {}
  __device__ void replay_start(uint32_t) {}
  __device__ void pass_begin() {}
  __device__ void pass_end(uint32_t) {}
  __device__ void framed(bool) {}
  __device__ void slow_path() {}
  __device__ void part_begin() {}
  __device__ void part_end(uint32_t) {}
  __device__ void exit(uint32_t) {}
#endif
#ifdef RHP_CLOCK
  unsigned long long clk_t0 = 0, clk_r0 = 0;
  __device__ void clock_start() { clk_t0 = __builtin_amdgcn_s_memtime(); clk_r0 = __builtin_amdgcn_s_memrealtime(); }
  __device__ void clock_end()
  {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      g_clock[0] = __builtin_amdgcn_s_memtime() - clk_t0;
      g_clock[1] = __builtin_amdgcn_s_memrealtime() - clk_r0;
    }
  }
#else
  __device__ void clock_start() {}
  __device__ void clock_end() {}
#endif
};

/* The exact parser's byte reader on the GPU: the aligned 16-byte line holding
 * the last byte read stays in registers, so its sequential scan makes one
 * global load per 16 bytes (the batch buffer is 16-aligned and padded) */
struct LineBytes {
  const uint8_t *b;
  uint64_t line;
  u32x4 c;
  __device__ uint32_t operator()(uint64_t p)
  {
    const uint64_t a = (uint64_t) (uintptr_t) b + p;
    const uint64_t l = a & ~(uint64_t) 15;
    if (l != line) {
      c = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>((uintptr_t) l);
      line = l;
    }
    const uint32_t q = (uint32_t) (a >> 2) & 3u;
    const uint32_t d = q == 0 ? c[0] : q == 1 ? c[1] : q == 2 ? c[2] : c[3];
    return (d >> (8u * ((uint32_t) a & 3u))) & 0xffu;
  }
};

/* n body bytes from src to dst (dst <= src, offsets from `in`), forward: the
 * in-place move of http_dechunk (http.c:155) for one thread.  Destination
 * blocks are whole aligned 16-byte stores built from aligned 16-byte source
 * lines (funnel-shifted by the constant src - dst), four blocks per memory
 * round trip; the partial first and last blocks are byte stores, so no byte
 * outside [dst, dst + n) -- another request's -- is written.  Loads read only
 * source bytes no earlier store has reached (each block's source lies past its
 * destination), apart from unused bytes of shared lines. */
struct DevMove {
  uint8_t *in;
  __device__ void operator()(uint64_t dst, uint64_t src, uint64_t n) const
  {
    typedef __attribute__((address_space(1))) const u32x4 gq;
    typedef __attribute__((address_space(1))) u32x4 gw;
    if (n == 0 || dst == src) return;
    const uintptr_t da = (uintptr_t) (in + dst), de = da + n, delta = (uintptr_t) (src - dst);
    const uint32_t q = (uint32_t) (delta >> 2) & 3u, r = (uint32_t) delta & 3u;
    /* block at destination A: source bytes [A + delta, A + delta + 16) from the
     * lines at (A + delta) & ~15 and the one after it */
    auto ld = [](uintptr_t a) -> u32x4 { return *reinterpret_cast<gq *>(a); };
    auto block = [&](const u32x4 &l0, const u32x4 &l1) {
      const uint32_t w[8] = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t lo = q == 0 ? w[j] : q == 1 ? w[j + 1] : q == 2 ? w[j + 2] : w[j + 3];
        const uint32_t hi = q == 0 ? w[j + 1] : q == 1 ? w[j + 2] : q == 2 ? w[j + 3] : w[j + 4];
        o[j] = __builtin_amdgcn_alignbyte(hi, lo, r);
      }
      return o;
    };
    auto partial = [&](uintptr_t A) {   /* bytes of block A inside [da, de): whole dwords, then bytes */
      typedef __attribute__((address_space(1))) uint32_t gw1;
      typedef __attribute__((address_space(1))) uint8_t gb1;
      const uintptr_t s0 = (A + delta) & ~(uintptr_t) 15;
      const u32x4 o = block(ld(s0), ld(s0 + 16));
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        const uintptr_t w = A + 4 * j;
        if (w >= da && w + 4 <= de) {
          *reinterpret_cast<gw1 *>(w) = o[j];
        } else if (w + 4 > da && w < de) {
#pragma unroll
          for (uint32_t k = 0; k < 4; k++)
            if (w + k >= da && w + k < de) *reinterpret_cast<gb1 *>(w + k) = (uint8_t) (o[j] >> (8 * k));
        }
      }
    };
    uintptr_t A = da & ~(uintptr_t) 15;
    if (A != da || A + 16 > de) {   /* a partial first block */
      partial(A);
      A += 16;
    }
#ifndef RHP_MOVE_UNROLL
#define RHP_MOVE_UNROLL 4
#endif
    constexpr int U = RHP_MOVE_UNROLL;   /* destination blocks per memory round trip */
    while (A + 16 * U <= de) {
      const uintptr_t s0 = (A + delta) & ~(uintptr_t) 15;
      u32x4 l[U + 1];
#pragma unroll
      for (int u = 0; u <= U; u++) l[u] = ld(s0 + 16 * u);
#pragma unroll
      for (int u = 0; u < U; u++) *reinterpret_cast<gw *>(A + 16 * u) = block(l[u], l[u + 1]);
      A += 16 * U;
    }
    while (A + 16 <= de) {
      const uintptr_t s0 = (A + delta) & ~(uintptr_t) 15;
      *reinterpret_cast<gw *>(A) = block(ld(s0), ld(s0 + 16));
      A += 16;
    }
    if (A < de) partial(A);
  }
};

/* http_dechunk on the GPU (rhp_scalar.h dechunk_t): size lines read through the
 * 16-byte line cache, payloads moved 16 bytes per store */
struct DevDechunk {
  __device__ int64_t operator()(uint8_t *in, uint64_t size, uint64_t *body_len, bool compact) const
  {
    LineBytes B{in, ~0ull, {0, 0, 0, 0}};
    DevMove M{in};
    return dechunk_t(B, M, size, body_len, compact);
  }
};

/* Exact scalar path for one request (phr or http mode).  Only called from the
 * post-loop replay, where inlining it lets it reuse the loop's dead registers. */
__device__ __forceinline__ void finish_exact(const Params &p, uint32_t i, uint64_t off, uint64_t len)
{
  rhp_req_t r;
  r.flags = RHP_F_EXACT | (p.lens || p.lens16 ? RHP_F_WIDE : 0u);   /* compact / dense: this request's records are wide */
  rhp_hdr_t *h = p.hdrs + (uint64_t) i * p.hs_req;
  if (p.mode == RHP_MODE_HTTP) {
    rhp_http_t x;
    LineBytes B{p.bytes_rw + off, ~0ull, {0, 0, 0, 0}};
    scalar_http_t(B, p.bytes_rw + off, len, p.max_headers, &r, h, p.hs_hdr, &x, p.compact, DevDechunk{});
    p.http[i] = x;
    mark_wide(p, i);
  } else {
    LineBytes B{p.bytes + off, ~0ull, {0, 0, 0, 0}};
    const uint64_t ll = p.last_len ? p.last_len[i] : 0;
    /* phr_parse_request runs is_complete first when last_len != 0
     * (picohttpparser.c:399-401); its -2 / -1 is the answer */
    const int pre = ll ? is_complete_t(B, len, ll) : 0;
    if (pre != 0) {
      r.ret = pre;
      r.method_len = r.path_off = r.path_len = 0;
      r.method_off = 0;
      r.minor_version = -1;
      r.num_headers = 0;
    } else {
      scalar_phr_t(B, len, p.max_headers, &r, h, p.hs_hdr);
    }
  }
  p.reqs[i] = r;
  if (p.dreq) p.dreq[i] = uint2{0u, RHP_DENSE_WIDE << 24};   /* dense: the record is the wide one */
}

/* 28 bytes at b (any alignment) as 7 dwords, from three aligned 16-byte loads:
 * the replay's scattered per-lane reads then cost 3 load instructions instead
 * of one per byte (the batch buffer is 16-aligned and padded) */
__device__ __forceinline__ void load28(const uint8_t *b, uint32_t (&d)[7])
{
  typedef __attribute__((address_space(1))) const u32x4 gq;
  const uintptr_t a = (uintptr_t) b, l = a & ~(uintptr_t) 15;
  const u32x4 q0 = *reinterpret_cast<gq *>(l), q1 = *reinterpret_cast<gq *>(l + 16), q2 = *reinterpret_cast<gq *>(l + 32);
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

/* Case-insensitive compare of the first n <= 28 bytes of d (a header name
 * already in registers) with a lower-case literal: OR 0x20 folds letters; the
 * one non-letter, '-', could only collide with CR, which a parsed name cannot
 * hold (tchar only).  For a literal of letters only ("chunked") the compare is
 * exact for any bytes: x | 0x20 equals a lower-case letter only for that
 * letter and its upper case. */
template <uint32_t N>
__device__ __forceinline__ bool name_is(const uint32_t (&d)[7], const char (&lit)[N])
{
  constexpr uint32_t n = N - 1;
  uint32_t diff = 0;
#pragma unroll
  for (uint32_t j = 0; j < n; j++) diff |= (RHP_BYTE(d, j) | 0x20u) ^ (uint32_t) lit[j];
  return diff == 0;
}

/* strtoull over a header value of n bytes at s (rhp_scalar.h strtoull10), its
 * first 28 bytes already in d; the byte walk continues past them only for
 * longer values */
__device__ __forceinline__ uint64_t strtoull10_gpu(const uint8_t *s, const uint32_t (&d)[7], uint32_t n)
{
  uint32_t st = 0;
  bool neg = false, ovf = false;
  uint64_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < 28; j++) num_step(j < n ? RHP_BYTE(d, j) : 0u, st, neg, ovf, v);
  for (uint32_t j = 28; st != 2 && j < n; j++) num_step(s[j], st, neg, ovf, v);
  return ovf ? ~0ull : neg ? 0 - v : v;
}

/* http_frame (rhp_scalar.h) for the replay's common case, from the decode's
 * hints (cand, crec: see the decode state) -- GET, no candidate header, or one
 * or two candidates (the second's record is read from hdrs): the final record
 * is written, kFrameDone, unless the only Transfer-Encoding's value is
 * "chunked" (any case): kFrameChunked, the body (ret, len) is de-framed by the
 * replay's second pass.  Three or more candidates, or an overflowed candidate
 * set: kFrameSlow, http_frame.  Reads no method byte and, for one candidate,
 * no header record: on batches larger than the caches those re-reads are HBM
 * traffic.  The candidates' names and values are loaded together, one memory
 * round trip. */
enum : int { kFrameDone = 0, kFrameSlow = 1, kFrameChunked = 2 };
template <class Rec>
__device__ __forceinline__ int http_frame_fast(const uint8_t *b, uint64_t len, int32_t ret, rhp_http_t &x,
                                               uint32_t cand, uint32_t crec_lo, uint32_t crec_hi, Rec &&rec)
{
  const int64_t n = ret;
  rhp_http_t o = {1, 0, (uint64_t) n, 0};
  const uint32_t hdr = cand & 0x3fffffffu;
  if (!(cand & 0x40000000u) && hdr != 0) {   /* not GET (http.c:198-202), some candidate */
    const uint32_t rest = hdr & (hdr - 1u);
    if ((cand >> 31) || (rest & (rest - 1u)) != 0) return kFrameSlow;
    /* up to two candidates (a Content-Length beside a Transfer-Encoding is the
     * usual second one): the second's record is one more load, and all four
     * strings are read together.  A candidate's name is never RHP_NAME_NULL
     * (its length is 14 or 17). */
    uint32_t lo[2] = {crec_lo, 0u}, hi[2] = {crec_hi, 0u};
    if (rest) {
      const uint2 r = rec((uint32_t) __builtin_ctz(rest));   /* record of header index j (the second candidate) */
      lo[1] = r.x; hi[1] = r.y;
    }
    uint32_t dn[2][7], dv[2][7];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      if (c == 0 || rest) {
        load28(b + (lo[c] & 0xffffu), dn[c]);
        load28(b + (hi[c] & 0xffffu), dv[c]);
      }
    }
    /* the first Transfer-Encoding and the first Content-Length, in header order
     * (http.c:209-216); indices chosen by selects, not by a dynamic register
     * index */
    bool is_te[2], is_cl[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      is_te[c] = (c == 0 || rest) && (lo[c] >> 16) == 17u && name_is(dn[c], "transfer-encoding");
      is_cl[c] = (c == 0 || rest) && (lo[c] >> 16) == 14u && name_is(dn[c], "content-length");
    }
    const bool te1 = !is_te[0], cl1 = !is_cl[0];
    const bool has_te = is_te[0] || is_te[1], has_cl = is_cl[0] || is_cl[1];
    const uint32_t te_hi = te1 ? hi[1] : hi[0], cl_hi = cl1 ? hi[1] : hi[0];
    const bool te_set = has_te && (te_hi >> 16) != 0, cl_set = has_cl && (cl_hi >> 16) != 0;
    if (cl_set && te_set) {
      o.result = -1; o.consumed = 0;
    } else if (te_set) {
      /* Transfer-Encoding alone: "chunked" (http.c:221-224, data_equal_case)
       * de-frames the body, anything else is -1 */
      uint32_t dt[7];
#pragma unroll
      for (int j = 0; j < 7; j++) dt[j] = te1 ? dv[1][j] : dv[0][j];
      if ((te_hi >> 16) == 7u && name_is(dt, "chunked")) return kFrameChunked;
      o.result = -1; o.consumed = 0;
    } else if (cl_set) {
      uint32_t dc[7];
#pragma unroll
      for (int j = 0; j < 7; j++) dc[j] = cl1 ? dv[1][j] : dv[0][j];
      const uint64_t size = strtoull10_gpu(b + (cl_hi & 0xffffu), dc, cl_hi >> 16);
      if (len < (uint64_t) n + size) {
        o.result = 0; o.consumed = 0;
      } else {
        o.body_kind = 1; o.body_len = size; o.consumed = (uint64_t) n + size;
      }
    }
  }
  x = o;
  return kFrameDone;
}

enum : uint32_t { kMoveChunks = 8, kStageBody = 2048, kStageBodies = 4 };

/* A chunked body's validation (http_dechunk's first pass, http.c:134-150) as
 * a walk one size line per step: a step parses the 17-20 bytes from the line's
 * start (one_chunk_window; a longer line goes to one_chunk_t) in the two
 * aligned lines the previous step loaded, and loads the next line's.  The walk keeps
 * the first kMoveChunks chunks' data spans.  One step per memory round trip:
 * the replay runs the next round's walks inside this round's payload moves
 * (staged_moves), one step per body group, so the walk's chain of round trips
 * hides behind the moves. */
struct ChunkWalk {
  uint8_t *in;          /* the body's first byte */
  uint64_t size, off;   /* bytes of the body; the next size line's offset */
  uint64_t sum, region; /* data bytes; framed bytes up to the last data byte */
  int32_t res;          /* when done: 1 valid, 0 need more, -1 malformed */
  uint32_t k;           /* data chunks */
  uint32_t span[kMoveChunks];   /* chunk c's data: (off | len << 16) from `in` (exact while region <= 0xffff) */
  bool live;
  u32x4 q[2];           /* the two aligned lines from the next size line's start, loading */
  __device__ __forceinline__ void issue()
  {
    typedef __attribute__((address_space(1))) const u32x4 gq;
    const uintptr_t l = (uintptr_t) (in + off) & ~(uintptr_t) 15;
#pragma unroll
    for (int j = 0; j < 2; j++) q[j] = *reinterpret_cast<gq *>(l + 16 * j);
  }
  __device__ __forceinline__ void begin(uint8_t *body, uint64_t n)
  {
    in = body; size = n; off = sum = region = 0; res = 0; k = 0; live = true;
    issue();
  }
  __device__ __forceinline__ void step()
  {
    if (!live) return;
    const uintptr_t a = (uintptr_t) (in + off);
    const uint32_t w[9] = {q[0][0], q[0][1], q[0][2], q[0][3], q[1][0], q[1][1], q[1][2], q[1][3], 0u};
    const uint32_t qd = (uint32_t) (a >> 2) & 3u, sh = (uint32_t) a & 3u;
    uint32_t x[6], W[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 6; m++) x[m] = qd == 0 ? w[m] : qd == 1 ? w[m + 1] : qd == 2 ? w[m + 2] : w[m + 3];
#pragma unroll
    for (int m = 0; m < 5; m++) W[m] = __builtin_amdgcn_alignbyte(x[m + 1], x[m], sh);
    int64_t r;
    uint64_t doff = 0, dlen = 0;
    /* W holds 20 bytes from the line's start, of them 32 - (a & 15) >= 17 in the two lines */
    /* the common line without a byte loop (one_chunk_head), else the windowed
     * state machine, else the byte-wise parse past the window */
    const uint32_t nw = min(20u, 32u - ((uint32_t) a & 15u));
    if (!one_chunk_head<5>(W, nw, size - off, &r, &doff, &dlen) && !one_chunk_window(W, nw, size - off, &r, &doff, &dlen)) {
      LineBytes B{in, ~0ull, {0, 0, 0, 0}};
      r = one_chunk_t(B, off, size, &doff, &dlen);
    }
    if (r <= 0) {
      res = (int32_t) r;
      live = false;
      return;
    }
    if (dlen) {
      const uint32_t sp = (uint32_t) (off + doff) | (uint32_t) dlen << 16;
#pragma unroll
      for (uint32_t j = 0; j < kMoveChunks; j++) span[j] = j == k ? sp : span[j];   /* every element stored: no indexed store */
      k++;
      region = off + doff + dlen;
    }
    off += (uint64_t) r;
    sum += dlen;
    if (!dlen) {   /* the last chunk */
      res = 1;
      live = false;
      return;
    }
    issue();
  }
};

/* The body's record and payload moves once its walk is done (http.c:150-160).
 * The moves -- each chunk's data down to the running body end, in order --
 * go one of two ways:
 *  - staged by the wave (staged_moves, below), when the body has at most
 *    kMoveChunks chunks and its framed bytes fit a kStageBody slot: the spans
 *    go to *sb and the function returns true;
 *  - by this thread (DevMove from the kept spans, or from a second walk of
 *    the size lines for a body of more chunks or beyond 64 KiB), returning
 *    false. */
struct StagedBody {
  uint64_t base;           /* the body's first byte: the de-framed body goes to [base, base + len) */
  uint32_t nch, region;    /* data chunks; framed bytes up to the last data byte */
  uint32_t size;           /* the body's bytes up to the request's end (capped at 2 * kStageBody) */
  uint32_t span[kMoveChunks];   /* chunk c: its slot shift src - dst | the body offset where chunk c + 1 starts << 16
                                   (a chunk past the body's: 0 | L << 16; both < kStageBody) */
};
__device__ __forceinline__ bool finish_chunked(const ChunkWalk &w, int32_t ret, rhp_http_t *x, bool compact,
                                               StagedBody *sb)
{
  rhp_http_t o = {1, compact ? 1u : (uint32_t) RHP_BODY_CHUNKED_PENDING, 0, 0};
  if (w.res <= 0) {
    o.result = (int32_t) w.res;
    *x = o;
    return false;
  }
  o.body_len = w.sum;
  o.consumed = (uint64_t) ret + w.off;
  *x = o;
  if (!compact) return false;
  if (sb && w.k <= kMoveChunks && ((uint32_t) (uintptr_t) w.in & 15u) + w.region + 20u <= kStageBody) {
    sb->base = (uint64_t) (uintptr_t) w.in;
    sb->nch = w.k;
    sb->region = (uint32_t) w.region;
    sb->size = (uint32_t) min(w.size, (uint64_t) (2 * kStageBody));
    uint32_t cdv = 0;   /* the chunk table entries of staged_moves: dl | cd_next << 16 (see StagedBody) */
#pragma unroll
    for (uint32_t j = 0; j < kMoveChunks; j++) {
      const uint32_t sp = j < w.k ? w.span[j] : 0u;
      const uint32_t dl = j < w.k ? (sp & 0xffffu) - cdv : 0u;
      cdv += sp >> 16;
      sb->span[j] = dl | cdv << 16;
    }
    return true;
  }
  DevMove M{w.in};
  uint64_t total = 0;
  if (w.k <= kMoveChunks && w.region <= 0xffffu) {
#pragma unroll
    for (uint32_t j = 0; j < kMoveChunks; j++) {
      if (j < w.k) {
        M(total, w.span[j] & 0xffffu, w.span[j] >> 16);
        total += w.span[j] >> 16;
      }
    }
    return false;
  }
  LineBytes B{w.in, ~0ull, {0, 0, 0, 0}};
  uint64_t off = 0, doff = 0, dlen = 0;
  do {
    const int64_t res = one_chunk_t(B, off, w.size, &doff, &dlen);
    M(total, off + doff, dlen);
    off += (uint64_t) res;
    total += dlen;
  } while (dlen);
  return false;
}

/* a chunked body walked and finished by this thread alone */
__device__ __forceinline__ bool frame_chunked(uint8_t *b, uint64_t len, int32_t ret, rhp_http_t *x, bool compact,
                                              StagedBody *sb = nullptr)
{
  ChunkWalk w;
  w.begin(b + ret, len - (uint64_t) ret);
  while (w.live) w.step();
  return finish_chunked(w, ret, x, compact, sb);
}

/* The wave's payload moves for the bodies of the lanes in `m` (their spans in
 * those lanes' *sb), kStageBodies bodies per group:
 *  1. the wave loads each body's framed bytes [base & ~15, base + region) as
 *     whole 16-byte lines, 64 lanes side by side (1 KiB per instruction, every
 *     line fetched once), and writes them to the body's LDS slot; the next
 *     group's lines are loaded while this group is built;
 *  2. lane j builds the j-th aligned 16-byte block of the de-framed body: body
 *     offset t lies at slot offset lead + t + delta(c), delta(c) = src(c) -
 *     dst(c) for the chunk c holding t, so the block is five dwords read at the
 *     lane's own slot address and funnel-shifted (the chunk of its first byte),
 *     with the bytes from the next chunk's start on taken the same way from
 *     that chunk (rarely a third: a general pass over the chunks), and stored:
 *     1 KiB of contiguous lines per wave store, only the body's bytes in the
 *     first and last block.
 * Every global load of a group lands before its stores (each chunk's data lies
 * at or past its destination, and bodies do not overlap).  Slot reads stay
 * below lead + region + 20 <= kStageBody (frame_chunked's staging test). */
/* bytes of a wave's chunk tables (staged_moves: one per body slot) */
constexpr uint32_t kChunkTab = 4u * (kMoveChunks + 1u), kChunkTabWave = kChunkTab * kStageBodies;
template <class Step>
__device__ __forceinline__ void staged_moves(uint64_t m, const StagedBody &sb, uint32_t lane, uint32_t stage, uint32_t ctab,
                                             Step &&step)
{
  typedef __attribute__((address_space(1))) const u32x4 gq;
  typedef __attribute__((address_space(1))) u32x4 gw;
  typedef __attribute__((address_space(1))) uint8_t gb1;
  typedef __attribute__((address_space(1))) uint32_t gw1;
  typedef __attribute__((address_space(3))) u32x4 lq;
  typedef __attribute__((address_space(3))) const uint32_t l1;
  constexpr uint32_t kLinesPerLane = kStageBody / 1024u;   /* 16-byte lines per lane per body */
  struct Group {
    uint32_t owner[kStageBodies];   /* the lane whose body slot q holds (a valid lane for an empty slot) */
    uint32_t have;                  /* bit q: slot q holds a body */
    uint32_t wide;                  /* bit q: slot q's body has lines past the first 64 (their loads were made) */
  };
  auto take = [&](Group &g) {
    g.have = 0;
#pragma unroll
    for (uint32_t q = 0; q < kStageBodies; q++) {
      g.owner[q] = m ? (uint32_t) __builtin_ctzll(m) : g.owner[0];
      if (m) g.have |= 1u << q;
      m &= m - 1u;   /* 0 stays 0 */
    }
  };
  auto base_of = [&](uint32_t owner) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t) sb.base, owner);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t) (sb.base >> 32), owner);
    return (uint64_t) lo | (uint64_t) hi << 32;
  };
  typedef u32x4 Lines[kStageBodies][kLinesPerLane];
  /* a group's framed lines (lines past a body's region load its first line;
   * an empty slot loads its group's first body's first line) */
  auto load = [&](Group &g, Lines &raw) {
    g.wide = 0;
#pragma unroll
    for (uint32_t q = 0; q < kStageBodies; q++) {
      const uint64_t base = base_of(g.owner[q]);
      const uint32_t region = (g.have >> q & 1u) ? __builtin_amdgcn_readlane(sb.region, g.owner[q]) : 0u;
      const uint64_t la = base & ~(uint64_t) 15;
      const uint32_t lines = (((uint32_t) base & 15u) + region + 15u) >> 4;   /* 32-bit: region < kStageBody */
#pragma unroll
      for (uint32_t h = 0; h < kLinesPerLane; h++) {
        const uint32_t line = lane + 64u * h;
        if (h == 0 || 64u * h < lines) {   /* wave-uniform: a body of at most 64 lines loads one line per lane */
          raw[q][h] = *reinterpret_cast<gq *>((uintptr_t) (la + (line < lines ? 16u * line : 0u)));
          if (h) g.wide |= 1u << q;
        }
      }
    }
  };
  /* five slot dwords at the lane's byte position P, funnel-shifted to P */
  auto fetch = [&](uint32_t slot, uint32_t P) {
    const l1 *d = reinterpret_cast<const l1 *>((size_t) (slot + (P & ~3u)));
    const uint32_t w0 = d[0], w1 = d[1], w2 = d[2], w3 = d[3], w4 = d[4], r = P & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
                 __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r)};
  };
  /* out's bytes k >= s (0 < s < 16) from o */
  /* the bytes k >= s (0 <= s <= 16) of a 16-byte block as a mask: two 64-bit
   * shifts and their selects, not a clamp and shift per dword */
  auto from_mask = [](int32_t s) -> u32x4 {
    const uint32_t a = 8u * (uint32_t) min(max(s, 0), 16);   /* bits below the first byte taken */
    const uint64_t lo = a >= 64u ? 0ull : ~0ull << a;
    const uint64_t hi = a <= 64u ? ~0ull : a >= 128u ? 0ull : ~0ull << (a - 64u);
    return u32x4{(uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32)};
  };
  auto merge_from = [&](u32x4 &out, const u32x4 &o, int32_t s) {
    const u32x4 msk = from_mask(s);
#pragma unroll
    for (int j = 0; j < 4; j++) out[j] = (o[j] & msk[j]) | (out[j] & ~msk[j]);
  };
  auto build = [&](uint32_t q, uint32_t owner) {
    const uint64_t base = base_of(owner);
    /* the body's chunk table T[c] = dl[c] | cd[c + 1] << 16 (dl: chunk c's slot
     * shift src - dst, cd: body offsets of the chunk starts; finish_chunked
     * packed them), T[kMoveChunks] = L << 16 */
    uint32_t T[kMoveChunks];
#pragma unroll
    for (uint32_t c = 0; c < kMoveChunks; c++) T[c] = __builtin_amdgcn_readlane(sb.span[c], owner);
    const int32_t L = (int32_t) (T[kMoveChunks - 1] >> 16);   /* spans past the body's chunks are empty */
    const int32_t size = (int32_t) __builtin_amdgcn_readlane(sb.size, owner);
    const uint32_t lead = (uint32_t) base & 15u;
    const uint64_t a0 = base - lead;
    const uint32_t blocks = (lead + (uint32_t) L + 15u) >> 4;
    const uint32_t slot = stage + kStageBody * q;
    /* The table in LDS, written by one lane: a lane reads its block's chunk c
     * and the next one as T[c], T[c + 1] with one ds_read2_b32 instead of
     * selecting them from the scalars (a select chain with a v_mov per scalar
     * operand: ~70 instructions per block, chunked config) */
    typedef __attribute__((address_space(3))) uint32_t lq1;
    typedef __attribute__((address_space(3))) u32x4 lq4;
    const uint32_t tab = ctab + kChunkTab * q;
    if (lane == 0) {
      *reinterpret_cast<lq4 *>((size_t) tab) = u32x4{T[0], T[1], T[2], T[3]};
      *reinterpret_cast<lq4 *>((size_t) (tab + 16u)) = u32x4{T[4], T[5], T[6], T[7]};
      *reinterpret_cast<lq1 *>((size_t) (tab + 32u)) = (uint32_t) L << 16;
    }
    __builtin_amdgcn_wave_barrier();   /* the wave's LDS accesses stay in order: every lane reads T after lane 0 wrote it */
    for (uint32_t b = lane; b < blocks; b += 64u) {
      /* block b: body offsets [t0, t0 + 16); chunk c holds its first byte (the
       * chunks past nch start at L > t0: they never count) */
      const int32_t t0 = (int32_t) (16u * b) - (int32_t) lead;
      uint32_t c = 0;
      /* chunk j >= 1 starts at or below t0 (cd[j] = T[j - 1] >> 16 <= t0): compared on
       * the packed entry against t0 << 16 | 0xffff, so the boundaries need no unpacking;
       * a chunk start is >= 1 (entries >= 1 << 16), so t0 < 0 compares against 0 */
      const uint32_t t0u = t0 < 0 ? 0u : (uint32_t) t0 << 16 | 0xffffu;
#pragma unroll
      for (uint32_t j = 1; j < kMoveChunks; j++) c += T[j - 1] <= t0u ? 1u : 0u;
      const uint32_t T0 = *reinterpret_cast<const lq1 *>((size_t) (tab + 4u * c));
      uint32_t Tn = *reinterpret_cast<const lq1 *>((size_t) (tab + 4u * c + 4u));
      u32x4 out = fetch(slot, 16u * b + (T0 & 0xffffu));
      /* the chunks that start inside the block, in order (usually none or one;
       * a chunk of < 16 bytes brings the next): chunk j's bytes from its start
       * e on (T[j - 1] >> 16 = cd[j]; a real chunk while e < L) */
      int32_t ej = (int32_t) (T0 >> 16);
      uint32_t tj = tab + 4u * c + 8u;
      bool more = ej < L && ej < t0 + 16;
      while (__builtin_amdgcn_ballot_w64(more)) {
        if (more) {
          merge_from(out, fetch(slot, 16u * b + (Tn & 0xffffu)), ej - t0);
          ej = (int32_t) (Tn >> 16);
          more = ej < L && ej < t0 + 16;
          if (more) {
            Tn = *reinterpret_cast<const lq1 *>((size_t) tj);
            tj += 4u;
          }
        }
      }
      const uintptr_t A = (uintptr_t) (a0 + 16u * b);
      /* the body's first and last block keep the bytes around the body: the
       * slot holds this line as it is in memory, and where the line lies in
       * the request (its header bytes before the body, its framing after) the
       * whole line is stored, those bytes unchanged; a line reaching into the
       * next request is written byte by byte (the caller may be filling that
       * request while this one parses) */
      const bool inner = t0 >= 0 && t0 + 16 <= L;
      const bool whole = inner || t0 + 16 <= size;
      if (!inner && whole) {
        const u32x4 orig = *reinterpret_cast<const lq *>((size_t) (slot + 16u * b));
        /* the body's bytes [kb, ke) of the block from out, the rest as in memory */
        const u32x4 mb = from_mask(-t0), me = from_mask(L - t0);
#pragma unroll
        for (int32_t j = 0; j < 4; j++) {
          const uint32_t msk = mb[j] & ~me[j];
          out[j] = (out[j] & msk) | (orig[j] & ~msk);
        }
      }
      if (whole) {
        *reinterpret_cast<gw *>(A) = out;
      } else {   /* only the body's bytes */
        const int32_t kb = max(-t0, 0), ke = min(L - t0, 16);
#pragma unroll
        for (int32_t j = 0; j < 4; j++) {
          if (kb <= 4 * j && 4 * j + 4 <= ke) {
            *reinterpret_cast<gw1 *>(A + 4 * j) = out[j];
          } else {
#pragma unroll
            for (int32_t z = 0; z < 4; z++)
              if (4 * j + z >= kb && 4 * j + z < ke) *reinterpret_cast<gb1 *>(A + 4 * j + z) = (uint8_t) (out[j] >> (8 * z));
          }
        }
      }
    }
  };
  auto to_slots = [&](const Group &g, const Lines &raw) {
#pragma unroll
    for (uint32_t q = 0; q < kStageBodies; q++)
#pragma unroll
      for (uint32_t h = 0; h < kLinesPerLane; h++)
        if (h == 0 || (g.wide >> q & 1u))   /* lines past a body's region were not loaded: their slot bytes are not read */
          *reinterpret_cast<lq *>((size_t) (stage + kStageBody * q + 16u * (lane + 64u * h))) = raw[q][h];
    wait_lgkm0();   /* the wave's slots are written (a wave reads its own) */
  };
  auto build_group = [&](const Group &g) {
#pragma unroll
    for (uint32_t q = 0; q < kStageBodies; q++)
      if (g.have >> q & 1u) build(q, g.owner[q]);
  };
  Lines ra;
  Group g;
  take(g);
  load(g, ra);
  while (g.have) {
    to_slots(g, ra);
    step();   /* the caller's per-group work (the next round's walks): its loads go out before the next group's */
    Group gn;
    take(gn);
    if (gn.have) load(gn, ra);   /* in flight while this group is built (a second group in flight: slower) */
    build_group(g);
    g = gn;
  }
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

/* one byte of LDS at address a (the table is at LDS address 0) */
__device__ __forceinline__ uint32_t lds_u8(uint32_t a)
{
  return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t *>((size_t) a);
}

/* LDS address of pair index st's entry for code c (rhp_dfa.h row geometry):
 * st * 256 + c is one v_perm; another stride one v_mad_u32_u24 */
__device__ __forceinline__ uint32_t row_addr(uint32_t st, uint32_t c)
{
  if constexpr (kStride == 256u) return __builtin_amdgcn_perm(st, c, 0x0c0c0400u);
  else return __umul24(st, kStride) + c;
}

/* keep the compiler from sinking the computation of x into a branch */
__device__ __forceinline__ void opaque(uint32_t &x) { asm("" : "+v"(x)); }

/* Write-through record stores.  With `wt` (a wave-uniform flag) the loop's
 * record stores carry sc1: the line goes to memory and leaves L2, so a launch
 * ends with no dirty record lines for the kernel boundary's L2 write-back to
 * drain (MI355X_MICROARCH.md, store flavours and the boundary row).  That pays
 * where a wave's records are whole lines -- header-major or compact records of
 * a range whose requests are even (config 2: 70.2 -> 67.1 us, the ceiling
 * ubench 53.9 -> 52.1 us, profiles/r04/) -- and costs where they are not:
 * request-major records, or an uneven range's (config 3 +12 %), whose partial
 * lines plain stores merge in L2 first; http records gained nothing (+2 %).
 * The host enables it per launch (Params::wt_records), the kernel per range. */
#define RHP_STORE_LANES(INSN, mask, dst, v, wt)                                                   \
  do {                                                                                            \
    uint64_t saved_;                                                                              \
    if (wt)                                                                                       \
      asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, %1\n\t" INSN " %2, %3, off sc1\n\t"     \
                   "s_mov_b64 exec, %0\n\ts_nop 1"                                              \
                   : "=&s"(saved_) : "s"(mask), "v"(dst), "v"(v) : "memory");                    \
    else                                                                                          \
      asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, %1\n\t" INSN " %2, %3, off\n\t"         \
                   "s_mov_b64 exec, %0\n\ts_nop 1"                                              \
                   : "=&s"(saved_) : "s"(mask), "v"(dst), "v"(v) : "memory");                    \
  } while (0)

/* one header record (8 B) for the lanes in `mask` (a ballot), as straight-line
 * code: exec is restored before the asm ends; the trailing s_nop covers the
 * store-data read hazard */
__device__ __forceinline__ void store_rec_lanes(uint64_t mask, rhp_hdr_t *dst, u32x2 v, bool wt)
{
  RHP_STORE_LANES("global_store_dwordx2", mask, dst, v, wt);
}
/* the same for a compact header record (RHP_LAYOUT_COMPACT: name_len |
 * value_len << 16) */
__device__ __forceinline__ void store_len_lanes(uint64_t mask, uint32_t *dst, uint32_t v, bool wt)
{
  RHP_STORE_LANES("global_store_dword", mask, dst, v, wt);
}
/* the same for a dense header record (RHP_LAYOUT_DENSE: name_len | value_len << 6) */
__device__ __forceinline__ void store_len16_lanes(uint64_t mask, uint16_t *dst, uint32_t v, bool wt)
{
  RHP_STORE_LANES("global_store_short", mask, dst, v, wt);
}
/* a dense header record (RHP_LAYOUT_DENSE: name_len | value_len << 6) for the
 * lanes in `mask`; one whose lengths do not fit stores RHP_DENSE_OVERFLOW and
 * its u32 lengths in the overflow area (rare: the lanes that need it, after a
 * ballot) */
__device__ __forceinline__ void store_dense_lanes(uint64_t mask, const Params &p, uint32_t hx, uint32_t nlen, uint32_t vlen, bool wt)
{
  const bool fits = max(nlen << 4, vlen) <= RHP_DENSE_VALUE_MAX;
  store_len16_lanes(mask, p.lens16 + hx, fits ? nlen | vlen << 6 : RHP_DENSE_OVERFLOW, wt);
  const uint64_t over = mask & __builtin_amdgcn_ballot_w64(!fits);
  if (over) store_len_lanes(over, p.ovf32 + hx, nlen | vlen << 16, false);
}
/* the request record (16 B) for the active lanes */
__device__ __forceinline__ void store_req(rhp_req_t *dst, u32x4 v, bool wt)
{
  if (wt) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
  else *GLOBAL(u32x4, dst) = v;
}
__device__ __forceinline__ void store_http(rhp_http_t *dst, const rhp_http_t &x)
{
  typedef uint32_t u32x2a8 __attribute__((ext_vector_type(2), aligned(8)));
  u32x2a8 v[3];
  __builtin_memcpy(v, &x, sizeof x);
  __attribute__((address_space(1))) u32x2a8 *q = GLOBAL(u32x2a8, dst);
  q[0] = v[0];
  q[1] = v[1];
  q[2] = v[2];
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
 *
 * Per lane there are two requests in flight: the one being WALKED (wcur: the
 * window that landed this iteration) and the one being DECODED (dcur: the
 * events of the window walked in the previous iteration) -- the same request
 * unless the lane switched between the two windows.
 */
/* REC: the records the loop writes: 0 rhp_hdr_t (request- or header-major), 1
 * compact (u32 lengths; http mode: compact http records too), 2 dense (u16
 * lengths and 8-byte request records, phr mode) */
enum : int { kRecWide = 0, kRecCompact = 1, kRecDense = 2 };
template <int WAVES, bool LATE, bool HTTP, int REC>
__global__ __launch_bounds__(WAVES * 64, RHP_WAVES_PER_SIMD) void rhp_dfa_kernel(Params p)
{
  constexpr bool COMPACT = REC != kRecWide;   /* lengths, offsets by the running sum */
  constexpr bool DENSE = REC == kRecDense;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  Diag dg;   /* diagnostic builds only; nothing in product builds */
  dg.entry();
  dg.clock_start();

  const uint32_t maxh = p.max_headers;
  constexpr bool http = HTTP;   /* p.mode == RHP_MODE_HTTP (the launch picks the instance) */
  /* Window geometry.  Windows are 128 bytes (whole HBM lines).  The http form
   * can walk kHttpXParts 16-byte parts more (RHP_HTTP_XPARTS, rhp_dfa.h), so a
   * header section that fits (config 5: 133 B) is walked, decoded and framed in
   * one iteration where 128 B takes two; the extension parts go to a staging
   * area of their own (xstage: part 8 + k of every lane's window at 1024 k +
   * 16 lane), fetched by kXParts more LDS-DMA loads per issue, and the
   * staging leaves room for 12 waves.  Measured with 2 parts (160 B,
   * profiles/r04/e/): config 5 +2-4 % (the fewer waves cost more than the
   * iterations saved) and no fewer bytes fetched (the 32 B of the next line
   * cost its whole line), so the default is 0. */
  constexpr uint32_t kXParts = (LATE && HTTP) ? kHttpXParts : 0u;
  /* Phase lock (http form, RHP_PHASE_LOCK): a lane walks the first window of a
   * request only on even iterations.  Header sections of one or two windows
   * (config 5: 133 B) then keep every lane of a wave in step -- first windows on
   * even iterations, second windows on odd ones -- and on an odd iteration
   * every lane reaches its terminal within the window's first parts, where the
   * walk stops (walk()).  A lane whose request ended in its first window idles
   * one iteration; without the lock the lanes drift out of step after the
   * first such request and no walk ever stops early. */
  constexpr bool kPhaseLock = RHP_PHASE_LOCK && LATE && HTTP;
  uint32_t it_odd = 0;   /* wave-uniform: this iteration's number is odd */
  constexpr uint32_t kWParts = kParts + kXParts;   /* 16-byte parts per window */
  constexpr uint32_t kWBlock = 16u * kWParts;      /* window bytes */
  constexpr uint32_t kWEv = kWBlock / 32u;         /* 32-bit event words per window */
  static_assert(kWBlock % 32u == 0, "whole event words per window");

  /* ---- request pool ----
   * Workgroup g owns requests [g*span, (g+1)*span) (host: span = n / grid).
   * Lanes that need their next request take it from the workgroup's LDS
   * counter (one atomic per wave and refill, for all of the wave's lanes that
   * need one), so the waves of a workgroup drain one shared range request by
   * request and finish together; no global atomic is ever touched.
   * Window addresses are u32 byte offsets from `base` (the 4-aligned start of
   * the range; a range below 4 GiB is checked after the prologue loads). */
  const uint32_t wg_lo = min(blockIdx.x * p.span, p.n), wg_hi = min(wg_lo + p.span, p.n);
  /* the first WAVES * 64 requests of the range go to the threads in order
   * (first_n); refills hand out the rest from the LDS counter */
  const uint32_t first_n = min(wg_hi - wg_lo, (uint32_t) (WAVES * 64));
  uint32_t *wg_counter = reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave);
  uint32_t *wg_deferred = wg_counter + 1;   /* some request of the range needs the replay */
  /* Longest first.  With lengths as uneven as config 3's, the requests drawn
   * last decide when a wave finishes: a lane's last requests (the one it walks
   * and the one it holds) are committed when the pool runs dry, so an uneven
   * range is handed out in descending window count (a counting sort over the
   * range before the first hand-out, in the idle waves' staging buffers): the
   * longest start at iteration 0, the last ones handed out are the shortest.
   * Ranges above kOrderSpan keep plain order. */
  const bool order_on = wg_hi - wg_lo <= kOrderSpan;
  bool sorted = false;   /* refills take the range in `order` (an uneven range) */
  bool pool_dry = wg_lo >= wg_hi;
  /* The prologue's global reads all go out at once (one round trip): the
   * table, the range's end offsets and every thread's first request. */
  u32x4 tab[(kTable2Bytes / 16 + WAVES * 64 - 1) / (WAVES * 64)];
  {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(&g_table);
#pragma unroll
    for (uint32_t j = 0; j < sizeof tab / sizeof tab[0]; j++) {
      const uint32_t k = tid + j * WAVES * 64;
      if (k < kTable2Bytes / 16) tab[j] = src[k];
    }
  }
  const uint64_t o_lo = pool_dry ? 0 : p.offsets[wg_lo], o_hi = pool_dry ? 0 : p.offsets[wg_hi];
  /* Window starts.  phr mode fetches a request's first window from the
   * 128-byte line holding its first byte (kLead = 127: up to 127 bytes before
   * the request are walked in S_PRE, zeroed), so every window is a whole HBM
   * line (a 128-byte aligned buffer: lines are counted from p.bytes, so the
   * geometry, and with it the rare choice between the DFA and the exact path
   * the emulator mirrors, does not depend on the buffer's address) and no line
   * is fetched by two windows of one request.  http mode fetches from the dword
   * holding it (kLead = 3): its requests are framed from the window (the GET
   * check, frame_window) at positions the 4-byte alignment keeps in the first
   * part. */
  constexpr uint32_t kLead = HTTP ? 3u : 127u;
  const uint64_t base = o_lo & ~(uint64_t) kLead;
  if (o_hi - base >= 0xFFFF0000ull) {
    /* The window offsets below are u32 from `base`: a workgroup whose range
     * spans ~4 GiB (a request of that size among its requests) parses its
     * range with the exact path, one request per thread.  Every other range of
     * the batch, wherever it lies, runs the DFA. */
    for (uint32_t i = wg_lo + tid; i < wg_hi; i += WAVES * 64) {
      const uint64_t off = p.offsets[i];
      finish_exact(p, i, off, p.offsets[i + 1] - off);
    }
    return;
  }
  const uint8_t *wbytes = p.bytes + base;
  /* the range's bytes as a raw buffer: window loads take 32-bit offsets from
   * base (the range is below 4 GiB, checked above), no 64-bit address per load */
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(wbytes), 0, -1, 0x00020000);

  /* ---- walk state (the request whose window landed) ---- */
  uint32_t st = kPark;                 /* table index (rhp_dfa.h idx2) */
  int32_t wpos = 0;                    /* request-relative position of the window's first byte */
  bool wact = false;                   /* wcur is live: its walk has not ended */
  uint32_t wcur = 0, wlen = 0, wget = 0, cur_ptr = 0;
  uint32_t wlead = 0;                  /* bytes before wcur in its first window (wnew) */
  uint32_t woff = 0;                   /* wcur's first byte, offset from base (LATE http framing) */
  uint32_t ev[kWEv];                   /* events of the window being walked (32 bytes per word) */
  bool pend_ok = false;                /* pend: the lane's next request */
  uint32_t pend = 0;
  uint32_t pend_o0 = 0, pend_o1 = 0;   /* low dwords of offsets[pend], offsets[pend+1] as loaded */
  uint32_t nw = 0;                     /* next window: byte offset from base | kind (0 none, 1
                                          continuation, 2 first window of pend); windows are 4-aligned */
  u32x4 W[kWParts];                    /* the window in registers */
  const uint32_t stage = __builtin_amdgcn_readfirstlane(kLdsTable + (tid >> 6) * kStageWave);   /* wave-uniform */
  /* the extension parts of the wave's windows (kXParts > 0): after the pool area */
  const uint32_t xstage = __builtin_amdgcn_readfirstlane(kLdsTable + WAVES * kStageWave + kPoolBytes + 4u * kOrderBuckets +
                                                         (tid >> 6) * 1024u * kXParts);
  /* the first window of the request starting at (low dword) o0, offset from
   * base, and the number of bytes before the request in it (see kLead) */
  auto first_win = [&](uint32_t o0) -> uint32_t { return (o0 - (uint32_t) base) & ~kLead; };
  auto lead_of = [&](uint32_t o0) -> uint32_t { return (o0 - (uint32_t) base) & kLead; };
  /* LDS address of part q of this lane's window */
  auto part_lds = [&](uint32_t q) -> uint32_t {
    return q < kParts ? stage + stage_off(lane, q) : xstage + 1024u * (q - kParts) + 16u * lane;
  };

  /* ---- decode state (the request whose previous window is decoded) ----
   *   kn   request-line events consumed (0 ME, 1 PE, 2 RL, 3 done) | minor << 3
   *   me, pe  positions of ME and PE (method end, path end)
   *   rl   method_len | path_len << 16
   *   nh   header records completed;  ls: start of the open header line
   *   t    1: the open line's colon (CO at pco) was seen, its LF not yet
   *   ovf  0, or 1 + the line start at which max_headers overflowed
   * http mode, framing hints for the replay: cand bits 0..29 = headers whose
   * name length is 14 or 17 (bit 31: such a header at index >= 30), bit 30 =
   * the method is GET; crec = the first such header's record */
  bool dhas = false;
  uint32_t dcur = 0, dlen = 0, st_prev = kPark, doff = 0;
  int32_t dpos = 0;                    /* position of the decoded window's first byte */
  uint32_t evp[kWEv];                  /* its events */
  uint32_t kn = 0, me = 0, pe = 0, rl = 0, nh = 0, ls = 0, t = 0, pco = 0, ovf = 0;
  uint32_t cand = 0, crec_lo = 0, crec_hi = 0;
  /* http framing in the late-issue kernel (http.c:196-218), from the
   * staging buffer while the decoded window is still in it: the request's
   * first framing candidate (a header whose name is 14 or 17 bytes long) is
   * evaluated when its record completes -- or, when its line is still open
   * at the window's end, its name and the value bytes so far are, the value's
   * number carried into the next window.  fr flags (kFr*), fv the number. */
  uint32_t fr = 0;
  uint64_t fv = 0;
#pragma unroll
  for (int w = 0; w < (int) kWEv; w++) ev[w] = evp[w] = 0;

  /* give every lane without a pending request one from the pool; the offsets
   * loads are only consumed at the top of the next block */
  auto take = [&](uint32_t i) {
    /* only the low dwords: the range is below 4 GiB, so offsets relative to
     * `base` and lengths are exact modulo 2^32 */
    const uint32_t *o = reinterpret_cast<const uint32_t *>(p.offsets + i);
    pend = i;
    pend_o0 = *GLOBAL(const uint32_t, o);
    pend_o1 = *GLOBAL(const uint32_t, o + 2);
    pend_ok = true;
  };
  /* an uneven range's order: the range's requests (u16, range-relative) by
   * descending window count, then the histogram / bucket cursors */
  /* in the last waves' staging: one wave's for a range of up to kStageWave / 2
   * requests (config 3 at 1M: 4096 per workgroup), two waves' up to kOrderSpan */
  const uint32_t order_waves = 2u * (wg_hi - wg_lo) <= kStageWave ? 1u : kOrderWaves;
  uint16_t *order = reinterpret_cast<uint16_t *>(lds + kLdsTable + (WAVES - order_waves) * kStageWave);
  uint32_t *bucket = reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave + kPoolBytes);   /* past the pool */
  static_assert(2 * kOrderSpan <= kOrderWaves * kStageWave, "the order fits the last kOrderWaves waves' staging");
  auto refill_pend = [&]() {
    /* Just in time (early form, longest-first ranges): a lane takes its next
     * request only when its current one has at most two windows left -- the
     * pending request's offsets must have landed by the iteration that issues
     * its first window, no earlier commitment is needed.  A lane deep in a long
     * request leaves the pool to the lanes that finish first, so the range
     * stays longest first per lane, not per hand-out round (config 3 -4.5 %). */
    const bool need = !pend_ok && !(!LATE && sorted && wact && wpos + (int32_t) (2u * kBlock) < (int32_t) wlen);
    uint64_t want = __ballot(need);
    if (!want || pool_dry) return;
    const uint32_t cnt = (uint32_t) __popcll(want);
    uint32_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(wg_counter, cnt);
    b0 = wg_lo + __builtin_amdgcn_readfirstlane(b0);
    if (b0 + cnt >= wg_hi) pool_dry = true;
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) want, 0));
    const uint32_t i = b0 + rank;
    if (need && i < wg_hi) take(sorted ? wg_lo + order[i - wg_lo] : i);
  };

  /* the longest-first order of an uneven range (see order_on): a counting sort
   * by window count, descending; every thread of the workgroup takes part (the
   * caller's barriers: the histogram zeroed before, the order complete after) */
  const uint32_t span_n = wg_hi - wg_lo;
  auto sort_range = [&]() {
    constexpr uint32_t kPer = kOrderSpan / (WAVES * 64);   /* requests per thread */
    uint32_t wc[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
      const uint32_t k = tid + j * WAVES * 64;
      wc[j] = 0;
      if (k < span_n) {
        const uint64_t o = p.offsets[wg_lo + k], len = p.offsets[wg_lo + k + 1] - o;
        wc[j] = (uint32_t) min((len + lead_of((uint32_t) o) + kBlock - 1u) / kBlock, (uint64_t) kOrderBuckets - 1u);
        atomicAdd(&bucket[wc[j]], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {   /* exclusive prefix of the counts from the longest bucket down */
      const uint32_t b = kOrderBuckets - 1u - tid, c = bucket[b];
      uint32_t x = c;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t) __shfl_up((int) x, d);
        x += tid >= d ? y : 0u;
      }
      bucket[b] = x - c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
      const uint32_t k = tid + j * WAVES * 64;
      if (k < span_n) order[atomicAdd(&bucket[wc[j]], 1u)] = (uint16_t) k;
    }
  };

  /* the replay's work list: requests finalize deferred, as offsets in the
   * range (u16); on overflow (or ranges over 64K requests) the replay scans
   * the whole range */
  uint32_t *defer_n = wg_counter + 5;
  uint16_t *defer_list = reinterpret_cast<uint16_t *>(wg_counter + kPoolWords);
  auto defer = [&](uint32_t i) {
    *wg_deferred = 1u;
    const uint32_t at = atomicAdd(defer_n, 1u);
    if (at < kDeferCap) defer_list[at] = (uint16_t) (i - wg_lo);
  };

  /* ---- decode ----
   * The decoded window's events as four 32-bit words mq[q] (bytes 32q..32q+31
   * of the window at dpos), the terminal taken off.  The grammar fixes their
   * order (rhp_dfa.h): ME PE RL, then per header line its colon (CO) and its LF
   * (EOL).  Per word, the request-line events of lanes still in the request
   * line go through a small loop; in the header region the events alternate,
   * so a prefix XOR splits the word into its CO and EOL bits and one loop
   * iteration completes one record:
   *   name = [ls, co), value = [co + 2, eol - 1), next ls = eol + 1.
   * The max_headers check (picohttpparser.c:281-284) fires at the CO of a line
   * that starts while nh == maxh; decoding stops there (dstop), so nh never
   * exceeds maxh and every completed record is stored.  Updates are written as
   * arithmetic on the conditions (m & (m - c), x + c * d) so the compiler emits
   * straight-line code, not exec-masked branches. */
  uint32_t mq[kWEv];
  uint32_t term_pos = 0xffffffffu, dstop = 0;
  /* hx: index in hdrs of the decoded request's next header record (set per
   * window from dcur and nh, not carried across the walk; the host keeps
   * n * max_headers below 2^32) */
  uint32_t hx = 0;
  bool wt = false;   /* write-through record stores (set once the range is known even, below) */
  auto word = [&](uint32_t m, uint32_t base) {
    m &= dstop - 1u;   /* nothing after a max_headers stop */
    if (!__builtin_amdgcn_ballot_w64(m != 0)) return;
    /* request line: ME -> method_len = ME (the DFA path parses the method from
     * byte 0); PE -> path = [ME + 1, PE), the first header line starts at
     * PE + 11; RL at the CR of "HTTP/1.0" (PE + 9) or the LF of "HTTP/1.1" */
    while (__builtin_amdgcn_ballot_w64(m != 0 && (kn & 7u) < 3u)) {
      const uint32_t v = m != 0 && (kn & 7u) < 3u;
      const uint32_t ep = base + (uint32_t) __builtin_ctz(m | 0x80000000u);
      m &= m - v;
      const uint32_t k = v ? kn & 7u : 7u;
      const uint32_t mv = ((ep - pe - 9u) & 1u) << 3;
      rl = k == 1u ? me | ((ep - me - 1u) << 16) : rl;
      ls = k == 1u ? ep + 11u : ls;
      me = k == 0u ? ep : me;
      pe = k == 1u ? ep : pe;
      kn += (k < 3u) + (k == 2u ? mv : 0u);
    }
    if (!__builtin_amdgcn_ballot_w64(m != 0)) return;
    /* prefix XOR: bit i = parity of the events at or below i, 1 at the 1st,
     * 3rd, ... event of the word */
    uint32_t px = m ^ (m << 1);
    px ^= px << 2; px ^= px << 4; px ^= px << 8; px ^= px << 16;
    const uint32_t odd = m & px;
    uint32_t com = t ? m ^ odd : odd;    /* t = 1: the word opens with an EOL */
    uint32_t eolm = m ^ com;
    if (!__builtin_amdgcn_ballot_w64(nh + (uint32_t) __builtin_popcount(eolm) >= maxh)) {
      /* no lane can reach max_headers in this word: no capacity checks.  The
       * lanes with a record in the word loop over their records under exec
       * (a lane leaves the loop after its last record), one record per trip;
       * the store flavour is chosen outside the loop */
#ifndef RHP_DECODE_SELECT
      if (eolm != 0) {
        auto records = [&](auto wt_c) __attribute__((always_inline)) {
          do {
            const uint32_t e = base + (uint32_t) __builtin_ctz(eolm);
            const uint32_t co = t ? pco : base + (uint32_t) __builtin_ctz(com | 0x80000000u);
            com = t ? com : com & (com - 1u);
            eolm &= eolm - 1u;
            const uint32_t nlen = co - ls, vlen = e - co - 3u;
            if constexpr (DENSE) {
              uint16_t *q = p.lens16 + hx;
              const bool fits = max(nlen << 4, vlen) <= RHP_DENSE_VALUE_MAX;   /* name <= 62, value <= 1007 */
              const uint32_t v16 = fits ? nlen | vlen << 6 : RHP_DENSE_OVERFLOW;
              if constexpr (decltype(wt_c)::value)
                asm volatile("global_store_short %0, %1, off sc1" ::"v"(q), "v"(v16) : "memory");
              else *GLOBAL(uint16_t, q) = (uint16_t) v16;
              if (!fits) *GLOBAL(uint32_t, p.ovf32 + hx) = nlen | vlen << 16;   /* rare: the overflow area */
            } else if constexpr (COMPACT) {
              uint32_t *q = p.lens + hx;
#ifdef RHP_DIAG_NO_RECSTORE   /* diagnostic: the records computed, not stored (the stores' share) */
              asm volatile("" ::"v"(q), "v"(nlen | vlen << 16));
#else
              if constexpr (decltype(wt_c)::value)
                asm volatile("global_store_dword %0, %1, off sc1" ::"v"(q), "v"(nlen | vlen << 16) : "memory");
              else *GLOBAL(uint32_t, q) = nlen | vlen << 16;
#endif
            } else {
              rhp_hdr_t *q = p.hdrs + hx;
              const u32x2 v = u32x2{ls | nlen << 16, (co + 2u) | vlen << 16};
              if constexpr (decltype(wt_c)::value)
                asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(q), "v"(v) : "memory");
              else *GLOBAL(u32x2, q) = v;
            }
            if (http) {   /* uniform: framing candidates only in http mode */
              const bool cnd = nlen == 14u || nlen == 17u;
              const bool first = cnd && (cand & 0xbfffffffu) == 0;
              crec_lo = first ? ls | nlen << 16 : crec_lo;
              crec_hi = first ? (co + 2u) | vlen << 16 : crec_hi;
              cand |= cnd ? (nh < 30u ? 1u << nh : 0x80000000u) : 0u;
            }
            ls = e + 1u;
            nh++;
            hx += p.rec_hdr;
            t = 0;
          } while (eolm != 0);
        };
        if (wt) records(std::true_type{});
        else records(std::false_type{});
      }
#else
      /* Straight-line body for every lane: a lane whose word is done (eolm ==
       * 0) computes a dead record, stores nothing and keeps its state */
      while (uint64_t st_m = __builtin_amdgcn_ballot_w64(eolm != 0)) {
        const bool has = eolm != 0;
        const uint32_t e = base + (uint32_t) __builtin_ctz(eolm | 0x80000000u);
        const uint32_t co = t ? pco : base + (uint32_t) __builtin_ctz(com | 0x80000000u);
        const uint32_t lo = ls | ((co - ls) << 16), hi = (co + 2u) | ((e - co - 3u) << 16);
        if constexpr (DENSE) store_dense_lanes(st_m, p, hx, co - ls, e - co - 3u, wt);
        else if constexpr (COMPACT) store_len_lanes(st_m, p.lens + hx, (co - ls) | ((e - co - 3u) << 16), wt);
        else store_rec_lanes(st_m, p.hdrs + hx, u32x2{lo, hi}, wt);
        if (http) {   /* uniform: framing candidates only in http mode */
          const uint32_t nlen = co - ls;
          const bool cnd = has && (nlen == 14u || nlen == 17u);
          const bool first = cnd && (cand & 0xbfffffffu) == 0;
          crec_lo = first ? lo : crec_lo;
          crec_hi = first ? hi : crec_hi;
          cand |= cnd ? (nh < 30u ? 1u << nh : 0x80000000u) : 0u;
        }
        com &= com - (uint32_t) (has && !t);
        eolm &= eolm - 1u;
        ls = has ? e + 1u : ls;
        nh += (uint32_t) has;
        hx += has ? p.rec_hdr : 0u;
        t = has ? 0u : t;
      }
#endif
      /* a colon left open at the end of the word: a later word (or window) has its LF */
      if (com) {
        pco = base + (uint32_t) __builtin_ctz(com);
        t = 1;
      }
      return;
    }
    while (__builtin_amdgcn_ballot_w64(eolm != 0)) {
      const bool has = eolm != 0;
      const uint32_t e = base + (uint32_t) __builtin_ctz(eolm | 0x80000000u);
      const uint32_t co = t ? pco : base + (uint32_t) __builtin_ctz(com | 0x80000000u);
      const bool nl = has && !t;                   /* this record's CO is in the word */
      const bool stop = nl && nh == maxh;          /* a line starts at capacity: -1 (or exact) */
      const bool rec = has && !stop;
      const uint32_t lo = ls | ((co - ls) << 16), hi = (co + 2u) | ((e - co - 3u) << 16);
      const uint64_t st_m = __builtin_amdgcn_ballot_w64(rec);
      if (st_m) {
        if constexpr (DENSE) store_dense_lanes(st_m, p, hx, co - ls, e - co - 3u, wt);
        else if constexpr (COMPACT) store_len_lanes(st_m, p.lens + hx, (co - ls) | ((e - co - 3u) << 16), wt);
        else store_rec_lanes(st_m, p.hdrs + hx, u32x2{lo, hi}, wt);
      }
      if (http) {
        const uint32_t nlen = co - ls;
        const bool cnd = rec && (nlen == 14u || nlen == 17u);
        const bool first = cnd && (cand & 0xbfffffffu) == 0;
        crec_lo = first ? lo : crec_lo;
        crec_hi = first ? hi : crec_hi;
        cand |= cnd ? (nh < 30u ? 1u << nh : 0x80000000u) : 0u;
      }
      ovf = stop && ovf == 0 ? ls + 1u : ovf;
      dstop |= stop ? 1u : 0u;
      com = stop ? 0u : nl ? com & (com - 1u) : com;
      eolm = stop ? 0u : rec ? eolm & (eolm - 1u) : eolm;
      ls = rec ? e + 1u : ls;
      nh += rec ? 1u : 0u;
      hx += rec ? p.rec_hdr : 0u;
      t = rec ? 0u : t;
    }
    const bool open = com != 0;
    const bool stop = open && nh == maxh;
    ovf = stop && ovf == 0 ? ls + 1u : ovf;
    dstop |= stop ? 1u : 0u;
    pco = open && !stop ? base + (uint32_t) __builtin_ctz(com) : pco;
    t = open && !stop ? 1u : t;
  };
  auto decode_window = [&]() {
#pragma unroll
    for (int q = 0; q < (int) kWEv; q++) word(mq[q], (uint32_t) dpos + 32u * (uint32_t) q);
  };
  /* The framing candidate's evaluation after a window's decode (see fr).  A
   * lane that needs bytes reads the 36 bytes from one position r of the
   * window at once (ten aligned ds_read_b32 from the staging buffer, whose
   * 16-byte parts hold whole dwords): a fresh candidate's name (compared
   * with both names) and its value from r + 16 (the one SP after the colon),
   * or the continuation of a Content-Length value from r. */
  /* frame_read: which bytes the lane needs and their LDS reads (issued; the
   * caller waits for them); frame_eval: the rest.  Split so that the next
   * window's issue, which refills the staging buffer, goes out between the
   * two */
  struct FrameIn {
    bool need, fresh, rec_done;
    uint32_t r, n, nl, value_len;
    uint32_t raw[10];
  };
  auto frame_read = [&](FrameIn &fi, uint32_t crec_before) __attribute__((always_inline)) {
    const uint32_t wend = (uint32_t) dpos + kWBlock;
    const uint32_t hdr = cand & 0x3fffffffu;
    const bool rec_done = (crec_lo | (cand & 0xbfffffffu)) != crec_before && hdr != 0 && (hdr & (hdr - 1u)) == 0 &&
                          !(cand >> 31);
    const uint32_t value_len = crec_hi >> 16;
    bool need = false, fresh = false;
    uint32_t r = 0, n = 0, nl = 0;
    if (fr & kFrDefer) {
    } else if (rec_done) {   /* the first candidate's record completed in this window */
      const uint32_t name_off = crec_lo & 0xffffu, name_len = crec_lo >> 16, value_off = crec_hi & 0xffffu;
      if (fr & kFrCarry) {   /* a Content-Length value that started in an earlier window */
        r = max(value_off, (uint32_t) dpos);
        n = value_off + value_len - r;
        need = true;
      } else if (fr & kFrTeName) {
        fr = (fr & ~kFrTeName) | (value_len != 0 ? kFrTe : 0u);
      } else if (fr & kFrNeither) {
      } else if (name_off < (uint32_t) dpos) {
        fr |= kFrDefer;   /* the name began in an earlier window */
      } else {
        r = name_off; nl = name_len; n = value_len; fresh = need = true;
      }
    } else if (t && (cand & 0xbfffffffu) == 0) {   /* its line may be open at the window's end */
      const uint32_t nlen = pco - ls;
      if (fr & kFrCarry) {
        r = max(pco + 2u, (uint32_t) dpos);
        n = wend > r ? wend - r : 0u;
        need = n != 0;
      } else if (!(fr & (kFrTeName | kFrNeither)) && (nlen == 14u || nlen == 17u)) {
        if (ls < (uint32_t) dpos) {
          fr |= kFrDefer;
        } else {
          r = ls; nl = nlen; n = wend > ls + 16u ? wend - ls - 16u : 0u; fresh = need = true;
        }
      }
    }
    fi.need = need;
    fi.fresh = fresh;
    fi.rec_done = rec_done;
    fi.r = r;
    fi.n = n;
    fi.nl = nl;
    fi.value_len = value_len;
    if (!__builtin_amdgcn_ballot_w64(need)) return;
    if (!need) return;
    const uint32_t b0 = (r - (uint32_t) dpos) & ~3u;
#pragma unroll
    for (uint32_t k = 0; k < 10; k++) {   /* bytes past the window wrap inside the lane's window: never used */
      const uint32_t b = b0 + 4u * k;
      fi.raw[k] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(
          (size_t) (part_lds((b >> 4) % kWParts) + (b & 15u)));
    }
  };
  auto frame_eval = [&](FrameIn &fi) __attribute__((always_inline)) {
    if (!__builtin_amdgcn_ballot_w64(fi.need)) return;
    if (!fi.need) return;
    const bool fresh = fi.fresh, rec_done = fi.rec_done;
    const uint32_t r = fi.r, n = fi.n, nl = fi.nl, value_len = fi.value_len;
    uint32_t d[9];
    const uint32_t sh = (r - (uint32_t) dpos) & 3u;
#pragma unroll
    for (uint32_t k = 0; k < 9; k++) d[k] = __builtin_amdgcn_alignbyte(fi.raw[k + 1], fi.raw[k], sh);
    bool digits = !fresh;
    if (fresh) {
      /* case-insensitive compares (OR 0x20: the one non-letter, '-', could
       * only collide with CR, which no name holds) */
      /* "content-length", "transfer-encoding" as little-endian dwords */
      constexpr uint32_t kCl[3] = {0x746e6f63u, 0x2d746e65u, 0x676e656cu};
      constexpr uint32_t kTe[4] = {0x6e617274u, 0x72656673u, 0x636e652du, 0x6e69646fu};
      uint32_t dcl = 0, dte = 0;
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t x = d[k] | 0x20202020u;
        dte |= x ^ kTe[k];
        if (k < 3) dcl |= x ^ kCl[k];
      }
      dcl |= ((d[3] | 0x2020u) ^ ((uint32_t) 'h' << 8 | 't')) & 0xffffu;   /* "th" */
      dte |= ((d[4] | 0x20u) ^ 'g') & 0xffu;
      if (nl == 14u && dcl == 0) {
        if (rec_done) {
          if (value_len > kFrMaxValue) fr |= kFrDefer;
          else if (value_len != 0) { fr |= kFrCl; digits = true; }
        } else {
          fr |= kFrCarry;
          digits = true;
        }
      } else if (nl == 17u && dte == 0) {
        if (rec_done) {
          fr |= value_len != 0 ? kFrTe : 0u;
          /* "chunked" right after ": " (value bytes 19..25 of the line) */
          const uint32_t value_off = crec_hi & 0xffffu;
          if (value_len == 7u && value_off == r + 19u && ((d[4] >> 24) | 0x20u) == 'c' &&
              (d[5] | 0x20202020u) == 0x6b6e7568u && ((d[6] | 0x2020u) & 0xffffu) == 0x6465u)
            fr |= kFrChunked;
        } else {
          fr |= kFrTeName;
        }
      } else if (!rec_done) {
        fr |= kFrNeither;
      }
    } else if (rec_done) {
      fr = (fr & ~kFrCarry) | (value_len != 0 ? kFrCl : 0u);   /* an empty value is no Content-Length */
    }
    if (digits) {
      /* strtoull (rhp_scalar.h num_step) over the value bytes: a fast-path
       * value starts with neither OWS nor a CTL, so only the sign and the
       * digit run matter; up to 12 bytes per window here, more -> the replay */
      /* one byte per trip, straight-line (selects, no exec-masked branches: the
       * branchy form spent ~25 scalar instructions per trip on exec masks); the
       * 12 value bytes shift down a byte per trip */
      uint32_t w0 = fresh ? d[4] : d[0], w1 = fresh ? d[5] : d[1], w2 = fresh ? d[6] : d[2];
      const uint32_t m = min(n, 12u);
      for (uint32_t j = 0; __builtin_amdgcn_ballot_w64(j < m && !(fr & kFrStop)); j++) {
        const bool act = j < m && !(fr & kFrStop);
        const uint32_t c = w0 & 0xffu, dg = c - '0';
        w0 = __builtin_amdgcn_alignbyte(w1, w0, 1);
        w1 = __builtin_amdgcn_alignbyte(w2, w1, 1);
        w2 >>= 8;
        const bool sign = !(fr & kFrDigits) && (c == '+' || c == '-');
        const bool dig = dg < 10u;
        const uint32_t flags = sign ? kFrDigits | (c == '-' ? kFrNeg : 0u) : dig ? kFrDigits : kFrStop;
        fr = act ? (fr + (1u << kFrCountSh)) | flags : fr;
        fv = act && !sign && dig ? fv * 10u + dg : fv;
      }
      if ((n > 12u && !(fr & kFrStop)) || ((fr >> kFrCountSh) & 0xffu) > kFrMaxValue) fr |= kFrDefer;
    }
  };
  auto frame_window = [&](uint32_t crec_before) __attribute__((always_inline)) {
    FrameIn fi;
    frame_read(fi, crec_before);
    frame_eval(fi);
  };
  /* set up the decode of the window walked last iteration */
  auto decode_begin = [&]() {
    const uint32_t e = st_prev;
    const bool slow = is_slow2(e);
    const bool term_ev = is_done2(e) || is_err2(e);
    const uint32_t live = (slow || !dhas || ovf) ? 0u : 0xffffffffu;
#pragma unroll
    for (int q = 0; q < (int) kWEv; q++) mq[q] = evp[q] & live;
    term_pos = 0xffffffffu;
    dstop = 0;
    hx = dcur * p.rec_req + nh * p.rec_hdr;
    if (term_ev) {   /* the terminal is the window's last event: take it off the mask */
      /* the last word with an event (selects, no dynamic register index) */
      int q = 0;
      uint32_t w = mq[0];
#pragma unroll
      for (int k = 1; k < (int) kWEv; k++) {
        q = mq[k] ? k : q;
        w = mq[k] ? mq[k] : w;
      }
      const uint32_t bt = 31u - (uint32_t) __builtin_clz(w | 1u);
      if (w) term_pos = (uint32_t) dpos + 32u * (uint32_t) q + bt;
      w &= ~(1u << bt);
#pragma unroll
      for (int k = 0; k < (int) kWEv; k++) mq[k] = k == q ? w : mq[k];
    }
  };
  /*
   * Finalize dcur when its outcome is known (decisions mirrored by rhp_emu.cpp):
   *   ok    DONE at term < len (and term < RHP_MAX_LEN, the records' range)
   *   bad   ERR at term < len, or max_headers overflow at a line start < len
   *   exact SLOW, a terminal at/after len, or no terminal by the end of the buffer
   * Returns true when dcur was finalized.
   */
  auto decode_end = [&]() -> bool {
    const uint32_t e = st_prev;
    const bool ovfl = ovf != 0;
    const bool term_ev = is_done2(e) || is_err2(e);
    const bool fin = dhas && (ovfl || is_slow2(e) || term_ev || (uint32_t) dpos + kWBlock >= dlen);
    if (!fin) return false;
    bool ok = !ovfl && is_done2(e) && term_pos < dlen && term_pos < RHP_MAX_LEN;
    /* an ERR between the path and the request-line end (the version, kn == 2)
     * is -1 only when the version's 9 bytes are there (picohttpparser.c:248-251):
     * len >= PE + 10 */
    bool bad = ovfl ? ovf - 1u < dlen
                    : (is_err2(e) && term_pos < dlen && ((kn & 7u) != 2u || pe + 10u <= dlen));
#ifdef RHP_DIAG_NO_WALK
    ok = false;   /* diagnostic: nothing was walked; every request ends at its last window, -1, no replay */
    bad = true;
#endif
    if (!http && p.last_len) {
      /* last_len != 0 (rare: a batch that carries it): is_complete runs first
       * (picohttpparser.c:399-401).  Scanning from last_len - 3 at or before
       * the first CR of the final CRLFCRLF of a request the DFA accepted, it
       * meets only CRLF line ends and stops at that empty line: the parse
       * stands.  Anything else (a later start, an ERR) takes the exact path. */
      const uint64_t ll = p.last_len[dcur];
      if (ll != 0) {
        ok = ok && (ll < 3u || ll <= term_pos);
        bad = false;
      }
    }
    /* dense records (phr mode): a DFA record whose method is longer than 255
     * bytes takes the exact path (the wide records) */
    if constexpr (DENSE) ok = ok && (rl & 0xffffu) <= 255u;
    /* the record as four dwords (rhp.h rhp_req_t: ret; method_len, path_off;
     * path_len, method_off 0, minor_version; num_headers, flags) */
    u32x4 rq = u32x4{0u, 0u, 0xff000000u, 0u};   /* minor_version -1 */
    if (ok) {
      rq = u32x4{term_pos + 1u, (rl & 0xffffu) | ((rl + 1u) << 16), (rl >> 16) | (((kn >> 3) & 1u) << 24), nh};
      if (http) {
        /* framing (http.c:196-218): in the late-issue kernel the common cases
         * (GET, no Content-Length / Transfer-Encoding candidate, one
         * Content-Length) are framed here, the candidate's line read back from
         * L2 right after its walk; the rest in the replay, from the hints left
         * in the record it will overwrite */
        bool framed = false;
        if constexpr (LATE) {
          /* GET or no candidate: no body; one candidate: its evaluation (a
           * Content-Length value, or neither name); several, a
           * Transfer-Encoding with a value (chunked) or no evaluation: the
           * replay */
          const uint32_t hdr = cand & 0x3fffffffu, ret = term_pos + 1u;
          const bool get = (cand & 0x40000000u) != 0;
          const bool one = !(cand >> 31) && hdr != 0 && (hdr & (hdr - 1)) == 0;
          if (get || (hdr == 0 && !(cand >> 31)) || (one && !(fr & (kFrDefer | kFrTe | kFrCarry | kFrTeName)))) {
            rhp_http_t x = {1, 0, (uint64_t) ret, 0};
            if (!get && (fr & kFrCl)) {
              const uint64_t size = (fr & kFrNeg) ? 0 - fv : fv;
              if (dlen < (uint64_t) ret + size) {
                x.result = 0; x.consumed = 0;
              } else {
                x.body_kind = 1; x.body_len = size; x.consumed = (uint64_t) ret + size;
              }
            }
            if constexpr (COMPACT) put_http(p, dcur, x);
            else store_http(p.http + dcur, x);
            framed = true;
          }
        }
        if (!framed) {
          defer(dcur);
          typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
          bool chunked = false;
          if constexpr (LATE) {
            const uint32_t hdr = cand & 0x3fffffffu;
            chunked = !(cand >> 30) && hdr != 0 && (hdr & (hdr - 1)) == 0 && (fr & (kFrChunked | kFrDefer)) == kFrChunked;
          }
          *GLOBAL(u32x4a4, &p.http[dcur]) =
              u32x4a4{cand, kHintFrame | (chunked ? kHintChunked : 0u) | (term_pos + 1u), crec_lo, crec_hi};
        }
      }
    } else if (bad) {
      rq[0] = 0xffffffffu;   /* -1 */
      if (http) {
        if constexpr (COMPACT) store_hc(p, dcur, 0xffu, 0u);   /* result -1 */
        else store_http_bad(p.http + dcur);
      }
    } else {
      rq[3] = (uint32_t) kDeferExact << 16;   /* exact path: replay */
      defer(dcur);
      if (http) {
        typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
        *GLOBAL(u32x4a4, &p.http[dcur]) = u32x4a4{0u, kHintExact, 0u, 0u};
      }
    }
    if constexpr (DENSE) {
      /* rhp_req_dense_t: ret | path_len << 16; method_len | num_headers << 8 |
       * minor << 16 | flags << 24 (bad: RHP_DENSE_BAD; exact: wide, deferred) */
      const uint32_t w1 = ok ? (rl & 0xffu) | (nh << 8) | (((kn >> 3) & 1u) << 16)
                             : bad ? RHP_DENSE_BAD << 24 : (kDeferDense | RHP_DENSE_WIDE) << 24;
      const u32x2 v = u32x2{ok ? (term_pos + 1u) | (rl & 0xffff0000u) : 0u, w1};
      uint2 *q = p.dreq + dcur;
      if (wt) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(q), "v"(v) : "memory");
      else *GLOBAL(u32x2, q) = v;
    } else {
      store_req(p.reqs + dcur, rq, wt);
    }
    dhas = false;
    return true;
  };

  /* Pair codes by two lookups.  Form 1 (rhp_dfa.h code_row): A = the row of
   * class(b1), B = class(b0) * 16 + class(b1) from that row: the code read's
   * address is one v_perm, but lanes whose b0 share an LDS bank and whose b1
   * differ in class read different rows there (a bank conflict: 3.25 LDS cycles
   * per read on config 2 where 2 is conflict free, tools/lds_conflicts.py).
   * Form 2 (RHP_CODE_FORM=2): A = class(b1), B = class(b0) * 16, each from one
   * 256-byte row (conflict free for bytes < 0x80), code = A | B: one more
   * v_or per pair.  The table sits at LDS address 0, so a v_perm result is the
   * address itself. */
  auto look_a = [&](uint32_t dw, int j) -> uint32_t {
    return lds_u8(__builtin_amdgcn_perm(kCodeForm == 2 ? kClassRow : kClassRowR, dw, 0x0c0c0400u | (uint32_t) (2 * (j & 1) + 1)));
  };
  auto look_b = [&](uint32_t a, uint32_t dw, int j) -> uint32_t {
    return lds_u8(__builtin_amdgcn_perm(kCodeForm == 2 ? kClassRow16 : a, dw, 0x0c0c0400u | (uint32_t) (2 * (j & 1))));
  };
  auto code_of = [&](uint32_t a, uint32_t b) -> uint32_t { return kCodeForm == 2 ? (a | b) : b; };
  auto codes_a = [&](const u32x4 &chunk, uint32_t (&r)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = look_a(chunk[j >> 1], j);
  };
  auto codes_b = [&](const u32x4 &chunk, const uint32_t (&r)[8], uint32_t (&c)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = code_of(r[j], look_b(r[j], chunk[j >> 1], j));
  };
  /* The walk of the window in W: part 0's codes first, then per chained step
   * one independent lookup pair for the next part behind the step's read (its
   * A read, and the B read of the step before, whose A has landed by then).
   * LDS returns in order, so a step waits only for its own read while the
   * lookups fly behind it (issued ahead of it, a batch of eight delayed every
   * fourth step: config 2 +3 %). */
  auto walk = [&]() {
    uint32_t c[8], r[8];
#if defined(RHP_DIAG_EXTRA_LDS) || defined(RHP_DIAG_EXTRA_VALU)
    uint32_t xacc = 0;   /* diagnostic: one more LDS read / three more VALU per pair (the walk's sensitivity) */
#endif
    codes_a(W[0], r);
    codes_b(W[0], r, c);
#pragma unroll
    for (int q = 0; q < (int) kWParts; q++) {
      const bool nx = q + 1 < (int) kWParts;
      uint32_t cn[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        st = lds_u8(row_addr(st, c[j]));
        __builtin_amdgcn_sched_barrier(0);   /* the chained read issues first */
        if (nx) r[j] = look_a(W[q + 1][j >> 1], j);
        if (nx && j > 0) cn[j - 1] = look_b(r[j - 1], W[q + 1][(j - 1) >> 1], j - 1);
#ifdef RHP_DIAG_EXTRA_LDS
        if (nx) xacc += lds_u8(__builtin_amdgcn_perm(kClassRow, W[q + 1][j >> 1], 0x0c0c0400u | (uint32_t) (2 * (j & 1))));
#endif
#ifdef RHP_DIAG_EXTRA_VALU
        if (nx) {
          uint32_t y = __builtin_amdgcn_perm(W[q + 1][j >> 1], W[q + 1][j >> 1], 0x0c0c0001u + 0x202u * (uint32_t) (j & 1));
          opaque(y);
          y = y ^ ((y >> 6) & 0x7cu);
          opaque(y);
          xacc += y;
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
        ev_shift2(ev[q >> 1], st);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (nx) {
        cn[7] = look_b(r[7], W[q + 1][3], 7);
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = code_of(r[j], cn[j]);
      }
      /* phase-locked http form: once every lane of the wave is terminal (or
       * parked) the rest of the window changes nothing -- terminal states are
       * absorbing and fire no event -- so the walk stops at the end of an event
       * word (q odd: the word holds its 16 steps) */
      if constexpr (kPhaseLock)
        if ((q & 1) && nx && !__builtin_amdgcn_ballot_w64(st >= kLiveIdx)) break;
    }
#if defined(RHP_DIAG_EXTRA_LDS) || defined(RHP_DIAG_EXTRA_VALU)
    asm volatile("" ::"v"(xacc));
#endif
  };

  /* The bytes of a first window before its request (wlead of them) zeroed in
   * the registers: S_PRE walks them (rhp_dfa.h) */
  auto zero_lead = [&](bool wnew) {
    if (!__builtin_amdgcn_ballot_w64(wnew && wlead != 0)) return;
    const int32_t l8 = wnew ? (int32_t) (8u * wlead) : 0;
#pragma unroll
    for (uint32_t q = 0; q < kLead / 16u + 1u && q < kWParts; q++)
#pragma unroll
      for (uint32_t d = 0; d < 4u; d++) {
        /* the dword's bytes before the request: a v_sub, a v_med3, a 64-bit shift, a v_and */
        const int32_t sh = min(max(l8 - (int32_t) (128u * q + 32u * d), 0), 32);
        W[q][d] &= (uint32_t) (~0ull << sh);
      }
  };

  /* LDS-DMA of every lane's next window (nw) into the staging buffer:
   * kParts loads of 1 KiB (see stage_off) */
  /* In two halves: issue_prep exchanges the window addresses (the shuffles,
   * one LDS round trip for the lot), issue_go makes the loads once the caller
   * has waited for its LDS reads -- the shuffles are issued before the reads
   * the wait is for, so the issue costs no round trip of its own */
  struct Issue {
    uint32_t a[kParts];
    uint32_t src;
  };
  auto issue_prep = [&](Issue &is) {
    /* a lane without a next window fetches the range's first bytes instead
     * (its staging slot is not read), so no load needs a branch */
    is.src = (nw & 3u) ? (nw & ~3u) : 0u;
#pragma unroll
    for (int i = 0; i < (int) kParts; i++) is.a[i] = (uint32_t) __shfl((int) is.src, (int) dma_window((uint32_t) i, lane));
  };
  auto issue_go = [&](const Issue &is) {
    const uint32_t src = is.src;
    const uint32_t (&a)[kParts] = is.a;
    /* Cache policy per wave and window: when every window is one whole HBM
     * line (line-aligned requests), no line is read by two windows and the
     * loads go non-temporal (config 2 +19 %, config 5 +9 %); windows that
     * straddle lines share their edge lines with the neighbouring requests'
     * windows, which then hit in L2 (non-temporal: config 3 -5 %) */
    const bool aligned = !(nw & 3u) || ((uint32_t) (uintptr_t) (wbytes + src) & (kBlock - 1u)) == 0;
#ifdef RHP_NO_NT
    const bool nt = false && aligned;
#else
    const bool nt = !__builtin_amdgcn_ballot_w64(!aligned);
#endif
    /* one branch per issue, not one per load (the cache policy is an immediate) */
#define RHP_ISSUE_LOADS(AUX)                                                                             \
    _Pragma("unroll") for (int i = 0; i < (int) kParts; i++) {                                           \
      const uint32_t part = dma_part(dma_window((uint32_t) i, lane), lane);                              \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc,                                                    \
          (__attribute__((address_space(3))) void *) (lds + stage + 1024u * i), 16, a[i] + 16u * part,   \
          0, 0, AUX);                                                                                    \
    }
    if (nt) { RHP_ISSUE_LOADS(2) } else { RHP_ISSUE_LOADS(0) }
#undef RHP_ISSUE_LOADS
    /* the extension parts: lane j's own window, part 8 + k at xstage + 1024 k + 16 j */
#pragma unroll
    for (uint32_t k = 0; k < kXParts; k++)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (__attribute__((address_space(3))) void *) (lds + xstage + 1024u * k),
                                               16, src + kBlock + 16u * k, 0, 0, 0);
  };
  auto issue = [&]() {
    Issue is;
    issue_prep(is);
    issue_go(is);
  };

  /* Uneven ranges (config 3) order the hand-out from the first request on;
   * the test reads the first 64 requests of the range, the same in every wave,
   * so every wave takes the same branch without a barrier */
  const bool may_order = order_on && span_n > first_n;
  uint32_t s0 = 0, s1 = 0;
  if (may_order) {
    const uint32_t *so = reinterpret_cast<const uint32_t *>(p.offsets + wg_lo + min(lane, span_n - 1u));
    s0 = *GLOBAL(const uint32_t, so);
    s1 = *GLOBAL(const uint32_t, so + 2);
  }
  if (tid < first_n) take(wg_lo + tid);
  /* the table into LDS, the pool counter past the requests handed out, the
   * long-request bitmap cleared */
#pragma unroll
  for (uint32_t j = 0; j < sizeof tab / sizeof tab[0]; j++) {
    const uint32_t k = tid + j * WAVES * 64;
    if (k < kTable2Bytes / 16) reinterpret_cast<u32x4 *>(lds)[k] = tab[j];
  }
  for (uint32_t k = tid; k < kPoolWords; k += WAVES * 64)
    reinterpret_cast<uint32_t *>(lds + kLdsTable + WAVES * kStageWave)[k] = k == 0 ? first_n : 0u;
  wait_vm0();   /* the pending offsets */
  dg.loads_landed();
  const bool uneven =
      may_order && __builtin_amdgcn_ballot_w64((uint64_t) (s1 - s0) * span_n > 2u * (o_hi - o_lo)) != 0;
  wt = p.wt_records && !uneven;
#ifdef RHP_DIAG_NO_WT   /* diagnostic: plain record stores everywhere */
  wt = false;
#endif
  /* An uneven range runs on 15 of the 16 waves (14 when its order needs two
   * waves' staging; the others hold the hand-out order and only join the
   * barriers and the replay).
   * Round 3, traffic-bound with 4-aligned windows: 16 waves 422 us, 12 waves 398
   * us, 8 waves 474 us; round 5, after line windows the loop is latency-bound and
   * more waves pay again: 12 waves 282 us, 13: 278, 14: 277 (profiles/r05/config3/). */
#ifndef RHP_UNEVEN_WAVES
#define RHP_UNEVEN_WAVES 15
#endif
  /* the order lives in the last order_waves waves' staging (sort_range): they
   * must not walk, so at least one wave stays idle whatever the knobs (the http
   * instance has fewer waves with RHP_HTTP_XPARTS > 0) */
  constexpr uint32_t kUnevenWaves = (uint32_t) WAVES - 1u < (uint32_t) RHP_UNEVEN_WAVES ? (uint32_t) WAVES - 1u
                                                                                     : (uint32_t) RHP_UNEVEN_WAVES;
  static_assert(kUnevenWaves + 1u <= (uint32_t) WAVES, "an idle wave's staging holds the hand-out order");
  bool idle_wave = false;
  if (uneven) {
    /* the whole range longest first, the first hand-out included: a long
     * request never waits behind another one in a lane, and the requests
     * committed when the pool runs dry are the shortest (the barriers: the
     * histogram zeroed before the sort; the order complete and the counter
     * reset before the first refill) */
    pend_ok = false;
    sorted = true;
    idle_wave = (tid >> 6) >= min(kUnevenWaves, (uint32_t) WAVES - order_waves);
    if (tid < kOrderBuckets) bucket[tid] = 0u;
    __syncthreads();
    if (tid == 0) *wg_counter = 0;
    sort_range();
    __syncthreads();
    if (!idle_wave) {
      refill_pend();
      wait_vm0();
      nw = pend_ok ? first_win(pend_o0) | 2u : 0u;
      issue();
    }
  } else {
    /* the barrier that makes the table and the pool area initialized, then each
     * wave's first windows: a wave enters the loop as soon as its own loads are
     * issued, not when the slowest wave's are -- the first issue waits on a
     * chip-wide burst of 32 MB (round 5: config 5 -3 %, config 2 +-0) */
    __syncthreads();
    nw = pend_ok ? first_win(pend_o0) | 2u : 0u;
    issue();
  }

  /*
   * One iteration = one 128-byte window per lane.
   * [A] the window issued one iteration earlier has landed (the loop's only
   * VMEM wait) -> [C] switch the walk to it -> [D] hand out pending requests
   * -> [E] issue the next window into the buffer [A] just read -> decode the
   * previous window -> [F] walk this one -> [G] finalize the
   * decoded request if it ended, hand the decode over to the walked window.
   */
  dg.loop_start();
  /* The SIMD issues by priority, then age: with equal priorities the waves
   * dispatched last in a workgroup run slowest and finish its range last.
   * Rotating every wave's priority each iteration (phase by wave) shares the
   * issue slots evenly (config 2 -1 %, configs 3 and 5 -3 %). */
#ifndef RHP_PRIO_PHASE_SHIFT
#define RHP_PRIO_PHASE_SHIFT 6
#endif
#ifndef RHP_PRIO_MODE
#define RHP_PRIO_MODE 0
#endif
  uint32_t prio_it = (tid >> RHP_PRIO_PHASE_SHIFT) & 3u;
#if RHP_PRIO_MODE == 1
  /* static, graded by dispatch order: the younger a wave on its SIMD, the higher */
  switch ((tid >> 8) & 3u) {
  case 0: __builtin_amdgcn_s_setprio(0); break;
  case 1: __builtin_amdgcn_s_setprio(1); break;
  case 2: __builtin_amdgcn_s_setprio(2); break;
  default: __builtin_amdgcn_s_setprio(3);
  }
#elif RHP_PRIO_MODE == 2
  if ((tid >> 9) & 1u) __builtin_amdgcn_s_setprio(1);   /* static: the younger half of the workgroup */
#endif
  while (!idle_wave) {
#if RHP_PRIO_MODE == 0
    prio_it = (prio_it + 1u) & 3u;
    switch (prio_it) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3);
    }
#elif RHP_PRIO_MODE == 3
    /* the gap between the window's landing and the next window's issue at the
     * top priority; the rest of the iteration rotates among 0-2 (below) */
    __builtin_amdgcn_s_setprio(3);
#endif
    dg.mark();
    /* [A] */
    wait_vm0();   /* the window's LDS-DMA has landed (and the pending offsets, and older stores) */
    dg.section(0);
    const uint32_t p_o0 = pend_o0, p_o1 = pend_o1;
#pragma unroll
    for (int q = 0; q < (int) kWParts; q++) W[q] = *reinterpret_cast<const u32x4 *>(lds + part_lds((uint32_t) q));
    /* [C] */
    const uint32_t nw_kind = nw & 3u;
    bool wnew = false;
    if (nw_kind == 2) {   /* pend's first window: the walk switches to pend */
      wcur = pend;
      wlen = p_o1 - p_o0;
      if constexpr (LATE) woff = p_o0 - (uint32_t) base;
      pend_ok = false;
      wlead = lead_of(p_o0);
      wpos = -(int32_t) wlead;
      wact = true;
      wnew = true;
      uint32_t first;   /* the request's first byte */
      if constexpr (HTTP) {
        /* GET: the request's first four bytes are "GET " (the DFA path parses
         * the method from byte 0), read from the window already in registers */
        const uint32_t head = __builtin_amdgcn_alignbyte(W[0][1], W[0][0], wlead);
        wget = head == ('G' | 'E' << 8 | 'T' << 16 | (uint32_t) ' ' << 24) ? 0x40000000u : 0u;
        first = head & 0xffu;
      } else {
        /* from the staging buffer (before the next issue refills it) */
        first = lds_u8(stage + stage_off(lane, wlead >> 4) + (wlead & 15u));
      }
      /* S_PRE walks the zeroed bytes before the request (rhp_dfa.h): a first
       * byte of their class goes to the exact path */
      st = idx2(byte_class_ctlx(first) ? S_SLOW : S_PRE, 0);
    }
    if (nw_kind) cur_ptr = nw & ~3u;
    const bool walking = nw_kind != 0 && wact;   /* a live request's window landed */
    const bool pend_ready = pend_ok;   /* assigned before this block: its offsets are valid */
    if constexpr (!LATE) dg.section(kSecDecodeStamp, true);   /* early form, stamps: [A]'s window reads + [C] */
    Issue is;
    if constexpr (!LATE) {
      /* [E] next window: continuation of wcur, else the first window of a ready
       * pend (its addresses exchanged now, the loads made after [D]) */
      nw = 0;
      if (walking && (uint32_t) (wpos + (int32_t) kWBlock) < wlen) nw = (cur_ptr + kWBlock) | 1u;
      else if (pend_ready) nw = first_win(p_o0) | 2u;
      issue_prep(is);
#ifndef RHP_REFILL_FIRST
      /* the loads first, [D]'s refill (an LDS atomic round trip and the pending
       * offsets' loads) after them: from the window's landing to the next
       * window's issue a wave has nothing of its own in flight */
      dg.section(kSecFrameStamp, true);   /* stamps: the shuffles */
      wait_lgkm0();   /* [A]'s reads of the buffer and the shuffles are done */
      issue_go(is);
#endif
#if RHP_PRIO_MODE == 3
      prio_it = prio_it == 2u ? 0u : prio_it + 1u;
      switch (prio_it) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      default: __builtin_amdgcn_s_setprio(2);
      }
#endif
    }
    /* [D] */
    refill_pend();
    const bool any_walk = __builtin_amdgcn_ballot_w64(walking) != 0;
    const bool any_dec = __builtin_amdgcn_ballot_w64(dhas) != 0;
    dg.lanes(walking, pool_dry);
    if constexpr (!LATE) {
#ifdef RHP_REFILL_FIRST
      dg.section(kSecFrameStamp, true);   /* stamps: the shuffles and [D]'s refill */
      wait_lgkm0();   /* [A]'s reads of the buffer and the shuffles are done */
      issue_go(is);
#endif
      dg.section(1, true);
      /* [F] walk + decode of the previous window */
      decode_begin();
#ifndef RHP_DIAG_NO_DECODE   /* diagnostic builds only (records not written): the decode's share of the loop */
      if (any_dec) decode_window();
#endif
#pragma unroll
      for (int w = 0; w < (int) kWEv; w++) ev[w] = 0;
      dg.section(2, true, true);
      if (any_walk) {
        if (!walking) st = kPark;   /* idle lanes step in the parked terminal state */
        zero_lead(wnew);
#ifndef RHP_DIAG_NO_WALK   /* diagnostic builds only (every request then ends at its buffer's end): the walk's share */
#ifdef RHP_DIAG_WALK_TWICE   /* diagnostic: the window walked twice from the same state (same outputs): a walk's marginal cost */
        {
          uint32_t st0 = st;
          opaque(st0);
          walk();
          opaque(st);
          st = st0;
        }
#endif
        walk();
#endif
      }
    } else {
      /* [F] walk, then decode the walked window at once (not one behind): a
       * request is finalized -- and framed, from its header lines while they
       * are still in L2 -- in the iteration that walks its last window; [E]
       * then knows whether wcur's walk ended (no continuation is fetched past
       * a terminal: a body is never loaded), and a request taken in [D] is
       * ready (its offsets landed meanwhile), so a lane never idles an
       * iteration between two requests */
      (void) any_dec;
      dg.section(1);
#pragma unroll
      for (int w = 0; w < (int) kWEv; w++) ev[w] = 0;
      if (any_walk) {
        if (!walking) st = kPark;
        zero_lead(wnew);
#ifndef RHP_DIAG_NO_WALK   /* diagnostic builds only (see the early form) */
        walk();
#endif
      }
      dg.section(3, true);
      if (walking && wnew) {
        dcur = wcur;
        dlen = wlen;
        doff = woff;
        kn = me = pe = rl = nh = ls = t = pco = ovf = 0;
        cand = wget;
        crec_lo = crec_hi = 0;
        fr = 0;
        fv = 0;
      }
      dhas = walking;
      dpos = wpos;
      st_prev = st;
#pragma unroll
      for (int w = 0; w < (int) kWEv; w++) evp[w] = ev[w];
      decode_begin();
      const uint32_t crec_before = crec_lo | (cand & 0xbfffffffu);
#ifndef RHP_DIAG_NO_DECODE   /* diagnostic builds only (see the early form) */
      if (any_walk) decode_window();
#endif
      dg.section(kSecDecodeStamp, true);
#ifndef RHP_FRAME_JOINED
      /* the framing's reads of the staging buffer, the next window's issue,
       * then the framing's evaluation and the finalize (which the issue does
       * not wait for: a walk ends at a terminal, its last byte or a max_headers
       * stop, all known after the decode): the window has the evaluation and
       * the finalize to land in (config 5 78.4 -> 75.1 us same-box,
       * profiles/r06/ab/ab_r6m_post.txt; RHP_FRAME_JOINED: the issue after
       * the finalize, as before) */
      FrameIn fi;
      fi.need = false;
#ifndef RHP_DIAG_NO_FRAME
      if (http && any_walk) frame_read(fi, crec_before);
#endif
      if (walking && (ovf != 0 || is_done2(st) || is_err2(st) || is_slow2(st) ||
                      (uint32_t) (wpos + (int32_t) kWBlock) >= wlen))
        wact = false;
      nw = 0;
      if (walking && wact) nw = (cur_ptr + kWBlock) | 1u;
      else if (pend_ok && (!kPhaseLock || it_odd)) nw = first_win(pend_o0) | 2u;   /* the next iteration is even */
      Issue is;
      issue_prep(is);   /* the address shuffles go out with the framing's reads */
      wait_lgkm0();     /* the framing's reads of the buffer are done */
      issue_go(is);
#ifndef RHP_DIAG_NO_FRAME
      if (http && any_walk) frame_eval(fi);
#endif
      dg.section(kSecFrameStamp, true);
      if (any_walk) (void) decode_end();
      dg.section(2, true);
#else
#ifndef RHP_DIAG_NO_FRAME   /* diagnostic builds only: the in-loop framing's share */
      if (http && any_walk) frame_window(crec_before);
#endif
      dg.section(kSecFrameStamp, true);
      const bool done = any_walk ? decode_end() : false;
      dg.section(2, true);
      /* the walk of wcur ends with this window: finalized (a terminal, a
       * max_headers stop), or its last byte */
      if (walking && (done || is_done2(st) || is_err2(st) || is_slow2(st) ||
                      (uint32_t) (wpos + (int32_t) kWBlock) >= wlen))
        wact = false;
      /* [E] (the decode above read the staging buffer the issue refills) */
      nw = 0;
      if (walking && wact) nw = (cur_ptr + kWBlock) | 1u;
      else if (pend_ok && (!kPhaseLock || it_odd)) nw = first_win(pend_o0) | 2u;   /* the next iteration is even */
      wait_lgkm0();   /* the decode's reads of the buffer are done */
      issue();
#endif
    }
    dg.section(LATE ? 4 : 3, true);
    /* [G] */
    if constexpr (!LATE) {
    const bool done = any_dec ? decode_end() : false;
    if (done && !wnew) wact = false;   /* decoded request ended (max_headers stop): stop its walk */
    /* hand the decode over to the walked window */
    if (walking && wact) {
      if (wnew) {
        dcur = wcur;
        dlen = wlen;
        if constexpr (LATE) doff = woff;
        kn = me = pe = rl = nh = ls = t = pco = ovf = 0;
        cand = wget;
        crec_lo = crec_hi = 0;
      }
      dhas = true;
      dpos = wpos;
      st_prev = st;
#pragma unroll
      for (int w = 0; w < (int) kWEv; w++) evp[w] = ev[w];
      /* the walk of wcur ends with this window: a terminal, or its last byte */
      if (is_done2(st) || is_err2(st) || is_slow2(st) || (uint32_t) (wpos + (int32_t) kWBlock) >= wlen) wact = false;
    } else {
      dhas = false;
    }
    }
    wpos += (int32_t) kWBlock;
    it_odd ^= 1u;
    dg.iteration_end();
    if (!__ballot(dhas || nw || pend_ok)) break;
  }
  dg.loop_end(WAVES);
  dg.clock_end();

  /* Replay: the rare paths run here, after the DFA loop, so none of their
   * registers are live in it.  Once every wave of the workgroup is done, the
   * workgroup finishes what finalize deferred, in two passes over its range:
   * (1) one request per thread, http_read_request framing of the DFA-parsed
   * requests from the decode's hints (no dependent loads), listing in LDS the
   * requests that need a serial scalar path -- the exact parse, general
   * framing; (2) the listed requests, one per thread.  A scalar path takes
   * many dependent loads; in pass 1 a wave would wait for it whenever one of
   * its 64 requests needed one (config 5: most iterations), listed they run
   * side by side.  Nothing to do -> no pass at all. */
  wait_vm0();   /* no window load still writes the staging area (reused below) */
  __syncthreads();
  dg.replay_start(WAVES);
  if (*wg_deferred) {
    /* the kernel's arguments loaded again (through an opaque pointer, so the
     * loads are not merged with the kernel's own): the replay's many uses of
     * them then keep no scalar registers busy through the loop, where they
     * were spilled to vector lanes (http kernel: 117 more instructions per
     * loop iteration, config 5 +4 %) */
#if defined(__HIP_DEVICE_COMPILE__)   /* the device pass (the host pass only checks the body) */
    typedef __attribute__((address_space(4))) const Params kParams;
    kParams *pa = (kParams *) __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(pa));
    const Params &p_kernel = p;
    const Params p = HTTP ? *pa : p_kernel;   /* the phr kernels had no such spills (config 3 +1-3 % with the reload) */
#endif
    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    /* what a request needs first: in http mode the hint left in its http
     * record says what to do (and holds ret), so neither the request record is
     * read nor its flags written back.  Pass 1 fetches it one request ahead. */
    struct Head {
      uint64_t off, end;
      u32x4a4 hint;
      uint32_t f;
    };
    auto head = [&](uint32_t k) {
      Head h = {0, 0, u32x4a4{0u, 0u, 0u, 0u}, 0u};
      if (k < wg_hi) {
        h.off = p.offsets[k];
        h.end = p.offsets[k + 1];
        if (http) h.hint = *GLOBAL(const u32x4a4, &p.http[k]);
        else if (DENSE) h.f = (p.dreq[k].y >> 24) & kDeferDense ? kDeferExact : 0u;
        else h.f = p.reqs[k].flags;
      }
      return h;
    };
    auto what = [&](const Head &h) {
      return http ? h.hint[1] & (kHintExact | kHintFrame) : (h.f & kDeferExact) ? kHintExact : 0u;
    };
    /* the serial paths; http_frame_fast declined (or the request is exact):
     * its http record still holds the hint */
    auto finish_slow = [&](uint32_t i, const Head &h) {
      const uint32_t f = what(h);
      if ((f & kHintExact) || p.hc) {   /* compact records: http_frame has no rhp_hdr_t to read, the exact path frames */
        finish_exact(p, i, h.off, h.end - h.off);
      } else {
        const uint32_t cand = h.hint[0];
        http_frame(p.bytes_rw + h.off, h.end - h.off, p.reqs[i], p.hdrs + (uint64_t) i * p.hs_req, p.hs_hdr,
                   &p.http[i], (cand >> 31) ? ~0ull : (uint64_t) (cand & 0x3fffffffu), p.compact, DevDechunk{});
      }
    };
    /* http_frame_fast from request i's hint; its record stored when it settles
     * the request.  The second candidate's record (index j): from hdrs, or, in
     * the compact layout, summed from the lengths after the first one's */
    auto frame_fast = [&](uint32_t i, const Head &h) {
      const uint32_t cand = h.hint[0], crec_hi = h.hint[3];
      /* header k's u32 lengths (compact), or from the dense u16 / its overflow area */
      auto len32 = [&](uint32_t k) -> uint32_t {
        const uint64_t at = (uint64_t) k * p.rec_hdr + (uint64_t) i * p.rec_req;
        if constexpr (!DENSE) return p.lens[at];
        const uint32_t l = p.lens16[at];
        return l == RHP_DENSE_OVERFLOW ? p.ovf32[at] : (l & 63u) | (l >> 6) << 16;
      };
      auto rec = [&](uint32_t j) -> uint2 {
        if (!p.hc) return *reinterpret_cast<const uint2 *>(p.hdrs + (uint64_t) i * p.hs_req + (uint64_t) j * p.hs_hdr);
        uint32_t at = (crec_hi & 0xffffu) + (crec_hi >> 16) + 2u;   /* the line after the first candidate's */
        for (uint32_t k = (uint32_t) __builtin_ctz(cand & 0x3fffffffu) + 1u; k < j; k++) {
          const uint32_t l = len32(k);
          at += (l & 0xffffu) + (l >> 16) + 4u;
        }
        const uint32_t l = len32(j);
        return uint2{at | (l & 0xffffu) << 16, (at + (l & 0xffffu) + 2u) | (l >> 16) << 16};
      };
      rhp_http_t o;
      const int fr = http_frame_fast(p.bytes_rw + h.off, h.end - h.off, (int32_t) (h.hint[1] & 0xffffu), o, cand,
                                     h.hint[2], crec_hi, rec);
      if (fr == kFrameDone) put_http(p, i, o);
      return fr;
    };
    /* the list lives where the DFA table was (idle now); the staging area
     * holds the chunked bodies' LDS slots (staged_moves) */
    uint32_t *slow = reinterpret_cast<uint32_t *>(lds);
    uint32_t *slow_n = wg_counter + 4;                                 /* 0 since the prologue */
    constexpr uint32_t kSlowCap = (kLdsTable - (uint32_t) WAVES * kChunkTabWave) / 4;   /* the chunk tables at the area's end */
    static_assert(kStageBody * kStageBodies <= kStageWave, "a wave's body slots fit its staging");
    dg.pass_begin();
    /* the deferred requests: the list finalize kept, or the whole range when
     * it overflowed */
    const uint32_t nd = *defer_n;
    const bool use_list = nd <= kDeferCap && wg_hi - wg_lo <= 65536u;
    const uint32_t cnt = use_list ? nd : wg_hi - wg_lo;
    auto req_at = [&](uint32_t k) { return wg_lo + (use_list ? (uint32_t) defer_list[k] : k); };
    auto head_at = [&](uint32_t k) { return head(k < cnt ? req_at(k) : wg_hi); };
    /* http mode with the list overflowed (most of the range deferred, e.g. every
     * request chunked): no first pass -- the second pass takes the range itself
     * and frames each request in its round (a scan of its own cost the replay
     * ~6 %) */
    const bool direct = http && !use_list;
    Head nx = head_at(direct ? cnt : tid);
    for (uint32_t k = tid; k < cnt && !direct; k += WAVES * 64) {
      const uint32_t i = req_at(k);
      const Head cur = nx;
      nx = head_at(k + WAVES * 64);
      const uint32_t f = what(cur);
      if (!f) continue;
      const int fr = (f & kHintExact)                 ? kFrameSlow
                     : (cur.hint[1] & kHintChunked) ? kFrameChunked   /* settled in the loop */
                                                    : frame_fast(i, cur);
      dg.framed(fr == kFrameDone);
      if (fr != kFrameDone) {
        /* listed: the range-relative index, bit 31 = a chunked body to de-frame */
        const uint32_t at = atomicAdd(slow_n, 1u);
        if (at < kSlowCap) slow[at] = (i - wg_lo) | (fr == kFrameChunked ? 0x80000000u : 0u);
        else if (fr == kFrameChunked) {   /* list full (a range of > kSlowCap such requests) */
          frame_chunked(p.bytes_rw + cur.off, cur.end - cur.off, (int32_t) (cur.hint[1] & 0xffffu), &p.http[i], p.compact);
          mark_wide(p, i);
        } else finish_slow(i, cur);
      }
    }
    dg.pass_end(1);
    __syncthreads();
    dg.pass_begin();
    const uint32_t ns = direct ? cnt : min(*slow_n, kSlowCap);
    /* wave-uniform rounds of 64 entries: the chunked bodies the lanes walked
     * are moved by the whole wave (staged_moves), and the next round's walks
     * step inside those moves */
    ChunkWalk w;
    w.live = false;
    uint32_t wi = 0;
    int32_t wret = 0;
    bool walking = false;
    auto start_round = [&](uint32_t kb, uint32_t ke) {   /* entries [kb, ke), at most 64 */
      const uint32_t k = kb + lane;
      walking = false;
      w.live = false;
      dg.part_begin();
      if (k < ke) {
        uint32_t e, i;
        Head h;
        if (direct) {   /* the range in order: what the first pass would have done */
          i = wg_lo + k;
          h = head(i);
          const uint32_t f = what(h);
          const int fr = !f                              ? kFrameDone
                         : (f & kHintExact)              ? kFrameSlow
                         : (h.hint[1] & kHintChunked)    ? kFrameChunked
                                                         : frame_fast(i, h);
          e = fr == kFrameDone ? 0x40000000u : fr == kFrameChunked ? 0x80000000u : 0u;
        } else {
          e = slow[k];
          i = wg_lo + (e & 0x7fffffffu);
          h = head(i);
        }
        if (e & 0x40000000u) {
          /* framed (or nothing to do) */
        } else if (http && (e >> 31)) {   /* chunked bodies: http mode only */
          wi = i;
          wret = (int32_t) (h.hint[1] & 0xffffu);
          w.begin(p.bytes_rw + h.off + (uint32_t) wret, (h.end - h.off) - (uint64_t) wret);
          walking = true;
        } else {
          finish_slow(i, h);
        }
        dg.slow_path();
      }
      dg.part_end(4);
    };
    /* Rounds are claimed from an LDS counter, not dealt out by wave index: the
     * waves a SIMD dispatched last run the replay's moves up to ~55 % slower
     * (RHP_STAMPS, chunked: 500 vs 780 us for the same four rounds, the
     * workgroup's end set by its slowest wave), so the faster waves take more
     * rounds (round 5) */
    uint32_t *round_next = wg_counter + 2;   /* entries claimed; 0 since the prologue */
    /* A round is at most 64 entries (one per lane).  Near the end of the range
     * the rounds shrink (32, then 16 entries: RHP_TAIL_ROUNDS), so the last ones
     * -- a 64-body round of chunked moves is ~150 us of one wave -- end closer
     * together; a wave judges "near the end" from its own last claim */
    auto claim = [&](uint32_t last) -> uint2 {
      uint32_t want = 64u;
#ifdef RHP_TAIL_ROUNDS
      const uint32_t left = ns > last ? ns - last : 0u;
      want = left > 32u * WAVES * 2u ? 64u : left > 16u * WAVES * 2u ? 32u : 16u;
#endif
      (void) last;
      uint32_t r = 0;
      if (lane == 0) r = atomicAdd(round_next, want);
      r = __builtin_amdgcn_readfirstlane(r);
      return uint2{r, min(r + want, ns)};
    };
    uint2 kr = claim(0u);
    if (kr.x < ns) start_round(kr.x, kr.y);
    while (kr.x < ns) {
      const uint2 kn = claim(kr.y);
      if constexpr (http) {
        dg.part_begin();
        while (__builtin_amdgcn_ballot_w64(w.live)) w.step();   /* what the last round's moves left */
        StagedBody sb;
        const bool staged = walking && finish_chunked(w, wret, &p.http[wi], p.compact, &sb);
        if (walking) mark_wide(p, wi);
        dg.part_end(4);
        const uint64_t m = __builtin_amdgcn_ballot_w64(staged);
        if (kn.x < ns) start_round(kn.x, kn.y);
        else walking = w.live = false;
        dg.part_begin();
        if (m) staged_moves(m, sb, lane, stage, kLdsTable - (uint32_t) WAVES * kChunkTabWave + (tid >> 6) * kChunkTabWave,
                            [&]() { w.step(); });
        dg.part_end(5);
      } else {
        if (kn.x < ns) start_round(kn.x, kn.y);
      }
      kr = kn;
    }
    dg.pass_end(0);
  }
  dg.exit(WAVES);
}

/* rhp_pack_dense (rhp.h): one thread per record slot, the dense encodings of
 * its request-major records (the host expands them: reactor/batch.c) */
__global__ __launch_bounds__(256) void rhp_pack_dense_kernel(const rhp_req_t *reqs, const rhp_hdr_t *hdrs,
                                                             const rhp_http_t *http, uint32_t n, uint32_t m, uint2 *dreq,
                                                             uint2 *hc, uint16_t *lens16)
{
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const rhp_req_t r = reqs[i];
  const rhp_http_t x = http[i];
  /* the http record: compact when its consumed follows from ret (rhp.h) */
  const uint64_t cons = x.result == 1 ? (uint64_t) (uint32_t) r.ret + (x.body_kind == 1 ? x.body_len : 0u) : 0u;
  const bool hok = x.consumed == cons && x.body_kind <= 1u && !(x.body_len >> 32) && (x.result != 1 || r.ret > 0);
  hc[i] = hok ? uint2{((uint32_t) x.result & 0xffu) | x.body_kind << 8, (uint32_t) x.body_len} : uint2{RHP_HTTP_WIDE << 16, 0u};
  /* the request: dense when the DFA's regular form holds it and the http
   * record is compact (a de-framed chunked body moves its request's bytes:
   * the wide records' offsets are the moved ones) */
  bool reg = hok && x.result == 1 && r.ret > 0 && r.ret <= (int32_t) RHP_MAX_LEN && r.method_off == 0 && r.method_len <= 255u &&
             r.path_off == r.method_len + 1u && r.num_headers <= m;
  uint32_t at = (uint32_t) r.path_off + r.path_len + 11u;
  const uint32_t nh = reg ? r.num_headers : 0u;
  for (uint32_t k = 0; k < nh; k++) {
    const rhp_hdr_t h = hdrs[(uint64_t) i * m + k];
    reg = reg && h.name_off == at && h.value_off == at + h.name_len + 2u &&
          max((uint32_t) h.name_len << 4, (uint32_t) h.value_len) <= RHP_DENSE_VALUE_MAX;
    at += (uint32_t) h.name_len + h.value_len + 4u;
    lens16[(uint64_t) k * n + i] = (uint16_t) (h.name_len | (uint32_t) h.value_len << 6);
  }
  dreq[i] = reg ? uint2{(uint32_t) r.ret | (uint32_t) r.path_len << 16,
                        r.method_len | (uint32_t) r.num_headers << 8 | ((uint32_t) (uint8_t) r.minor_version) << 16}
                : uint2{0u, RHP_DENSE_WIDE << 24};
}

/* rhp_fixup_sessions: one wave per session.  The wave first takes the
 * session's leading pieces whose speculative record is the whole piece -- a
 * request that ended exactly at the piece's end with no chunked body to
 * de-frame, the common case of pipelined input -- 64 pieces per step: the
 * sequential walk of the reference's loop would take each of them as it is, in
 * its own slot (rhp_scalar.h fixup_session_t), so only req_start is written.
 * From the first other piece on, lane 0 walks the rest as that loop does. */
__global__ __launch_bounds__(256) void rhp_fixup_kernel(Params p, const rhp_session_t *sessions, uint32_t n_sessions,
                                                       rhp_session_result_t *results, uint64_t *req_start)
{
  const FixupIO io{p.bytes_rw, p.offsets, p.reqs, p.hdrs, p.http, p.hs_req, p.hs_hdr, p.max_headers};
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (k >= n_sessions) return;   /* wave-uniform */
  const rhp_session_t ss = sessions[k];
  uint32_t from = ss.piece_lo;
  while (from < ss.piece_hi) {
    const uint32_t j = from + lane;
    bool whole = false;
    uint64_t a = 0;
    if (j < ss.piece_hi) {
      const rhp_http_t x = p.http[j];
      a = p.offsets[j];
      whole = x.result == 1 && x.body_kind != RHP_BODY_CHUNKED_PENDING && x.consumed == p.offsets[j + 1] - a;
    }
    const uint64_t other = __builtin_amdgcn_ballot_w64(!whole && j < ss.piece_hi);
    const uint32_t stop = other ? from + (uint32_t) __builtin_ctzll(other) : min(from + 64u, ss.piece_hi);
    if (j < stop) req_start[j] = a;
    from = stop;
    if (other) break;
  }
  if (lane == 0)
    fixup_session_t(io, ss.piece_lo, ss.piece_hi, req_start, &results[k],
                    [&](uint64_t at) { return LineBytes{p.bytes_rw + at, ~0ull, {0, 0, 0, 0}}; }, DevDechunk{}, from);
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
std::atomic<uint64_t> g_attr[kMaxDevices];   /* bit 8(w/4)+4compact+2late+http: the LDS attribute of rhp_dfa_kernel<w, late, http, compact> is set */
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

template <int WAVES, bool LATE, bool HTTP, int REC>
int launch_dfa(const Params &prm, hipStream_t s, int dev, int cus)
{
  constexpr uint32_t kX = (LATE && HTTP) ? kHttpXParts : 0u;
  /* table, staging, pool area, the order's bucket cursors past it (the kernel's
   * `bucket`), the extension parts: one sum for the launch and the check */
  constexpr size_t lds_bytes = kLdsTable + (size_t) WAVES * kStageWave + kPoolBytes + 4u * kOrderBuckets +
                               (size_t) WAVES * 1024u * kX;
  static_assert(lds_bytes <= 160u * 1024u, "the workgroup's LDS fits the CU's 160 KiB");
  const uint64_t bit = 1ull << ((3 * (WAVES / 4) + REC) * 4 + (LATE ? 2 : 0) + (HTTP ? 1 : 0));   /* < 64: WAVES 8/12/16 */
  if (!(g_attr[dev].load(std::memory_order_acquire) & bit)) {
    /* idempotent: two threads of one device may both set it */
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&rhp_dfa_kernel<WAVES, LATE, HTTP, REC>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds_bytes);
    if (e != hipSuccess) return (int) e;
    g_attr[dev].fetch_or(bit, std::memory_order_release);
  }
  /* one workgroup per CU (the staging buffers take the LDS) */
  uint32_t grid = (uint32_t) cus;
  uint32_t need = (prm.n + 64 * WAVES - 1) / (64 * WAVES);
  if (grid > need) grid = need > 0 ? need : 1;
  /* each workgroup owns a contiguous n/grid share of the requests */
  Params q = prm;
  q.span = (prm.n + grid - 1) / grid;
  hipLaunchKernelGGL((rhp_dfa_kernel<WAVES, LATE, HTTP, REC>), dim3(grid), dim3(WAVES * 64), lds_bytes, s, q);
  return (int) hipGetLastError();
}

/* waves per workgroup of the phr-mode kernels (16: four per SIMD) */
#ifndef RHP_PHR_WAVES
#define RHP_PHR_WAVES 16
#endif

/* the late-issue form: http mode (frames requests in the loop), or on request
 * (RHP_IMPL_DFA_LATE, parity tests of that form in phr mode) */
bool late_issue(uint32_t mode) { return t_impl == RHP_IMPL_DFA_LATE || mode == RHP_MODE_HTTP; }
}  // namespace

extern "C" {

const char *rhp_version(void) { return "rhp 0.5.0 (gfx950)"; }

#ifdef RHP_STAMPS
/* diagnostic build only: the per-wave stamps (8192 x kStampSlots u64) */
int rhp_debug_stamps(unsigned long long *host)
{
  return (int) hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps), 0, hipMemcpyDeviceToHost);
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
  if (impl != RHP_IMPL_DFA && impl != RHP_IMPL_EXACT && impl != RHP_IMPL_DFA_LATE) return -22;
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
  if ((uint64_t) b->n * b->max_headers > 0xffffffffull) return -22;   /* record indices are 32-bit */
  if (b->mode == RHP_MODE_HTTP && (!b->http || !b->bytes_rw)) return -22;
  if (b->mode != RHP_MODE_PHR && b->mode != RHP_MODE_HTTP) return -22;
  if (b->layout != RHP_LAYOUT_REQUEST_MAJOR && b->layout != RHP_LAYOUT_HEADER_MAJOR &&
      !(b->layout == RHP_LAYOUT_COMPACT && !(b->flags & RHP_BATCH_SPECULATIVE)) &&
      !(b->layout == RHP_LAYOUT_DENSE || b->layout == RHP_LAYOUT_DENSE_RM))
    return -22;   /* compact: not speculative; dense: below */
  if (b->last_len && b->mode != RHP_MODE_PHR) return -22;   /* http_read_request passes last_len 0 */
  if ((b->flags & ~RHP_BATCH_SPECULATIVE) || ((b->flags & RHP_BATCH_SPECULATIVE) && b->mode != RHP_MODE_HTTP)) return -22;
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
  prm.last_len = b->last_len;
  prm.compact = !(b->flags & RHP_BATCH_SPECULATIVE);
  prm.n = b->n;
  prm.max_headers = b->max_headers;
  prm.mode = b->mode;
  prm.span = 0;
  const bool hmajor = b->layout == RHP_LAYOUT_HEADER_MAJOR;
  const bool compact = b->layout == RHP_LAYOUT_COMPACT;
  const bool dense = b->layout == RHP_LAYOUT_DENSE || b->layout == RHP_LAYOUT_DENSE_RM;
  if (dense && (b->mode == RHP_MODE_HTTP ? b->layout != RHP_LAYOUT_DENSE || (b->flags & RHP_BATCH_SPECULATIVE) : false))
    return -22;   /* http mode: header-major dense records, not speculative */
  prm.hs_req = hmajor ? 1u : b->max_headers;
  prm.hs_hdr = hmajor ? b->n : 1u;
  prm.lens = nullptr;
  prm.hc = nullptr;
  prm.dreq = nullptr;
  prm.lens16 = nullptr;
  prm.ovf32 = nullptr;
  prm.rec_req = prm.hs_req;
  prm.rec_hdr = prm.hs_hdr;
  prm.wt_records = b->mode == RHP_MODE_PHR && b->layout != RHP_LAYOUT_REQUEST_MAJOR && b->layout != RHP_LAYOUT_DENSE_RM;
  if (dense) {   /* 8-byte request records and u16 lengths (header-major), the wide ones behind them */
    prm.dreq = reinterpret_cast<uint2 *>(b->reqs);
    prm.reqs = reinterpret_cast<rhp_req_t *>(reinterpret_cast<uint8_t *>(b->reqs) + RHP_DENSE_REQ_WIDE_OFF(b->n));
    prm.lens16 = reinterpret_cast<uint16_t *>(b->hdrs);
    prm.ovf32 = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(b->hdrs) + RHP_DENSE_OVF_OFF(b->n, b->max_headers));
    prm.hdrs = reinterpret_cast<rhp_hdr_t *>(reinterpret_cast<uint8_t *>(b->hdrs) + RHP_DENSE_WIDE_OFF(b->n, b->max_headers));
    prm.hs_req = b->max_headers;   /* the exact path's wide records: request-major */
    prm.hs_hdr = 1u;
    const bool rm = b->layout == RHP_LAYOUT_DENSE_RM;   /* the u16 lengths request-major or header-major */
    prm.rec_req = rm ? b->max_headers : 1u;
    prm.rec_hdr = rm ? 1u : b->n;
    if (b->mode == RHP_MODE_HTTP) {   /* the compact http records, as RHP_LAYOUT_COMPACT's */
      prm.hc = reinterpret_cast<uint2 *>(b->http);
      prm.http = reinterpret_cast<rhp_http_t *>(reinterpret_cast<uint8_t *>(b->http) + RHP_COMPACT_HTTP_WIDE_OFF(b->n));
    }
  }
  if (compact) {   /* lengths header-major at hdrs, the wide records request-major behind them */
    prm.lens = reinterpret_cast<uint32_t *>(b->hdrs);
    prm.hdrs = reinterpret_cast<rhp_hdr_t *>(reinterpret_cast<uint8_t *>(b->hdrs) + RHP_COMPACT_WIDE_OFF(b->n, b->max_headers));
    prm.rec_req = 1u;
    prm.rec_hdr = b->n;
    if (b->mode == RHP_MODE_HTTP) {   /* 8-byte http records, the wide ones (and the replay's hints) behind them */
      prm.hc = reinterpret_cast<uint2 *>(b->http);
      prm.http = reinterpret_cast<rhp_http_t *>(reinterpret_cast<uint8_t *>(b->http) + RHP_COMPACT_HTTP_WIDE_OFF(b->n));
    }
  }

  /* the DFA kernel addresses windows with u32 offsets from its workgroup's
   * range start; a range of ~4 GiB runs the exact path inside it */
  if (t_impl == RHP_IMPL_EXACT) {
    uint32_t grid = (b->n + 255) / 256;
    if (grid > (uint32_t) cus * 8) grid = (uint32_t) cus * 8;
    hipLaunchKernelGGL(rhp_exact_kernel, dim3(grid), dim3(256), 0, s, prm);
    return (int) hipGetLastError();
  }
  const bool late = late_issue(b->mode);
  if (b->mode == RHP_MODE_HTTP)
    return dense     ? launch_dfa<kHttpWaves, true, true, kRecDense>(prm, s, dev, cus)
           : compact ? launch_dfa<kHttpWaves, true, true, kRecCompact>(prm, s, dev, cus)
                     : launch_dfa<kHttpWaves, true, true, kRecWide>(prm, s, dev, cus);
  constexpr int W = RHP_PHR_WAVES;
  if (dense) return late ? launch_dfa<W, true, false, kRecDense>(prm, s, dev, cus) : launch_dfa<W, false, false, kRecDense>(prm, s, dev, cus);
  if (compact) return late ? launch_dfa<W, true, false, kRecCompact>(prm, s, dev, cus) : launch_dfa<W, false, false, kRecCompact>(prm, s, dev, cus);
  if (late) return launch_dfa<W, true, false, kRecWide>(prm, s, dev, cus);
  return launch_dfa<W, false, false, kRecWide>(prm, s, dev, cus);
}

int rhp_pack_dense(const rhp_batch_t *b, rhp_req_dense_t *dreq, rhp_http_compact_t *hc, uint16_t *lens16, void *stream)
{
  if (!b || (b->n && (!b->reqs || !b->http || !dreq || !hc || (b->max_headers && (!b->hdrs || !lens16))))) return -22;
  if (b->mode != RHP_MODE_HTTP || b->layout != RHP_LAYOUT_REQUEST_MAJOR || b->max_headers > RHP_MAX_HEADERS) return -22;
  if (b->n == 0) return 0;
  hipLaunchKernelGGL(rhp_pack_dense_kernel, dim3((b->n + 255u) / 256u), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     b->reqs, b->hdrs, b->http, b->n, b->max_headers, reinterpret_cast<uint2 *>(dreq),
                     reinterpret_cast<uint2 *>(hc), lens16);
  return (int) hipGetLastError();
}

int rhp_fixup_sessions(const rhp_batch_t *b, const rhp_session_t *sessions, uint32_t n_sessions,
                       rhp_session_result_t *results, uint64_t *req_start, void *stream)
{
  if (!b || (n_sessions && (!sessions || !results || !req_start))) return -22;
  if (n_sessions == 0) return 0;
  if (b->mode != RHP_MODE_HTTP || !(b->flags & RHP_BATCH_SPECULATIVE)) return -22;
  if (!b->bytes_rw || !b->offsets || !b->reqs || !b->http || (b->max_headers && !b->hdrs)) return -22;
  if (b->layout != RHP_LAYOUT_REQUEST_MAJOR && b->layout != RHP_LAYOUT_HEADER_MAJOR) return -22;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Params prm = {};
  prm.bytes = b->bytes;
  prm.bytes_rw = b->bytes_rw;
  prm.offsets = b->offsets;
  prm.reqs = b->reqs;
  prm.hdrs = b->hdrs;
  prm.http = b->http;
  prm.n = b->n;
  prm.max_headers = b->max_headers;
  prm.mode = b->mode;
  prm.compact = true;
  const bool hmajor = b->layout == RHP_LAYOUT_HEADER_MAJOR;
  prm.hs_req = hmajor ? 1u : b->max_headers;
  prm.hs_hdr = hmajor ? b->n : 1u;
  prm.lens = nullptr;
  prm.rec_req = prm.hs_req;
  prm.rec_hdr = prm.hs_hdr;
  prm.wt_records = false;
  const uint32_t grid = (n_sessions + 3u) / 4u;   /* four sessions (waves) per workgroup */
  hipLaunchKernelGGL(rhp_fixup_kernel, dim3(grid), dim3(256), 0, s, prm, sessions, n_sessions, results, req_start);
  return (int) hipGetLastError();
}

}  // extern "C"
