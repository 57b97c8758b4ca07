/*
 * batch.c -- the session parser behind the server: one rhp_parse_batch call
 * (include/rhp.h) over the packed unconsumed input of every session that has
 * bytes to parse in a reactor round.
 *
 * "gpu" (default): a round is packed into one of REACTOR_BATCH_SLOTS pinned
 * host slots, then H2D copies, the MI355X kernel and the D2H copies of the
 * records are queued on this thread's HIP stream and the call returns.  A host
 * function queued behind them writes the thread's eventfd, which the server
 * polls from the reactor loop (the reference's reactor_async pattern,
 * reactor.c:316-330: work off the loop, completion by eventfd), so the loop
 * keeps serving sockets, and the server packs the next round, while a round
 * parses.  The parser is the product path: when RHP_REACTOR_PARSER is unset or
 * "gpu" and no GPU or librhp.so is usable, the process stops with an error (no
 * silent fallback).
 * "host": the product's exact scalar parser (rhp_cpu_parse_batch) in place,
 * synchronously, selected explicitly for CPU-only hosts and the CPU suite.
 * "host-async": the same parser on a worker thread with the gpu mode's
 * completion protocol (slots, eventfd), so the CPU suite exercises the
 * server's pipelined rounds.
 *
 * Replies (RHP_REACTOR_WRITER): "gpu" serializes the replies a round's
 * dispatch produced in one rhp_write_responses call (http_write_response for
 * the whole round, include/rhp.h); "host-batch" runs the same round-batched
 * protocol with the host serializer (CPU tests); unset or "host": each reply
 * is written as the reference does, when the handler responds.
 */
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <stdbool.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <hip/hip_runtime_api.h>

#include "reactor.h"
#include "reactor_batch.h"
#include "rhp.h"
#include "rhp_host.h"

enum { PARSER_UNSET, PARSER_GPU, PARSER_HOST, PARSER_HOST_ASYNC };

/* A slot's round lives in ONE buffer, the same layout on the host (pinned) and
 * the device: the input [bytes + RHP_PAD | offsets | sessions] goes over in one
 * H2D copy; then
 * [bytes | offsets | sessions | reqs | hdrs | http | req_start | session results | dreq | hc | lens16]:
 * the batch's own records (request-major, what rhp_fixup_sessions works on),
 * the session results and, round 6, their dense copies (rhp_pack_dense:
 * 8-byte request and http records, u16 header lengths header-major).  One D2H
 * copy brings back the session results, the dense records and the length rows
 * the round's requests use (the records had come back
 * request-major at 176 B per request); a slot the dense form cannot hold (the
 * exact path's irregular records, a de-framed chunked body) has the batch's own
 * records fetched for the round, and the bytes come back only for chunked
 * bodies (reactor_batch_result). */
typedef struct slot
{
  size_t       cap;          /* bytes of h_buf / d_buf */
  uint8_t     *h_buf, *d_buf;
  size_t       in_size, out_size;   /* this round: the input prefix, the whole layout */
  size_t       o_off, o_sess, o_req, o_hdr, o_http, o_start, o_sres, o_dreq, o_hc, o_lens;
  rhp_req_dense_t    *h_dreq;
  rhp_http_compact_t *h_hc;
  uint16_t           *h_lens;
  uint32_t            rows;   /* length rows the round's D2H copy brought back */
  uint8_t     *h_bytes;      /* = h_buf */
  uint64_t    *h_off;
  rhp_req_t   *h_req;
  rhp_hdr_t   *h_hdr;
  rhp_http_t  *h_http;
  uint64_t    *h_start;      /* rhp_fixup_sessions: where each record slot's request starts */
  rhp_session_t        *h_sess;
  rhp_session_result_t *h_sres;
  uint32_t     n, n_sess;
  size_t       bytes;
  uint64_t     t_submit;
  /* RHP_REACTOR_STATS=2 (the per-phase timeline): timing events around the
   * round's H2D, parse, fix-up and D2H, and host clocks of its submit's end and
   * of the completion thread's wake-up */
  hipEvent_t   tev[5];
  uint64_t     t_enqueued, t_wake, t_h2d_call, t_launch_calls;
} slot_t;

typedef struct batch_state
{
  int          parser;
  hipStream_t  stream;
  hipStream_t  wstream;      /* the gpu writer's own stream: its syncs never wait for a queued parse round */
  int          efd;          /* gpu: written once per completed round */
  slot_t       slot[REACTOR_BATCH_SLOTS];
  void        *d_work;
  int          diag_host;   /* RHP_REACTOR_DIAG=hostparse: gpu-mode buffers, host parse (diagnostic) */
  int          pack;        /* gpu: the dense copy-back (RHP_REACTOR_PACK=0: the request-major records, A/B) */
  uint32_t     rows_hint;   /* length rows the last round used: the next round's D2H copies as many */
  /* gpu: how a round's completion reaches the eventfd (RHP_REACTOR_COMPLETE):
   * COMPLETE_HOSTFUNC a hipLaunchHostFunc behind the round's copies (the HIP
   * runtime's callback thread writes the eventfd); COMPLETE_EVENT a waiter
   * thread of ours blocks in hipEventSynchronize on the round's event
   * (hipEventBlockingSync) and writes it; COMPLETE_SPIN the waiter polls
   * hipEventQuery (lowest latency, one busy core while rounds are in flight) */
  int             complete;
  hipEvent_t      ev[REACTOR_BATCH_SLOTS];
  /* host-async, and the gpu waiter: the worker's queue of submitted slots (in order) */
  pthread_t       worker;
  pthread_mutex_t mu;
  pthread_cond_t  cv;
  int             q[REACTOR_BATCH_SLOTS], q_head, q_n;
  /* the round-batched writer */
  int             writer;
  size_t          w_cap_arena, w_cap_n, w_cap_f, w_cap_out;
  void           *dw_arena, *dw_resps, *dw_fields, *dw_out, *dw_off, *dw_work;
  uint8_t        *hw_out;
  uint64_t       *hw_off;
  /* the waiter / worker thread: started once, stopped and joined at teardown */
  int             have_worker, stop;
  hipStream_t     cstream;   /* gpu: D2H of a round's de-framed bytes, when it has chunked bodies */
  int             delay_us;   /* RHP_REACTOR_DELAY_COMPLETION_US (tests): the completion thread sleeps before its write */
  /* the host-batch writer's reply buffer and offsets (freed at teardown) */
  buffer_t        hb_buf;
  uint64_t       *hb_off;
  size_t          hb_cap;
} batch_state_t;

/* One parser per reactor thread, on the heap: the waiter / worker thread holds
 * a pointer to it, so it must outlive the thread's TLS.  A thread-exit hook
 * (pthread key destructor) stops and joins that thread, waits for the rounds
 * in flight, and frees the events, streams and buffers. */
static __thread batch_state_t *B;
static pthread_key_t   batch_key;
static pthread_once_t  batch_once = PTHREAD_ONCE_INIT;
static void batch_teardown(void *);
static void batch_key_init(void)
{
  if (pthread_key_create(&batch_key, batch_teardown) != 0)
    abort();
}

/* RHP_REACTOR_STATS=1: rounds, requests and submit -> result time of every
 * thread, printed at exit */
static uint64_t st_rounds, st_requests, st_ns;
static int      st_on;
/* RHP_REACTOR_STATS=2: sums over the rounds, ns (device phases from the events) */
enum { PH_SUBMIT, PH_H2D_CALL, PH_LAUNCH_CALLS, PH_H2D, PH_PARSE, PH_FIXUP, PH_D2H, PH_DEVICE, PH_WAKE, PH_LOOP, PH_COUNT };
static uint64_t st_phase[PH_COUNT], st_tl_rounds;
static const char *const st_phase_name[PH_COUNT] = {
  "submit (host: H2D, kernels, D2H enqueued)", "  of it the H2D call", "  of it the two launches",
  "H2D", "rhp_parse_batch", "rhp_fixup_sessions", "D2H records",
  "device span (H2D start -> D2H end)", "submit -> completion thread awake", "completion thread -> loop takes the result"};

static void host_parse(batch_state_t *b, int k);
static uint64_t now_ns(void);

/* The worker / waiter has finished the round at the head of the queue: the
 * eventfd is written BEFORE the entry leaves the queue, so once
 * reactor_batch_wait has seen the queue empty every completion is on the
 * eventfd (written after it, the last warm-up round's write could
 * land after reactor_batch_prepare drained the eventfd and finish the first
 * real round early).  The loop thread may hear of the round and submit its
 * slot again before the entry leaves: reactor_batch_submit waits for room.
 * Called with b->mu unlocked; returns with it locked. */
static void round_complete(batch_state_t *b)
{
  if (b->delay_us)   /* test knob: a late completion write (RHP_REACTOR_DELAY_COMPLETION_US) */
    usleep((useconds_t) b->delay_us);
  const uint64_t one = 1;
  ssize_t r = write(b->efd, &one, sizeof one);
  (void) r;
  pthread_mutex_lock(&b->mu);
  b->q_head = (b->q_head + 1) % REACTOR_BATCH_SLOTS;
  b->q_n--;
  pthread_cond_broadcast(&b->cv);
}

/* queue slot k for the worker / waiter (in submission order) */
static void queue_slot(batch_state_t *b, int k)
{
  pthread_mutex_lock(&b->mu);
  while (b->q_n >= REACTOR_BATCH_SLOTS)   /* a completed round whose entry has not left yet */
    pthread_cond_wait(&b->cv, &b->mu);
  b->q[(b->q_head + b->q_n) % REACTOR_BATCH_SLOTS] = k;
  b->q_n++;
  pthread_cond_broadcast(&b->cv);
  pthread_mutex_unlock(&b->mu);
}

/* host-async worker: the state is its creator's (B is per thread) */
static void *host_worker(void *arg)
{
  batch_state_t *b = arg;
  pthread_mutex_lock(&b->mu);
  for (;;)
  {
    while (!b->q_n && !b->stop)
      pthread_cond_wait(&b->cv, &b->mu);
    if (!b->q_n)
      break;   /* stopped, nothing queued */
    const int k = b->q[b->q_head];
    pthread_mutex_unlock(&b->mu);
    host_parse(b, k);
    round_complete(b);
  }
  pthread_mutex_unlock(&b->mu);
  return NULL;
}

enum { COMPLETE_HOSTFUNC, COMPLETE_EVENT, COMPLETE_SPIN };

/* gpu completion waiter (COMPLETE_EVENT / COMPLETE_SPIN): the state is its
 * creator's (B is per thread) */
static void *gpu_waiter(void *arg)
{
  batch_state_t *b = arg;
  pthread_mutex_lock(&b->mu);
  for (;;)
  {
    while (!b->q_n && !b->stop)
      pthread_cond_wait(&b->cv, &b->mu);
    if (!b->q_n)
      break;   /* stopped, nothing queued */
    const int k = b->q[b->q_head];
    pthread_mutex_unlock(&b->mu);
    if (b->complete == COMPLETE_SPIN)
    {
      while (hipEventQuery(b->ev[k]) == hipErrorNotReady)
        ;
    }
    else
      (void) hipEventSynchronize(b->ev[k]);
    if (st_on == 2)
      b->slot[k].t_wake = now_ns();
    round_complete(b);
  }
  pthread_mutex_unlock(&b->mu);
  return NULL;
}

static uint64_t now_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t) ts.tv_sec * 1000000000u + (uint64_t) ts.tv_nsec;
}

static void print_stats(void)
{
  const uint64_t tr = __atomic_load_n(&st_tl_rounds, __ATOMIC_RELAXED);
  if (st_on == 2 && tr)
  {
    fprintf(stderr, "reactor round timeline (mean over %llu gpu rounds, us):\n", (unsigned long long) tr);
    for (int k = 0; k < PH_COUNT; k++)
      fprintf(stderr, "  %-48s %9.1f\n", st_phase_name[k], (double) st_phase[k] / 1e3 / (double) tr);
  }
  const uint64_t r = __atomic_load_n(&st_rounds, __ATOMIC_RELAXED), q = __atomic_load_n(&st_requests, __ATOMIC_RELAXED);
  const uint64_t ns = __atomic_load_n(&st_ns, __ATOMIC_RELAXED);
  fprintf(stderr, "reactor parser %s: %llu rounds, %llu requests (%.1f per round), %.1f us per round (submit to result)\n",
          getenv("RHP_REACTOR_PARSER") ? getenv("RHP_REACTOR_PARSER") : "gpu", (unsigned long long) r,
          (unsigned long long) q, r ? (double) q / (double) r : 0.0, r ? (double) ns / 1e3 / (double) r : 0.0);
}

static void die(const char *what, int e)
{
  fprintf(stderr, "reactor: GPU request parser unavailable (%s: %d); set RHP_REACTOR_PARSER=host to parse on the host\n",
          what, e);
  abort();
}

#define HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) die(#x, (int) e_); } while (0)

static void stats_init(void)
{
  const char *st = getenv("RHP_REACTOR_STATS");
  if ((st_on = st && (*st == '1' || *st == '2') ? *st - '0' : 0))
    atexit(print_stats);
}

static int parser(void)
{
  if (!B)
  {
    static pthread_once_t stats_once = PTHREAD_ONCE_INIT;
    pthread_once(&stats_once, stats_init);
    pthread_once(&batch_once, batch_key_init);
    if (!(B = calloc(1, sizeof *B)))
      abort();
    if (pthread_setspecific(batch_key, B) != 0)
      abort();
  }
  if (B->parser == PARSER_UNSET)
  {
    const char *e = getenv("RHP_REACTOR_PARSER");
    B->parser = !e ? PARSER_GPU : strcmp(e, "host") == 0 ? PARSER_HOST : strcmp(e, "host-async") == 0 ? PARSER_HOST_ASYNC
                                                                                                       : PARSER_GPU;
    const char *dl = getenv("RHP_REACTOR_DELAY_COMPLETION_US");
    B->delay_us = dl ? atoi(dl) : 0;
    const char *dg = getenv("RHP_REACTOR_DIAG");
    B->diag_host = dg && strcmp(dg, "hostparse") == 0;
    /* the dense copy-back: gpu and host-async (the gpu protocol on the CPU) by
     * default, RHP_REACTOR_PACK=0 / 1 to choose */
    const char *pk = getenv("RHP_REACTOR_PACK");
    B->pack = pk ? strcmp(pk, "0") != 0 : B->parser != PARSER_HOST;
    B->rows_hint = 4;
    B->efd = -1;
    if (B->parser == PARSER_GPU)
    {
      int n = 0;
      HIP(hipGetDeviceCount(&n));
      if (n < 1)
        die("hipGetDeviceCount", 0);
      HIP(hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking));
      const char *c = getenv("RHP_REACTOR_COMPLETE");
      B->complete = !c ? COMPLETE_EVENT : strcmp(c, "hostfunc") == 0 ? COMPLETE_HOSTFUNC
                                       : strcmp(c, "spin") == 0   ? COMPLETE_SPIN
                                                                  : COMPLETE_EVENT;
      if (B->complete != COMPLETE_HOSTFUNC)
        for (int k = 0; k < REACTOR_BATCH_SLOTS; k++)
          HIP(hipEventCreateWithFlags(&B->ev[k], hipEventDisableTiming |
                                                    (B->complete == COMPLETE_EVENT ? hipEventBlockingSync : 0)));
    }
    if (B->parser != PARSER_HOST)
    {
      B->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      if (B->efd < 0)
        die("eventfd", errno);
    }
    if (B->parser == PARSER_HOST_ASYNC || (B->parser == PARSER_GPU && B->complete != COMPLETE_HOSTFUNC))
    {
      pthread_mutex_init(&B->mu, NULL);
      pthread_cond_init(&B->cv, NULL);
      if (pthread_create(&B->worker, NULL, B->parser == PARSER_GPU ? gpu_waiter : host_worker, B) != 0)
        abort();
      B->have_worker = 1;
    }
  }
  return B->parser;
}

const char *reactor_parser_name(void)
{
  const int p = parser();
  return p == PARSER_GPU ? "gpu" : p == PARSER_HOST_ASYNC ? "host-async" : "host";
}

int reactor_batch_async(void)
{
  return parser() != PARSER_HOST;
}

int reactor_batch_fd(void)
{
  (void) parser();
  return B->efd;
}

/* The slots the loop packs rounds into and dispatches from: ordinary pages
 * registered with the runtime (pinned, DMA-able).  hipHostMalloc'd memory is
 * as fast for the copies but the CPU writes it at half the speed and reads it
 * 25 % slower (tools/h2d_probe.c: 27 vs 60 GB/s written, 26 vs 35 GB/s read),
 * and the loop's pack and dispatch are CPU passes over it. */
static void *host_alloc(size_t n)
{
  void *p = NULL;
  if (B->parser == PARSER_GPU)
  {
    n = (n + 4095u) & ~(size_t) 4095u;
    if (!(p = aligned_alloc(4096, n)))
      abort();
    HIP(hipHostRegister(p, n, hipHostRegisterDefault));
  }
  else if (!(p = malloc(n)))
    abort();
  return p;
}

static void host_free(void *p)
{
  if (!p)
    return;
  if (B->parser == PARSER_GPU)
    (void) hipHostUnregister(p);
  free(p);
}

static void dev_free(void **p)
{
  if (*p)
    (void) hipFree(*p);
  *p = NULL;
}

static size_t up16(size_t x) { return (x + 15u) & ~(size_t) 15u; }

uint8_t *reactor_batch_reserve(int k, size_t bytes, uint32_t n, uint32_t n_sessions)
{
  (void) parser();
  slot_t *s = &B->slot[k];
  s->o_off = up16(bytes + RHP_PAD);
  s->o_sess = s->o_off + up16((n + 1u) * sizeof(uint64_t));
  s->in_size = s->o_sess + up16(n_sessions * sizeof(rhp_session_t));
  s->o_req = s->in_size;
  s->o_hdr = s->o_req + up16(n * sizeof(rhp_req_t));
  s->o_http = s->o_hdr + up16((size_t) n * REACTOR_BATCH_HEADERS * sizeof(rhp_hdr_t));
  s->o_start = s->o_http + up16(n * sizeof(rhp_http_t));
  s->o_sres = s->o_start + up16(n * sizeof(uint64_t));
  s->o_dreq = s->o_sres + up16(n_sessions * sizeof(rhp_session_result_t));
  s->o_hc = s->o_dreq + up16(n * sizeof(rhp_req_dense_t));
  s->o_lens = s->o_hc + up16(n * sizeof(rhp_http_compact_t));
  s->out_size = s->o_lens + up16((size_t) n * REACTOR_BATCH_HEADERS * sizeof(uint16_t));
  if (s->out_size > s->cap)
  {
    /* generous first capacities: growing pinned and device buffers costs
     * milliseconds per step (page pinning, frees that synchronise) */
    size_t c = s->cap ? s->cap : 4u << 20;
    while (c < s->out_size)
      c *= 2;
    host_free(s->h_buf);
    s->h_buf = host_alloc(c);
    if (B->parser == PARSER_GPU)
    {
      dev_free((void **) &s->d_buf);
      HIP(hipMalloc((void **) &s->d_buf, c));
      if (!B->d_work)
      {
        HIP(hipMalloc(&B->d_work, RHP_WORK_WORDS * sizeof(uint32_t)));
        HIP(hipMemsetAsync(B->d_work, 0, RHP_WORK_WORDS * sizeof(uint32_t), B->stream));
      }
    }
    s->cap = c;
  }
  s->h_bytes = s->h_buf;
  s->h_off = (uint64_t *) (s->h_buf + s->o_off);
  s->h_sess = (rhp_session_t *) (s->h_buf + s->o_sess);
  s->h_req = (rhp_req_t *) (s->h_buf + s->o_req);
  s->h_hdr = (rhp_hdr_t *) (s->h_buf + s->o_hdr);
  s->h_http = (rhp_http_t *) (s->h_buf + s->o_http);
  s->h_start = (uint64_t *) (s->h_buf + s->o_start);
  s->h_sres = (rhp_session_result_t *) (s->h_buf + s->o_sres);
  s->h_dreq = (rhp_req_dense_t *) (s->h_buf + s->o_dreq);
  s->h_hc = (rhp_http_compact_t *) (s->h_buf + s->o_hc);
  s->h_lens = (uint16_t *) (s->h_buf + s->o_lens);
  return s->h_bytes;
}

uint64_t *reactor_batch_offsets(int k)
{
  return B->slot[k].h_off;
}

rhp_session_t *reactor_batch_sessions(int k)
{
  return B->slot[k].h_sess;
}

/* runs on a HIP runtime thread once the round's copies have landed: wake the
 * reactor loop (write(2) on an eventfd; no HIP call here) */
static void round_done(void *arg)
{
  const uint64_t one = 1;
  ssize_t r = write((int) (intptr_t) arg, &one, sizeof one);
  (void) r;
}

static void host_parse(batch_state_t *st, int k)
{
  slot_t *s = &st->slot[k];
  rhp_batch_t b = {
    .bytes = s->h_bytes, .bytes_rw = s->h_bytes, .offsets = s->h_off, .bytes_size = s->bytes + RHP_PAD, .n = s->n,
    .max_headers = REACTOR_BATCH_HEADERS, .mode = RHP_MODE_HTTP, .reqs = s->h_req, .hdrs = s->h_hdr, .http = s->h_http,
    .flags = RHP_BATCH_SPECULATIVE};
  (void) rhp_cpu_parse_batch(&b);
  (void) rhp_cpu_fixup_sessions(&b, s->h_sess, s->n_sess, s->h_sres, s->h_start);
  if (st->pack)   /* the gpu mode's dense records (host-async: its copy-back protocol on the CPU) */
    (void) rhp_cpu_pack_dense(&b, s->h_dreq, s->h_hc, s->h_lens);
}

void reactor_batch_submit(int k, uint32_t n, size_t bytes, uint32_t n_sessions)
{
  slot_t *s = &B->slot[k];
  s->n = n;
  s->n_sess = n_sessions;
  s->bytes = bytes;
  s->t_submit = st_on ? now_ns() : 0;
  memset(s->h_bytes + bytes, 0, RHP_PAD);
  s->h_off[n] = bytes;
  if (B->parser == PARSER_HOST_ASYNC)
  {
    queue_slot(B, k);
    return;
  }
  if (B->parser == PARSER_HOST || B->diag_host)
  {
    host_parse(B, k);
    if (B->parser == PARSER_GPU)
      round_done((void *) (intptr_t) B->efd);   /* diagnostic mode keeps the asynchronous protocol */
    return;
  }
  const bool tl = st_on == 2;
  if (tl)
  {
    if (!s->tev[0])
      for (int e = 0; e < 5; e++)
        HIP(hipEventCreate(&s->tev[e]));
    HIP(hipEventRecord(s->tev[0], B->stream));
  }
  const uint64_t t_h2d0 = tl ? now_ns() : 0;
  HIP(hipMemcpyAsync(s->d_buf, s->h_buf, s->in_size, hipMemcpyHostToDevice, B->stream));   /* bytes, offsets, sessions */
  const uint64_t t_h2d1 = tl ? now_ns() : 0;
  s->t_h2d_call = t_h2d1 - t_h2d0;
  if (tl)
  {
    HIP(hipEventRecord(s->tev[1], B->stream));
    static int once;
    if (!once++)
    {
      hipPointerAttribute_t pa;
      memset(&pa, 0, sizeof pa);
      const hipError_t e = hipPointerGetAttributes(&pa, s->h_buf);
      fprintf(stderr, "reactor round timeline: slot buffer %p: hipPointerGetAttributes %d, type %d (host pinned = %d)\n",
              (void *) s->h_buf, (int) e, (int) pa.type, (int) hipMemoryTypeHost);
    }
  }
  const uint64_t t_l0 = tl ? now_ns() : 0;
  /* the pieces speculatively, then every session walked in order from its
   * true request boundaries (include/rhp.h rhp_fixup_sessions): all of a
   * round's pipelined requests, bodies included, in this one round */
  uint8_t *d = s->d_buf;
  rhp_batch_t b = {
    .bytes = d, .bytes_rw = d, .offsets = (const uint64_t *) (d + s->o_off), .bytes_size = bytes + RHP_PAD, .n = n,
    .max_headers = REACTOR_BATCH_HEADERS, .mode = RHP_MODE_HTTP, .reqs = (rhp_req_t *) (d + s->o_req),
    .hdrs = (rhp_hdr_t *) (d + s->o_hdr), .http = (rhp_http_t *) (d + s->o_http), .work = B->d_work,
    .flags = RHP_BATCH_SPECULATIVE};
  int rc = rhp_parse_batch(&b, B->stream);
  if (rc != 0)
    die("rhp_parse_batch", rc);
  if (tl)
    HIP(hipEventRecord(s->tev[2], B->stream));
  rc = rhp_fixup_sessions(&b, (const rhp_session_t *) (d + s->o_sess), n_sessions,
                          (rhp_session_result_t *) (d + s->o_sres), (uint64_t *) (d + s->o_start), B->stream);
  if (rc != 0)
    die("rhp_fixup_sessions", rc);
  if (tl)
  {
    HIP(hipEventRecord(s->tev[3], B->stream));
    s->t_launch_calls = now_ns() - t_l0;
  }
  /* the records: one asynchronous copy (the bytes, de-framed in place where a
   * body is chunked, http.c:155, come back only for a round that has such a
   * body: reactor_batch_result).  Dense (B->pack): the session results, the
   * 8-byte request and http records and as many u16 length rows as the last
   * round used; the request-major records otherwise. */
  if (B->pack)
  {
    rc = rhp_pack_dense(&b, (rhp_req_dense_t *) (d + s->o_dreq), (rhp_http_compact_t *) (d + s->o_hc),
                        (uint16_t *) (d + s->o_lens), B->stream);
    if (rc != 0)
      die("rhp_pack_dense", rc);
    s->rows = B->rows_hint < REACTOR_BATCH_HEADERS ? B->rows_hint : REACTOR_BATCH_HEADERS;
    const size_t end = s->o_lens + (size_t) s->rows * n * sizeof(uint16_t);
    HIP(hipMemcpyAsync(s->h_buf + s->o_sres, s->d_buf + s->o_sres, end - s->o_sres, hipMemcpyDeviceToHost, B->stream));
  }
  else
    HIP(hipMemcpyAsync(s->h_buf + s->o_req, s->d_buf + s->o_req, s->o_dreq - s->o_req, hipMemcpyDeviceToHost, B->stream));
  if (tl)
  {
    HIP(hipEventRecord(s->tev[4], B->stream));
    s->t_enqueued = now_ns();
  }
  if (B->complete == COMPLETE_HOSTFUNC)
  {
    HIP(hipLaunchHostFunc(B->stream, round_done, (void *) (intptr_t) B->efd));
    return;
  }
  HIP(hipEventRecord(B->ev[k], B->stream));
  queue_slot(B, k);
}

int reactor_batch_completed(void)
{
  uint64_t v = 0;
  if (read(B->efd, &v, sizeof v) != (ssize_t) sizeof v)
    return 0;
  return (int) v;
}

void reactor_batch_wait(void)
{
  if (!B)
    return;
  if (B->parser == PARSER_GPU)
    HIP(hipStreamSynchronize(B->stream));
  if (B->parser == PARSER_HOST_ASYNC || (B->parser == PARSER_GPU && B->complete != COMPLETE_HOSTFUNC))
  {
    pthread_mutex_lock(&B->mu);
    while (B->q_n)
      pthread_cond_wait(&B->cv, &B->mu);
    pthread_mutex_unlock(&B->mu);
  }
}

void reactor_batch_result(int k, reactor_batch_result_t *out)
{
  slot_t *s = &B->slot[k];
  if (st_on)
  {
    __atomic_fetch_add(&st_rounds, 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&st_requests, s->n, __ATOMIC_RELAXED);
    const uint64_t t_result = now_ns();
    __atomic_fetch_add(&st_ns, t_result - s->t_submit, __ATOMIC_RELAXED);
    if (st_on == 2 && B->parser == PARSER_GPU && s->tev[0] && s->t_wake)
    {
      float ms[5] = {0, 0, 0, 0, 0};
      for (int e = 1; e < 5; e++)
        (void) hipEventElapsedTime(&ms[e], s->tev[e - 1], s->tev[e]);
      float span = 0;
      (void) hipEventElapsedTime(&span, s->tev[0], s->tev[4]);
      const uint64_t add[PH_COUNT] = {s->t_enqueued - s->t_submit, s->t_h2d_call, s->t_launch_calls,
                                      (uint64_t) (ms[1] * 1e6f), (uint64_t) (ms[2] * 1e6f),
                                      (uint64_t) (ms[3] * 1e6f), (uint64_t) (ms[4] * 1e6f), (uint64_t) (span * 1e6f),
                                      s->t_wake - s->t_submit, t_result - s->t_wake};
      for (int k2 = 0; k2 < PH_COUNT; k2++)
        __atomic_fetch_add(&st_phase[k2], add[k2], __ATOMIC_RELAXED);
      __atomic_fetch_add(&st_tl_rounds, 1, __ATOMIC_RELAXED);
      s->t_wake = 0;
    }
  }
  bool wide = !B->pack || (B->parser == PARSER_GPU && B->diag_host);   /* the request-major records are on the host */
  if (!wide)
  {
    /* the dense copy-back (reactor_batch_submit): the length rows the owned
     * slots' dense requests use beyond the ones copied, and the batch's own
     * records when some owned slot is wide (the exact path's, a de-framed
     * chunked body); the next round copies as many rows as this one used */
    uint32_t rows = 0;
    for (uint32_t q = 0; q < s->n_sess; q++)
      for (uint32_t i = s->h_sess[q].piece_lo; i < s->h_sess[q].piece_lo + s->h_sres[q].n_slots && i < s->n; i++)
      {
        /* a wide http record's request is wide too (rhp_pack_dense) */
        const bool hw = s->h_hc[i].flags & RHP_HTTP_WIDE;
        const bool rw = !hw && s->h_hc[i].result == 1 && (s->h_dreq[i].flags & RHP_DENSE_WIDE);
        wide |= hw || rw;
        if (!hw && s->h_hc[i].result == 1 && !rw && s->h_dreq[i].num_headers > rows)
          rows = s->h_dreq[i].num_headers;
      }
    bool sync = false;
    const bool dev = B->parser == PARSER_GPU;   /* host-async: every record is on the host already */
    if (dev && !B->cstream)
      HIP(hipStreamCreateWithFlags(&B->cstream, hipStreamNonBlocking));
    if (dev && rows > s->rows)
    {
      const size_t a = s->o_lens + (size_t) s->rows * s->n * sizeof(uint16_t), e = s->o_lens + (size_t) rows * s->n * sizeof(uint16_t);
      HIP(hipMemcpyAsync(s->h_buf + a, s->d_buf + a, e - a, hipMemcpyDeviceToHost, B->cstream));
      sync = true;
    }
    if (dev && wide)
    {
      HIP(hipMemcpyAsync(s->h_buf + s->o_req, s->d_buf + s->o_req, s->o_sres - s->o_req, hipMemcpyDeviceToHost, B->cstream));
      sync = true;
    }
    if (sync)
      HIP(hipStreamSynchronize(B->cstream));
    B->rows_hint = rows ? rows : 1;
  }
  if (B->parser == PARSER_GPU && !B->diag_host && wide)
  {
    /* only the records came back (reactor_batch_submit): the bytes, de-framed
     * in place by the fix-up, are fetched when some request of the round has a
     * chunked body (the server copies that body from them, server.c) */
    /* only the requests whose chunked body was de-framed: their byte ranges
     * [req_start, + consumed), adjacent ones merged into one copy, or the span
     * from the first to the last when they are many (the whole
     * input came back for one such request) */
    enum { MAX_RUNS = 16 };
    uint64_t run_lo[MAX_RUNS], run_hi[MAX_RUNS], span_lo = 0, span_hi = 0;
    uint32_t runs = 0;
    /* only the record slots the fix-up filled: slots [piece_lo, piece_lo +
     * n_slots) of each session (the slots after them keep the
     * speculative records, whose req_start is whatever the device buffer held);
     * the ranges are clamped to the round's bytes */
    for (uint32_t q = 0; q < s->n_sess; q++)
    for (uint32_t i = s->h_sess[q].piece_lo; i < s->h_sess[q].piece_lo + s->h_sres[q].n_slots && i < s->n; i++)
    {
      const rhp_http_t *x = &s->h_http[i];
      if (!(x->result == 1 && x->body_kind && x->consumed != (uint64_t) s->h_req[i].ret + x->body_len))
        continue;
      const uint64_t a = s->h_start[i] < s->bytes ? s->h_start[i] : s->bytes;
      const uint64_t b = x->consumed < s->bytes - a ? a + x->consumed : s->bytes;
      if (b <= a)
        continue;
      span_lo = runs && span_lo < a ? span_lo : a;
      span_hi = b > span_hi ? b : span_hi;
      if (runs && runs <= MAX_RUNS && a <= run_hi[runs - 1])
        run_hi[runs - 1] = b > run_hi[runs - 1] ? b : run_hi[runs - 1];
      else
      {
        if (runs < MAX_RUNS)
        {
          run_lo[runs] = a;
          run_hi[runs] = b;
        }
        runs++;
      }
    }
    if (runs)
    {
      if (!B->cstream)
        HIP(hipStreamCreateWithFlags(&B->cstream, hipStreamNonBlocking));
      if (runs > MAX_RUNS)
        HIP(hipMemcpyAsync(s->h_buf + span_lo, s->d_buf + span_lo, span_hi - span_lo, hipMemcpyDeviceToHost, B->cstream));
      else
        for (uint32_t r = 0; r < runs; r++)
          HIP(hipMemcpyAsync(s->h_buf + run_lo[r], s->d_buf + run_lo[r], run_hi[r] - run_lo[r], hipMemcpyDeviceToHost,
                             B->cstream));
      HIP(hipStreamSynchronize(B->cstream));
    }
  }
  out->bytes = s->h_bytes;
  out->reqs = s->h_req;
  out->hdrs = s->h_hdr;
  out->n = s->n;
  out->http = s->h_http;
  out->offsets = s->h_off;
  out->sessions = s->h_sess;
  out->session_results = s->h_sres;
  out->req_start = s->h_start;
  out->n_sessions = s->n_sess;
  out->dense = B->pack && !(B->parser == PARSER_GPU && B->diag_host);
  out->dreq = s->h_dreq;
  out->hc = s->h_hc;
  out->lens16 = s->h_lens;
}

void reactor_batch_record(const reactor_batch_result_t *r, uint32_t i, rhp_req_t *req, rhp_http_t *x, rhp_hdr_t *h,
                          const rhp_hdr_t **hp)
{
  if (!r->dense)
  {
    *req = r->reqs[i];
    *x = r->http[i];
    *hp = r->hdrs + (size_t) i * REACTOR_BATCH_HEADERS;
    return;
  }
  const rhp_http_compact_t c = r->hc[i];
  const rhp_req_dense_t d = r->dreq[i];
  const int result = c.flags & RHP_HTTP_WIDE ? r->http[i].result : c.result;
  const bool rw = result == 1 && (d.flags & RHP_DENSE_WIDE);
  if (rw)
  {
    *req = r->reqs[i];
    *hp = r->hdrs + (size_t) i * REACTOR_BATCH_HEADERS;
  }
  else
  {
    /* rhp.h dense records: path_off = method_len + 1, the header offsets a running sum */
    memset(req, 0, sizeof *req);
    req->ret = d.ret;
    req->method_len = d.method_len;
    req->path_off = (uint16_t) (d.method_len + 1u);
    req->path_len = d.path_len;
    req->minor_version = (int8_t) d.minor_version;
    req->num_headers = d.num_headers;
    uint32_t at = (uint32_t) req->path_off + req->path_len + 11u;
    for (uint32_t k = 0; k < d.num_headers && result == 1; k++)
    {
      const uint32_t l = r->lens16[(size_t) k * r->n + i], nl = l & 63u, vl = l >> 6;
      h[k] = (rhp_hdr_t) {(uint16_t) at, (uint16_t) nl, (uint16_t) (at + nl + 2u), (uint16_t) vl};
      at += nl + vl + 4u;
    }
    *hp = h;
  }
  if (c.flags & RHP_HTTP_WIDE)
    *x = r->http[i];
  else
  {
    x->result = c.result;
    x->body_kind = c.body_kind;
    x->body_len = c.body_len;
    x->consumed = c.result == 1 ? (uint64_t) (uint32_t) req->ret + (c.body_kind == 1 ? c.body_len : 0u) : 0u;
  }
}

enum { WRITER_HOST, WRITER_HOST_BATCH, WRITER_GPU };

int reactor_batch_writer(void)
{
  (void) parser();
  if (B->writer == 0)
  {
    const char *e = getenv("RHP_REACTOR_WRITER");
    B->writer = 1 + (!e ? WRITER_HOST : strcmp(e, "gpu") == 0 ? WRITER_GPU : strcmp(e, "host-batch") == 0 ? WRITER_HOST_BATCH
                                                                                                        : WRITER_HOST);
    if (B->writer == 1 + WRITER_GPU && B->parser != PARSER_GPU)
    {
      /* the gpu writer runs on the gpu parser's device */
      fprintf(stderr, "reactor: RHP_REACTOR_WRITER=gpu needs RHP_REACTOR_PARSER=gpu\n");
      abort();
    }
    if (B->writer == 1 + WRITER_GPU)
      HIP(hipStreamCreateWithFlags(&B->wstream, hipStreamNonBlocking));
  }
  return B->writer - 1 != WRITER_HOST;
}

static void grow_dev(void **p, size_t *cap, size_t need)
{
  if (need <= *cap)
    return;
  size_t c = *cap ? *cap : 1u << 16;
  while (c < need)
    c *= 2;
  dev_free(p);
  HIP(hipMalloc(p, c));
  *cap = c;
}

/* n replies in one pass: out_off[0..n] and the bytes out[0, out_off[n]) */
void reactor_batch_write(const uint8_t *arena, size_t arena_n, const rhp_resp_t *resps, uint32_t n,
                         const rhp_resp_field_t *fields, uint32_t n_fields, const char *date, const uint8_t **out,
                         const uint64_t **out_off)
{
  if (B->writer - 1 == WRITER_HOST_BATCH)
  {
    /* the host serializer, into one buffer in reply order (the thread's
     * parser state holds it: batch_teardown frees it) */
    buffer_t buf = B->hb_buf;
    if (n + 1 > B->hb_cap)
    {
      B->hb_cap = n + 1 > 2 * B->hb_cap ? n + 1 : 2 * B->hb_cap;
      if (!(B->hb_off = realloc(B->hb_off, B->hb_cap * sizeof *B->hb_off)))
        abort();
    }
    uint64_t *off = B->hb_off;
    buffer_clear(&buf);
    stream_t tmp;   /* http_write_response appends to a stream's output buffer */
    memset(&tmp, 0, sizeof tmp);
    tmp.output = buf;
    for (uint32_t i = 0; i < n; i++)
    {
      off[i] = buffer_size(&tmp.output);
      const rhp_resp_t *r = &resps[i];
      http_field_t f[64];
      const uint32_t nf = r->fields_count < 64 ? r->fields_count : 64;
      for (uint32_t k = 0; k < nf; k++)
        f[k] = http_field_define(data(arena + fields[r->fields_first + k].name.off, fields[r->fields_first + k].name.len),
                                 data(arena + fields[r->fields_first + k].value.off, fields[r->fields_first + k].value.len));
      http_write_response(&tmp, data(arena + r->status.off, r->status.len), data(date, RHP_DATE_LEN),
                          data(arena + r->type.off, r->type.len), data(arena + r->body.off, r->body.len), f, nf);
    }
    off[n] = buffer_size(&tmp.output);
    B->hb_buf = tmp.output;
    *out = buffer_base(&B->hb_buf);
    *out_off = off;
    (void) arena_n;
    (void) n_fields;
    return;
  }
  /* gpu: H2D of the round's replies, rhp_write_responses, D2H (synchronous, on
   * the writer's own stream: the next parse round, already queued on
   * B->wstream, keeps running meanwhile) */
  grow_dev(&B->dw_arena, &B->w_cap_arena, arena_n + 16);
  size_t cap_n = B->w_cap_n;
  grow_dev(&B->dw_resps, &B->w_cap_n, (size_t) n * sizeof *resps + 16);
  if (B->w_cap_n != cap_n || !B->hw_off)
  {
    dev_free(&B->dw_off);
    dev_free(&B->dw_work);
    if (B->hw_off)
      (void) hipHostFree(B->hw_off);
    const size_t rn = B->w_cap_n / sizeof *resps + 1;
    HIP(hipMalloc(&B->dw_off, rn * sizeof(uint64_t)));
    HIP(hipMalloc(&B->dw_work, RHP_RESP_WORK_WORDS(rn) * sizeof(uint64_t)));
    HIP(hipHostMalloc((void **) &B->hw_off, rn * sizeof(uint64_t), hipHostMallocDefault));
  }
  grow_dev(&B->dw_fields, &B->w_cap_f, (size_t) n_fields * sizeof *fields + 16);
  HIP(hipMemcpyAsync(B->dw_arena, arena, arena_n, hipMemcpyHostToDevice, B->wstream));
  HIP(hipMemcpyAsync(B->dw_resps, resps, (size_t) n * sizeof *resps, hipMemcpyHostToDevice, B->wstream));
  if (n_fields)
    HIP(hipMemcpyAsync(B->dw_fields, fields, (size_t) n_fields * sizeof *fields, hipMemcpyHostToDevice, B->wstream));
  for (int pass = 0; pass < 2; pass++)
  {
    rhp_resp_batch_t w = {.arena = B->dw_arena, .resps = B->dw_resps, .fields = n_fields ? B->dw_fields : NULL, .n = n,
                          .date_len = RHP_DATE_LEN, .date = date, .out_off = B->dw_off, .out = B->dw_out,
                          .out_size = B->w_cap_out, .work = B->dw_work};
    int rc = rhp_write_responses(&w, B->wstream);
    if (rc != 0)
      die("rhp_write_responses", rc);
    HIP(hipMemcpyAsync(B->hw_off, B->dw_off, ((size_t) n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, B->wstream));
    HIP(hipStreamSynchronize(B->wstream));
    if (B->hw_off[n] <= B->w_cap_out)
      break;
    /* the output did not fit: grow it and write again (rhp.h) */
    size_t c = B->w_cap_out ? B->w_cap_out : 1u << 20;
    while (c < B->hw_off[n])
      c *= 2;
    dev_free(&B->dw_out);
    HIP(hipMalloc(&B->dw_out, c));
    if (B->hw_out)
      (void) hipHostFree(B->hw_out);
    HIP(hipHostMalloc((void **) &B->hw_out, c, hipHostMallocDefault));
    B->w_cap_out = c;
  }
  HIP(hipMemcpyAsync(B->hw_out, B->dw_out, B->hw_off[n], hipMemcpyDeviceToHost, B->wstream));
  HIP(hipStreamSynchronize(B->wstream));
  *out = B->hw_out;
  *out_off = B->hw_off;
}

/* thread exit (pthread key destructor): the rounds in flight complete, the
 * waiter / worker thread is stopped and joined, then every resource goes */
static void batch_teardown(void *arg)
{
  batch_state_t *b = arg;
  B = b;   /* the thread's TLS pointer may already be cleared */
  if (b->parser == PARSER_GPU)
    (void) hipStreamSynchronize(b->stream);
  if (b->have_worker)
  {
    pthread_mutex_lock(&b->mu);
    b->stop = 1;
    pthread_cond_broadcast(&b->cv);
    pthread_mutex_unlock(&b->mu);
    (void) pthread_join(b->worker, NULL);
    pthread_mutex_destroy(&b->mu);
    pthread_cond_destroy(&b->cv);
  }
  for (int k = 0; k < REACTOR_BATCH_SLOTS; k++)
  {
    if (b->parser == PARSER_GPU && b->slot[k].tev[0])
      for (int e = 0; e < 5; e++)
        (void) hipEventDestroy(b->slot[k].tev[e]);
    host_free(b->slot[k].h_buf);
    if (b->parser == PARSER_GPU)
      dev_free((void **) &b->slot[k].d_buf);
  }
  if (b->parser == PARSER_GPU)
  {
    if (b->complete != COMPLETE_HOSTFUNC)
      for (int k = 0; k < REACTOR_BATCH_SLOTS; k++)
        (void) hipEventDestroy(b->ev[k]);
    if (b->writer == 1 + WRITER_GPU)
    {
      (void) hipStreamSynchronize(b->wstream);
      dev_free(&b->dw_arena);
      dev_free(&b->dw_resps);
      dev_free(&b->dw_fields);
      dev_free(&b->dw_out);
      dev_free(&b->dw_off);
      dev_free(&b->dw_work);
      if (b->hw_out)
        (void) hipHostFree(b->hw_out);
      if (b->hw_off)
        (void) hipHostFree(b->hw_off);
      (void) hipStreamDestroy(b->wstream);
    }
    dev_free(&b->d_work);
    if (b->cstream)
      (void) hipStreamDestroy(b->cstream);
    (void) hipStreamDestroy(b->stream);
  }
  if (b->efd >= 0)
    close(b->efd);
  buffer_destruct(&b->hb_buf);
  free(b->hb_off);
  free(b);
  B = NULL;
}

void reactor_batch_release(void)
{
  if (!B)
    return;
  /* on the owning thread, while the HIP runtime's per-thread state is intact;
   * the key's destructor is the fallback for threads that exit without it */
  (void) pthread_setspecific(batch_key, NULL);
  batch_teardown(B);
}

void reactor_batch_prepare(void)
{
  if (parser() != PARSER_GPU || B->diag_host || B->slot[0].cap || B->slot[1].cap)
    return;   /* host parsers need no warm-up; slots in use: the thread's rounds have begun */
  /* Everything a first round would otherwise pay inside a client's burst: the
   * pinned and device slots at their first capacity, the code object's load,
   * the kernels' first launches and the completion path, by one round of one
   * request through the whole protocol, waited for here. */
  static const char warm[] = "GET / HTTP/1.1\r\nHost: warm-up\r\n\r\n";
  const size_t n = sizeof warm - 1;
  /* The first copy of a size the runtime hands to the DMA engine costs ~1.4 ms
   * (tools/h2d_probe.c: 1427 us for the first 128-KiB copy of a process, 2 us
   * after; a round of one request copies too little to reach that path), so
   * the slots' whole capacity goes over and back once here */
  for (int k = 0; k < REACTOR_BATCH_SLOTS; k++)
  {
    slot_t *s = &B->slot[k];
    (void) reactor_batch_reserve(k, n, 1, 1);
    memset(s->h_buf, 0, s->cap);
    HIP(hipMemcpyAsync(s->d_buf, s->h_buf, s->cap, hipMemcpyHostToDevice, B->stream));
    HIP(hipMemcpyAsync(s->h_buf, s->d_buf, s->cap, hipMemcpyDeviceToHost, B->stream));
  }
  HIP(hipStreamSynchronize(B->stream));
  for (int k = REACTOR_BATCH_SLOTS - 1; k >= 0; k--)
  {
    uint8_t *h = reactor_batch_reserve(k, n, 1, 1);
    memcpy(h, warm, n);
    reactor_batch_offsets(k)[0] = 0;
    rhp_session_t *ss = reactor_batch_sessions(k);
    ss[0].piece_lo = 0;
    ss[0].piece_hi = 1;
    reactor_batch_submit(k, 1, n, 1);
  }
  /* the warm-up rounds' completions are nobody's: exactly that many are read
   * off the eventfd, waiting for each (whatever the completion path) */
  for (int left = REACTOR_BATCH_SLOTS; left > 0;)
  {
    struct pollfd pfd = {.fd = B->efd, .events = POLLIN};
    if (poll(&pfd, 1, -1) < 0 && errno != EINTR)
      die("poll", errno);
    uint64_t v = 0;
    if (read(B->efd, &v, sizeof v) == (ssize_t) sizeof v)
      left -= (int) v;
  }
  reactor_batch_wait();
}
