/*
 * server.c -- the HTTP server of the libreactor surface (reference
 * src/reactor/server.c, server.h:37-45) with the receive path on the MI355X
 * batch parser.
 *
 * The reference parses a session synchronously when its recv completes
 * (server_session_read, server.c:37-65): parse, SERVER_REQUEST, repeat while
 * the session is READY, then flush.  Here a session that received bytes is
 * queued, and once per reactor round (a reactor_next call) every queued
 * session's unconsumed input is parsed in ONE batch (batch.c), after which
 * SERVER_REQUEST is dispatched per request in session order -- the same flags
 * (READY / PROCESSING), the same abort handling, the same -1 -> close and
 * 0 -> wait outcomes.
 *
 * With the gpu parser a round is asynchronous: it is packed into a batch slot
 * and submitted, the loop goes on serving sockets, and the round is dispatched
 * when its completion arrives on the batch eventfd (polled only while rounds
 * are in flight).  Up to REACTOR_BATCH_SLOTS rounds are in flight per thread:
 * sessions that received bytes meanwhile are packed into the next slot while
 * the first parses; a session belongs to one round at a time.  Rounds complete
 * and dispatch in submission order.
 *
 * Pipelined input: a session's input is split after
 * every empty line (LF LF, LF CR LF: where a header section can end) into
 * pieces of one speculative batch, and the device's fix-up pass
 * (include/rhp.h rhp_fixup_sessions) walks every session from its true
 * request boundaries -- taking a piece's result where more input cannot change
 * it, parsing again where a body ran past its piece -- so all of a round's
 * pipelined requests, bodies (Content-Length, chunked) and LF-only line ends
 * included, are parsed in that one round, as the reference's
 * server_session_read loop (server.c:37-65) parses them in one pass.
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/epoll.h>

#include "reactor.h"
#include "reactor_batch.h"
#include "rhp.h"

#define container_of(p, T, m) ((T *) ((char *) (p) - offsetof(T, m)))

static void list_init(list_t *l) { l->next = l->prev = l; }
static bool list_is_empty(const list_t *l) { return l->next == l; }
static void list_push(list_t *head, list_t *node)
{
  node->prev = head->prev;
  node->next = head;
  head->prev->next = node;
  head->prev = node;
}
static void list_unlink(list_t *node)
{
  node->prev->next = node->next;
  node->next->prev = node->prev;
  list_init(node);
}

/* ---------------------------------------------------------------- date */

static __thread char server_date[30];

static void server_date_update(void)
{
  static const char days[] = "SunMonTueWedThuFriSat", months[] = "JanFebMarAprMayJunJulAugSepOctNovDec";
  time_t t = (time_t) ((reactor_now() + 10000000) / 1000000000);
  struct tm tm;
  char text[64];
  (void) gmtime_r(&t, &tm);
  snprintf(text, sizeof text, "%.3s, %02d %.3s %04d %02d:%02d:%02d GMT", days + 3 * tm.tm_wday, tm.tm_mday,
           months + 3 * tm.tm_mon, tm.tm_year + 1900, tm.tm_hour, tm.tm_min, tm.tm_sec);
  memcpy(server_date, text, 29);   /* "Wed, 16 Aug 2023 10:29:23 GMT" */
}

/* ------------------------------------------------------------- session */

static void server_batch_run(reactor_event_t *);
static void server_rounds_drain(server_t *);

static void server_queue(server_session_t *s)
{
  server_t *server = s->server;
  if (list_is_empty(&s->queued))
    list_push(&server->queue, &s->queued);
  if (!server->batch)
    server->batch = reactor_next(server_batch_run, server);
}

/* a session taking part in a batch round is only marked; the round frees it */
static void server_session_free(server_session_t *s)
{
  stream_destruct(&s->stream);
  list_unlink(&s->link);
  list_unlink(&s->queued);
  if (s->in_round)
    s->dead = true;
  else
    free(s);
}

static void server_session_close(server_session_t *s)
{
  stream_close(&s->stream);
  if (s->abort)
    *s->abort = true;
  if (s->next)
  {
    reactor_cancel(s->next, NULL, NULL);
    s->next = 0;
  }
  list_unlink(&s->queued);
  if (s->flags & SERVER_SESSION_READY)
    server_session_free(s);
}

static void server_session_next(reactor_event_t *event)
{
  server_session_t *s = event->state;
  s->next = 0;
  server_queue(s);
}

static void server_session_stream(reactor_event_t *event)
{
  server_session_t *s = event->state;
  if (reactor_likely(event->type == STREAM_READ))
    server_queue(s);
  else
    server_session_close(s);
}

static void server_create_session(server_t *server, int fd)
{
  server_session_t *s = calloc(1, sizeof *s);
  if (!s)
    abort();
  s->user = server->user;
  s->flags = SERVER_SESSION_READY;
  s->server = server;
  list_init(&s->queued);
  list_push(&server->sessions, &s->link);
  stream_construct(&s->stream, server_session_stream, s);
  stream_open(&s->stream, fd, 0);
}

static void server_accept(reactor_event_t *event)
{
  server_t *server = event->state;
  switch (event->type)
  {
  case NETWORK_ACCEPT:
    server_create_session(server, (int) event->data);
    break;
  case NETWORK_ACCEPT_BIND:
    break;
  default:
    server->accept = 0;
    reactor_call(&server->user, SERVER_ERROR, 0);
    break;
  }
}

static void server_timeout(reactor_event_t *event)
{
  (void) event;
  server_date_update();
}

/* --------------------------------------------------------------- batch */

typedef struct piece
{
  server_session_t *session;
  uint64_t          start;   /* offset in the session's unconsumed input */
  uint64_t          len;
  uint32_t          index;   /* request index in the batch */
} piece_t;

typedef struct round
{
  server_t          *server;
  server_session_t **sessions;
  size_t             n_sessions, cap_sessions;
  piece_t           *pieces;
  size_t             n_pieces, cap_pieces;
} round_t;

/* the rounds in flight on this thread, in submission order (slot = index);
 * the slots are shared by every server of the thread */
static __thread struct
{
  round_t    r[REACTOR_BATCH_SLOTS];
  int        head, count;
  reactor_t  poll;       /* the batch eventfd, registered while count > 0 */
  server_t **waiting;    /* servers turned away while every slot was in flight */
  size_t     n_waiting, cap_waiting;
  int        servers;    /* constructed and not yet destructed on this thread */
} R;

/* the last server of the thread is gone: the rounds' arrays go too */
static void rounds_release(void)
{
  for (int k = 0; k < REACTOR_BATCH_SLOTS; k++)
  {
    free(R.r[k].sessions);
    free(R.r[k].pieces);
    R.r[k] = (round_t) {0};
  }
  free(R.waiting);
  R.waiting = NULL;
  R.n_waiting = R.cap_waiting = 0;
}


static void *grow(void *p, size_t *cap, size_t need, size_t elem)
{
  if (need <= *cap)
    return p;
  size_t c = *cap ? *cap * 2 : 64;
  while (c < need)
    c *= 2;
  p = realloc(p, c * elem);
  if (!p)
    abort();
  *cap = c;
  return p;
}

/* Round-batched replies (reactor_batch_writer): while a round is dispatched,
 * server_respond records each reply (its strings copied into an arena), and
 * the round's sessions are flushed only after one reactor_batch_write call has
 * serialized all of them, in reply order. */
static __thread struct
{
  bool               on;          /* collecting: a round is being dispatched */
  uint8_t           *arena;
  size_t             arena_n, arena_cap;
  rhp_resp_t        *resps;
  server_session_t **owner;
  size_t             n, cap, cap_owner;
  rhp_resp_field_t  *fields;
  size_t             nf, cap_f;
} W;

static rhp_span_t w_span(data_t d)
{
  const size_t n = data_size(d);
  W.arena = grow(W.arena, &W.arena_cap, W.arena_n + n + 4, 1);
  if (n)
    memcpy(W.arena + W.arena_n, data_base(d), n);
  const rhp_span_t sp = {.off = (uint32_t) W.arena_n, .len = (uint32_t) n};
  W.arena_n += n;
  return sp;
}

static void w_record(server_session_t *s, string_t status, string_t type, data_t body, http_field_t *fields,
                     size_t fields_count)
{
  W.resps = grow(W.resps, &W.cap, W.n + 1, sizeof *W.resps);
  W.owner = grow(W.owner, &W.cap_owner, W.n + 1, sizeof *W.owner);
  W.fields = grow(W.fields, &W.cap_f, W.nf + fields_count + 1, sizeof *W.fields);
  rhp_resp_t *r = &W.resps[W.n];
  r->status = w_span(status);
  r->type = w_span(type);
  r->body = w_span(body);
  r->fields_first = (uint32_t) W.nf;
  r->fields_count = (uint32_t) fields_count;
  for (size_t k = 0; k < fields_count; k++)
  {
    W.fields[W.nf].name = w_span(fields[k].name);
    W.fields[W.nf].value = w_span(fields[k].value);
    W.nf++;
  }
  W.owner[W.n++] = s;
}

/* serialize the recorded replies into their sessions' output, then flush the
 * round's sessions */
static void w_flush_round(round_t *r)
{
  if (W.n)
  {
    const uint8_t *out;
    const uint64_t *off;
    reactor_batch_write(W.arena, W.arena_n, W.resps, (uint32_t) W.n, W.fields, (uint32_t) W.nf, server_date, &out, &off);
    for (size_t i = 0; i < W.n; i++)
    {
      server_session_t *s = W.owner[i];
      if (!s->dead && stream_is_open(&s->stream))
        stream_write(&s->stream, data(out + off[i], off[i + 1] - off[i]));
    }
  }
  W.n = W.nf = W.arena_n = 0;
  for (size_t i = 0; i < r->n_sessions; i++)
    if (!r->sessions[i]->dead && stream_is_open(&r->sessions[i]->stream))
      stream_flush(&r->sessions[i]->stream);
}

/* the end of the first empty line at or after p (LF LF or LF CR LF: where a
 * header section can end, picohttpparser.c:266-275), or NULL */
static const uint8_t *find_empty_line(const uint8_t *p, const uint8_t *end)
{
  while (p < end)
  {
    const uint8_t *q = memchr(p, '\n', (size_t) (end - p));
    if (!q || q + 1 >= end)
      return NULL;
    if (q[1] == '\n')
      return q + 2;
    if (q[1] == '\r' && q + 2 < end && q[2] == '\n')
      return q + 3;
    p = q + 1;
  }
  return NULL;
}

/* dispatch the requests the fix-up found in one session's input, in order
 * (record slots lo, lo + 1, ...); false: the session needs another batch over
 * the rest of its input */
static bool server_session_dispatch(server_session_t *s, uint32_t lo, const rhp_session_result_t *sr,
                                    const reactor_batch_result_t *res)
{
  bool abort = false;
  uint32_t m = 0;
  bool more = false;
  while (s->flags & SERVER_SESSION_READY)
  {
    data_t in = stream_read(&s->stream);
    if (m == sr->n_slots)
    {
      more = sr->more || !data_empty(in);   /* pieces ran out, or bytes that arrived during the round */
      break;
    }
    const uint32_t i = lo + m;
    rhp_req_t rq;
    rhp_http_t hx;
    rhp_hdr_t hbuf[REACTOR_BATCH_HEADERS];
    const rhp_hdr_t *hp;
    reactor_batch_record(res, i, &rq, &hx, hbuf, &hp);
    const rhp_http_t *x = &hx;
    int result = x->result;
    size_t consumed = 0;
    if (result == RHP_RET_TOOLONG)
    {
      /* a header section the batch records cannot hold (> RHP_MAX_LEN): the
       * pointer-based host parser answers for this request; the rest of the
       * input goes to the next batch */
      s->request.fields_count = REACTOR_BATCH_HEADERS;
      const size_t before = data_size(in);
      result = http_read_request(&s->stream, &s->request.method, &s->request.target, &s->request.body,
                                 s->request.fields, &s->request.fields_count);
      consumed = before - data_size(stream_read(&s->stream));
    }
    if (result == -1)
    {
      server_session_close(s);
      return true;
    }
    if (result == 0)
      break;   /* incomplete (a TOOLONG request too): the session waits for more bytes */
    if (x->result == RHP_RET_TOOLONG)
      more = true;   /* parsed on the host: the rest of the input goes to the next batch */
    if (x->result != RHP_RET_TOOLONG)
    {
      uint8_t *base = data_base(in);
      if (x->body_kind && x->consumed != (uint64_t) rq.ret + x->body_len)
        memcpy(base, res->bytes + res->req_start[i], x->consumed);   /* chunked body, de-framed in place */
      reactor_http_fill(base, &rq, hp, 1, x,
                        &s->request.method, &s->request.target, &s->request.body, s->request.fields,
                        &s->request.fields_count);
      consumed = x->consumed;
      stream_consume(&s->stream, consumed);
    }
    m++;
    s->flags &= ~SERVER_SESSION_READY;
    s->flags |= SERVER_SESSION_PROCESSING;
    s->abort = &abort;
    reactor_call(&s->user, SERVER_REQUEST, (uintptr_t) s);
    if (reactor_unlikely(abort))
      return true;
    s->abort = NULL;
    s->flags &= ~SERVER_SESSION_PROCESSING;
    if (more)
      break;
  }
  if (!(s->flags & SERVER_SESSION_READY) && m < sr->n_slots)
    more = true;   /* an asynchronous reply: the rest is parsed again once the session is ready */
  if (!W.on)
    stream_flush(&s->stream);   /* round-batched replies: flushed after the round's write (w_flush_round) */
  return !more;
}

/* RHP_REACTOR_STATS=1: time per round phase (split+pack+submit, dispatch), at exit */
static int round_stats = -1;
static uint64_t rs_pack_ns, rs_dispatch_ns, rs_rounds;
static uint64_t rounds_total;   /* rounds submitted with input, every server of the process */

uint64_t reactor_batch_rounds(void) { return __atomic_load_n(&rounds_total, __ATOMIC_RELAXED); }
static uint64_t rs_now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t) ts.tv_sec * 1000000000u + (uint64_t) ts.tv_nsec;
}
static void rs_print(void)
{
  fprintf(stderr, "server rounds: %llu, split+pack+submit %.1f ms, dispatch %.1f ms\n", (unsigned long long) rs_rounds,
          (double) rs_pack_ns / 1e6, (double) rs_dispatch_ns / 1e6);
}

static void round_stats_init(void)
{
  if (round_stats < 0)
  {
    const char *st = getenv("RHP_REACTOR_STATS");
    if ((round_stats = st && (*st == '1' || *st == '2')))
      atexit(rs_print);
  }
}

/* the queued sessions not already in a round, split into pieces; false: none */
static bool round_build(server_t *server, round_t *r, size_t *bytes_out)
{
  r->server = server;
  r->n_sessions = r->n_pieces = 0;
  size_t bytes = 0;
  list_t *it = server->queue.next;
  while (it != &server->queue)
  {
    list_t *nx = it->next;
    server_session_t *s = container_of(it, server_session_t, queued);
    it = nx;
    if (s->in_round)
      continue;   /* stays queued: parsed in a round after its current one */
    list_unlink(&s->queued);
    if (!(s->flags & SERVER_SESSION_READY) || !stream_is_open(&s->stream))
      continue;
    r->sessions = grow(r->sessions, &r->cap_sessions, r->n_sessions + 1, sizeof *r->sessions);
    r->sessions[r->n_sessions++] = s;
    s->in_round = true;
    data_t in = stream_read(&s->stream);
    const uint8_t *b = data_base(in), *end = b + data_size(in), *p = b;
    while (p < end)
    {
      const uint8_t *q = find_empty_line(p, end);
      if (!q)
        q = end;
      r->pieces = grow(r->pieces, &r->cap_pieces, r->n_pieces + 1, sizeof *r->pieces);
      const uint32_t index = (uint32_t) r->n_pieces;
      r->pieces[index] = (piece_t) {.session = s, .start = (uint64_t) (p - b), .len = (uint64_t) (q - p),
                                    .index = index};
      r->n_pieces = index + 1u;
      p = q;
    }
    bytes += data_size(in);
  }
  *bytes_out = bytes;
  return r->n_sessions != 0;
}

/* dispatch a parsed round (slot k) and release its sessions */
static void round_finish(round_t *r, int k, bool dispatch)
{
  const uint64_t t0 = round_stats ? rs_now() : 0;
  reactor_batch_result_t res = {0};
  if (r->n_pieces)
    reactor_batch_result(k, &res);
  size_t i = 0;
  W.on = dispatch && reactor_batch_writer();
  /* batch session i is round session i (a session without input has no
   * pieces and no request) */
  for (; dispatch && r->n_pieces && i < r->n_sessions; i++)
  {
    server_session_t *s = r->sessions[i];
    if (!s->dead && !server_session_dispatch(s, res.sessions[i].piece_lo, &res.session_results[i], &res) && !s->dead)
      server_queue(s);   /* the rest of its input in a later batch */
  }
  if (W.on)
  {
    W.on = false;
    w_flush_round(r);
  }
  for (i = 0; i < r->n_sessions; i++)
  {
    r->sessions[i]->in_round = false;
    if (r->sessions[i]->dead)
      free(r->sessions[i]);
  }
  server_t *server = r->server;
  r->n_sessions = r->n_pieces = 0;
  if (dispatch && !list_is_empty(&server->queue) && !server->batch)
    server->batch = reactor_next(server_batch_run, server);   /* sessions that waited for this round */
  if (round_stats)
    rs_dispatch_ns += rs_now() - t0;
}

/* A server whose batch round found every slot in flight waits here; the next
 * completion re-arms every waiting server (not only the one whose round
 * completed: the slots are shared by all servers of the thread) */
static void server_wait_slot(server_t *server)
{
  for (size_t i = 0; i < R.n_waiting; i++)
    if (R.waiting[i] == server)
      return;
  R.waiting = grow(R.waiting, &R.cap_waiting, R.n_waiting + 1, sizeof *R.waiting);
  R.waiting[R.n_waiting++] = server;
}

static void server_wait_remove(server_t *server)
{
  for (size_t i = 0; i < R.n_waiting; i++)
    if (R.waiting[i] == server)
      R.waiting[i--] = R.waiting[--R.n_waiting];
}

static void server_wake_waiting(void)
{
  while (R.n_waiting)
  {
    server_t *server = R.waiting[--R.n_waiting];
    if (!list_is_empty(&server->queue) && !server->batch)
      server->batch = reactor_next(server_batch_run, server);
  }
}

static void server_batch_ready(reactor_event_t *event)
{
  (void) event;
  for (int c = reactor_batch_completed(); c > 0 && R.count; c--)
  {
    const int k = R.head;
    R.head = (R.head + 1) % REACTOR_BATCH_SLOTS;
    R.count--;
    round_finish(&R.r[k], k, true);
  }
  if (R.count < REACTOR_BATCH_SLOTS)
    server_wake_waiting();
  if (!R.count && R.poll)
  {
    reactor_poll_remove(R.poll);
    R.poll = 0;
  }
}

static void server_batch_run(reactor_event_t *event)
{
  server_t *server = event->state;
  server->batch = 0;
  round_stats_init();
  if (R.count == REACTOR_BATCH_SLOTS)
  {
    server_wait_slot(server);   /* every slot in flight: the next completion schedules this again */
    return;
  }
  const uint64_t t0 = round_stats ? rs_now() : 0;
  const int k = (R.head + R.count) % REACTOR_BATCH_SLOTS;
  round_t *r = &R.r[k];
  size_t bytes = 0;
  if (!round_build(server, r, &bytes))
    return;
  /* pack every session's input, back to back, and parse all pieces at once */
  if (r->n_pieces)
  {
    uint8_t *h = reactor_batch_reserve(k, bytes, (uint32_t) r->n_pieces, (uint32_t) r->n_sessions);
    uint64_t *off = reactor_batch_offsets(k);
    rhp_session_t *ss = reactor_batch_sessions(k);
    size_t at = 0, q = 0;
    for (size_t i = 0; i < r->n_sessions; i++)
    {
      data_t in = stream_read(&r->sessions[i]->stream);
      memcpy(h + at, data_base(in), data_size(in));
      ss[i].piece_lo = (uint32_t) q;
      for (; q < r->n_pieces && r->pieces[q].session == r->sessions[i]; q++)
        off[q] = at + r->pieces[q].start;
      ss[i].piece_hi = (uint32_t) q;
      at += data_size(in);
    }
    reactor_batch_submit(k, (uint32_t) r->n_pieces, bytes, (uint32_t) r->n_sessions);
    __atomic_fetch_add(&rounds_total, 1, __ATOMIC_RELAXED);
  }
  if (round_stats)
  {
    rs_pack_ns += rs_now() - t0;
    rs_rounds++;
  }
  if (!r->n_pieces || !reactor_batch_async())
  {
    round_finish(r, k, true);   /* parsed in place (host parser), or nothing to parse */
    return;
  }
  R.count++;
  if (!R.poll)
    R.poll = reactor_poll(server_batch_ready, NULL, reactor_batch_fd(), EPOLLIN);
}

/* teardown: every round in flight completes; this server's are released
 * without dispatch, other servers' are dispatched */
static void server_rounds_drain(server_t *server)
{
  if (!R.count)
    return;
  reactor_batch_wait();
  (void) reactor_batch_completed();
  while (R.count)
  {
    const int k = R.head;
    R.head = (R.head + 1) % REACTOR_BATCH_SLOTS;
    R.count--;
    round_finish(&R.r[k], k, R.r[k].server != server);
  }
  if (R.poll)
  {
    reactor_poll_remove(R.poll);
    R.poll = 0;
  }
  server_wake_waiting();   /* other servers of the thread that waited for a slot */
}

/* -------------------------------------------------------------- public */

void server_construct(server_t *server, reactor_callback_t *callback, void *state)
{
  *server = (server_t) {.user = reactor_user_define(callback, state)};
  R.servers++;
  list_init(&server->sessions);
  list_init(&server->queue);
  timeout_construct(&server->timeout, server_timeout, NULL);
}

void server_destruct(server_t *server)
{
  server_close(server);
  timeout_destruct(&server->timeout);
  server_wait_remove(server);
  server_rounds_drain(server);
  while (!list_is_empty(&server->sessions))
  {
    server_session_t *s = container_of(server->sessions.next, server_session_t, link);
    if (s->next)
      reactor_cancel(s->next, NULL, NULL);
    if (s->abort)
      *s->abort = true;
    server_session_free(s);
  }
  if (server->batch)
    reactor_cancel(server->batch, NULL, NULL);
  server->batch = 0;
  if (--R.servers <= 0 && !R.count)
  {
    R.servers = 0;
    rounds_release();
  }
}

void server_open(server_t *server, const char *host, int port)
{
  server->accept = network_accept(server_accept, server, host, port, NETWORK_REUSEADDR);
  reactor_batch_prepare();   /* the parser's setup before any client's first burst */
  timeout_set(&server->timeout, (reactor_now() / 1000000000) * 1000000000, 1000000000);
  server_date_update();
}

void server_open_socket(server_t *server, int socket)
{
  server->accept = network_accept_socket(server_accept, server, socket);
  reactor_batch_prepare();   /* the parser's setup before any client's first burst */
  timeout_set(&server->timeout, (reactor_now() / 1000000000) * 1000000000, 1000000000);
  server_date_update();
}

void server_close(server_t *server)
{
  if (server->accept)
  {
    network_cancel(server->accept);
    server->accept = 0;
  }
  timeout_clear(&server->timeout);
}

void server_disconnect(server_session_t *session)
{
  session->flags |= SERVER_SESSION_READY;
  server_session_close(session);
}

void server_respond(server_session_t *session, string_t status, string_t type, data_t body, http_field_t *fields,
                    size_t fields_count)
{
  session->flags |= SERVER_SESSION_READY;
  if (reactor_likely(stream_is_open(&session->stream)))
  {
    if (W.on && (session->flags & SERVER_SESSION_PROCESSING) && session->in_round)
      w_record(session, status, type, body, fields, fields_count);   /* serialized with the round's replies */
    else
      http_write_response(&session->stream, status, data(server_date, 29), type, body, fields, fields_count);
    if (!(session->flags & SERVER_SESSION_PROCESSING))
    {
      stream_flush(&session->stream);
      session->next = reactor_next(server_session_next, session);
    }
  }
  else
  {
    server_session_close(session);
  }
}

void server_ok(server_session_t *session, string_t type, string_t body, http_field_t *fields, size_t fields_count)
{
  server_respond(session, string("200 OK"), type, body, fields, fields_count);
}

void server_plain(server_session_t *session, data_t body, http_field_t *fields, size_t fields_count)
{
  server_respond(session, string("200 OK"), string("text/plain"), body, fields, fields_count);
}
