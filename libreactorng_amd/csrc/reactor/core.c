/*
 * core.c -- data/string/buffer helpers, the event loop, timeouts, the accept
 * side of the network module and buffered streams: the host plumbing around
 * the HTTP receive path (reference src/reactor/{data,string,buffer,reactor,
 * timeout,network,stream}.c), written for epoll.
 *
 * Semantics kept from the reference: reactor_next calls run at the top of the
 * next loop round (reactor.c:264-276); reactor_loop runs while anything is
 * registered (reactor.c:251-255); a stream delivers STREAM_READ after bytes
 * arrived and STREAM_CLOSE on end of file (stream.c:23-44), keeps unconsumed
 * input across reads (stream.c:65-84) and sends only flushed output
 * (stream.c:97-120, 203-207).  Input buffers keep RHP_PAD zero bytes after the
 * received data, the batch contract of the parser (include/rhp.h).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <time.h>
#include <unistd.h>
#include <netinet/in.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/timerfd.h>

#include "reactor.h"
#include "reactor_batch.h"
#include "rhp.h"

/* ---------------------------------------------------------------- data */

data_t data(const void *base, size_t size) { return (data_t) {.iov = {.iov_base = (void *) base, .iov_len = size}}; }
data_t data_null(void) { return data(NULL, 0); }
data_t data_string(const char *s) { return data(s, strlen(s)); }
data_t data_offset(const data_t d, size_t n) { return data((char *) d.iov.iov_base + n, d.iov.iov_len - n); }
data_t data_select(const data_t d, size_t n) { return data(d.iov.iov_base, n); }
size_t data_size(const data_t d) { return d.iov.iov_len; }
bool data_empty(const data_t d) { return d.iov.iov_len == 0; }
void *data_base(const data_t d) { return d.iov.iov_base; }
void *data_end(const data_t d) { return (char *) d.iov.iov_base + d.iov.iov_len; }

bool data_equal(const data_t a, const data_t b)
{
  return a.iov.iov_len == b.iov.iov_len && (a.iov.iov_len == 0 || memcmp(a.iov.iov_base, b.iov.iov_base, a.iov.iov_len) == 0);
}

/* ASCII case-insensitive (the reference uses memcasecmp in the C locale, data.c:11-28) */
bool data_equal_case(const data_t a, const data_t b)
{
  if (a.iov.iov_len != b.iov.iov_len)
    return false;
  const unsigned char *p = a.iov.iov_base, *q = b.iov.iov_base;
  for (size_t i = 0; i < a.iov.iov_len; i++)
  {
    unsigned x = p[i], y = q[i];
    x = x - 'a' < 26u ? x - 32u : x;
    y = y - 'a' < 26u ? y - 32u : y;
    if (x != y)
      return false;
  }
  return true;
}

string_t string(const char *s) { return data_string(s); }
string_t string_data(const data_t d) { return d; }
string_t string_null(void) { return data_null(); }
size_t string_size(const string_t s) { return data_size(s); }
bool string_empty(const string_t s) { return data_empty(s); }
char *string_base(const string_t s) { return data_base(s); }
bool string_equal(const string_t a, const string_t b) { return data_equal(a, b); }
bool string_equal_case(const string_t a, const string_t b) { return data_equal_case(a, b); }

/* -------------------------------------------------------------- buffer */

void buffer_construct(buffer_t *b) { *b = (buffer_t) {.data = data_null(), .capacity = 0}; }
void buffer_destruct(buffer_t *b) { free(data_base(b->data)); buffer_construct(b); }
data_t buffer_data(const buffer_t *b) { return b->data; }
size_t buffer_size(const buffer_t *b) { return data_size(b->data); }
size_t buffer_capacity(const buffer_t *b) { return b->capacity; }
void *buffer_base(const buffer_t *b) { return data_base(b->data); }
void *buffer_end(const buffer_t *b) { return data_end(b->data); }

/* power-of-two capacity (buffer.c:6-17, 56-64), plus RHP_PAD zero bytes past
 * it that nothing writes: the parser's reads past the input (the SP skip of
 * picohttpparser.c:356-362) stay inside the allocation and stop there */
void buffer_reserve(buffer_t *b, size_t capacity)
{
  if (capacity <= b->capacity)
    return;
  size_t c = b->capacity ? b->capacity : 64;
  while (c < capacity)
    c *= 2;
  char *p = realloc(data_base(b->data), c + RHP_PAD);
  if (!p)
    abort();
  memset(p + c, 0, RHP_PAD);
  b->data.iov.iov_base = p;
  b->capacity = c;
}

void buffer_resize(buffer_t *b, size_t size)
{
  buffer_reserve(b, size);
  b->data.iov.iov_len = size;
}

void buffer_append(buffer_t *b, data_t d)
{
  size_t n = buffer_size(b);
  buffer_resize(b, n + data_size(d));
  if (data_size(d))
    memcpy((char *) buffer_base(b) + n, data_base(d), data_size(d));
}

void buffer_erase(buffer_t *b, size_t at, size_t n)
{
  if (n == 0)
    return;
  memmove((char *) buffer_base(b) + at, (char *) buffer_base(b) + at + n, buffer_size(b) - at - n);
  b->data.iov.iov_len -= n;
}

data_t buffer_allocate(buffer_t *b, size_t n)
{
  size_t at = buffer_size(b);
  buffer_resize(b, at + n);
  return data((char *) buffer_base(b) + at, n);
}

void buffer_clear(buffer_t *b) { b->data.iov.iov_len = 0; }

/* ------------------------------------------------------------- reactor */

typedef struct poll_user
{
  reactor_user_t  user;
  int             fd;
  int             dead;
} poll_user_t;

static __thread struct
{
  int              ref;
  int              epfd;
  size_t           users;        /* live polls + queued deferred calls */
  reactor_user_t **next;         /* deferred calls for the next round */
  size_t           next_n, next_cap;
  poll_user_t    **dead;         /* removed polls, freed after the round */
  size_t           dead_n, dead_cap;
  reactor_time_t   time;
} core;

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

reactor_event_t reactor_event_define(void *state, int type, uint64_t data)
{
  return (reactor_event_t) {.state = state, .type = type, .data = data};
}

reactor_user_t reactor_user_define(reactor_callback_t *callback, void *state)
{
  return (reactor_user_t) {.callback = callback, .state = state};
}

void reactor_user_construct(reactor_user_t *user, reactor_callback_t *callback, void *state)
{
  *user = reactor_user_define(callback, state);
}

void reactor_construct(void)
{
  if (!core.ref)
  {
    signal(SIGPIPE, SIG_IGN);
    core.epfd = epoll_create1(EPOLL_CLOEXEC);
    if (core.epfd < 0)
      abort();
  }
  core.ref++;
}

static void reactor_reap(void)
{
  for (size_t i = 0; i < core.dead_n; i++)
    free(core.dead[i]);
  core.dead_n = 0;
}

void reactor_destruct(void)
{
  if (--core.ref)
    return;
  /* the thread's batch parser state (streams, events, pinned and device slots,
   * its completion thread) released here, on the owning thread;
   * kept while the reactor lives, so servers opened one after another reuse
   * its slots at the capacity they grew to */
  reactor_batch_release();
  for (size_t i = 0; i < core.next_n; i++)
    free(core.next[i]);
  free(core.next);
  reactor_reap();
  free(core.dead);
  close(core.epfd);
  memset(&core, 0, sizeof core);
}

reactor_time_t reactor_now(void)
{
  if (!core.time)
  {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME_COARSE, &ts);
    core.time = (reactor_time_t) ts.tv_sec * 1000000000ULL + (reactor_time_t) ts.tv_nsec;
  }
  return core.time;
}

void reactor_call(reactor_user_t *user, int type, uint64_t value)
{
  if (user->callback)
    user->callback((reactor_event_t[]) {reactor_event_define(user->state, type, value)});
}

reactor_t reactor_next(reactor_callback_t *callback, void *state)
{
  reactor_user_t *user = malloc(sizeof *user);
  if (!user)
    abort();
  *user = reactor_user_define(callback, state);
  core.next = grow(core.next, &core.next_cap, core.next_n + 1, sizeof *core.next);
  core.next[core.next_n++] = user;
  core.users++;
  return (reactor_t) (uintptr_t) user | 1u;
}

/* a deferred call keeps its slot and runs with the new callback (NULL: nothing),
 * as the reference's reactor_cancel redirects a pending operation (reactor.c:306-314) */
void reactor_cancel(reactor_t id, reactor_callback_t *callback, void *state)
{
  if (!id)
    return;
  reactor_user_t *user = (reactor_user_t *) (uintptr_t) (id & ~(reactor_t) 1);
  *user = reactor_user_define(callback, state);
}

reactor_t reactor_poll(reactor_callback_t *callback, void *state, int fd, uint32_t events)
{
  poll_user_t *p = calloc(1, sizeof *p);
  if (!p)
    abort();
  p->user = reactor_user_define(callback, state);
  p->fd = fd;
  struct epoll_event ev = {.events = events, .data.ptr = p};
  if (epoll_ctl(core.epfd, EPOLL_CTL_ADD, fd, &ev) == -1)
  {
    free(p);
    return 0;
  }
  core.users++;
  return (reactor_t) (uintptr_t) p;
}

void reactor_poll_update(reactor_t id, uint32_t events)
{
  poll_user_t *p = (poll_user_t *) (uintptr_t) id;
  struct epoll_event ev = {.events = events, .data.ptr = p};
  (void) epoll_ctl(core.epfd, EPOLL_CTL_MOD, p->fd, &ev);
}

void reactor_poll_remove(reactor_t id)
{
  poll_user_t *p = (poll_user_t *) (uintptr_t) id;
  if (!p || p->dead)
    return;
  (void) epoll_ctl(core.epfd, EPOLL_CTL_DEL, p->fd, NULL);
  p->dead = 1;
  core.users--;
  core.dead = grow(core.dead, &core.dead_cap, core.dead_n + 1, sizeof *core.dead);
  core.dead[core.dead_n++] = p;
}

/* RHP_REACTOR_STATS=1: epoll_wait calls and the time blocked in them, at exit */
static int core_stats = -1;
static uint64_t core_wait_ns, core_waits, core_next_ns, core_events_ns, core_events, core_events_cpu_ns;
static uint64_t core_cpu_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t) ts.tv_sec * 1000000000u + (uint64_t) ts.tv_nsec;
}
static uint64_t core_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t) ts.tv_sec * 1000000000u + (uint64_t) ts.tv_nsec;
}
static void core_print_stats(void)
{
  fprintf(stderr, "reactor loop: %llu epoll_wait calls, %.1f ms blocked; deferred calls %.1f ms; %llu events handled in %.1f ms"
          " (thread CPU %.1f ms)\n", (unsigned long long) core_waits, (double) core_wait_ns / 1e6, (double) core_next_ns / 1e6,
          (unsigned long long) core_events, (double) core_events_ns / 1e6, (double) core_events_cpu_ns / 1e6);
}

void reactor_loop_once(void)
{
  if (core_stats < 0)
  {
    const char *st = getenv("RHP_REACTOR_STATS");
    core_stats = st && (*st == '1' || *st == '2');
    if (core_stats)
      atexit(core_print_stats);
  }
  const uint64_t n0 = core_stats > 0 ? core_ns() : 0;
  if (core.next_n)
  {
    reactor_user_t **run = core.next;
    size_t n = core.next_n;
    core.next = NULL;
    core.next_n = core.next_cap = 0;
    core.time = 0;
    for (size_t i = 0; i < n; i++)
    {
      reactor_call(run[i], REACTOR_CALL, 0);
      free(run[i]);
      core.users--;
    }
    free(run);
  }
  if (core_stats > 0)
    core_next_ns += core_ns() - n0;
  if (core.users > core.next_n)
  {
    struct epoll_event ev[256];
    struct timespec w0, w1;
    if (core_stats) clock_gettime(CLOCK_MONOTONIC, &w0);
    int n = epoll_wait(core.epfd, ev, 256, core.next_n ? 0 : -1);
    if (core_stats)
    {
      clock_gettime(CLOCK_MONOTONIC, &w1);
      core_wait_ns += (uint64_t) (w1.tv_sec - w0.tv_sec) * 1000000000u + (uint64_t) w1.tv_nsec - (uint64_t) w0.tv_nsec;
      core_waits++;
    }
    core.time = 0;
    const uint64_t e0 = core_stats > 0 ? core_ns() : 0, c0 = core_stats > 0 ? core_cpu_ns() : 0;
    for (int i = 0; i < n; i++)
    {
      poll_user_t *p = ev[i].data.ptr;
      if (!p->dead)
        reactor_call(&p->user, REACTOR_CALL, ev[i].events);
    }
    if (core_stats > 0)
    {
      core_events_ns += core_ns() - e0;
      core_events_cpu_ns += core_cpu_ns() - c0;
      core_events += n > 0 ? (uint64_t) n : 0;
    }
    reactor_reap();
  }
}

void reactor_loop(void)
{
  while (core.users)
    reactor_loop_once();
}

/* ------------------------------------------------------------- timeout */

static void timeout_ready(reactor_event_t *event)
{
  timeout_t *t = event->state;
  uint64_t n = 0;
  if (read(t->fd, &n, sizeof n) != (ssize_t) sizeof n)
    return;
  reactor_call(&t->user, TIMEOUT_EXPIRE, n);
}

void timeout_construct(timeout_t *t, reactor_callback_t *callback, void *state)
{
  *t = (timeout_t) {.user = reactor_user_define(callback, state), .fd = -1};
}

/* absolute expiry `time` (ns, CLOCK_REALTIME), then every `delay` ns
 * (the reference arms IORING_TIMEOUT_ABS|REALTIME, timeout.c:7-12) */
void timeout_set(timeout_t *t, reactor_time_t time, reactor_time_t delay)
{
  if (t->fd < 0)
  {
    t->fd = timerfd_create(CLOCK_REALTIME, TFD_NONBLOCK | TFD_CLOEXEC);
    if (t->fd < 0)
      return;
    t->poll = reactor_poll(timeout_ready, t, t->fd, EPOLLIN);
  }
  if (!time)
    time = 1;
  struct itimerspec its = {
    .it_interval = {.tv_sec = (time_t) (delay / 1000000000ULL), .tv_nsec = (long) (delay % 1000000000ULL)},
    .it_value = {.tv_sec = (time_t) (time / 1000000000ULL), .tv_nsec = (long) (time % 1000000000ULL)}};
  (void) timerfd_settime(t->fd, TFD_TIMER_ABSTIME, &its, NULL);
}

void timeout_clear(timeout_t *t)
{
  if (t->fd >= 0)
  {
    reactor_poll_remove(t->poll);
    close(t->fd);
    t->fd = -1;
    t->poll = 0;
  }
}

void timeout_destruct(timeout_t *t)
{
  timeout_clear(t);
}

/* ------------------------------------------------------------- network */

typedef struct accept_task
{
  reactor_user_t  user;
  int             fd;
  int             own;       /* fd created here (closed on cancel) */
  int             port;
  int             flags;
  char           *host;
  reactor_t       poll;
  reactor_t       next;
} accept_task_t;

static void accept_ready(reactor_event_t *event)
{
  accept_task_t *t = event->state;
  for (;;)
  {
    int fd = accept4(t->fd, NULL, NULL, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd >= 0)
    {
      reactor_t self = t->poll;
      reactor_call(&t->user, NETWORK_ACCEPT, (uint64_t) fd);
      if (t->poll != self || !t->poll)
        return;   /* cancelled by the callback */
      continue;
    }
    if (errno == EINTR || errno == ECONNABORTED)
      continue;
    if (errno != EAGAIN && errno != EWOULDBLOCK)
      reactor_call(&t->user, NETWORK_ERROR, (uint64_t) errno);
    return;
  }
}

static int listen_socket(const char *host, int port, int flags)
{
  struct addrinfo hints = {.ai_family = AF_UNSPEC, .ai_socktype = SOCK_STREAM, .ai_flags = AI_PASSIVE | AI_NUMERICSERV};
  struct addrinfo *ai = NULL;
  char service[16];
  snprintf(service, sizeof service, "%d", port);
  if (getaddrinfo(host, service, &hints, &ai) != 0 || !ai)
    return -1;
  int fd = socket(ai->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd >= 0)
  {
    if (flags & NETWORK_REUSEADDR)
      (void) setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, (int[]) {1}, sizeof(int));
    if (flags & NETWORK_REUSEPORT)
      (void) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, (int[]) {1}, sizeof(int));
    if (bind(fd, ai->ai_addr, ai->ai_addrlen) == -1 || listen(fd, SOMAXCONN) == -1)
    {
      close(fd);
      fd = -1;
    }
  }
  freeaddrinfo(ai);
  return fd;
}

/* runs inside the loop, like the reference's resolve -> socket step (network.c:292-346) */
static void accept_start(reactor_event_t *event)
{
  accept_task_t *t = event->state;
  t->next = 0;
  t->fd = listen_socket(t->host, t->port, t->flags);
  if (t->fd < 0)
  {
    reactor_call(&t->user, NETWORK_ERROR, (uint64_t) errno);
    return;
  }
  t->poll = reactor_poll(accept_ready, t, t->fd, EPOLLIN);
  reactor_call(&t->user, NETWORK_ACCEPT_BIND, (uint64_t) t->fd);
}

static void accept_error(reactor_event_t *event)
{
  accept_task_t *t = event->state;
  t->next = 0;
  reactor_call(&t->user, NETWORK_ERROR, EBADF);
}

network_t network_accept(reactor_callback_t *callback, void *state, const char *host, int port, int flags)
{
  accept_task_t *t = calloc(1, sizeof *t);
  if (!t)
    abort();
  t->user = reactor_user_define(callback, state);
  t->fd = -1;
  t->own = 1;
  t->port = port;
  t->flags = flags;
  t->host = strdup(host ? host : "0.0.0.0");
  t->next = reactor_next(accept_start, t);
  return (network_t) (uintptr_t) t;
}

network_t network_accept_socket(reactor_callback_t *callback, void *state, int fd)
{
  accept_task_t *t = calloc(1, sizeof *t);
  if (!t)
    abort();
  t->user = reactor_user_define(callback, state);
  t->fd = fd;
  int fl = fd >= 0 ? fcntl(fd, F_GETFL) : -1;
  if (fl != -1)
    (void) fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  t->poll = fl != -1 ? reactor_poll(accept_ready, t, fd, EPOLLIN) : 0;
  if (!t->poll)
    t->next = reactor_next(accept_error, t);
  return (network_t) (uintptr_t) t;
}

static void accept_free(reactor_event_t *event)
{
  accept_task_t *t = event->state;
  free(t->host);
  free(t);
}

void network_cancel(network_t id)
{
  accept_task_t *t = (accept_task_t *) (uintptr_t) id;
  if (!t)
    return;
  if (t->next)
    reactor_cancel(t->next, NULL, NULL);
  if (t->poll)
    reactor_poll_remove(t->poll);
  t->poll = 0;
  if (t->own && t->fd >= 0)
    close(t->fd);
  t->fd = -1;
  t->user = reactor_user_define(NULL, NULL);
  (void) reactor_next(accept_free, t);   /* freed after any callback still running on it */
}

/* -------------------------------------------------------------- stream */

enum { STREAM_BLOCK = 16384 };   /* recv size, as the reference (stream.c:8) */

static void stream_send(stream_t *s)
{
  while (s->output_sent < s->output_flushed)
  {
    ssize_t n = send(s->fd, (char *) buffer_base(&s->output) + s->output_sent, s->output_flushed - s->output_sent,
                     MSG_NOSIGNAL);
    if (n > 0)
    {
      s->output_sent += (size_t) n;
      continue;
    }
    if (n < 0 && errno == EINTR)
      continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))
    {
      if (!s->output_wait && s->poll)
        reactor_poll_update(s->poll, (s->flags & STREAM_WRITE_ONLY ? 0 : EPOLLIN) | EPOLLOUT);
      s->output_wait = true;
      return;
    }
    /* peer gone: drop the output; the read side reports the close */
    s->output_sent = s->output_flushed;
    break;
  }
  buffer_erase(&s->output, 0, s->output_sent);
  s->output_flushed -= s->output_sent;
  s->output_sent = 0;
  if (s->output_wait && s->poll)
    reactor_poll_update(s->poll, s->flags & STREAM_WRITE_ONLY ? 0 : EPOLLIN);
  s->output_wait = false;
}

static void stream_receive(stream_t *s)
{
  if (s->input_consumed)
  {
    buffer_erase(&s->input, 0, s->input_consumed);
    s->input_consumed = 0;
  }
  size_t got = 0;
  int closed = 0, error = 0;
  for (;;)
  {
    buffer_reserve(&s->input, buffer_size(&s->input) + STREAM_BLOCK + RHP_PAD);
    ssize_t n = recv(s->fd, buffer_end(&s->input), STREAM_BLOCK, 0);
    if (n > 0)
    {
      buffer_resize(&s->input, buffer_size(&s->input) + (size_t) n);
      got += (size_t) n;
      if (n < STREAM_BLOCK)
        break;
      continue;
    }
    if (n == 0)
      closed = 1;
    else if (errno == EINTR)
      continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK)
      error = errno;
    break;
  }
  memset(buffer_end(&s->input), 0, RHP_PAD);
  if (got)
  {
    bool abort = false;
    s->abort = &abort;
    reactor_call(&s->user, STREAM_READ, 0);
    if (abort)
      return;
    s->abort = NULL;
  }
  if (closed)
    reactor_call(&s->user, STREAM_CLOSE, 0);
  else if (error)
    reactor_call(&s->user, STREAM_ERROR, (uint64_t) error);
}

static void stream_ready(reactor_event_t *event)
{
  stream_t *s = event->state;
  uint32_t ev = (uint32_t) event->data;
  if (ev & EPOLLOUT)
    stream_send(s);
  if (s->fd >= 0 && (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) && !(s->flags & STREAM_WRITE_ONLY))
    stream_receive(s);
}

void stream_construct(stream_t *s, reactor_callback_t *callback, void *state)
{
  *s = (stream_t) {.user = reactor_user_define(callback, state), .fd = -1};
  buffer_construct(&s->input);
  buffer_construct(&s->output);
}

void stream_destruct(stream_t *s)
{
  stream_close(s);
  if (s->abort)
    *s->abort = true;
  s->abort = NULL;
  buffer_destruct(&s->input);
  buffer_destruct(&s->output);
}

void stream_open(stream_t *s, int fd, int flags)
{
  s->fd = fd;
  s->flags = flags;
  int fl = fcntl(fd, F_GETFL);
  if (fl != -1)
    (void) fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  s->poll = reactor_poll(stream_ready, s, fd, flags & STREAM_WRITE_ONLY ? 0 : EPOLLIN);
}

int stream_fd(stream_t *s) { return s->fd; }
bool stream_is_open(stream_t *s) { return s->fd >= 0; }

void stream_close(stream_t *s)
{
  if (s->poll)
    reactor_poll_remove(s->poll);
  s->poll = 0;
  if (s->fd >= 0)
    close(s->fd);
  s->fd = -1;
}

data_t stream_read(stream_t *s) { return data_offset(buffer_data(&s->input), s->input_consumed); }
void stream_consume(stream_t *s, size_t n) { s->input_consumed += n; }
void *stream_allocate(stream_t *s, size_t n) { return data_base(buffer_allocate(&s->output, n)); }

void stream_write(stream_t *s, data_t d)
{
  if (data_size(d))
    memcpy(stream_allocate(s, data_size(d)), data_base(d), data_size(d));
}

void stream_flush(stream_t *s)
{
  s->output_flushed = buffer_size(&s->output);
  if (s->fd >= 0 && !s->output_wait)
    stream_send(s);
}
