/*
 * server_test.c -- end-to-end test of libreactor.so's HTTP server over
 * loopback: the server runs in the reactor loop of the main thread (its
 * sessions parsed in batches by the parser RHP_REACTOR_PARSER selects); a
 * client thread plays the cases of the reference's test/server.c:150-160 (same
 * requests, same callback behaviour: /abort, /next1, /next2, invalid input,
 * an immediate close) plus BASELINE config 1 (16 pipelined 128-byte GETs in one
 * write), request bodies (Content-Length and chunked) and a many-connection
 * pipelined load.
 * usage: server_test [connections] [requests-per-connection]; exit 0 = pass.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>

#include "reactor.h"

static int port, port2;
static int stop_pipe[2];
static atomic_long calls;
static int failures;

#define CHECK(cond, ...) do { if (!(cond)) { failures++; printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); fflush(stdout); } } while (0)

/* ---------------------------------------------------------------- server */

static void server_next1(reactor_event_t *event)
{
  server_respond((server_session_t *) event->state, string("200 OK"), string("text/plain"), string("ok"), NULL, 0);
}

static void server_next2(reactor_event_t *event)
{
  server_session_t *session = (server_session_t *) event->state;
  server_ok(session, string("text/plain"), string("ok"), NULL, 0);
  server_disconnect(session);
}

static void server_callback(reactor_event_t *event)
{
  server_session_t *session = (server_session_t *) event->data;
  atomic_fetch_add(&calls, 1);
  if (event->type != SERVER_REQUEST)
    return;
  if (string_equal(session->request.target, string("/abort")))
  {
    server_plain(session, string("no"), NULL, 0);
    server_disconnect(session);
  }
  else if (string_equal(session->request.target, string("/next1")))
    reactor_next(server_next1, session);
  else if (string_equal(session->request.target, string("/next2")))
    reactor_next(server_next2, session);
  else if (string_equal(session->request.target, string("/body")))
    server_plain(session, session->request.body, NULL, 0);   /* echo the request body */
  else if (string_equal(session->request.target, string("/len")))
  {
    /* the body's length and a checksum of its bytes (large bodies) */
    char text[64];
    const unsigned char *b = data_base(session->request.body);
    unsigned long sum = 0;
    for (size_t i = 0; i < data_size(session->request.body); i++)
      sum = sum * 31 + b[i];
    snprintf(text, sizeof text, "%zu %lu", data_size(session->request.body), sum);
    server_plain(session, string(text), NULL, 0);
  }
  else
    server_plain(session, string("ok"), NULL, 0);
}

static server_t server, server2;   /* two servers on one reactor thread share its batch slots */

static void stop_ready(reactor_event_t *event)
{
  reactor_poll_remove(*(reactor_t *) event->state);
  server_destruct(&server);
  server_destruct(&server2);
}

/* ---------------------------------------------------------------- client */

static int client_port(int p)
{
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001), .sin_port = htons(p)};
  int c = socket(AF_INET, SOCK_STREAM, 0);
  struct timeval tv = {.tv_sec = 10};
  (void) setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  (void) setsockopt(c, IPPROTO_TCP, TCP_NODELAY, (int[]) {1}, sizeof(int));
  if (connect(c, (struct sockaddr *) &sin, sizeof sin) != 0)
  {
    CHECK(0, "connect: %s", strerror(errno));
    close(c);
    return -1;
  }
  return c;
}

static int client(void) { return client_port(port); }

static void send_all(int c, const char *p, size_t n)
{
  while (n)
  {
    ssize_t k = send(c, p, n, MSG_NOSIGNAL);
    if (k <= 0)
      return;
    p += k;
    n -= (size_t) k;
  }
}

typedef struct reader
{
  char    buf[1 << 16];
  size_t  len;
  int     eof;
} reader_t;

/* one response: status code, body into `body` (NUL-terminated); 0 on EOF/timeout */
static int read_response(int c, reader_t *r, char *body, size_t cap)
{
  for (;;)
  {
    char *end = memmem(r->buf, r->len, "\r\n\r\n", 4);
    if (end)
    {
      size_t head = (size_t) (end - r->buf) + 4;
      char *cl = memmem(r->buf, head, "Content-Length: ", 16);
      size_t blen = cl ? strtoul(cl + 16, NULL, 10) : 0;
      if (r->len >= head + blen)
      {
        int code = strncmp(r->buf, "HTTP/1.1 ", 9) == 0 ? atoi(r->buf + 9) : -1;
        size_t k = blen < cap - 1 ? blen : cap - 1;
        memcpy(body, r->buf + head, k);
        body[k] = 0;
        memmove(r->buf, r->buf + head + blen, r->len - head - blen);
        r->len -= head + blen;
        return code;
      }
    }
    if (r->eof)
      return 0;
    ssize_t n = recv(c, r->buf + r->len, sizeof r->buf - r->len, 0);
    if (n <= 0)
    {
      r->eof = 1;
      if (r->len == 0)
        return 0;
    }
    else
      r->len += (size_t) n;
  }
}

static int at_eof(int c, reader_t *r)
{
  if (r->len)
    return 0;
  char x;
  ssize_t n = recv(c, &x, 1, 0);
  return n == 0;
}

/* one case: send `req` (`n` bytes, in writes of at most `piece` bytes, 0: one
 * write), expect `responses` 200s with body `want` (NULL: any), then EOF or not */
static void run_case_n(const char *name, const char *req, size_t n, size_t piece, int responses, const char *want,
                       int expect_eof)
{
  static reader_t r;
  char body[256];
  long before = atomic_load(&calls);
  int c = client();
  if (c < 0)
    return;
  r.len = 0;
  r.eof = 0;
  for (size_t at = 0; req && at < n;)
  {
    size_t k = piece && n - at > piece ? piece : n - at;
    send_all(c, req + at, k);
    at += k;
    if (piece)
      usleep(2000);
  }
  int got = 0;
  for (int i = 0; i < responses; i++)
  {
    int code = read_response(c, &r, body, sizeof body);
    if (code != 200)
      break;
    CHECK(!want || strcmp(body, want) == 0, "%s: body '%s', want '%s'", name, body, want);
    got++;
  }
  CHECK(got == responses, "%s: %d responses, want %d", name, got, responses);
  if (expect_eof)
    CHECK(at_eof(c, &r), "%s: connection left open", name);
  close(c);
  usleep(20000);
  printf("case %-22s responses %d  callbacks %ld\n", name, got, atomic_load(&calls) - before);
  fflush(stdout);
}

static void run_case(const char *name, const char *req, int responses, const char *want, int expect_eof)
{
  run_case_n(name, req, req ? strlen(req) : 0, 0, responses, want, expect_eof);
}

/* a POST /len request with an n-byte body of 'x' .. 'z' */
static char *big_post(size_t n, size_t *total, char *want, size_t want_cap)
{
  char head[128];
  int h = snprintf(head, sizeof head, "POST /len HTTP/1.1\r\nHost: x\r\nContent-Length: %zu\r\n\r\n", n);
  char *req = malloc((size_t) h + n + 1);
  memcpy(req, head, (size_t) h);
  unsigned long sum = 0;
  for (size_t i = 0; i < n; i++)
  {
    req[h + i] = (char) ('x' + i % 3);
    sum = sum * 31 + (unsigned char) req[h + i];
  }
  req[h + n] = 0;
  *total = (size_t) h + n;
  snprintf(want, want_cap, "%zu %lu", n, sum);
  return req;
}

/* inputs longer than 64 KiB (the reference parses any
 * length, http.c:177-234, buffer.c:56-64) */
static void long_cases(void)
{
  char want[64];
  size_t n;
  char *req = big_post(200000, &n, want, sizeof want);
  run_case_n("post 200 KB", req, n, 0, 1, want, 0);
  free(req);
  req = big_post(1u << 20, &n, want, sizeof want);
  run_case_n("post 1 MiB in 16 KiB", req, n, 16384, 1, want, 0);
  free(req);
  /* ~70 KiB of pipelined GETs in one write */
  const char get[] = "GET /plaintext HTTP/1.1\r\nHost: tfb\r\n\r\n";
  const size_t one = sizeof get - 1, count = 72000 / one;
  req = malloc(one * count + 1);
  for (size_t i = 0; i < count; i++)
    memcpy(req + one * i, get, one);
  req[one * count] = 0;
  run_case_n("pipelined 70 KiB GETs", req, one * count, 0, (int) count, "ok", 0);
  free(req);
  /* a header section longer than the batch records hold (RHP_RET_TOOLONG) */
  const char pre[] = "GET / HTTP/1.1\r\nX-Big: ";
  const size_t v = 70000;
  req = malloc(sizeof pre - 1 + v + 5);
  memcpy(req, pre, sizeof pre - 1);
  memset(req + sizeof pre - 1, 'v', v);
  memcpy(req + sizeof pre - 1 + v, "\r\n\r\n", 5);
  run_case_n("header section 70 KB", req, sizeof pre - 1 + v + 4, 0, 1, "ok", 0);
  free(req);
  /* the same header section on a POST whose Content-Length body has not all
   * arrived: the host parser answers 0 for it, and the session waits for bytes
   * (a bounded number of rounds, not one round after another: ADVICE r3) */
  {
    const char post[] = "POST /body HTTP/1.1\r\nContent-Length: 10\r\nX-Big: ";
    const size_t head = sizeof post - 1 + v + 4;
    req = malloc(head + 10 + 1);
    memcpy(req, post, sizeof post - 1);
    memset(req + sizeof post - 1, 'v', v);
    memcpy(req + sizeof post - 1 + v, "\r\n\r\n0123456789", 15);
    static reader_t r;
    char body[256];
    r.len = 0;
    r.eof = 0;
    int c = client();
    if (c >= 0)
    {
      send_all(c, req, head + 4);   /* 4 of the 10 body bytes */
      usleep(100000);
      const uint64_t r0 = reactor_batch_rounds();
      usleep(200000);
      const uint64_t idle = reactor_batch_rounds() - r0;
      CHECK(idle <= 2, "toolong post, partial body: %llu rounds while waiting for bytes", (unsigned long long) idle);
      send_all(c, req + head + 4, 6);
      const int code = read_response(c, &r, body, sizeof body);
      CHECK(code == 200 && strcmp(body, "0123456789") == 0, "toolong post: code %d body '%s'", code, body);
      close(c);
      usleep(20000);
      printf("case %-22s idle rounds %llu\n", "toolong post, partial", (unsigned long long) idle);
      fflush(stdout);
    }
    free(req);
  }
}

static const char tfb[] = "GET /plaintext HTTP/1.1\r\nHost: tfb-server:8080\r\nAccept: text/plain\r\n"
                          "Connection: keep-alive\r\nUser-Agent: wrk/4.2.0 (tfb-load)\r\n\r\n";

typedef struct load_arg
{
  int   requests;
  int   port;
  long  got;
} load_arg_t;

static void *load_client(void *p)
{
  load_arg_t *a = p;
  static __thread reader_t r;
  char body[64];
  int c = client_port(a->port);
  if (c < 0)
    return NULL;
  r.len = 0;
  r.eof = 0;
  size_t one = strlen(tfb);
  char *req = malloc(one * (size_t) a->requests);
  for (int i = 0; i < a->requests; i++)
    memcpy(req + one * (size_t) i, tfb, one);
  send_all(c, req, one * (size_t) a->requests);
  for (int i = 0; i < a->requests; i++)
    if (read_response(c, &r, body, sizeof body) == 200 && strcmp(body, "ok") == 0)
      a->got++;
  free(req);
  close(c);
  return NULL;
}

static int conns = 32, per_conn = 64;

static void *client_main(void *unused)
{
  (void) unused;
  /* the reference's cases (test/server.c:150-160) */
  run_case("get", "GET / HTTP/1.0\r\n\r\n", 1, "ok", 0);
  run_case("get+partial", "GET / HTTP/1.0\r\n\r\nGET", 1, "ok", 0);
  run_case("abort", "GET /abort HTTP/1.0\r\n\r\n", 0, NULL, 1);   /* closed before the reply is flushed, as the reference */
  run_case("next1", "GET /next1 HTTP/1.0\r\n\r\n", 1, "ok", 0);
  run_case("next2", "GET /next2 HTTP/1.0\r\n\r\n", 1, "ok", 1);
  run_case("next1 x2 pipelined", "GET /next1 HTTP/1.0\r\n\r\nGET /next1 HTTP/1.0\r\n\r\n", 2, "ok", 0);
  run_case("invalid", "i n v a l i d", 0, NULL, 1);
  run_case("connect+close", NULL, 0, NULL, 0);
  /* BASELINE config 1: 16 pipelined 128-byte GETs in one write */
  {
    char req[16 * 128 + 1];
    for (int i = 0; i < 16; i++)
      memcpy(req + 128 * i, tfb, 128);
    req[16 * 128] = 0;
    CHECK(strlen(tfb) == 128, "template is %zu bytes", strlen(tfb));
    run_case("config1 16 pipelined", req, 16, "ok", 0);
  }
  /* bodies: Content-Length, chunked (de-framed in place), a GET behind them */
  run_case("post content-length", "POST /body HTTP/1.1\r\nContent-Length: 5\r\n\r\nhelloGET / HTTP/1.1\r\n\r\n", 2, NULL, 0);
  run_case("post chunked", "POST /body HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n",
           1, "hello world", 0);
  run_case("lf line ends x2", "GET / HTTP/1.1\n\nGET / HTTP/1.1\n\n", 2, "ok", 0);
  long_cases();
  /* load: many connections, pipelined, on both servers at once (a server
   * turned away while the other's rounds hold every batch slot must be
   * re-armed by the next completion: ADVICE r2) */
  for (int phase = 0; phase < 2; phase++)
  {
    pthread_t t[256];
    load_arg_t a[256];
    int n = conns < 256 ? conns : 256;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < n; i++)
    {
      a[i] = (load_arg_t) {.requests = per_conn, .port = phase && (i & 1) ? port2 : port};
      pthread_create(&t[i], NULL, load_client, &a[i]);
    }
    long total = 0;
    for (int i = 0; i < n; i++)
    {
      pthread_join(t[i], NULL);
      total += a[i].got;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double s = (double) (t1.tv_sec - t0.tv_sec) + (double) (t1.tv_nsec - t0.tv_nsec) * 1e-9;
    CHECK(total == (long) n * per_conn, "load: %ld responses, want %ld", total, (long) n * per_conn);
    printf("load %d connections x %d pipelined%s: %ld responses in %.3f s (%.0f req/s)\n", n, per_conn,
           phase ? " (two servers)" : "", total, s, (double) total / s);
  }
  if (write(stop_pipe[1], "x", 1) != 1)
    abort();
  return NULL;
}

int main(int argc, char **argv)
{
  if (argc > 1)
    conns = atoi(argv[1]);
  if (argc > 2)
    per_conn = atoi(argv[2]);
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001)};
  socklen_t len = sizeof sin;
  int s = socket(AF_INET, SOCK_STREAM, 0);
  (void) setsockopt(s, SOL_SOCKET, SO_REUSEADDR, (int[]) {1}, sizeof(int));
  if (bind(s, (struct sockaddr *) &sin, sizeof sin) != 0 || listen(s, 4096) != 0 ||
      getsockname(s, (struct sockaddr *) &sin, &len) != 0)
    return 2;
  port = ntohs(sin.sin_port);
  struct sockaddr_in sin2 = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001)};
  int s2 = socket(AF_INET, SOCK_STREAM, 0);
  (void) setsockopt(s2, SOL_SOCKET, SO_REUSEADDR, (int[]) {1}, sizeof(int));
  len = sizeof sin2;
  if (bind(s2, (struct sockaddr *) &sin2, sizeof sin2) != 0 || listen(s2, 4096) != 0 ||
      getsockname(s2, (struct sockaddr *) &sin2, &len) != 0)
    return 2;
  port2 = ntohs(sin2.sin_port);
  if (pipe(stop_pipe) != 0)
    return 2;

  reactor_construct();
  server_construct(&server, server_callback, NULL);
  server_open_socket(&server, s);
  server_construct(&server2, server_callback, NULL);
  server_open_socket(&server2, s2);
  reactor_t stop = reactor_poll(stop_ready, &stop, stop_pipe[0], EPOLLIN);
  printf("parser: %s\n", reactor_parser_name());
  pthread_t t;
  pthread_create(&t, NULL, client_main, NULL);
  reactor_loop();
  pthread_join(t, NULL);
  reactor_destruct();
  close(s);
  close(s2);
  printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures != 0;
}
