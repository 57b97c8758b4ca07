/*
 * burst_test.c -- server throughput at a given round size.  C clients connect
 * and each sends P pipelined plaintext GETs (BASELINE config 1's 128-byte TFB
 * request) BEFORE the server's loop starts, so the first reactor rounds see
 * all C x P requests at once (round size = C x P unless the kernel splits
 * reads); the server answers every request "ok" and the clients count the
 * responses.  Reported: wall time from the loop's start to the last response
 * and requests per second, per repetition (a fresh server each time).
 *
 * usage: burst_test [conns=64] [pipelined=64] [repetitions=5]
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "reactor.h"

static const char tfb[] = "GET /plaintext HTTP/1.1\r\nHost: tfb-server:8080\r\nAccept: text/plain\r\n"
                          "Connection: keep-alive\r\nUser-Agent: wrk/4.2.0 (tfb-load)\r\n\r\n";

static int port, conns = 64, per_conn = 64;
static int stop_pipe[2];
static atomic_int ready, done;
static atomic_long answered;

static void server_callback(reactor_event_t *event)
{
  if (event->type == SERVER_REQUEST)
    server_plain((server_session_t *) event->data, data_string("ok"), NULL, 0);
}

/* wakes the loop once the last client is done (the loop re-checks `done`) */
static void stop_ready(reactor_event_t *event)
{
  (void) event;
  char c;
  if (read(stop_pipe[0], &c, 1) != 1)
    abort();
}

static int count_responses(const char *p, size_t n)
{
  int k = 0;
  for (const char *q = p; (q = memmem(q, (size_t) (p + n - q), "\r\n\r\nok", 6)); q += 6)
    k++;
  return k;
}

static void *client(void *unused)
{
  (void) unused;
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_port = htons((uint16_t) port),
                            .sin_addr.s_addr = htonl(0x7f000001)};
  int c = socket(AF_INET, SOCK_STREAM, 0);
  if (connect(c, (struct sockaddr *) &sin, sizeof sin) != 0)
    abort();
  const size_t one = strlen(tfb);
  char *req = malloc(one * (size_t) per_conn);
  for (int i = 0; i < per_conn; i++)
    memcpy(req + one * (size_t) i, tfb, one);
  for (size_t at = 0; at < one * (size_t) per_conn;)
  {
    ssize_t w = write(c, req + at, one * (size_t) per_conn - at);
    if (w <= 0)
      abort();
    at += (size_t) w;
  }
  free(req);
  atomic_fetch_add(&ready, 1);
  /* every response ends in "\r\n\r\nok": read until all are in */
  size_t cap = 256 * (size_t) per_conn + 4096, n = 0;
  char *buf = malloc(cap);
  int got = 0;
  while (got < per_conn)
  {
    if (n == cap)
      buf = realloc(buf, cap *= 2);
    ssize_t r = read(c, buf + n, cap - n);
    if (r <= 0)
      break;
    n += (size_t) r;
    got = count_responses(buf, n);
  }
  free(buf);
  atomic_fetch_add(&answered, got);
  close(c);
  if (atomic_fetch_add(&done, 1) + 1 == conns)
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
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  reactor_construct();
  printf("parser: %s, %d connections x %d pipelined per burst\n", reactor_parser_name(), conns, per_conn);
  int failures = 0;
  for (int rep = 0; rep < reps; rep++)
  {
    struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001)};
    socklen_t len = sizeof sin;
    int s = socket(AF_INET, SOCK_STREAM, 0);
    (void) setsockopt(s, SOL_SOCKET, SO_REUSEADDR, (int[]) {1}, sizeof(int));
    if (bind(s, (struct sockaddr *) &sin, sizeof sin) != 0 || listen(s, 4096) != 0 ||
        getsockname(s, (struct sockaddr *) &sin, &len) != 0 || pipe(stop_pipe) != 0)
      return 2;
    port = ntohs(sin.sin_port);
    atomic_store(&ready, 0);
    atomic_store(&done, 0);
    atomic_store(&answered, 0);
    pthread_t *t = calloc((size_t) conns, sizeof *t);
    for (int i = 0; i < conns; i++)
      pthread_create(&t[i], NULL, client, NULL);
    while (atomic_load(&ready) < conns)
      usleep(100);
    usleep(2000);   /* let the last bytes land in the socket buffers */

    server_t server;
    server_construct(&server, server_callback, NULL);
    server_open_socket(&server, s);
    reactor_t stop = reactor_poll(stop_ready, NULL, stop_pipe[0], EPOLLIN);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    while (atomic_load(&done) < conns)
      reactor_loop_once();
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int i = 0; i < conns; i++)
      pthread_join(t[i], NULL);
    free(t);
    reactor_poll_remove(stop);
    server_destruct(&server);
    close(s);
    close(stop_pipe[0]);
    close(stop_pipe[1]);
    const double sec = (double) (t1.tv_sec - t0.tv_sec) + (double) (t1.tv_nsec - t0.tv_nsec) * 1e-9;
    const long want = (long) conns * per_conn, got = atomic_load(&answered);
    if (got != want)
      failures++;
    printf("burst %d: %ld/%ld responses in %.3f ms (%.0f req/s)\n", rep, got, want, sec * 1e3, (double) got / sec);
    fflush(stdout);
  }
  reactor_destruct();
  printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures != 0;
}
