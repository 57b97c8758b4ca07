/*
 * echo_test.c -- what the server hands to SERVER_REQUEST, per request, for a
 * byte stream sent over one connection in chunks.  The handler answers each
 * request with a body that serializes the parsed request: method, target,
 * every field (name, value) and the body, each as a u32 length + bytes, and
 * the field count before the fields.  The client sends the input file in
 * chunks of <chunk> bytes (a pause after each, so rounds see partial input),
 * reads responses until the server closes or stays silent for 300 ms, and
 * writes everything it received to <out>.  tests/test_reactor.py compares the
 * decoded requests with the oracle's sequential http_read_request loop over
 * the same stream (reference server.c:37-65 + http.c:177-234).
 *
 * usage: echo_test <in> <chunk> <out>
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include "reactor.h"

static int port, stop_pipe[2];
static const char *in_path, *out_path;
static size_t chunk;
static volatile int done;

static uint8_t enc[1 << 22];
static size_t enc_n;

static void put(const void *p, size_t n)
{
  const uint32_t len = (uint32_t) n;
  if (enc_n + 4 + n > sizeof enc)
    abort();
  memcpy(enc + enc_n, &len, 4);
  memcpy(enc + enc_n + 4, p, n);
  enc_n += 4 + n;
}

static void server_callback(reactor_event_t *event)
{
  if (event->type != SERVER_REQUEST)
    return;
  server_session_t *s = (server_session_t *) event->data;
  http_request_t *r = &s->request;
  enc_n = 0;
  put(data_base(r->method), data_size(r->method));
  put(data_base(r->target), data_size(r->target));
  const uint32_t nf = (uint32_t) r->fields_count;
  put(&nf, 4);
  for (size_t i = 0; i < r->fields_count; i++)
  {
    put(data_base(r->fields[i].name), data_size(r->fields[i].name));
    put(data_base(r->fields[i].value), data_size(r->fields[i].value));
  }
  put(data_base(r->body), data_size(r->body));
  server_respond(s, string("200 OK"), string("application/octet-stream"), data(enc, enc_n), NULL, 0);
}

static void stop_ready(reactor_event_t *event)
{
  (void) event;
  char c;
  if (read(stop_pipe[0], &c, 1) != 1)
    abort();
}

static void *client(void *unused)
{
  (void) unused;
  FILE *f = fopen(in_path, "rb");
  if (!f)
    abort();
  fseek(f, 0, SEEK_END);
  const size_t n = (size_t) ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *in = malloc(n + 1);
  if (fread(in, 1, n, f) != n)
    abort();
  fclose(f);
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_port = htons((uint16_t) port),
                            .sin_addr.s_addr = htonl(0x7f000001)};
  int c = socket(AF_INET, SOCK_STREAM, 0);
  if (connect(c, (struct sockaddr *) &sin, sizeof sin) != 0)
    abort();
  size_t cap = 1 << 20, got = 0;
  uint8_t *out = malloc(cap);
  for (size_t at = 0; at < n;)
  {
    const size_t k = n - at < chunk ? n - at : chunk;
    if (write(c, in + at, k) != (ssize_t) k)
      break;   /* the server closed (a bad request) */
    at += k;
    usleep(500);
  }
  for (;;)
  {
    struct pollfd pfd = {.fd = c, .events = POLLIN};
    if (poll(&pfd, 1, 300) <= 0)
      break;
    if (got == cap)
      out = realloc(out, cap *= 2);
    const ssize_t r = read(c, out + got, cap - got);
    if (r <= 0)
      break;
    got += (size_t) r;
  }
  FILE *o = fopen(out_path, "wb");
  if (!o || fwrite(out, 1, got, o) != got)
    abort();
  fclose(o);
  free(in);
  free(out);
  close(c);
  done = 1;
  if (write(stop_pipe[1], "x", 1) != 1)
    abort();
  return NULL;
}

int main(int argc, char **argv)
{
  if (argc != 4)
    return 2;
  in_path = argv[1];
  chunk = (size_t) atol(argv[2]);
  out_path = argv[3];
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001)};
  socklen_t len = sizeof sin;
  int s = socket(AF_INET, SOCK_STREAM, 0);
  if (bind(s, (struct sockaddr *) &sin, sizeof sin) != 0 || listen(s, 16) != 0 ||
      getsockname(s, (struct sockaddr *) &sin, &len) != 0 || pipe(stop_pipe) != 0)
    return 2;
  port = ntohs(sin.sin_port);
  reactor_construct();
  server_t server;
  server_construct(&server, server_callback, NULL);
  server_open_socket(&server, s);
  reactor_t stop = reactor_poll(stop_ready, NULL, stop_pipe[0], EPOLLIN);
  printf("parser: %s\n", reactor_parser_name());
  pthread_t t;
  pthread_create(&t, NULL, client, NULL);
  while (!done)
    reactor_loop_once();
  pthread_join(t, NULL);
  reactor_poll_remove(stop);
  server_destruct(&server);
  reactor_destruct();
  close(s);
  printf("OK\n");
  return 0;
}
