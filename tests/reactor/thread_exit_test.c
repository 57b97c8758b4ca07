/*
 * thread_exit_test.c -- a reactor thread that serves with the batch parser and
 * then exits, three times over: the parser's per-thread state
 * (slots, events, the completion waiter or host worker thread) must be torn
 * down when its thread exits -- the waiter stopped and joined before the state
 * it uses is freed -- and a new thread must get a fresh one.  Runs with the
 * parser RHP_REACTOR_PARSER selects (gpu on the MI355X, host-async on CPU).
 * exit 0 = pass.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/epoll.h>
#include <sys/socket.h>

#include "reactor.h"

static int failures;
#define CHECK(cond, ...) do { if (!(cond)) { failures++; printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); fflush(stdout); } } while (0)

typedef struct run
{
  int       listen_fd, stop_pipe[2], port;
  server_t  server;
  reactor_t stop;
} run_t;

static void callback(reactor_event_t *event)
{
  if (event->type == SERVER_REQUEST)
    server_plain((server_session_t *) event->data, string("ok"), NULL, 0);
}

static void stop_ready(reactor_event_t *event)
{
  run_t *r = event->state;
  reactor_poll_remove(r->stop);
  server_destruct(&r->server);
}

static void *server_thread(void *arg)
{
  run_t *r = arg;
  reactor_construct();
  server_construct(&r->server, callback, NULL);
  server_open_socket(&r->server, r->listen_fd);
  r->stop = reactor_poll(stop_ready, r, r->stop_pipe[0], EPOLLIN);
  reactor_loop();
  reactor_destruct();
  return NULL;   /* the batch parser's thread-exit hook runs here */
}

/* 64 pipelined GETs on one connection, all answered "ok" */
static int client_round(int port)
{
  struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001), .sin_port = htons(port)};
  int c = socket(AF_INET, SOCK_STREAM, 0);
  struct timeval tv = {.tv_sec = 10};
  (void) setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  if (connect(c, (struct sockaddr *) &sin, sizeof sin) != 0)
  {
    close(c);
    return 0;
  }
  const char get[] = "GET / HTTP/1.1\r\nHost: x\r\n\r\n";
  char req[64 * sizeof get];
  for (int i = 0; i < 64; i++)
    memcpy(req + i * (sizeof get - 1), get, sizeof get - 1);
  const size_t n = 64 * (sizeof get - 1);
  if (send(c, req, n, MSG_NOSIGNAL) != (ssize_t) n)
  {
    close(c);
    return 0;
  }
  char buf[1 << 16];
  size_t len = 0;
  int oks = 0;
  while (oks < 64)
  {
    ssize_t k = recv(c, buf + len, sizeof buf - len - 1, 0);
    if (k <= 0)
      break;
    len += (size_t) k;
    buf[len] = 0;
    oks = 0;
    for (char *p = buf; (p = strstr(p, "\r\n\r\nok")); p += 6)
      oks++;
  }
  close(c);
  return oks;
}

int main(void)
{
  for (int it = 0; it < 3; it++)
  {
    run_t r = {0};
    struct sockaddr_in sin = {.sin_family = AF_INET, .sin_addr.s_addr = htonl(0x7f000001)};
    socklen_t len = sizeof sin;
    r.listen_fd = socket(AF_INET, SOCK_STREAM, 0);
    if (bind(r.listen_fd, (struct sockaddr *) &sin, sizeof sin) != 0 || listen(r.listen_fd, 64) != 0 ||
        getsockname(r.listen_fd, (struct sockaddr *) &sin, &len) != 0 || pipe(r.stop_pipe) != 0)
      return 2;
    r.port = ntohs(sin.sin_port);
    pthread_t t;
    if (pthread_create(&t, NULL, server_thread, &r) != 0)
      return 2;
    const int oks = client_round(r.port);
    CHECK(oks == 64, "thread %d: %d of 64 responses", it, oks);
    if (write(r.stop_pipe[1], "x", 1) != 1)
      return 2;
    pthread_join(t, NULL);
    close(r.listen_fd);
    close(r.stop_pipe[0]);
    close(r.stop_pipe[1]);
    printf("thread %d: %d responses, exited\n", it, oks);
    fflush(stdout);
  }
  usleep(100000);   /* a waiter left running on freed state would fault about now */
  printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures != 0;
}
