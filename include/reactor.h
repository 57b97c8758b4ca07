/*
 * reactor.h -- the libreactor surface of the HTTP receive path, host C, with
 * the request parse on the MI355X batch parser (include/rhp.h).
 *
 * Declares the part of the reference's public API (src/reactor.h:23-46) that
 * the HTTP server, its callers and its request parse use, so that the
 * reference's example/server.c compiles and links unchanged against
 * libreactorng_amd/libreactor.so:
 *
 *   data / string   src/reactor/data.h:10-41, src/reactor/string.h:7-29
 *   buffer          src/reactor/buffer.h
 *   reactor         src/reactor/reactor.h:14-52 (an epoll loop here; io_uring there)
 *   timeout         src/reactor/timeout.h
 *   network         src/reactor/network.h:10-21 (the accept side)
 *   stream          src/reactor/stream.h:7-52
 *   http            src/reactor/http.h:4-37
 *   server          src/reactor/server.h:4-45
 *
 * Server sessions parse their input through rhp_parse_batch: once per reactor
 * round, every session that received bytes is parsed in ONE batch launch and
 * SERVER_REQUEST is then dispatched per request in order (SURVEY.md §8f rows 1
 * and 2).  The types are this library's own (only the API and
 * the callback semantics follow the reference), so code that stack-allocates
 * server_t, as example/server.c:10 does, compiles against this header.
 */
#ifndef REACTOR_H_INCLUDED
#define REACTOR_H_INCLUDED

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>
#include <sys/uio.h>

#define REACTOR_VERSION       "0.9.2-rhp"
#define REACTOR_VERSION_MAJOR 0
#define REACTOR_VERSION_MINOR 9
#define REACTOR_VERSION_PATCH 2

#define reactor_likely(x)   __builtin_expect(!!(x), 1)
#define reactor_unlikely(x) __builtin_expect(!!(x), 0)

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- data */

typedef struct data data_t;
struct data
{
  struct iovec iov;
};

data_t   data(const void *, size_t);
data_t   data_null(void);
data_t   data_string(const char *);
data_t   data_offset(const data_t, size_t);
data_t   data_select(const data_t, size_t);
size_t   data_size(const data_t);
bool     data_empty(const data_t);
void    *data_base(const data_t);
void    *data_end(const data_t);
bool     data_equal(const data_t, const data_t);
bool     data_equal_case(const data_t, const data_t);

typedef data_t string_t;

string_t string(const char *);
string_t string_data(const data_t);
string_t string_null(void);
size_t   string_size(const string_t);
bool     string_empty(const string_t);
char    *string_base(const string_t);
bool     string_equal(const string_t, const string_t);
bool     string_equal_case(const string_t, const string_t);

/* -------------------------------------------------------------- buffer */

typedef struct buffer buffer_t;
struct buffer
{
  data_t  data;
  size_t  capacity;
};

void    buffer_construct(buffer_t *);
void    buffer_destruct(buffer_t *);
data_t  buffer_data(const buffer_t *);
size_t  buffer_size(const buffer_t *);
size_t  buffer_capacity(const buffer_t *);
void   *buffer_base(const buffer_t *);
void   *buffer_end(const buffer_t *);
void    buffer_reserve(buffer_t *, size_t);
void    buffer_resize(buffer_t *, size_t);
void    buffer_append(buffer_t *, data_t);
void    buffer_erase(buffer_t *, size_t, size_t);
data_t  buffer_allocate(buffer_t *, size_t);
void    buffer_clear(buffer_t *);

/* ---------------------------------------------------------------- list */

typedef struct list list_t;
struct list
{
  list_t *next;
  list_t *prev;
};

/* ------------------------------------------------------------- reactor */

enum
{
  REACTOR_CALL,
  REACTOR_RETURN
};

typedef struct reactor_event reactor_event_t;
typedef struct reactor_user  reactor_user_t;
typedef uint64_t             reactor_time_t;
typedef uint64_t             reactor_t;
typedef void                (reactor_callback_t)(reactor_event_t *);

struct reactor_event
{
  void     *state;
  int       type;
  uint64_t  data;
};

struct reactor_user
{
  reactor_callback_t *callback;
  void               *state;
};

reactor_event_t reactor_event_define(void *, int, uint64_t);
reactor_user_t  reactor_user_define(reactor_callback_t *, void *);
void            reactor_user_construct(reactor_user_t *, reactor_callback_t *, void *);

void            reactor_construct(void);
void            reactor_destruct(void);
reactor_time_t  reactor_now(void);
void            reactor_loop(void);
void            reactor_loop_once(void);
void            reactor_call(reactor_user_t *, int, uint64_t);
void            reactor_cancel(reactor_t, reactor_callback_t *, void *);
reactor_t       reactor_next(reactor_callback_t *, void *);

/* fd readiness, this library's loop primitive (the reference submits io_uring
 * operations instead); the callback receives the epoll event bits as data */
reactor_t       reactor_poll(reactor_callback_t *, void *, int, uint32_t);
void            reactor_poll_update(reactor_t, uint32_t);
void            reactor_poll_remove(reactor_t);

/* ------------------------------------------------------------- timeout */

enum
{
  TIMEOUT_ERROR,
  TIMEOUT_EXPIRE
};

typedef struct timeout timeout_t;
struct timeout
{
  reactor_user_t  user;
  int             fd;
  reactor_t       poll;
};

void timeout_construct(timeout_t *, reactor_callback_t *, void *);
void timeout_destruct(timeout_t *);
void timeout_set(timeout_t *, reactor_time_t, reactor_time_t);
void timeout_clear(timeout_t *);

/* ------------------------------------------------------------- network */

enum
{
  NETWORK_ERROR,
  NETWORK_ACCEPT,
  NETWORK_ACCEPT_BIND
};

enum
{
  NETWORK_REUSEADDR = 0x01,
  NETWORK_REUSEPORT = 0x02
};

typedef uint64_t network_t;

network_t network_accept(reactor_callback_t *, void *, const char *, int, int);
network_t network_accept_socket(reactor_callback_t *, void *, int);
void      network_cancel(network_t);

/* -------------------------------------------------------------- stream */

enum
{
  STREAM_ERROR,
  STREAM_READ,
  STREAM_CLOSE
};

enum
{
  STREAM_WRITE_ONLY = 0x01
};

typedef struct stream stream_t;
struct stream
{
  reactor_user_t  user;
  int             fd;
  int             flags;
  bool           *abort;
  reactor_t       poll;
  buffer_t        input;
  size_t          input_consumed;
  buffer_t        output;
  size_t          output_flushed;
  size_t          output_sent;
  bool            output_wait;
};

void    stream_construct(stream_t *, reactor_callback_t *, void *);
void    stream_destruct(stream_t *);
void    stream_open(stream_t *, int, int);
int     stream_fd(stream_t *);
bool    stream_is_open(stream_t *);
void    stream_close(stream_t *);
data_t  stream_read(stream_t *);
void    stream_consume(stream_t *, size_t);
void   *stream_allocate(stream_t *, size_t);
void    stream_write(stream_t *, data_t);
void    stream_flush(stream_t *);

/* ---------------------------------------------------------------- http */

typedef struct http_field   http_field_t;
typedef struct http_request http_request_t;

struct http_field
{
  string_t  name;
  string_t  value;
};

struct http_request
{
  string_t      method;
  string_t      target;
  data_t        body;
  http_field_t  fields[16];
  size_t        fields_count;
};

http_field_t http_field_define(string_t, string_t);
string_t     http_field_lookup(http_field_t *, size_t, string_t);
int          http_read_request(stream_t *, string_t *, string_t *, data_t *, http_field_t *, size_t *);
void         http_write_response(stream_t *, string_t, string_t, string_t, data_t, http_field_t *, size_t);

/* -------------------------------------------------------------- server */

enum
{
  SERVER_ERROR,
  SERVER_REQUEST
};

enum
{
  SERVER_SESSION_READY      = 0x01,
  SERVER_SESSION_PROCESSING = 0x02
};

typedef struct server         server_t;
typedef struct server_session server_session_t;

struct server
{
  reactor_user_t  user;
  network_t       accept;
  timeout_t       timeout;
  list_t          sessions;   /* every session of this server */
  list_t          queue;      /* sessions waiting for the next parse batch */
  reactor_t       batch;      /* the scheduled batch round, or 0 */
};

struct server_session
{
  reactor_user_t  user;
  http_request_t  request;
  stream_t        stream;
  int             flags;
  bool           *abort;
  reactor_t       next;
  /* this library */
  server_t       *server;
  list_t          link;       /* in server->sessions */
  list_t          queued;     /* in server->queue (self-linked when not queued) */
  bool            exact;      /* unused (kept for the struct's layout) */
  bool            in_round;   /* taking part in the running batch round */
  bool            dead;       /* freed while in a round (the round releases it) */
};

void server_construct(server_t *, reactor_callback_t *, void *);
void server_destruct(server_t *);
void server_open(server_t *, const char *, int);
void server_open_socket(server_t *, int);
void server_close(server_t *);
void server_disconnect(server_session_t *);
void server_respond(server_session_t *, string_t, string_t, data_t, http_field_t *, size_t);
void server_ok(server_session_t *, string_t, data_t, http_field_t *, size_t);
void server_plain(server_session_t *, data_t, http_field_t *, size_t);

/* ------------------------------------------------- batch parser binding */

/* Which parser server sessions use (read once, from RHP_REACTOR_PARSER):
 * "gpu" (default) = rhp_parse_batch on the MI355X, failing loudly when no GPU
 * or librhp.so is usable; "host" = the product's exact scalar parser
 * (rhp_scalar.h) on the host, for CPU-only hosts and tests. */
const char *reactor_parser_name(void);

/* Diagnostic: batch rounds submitted with input so far (all servers of the
 * process; tests bound the rounds a waiting session may cost). */
uint64_t reactor_batch_rounds(void);

#ifdef __cplusplus
}
#endif

#endif /* REACTOR_H_INCLUDED */
