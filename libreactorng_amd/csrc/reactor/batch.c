/*
 * batch.c -- the session parser behind the server: one rhp_parse_batch call
 * (include/rhp.h) over the packed unconsumed input of every session that has
 * bytes to parse in a reactor round.
 *
 * "gpu" (default): pinned host staging -> hipMemcpyAsync H2D -> the MI355X
 * kernel -> D2H of the records, on one HIP stream of this thread.  The parser
 * is the product path: when RHP_REACTOR_PARSER is unset or "gpu" and no GPU or
 * librhp.so is usable, the process stops with an error (no silent fallback).
 * "host": the product's exact scalar parser (rhp_cpu_parse_batch) in place,
 * selected explicitly for CPU-only hosts and the CPU test suite.
 */
#define __HIP_PLATFORM_AMD__ 1
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <hip/hip_runtime_api.h>

#include "reactor.h"
#include "reactor_batch.h"
#include "rhp.h"
#include "rhp_host.h"

enum { PARSER_UNSET, PARSER_GPU, PARSER_HOST };

static __thread struct
{
  int          parser;
  size_t       cap_bytes, cap_n, cap_h;
  uint8_t     *h_bytes;      /* pinned (gpu) or malloc'd (host) staging */
  uint64_t    *h_off;
  rhp_req_t   *h_req;
  rhp_hdr_t   *h_hdr;
  rhp_http_t  *h_http;
  void        *d_bytes, *d_off, *d_req, *d_hdr, *d_http, *d_work;
  hipStream_t  stream;
  /* RHP_REACTOR_STATS=1: rounds, requests and time spent in the parser, printed at exit */
  int          stats;
  int          diag_host;   /* RHP_REACTOR_DIAG=hostparse: gpu-mode buffers, host parse (diagnostic) */
  uint64_t     st_rounds, st_requests, st_ns;
} B;

static uint64_t now_ns(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t) ts.tv_sec * 1000000000u + (uint64_t) ts.tv_nsec;
}

static void print_stats(void)
{
  fprintf(stderr, "reactor parser %s: %llu rounds, %llu requests (%.1f per round), %.1f us per round\n",
          B.parser == PARSER_GPU ? "gpu" : "host", (unsigned long long) B.st_rounds, (unsigned long long) B.st_requests,
          B.st_rounds ? (double) B.st_requests / (double) B.st_rounds : 0.0,
          B.st_rounds ? (double) B.st_ns / 1e3 / (double) B.st_rounds : 0.0);
}

static void die(const char *what, int e)
{
  fprintf(stderr, "reactor: GPU request parser unavailable (%s: %d); set RHP_REACTOR_PARSER=host to parse on the host\n",
          what, e);
  abort();
}

#define HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) die(#x, (int) e_); } while (0)

static int parser(void)
{
  if (B.parser == PARSER_UNSET)
  {
    const char *e = getenv("RHP_REACTOR_PARSER");
    B.parser = e && strcmp(e, "host") == 0 ? PARSER_HOST : PARSER_GPU;
    const char *st = getenv("RHP_REACTOR_STATS");
    if ((B.stats = st && *st == '1'))
      atexit(print_stats);
    const char *dg = getenv("RHP_REACTOR_DIAG");
    B.diag_host = dg && strcmp(dg, "hostparse") == 0;
    if (B.parser == PARSER_GPU)
    {
      int n = 0;
      HIP(hipGetDeviceCount(&n));
      if (n < 1)
        die("hipGetDeviceCount", 0);
      HIP(hipStreamCreateWithFlags(&B.stream, hipStreamNonBlocking));
    }
  }
  return B.parser;
}

const char *reactor_parser_name(void)
{
  return parser() == PARSER_GPU ? "gpu" : "host";
}

static void *host_alloc(size_t n)
{
  void *p = NULL;
  if (B.parser == PARSER_GPU)
    HIP(hipHostMalloc(&p, n, hipHostMallocDefault));
  else if (!(p = malloc(n)))
    abort();
  return p;
}

static void host_free(void *p)
{
  if (!p)
    return;
  if (B.parser == PARSER_GPU)
    (void) hipHostFree(p);
  else
    free(p);
}

static void dev_free(void **p)
{
  if (*p)
    (void) hipFree(*p);
  *p = NULL;
}

uint8_t *reactor_batch_reserve(size_t bytes, uint32_t n)
{
  (void) parser();
  const uint64_t t0 = B.stats ? now_ns() : 0;
  const size_t need = bytes + RHP_PAD;
  if (need > B.cap_bytes)
  {
    /* generous first capacities: growing pinned and device buffers costs
     * milliseconds per step (page pinning, frees that synchronise) */
    size_t c = B.cap_bytes ? B.cap_bytes : 1u << 20;
    while (c < need)
      c *= 2;
    host_free(B.h_bytes);
    B.h_bytes = host_alloc(c);
    if (B.parser == PARSER_GPU)
    {
      dev_free(&B.d_bytes);
      HIP(hipMalloc(&B.d_bytes, c));
    }
    B.cap_bytes = c;
  }
  if (n + 1 > B.cap_n)
  {
    size_t c = B.cap_n ? B.cap_n : 4096;
    while (c < n + 1u)
      c *= 2;
    host_free(B.h_off);
    host_free(B.h_req);
    host_free(B.h_hdr);
    host_free(B.h_http);
    B.h_off = host_alloc(c * sizeof *B.h_off);
    B.h_req = host_alloc(c * sizeof *B.h_req);
    B.h_hdr = host_alloc(c * REACTOR_BATCH_HEADERS * sizeof *B.h_hdr);
    B.h_http = host_alloc(c * sizeof *B.h_http);
    if (B.parser == PARSER_GPU)
    {
      dev_free(&B.d_off);
      dev_free(&B.d_req);
      dev_free(&B.d_hdr);
      dev_free(&B.d_http);
      HIP(hipMalloc(&B.d_off, c * sizeof *B.h_off));
      HIP(hipMalloc(&B.d_req, c * sizeof *B.h_req));
      HIP(hipMalloc(&B.d_hdr, c * REACTOR_BATCH_HEADERS * sizeof *B.h_hdr));
      HIP(hipMalloc(&B.d_http, c * sizeof *B.h_http));
      if (!B.d_work)
      {
        HIP(hipMalloc(&B.d_work, RHP_WORK_WORDS * sizeof(uint32_t)));
        HIP(hipMemsetAsync(B.d_work, 0, RHP_WORK_WORDS * sizeof(uint32_t), B.stream));
      }
    }
    B.cap_n = c;
  }
  if (B.stats)
    B.st_ns += now_ns() - t0;
  return B.h_bytes;
}

uint64_t *reactor_batch_offsets(void)
{
  return B.h_off;
}

int reactor_batch_run(uint32_t n, size_t bytes, reactor_batch_result_t *out)
{
  const uint64_t t0 = B.stats ? now_ns() : 0;
  memset(B.h_bytes + bytes, 0, RHP_PAD);
  B.h_off[n] = bytes;
  if (B.parser == PARSER_HOST || B.diag_host)
  {
    rhp_batch_t b = {
      .bytes = B.h_bytes, .bytes_rw = B.h_bytes, .offsets = B.h_off, .bytes_size = bytes + RHP_PAD, .n = n,
      .max_headers = REACTOR_BATCH_HEADERS, .mode = RHP_MODE_HTTP, .reqs = B.h_req, .hdrs = B.h_hdr, .http = B.h_http};
    (void) rhp_cpu_parse_batch(&b);
  }
  else
  {
    HIP(hipMemcpyAsync(B.d_bytes, B.h_bytes, bytes + RHP_PAD, hipMemcpyHostToDevice, B.stream));
    HIP(hipMemcpyAsync(B.d_off, B.h_off, (n + 1) * sizeof *B.h_off, hipMemcpyHostToDevice, B.stream));
    rhp_batch_t b = {
      .bytes = B.d_bytes, .bytes_rw = B.d_bytes, .offsets = B.d_off, .bytes_size = bytes + RHP_PAD, .n = n,
      .max_headers = REACTOR_BATCH_HEADERS, .mode = RHP_MODE_HTTP, .reqs = B.d_req, .hdrs = B.d_hdr, .http = B.d_http,
      .work = B.d_work};
    int rc = rhp_parse_batch(&b, B.stream);
    if (rc != 0)
      die("rhp_parse_batch", rc);
    HIP(hipMemcpyAsync(B.h_req, B.d_req, n * sizeof *B.h_req, hipMemcpyDeviceToHost, B.stream));
    HIP(hipMemcpyAsync(B.h_hdr, B.d_hdr, (size_t) n * REACTOR_BATCH_HEADERS * sizeof *B.h_hdr, hipMemcpyDeviceToHost,
                       B.stream));
    HIP(hipMemcpyAsync(B.h_http, B.d_http, n * sizeof *B.h_http, hipMemcpyDeviceToHost, B.stream));
    HIP(hipStreamSynchronize(B.stream));
    /* chunked bodies were de-framed in place in device memory (http.c:155):
     * bring those bytes back so the caller sees the rewritten input */
    for (uint32_t i = 0; i < n; i++)
    {
      const rhp_http_t *x = &B.h_http[i];
      if (x->result == 1 && x->body_kind && x->consumed != (uint64_t) B.h_req[i].ret + x->body_len)
        HIP(hipMemcpy(B.h_bytes + B.h_off[i], (uint8_t *) B.d_bytes + B.h_off[i], x->consumed,
                      hipMemcpyDeviceToHost));
    }
  }
  if (B.stats)
  {
    B.st_rounds++;
    B.st_requests += n;
    B.st_ns += now_ns() - t0;
  }
  out->bytes = B.h_bytes;
  out->reqs = B.h_req;
  out->hdrs = B.h_hdr;
  out->n = n;
  out->http = B.h_http;
  return 0;
}
