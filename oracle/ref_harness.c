/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives the REAL reference (compiled from /root/reference by oracle/Makefile into
 * oracle/_ref/libref.so, never committed) over a packed batch and emits the
 * canonical records of oracle/rhp_oracle.h.  Used to pin the restatement
 * (oracle/diff_fuzz.c) and to generate tests/golden/ fixtures.
 *
 *   phr_parse_request  src/picohttpparser/picohttpparser.c:383-409
 *   http_read_request  src/reactor/http.c:177-234 (driven like test/http.c:121-141,
 *                      but with the stream's input pointing into the batch so the
 *                      bytes after each request are the batch's own bytes)
 */
#include <string.h>
#include <reactor.h>
#include "picohttpparser/picohttpparser.h"
#include "rhp_oracle.h"

static void ref_canon(orc_req_t *r, orc_hdr_t *h, uint32_t max_headers)
{
  int32_t ret = r->ret;
  memset(r, 0, sizeof *r);
  r->ret = ret;
  memset(h, 0, sizeof *h * max_headers);
}

static int ref_phr_one_last(const uint8_t *buf, size_t len, orc_req_t *req, orc_hdr_t *hdrs,
                            uint32_t max_headers, struct phr_header *tmp, size_t last_len)
{
  const char *method, *path;
  size_t method_len, path_len, num = max_headers;
  int minor;
  int r = phr_parse_request((const char *) buf, len, &method, &method_len, &path, &path_len, &minor,
                            tmp, &num, last_len);
  memset(req, 0, sizeof *req);
  req->ret = r;
  if (r > 0) {
    req->minor_version = minor;
    req->num_headers = (uint32_t) num;
    req->method_off = method - (const char *) buf;
    req->method_len = (int64_t) method_len;
    req->path_off = path - (const char *) buf;
    req->path_len = (int64_t) path_len;
    for (size_t i = 0; i < num; i++) {
      hdrs[i].name_off = tmp[i].name ? tmp[i].name - (const char *) buf : -1;
      hdrs[i].name_len = (int64_t) tmp[i].name_len;
      hdrs[i].value_off = tmp[i].value - (const char *) buf;
      hdrs[i].value_len = (int64_t) tmp[i].value_len;
    }
  }
  return r;
}

static int ref_phr_one(const uint8_t *buf, size_t len, orc_req_t *req, orc_hdr_t *hdrs,
                       uint32_t max_headers, struct phr_header *tmp)
{
  return ref_phr_one_last(buf, len, req, hdrs, max_headers, tmp, 0);
}

/* phr_parse_request with a per-request last_len (is_complete runs first when it
 * is not 0, picohttpparser.c:197-223, 399-401) */
void ref_phr_batch_last(const uint8_t *bytes, const uint64_t *offsets, const uint64_t *last_len, uint32_t n,
                        uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs)
{
  struct phr_header tmp[256];
  if (max_headers > 256)
    max_headers = 256;
  for (uint32_t i = 0; i < n; i++) {
    orc_hdr_t *h = hdrs + (size_t) i * max_headers;
    memset(h, 0, sizeof *h * max_headers);
    int r = ref_phr_one_last(bytes + offsets[i], offsets[i + 1] - offsets[i], &reqs[i], h, max_headers, tmp,
                             last_len[i]);
    if (r <= 0)
      ref_canon(&reqs[i], h, max_headers);
  }
}

void ref_phr_batch(const uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                   uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs)
{
  struct phr_header tmp[256];
  if (max_headers > 256)
    max_headers = 256;
  for (uint32_t i = 0; i < n; i++) {
    orc_hdr_t *h = hdrs + (size_t) i * max_headers;
    memset(h, 0, sizeof *h * max_headers);
    int r = ref_phr_one(bytes + offsets[i], offsets[i + 1] - offsets[i], &reqs[i], h, max_headers, tmp);
    if (r <= 0)
      ref_canon(&reqs[i], h, max_headers);
  }
}

void ref_http_batch(uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                    uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs,
                    orc_http_t *https)
{
  struct phr_header tmp[256];
  http_field_t fields[256];
  if (max_headers > 256)
    max_headers = 256;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t *buf = bytes + offsets[i];
    size_t len = offsets[i + 1] - offsets[i];
    orc_hdr_t *h = hdrs + (size_t) i * max_headers;
    memset(h, 0, sizeof *h * max_headers);
    memset(&https[i], 0, sizeof https[i]);

    /* minor_version is local to http_read_request; take it from phr on the
     * untouched bytes (http.c:188-192 calls phr with the same arguments) */
    orc_req_t pre;
    ref_phr_one(buf, len, &pre, h, max_headers, tmp);
    memset(h, 0, sizeof *h * max_headers);

    stream_t s;
    memset(&s, 0, sizeof s);
    s.fd = -1;
    s.input.data = data(buf, len);
    s.input.capacity = len;
    s.input_consumed = 0;
    string_t method = string_null(), target = string_null();
    data_t body = data_null();
    size_t count = max_headers;
    int r = http_read_request(&s, &method, &target, &body, fields, &count);

    orc_req_t *req = &reqs[i];
    memset(req, 0, sizeof *req);
    https[i].result = r;
    if (r == 1) {
      req->ret = pre.ret;
      req->minor_version = pre.minor_version;
      req->num_headers = (uint32_t) count;
      req->method_off = (const uint8_t *) data_base(method) - buf;
      req->method_len = (int64_t) data_size(method);
      req->path_off = (const uint8_t *) data_base(target) - buf;
      req->path_len = (int64_t) data_size(target);
      for (size_t k = 0; k < count; k++) {
        h[k].name_off = data_base(fields[k].name) ? (const uint8_t *) data_base(fields[k].name) - buf : -1;
        h[k].name_len = (int64_t) data_size(fields[k].name);
        h[k].value_off = (const uint8_t *) data_base(fields[k].value) - buf;
        h[k].value_len = (int64_t) data_size(fields[k].value);
      }
      https[i].consumed = (uint64_t) s.input_consumed;
      if (data_base(body)) {
        https[i].body_kind = 1;
        https[i].body_off = (const uint8_t *) data_base(body) - buf;
        https[i].body_len = (uint64_t) data_size(body);
      }
    } else {
      req->ret = pre.ret;
      ref_canon(req, h, max_headers);
    }
  }
}

/* ---- CPU baseline: the reference parser itself, timed on the host cores ----
 * Each thread runs phr_parse_request (the reference's own -O3 build flags, see
 * oracle/Makefile) over its contiguous share of the batch, reps times, exactly
 * as libreactor's http_read_request calls it; returns elapsed ns. */
#include <pthread.h>
#include <time.h>

struct ref_mt_arg {
  const uint8_t *bytes;
  const uint64_t *offsets;
  uint32_t lo, hi, max_headers;
  int reps;
  long sum;
};

static void *ref_mt_worker(void *p)
{
  struct ref_mt_arg *a = p;
  struct phr_header tmp[256];
  long sum = 0;
  for (int rep = 0; rep < a->reps; rep++)
    for (uint32_t i = a->lo; i < a->hi; i++) {
      const char *method, *path;
      size_t method_len, path_len, num = a->max_headers;
      int minor;
      sum += phr_parse_request((const char *) a->bytes + a->offsets[i], a->offsets[i + 1] - a->offsets[i],
                               &method, &method_len, &path, &path_len, &minor, tmp, &num, 0);
    }
  a->sum = sum;
  return NULL;
}

uint64_t ref_phr_batch_mt(const uint8_t *bytes, const uint64_t *offsets, uint32_t n, uint32_t max_headers,
                          int threads, int reps, long *checksum)
{
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if (max_headers > 256) max_headers = 256;
  pthread_t tid[256];
  struct ref_mt_arg args[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    args[t] = (struct ref_mt_arg) {bytes, offsets, (uint32_t) ((uint64_t) n * t / threads),
                                   (uint32_t) ((uint64_t) n * (t + 1) / threads), max_headers, reps, 0};
    pthread_create(&tid[t], NULL, ref_mt_worker, &args[t]);
  }
  long sum = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tid[t], NULL);
    sum += args[t].sum;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (checksum) *checksum = sum;
  return (uint64_t) (t1.tv_sec - t0.tv_sec) * 1000000000ull + (uint64_t) (t1.tv_nsec - t0.tv_nsec);
}

/*
 * The REAL http_write_response (src/reactor/http.c:286-297) over a batch laid
 * out as orc_write_responses' arguments: one stream, output_waiting drained
 * after every response (as test/http.c:143-181 drives it).
 */
uint64_t ref_write_responses(const uint8_t *arena, const uint32_t *resps, const uint32_t *fields, uint32_t n,
                             const uint8_t *date, uint8_t *out, uint64_t *out_off)
{
  stream_t s;
  uint64_t o = 0;
  http_field_t f[64];
  stream_construct(&s, NULL, NULL);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t *r = resps + 8u * i;
    const uint32_t nf = r[7] < 64 ? r[7] : 64;
    for (uint32_t k = 0; k < nf; k++) {
      const uint32_t *x = fields + 4u * (r[6] + k);
      f[k] = http_field_define(data(arena + x[0], x[1]), data(arena + x[2], x[3]));
    }
    http_write_response(&s, data(arena + r[0], r[1]), data(date, 29), data(arena + r[2], r[3]),
                        data(arena + r[4], r[5]), nf ? f : NULL, nf);
    data_t d = buffer_data(&s.output_waiting);
    out_off[i] = o;
    if (out) memcpy(out + o, data_base(d), data_size(d));
    o += data_size(d);
    buffer_clear(&s.output_waiting);
  }
  out_off[n] = o;
  stream_destruct(&s);
  return o;
}

/* http_read_request over a stream per request (config 5's path, http.c:177-234),
 * threads x reps, on a private copy per thread (chunked bodies are rewritten in
 * place); returns elapsed ns */
struct ref_http_mt_arg {
  uint8_t *bytes;
  const uint64_t *offsets;
  uint32_t lo, hi, max_headers;
  int reps;
  long sum;
};

static void *ref_http_mt_worker(void *p)
{
  struct ref_http_mt_arg *a = p;
  http_field_t fields[256];
  long sum = 0;
  for (int rep = 0; rep < a->reps; rep++)
    for (uint32_t i = a->lo; i < a->hi; i++) {
      stream_t s;
      memset(&s, 0, sizeof s);
      s.fd = -1;
      s.input.data = data(a->bytes + a->offsets[i], a->offsets[i + 1] - a->offsets[i]);
      s.input.capacity = a->offsets[i + 1] - a->offsets[i];
      string_t method, target;
      data_t body;
      size_t count = a->max_headers;
      sum += http_read_request(&s, &method, &target, &body, fields, &count) + (long) s.input_consumed;
    }
  a->sum = sum;
  return NULL;
}

uint64_t ref_http_batch_mt(uint8_t *bytes, const uint64_t *offsets, uint32_t n, uint32_t max_headers,
                           int threads, int reps, long *checksum)
{
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if (max_headers > 256) max_headers = 256;
  pthread_t tid[256];
  struct ref_http_mt_arg args[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    args[t] = (struct ref_http_mt_arg) {bytes, offsets, (uint32_t) ((uint64_t) n * t / threads),
                                        (uint32_t) ((uint64_t) n * (t + 1) / threads), max_headers, reps, 0};
    pthread_create(&tid[t], NULL, ref_http_mt_worker, &args[t]);
  }
  long sum = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(tid[t], NULL);
    sum += args[t].sum;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (checksum)
    *checksum = sum;
  return (uint64_t) (t1.tv_sec - t0.tv_sec) * 1000000000ull + (uint64_t) (t1.tv_nsec - t0.tv_nsec);
}
