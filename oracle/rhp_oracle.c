/*
 * rhp_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the libreactor
 * request-receive parser, used as the parity checker for the MI355X kernels.
 *
 * Written from the reference's observable behaviour, position-indexed (no
 * pointer tricks, no SSE4.2): picohttpparser's SSE4.2 findchar_fast is a pure
 * accelerator whose results equal the scalar loops.
 *
 * Citations (all /root/reference/...):
 *   ADVANCE_TOKEN                src/picohttpparser/picohttpparser.c:71-94
 *   token_char_map               src/picohttpparser/picohttpparser.c:96-103
 *   get_token_to_eol             src/picohttpparser/picohttpparser.c:134-195
 *   parse_http_version           src/picohttpparser/picohttpparser.c:245-261
 *   parse_headers                src/picohttpparser/picohttpparser.c:263-339
 *   parse_request                src/picohttpparser/picohttpparser.c:341-381
 *   phr_parse_request            src/picohttpparser/picohttpparser.c:383-409
 *   http_chunk_size/chunk/dechunk src/reactor/http.c:73-160
 *   http_field_lookup            src/reactor/http.c:167-175 (+ memcasecmp data.c:11-28)
 *   http_read_request            src/reactor/http.c:177-234
 */
#define _GNU_SOURCE
#include "rhp_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ERR_BAD (-1)
#define ERR_PARTIAL (-2)

/* RFC 7230 tchar, same membership as token_char_map (picohttpparser.c:96-103) */
static int orc_is_tchar(uint8_t c)
{
  if (c >= '0' && c <= '9') return 1;
  if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return 1;
  switch (c) {
  case '!': case '#': case '$': case '%': case '&': case '\'': case '*':
  case '+': case '-': case '.': case '^': case '_': case '`': case '|': case '~':
    return 1;
  default:
    return 0;
  }
}

static int orc_is_ctl_or_del(uint8_t c) { return c < 0x20 || c == 0x7f; }

/* ADVANCE_TOKEN: scan to the first SP; CTL/DEL -> -1; reaching exactly `len`
 * -> -2.  The EOF test is an equality test (buf == buf_end), so a scan that
 * started beyond the end never sees EOF (picohttpparser.c:55-59,76-91). */
static int orc_token(const uint8_t *b, size_t len, size_t *p, int64_t *off, int64_t *tlen)
{
  size_t q = *p;
  if (q == len)
    return ERR_PARTIAL;
  for (;;) {
    uint8_t c = b[q];
    if (c == ' ')
      break;
    if (orc_is_ctl_or_del(c))
      return ERR_BAD;
    ++q;
    if (q == len)
      return ERR_PARTIAL;
  }
  *off = (int64_t) *p;
  *tlen = (int64_t) (q - *p);
  *p = q;
  return 0;
}

/* CR must be followed by LF; EOF in between is partial (EXPECT_CHAR) */
static int orc_crlf_tail(const uint8_t *b, size_t len, size_t *p)
{
  ++*p;                          /* past CR */
  if (*p == len)
    return ERR_PARTIAL;
  if (b[(*p)++] != '\n')
    return ERR_BAD;
  return 0;
}

int orc_phr_parse_request(const uint8_t *b, size_t len, orc_req_t *req,
                          orc_hdr_t *hdrs, size_t max_headers)
{
  size_t p = 0;
  int r;

  memset(req, 0, sizeof *req);
  req->minor_version = -1;
  req->method_off = req->path_off = -1;

  /* one optional leading empty line (parse_request :345-352) */
  if (p == len)
    return req->ret = ERR_PARTIAL;
  if (b[p] == '\r') {
    if ((r = orc_crlf_tail(b, len, &p)) != 0)
      return req->ret = r;
  } else if (b[p] == '\n') {
    ++p;
  }

  /* method, then >=1 SP with no EOF test (:355-358) */
  if ((r = orc_token(b, len, &p, &req->method_off, &req->method_len)) != 0)
    return req->ret = r;
  do ++p; while (b[p] == ' ');
  /* path, then SPs (:359-362) */
  if ((r = orc_token(b, len, &p, &req->path_off, &req->path_len)) != 0)
    return req->ret = r;
  do ++p; while (b[p] == ' ');
  if (req->method_len == 0 || req->path_len == 0)
    return req->ret = ERR_BAD;

  /* "HTTP/1.<digit>" needs 9 bytes left (signed test) (:245-261) */
  if ((int64_t) len - (int64_t) p < 9)
    return req->ret = ERR_PARTIAL;
  {
    static const char lit[7] = {'H', 'T', 'T', 'P', '/', '1', '.'};
    for (int k = 0; k < 7; k++)
      if (b[p + k] != (uint8_t) lit[k])
        return req->ret = ERR_BAD;
    uint8_t d = b[p + 7];
    if (d < '0' || d > '9')
      return req->ret = ERR_BAD;
    req->minor_version = d - '0';
    p += 8;
  }
  /* end of request line: CRLF or LF (:370-378) */
  if (b[p] == '\r') {
    if ((r = orc_crlf_tail(b, len, &p)) != 0)
      return req->ret = r;
  } else if (b[p] == '\n') {
    ++p;
  } else {
    return req->ret = ERR_BAD;
  }

  /* header lines (:263-339) */
  size_t n = 0;
  for (;; ++n) {
    if (p == len) {
      req->num_headers = (uint32_t) n;
      return req->ret = ERR_PARTIAL;
    }
    if (b[p] == '\r') {
      if ((r = orc_crlf_tail(b, len, &p)) != 0)
        return req->ret = r;
      break;
    }
    if (b[p] == '\n') {
      ++p;
      break;
    }
    if (n == max_headers)
      return req->ret = ERR_BAD;
    orc_hdr_t *h = &hdrs[n];
    if (!(n != 0 && (b[p] == ' ' || b[p] == '\t'))) {
      size_t name = p;
      for (;;) {
        uint8_t c = b[p];
        if (c == ':')
          break;
        if (!orc_is_tchar(c))
          return req->ret = ERR_BAD;
        ++p;
        if (p == len)
          return req->ret = ERR_PARTIAL;
      }
      if (p == name)
        return req->ret = ERR_BAD;
      h->name_off = (int64_t) name;
      h->name_len = (int64_t) (p - name);
      ++p;
      for (;; ++p) {
        if (p == len)
          return req->ret = ERR_PARTIAL;
        if (!(b[p] == ' ' || b[p] == '\t'))
          break;
      }
    } else {
      h->name_off = -1;          /* obs-fold continuation: name == NULL */
      h->name_len = 0;
    }
    /* get_token_to_eol: stop at CTL other than HT, or DEL */
    size_t vs = p, vlen;
    uint8_t c;
    for (;; ++p) {
      if (p == len)
        return req->ret = ERR_PARTIAL;
      c = b[p];
      if ((c < 0x20 && c != '\t') || c == 0x7f)
        break;
    }
    if (c == '\r') {
      if ((r = orc_crlf_tail(b, len, &p)) != 0)
        return req->ret = r;
      vlen = p - 2 - vs;
    } else if (c == '\n') {
      vlen = p - vs;
      ++p;
    } else {
      return req->ret = ERR_BAD;
    }
    /* trim trailing SP / HT (:327-336) */
    while (vlen > 0 && (b[vs + vlen - 1] == ' ' || b[vs + vlen - 1] == '\t'))
      --vlen;
    h->value_off = (int64_t) vs;
    h->value_len = (int64_t) vlen;
    req->num_headers = (uint32_t) (n + 1);
  }
  req->num_headers = (uint32_t) n;
  return req->ret = (int32_t) p;
}

/* ---- http_read_request (http.c:177-234) ---- */

static int orc_upper(int c) { return (c >= 'a' && c <= 'z') ? c - 32 : c; }

/* string_equal_case: equal sizes and memcasecmp == 0 (data.c:11-28,120-123) */
static int orc_name_is(const uint8_t *b, const orc_hdr_t *h, const char *name)
{
  size_t n = strlen(name);
  if (h->name_off < 0 || (size_t) h->name_len != n)
    return 0;
  for (size_t i = 0; i < n; i++)
    if (orc_upper(b[h->name_off + i]) != orc_upper((uint8_t) name[i]))
      return 0;
  return 1;
}

/* http_field_lookup: first matching field (http.c:167-175) */
static const orc_hdr_t *orc_lookup(const uint8_t *b, const orc_hdr_t *hdrs, size_t n, const char *name)
{
  for (size_t i = 0; i < n; i++)
    if (orc_name_is(b, &hdrs[i], name))
      return &hdrs[i];
  return NULL;
}

/* glibc strtoull(s, NULL, 10) in the C locale: skip isspace, optional sign,
 * decimal digits, saturate to ULLONG_MAX on overflow, negate for '-'. */
static uint64_t orc_strtoull10(const uint8_t *s)
{
  while (*s == ' ' || (*s >= '\t' && *s <= '\r'))
    s++;
  int neg = 0;
  if (*s == '+' || *s == '-')
    neg = (*s++ == '-');
  uint64_t v = 0;
  int overflow = 0;
  while (*s >= '0' && *s <= '9') {
    uint64_t d = (uint64_t) (*s++ - '0');
    if (v > (UINT64_MAX - d) / 10)
      overflow = 1;
    v = v * 10 + d;
  }
  if (overflow)
    return UINT64_MAX;
  return neg ? (uint64_t) 0 - v : v;
}

/* glibc strtoul(s, NULL, 16) restricted to what http_chunk_size feeds it: a
 * non-empty run of hex digits.  Saturates to ULONG_MAX on overflow. */
static uint64_t orc_strtoul16(const uint8_t *s)
{
  uint64_t v = 0;
  int overflow = 0;
  for (;; s++) {
    int d;
    if (*s >= '0' && *s <= '9') d = *s - '0';
    else if (*s >= 'a' && *s <= 'f') d = *s - 'a' + 10;
    else if (*s >= 'A' && *s <= 'F') d = *s - 'A' + 10;
    else break;
    if (v >> 60)
      overflow = 1;
    v = (v << 4) | (uint64_t) d;
  }
  return overflow ? UINT64_MAX : v;
}

static int orc_isblank(uint8_t c) { return c == ' ' || c == '\t'; }
static int orc_isxdigit(uint8_t c)
{
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}

/* http_chunk_size (http.c:73-116): returns bytes of the size line, 0 (need
 * more) or -1.  The line scans are bounded by the first '\n' in the input. */
static int64_t orc_chunk_size(const uint8_t *in, size_t size, uint64_t *csize)
{
  if (!memchr(in, '\n', size))
    return 0;
  const uint8_t *p = in;
  while (orc_isblank(*p)) p++;
  const uint8_t *digits = p;
  while (orc_isxdigit(*p)) p++;
  if (digits == p)
    return -1;
  while (orc_isblank(*p)) p++;
  if (*p == ';') {
    while (*p != '\n') p++;
    if (p[-1] != '\r')
      return -1;
  } else {
    if (*p != '\r')
      return -1;
    p++;
  }
  if (*p != '\n')
    return -1;
  p++;
  *csize = orc_strtoul16(digits);
  if (*csize == UINT64_MAX)
    return -1;
  return (int64_t) (p - in);
}

/* http_chunk (http.c:118-132): the 2 bytes after the data are skipped unchecked */
static int64_t orc_chunk(const uint8_t *in, size_t size, size_t *coff, uint64_t *clen)
{
  uint64_t cs = 0;
  int64_t n = orc_chunk_size(in, size, &cs);
  if (n <= 0)
    return n;
  if ((uint64_t) n + 2 > size)
    return 0;
  if (cs > size - (uint64_t) n - 2)
    return 0;
  *coff = (size_t) n;
  *clen = cs;
  return (int64_t) (cs + (uint64_t) n + 2);
}

/* http_dechunk (http.c:134-160): validate every chunk up to the empty one, then
 * compact the chunk payloads to the start of `in` (in place).  Returns bytes
 * of framing consumed, 0 or -1; *body_len = payload bytes. */
static int64_t orc_dechunk(uint8_t *in, size_t size, uint64_t *body_len)
{
  size_t offset = 0, coff = 0;
  uint64_t clen = 0;
  int64_t n;
  do {
    n = orc_chunk(in + offset, size - offset, &coff, &clen);
    if (n <= 0)
      return n;
    offset += (size_t) n;
  } while (clen);

  uint64_t total = 0;
  offset = 0;
  do {
    n = orc_chunk(in + offset, size - offset, &coff, &clen);
    memmove(in + total, in + offset + coff, clen);
    offset += (size_t) n;
    total += clen;
  } while (clen);
  *body_len = total;
  return (int64_t) offset;
}

int orc_http_read_request(uint8_t *b, size_t len, orc_req_t *req,
                          orc_hdr_t *hdrs, size_t max_headers, orc_http_t *http)
{
  memset(http, 0, sizeof *http);
  /* records carry the phr status too; on empty input phr reports -2 without
   * reading, so computing it first changes nothing observable */
  int n = orc_phr_parse_request(b, len, req, hdrs, max_headers);
  if (len == 0)
    return http->result = 0;      /* data_empty(input) (http.c:185-186) */
  if (n <= 0)
    return http->result = (n == -1 ? -1 : 0);

  if (req->method_len == 3 && memcmp(b + req->method_off, "GET", 3) == 0) {
    http->consumed = (uint64_t) n;  /* GET fast path (http.c:198-202) */
    return http->result = 1;
  }
  const orc_hdr_t *te = orc_lookup(b, hdrs, req->num_headers, "Transfer-Encoding");
  const orc_hdr_t *cl = orc_lookup(b, hdrs, req->num_headers, "Content-Length");
  int te_set = te && te->value_len != 0;
  int cl_set = cl && cl->value_len != 0;

  if (cl_set) {                   /* http.c:208-218 */
    if (te_set)
      return http->result = -1;
    uint64_t size = orc_strtoull10(b + cl->value_off);
    if ((uint64_t) len < (uint64_t) n + size)
      return http->result = 0;
    http->body_kind = 1;
    http->body_off = n;
    http->body_len = size;
    http->consumed = (uint64_t) n + size;
    return http->result = 1;
  }
  if (te_set) {                   /* http.c:221-230 */
    static const char chunked[] = "Chunked";
    int eq = (size_t) te->value_len == sizeof chunked - 1;
    for (size_t i = 0; eq && i < sizeof chunked - 1; i++)
      eq = orc_upper(b[te->value_off + i]) == orc_upper((uint8_t) chunked[i]);
    if (!eq)
      return http->result = -1;
    uint64_t blen = 0;
    int64_t size = orc_dechunk(b + n, len - (size_t) n, &blen);
    if (size <= 0)
      return http->result = (int32_t) size;
    http->body_kind = 1;
    http->body_off = n;
    http->body_len = blen;
    http->consumed = (uint64_t) n + (uint64_t) size;
    return http->result = 1;
  }
  http->consumed = (uint64_t) n;
  return http->result = 1;
}

/* ---- batch drivers ---- */

static void orc_canon_req(orc_req_t *r, orc_hdr_t *h, uint32_t max_headers)
{
  int32_t ret = r->ret;
  memset(r, 0, sizeof *r);
  r->ret = ret;
  memset(h, 0, sizeof *h * max_headers);
}

void orc_phr_batch(const uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                   uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs)
{
  for (uint32_t i = 0; i < n; i++) {
    orc_hdr_t *h = hdrs + (size_t) i * max_headers;
    memset(h, 0, sizeof *h * max_headers);
    int r = orc_phr_parse_request(bytes + offsets[i], offsets[i + 1] - offsets[i], &reqs[i], h, max_headers);
    if (r <= 0)
      orc_canon_req(&reqs[i], h, max_headers);
  }
}

void orc_http_batch(uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                    uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs,
                    orc_http_t *https)
{
  for (uint32_t i = 0; i < n; i++) {
    orc_hdr_t *h = hdrs + (size_t) i * max_headers;
    memset(h, 0, sizeof *h * max_headers);
    int r = orc_http_read_request(bytes + offsets[i], offsets[i + 1] - offsets[i], &reqs[i], h,
                                  max_headers, &https[i]);
    if (r <= 0) {
      orc_canon_req(&reqs[i], h, max_headers);
      memset(&https[i], 0, sizeof https[i]);
      https[i].result = r;
    }
  }
}

struct orc_mt_arg {
  const uint8_t *bytes;
  const uint64_t *offsets;
  uint32_t lo, hi, max_headers;
  orc_req_t *reqs;
  orc_hdr_t *hdrs;
  int reps;
};

static void *orc_mt_worker(void *varg)
{
  struct orc_mt_arg *a = varg;
  for (int rep = 0; rep < a->reps; rep++)
    for (uint32_t i = a->lo; i < a->hi; i++)
      orc_phr_parse_request(a->bytes + a->offsets[i], a->offsets[i + 1] - a->offsets[i], &a->reqs[i],
                            a->hdrs + (size_t) i * a->max_headers, a->max_headers);
  return NULL;
}

uint64_t orc_phr_batch_mt(const uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                          uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs,
                          int threads, int reps)
{
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  struct orc_mt_arg args[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < threads; t++) {
    args[t] = (struct orc_mt_arg) {bytes, offsets, (uint32_t) ((uint64_t) n * t / threads),
                                   (uint32_t) ((uint64_t) n * (t + 1) / threads), max_headers,
                                   reqs, hdrs, reps};
    pthread_create(&tid[t], NULL, orc_mt_worker, &args[t]);
  }
  for (int t = 0; t < threads; t++)
    pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (uint64_t) (t1.tv_sec - t0.tv_sec) * 1000000000ull + (uint64_t) (t1.tv_nsec - t0.tv_nsec);
}

/*
 * http_write_response (src/reactor/http.c:286-297) restated for a batch, TEST
 * INFRASTRUCTURE ONLY.  resps: n x {status off,len, type off,len, body off,len,
 * fields_first, fields_count}; fields: {name off,len, value off,len}; strings are
 * spans of `arena`; `date` is 29 bytes.  Response i goes to out[out_off[i],
 * out_off[i+1]) in the reference's push order: status line (:250-252), Server,
 * Date, Content-Type, Content-Length fields (:253-256, http_push_field :61-69),
 * the extra fields (:279-280), the empty line and the body (:257-258).  The length
 * is printed in decimal (http_u32_sprint :17-44).  out == NULL: offsets only.
 * Returns the total size.
 */
static uint64_t orc_put(uint8_t *out, uint64_t o, const void *src, size_t len)
{
  if (out) memcpy(out + o, src, len);
  return o + len;
}

uint64_t orc_write_responses(const uint8_t *arena, const uint32_t *resps, const uint32_t *fields, uint32_t n,
                             const uint8_t *date, uint8_t *out, uint64_t *out_off)
{
  uint64_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t *r = resps + 8u * i;
    char digits[16];
    const int nd = snprintf(digits, sizeof digits, "%u", r[5]);
    out_off[i] = o;
    o = orc_put(out, o, "HTTP/1.1 ", 9);
    o = orc_put(out, o, arena + r[0], r[1]);
    o = orc_put(out, o, "\r\nServer: *\r\nDate: ", 19);
    o = orc_put(out, o, date, 29);
    o = orc_put(out, o, "\r\nContent-Type: ", 16);
    o = orc_put(out, o, arena + r[2], r[3]);
    o = orc_put(out, o, "\r\nContent-Length: ", 18);
    o = orc_put(out, o, digits, (size_t) nd);
    o = orc_put(out, o, "\r\n", 2);
    for (uint32_t f = 0; f < r[7]; f++) {
      const uint32_t *x = fields + 4u * (r[6] + f);
      o = orc_put(out, o, arena + x[0], x[1]);
      o = orc_put(out, o, ": ", 2);
      o = orc_put(out, o, arena + x[2], x[3]);
      o = orc_put(out, o, "\r\n", 2);
    }
    o = orc_put(out, o, "\r\n", 2);
    o = orc_put(out, o, arena + r[4], r[5]);
  }
  out_off[n] = o;
  return o;
}
