/*
 * http.c -- the http module of the libreactor surface (reference
 * src/reactor/http.c, http.h:34-37).
 *
 *   http_read_request    one request from a stream (http.c:177-234): the same
 *                        contract, answered by the product's exact parser on
 *                        the host (rhp_cpu_parse_batch, a batch of one).  The
 *                        server does not call it: sessions are parsed in
 *                        batches on the GPU (server.c).
 *   http_write_response  the response serializer (http.c:236-297): status
 *                        line, Server / Date / Content-Type / Content-Length,
 *                        the caller's fields, blank line, body.
 *   http_field_define / http_field_lookup (http.c:162-175).
 */
#include <stdio.h>
#include <string.h>

#include "reactor.h"
#include "rhp.h"
#include "rhp_host.h"

http_field_t http_field_define(string_t name, string_t value)
{
  return (http_field_t) {.name = name, .value = value};
}

/* the first field whose name equals `name` ignoring ASCII case, else string_null() */
string_t http_field_lookup(http_field_t *fields, size_t fields_count, string_t name)
{
  for (size_t i = 0; i < fields_count; i++)
    if (string_equal_case(fields[i].name, name))
      return fields[i].value;
  return string_null();
}

/* request records (offsets into `base`) -> the reference's output iovecs */
void reactor_http_fill(const uint8_t *base, const rhp_req_t *r, const rhp_hdr_t *h, const rhp_http_t *x,
                       string_t *method, string_t *target, data_t *body, http_field_t *fields, size_t *fields_count)
{
  *method = data(base + r->method_off, r->method_len);
  *target = data(base + r->path_off, r->path_len);
  for (uint32_t k = 0; k < r->num_headers; k++)
  {
    fields[k].name = h[k].name_off == RHP_NAME_NULL ? data_null() : data(base + h[k].name_off, h[k].name_len);
    fields[k].value = data(base + h[k].value_off, h[k].value_len);
  }
  *fields_count = r->num_headers;
  *body = x->body_kind ? data(base + r->ret, x->body_len) : data_null();
}

int http_read_request(stream_t *stream, string_t *method, string_t *target, data_t *body, http_field_t *fields,
                      size_t *fields_count)
{
  data_t input = stream_read(stream);
  if (data_empty(input))
    return 0;
  rhp_hdr_t h[RHP_MAX_HEADERS];
  rhp_req_t r;
  rhp_http_t x;
  uint64_t offsets[2] = {0, data_size(input)};
  uint32_t maxh = *fields_count < RHP_MAX_HEADERS ? (uint32_t) *fields_count : RHP_MAX_HEADERS;
  rhp_batch_t b = {
    .bytes = data_base(input), .bytes_rw = data_base(input), .offsets = offsets,
    .bytes_size = data_size(input) + RHP_PAD, .n = 1, .max_headers = maxh, .mode = RHP_MODE_HTTP,
    .reqs = &r, .hdrs = h, .http = &x};
  (void) rhp_cpu_parse_batch(&b);
  if (x.result != 1)
    return x.result;
  reactor_http_fill(data_base(input), &r, h, &x, method, target, body, fields, fields_count);
  stream_consume(stream, x.consumed);
  return 1;
}

/* ------------------------------------------------------------ response */

static char *put(char *p, data_t d)
{
  if (data_size(d))
    memcpy(p, data_base(d), data_size(d));
  return p + data_size(d);
}

static char *put_field(char *p, data_t name, data_t value)
{
  p = put(p, name);
  *p++ = ':';
  *p++ = ' ';
  p = put(p, value);
  *p++ = '\r';
  *p++ = '\n';
  return p;
}

/* decimal digits of a u32 (the reference formats data_size(body) as uint32_t, http.c:243-245) */
static size_t u32_print(uint32_t n, char out[16])
{
  char tmp[16];
  size_t k = 0;
  do
  {
    tmp[k++] = (char) ('0' + n % 10);
    n /= 10;
  } while (n);
  for (size_t i = 0; i < k; i++)
    out[i] = tmp[k - 1 - i];
  return k;
}

void http_write_response(stream_t *stream, string_t status, string_t date, string_t type, data_t body,
                         http_field_t *fields, size_t fields_count)
{
  char len[16];
  data_t length = data(len, u32_print((uint32_t) data_size(body), len));
  size_t size = 9 + data_size(status) + 2 + 11 + (8 + data_size(date)) + (16 + data_size(type)) +
                (18 + data_size(length)) + 2 + data_size(body);
  for (size_t i = 0; i < fields_count; i++)
    size += data_size(fields[i].name) + 2 + data_size(fields[i].value) + 2;
  char *p = stream_allocate(stream, size);
  p = put(p, string("HTTP/1.1 "));
  p = put(p, status);
  p = put(p, string("\r\n"));
  p = put_field(p, string("Server"), string("*"));
  p = put_field(p, string("Date"), date);
  p = put_field(p, string("Content-Type"), type);
  p = put_field(p, string("Content-Length"), length);
  for (size_t i = 0; i < fields_count; i++)
    p = put_field(p, fields[i].name, fields[i].value);
  p = put(p, string("\r\n"));
  (void) put(p, body);
}
