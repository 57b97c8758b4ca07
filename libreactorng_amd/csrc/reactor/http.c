/*
 * http.c -- the http module of the libreactor surface (reference
 * src/reactor/http.c, http.h:34-37).
 *
 *   http_read_request    one request from a stream (http.c:177-234): the same
 *                        contract, answered by the product's exact parser on
 *                        the host with pointer outputs (rhp_http_read_cpu, no
 *                        length limit).  The server parses sessions in batches
 *                        on the GPU (server.c) and uses it only for requests
 *                        the batch records cannot hold (RHP_RET_TOOLONG).
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
void reactor_http_fill(const uint8_t *base, const rhp_req_t *r, const rhp_hdr_t *h, size_t hs, const rhp_http_t *x,
                       string_t *method, string_t *target, data_t *body, http_field_t *fields, size_t *fields_count)
{
  *method = data(base + r->method_off, r->method_len);
  *target = data(base + r->path_off, r->path_len);
  for (uint32_t k = 0; k < r->num_headers; k++)
  {
    const rhp_hdr_t *o = &h[k * hs];   /* record k at h[k * hs] (hs = 1 request-major, n header-major; rhp.h) */
    fields[k].name = o->name_off == RHP_NAME_NULL ? data_null() : data(base + o->name_off, o->name_len);
    fields[k].value = data(base + o->value_off, o->value_len);
  }
  *fields_count = r->num_headers;
  *body = x->body_kind ? data(base + r->ret, x->body_len) : data_null();
}

int http_read_request(stream_t *stream, string_t *method, string_t *target, data_t *body, http_field_t *fields,
                      size_t *fields_count)
{
  data_t input = stream_read(stream);
  rhp_http_req_t r;
  rhp_phr_header_t h[RHP_MAX_HEADERS];
  size_t n = *fields_count < RHP_MAX_HEADERS ? *fields_count : RHP_MAX_HEADERS;
  int result = rhp_http_read_cpu(data_base(input), data_size(input), &r, h, &n);
  if (result != 1)
    return result;
  *method = data(r.method, r.method_len);
  *target = data(r.target, r.target_len);
  for (size_t k = 0; k < n; k++)
  {
    fields[k].name = h[k].name ? data(h[k].name, h[k].name_len) : data_null();
    fields[k].value = data(h[k].value, h[k].value_len);
  }
  *fields_count = n;
  *body = r.body ? data(r.body, r.body_len) : data_null();
  stream_consume(stream, r.consumed);
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
