/* reactor_batch.h -- internal: the server's batch parse (batch.c) */
#ifndef REACTOR_BATCH_H
#define REACTOR_BATCH_H

#include <stddef.h>
#include <stdint.h>
#include "rhp.h"

#define REACTOR_BATCH_HEADERS 16u   /* fields_count = 16 per request (server.c:44 of the reference) */

typedef struct reactor_batch_result
{
  const uint8_t    *bytes;   /* the packed input after the parse (chunked bodies de-framed) */
  const rhp_req_t  *reqs;
  const rhp_hdr_t  *hdrs;    /* REACTOR_BATCH_HEADERS per request, header-major (stride n) */
  uint32_t          n;
  const rhp_http_t *http;
} reactor_batch_result_t;

/* staging for `bytes` packed input bytes (+ RHP_PAD) and n segments */
uint8_t  *reactor_batch_reserve(size_t bytes, uint32_t n);
uint64_t *reactor_batch_offsets(void);
/* parse the n segments (offsets[0..n-1], offsets[n] = bytes) in http_read_request mode */
int       reactor_batch_run(uint32_t n, size_t bytes, reactor_batch_result_t *out);

/* records (offsets into base) -> the reference's output iovecs (http.c) */
struct http_field;
void reactor_http_fill(const uint8_t *base, const rhp_req_t *r, const rhp_hdr_t *h, size_t hs, const rhp_http_t *x,
                       data_t *method, data_t *target, data_t *body, struct http_field *fields, size_t *fields_count);

#endif
