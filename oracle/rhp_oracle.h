/*
 * rhp_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * A from-scratch CPU restatement of libreactor's HTTP request-receive path:
 *   - picohttpparser phr_parse_request   /root/reference/src/picohttpparser/picohttpparser.c:383-409
 *   - libreactor http_read_request       /root/reference/src/reactor/http.c:177-234
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code.  The product path (libreactorng_amd/librhp.so) never links it.
 *
 * Parity pin: the restatement is checked against the reference itself, compiled
 * from /root/reference into oracle/_ref/ (see oracle/Makefile), by the
 * differential fuzzer oracle/diff_fuzz.c and by tests/golden/ fixtures that the
 * compiled reference produced (tests/golden/make_golden.py).
 *
 * Canonical ("wide") records below are shared by the reference harness
 * (oracle/ref_harness.c) and the restatement so the two can be compared
 * byte for byte.  All offsets are relative to the start of each request.
 */
#ifndef RHP_ORACLE_H
#define RHP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one request of the phr_parse_request view (phr_parse_request outputs) */
typedef struct orc_req {
  int32_t  ret;          /* >0 bytes consumed, -1 malformed, -2 partial */
  int32_t  minor_version;
  uint32_t num_headers;
  uint32_t pad;
  int64_t  method_off, method_len;
  int64_t  path_off, path_len;
} orc_req_t;

/* struct phr_header, as offsets; name_off == -1 encodes name == NULL (obs-fold) */
typedef struct orc_hdr {
  int64_t name_off, name_len;
  int64_t value_off, value_len;
} orc_hdr_t;

/* http_read_request view */
typedef struct orc_http {
  int32_t  result;       /* 1 request ready, 0 need more, -1 malformed */
  int32_t  body_kind;    /* 0 = data_null(), 1 = body present */
  uint64_t consumed;     /* bytes passed to stream_consume (mod 2^64) */
  int64_t  body_off;     /* body base - request base (if body_kind) */
  uint64_t body_len;
} orc_http_t;

/* scalar single-request restatements (buf must be readable beyond len: the
 * reference's SP-skip loops read past the end, picohttpparser.c:356-362) */
int orc_phr_parse_request(const uint8_t *buf, size_t len, orc_req_t *req,
                          orc_hdr_t *hdrs, size_t max_headers);
int orc_http_read_request(uint8_t *buf, size_t len, orc_req_t *req,
                          orc_hdr_t *hdrs, size_t max_headers, orc_http_t *http);

/* batch drivers over a packed batch (bytes, offsets[n+1]); hdrs is n*max_headers.
 * For ret <= 0 (phr) / result <= 0 (http) every field except the status is zeroed
 * so records compare canonically.  http mode may rewrite bytes (chunked bodies are
 * de-framed in place, http.c:134-160), exactly like the reference. */
void orc_phr_batch(const uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                   uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs);
void orc_http_batch(uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                    uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs,
                    orc_http_t *https);

/* multi-threaded phr batch (cpu_baseline leg of bench.py); returns ns elapsed */
uint64_t orc_phr_batch_mt(const uint8_t *bytes, const uint64_t *offsets, uint32_t n,
                          uint32_t max_headers, orc_req_t *reqs, orc_hdr_t *hdrs,
                          int threads, int reps);

/* http_write_response (src/reactor/http.c:286-297) over a batch (rhp_oracle.c) */
uint64_t orc_write_responses(const uint8_t *arena, const uint32_t *resps, const uint32_t *fields, uint32_t n,
                             const uint8_t *date, uint8_t *out, uint64_t *out_off);
uint64_t ref_write_responses(const uint8_t *arena, const uint32_t *resps, const uint32_t *fields, uint32_t n,
                             const uint8_t *date, uint8_t *out, uint64_t *out_off);

#ifdef __cplusplus
}
#endif
#endif
