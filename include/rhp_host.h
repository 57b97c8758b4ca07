/*
 * rhp_host.h -- host-side entry points of librhp_host.so (no GPU).
 *
 *   rhp_cpu_parse_batch   the product's exact scalar parser (rhp_scalar.h, the
 *                         same code the kernel's rare paths run) over a batch in
 *                         host memory; the reactor's http_read_request and its
 *                         "host" session parser use it
 *   rhp_emu_parse_batch   CPU emulation of the kernel's DFA algorithm, block for
 *                         block (tests only); stats[3] = fast ok, fast -1, exact
 *   (both take an rhp_batch_t (include/rhp.h) whose pointers are host memory)
 *   rhp_expand_records    any layout's header records (the compact and dense
 *                         ones included) as rhp_hdr_t, on the host;
 *   rhp_expand_reqs       the dense layout's request records as rhp_req_t
 *
 *   rhp_phr_parse_request the same exact parser with phr_parse_request's own
 *                         signature and outputs (pointers into buf, no length
 *                         limit): a drop-in for
 *                         /root/reference/src/picohttpparser/picohttpparser.h:51-52
 *                         (last_len != 0 runs is_complete first, :197-223, :399-401)
 *   rhp_http_read_cpu     http_read_request (/root/reference/src/reactor/http.c:177-234)
 *                         over one buffer with pointer outputs: the reactor's
 *                         http_read_request, and the server's path for requests
 *                         whose records do not fit the batch format (RHP_RET_TOOLONG)
 */
#ifndef RHP_HOST_H
#define RHP_HOST_H

#include <stdint.h>
#include "rhp.h"

#ifdef __cplusplus
extern "C" {
#endif

int rhp_cpu_parse_batch(const rhp_batch_t *batch);
/* rhp_fixup_sessions (rhp.h) on the host, over a RHP_BATCH_SPECULATIVE batch
 * parsed by rhp_cpu_parse_batch; 0 or -22 */
int rhp_cpu_fixup_sessions(const rhp_batch_t *batch, const rhp_session_t *sessions, uint32_t n_sessions,
                           rhp_session_result_t *results, uint64_t *req_start);
int rhp_emu_parse_batch(const rhp_batch_t *batch, uint64_t *stats);
/* rhp_pack_dense (rhp.h) on the host, over host copies of the batch's records
 * (the reactor's host-async parser exercises the dense copy-back with it) */
int rhp_cpu_pack_dense(const rhp_batch_t *batch, rhp_req_dense_t *dreq, rhp_http_compact_t *hc, uint16_t *lens16);

/* A parsed batch's header records as rhp_hdr_t, out[i * max_headers + k]
 * (request-major), from host copies of its reqs and hdrs in the batch's
 * layout; records past num_headers and those of requests with ret <= 0 are
 * zeroed.  For RHP_LAYOUT_COMPACT / RHP_LAYOUT_DENSE this is the running sum
 * of rhp.h (the wide records for RHP_F_WIDE requests; reqs as rhp_expand_reqs
 * makes them).  `batch` supplies n, max_headers and
 * layout only.  0, or -22 on bad arguments. */
int rhp_expand_records(const rhp_batch_t *batch, const rhp_req_t *reqs, const void *hdrs, rhp_hdr_t *out);
/* A parsed batch's request records as rhp_req_t[n]: copied, or for
 * RHP_LAYOUT_DENSE expanded from rhp_req_dense_t and the wide area (rhp.h;
 * a dense record's flags become 0, a wide one's RHP_F_WIDE is set).  `reqs` is
 * the batch's reqs buffer as the parser left it.  0, or -22.  Expand the
 * requests first: rhp_expand_records and rhp_expand_http take rhp_req_t. */
int rhp_expand_reqs(const rhp_batch_t *batch, const void *reqs, rhp_req_t *out);
/* A batch's http records (RHP_MODE_HTTP) as rhp_http_t[n]: copied, or for
 * RHP_LAYOUT_COMPACT expanded from the compact records and their wide area
 * (rhp.h rhp_http_compact_t; consumed from reqs[i].ret).  0, or -22. */
int rhp_expand_http(const rhp_batch_t *batch, const rhp_req_t *reqs, const void *http, rhp_http_t *out);

/* struct phr_header (picohttpparser.h:42-47): name == NULL for an obs-fold line */
typedef struct rhp_phr_header {
  const char *name;
  size_t      name_len;
  const char *value;
  size_t      value_len;
} rhp_phr_header_t;

/* phr_parse_request: >0 bytes consumed, -1 malformed, -2 partial.  *num_headers
 * is the capacity on input and the count on output.  As the reference, it may
 * read bytes past buf + len while they are SP (picohttpparser.c:356-362). */
int rhp_phr_parse_request(const char *buf, size_t len, const char **method, size_t *method_len, const char **path,
                          size_t *path_len, int *minor_version, rhp_phr_header_t *headers, size_t *num_headers,
                          size_t last_len);

/* http_read_request's outputs for one buffer (http.c:177-234) */
typedef struct rhp_http_req {
  const char    *method;
  size_t         method_len;
  const char    *target;
  size_t         target_len;
  int            minor_version;
  const uint8_t *body;       /* NULL: data_null() */
  size_t         body_len;
  uint64_t       consumed;   /* bytes stream_consume() is given (result 1) */
} rhp_http_req_t;

/* 1 ready, 0 need more bytes (or empty), -1 malformed.  *fields_count is the
 * capacity on input, the count on output.  A chunked body is de-framed in place
 * (http.c:155), so buf is written. */
int rhp_http_read_cpu(uint8_t *buf, size_t len, rhp_http_req_t *req, rhp_phr_header_t *fields, size_t *fields_count);

/* Test hooks (tests/test_cpu_units.py): the GPU replay's windowed chunk-size-line
 * parse (rhp_scalar.h one_chunk_window: the nw <= 32 bytes at `line`, 32
 * readable; 0 = undecided) and the byte-wise one it must equal (one_chunk_t,
 * the size line at body offset `at`; the body readable to size + 64). */
int rhp_test_chunk_window(const uint8_t *line, uint32_t nw, uint64_t avail, int64_t *res, uint64_t *data_off,
                          uint64_t *data_len);
int64_t rhp_test_chunk_exact(const uint8_t *body, uint64_t at, uint64_t size, uint64_t *data_off, uint64_t *data_len);

#ifdef __cplusplus
}
#endif
#endif
