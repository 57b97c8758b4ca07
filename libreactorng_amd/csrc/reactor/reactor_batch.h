/* reactor_batch.h -- internal: the server's batch parse (batch.c) */
#ifndef REACTOR_BATCH_H
#define REACTOR_BATCH_H

#include <stddef.h>
#include <stdint.h>
#include "rhp.h"

#define REACTOR_BATCH_HEADERS 16u   /* fields_count = 16 per request (server.c:44 of the reference) */
#define REACTOR_BATCH_SLOTS   2     /* rounds in flight per thread: one parsing, one being packed */

typedef struct reactor_batch_result
{
  const uint8_t    *bytes;   /* the packed input after the parse (chunked bodies de-framed) */
  const uint64_t   *offsets; /* n + 1 */
  const rhp_req_t  *reqs;
  const rhp_hdr_t  *hdrs;    /* REACTOR_BATCH_HEADERS per request, request-major */
  uint32_t          n;
  const rhp_http_t *http;
  /* rhp_fixup_sessions: session m's requests are record slots
   * sessions[m].piece_lo + 0 .. + session_results[m].n_slots - 1, request j
   * starting at byte req_start[j] of `bytes` */
  const rhp_session_t        *sessions;
  const rhp_session_result_t *session_results;
  const uint64_t             *req_start;
  uint32_t                    n_sessions;
  /* gpu (round 6): the dense copies the round brought back (rhp_pack_dense);
   * reqs / hdrs / http / req_start are then valid only for slots marked wide.
   * Read a slot through reactor_batch_record. */
  int                         dense;
  const rhp_req_dense_t      *dreq;
  const rhp_http_compact_t   *hc;
  const uint16_t             *lens16;   /* header-major, n per row */
} reactor_batch_result_t;

/* record slot i of a result: its request, http and header records (expanded
 * from the dense copies into *req, *x and h[REACTOR_BATCH_HEADERS], or the
 * batch's own; *hp is the header records, one per request header, stride 1) */
void reactor_batch_record(const reactor_batch_result_t *r, uint32_t i, rhp_req_t *req, rhp_http_t *x, rhp_hdr_t *h,
                          const rhp_hdr_t **hp);

/* 1: rounds complete asynchronously (gpu parser) and each completion adds 1 to
 * the eventfd reactor_batch_fd(); 0: reactor_batch_submit parses in place */
int       reactor_batch_async(void);
/* once per thread, before its first round (server_open): the gpu parser's
 * slots, code object and first launches set up by one warm-up round, so no
 * client's first burst pays for them */
void      reactor_batch_prepare(void);
int       reactor_batch_fd(void);
/* the thread's parser state (streams, events, pinned and device slots, the
 * completion thread) released on this thread, e.g. when its last server goes;
 * every round must be complete.  The next round sets it up again. */
void      reactor_batch_release(void);
/* staging of slot k for `bytes` packed input bytes (+ RHP_PAD), n pieces and
 * n_sessions sessions */
uint8_t  *reactor_batch_reserve(int k, size_t bytes, uint32_t n, uint32_t n_sessions);
uint64_t *reactor_batch_offsets(int k);
rhp_session_t *reactor_batch_sessions(int k);
/* parse slot k's n pieces (offsets[0..n-1], offsets[n] = bytes) of
 * n_sessions sessions: a speculative http batch, then rhp_fixup_sessions;
 * slots complete in submission order */
void      reactor_batch_submit(int k, uint32_t n, size_t bytes, uint32_t n_sessions);
/* rounds completed since the last call (reads the eventfd; 0 if none) */
int       reactor_batch_completed(void);
/* block until every submitted round is complete (teardown) */
void      reactor_batch_wait(void);
/* the records of completed slot k */
void      reactor_batch_result(int k, reactor_batch_result_t *out);

/* 1: replies produced while a round is dispatched are serialized together
 * after it (RHP_REACTOR_WRITER=gpu | host-batch); 0: written at once */
int       reactor_batch_writer(void);
/* serialize n replies (spans of `arena`) as http_write_response does; out and
 * out_off (n + 1 offsets) stay valid until the next call */
void      reactor_batch_write(const uint8_t *arena, size_t arena_n, const rhp_resp_t *resps, uint32_t n,
                              const rhp_resp_field_t *fields, uint32_t n_fields, const char *date, const uint8_t **out,
                              const uint64_t **out_off);

/* records (offsets into base) -> the reference's output iovecs (http.c) */
struct http_field;
void reactor_http_fill(const uint8_t *base, const rhp_req_t *r, const rhp_hdr_t *h, size_t hs, const rhp_http_t *x,
                       data_t *method, data_t *target, data_t *body, struct http_field *fields, size_t *fields_count);

#endif
