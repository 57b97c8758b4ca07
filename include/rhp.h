/*
 * rhp.h -- MI355X batched HTTP/1.1 request parser: the C-ABI drop-in boundary.
 *
 * Replaces, for a batch of independent request buffers already in HBM:
 *   int phr_parse_request(const char *buf, size_t len, const char **method,
 *       size_t *method_len, const char **path, size_t *path_len, int *minor_version,
 *       struct phr_header *headers, size_t *num_headers, size_t last_len);
 *                       /root/reference/src/picohttpparser/picohttpparser.h:51-52
 *   int http_read_request(stream_t *, string_t *method, string_t *target, data_t *body,
 *       http_field_t *fields, size_t *fields_count);
 *                       /root/reference/src/reactor/http.h:36 (http.c:177-234)
 *
 * One call parses n requests.  Request i is bytes[offsets[i] .. offsets[i+1]) (its
 * `len`); the bytes after it (the next request, then >= RHP_PAD zero bytes after
 * the last one) are what the reference would read past the end.
 * Every pointer the reference returns into `buf` is returned here as an offset
 * from the request start (pointer - buf).  All buffers are device memory owned by
 * the caller; the call is asynchronous on `stream` (a hipStream_t).
 *
 * Requests of any length are parsed.  Records are compact (u16 offsets), so
 * the one answer they cannot carry is a successful parse whose header section
 * is longer than RHP_MAX_LEN bytes (phr ret > 65535): that request gets
 * ret = RHP_RET_TOOLONG (and in RHP_MODE_HTTP result = RHP_RET_TOOLONG) and no
 * other output; the caller parses it with a pointer-based parser
 * (rhp_phr_parse_request / rhp_http_read_cpu, include/rhp_host.h).  -1, -2 and
 * http results 0/-1 are exact at every length; body lengths and `consumed` are
 * u64.
 */
#ifndef RHP_H
#define RHP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RHP_PAD 256u            /* zero bytes required after the last request */
#define RHP_MAX_LEN 65535u      /* longest header section (phr ret) the u16 records hold */
#define RHP_MAX_HEADERS 64u     /* largest supported *num_headers capacity */
#define RHP_RET_TOOLONG (-3)

enum rhp_mode {
  RHP_MODE_PHR = 0,   /* phr_parse_request(buf, len, ..., &num_headers = max, last_len = 0) */
  RHP_MODE_HTTP = 1   /* http_read_request over a stream whose unconsumed input is the request */
};

/* phr_parse_request result for one request (16 B).  For ret <= 0 only `ret`
 * is meaningful (the reference leaves the other outputs unspecified). */
typedef struct rhp_req {
  int32_t  ret;            /* >0 bytes consumed, -1 malformed, -2 partial, RHP_RET_TOOLONG (ret > RHP_MAX_LEN) */
  uint16_t method_len;
  uint16_t path_off;
  uint16_t path_len;
  uint8_t  method_off;     /* 0, 1 or 2 (one optional leading CRLF / LF) */
  int8_t   minor_version;
  uint16_t num_headers;
  uint16_t flags;          /* RHP_F_* diagnostics, not part of parity */
} rhp_req_t;

#define RHP_F_EXACT 0x1u   /* resolved by the exact (scalar) device path, not the DFA */
#define RHP_F_WIDE  0x2u   /* RHP_LAYOUT_COMPACT: this request's header records are the wide ones */

/* struct phr_header as offsets (8 B); name_off == RHP_NAME_NULL encodes name ==
 * NULL (obs-fold continuation line, picohttpparser.c:318-321). */
typedef struct rhp_hdr {
  uint16_t name_off, name_len;
  uint16_t value_off, value_len;
} rhp_hdr_t;

#define RHP_NAME_NULL 0xFFFFu

/* Layout of the header records.  Request-major (the C array hdrs[n][max_headers],
 * the default): a request's records are contiguous.  Header-major
 * (hdrs[max_headers][n]): the records of one header index are contiguous across
 * requests, so the records a wave completes together for consecutive requests of
 * a uniform batch are whole lines (request-major writes them as one partial
 * line per request, which HBM handles at a fraction of its write rate:
 * profiles/r02/ubench_records.txt).  Records past num_headers are unspecified. */
enum rhp_layout {
  RHP_LAYOUT_REQUEST_MAJOR = 0,
  RHP_LAYOUT_HEADER_MAJOR = 1,
  RHP_LAYOUT_COMPACT = 2,     /* 4-byte header records, below (http mode: 8-byte http records too;
                                 not with RHP_BATCH_SPECULATIVE) */
  RHP_LAYOUT_DENSE = 3,       /* RHP_MODE_PHR: 8-byte request and 2-byte header records, below */
  RHP_LAYOUT_DENSE_RM = 4     /* the same, the header records request-major */
};
/* Compact records (RHP_LAYOUT_COMPACT).  A header line the DFA
 * parses is `name ": " value CRLF` and the first one starts right after the
 * request line `method SP path SP "HTTP/1." digit CRLF`, so its record is two
 * lengths: hdrs holds u32 lens[max_headers][n] (header-major), name_len |
 * value_len << 16, and the offsets follow by a running sum,
 *   name_off(0) = path_off + path_len + 11
 *   value_off(k) = name_off(k) + name_len(k) + 2
 *   name_off(k + 1) = value_off(k) + value_len(k) + 2.
 * A request whose flags hold RHP_F_WIDE (the exact path parsed it: leading
 * CRLF, OWS, obs-fold, bare LF, ...) has its records as rhp_hdr_t in the wide
 * area, wide[n][max_headers] (request-major) at byte RHP_COMPACT_WIDE_OFF(n, m)
 * of hdrs.  hdrs holds RHP_COMPACT_HDRS_BYTES(n, m) bytes; rhp_expand_records
 * (rhp_host.h) turns a batch's records into rhp_hdr_t on the host.  The
 * records a uniform batch writes shrink from 8 to 4 bytes per header (config
 * 2: 48 -> 32 B per request with the 16-B request record). */
#define RHP_COMPACT_WIDE_OFF(n, m) ((((size_t) (n) * (size_t) (m) * 4u) + 15u) & ~(size_t) 15u)
#define RHP_COMPACT_HDRS_BYTES(n, m) (RHP_COMPACT_WIDE_OFF(n, m) + (size_t) (n) * (size_t) (m) * 8u)
/* Dense records (RHP_LAYOUT_DENSE / RHP_LAYOUT_DENSE_RM, RHP_MODE_PHR; round
 * 6).  The compact layout's running-sum offsets with narrower fields, for the
 * DFA's records.  reqs holds rhp_req_dense_t dreq[n] (8 B) and, at byte
 * RHP_DENSE_REQ_WIDE_OFF(n), a wide area rhp_req_t wide[n]
 * (RHP_DENSE_REQS_BYTES(n) bytes in all).  hdrs holds u16 lens, name_len |
 * value_len << 6, at index k * n + i (RHP_LAYOUT_DENSE, header-major) or
 * i * m + k (RHP_LAYOUT_DENSE_RM, request-major); a header whose name is longer
 * than RHP_DENSE_NAME_MAX or value longer than RHP_DENSE_VALUE_MAX has
 * RHP_DENSE_OVERFLOW there and its u32 lengths, name_len | value_len << 16, at
 * the same index of the overflow area at byte RHP_DENSE_OVF_OFF(n, m); the wide
 * header records rhp_hdr_t wide[n][m] follow at RHP_DENSE_WIDE_OFF(n, m)
 * (RHP_DENSE_HDRS_BYTES(n, m) bytes in all).  A DFA request is dense when its
 * method is at most 255 bytes (path_off = method_len + 1, method_off = 0); any
 * other (and every request the exact path parses) is wide: dreq[i].flags holds
 * RHP_DENSE_WIDE, its records are wide[i] and the wide header records.
 * RHP_DENSE_BAD: ret = -1 (the other outputs unspecified, as in rhp_req_t).
 * Config 2 writes 8 + 4 x 2 = 16 B of records per request (compact: 32 B).
 * rhp_expand_reqs / rhp_expand_records (rhp_host.h) expand them on the host. */
typedef struct rhp_req_dense {
  uint16_t ret;           /* 1..65535 (the header section), when neither flag is set */
  uint16_t path_len;
  uint8_t  method_len;
  uint8_t  num_headers;
  uint8_t  minor_version;
  uint8_t  flags;         /* RHP_DENSE_WIDE, RHP_DENSE_BAD */
} rhp_req_dense_t;
#define RHP_DENSE_WIDE 1u
#define RHP_DENSE_BAD  2u
#define RHP_DENSE_NAME_MAX 62u    /* longest name a dense header record holds */
#define RHP_DENSE_VALUE_MAX 1007u /* longest value */
#define RHP_DENSE_REQ_WIDE_OFF(n) ((((size_t) (n) * 8u) + 15u) & ~(size_t) 15u)
#define RHP_DENSE_REQS_BYTES(n) (RHP_DENSE_REQ_WIDE_OFF(n) + (size_t) (n) * 16u)
#define RHP_DENSE_OVERFLOW 0xFFFFu
#define RHP_DENSE_OVF_OFF(n, m) ((((size_t) (n) * (size_t) (m) * 2u) + 15u) & ~(size_t) 15u)
#define RHP_DENSE_WIDE_OFF(n, m) (RHP_DENSE_OVF_OFF(n, m) + ((((size_t) (n) * (size_t) (m) * 4u) + 15u) & ~(size_t) 15u))
#define RHP_DENSE_HDRS_BYTES(n, m) (RHP_DENSE_WIDE_OFF(n, m) + (size_t) (n) * (size_t) (m) * 8u)

/* record k of request i in a batch of n requests with capacity m */
#define RHP_HDR(hdrs, layout, n, m, i, k) \
  ((hdrs)[(layout) == RHP_LAYOUT_HEADER_MAJOR ? (size_t) (k) * (n) + (i) : (size_t) (i) * (m) + (k)])

/* http_read_request result (24 B), RHP_MODE_HTTP only */
typedef struct rhp_http {
  int32_t  result;         /* 1 ready, 0 need more bytes / empty, -1 malformed, RHP_RET_TOOLONG */
  uint32_t body_kind;      /* 0: data_null(); 1: body = (req.ret, body_len);
                              RHP_BODY_CHUNKED_PENDING: a speculative batch's chunked body,
                              validated, not yet de-framed (rhp_fixup_sessions finishes it) */
  uint64_t consumed;       /* bytes stream_consume() is given (mod 2^64, http.c:216) */
  uint64_t body_len;
} rhp_http_t;

/* Compact http records (RHP_LAYOUT_COMPACT, RHP_MODE_HTTP): http holds
 * rhp_http_compact_t hc[n] (8 B) and, at byte RHP_COMPACT_HTTP_WIDE_OFF(n), a
 * wide area rhp_http_t wide[n]; RHP_COMPACT_HTTP_BYTES(n) bytes in all.  A
 * record without RHP_HTTP_WIDE holds result, body_kind and body_len, and
 * consumed = ret + (body_kind == 1 ? body_len : 0) for result 1, else 0 (the
 * DFA path's framing: no body, or a Content-Length body).  A record with
 * RHP_HTTP_WIDE (the exact path, a chunked body de-framed in place) is
 * wide[i].  rhp_expand_http (rhp_host.h) turns them into rhp_http_t.  With
 * the compact header records, a uniform batch writes 16 + 4 h + 8 bytes per
 * request (config 5: 40 B, was 16 + 8 h + 24 = 70 B header-major). */
typedef struct rhp_http_compact {
  int8_t   result;
  uint8_t  body_kind;
  uint8_t  flags;       /* RHP_HTTP_WIDE */
  uint8_t  reserved;
  uint32_t body_len;
} rhp_http_compact_t;
#define RHP_HTTP_WIDE 1u
#define RHP_COMPACT_HTTP_WIDE_OFF(n) ((((size_t) (n) * 8u) + 15u) & ~(size_t) 15u)
#define RHP_COMPACT_HTTP_BYTES(n) (RHP_COMPACT_HTTP_WIDE_OFF(n) + (size_t) (n) * 24u)

typedef struct rhp_batch {
  const uint8_t  *bytes;   /* device, 16-byte aligned: packed requests + RHP_PAD zero bytes */
  uint8_t        *bytes_rw;/* device, RHP_MODE_HTTP: same buffer, writable (chunked
                              bodies are de-framed in place, http.c:134-160; a request's
                              writes stay inside its own [offsets[i], offsets[i+1]), the
                              bytes around its body rewritten with their own values, so
                              the caller may fill other requests meanwhile); may be NULL
                              in RHP_MODE_PHR */
  const uint64_t *offsets; /* device: n + 1 offsets, non-decreasing */
  uint64_t        bytes_size; /* readable bytes at `bytes` (>= offsets[n] + RHP_PAD) */
  uint32_t        n;
  uint32_t        max_headers; /* headers capacity per request (*num_headers in) */
  uint32_t        mode;        /* enum rhp_mode */
  uint32_t        layout;      /* enum rhp_layout: where record k of request i lives in hdrs */
  rhp_req_t      *reqs;        /* device [n] (RHP_LAYOUT_DENSE: RHP_DENSE_REQS_BYTES(n) bytes,
                                  rhp_req_dense_t and the wide area) */
  rhp_hdr_t      *hdrs;        /* device [n * max_headers] records, laid out as `layout` says
                                  (n * max_headers < 2^32); RHP_LAYOUT_COMPACT:
                                  RHP_COMPACT_HDRS_BYTES(n, max_headers) bytes; RHP_LAYOUT_DENSE:
                                  RHP_DENSE_HDRS_BYTES(n, max_headers) bytes */
  rhp_http_t     *http;        /* device [n], RHP_MODE_HTTP (RHP_LAYOUT_COMPACT:
                                  RHP_COMPACT_HTTP_BYTES(n) bytes, rhp_http_compact_t) */
  uint32_t       *work;        /* reserved, may be NULL (device scratch of RHP_WORK_WORDS u32
                                  for future kernels; the current ones keep their scheduling
                                  state in LDS) */
  uint32_t        flags;       /* RHP_BATCH_* */
  uint32_t        reserved;
  const uint64_t *last_len;    /* device [n] or NULL (= all 0), RHP_MODE_PHR only:
                                  phr_parse_request's last_len per request
                                  (picohttpparser.c:383, 399-401): when last_len[i] != 0 the
                                  slowloris pre-check is_complete (:197-223) runs first and
                                  its -2 / -1 is the answer.  Contract: last_len[i] <= len
                                  (the reference reads before `buf_end` only then) */
} rhp_batch_t;

#define RHP_WORK_WORDS 64u
#define RHP_BODY_CHUNKED_PENDING 2u

/* rhp_batch_t.flags */
#define RHP_BATCH_SPECULATIVE 1u   /* RHP_MODE_HTTP: the requests may be speculative pieces of
                                      pipelined input (rhp_fixup_sessions below): nothing is
                                      written to bytes_rw (chunked bodies are validated and
                                      left framed, body_kind RHP_BODY_CHUNKED_PENDING) */

/* Parse a batch on `stream` (hipStream_t) of the calling thread's current
 * device.  Returns 0 on successful launch, a negative errno-style code for bad
 * arguments, or a positive hipError_t.  Thread-safe: one host thread per GPU
 * may call it concurrently (per-device state is cached per device id). */
int rhp_parse_batch(const rhp_batch_t *batch, void *stream);

/*
 * Pipelined input (the reference's server_session_read loop,
 * /root/reference/src/reactor/server.c:37-65, advancing by http.c:200, 216, 232).
 * A session's unconsumed input is split by the caller at every empty line (the
 * end of a header section: LF LF or LF CR LF) into pieces that are consecutive
 * requests of a RHP_BATCH_SPECULATIVE http batch, so every request's header
 * section ends a piece (#pieces >= #requests).  After rhp_parse_batch,
 * rhp_fixup_sessions walks each session in order, as http_read_request would be
 * called in a loop over the whole input: a piece that starts at the next request
 * boundary and whose result cannot change with more input (1 within the piece,
 * -1, RHP_RET_TOOLONG, or 0 for the session's last piece) is taken (a pending
 * chunked body is de-framed in place now); anything else (a body that ran past
 * its piece, a piece that started inside a body) is parsed again from the true
 * boundary over the rest of the session's input.  Request m of a session is
 * left in record slot piece_lo + m (reqs/hdrs/http of the batch), its start
 * in req_start[piece_lo + m].  One launch, one thread per session.  Any split
 * gives the reference's answers: with a coarser one (a piece holding several
 * requests) a piece whose records an earlier request of the walk has already
 * overwritten is parsed again from its boundary, and a session with more
 * requests than pieces stops with `more`.
 */
typedef struct rhp_session {
  uint32_t piece_lo, piece_hi;   /* the session's pieces: requests [piece_lo, piece_hi) of the
                                    batch, its bytes [offsets[piece_lo], offsets[piece_hi]) */
} rhp_session_t;

typedef struct rhp_session_result {
  uint32_t n_slots;   /* record slots filled: every one but the last has result 1; the last
                         one's result says where the session stopped (1: input used up) */
  uint32_t more;      /* 1: more requests than pieces (a coarser split than one per empty
                         line): the rest from offsets[piece_lo] + consumed needs another batch */
  uint64_t consumed;  /* bytes of the session's input taken by its result-1 requests */
} rhp_session_result_t;

/* Launch status as rhp_parse_batch.  `batch` is the speculative batch already
 * parsed on `stream`; sessions, results and req_start (u64 [n]) are device
 * memory. */
int rhp_fixup_sessions(const rhp_batch_t *batch, const rhp_session_t *sessions, uint32_t n_sessions,
                       rhp_session_result_t *results, uint64_t *req_start, void *stream);

/* Dense copies of a parsed http batch's records (round 6: what the reactor
 * copies back to the host, reactor/batch.c).  For each record slot i of a
 * RHP_MODE_HTTP batch in RHP_LAYOUT_REQUEST_MAJOR (speculative or not), after
 * the parse (and rhp_fixup_sessions, when used): the request record as
 * rhp_req_dense_t dreq[i], the http record as rhp_http_compact_t hc[i] and the
 * header lengths as u16 lens16[k * n + i], k < num_headers, in
 * RHP_LAYOUT_DENSE's encodings (a record whose consumed follows from ret and
 * body_len; a request whose http record is such a record and whose offsets
 * follow the running sum with names of at most RHP_DENSE_NAME_MAX and values of
 * at most RHP_DENSE_VALUE_MAX bytes -- a de-framed chunked body moves its
 * request's bytes, so that request stays wide).
 * Any other slot is marked RHP_HTTP_WIDE / RHP_DENSE_WIDE: its records are the
 * batch's own.  Device pointers; launch status as rhp_parse_batch. */
int rhp_pack_dense(const rhp_batch_t *batch, rhp_req_dense_t *dreq, rhp_http_compact_t *hc, uint16_t *lens16,
                   void *stream);

/* Which kernel implementation rhp_parse_batch uses (diagnostics / A-B tests). */
enum rhp_impl {
  RHP_IMPL_DFA = 0,    /* lane-per-request byte DFA with LDS tables (default) */
  RHP_IMPL_EXACT = 1,  /* lane-per-request exact scalar path only (slow reference path) */
  RHP_IMPL_DFA_LATE = 2 /* the DFA kernel in its late-issue form in both modes (the default
                           uses that form in RHP_MODE_HTTP only) */
};
int rhp_set_impl(int impl);   /* per calling thread */

/* Name of the kernel symbol the default implementation launches (for profiles). */
const char *rhp_kernel_name(void);

/* Library version string. */
const char *rhp_version(void);

/*
 * Batched response serialization: http_write_response (src/reactor/http.c:236-297,
 * decl http.h:37) for n responses at once, on the device.  Response i is written to
 * out[out_off[i], out_off[i+1]) byte for byte as the reference appends it to the
 * stream's output:
 *   "HTTP/1.1 " status CRLF "Server: *" CRLF "Date: " date CRLF
 *   "Content-Type: " type CRLF "Content-Length: " decimal(body_len) CRLF
 *   { name ": " value CRLF }  CRLF body
 * Every string of a response is a span of the device `arena`.  The date is one
 * 29-byte IMF-fixdate for the batch (the reactor's cached date; http.c:244 sizes
 * the response for exactly 29 date bytes, so other lengths are rejected).
 */
typedef struct rhp_span {
  uint32_t off, len;         /* bytes arena[off, off + len) */
} rhp_span_t;

typedef struct rhp_resp {
  rhp_span_t status;         /* e.g. "200 OK" */
  rhp_span_t type;           /* Content-Type value */
  rhp_span_t body;
  uint32_t   fields_first;   /* extra fields: fields[fields_first .. + fields_count) */
  uint32_t   fields_count;
} rhp_resp_t;

typedef struct rhp_resp_field {
  rhp_span_t name, value;
} rhp_resp_field_t;

#define RHP_DATE_LEN 29u

typedef struct rhp_resp_batch {
  const uint8_t          *arena;    /* device */
  const rhp_resp_t       *resps;    /* device [n] */
  const rhp_resp_field_t *fields;   /* device, may be NULL when no response has fields */
  uint32_t                n;
  uint32_t                date_len; /* must be RHP_DATE_LEN */
  const char             *date;     /* host, date_len bytes */
  uint64_t               *out_off;  /* device [n + 1]: written (exclusive prefix sum of sizes) */
  uint8_t                *out;      /* device, out_size bytes */
  uint64_t                out_size; /* when out_off[n] > out_size nothing is written to `out`
                                       (out_off still holds every size: grow and call again) */
  uint64_t               *work;     /* device scratch, >= RHP_RESP_WORK_WORDS(n) u64 */
} rhp_resp_batch_t;

#define RHP_RESP_WORK_WORDS(n) (((uint64_t) (n) + 4095u) / 4096u + 1u)

/* Launch status as rhp_parse_batch; four kernels on `stream` (sizes with tile
 * sums, two scan passes, copy). */
int rhp_write_responses(const rhp_resp_batch_t *batch, void *stream);


#ifdef __cplusplus
}
#endif
#endif
