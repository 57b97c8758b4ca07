/*
 * rhp_scalar.h -- exact scalar request parser, compiled for host and device.
 *
 * The DFA kernel (rhp_kernel.hip) hands a request to this path when its fast
 * table cannot decide it alone: the buffer ends before the request completes
 * (end-of-buffer semantics, including the past-the-end SP skips at
 * picohttpparser.c:356-362), obs-fold lines, an empty method, a bad version,
 * non-GET framing in http mode, requests longer than the DFA's capture area.
 * It is the executable form of the semantics the DFA table is derived from.
 *
 * Semantics followed (all /root/reference/...):
 *   phr_parse_request  src/picohttpparser/picohttpparser.c:71-94,134-195,245-409
 *   http_read_request  src/reactor/http.c:73-160,167-234; memcasecmp data.c:11-28
 */
#ifndef RHP_SCALAR_H
#define RHP_SCALAR_H

#include <stdint.h>
#include "rhp.h"

#if defined(__HIPCC__)
#define RHP_HD __host__ __device__ __forceinline__
#define RHP_HDM __host__ __device__ __forceinline__
#else
#define RHP_HD static inline
#define RHP_HDM inline
#endif

namespace rhp {

enum : int { kBad = -1, kPartial = -2 };

RHP_HD bool is_tchar(uint32_t c)
{
  /* token_char_map (picohttpparser.c:96-103) as two 64-bit row masks */
  const uint64_t lo = 0x03ff6cfa00000000ull;  /* 0x00-0x3f: ! # $ % & ' * + - . 0-9 */
  const uint64_t hi = 0x57ffffffc7fffffeull;  /* 0x40-0x7f: A-Z ^ _ ` a-z | ~ */
  if (c >= 128) return false;
  return ((c < 64 ? lo : hi) >> (c & 63)) & 1u;
}
RHP_HD bool is_ctl_del(uint32_t c) { return c < 0x20u || c == 0x7fu; }
RHP_HD bool is_ows(uint32_t c) { return c == ' ' || c == '\t'; }

/* Byte access for the exact parser.  PlainBytes indexes memory directly
 * (host); the GPU replay uses a reader that caches the aligned 16-byte line
 * holding the last byte read, so a sequential scan costs one global load per
 * 16 bytes instead of one dependent load per byte. */
struct PlainBytes {
  const uint8_t *b;
  RHP_HDM uint32_t operator()(uint64_t p) const { return b[p]; }
};

/* Where the exact parser puts its answer (the same parse, two encodings).
 *   OutRec  the batch records of rhp.h: offsets from the request start as u16.
 *           A header section longer than RHP_MAX_LEN (phr ret > 65535) cannot
 *           be encoded and gives RHP_RET_TOOLONG; every other answer (-1, -2,
 *           or a ret that fits) is the reference's, whatever the buffer length.
 *   OutPhr  (host, rhp_emu.cpp) phr_parse_request's own outputs: pointers into
 *           the buffer and size_t lengths, no limit (picohttpparser.h:51-52). */
struct OutRec {
  rhp_req_t *r;
  rhp_hdr_t *h;        /* record k at h[k * hs] (the batch's header-major layout: hs = n) */
  uint64_t hs;
  RHP_HDM void begin()
  {
    r->method_off = 0; r->method_len = 0; r->path_off = 0; r->path_len = 0;
    r->minor_version = -1; r->num_headers = 0;
  }
  RHP_HDM int fail(int code) { r->ret = code; return code; }
  RHP_HDM void header(uint32_t n, bool fold, uint64_t name, uint64_t name_len, uint64_t vs, uint64_t vlen)
  {
    rhp_hdr_t &o = h[n * hs];
    o.name_off = fold ? (uint16_t) RHP_NAME_NULL : (uint16_t) name;
    o.name_len = (uint16_t) name_len;
    o.value_off = (uint16_t) vs;
    o.value_len = (uint16_t) vlen;
  }
  RHP_HDM int done(uint64_t p, const uint64_t (&tok)[2][2], int minor, uint32_t n)
  {
    if (p > RHP_MAX_LEN) return fail(RHP_RET_TOOLONG);   /* u16 records cannot hold it */
    r->method_off = (uint8_t) tok[0][0];
    r->method_len = (uint16_t) (tok[0][1] - tok[0][0]);
    r->path_off = (uint16_t) tok[1][0];
    r->path_len = (uint16_t) (tok[1][1] - tok[1][0]);
    r->minor_version = (int8_t) minor;
    r->num_headers = (uint16_t) n;
    r->ret = (int32_t) p;
    return r->ret;
  }
};

/* Parse one request (parse_request, picohttpparser.c:341-381).  b may be read
 * beyond len (batch contract).  Headers go to out.header(0 .. max-1).  Returns
 * the phr status (or RHP_RET_TOOLONG from OutRec). */
template <class Bytes, class Out>
RHP_HD int scalar_phr_t(Bytes &B, uint64_t len, uint32_t max, Out &out)
{
  uint64_t p = 0;
  out.begin();
#define RHP_FAIL(code) do { return out.fail(code); } while (0)
#define RHP_EOF() do { if (p == len) RHP_FAIL(kPartial); } while (0)
#define RHP_CRLF() do { ++p; RHP_EOF(); if (B(p++) != '\n') RHP_FAIL(kBad); } while (0)
  RHP_EOF();
  if (B(p) == '\r') RHP_CRLF();
  else if (B(p) == '\n') ++p;

  uint64_t tok[2][2];              /* [method, path][start, end] */
  for (int t = 0; t < 2; t++) {
    tok[t][0] = p;
    RHP_EOF();
    for (;;) {
      uint32_t c = B(p);
      if (c == ' ') break;
      if (is_ctl_del(c)) RHP_FAIL(kBad);
      ++p;
      RHP_EOF();
    }
    tok[t][1] = p;
    do ++p; while (B(p) == ' ');   /* no EOF test: may run past len */
  }
  if (tok[0][1] == tok[0][0] || tok[1][1] == tok[1][0]) RHP_FAIL(kBad);
  if ((int64_t) len - (int64_t) p < 9) RHP_FAIL(kPartial);
  if (B(p) != 'H' || B(p + 1) != 'T' || B(p + 2) != 'T' || B(p + 3) != 'P' || B(p + 4) != '/' ||
      B(p + 5) != '1' || B(p + 6) != '.' || B(p + 7) - '0' > 9u)
    RHP_FAIL(kBad);
  int minor = (int) B(p + 7) - '0';
  p += 8;
  if (B(p) == '\r') RHP_CRLF();
  else if (B(p) == '\n') ++p;
  else RHP_FAIL(kBad);

  uint32_t n = 0;
  for (;;) {
    RHP_EOF();
    if (B(p) == '\r') { RHP_CRLF(); break; }
    if (B(p) == '\n') { ++p; break; }
    if (n == max) RHP_FAIL(kBad);
    uint64_t name = p, name_len = 0;
    bool fold = n != 0 && is_ows(B(p));
    if (!fold) {
      for (;;) {
        uint32_t c = B(p);
        if (c == ':') break;
        if (!is_tchar(c)) RHP_FAIL(kBad);
        ++p;
        RHP_EOF();
      }
      name_len = p - name;
      if (name_len == 0) RHP_FAIL(kBad);
      ++p;
      for (;; ++p) {
        RHP_EOF();
        if (!is_ows(B(p))) break;
      }
    }
    uint64_t vs = p;
    uint32_t c;
    for (;; ++p) {
      RHP_EOF();
      c = B(p);
      if ((c < 0x20u && c != '\t') || c == 0x7fu) break;
    }
    uint64_t ve = p;
    if (c == '\r') RHP_CRLF();
    else if (c == '\n') ++p;
    else RHP_FAIL(kBad);
    while (ve > vs && is_ows(B(ve - 1))) --ve;
    out.header(n, fold, name, name_len, vs, ve - vs);
    ++n;
  }
#undef RHP_CRLF
#undef RHP_EOF
#undef RHP_FAIL
  return out.done(p, tok, minor, n);
}

template <class Bytes>
RHP_HD int scalar_phr_t(Bytes &B, uint64_t len, uint32_t max, rhp_req_t *r, rhp_hdr_t *h, uint64_t hs)
{
  OutRec o{r, h, hs};
  return scalar_phr_t(B, len, max, o);
}

RHP_HD int scalar_phr(const uint8_t *b, uint64_t len, uint32_t max, rhp_req_t *r, rhp_hdr_t *h, uint64_t hs)
{
  PlainBytes B{b};
  return scalar_phr_t(B, len, max, r, h, hs);
}

/* is_complete (picohttpparser.c:197-223), the slowloris pre-check that
 * phr_parse_request runs first when last_len != 0 (:399-401): 0 when an empty
 * line ends the bytes seen (scanning from last_len - 3), else -2 / -1. */
template <class Bytes>
RHP_HD int is_complete_t(Bytes &B, uint64_t len, uint64_t last_len)
{
  uint64_t p = last_len < 3 ? 0 : last_len - 3;
  int ret_cnt = 0;
  for (;;) {
    if (p >= len) return kPartial;   /* CHECK_EOF; p > len only when last_len > len + 3 (off contract) */
    const uint32_t c = B(p);
    if (c == '\r') {
      ++p;
      if (p == len) return kPartial;
      if (B(p++) != '\n') return kBad;
      ++ret_cnt;
    } else if (c == '\n') {
      ++p;
      ++ret_cnt;
    } else {
      ++p;
      ret_cnt = 0;
    }
    if (ret_cnt == 2) return 0;
  }
}

RHP_HD int is_complete(const uint8_t *b, uint64_t len, uint64_t last_len)
{
  PlainBytes B{b};
  return is_complete_t(B, len, last_len);
}

/* ---- http_read_request framing (http.c:177-234) over a parsed request ---- */

RHP_HD uint32_t upper(uint32_t c) { return (c - 'a' < 26u) ? c - 32u : c; }

/* Header views for the framing: HdrsRec reads the batch records (offsets from
 * the request start b), a host view (rhp_emu.cpp) reads phr_header pointers. */
struct HdrsRec {
  const uint8_t *b;
  const rhp_hdr_t *h;
  uint64_t hs;         /* record i at h[i * hs] */
  RHP_HDM bool null(uint32_t i) const { return h[i * hs].name_off == RHP_NAME_NULL; }
  RHP_HDM const uint8_t *name(uint32_t i) const { return b + h[i * hs].name_off; }
  RHP_HDM uint64_t name_len(uint32_t i) const { return h[i * hs].name_len; }
  RHP_HDM const uint8_t *value(uint32_t i) const { return b + h[i * hs].value_off; }
  RHP_HDM uint64_t value_len(uint32_t i) const { return h[i * hs].value_len; }
};

/* Case-insensitive name compare.  All n bytes are read before any is tested
 * (no early exit), so on the GPU replay path they are independent loads: one
 * memory round trip instead of n dependent ones. */
template <class HV>
RHP_HD bool name_eq(const HV &hv, uint32_t i, const char *name, uint32_t n)
{
  if (hv.null(i) || hv.name_len(i) != n) return false;
  const uint8_t *s = hv.name(i);
  uint32_t diff = 0;
  for (uint32_t k = 0; k < n; k++) diff |= upper(s[k]) ^ upper((uint8_t) name[k]);
  return diff == 0;
}

/* strtoull(s, NULL, 10), glibc C locale (saturating, sign-negated), as a
 * state machine over bytes: 0 leading space, 1 digits (after an optional
 * sign), 2 done. */
RHP_HD void num_step(uint32_t c, uint32_t &st, bool &neg, bool &ovf, uint64_t &v)
{
  const bool digit = c - '0' < 10u;
  if (st == 0) {
    if (c == ' ' || c - '\t' < 5u) return;
    if (c == '+' || c == '-') { neg = c == '-'; st = 1; return; }
    st = digit ? 1u : 2u;
  } else if (st == 1 && !digit) {
    st = 2;
  }
  if (st != 1 || !digit) return;
  const uint64_t d = c - '0';
  /* v * 10 + d > 2^64 - 1  <=>  v > 1844674407370955161, or v equal to it and d > 5 */
  ovf |= v > 1844674407370955161ull || (v == 1844674407370955161ull && d > 5u);
  v = v * 10 + d;
}

/* strtoull over a header value of n bytes.  Reading stops at the value's end:
 * a parsed value starts with a byte that is neither OWS nor a CTL, so the
 * leading-space skip ends inside it, and the byte after it (trimmed OWS, CR or
 * LF) is no digit -- the same answer as strtoull running on past it.  The first
 * kNumWindow bytes are read up front (independent loads on the GPU replay). */
RHP_HD uint64_t strtoull10(const uint8_t *s, uint64_t n)
{
  constexpr int kNumWindow = 24;
  uint32_t w[kNumWindow];
  for (int i = 0; i < kNumWindow; i++) w[i] = (uint64_t) i < n ? s[i] : 0u;
  uint32_t st = 0;
  bool neg = false, ovf = false;
  uint64_t v = 0;
  for (int i = 0; i < kNumWindow; i++) num_step(w[i], st, neg, ovf, v);
  for (uint64_t i = kNumWindow; st != 2 && i < n; i++) num_step(s[i], st, neg, ovf, v);
  return ovf ? ~0ull : neg ? 0 - v : v;
}

RHP_HD int hexval(uint32_t c)
{
  if (c - '0' < 10u) return (int) (c - '0');
  if ((c | 0x20u) - 'a' < 6u) return (int) ((c | 0x20u) - 'a' + 10);
  return -1;
}

/* http_chunk_size + http_chunk (http.c:73-132) for the chunk whose size line
 * starts at byte `at` of a body of `size` bytes, read through B (B(p) = body
 * byte p): >0 bytes of this chunk (size line + data + 2), 0 need more, -1
 * malformed; *data_off (from `at`) / *data_len.  Only the size line is read:
 * the data bytes are skipped, and the reads stop at the line's LF. */
template <class Bytes>
RHP_HD int64_t one_chunk_t(Bytes &B, uint64_t at, uint64_t size, uint64_t *data_off, uint64_t *data_len)
{
  const uint64_t avail = size - at;
  uint64_t nl = 0;
  while (nl < avail && B(at + nl) != '\n') nl++;   /* memchr(input, '\n') */
  if (nl == avail) return 0;                      /* no '\n' yet */
  uint64_t p = at;
  while (is_ows(B(p))) p++;
  const uint64_t digits = p;
  while (hexval(B(p)) >= 0) p++;
  if (p == digits) return -1;
  const uint64_t digits_end = p;
  while (is_ows(B(p))) p++;
  if (B(p) == ';') {
    p = at + nl;                                   /* while (*p != '\n') p++ */
    if (B(p - 1) != '\r') return -1;
  } else {
    if (B(p) != '\r') return -1;
    p++;
  }
  if (B(p) != '\n') return -1;
  p++;
  uint64_t cs = 0;
  bool ovf = false;
  for (uint64_t q = digits; q < digits_end; q++) {
    ovf |= (cs >> 60) != 0;
    cs = (cs << 4) | (uint64_t) hexval(B(q));
  }
  if (ovf || cs == ~0ull) return -1;             /* strtoul == ULONG_MAX */
  const uint64_t n = p - at;
  if (n + 2 > avail) return 0;
  if (cs > avail - n - 2) return 0;
  *data_off = n;
  *data_len = cs;
  return (int64_t) (cs + n + 2);
}

/* one_chunk_t from a window W holding the `nw` (<= 32) bytes at `at` (little-
 * endian dwords; bytes past the buffer's end zero -- the batch is padded), one
 * pass over the size line as a state machine: the GPU replay loads the window
 * in one memory round trip where one_chunk_t's line cache takes one per line,
 * and twice when its LF search crosses a line.  Returns false when the window
 * cannot decide (no LF in it and more than nw bytes available); otherwise *res
 * and the data span are one_chunk_t's. */
RHP_HD bool one_chunk_window(const uint32_t (&W)[8], uint32_t nw, uint64_t avail, int64_t *res, uint64_t *data_off,
                             uint64_t *data_len)
{
  enum : uint32_t { kLead, kHex, kTrail, kExt, kCr, kErr };
  uint32_t st = kLead, nl = 32;
  bool prev_cr = false, ovf = false;
  uint64_t cs = 0;
  for (uint32_t j = 0; j < 32; j++) {
    if (j >= nw) break;
    const uint32_t c = (W[j >> 2] >> (8 * (j & 3))) & 0xffu;
    if (c == '\n') {   /* memchr's LF */
      nl = j;
      break;
    }
    const bool ows = is_ows(c);
    const uint32_t dg = c - '0', al = (c | 0x20u) - 'a';
    const bool hex = dg < 10u || al < 6u;
    if ((st == kLead || st == kHex) && hex) {
      ovf |= (cs >> 60) != 0;
      cs = (cs << 4) | (uint64_t) (dg < 10u ? dg : al + 10u);
      st = kHex;
    } else if (st == kLead) {
      st = ows ? kLead : kErr;   /* no digit before this byte: -1 */
    } else if (st == kHex || st == kTrail) {
      st = ows ? kTrail : c == ';' ? kExt : c == '\r' ? kCr : kErr;
    } else if (st == kCr) {
      st = kErr;                 /* CR not followed by LF */
    }
    prev_cr = c == '\r';
  }
  if (nl == 32 && avail > nw) return false;
  if (nl >= avail) {   /* no LF within the body yet */
    *res = 0;
    return true;
  }
  if (!(st == kCr || (st == kExt && prev_cr)) || ovf || cs == ~0ull) {
    *res = -1;
    return true;
  }
  const uint64_t n = nl + 1;
  if (n + 2 > avail || cs > avail - n - 2) {
    *res = 0;
    return true;
  }
  *data_off = n;
  *data_len = cs;
  *res = (int64_t) (cs + n + 2);
  return true;
}

/* one_chunk_window's answer for the common size line, without its byte loop's
 * branches (round 6, the GPU replay's size-line walk): the LF found by a
 * zero-byte test on the window's first ND dwords (nw <= 4 * ND), the state
 * machine run over the first 8 bytes only, every byte under a predicate.  A
 * line whose state is decided by its 8th byte -- an extension or its CR
 * reached, or an error --, or whose LF comes earlier, is answered here with
 * one_chunk_window's result; anything else (a longer run of OWS or hex digits)
 * returns false and the caller runs one_chunk_window.  At most 8 digits are
 * read, so the size fits 32 bits and never overflows. */
template <uint32_t ND>
RHP_HD bool one_chunk_head(const uint32_t (&W)[8], uint32_t nw, uint64_t avail, int64_t *res, uint64_t *data_off,
                           uint64_t *data_len)
{
  enum : uint32_t { kLead, kHex, kTrail, kExt, kCr, kErr };
  uint32_t nl = 32;   /* the first LF among the window's bytes, 32: none */
#pragma unroll
  for (int q = (int) ND - 1; q >= 0; q--) {   /* the lowest dword with an LF wins; the first zero byte is exact */
    const uint32_t t = W[q] ^ 0x0a0a0a0au;
    const uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;
    nl = z ? 4u * (uint32_t) q + ((uint32_t) __builtin_ctz(z) >> 3) : nl;
  }
  nl = nl < nw ? nl : 32u;
  if (nl == 32 && avail > nw) return false;
  if (nl >= avail) {   /* no LF within the body yet */
    *res = 0;
    return true;
  }
  uint32_t st = kLead, cs = 0;
  bool prev_cr = false;
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {
    const uint32_t c = (W[j >> 2] >> (8 * (j & 3))) & 0xffu;
    const bool live = j < nl;
    const bool ows = is_ows(c);
    const uint32_t dg = c - '0', al = (c | 0x20u) - 'a';
    const bool hex = dg < 10u || al < 6u;
    const bool dig = st <= kHex && hex;
    const uint32_t nst = dig ? kHex
                         : st == kLead ? (ows ? kLead : kErr)
                         : (st == kHex || st == kTrail) ? (ows ? kTrail : c == ';' ? kExt : c == '\r' ? kCr : kErr)
                         : st == kCr ? kErr : st;
    cs = live && dig ? (cs << 4) | (dg < 10u ? dg : al + 10u) : cs;
    st = live ? nst : st;
    prev_cr = live ? c == '\r' : prev_cr;
  }
  if (nl > 8) {   /* bytes 8 .. nl - 1 not run */
    if (st <= kTrail) return false;   /* OWS / digits / OWS still running: one_chunk_window decides */
    if (st == kCr) st = kErr;          /* byte 8 follows the CR: not its LF */
    const uint32_t b = nl - 1;         /* an extension: what counts is the byte before the LF */
    uint32_t wd = W[0];
#pragma unroll
    for (uint32_t q = 1; q < ND; q++) wd = (b >> 2) == q ? W[q] : wd;
    prev_cr = ((wd >> (8 * (b & 3))) & 0xffu) == '\r';
  }
  if (!(st == kCr || (st == kExt && prev_cr))) {
    *res = -1;
    return true;
  }
  const uint64_t n = nl + 1;
  if (n + 2 > avail || cs > avail - n - 2) {
    *res = 0;
    return true;
  }
  *data_off = n;
  *data_len = cs;
  *res = (int64_t) (cs + n + 2);
  return true;
}

/* http_dechunk (http.c:134-160): validate every chunk, then move the payloads
 * down in place, chunk by chunk (dst <= src: the compacted body never passes
 * the next size line).  B reads the body (B(p) = body byte p), move(dst, src, n)
 * copies n body bytes forward.  compact = false (speculative batches, rhp.h
 * RHP_BATCH_SPECULATIVE): validate only and report the payload length; nothing
 * is written. */
template <class Bytes, class Move>
RHP_HD int64_t dechunk_t(Bytes &B, Move &move, uint64_t size, uint64_t *body_len, bool compact)
{
  uint64_t off = 0, doff = 0, dlen = 0, sum = 0;
  do {
    int64_t n = one_chunk_t(B, off, size, &doff, &dlen);
    if (n <= 0) return n;
    off += (uint64_t) n;
    sum += dlen;
  } while (dlen);
  if (!compact) {
    *body_len = sum;
    return (int64_t) off;
  }
  uint64_t total = 0;
  off = 0;
  do {
    int64_t n = one_chunk_t(B, off, size, &doff, &dlen);
    move(total, off + doff, dlen);
    off += (uint64_t) n;
    total += dlen;
  } while (dlen);
  *body_len = total;
  return (int64_t) off;
}

/* the byte-wise form (host) */
struct PlainMove {
  uint8_t *in;
  RHP_HDM void operator()(uint64_t dst, uint64_t src, uint64_t n) const
  {
    for (uint64_t i = 0; i < n; i++) in[dst + i] = in[src + i];   /* dst <= src: forward copy */
  }
};
RHP_HD int64_t dechunk(uint8_t *in, uint64_t size, uint64_t *body_len, bool compact = true)
{
  PlainBytes B{in};
  PlainMove M{in};
  return dechunk_t(B, M, size, body_len, compact);
}

/* http_dechunk over the body at `in` (size bytes).  Plain: the byte-wise form;
 * the GPU passes its own (line-cached size-line reads, 16-byte moves). */
struct PlainDechunk {
  RHP_HDM int64_t operator()(uint8_t *in, uint64_t size, uint64_t *body_len, bool compact) const
  {
    return dechunk(in, size, body_len, compact);
  }
};

/* Framing decision given a successful phr parse (n = ret > 0) of a request of
 * len bytes at b: get = the method is "GET"; hv / nh = its headers.
 * cand: the header indices whose name could be Transfer-Encoding or
 * Content-Length (name length 17 or 14), as found by the kernel's decode; ~0
 * checks every header */
template <class HV, class DC = PlainDechunk>
RHP_HD void http_frame_t(uint8_t *b, uint64_t len, int64_t n, bool get, const HV &hv, uint32_t nh, rhp_http_t *x,
                         uint64_t cand = ~0ull, bool compact = true, const DC &dc = DC())
{
  /* one framing candidate (the common case): its name is read together with
   * its value digits, so the GPU replay makes fewer memory round trips */
  const bool one = cand != 0 && (cand & (cand - 1)) == 0;
  const uint32_t c = one ? (uint32_t) __builtin_ctzll(cand) : 0u;
  x->result = 1; x->body_kind = 0; x->consumed = (uint64_t) n; x->body_len = 0;
  if (get) return;                                /* GET fast path (http.c:198-202) */
  int te = -1, cl = -1;
  uint64_t size = 0;
  if (one) {
    if (c < nh) {
      const uint64_t vl = hv.value_len(c);
      size = vl ? strtoull10(hv.value(c), vl) : 0;   /* used only if the name is Content-Length */
      if (name_eq(hv, c, "Transfer-Encoding", 17)) te = (int) c;
      if (name_eq(hv, c, "Content-Length", 14)) cl = (int) c;
    }
  } else {
    for (uint32_t i = 0; i < nh; i++) {
      if (i < 64 && !((cand >> i) & 1u)) continue;
      if (te < 0 && name_eq(hv, i, "Transfer-Encoding", 17)) te = (int) i;
      if (cl < 0 && name_eq(hv, i, "Content-Length", 14)) cl = (int) i;
    }
    if (cl >= 0 && hv.value_len((uint32_t) cl) != 0) size = strtoull10(hv.value((uint32_t) cl), hv.value_len((uint32_t) cl));
  }
  const bool te_set = te >= 0 && hv.value_len((uint32_t) te) != 0;
  const bool cl_set = cl >= 0 && hv.value_len((uint32_t) cl) != 0;
  if (cl_set) {
    if (te_set) { x->result = -1; x->consumed = 0; return; }
    if (len < (uint64_t) n + size) { x->result = 0; x->consumed = 0; return; }
    x->body_kind = 1; x->body_len = size; x->consumed = (uint64_t) n + size;
    return;
  }
  if (te_set) {
    const char *ch = "CHUNKED";
    const uint8_t *v = hv.value((uint32_t) te);
    const uint64_t vl = hv.value_len((uint32_t) te);
    bool eq = vl == 7u;
    for (uint32_t i = 0; eq && i < 7; i++) eq = upper(v[i]) == (uint32_t) ch[i];
    if (!eq) { x->result = -1; x->consumed = 0; return; }
    uint64_t blen = 0;
    int64_t size = dc(b + n, len - (uint64_t) n, &blen, compact);
    if (size <= 0) { x->result = (int32_t) size; x->consumed = 0; return; }
    x->body_kind = compact ? 1u : RHP_BODY_CHUNKED_PENDING;
    x->body_len = blen; x->consumed = (uint64_t) n + (uint64_t) size;
  }
}

template <class DC = PlainDechunk>
RHP_HD void http_frame(uint8_t *b, uint64_t len, const rhp_req_t &r, const rhp_hdr_t *h, uint64_t hs, rhp_http_t *x,
                       uint64_t cand = ~0ull, bool compact = true, const DC &dc = DC())
{
  const bool get = r.method_len == 3 && ((b[r.method_off] == 'G') & (b[r.method_off + 1] == 'E') & (b[r.method_off + 2] == 'T'));
  http_frame_t(b, len, r.ret, get, HdrsRec{b, h, hs}, r.num_headers, x, cand, compact, dc);
}

/* phr status -> http_read_request result when the parse gave no request
 * (http.c:194-195); RHP_RET_TOOLONG (records cannot hold the request) is passed
 * on for the caller to parse it with a pointer-based parser */
RHP_HD int32_t http_result_of(int n) { return n == kBad ? -1 : n == RHP_RET_TOOLONG ? RHP_RET_TOOLONG : 0; }

/* Whole http_read_request for one request. */
template <class Bytes, class DC = PlainDechunk>
RHP_HD void scalar_http_t(Bytes &B, uint8_t *b, uint64_t len, uint32_t max, rhp_req_t *r, rhp_hdr_t *h, uint64_t hs,
                          rhp_http_t *x, bool compact = true, const DC &dc = DC())
{
  int n = scalar_phr_t(B, len, max, r, h, hs);
  x->body_kind = 0; x->consumed = 0; x->body_len = 0;
  if (len == 0) { x->result = 0; return; }
  if (n <= 0) { x->result = http_result_of(n); return; }
  http_frame(b, len, *r, h, hs, x, ~0ull, compact, dc);
}
RHP_HD void scalar_http(uint8_t *b, uint64_t len, uint32_t max, rhp_req_t *r, rhp_hdr_t *h, uint64_t hs, rhp_http_t *x)
{
  PlainBytes B{b};
  scalar_http_t(B, b, len, max, r, h, hs, x);
}

/* rhp_fixup_sessions (rhp.h) for one session: the pieces' speculative
 * results are taken where they are what http_read_request over the rest of
 * the input would return, and the rest is parsed again from the true request
 * boundaries; `mk(at)` gives a byte reader for the batch bytes at `at`.  The
 * loop is the reference's server_session_read (server.c:37-65): one
 * http_read_request per request, advancing by what it consumed. */
struct FixupIO {
  uint8_t *bytes_rw;
  const uint64_t *off;
  rhp_req_t *reqs;
  rhp_hdr_t *hdrs;
  rhp_http_t *http;
  uint64_t hs_req, hs_hdr;   /* record k of request i at hdrs[i * hs_req + k * hs_hdr] */
  uint32_t max_headers;
};

/* p_from (>= p_lo): the walk resumes at piece p_from, every piece before it
 * having been taken as it is (a whole-piece request whose records stay in
 * their slot and whose start req_start already holds) */
template <class MakeBytes, class DC = PlainDechunk>
RHP_HD void fixup_session_t(const FixupIO &io, uint32_t p_lo, uint32_t p_hi, uint64_t *req_start,
                            rhp_session_result_t *out, MakeBytes mk, const DC &dc = DC(), uint32_t p_from = ~0u)
{
  if (p_from == ~0u) p_from = p_lo;
  const uint64_t b_lo = io.off[p_lo], b_hi = io.off[p_hi];
  uint64_t pos = io.off[p_from];
  uint32_t slot = p_from, j = p_from, more = 0;
  while (pos < b_hi) {
    if (slot == p_hi) { more = 1; break; }
    while (j < p_hi && io.off[j] < pos) j++;
    rhp_http_t x;
    bool taken = false;
    /* piece j's speculative records are intact only while no earlier request
     * of this walk has been written over them (slots below `slot` have): a
     * piece that held more than one request -- a coarser split than the
     * server's -- puts later boundaries behind `slot`, and those requests are
     * parsed again from the true boundary */
    if (j < p_hi && io.off[j] == pos && j >= slot) {
      x = io.http[j];
      const uint64_t plen = io.off[j + 1] - pos;
      taken = (x.result == 1 && x.consumed <= plen) || x.result == -1 || x.result == RHP_RET_TOOLONG ||
              (x.result == 0 && j + 1 == p_hi);
    }
    if (taken) {
      const rhp_req_t r = io.reqs[j];
      if (x.result == 1 && x.body_kind == RHP_BODY_CHUNKED_PENDING) {
        /* a true request boundary now: de-frame its chunked body in place
         * (http.c:225-229, the memmove of http_dechunk) */
        uint64_t blen = 0;
        (void) dc(io.bytes_rw + pos + (uint64_t) r.ret, x.consumed - (uint64_t) r.ret, &blen, true);
        x.body_kind = 1;
      }
      if (j != slot) {
        io.reqs[slot] = r;
        const uint32_t nh = r.ret > 0 ? r.num_headers : 0u;
        for (uint32_t k = 0; k < nh; k++)
          io.hdrs[(uint64_t) slot * io.hs_req + k * io.hs_hdr] = io.hdrs[(uint64_t) j * io.hs_req + k * io.hs_hdr];
      }
      io.http[slot] = x;
    } else {
      auto B = mk(pos);
      scalar_http_t(B, io.bytes_rw + pos, b_hi - pos, io.max_headers, &io.reqs[slot],
                    io.hdrs + (uint64_t) slot * io.hs_req, io.hs_hdr, &x, true, dc);
      io.http[slot] = x;
    }
    req_start[slot] = pos;
    slot++;
    if (x.result != 1) break;
    pos += x.consumed;
  }
  out->n_slots = slot - p_lo;
  out->more = more;
  out->consumed = pos - b_lo;
}

}  // namespace rhp

#endif
