/*
 * rhp_dfa.h -- the byte DFA that the MI355X kernel runs, one request per lane.
 *
 * The table re-expresses phr_parse_request (picohttpparser.c:341-409) as a
 * transition table over (state, byte) whose u32 entries carry everything one
 * step needs, so a step is: entry = T[row(entry) + 4*byte] (one LDS read), plus
 * one LDS u16 write that records the byte position into a per-lane capture slot.
 *
 *   entry bits  0..15  LDS byte offset of the next state's row
 *   entry bits 16..23  capture slot, byte offset from the lane's capture pointer
 *   entry bits 24..31  capture pointer increment (a new header record starts)
 *
 * The DFA only decides what it can decide without knowing where the buffer
 * ends: every result is trusted only if the deciding byte lies before `len`
 * (the kernel checks), and paths whose reference behaviour depends on the end
 * of the buffer or that are rare (empty method, bad version literal, obs-fold
 * continuation lines) go to the SLOW terminal and are re-parsed by the exact
 * scalar path (rhp_scalar.h).  Both are checked against the oracle.
 *
 * Per-lane capture area (u16 positions, relative to the request start):
 *   request line record at cap0 (16 B): MS ME PS PE VD . TERM .
 *     MS/ME method start/end  PS/PE path start/end  VD version digit
 *   header record h at cap0 + 16 + 8h (8 B): LS CO VS VE
 *     LS line start (name)  CO colon  VS value start  VE value end (0 = empty)
 *   While header h is being parsed the capture pointer is cap0 + 16 + 8h and the
 *   no-event writes land in record h+1's LS slot (rewritten when h+1 starts),
 *   the terminal position in record h+1's CO slot.  VE slots must start at 0.
 */
#ifndef RHP_DFA_H
#define RHP_DFA_H

#include <stdint.h>

namespace rhp {

enum State : uint32_t {
  S_DONE = 0,     /* terminal: header section complete, TERM = position of final LF */
  S_ERR1,         /* terminal: -1 decided at TERM (trusted iff TERM < len)          */
  S_SLOW,         /* terminal: needs the exact scalar path                          */
  S_OVF,          /* terminal: forced by the kernel when headers exceed capacity    */
  S_SKIP3, S_SKIP2, S_SKIP1,   /* leading bytes of an unaligned 4-byte window   */
  S_START, S_START_CR, S_METHOD0, S_METHOD, S_SPSKIP1, S_PATH, S_SPSKIP2,
  S_V1, S_V2, S_V3, S_V4, S_V5, S_V6, S_V7, S_V8, S_CRLF_REQ,
  S_LINE0, S_LINE, S_NAME, S_COLON, S_VALUE, S_VWS, S_VCR, S_END_CR0, S_END_CR,
  S_COUNT
};

/* capture slots, byte offsets from the capture pointer */
enum Slot : uint32_t {
  /* request-line phase (pointer = cap0) */
  C_MS = 0, C_ME = 2, C_PS = 4, C_PE = 6, C_VD = 8, C_NONE_RL = 10, C_TERM_RL = 12,
  /* header phase (pointer = record h) */
  C_LS = 0, C_CO = 2, C_VS = 4, C_VE = 6, C_NONE_H = 8, C_TERM_H = 10,
  /* terminal self-loops, either phase (record h+1's VE, or cap0+14) */
  C_NONE_T = 14
};

enum : uint32_t {
  kRowBytes = 1040,          /* 256 entries + 4 pad: rows rotate LDS banks by 4 */
  kTableBytes = S_COUNT * kRowBytes,
  kRlBytes = 16,             /* request-line record */
  kHdrBytes = 8,             /* header record */
  kInc0 = 16,                /* first header: cap0 -> record 0 */
  kInc = 8
};

constexpr uint32_t row_of(uint32_t s) { return s * kRowBytes; }
constexpr uint32_t entry(uint32_t next, uint32_t slot, uint32_t inc = 0)
{
  return row_of(next) | (slot << 16) | (inc << 24);
}
constexpr uint32_t entry_next(uint32_t e) { return e & 0xffffu; }
constexpr uint32_t entry_slot(uint32_t e) { return (e >> 16) & 0xffu; }
constexpr uint32_t entry_inc(uint32_t e) { return e >> 24; }
constexpr bool is_terminal_row(uint32_t row) { return row < row_of(S_SKIP3); }

constexpr bool c_tchar(uint32_t c)
{
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '!' ||
         c == '#' || c == '$' || c == '%' || c == '&' || c == '\'' || c == '*' || c == '+' || c == '-' ||
         c == '.' || c == '^' || c == '_' || c == '`' || c == '|' || c == '~';
}
constexpr bool c_ctl(uint32_t c) { return c < 0x20u || c == 0x7fu; }   /* CTL or DEL */
constexpr bool c_ows(uint32_t c) { return c == ' ' || c == '\t'; }

/* one transition: the reference's behaviour on byte c in state s */
constexpr uint32_t step(uint32_t s, uint32_t c)
{
  switch (s) {
  case S_DONE: case S_ERR1: case S_SLOW: case S_OVF:
    return entry(s, C_NONE_T);
  case S_SKIP3: return entry(S_SKIP2, C_NONE_RL);
  case S_SKIP2: return entry(S_SKIP1, C_NONE_RL);
  case S_SKIP1: return entry(S_START, C_NONE_RL);
  case S_START:     /* one optional leading CRLF / LF (picohttpparser.c:345-352) */
    if (c == '\r') return entry(S_START_CR, C_NONE_RL);
    if (c == '\n') return entry(S_METHOD0, C_NONE_RL);
    return step(S_METHOD0, c);
  case S_START_CR:
    return c == '\n' ? entry(S_METHOD0, C_NONE_RL) : entry(S_ERR1, C_TERM_RL);
  case S_METHOD0:   /* ADVANCE_TOKEN(method) first byte (:71-94,:355) */
    if (c == ' ') return entry(S_SLOW, C_TERM_RL);          /* empty method */
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_RL);
    return entry(S_METHOD, C_MS);
  case S_METHOD:
    if (c == ' ') return entry(S_SPSKIP1, C_ME);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_RL);
    return entry(S_METHOD, C_NONE_RL);
  case S_SPSKIP1:   /* do ++buf while SP (:356-358), then path token (:359) */
    if (c == ' ') return entry(S_SPSKIP1, C_NONE_RL);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_RL);
    return entry(S_PATH, C_PS);
  case S_PATH:
    if (c == ' ') return entry(S_SPSKIP2, C_PE);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_RL);
    return entry(S_PATH, C_NONE_RL);
  case S_SPSKIP2:   /* SPs (:360-362), then "HTTP/1." + digit (:245-261) */
    if (c == ' ') return entry(S_SPSKIP2, C_NONE_RL);
    return c == 'H' ? entry(S_V1, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V1: return c == 'T' ? entry(S_V2, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V2: return c == 'T' ? entry(S_V3, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V3: return c == 'P' ? entry(S_V4, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V4: return c == '/' ? entry(S_V5, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V5: return c == '1' ? entry(S_V6, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V6: return c == '.' ? entry(S_V7, C_NONE_RL) : entry(S_SLOW, C_TERM_RL);
  case S_V7: return (c >= '0' && c <= '9') ? entry(S_V8, C_VD) : entry(S_SLOW, C_TERM_RL);
  case S_V8:        /* request line ends with CRLF or LF (:370-378) */
    if (c == '\r') return entry(S_CRLF_REQ, C_NONE_RL);
    if (c == '\n') return entry(S_LINE0, C_NONE_RL);
    return entry(S_ERR1, C_TERM_RL);
  case S_CRLF_REQ:
    return c == '\n' ? entry(S_LINE0, C_NONE_RL) : entry(S_ERR1, C_TERM_RL);
  case S_LINE0:     /* first header line (:266-311), obs-fold impossible */
    if (c == '\r') return entry(S_END_CR0, C_NONE_RL);
    if (c == '\n') return entry(S_DONE, C_TERM_RL);
    if (c_tchar(c)) return entry(S_NAME, C_LS, kInc0);
    return entry(S_ERR1, C_TERM_RL);
  case S_LINE:
    if (c == '\r') return entry(S_END_CR, C_NONE_H);
    if (c == '\n') return entry(S_DONE, C_TERM_H);
    if (c_tchar(c)) return entry(S_NAME, C_LS, kInc);
    if (c_ows(c)) return entry(S_SLOW, C_TERM_H);           /* obs-fold */
    return entry(S_ERR1, C_TERM_H);
  case S_NAME:      /* name bytes must be tchar up to ':' (:297-310) */
    if (c == ':') return entry(S_COLON, C_CO);
    if (c_tchar(c)) return entry(S_NAME, C_NONE_H);
    return entry(S_ERR1, C_TERM_H);
  case S_COLON:     /* OWS after ':' (:312-317), then get_token_to_eol (:134-195) */
    if (c_ows(c)) return entry(S_COLON, C_NONE_H);
    if (c == '\r') return entry(S_VCR, C_VS);
    if (c == '\n') return entry(S_LINE, C_VS);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_H);
    return entry(S_VALUE, C_VS);
  case S_VALUE:     /* VE = start of the latest OWS run, or the EOL (:327-336) */
    if (c_ows(c)) return entry(S_VWS, C_VE);
    if (c == '\r') return entry(S_VCR, C_VE);
    if (c == '\n') return entry(S_LINE, C_VE);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_H);
    return entry(S_VALUE, C_NONE_H);
  case S_VWS:
    if (c_ows(c)) return entry(S_VWS, C_NONE_H);
    if (c == '\r') return entry(S_VCR, C_NONE_H);
    if (c == '\n') return entry(S_LINE, C_NONE_H);
    if (c_ctl(c)) return entry(S_ERR1, C_TERM_H);
    return entry(S_VALUE, C_NONE_H);
  case S_VCR:
    return c == '\n' ? entry(S_LINE, C_NONE_H) : entry(S_ERR1, C_TERM_H);
  case S_END_CR0:   /* empty line ends the headers (:268-275) */
    return c == '\n' ? entry(S_DONE, C_TERM_RL) : entry(S_ERR1, C_TERM_RL);
  case S_END_CR:
    return c == '\n' ? entry(S_DONE, C_TERM_H) : entry(S_ERR1, C_TERM_H);
  default:
    return entry(S_SLOW, C_NONE_T);
  }
}

struct Table {
  uint32_t w[kTableBytes / 4];
};

constexpr Table make_table()
{
  Table t{};
  for (uint32_t s = 0; s < S_COUNT; s++) {
    for (uint32_t c = 0; c < 256; c++) t.w[(row_of(s) >> 2) + c] = step(s, c);
    for (uint32_t c = 256; c < kRowBytes / 4; c++) t.w[(row_of(s) >> 2) + c] = entry(S_SLOW, C_NONE_T);
  }
  return t;
}

/* bytes of per-lane capture area for a header capacity; the kernel checks the
 * header count every kCheckSteps bytes, and a header line is >= 3 bytes, so at
 * most kCheckSteps/3 + 1 records can start past capacity before the check, plus
 * one for the next-record slots. */
enum : uint32_t { kCheckSteps = 16 };
constexpr uint32_t cap_bytes(uint32_t max_headers)
{
  return kRlBytes + kHdrBytes * (max_headers + kCheckSteps / 3 + 3);
}

}  // namespace rhp

#endif
