/*
 * rhp_dfa.h -- the byte DFA that the MI355X kernel runs, one request per lane,
 * and the event decoder that turns its output into phr_parse_request records.
 *
 * The table re-expresses phr_parse_request (picohttpparser.c:341-409, headers
 * :263-339) as u8 entries over (state, byte).  State s has the index idx8(s)
 * and its row of 256 next-state indices lives at LDS byte idx8(s) * 256, so a
 * step is
 *
 *     a = v_perm(state, window dword, sel)   = state * 256 + byte
 *     state = T8[a]                          one ds_read_u8
 *     ev = v_alignbit(state, ev, 1)          bit 0 of the index -> event mask
 *
 * Events.  Plain states have even indices and event states odd ones, so bit 0
 * of an index says "the transition that entered this state is an event"; the
 * kernel shifts that bit into a per-lane 32-bit mask with one VALU op and
 * decodes the mask once per block.  For a request the fast path accepts, the
 * event sequence is fixed by the grammar:
 *
 *   ME  PE  RL              request line: method end (the SP; the path starts
 *                           right after it), path end (the next SP), RL = the
 *                           CR of "HTTP/1.0\r\n" or the LF of "HTTP/1.1\r\n" (so
 *                           the position encodes the minor version: RL - PE =
 *                           9 or 10)
 *   { CO  EOL }*            per header line: the colon (the value starts two
 *                           bytes later, after its one SP) and the LF that ends
 *                           the line
 *   T                       terminal: the final LF (DONE) or the byte at which
 *                           the reference returns -1 (ERR)
 *
 * Each event shifts its position into a 4-deep u16 history, which then holds
 * everything a record needs.  The DFA only decides what it can decide without
 * knowing where the buffer ends: a terminal is the reference's answer iff its
 * byte lies before `len`; constructs that are rare in real traffic or whose
 * answer depends on where the buffer ends go to the SLOW terminal and are
 * re-parsed by the exact scalar path (rhp_scalar.h): a leading empty line, an
 * empty method, more than one SP between request-line fields, minor versions
 * other than 0 and 1 (a version that is not "HTTP/1." + digit is ERR, trusted
 * when the version's 9 bytes are in the buffer), bare-LF line ends, anything but exactly one SP
 * after a header colon (":v", ":\tv", ":  v", ":\r\n"), OWS before a CR
 * (value trimming), obs-fold continuation lines.  A header section longer
 * than the u16 records hold (ret > RHP_MAX_LEN) is also handed to the exact
 * path, which answers RHP_RET_TOOLONG; requests of any length are walked.
 */
#ifndef RHP_DFA_H
#define RHP_DFA_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RHP_DHD __host__ __device__
#else
#define RHP_DHD
#endif

/* bytes of a lane's window per kernel loop iteration: the DFA steps this many
 * bytes between two decodes (kernel and emulator must agree) */
#ifndef RHP_BLOCK
#define RHP_BLOCK 64
#endif
/* http mode's window extension in 16-byte parts: its windows are RHP_BLOCK +
 * 16 * RHP_HTTP_XPARTS bytes (rhp_kernel.hip, window geometry; measured with 2
 * and not kept) */
#ifndef RHP_HTTP_XPARTS
#define RHP_HTTP_XPARTS 0
#endif
#define RHP_HTTP_BLOCK (RHP_BLOCK + 16 * RHP_HTTP_XPARTS)

namespace rhp {

enum State : uint32_t {
  /* plain rows (no event on entry) */
  S_DONE = 0, S_ERR, S_SLOW,                   /* terminals */
  S_PRE,                                       /* the window's bytes before the request's first */
  S_METHOD0, S_METHOD, S_PATH0, S_PATH,
  S_V1, S_V2, S_V3, S_V4, S_V5, S_V6, S_V7, S_V8_0, S_V8_1, S_CRLF_RL,
  S_LINE0, S_NAME, S_VAL0, S_VALUE, S_VWS, S_VCR, S_END_CR,
  S_NUM_PLAIN,
  /* event rows (an event fires on the transition that enters them) */
  S_DONE_E = S_NUM_PLAIN, S_ERR_E,             /* terminal events */
  S_SP1_E,       /* ME */
  S_SP2_E,       /* PE */
  S_CRLF_RL_E,   /* RL at the CR (HTTP/1.0) */
  S_LINE0_E,     /* RL at the LF (HTTP/1.1) */
  S_COLON_E,     /* CO */
  S_LINE_E,      /* EOL */
  S_COUNT
};

/* u8 index of a state: plain states even, event states odd */
RHP_DHD constexpr uint32_t idx8(uint32_t s)
{
  return s < S_NUM_PLAIN ? 2u * s : 2u * (s - S_NUM_PLAIN) + 1u;
}
enum : uint32_t {
  kRows8 = 2u * (S_NUM_PLAIN - 1u) + 1u,   /* highest index + 1 (the last plain state) */
  kTable8Bytes = kRows8 * 256u
};
static_assert(2u * (S_COUNT - S_NUM_PLAIN) - 1u < kRows8, "event indices fit below the last plain row");
static_assert(kRows8 <= 256u, "indices are bytes");

RHP_DHD constexpr bool is_done8(uint32_t e) { return e == idx8(S_DONE) || e == idx8(S_DONE_E); }
RHP_DHD constexpr bool is_err8(uint32_t e) { return e == idx8(S_ERR) || e == idx8(S_ERR_E); }
RHP_DHD constexpr bool is_slow8(uint32_t e) { return e == idx8(S_SLOW); }

constexpr bool c_tchar(uint32_t c)
{
  return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '!' ||
         c == '#' || c == '$' || c == '%' || c == '&' || c == '\'' || c == '*' || c == '+' || c == '-' ||
         c == '.' || c == '^' || c == '_' || c == '`' || c == '|' || c == '~';
}
constexpr bool c_ctl(uint32_t c) { return c < 0x20u || c == 0x7fu; }   /* CTL or DEL */
constexpr bool c_ows(uint32_t c) { return c == ' ' || c == '\t'; }
/* the byte class of 0x00: CTL or DEL other than HT, LF and CR (C_CTLX below) */
RHP_DHD constexpr bool byte_class_ctlx(uint32_t c) { return (c < 0x20u && c != '\t' && c != '\n' && c != '\r') || c == 0x7fu; }

/* one transition: the next state on byte c in state s (picohttpparser.c line refs) */
constexpr uint32_t step(uint32_t s, uint32_t c)
{
  switch (s) {
  case S_DONE: case S_DONE_E: return S_DONE;
  case S_ERR: case S_ERR_E: return S_ERR;
  case S_SLOW: return S_SLOW;
  case S_PRE:       /* a window starts at or before the request: the kernel zeroes the bytes
                       before its first one (a CTL, which then starts no request: the
                       kernel sends a request whose own first byte is such a CTL to the
                       exact path instead of walking it) */
    return byte_class_ctlx(c) ? S_PRE : step(S_METHOD0, c);
  case S_METHOD0:   /* optional leading empty line (:345-352) -> exact path; ADVANCE_TOKEN (:71-94) */
    if (c == '\r' || c == '\n' || c == ' ') return S_SLOW;
    return c_ctl(c) ? S_ERR_E : S_METHOD;
  case S_METHOD:
    if (c == ' ') return S_SP1_E;
    return c_ctl(c) ? S_ERR_E : S_METHOD;
  case S_SP1_E:     /* SP skip (:356-358): a second SP -> exact path; then the path token (:359) */
    if (c == ' ') return S_SLOW;
    return c_ctl(c) ? S_ERR_E : S_PATH;
  case S_PATH:
    if (c == ' ') return S_SP2_E;
    return c_ctl(c) ? S_ERR_E : S_PATH;
  case S_SP2_E:     /* "HTTP/1." + digit (:245-261) right after one SP (a second SP is
                       skipped by :360-362: exact path) */
    return c == 'H' ? S_V1 : c == ' ' ? S_SLOW : S_ERR_E;
  /* a mismatch in the version is -1 (EXPECT_CHAR_NO_CHECK, :252-258) when the
   * 9 bytes of the version are there (:248-251): finalize trusts an ERR before
   * the request-line end only when len >= PE + 10 (rhp_kernel.hip decode_end) */
  case S_V1: return c == 'T' ? S_V2 : S_ERR_E;
  case S_V2: return c == 'T' ? S_V3 : S_ERR_E;
  case S_V3: return c == 'P' ? S_V4 : S_ERR_E;
  case S_V4: return c == '/' ? S_V5 : S_ERR_E;
  case S_V5: return c == '1' ? S_V6 : S_ERR_E;
  case S_V6: return c == '.' ? S_V7 : S_ERR_E;
  case S_V7:        /* PARSE_INT (:259): minors 2-9 (and tchar letters, one class) -> exact path */
    return c == '0' ? S_V8_0 : c == '1' ? S_V8_1 : c_tchar(c) ? S_SLOW : S_ERR_E;
  case S_V8_0:      /* the request line ends with CRLF (:370-378); bare LF -> exact path */
    if (c == '\r') return S_CRLF_RL_E;
    return c == '\n' ? S_SLOW : S_ERR_E;
  case S_V8_1:
    if (c == '\r') return S_CRLF_RL;
    return c == '\n' ? S_SLOW : S_ERR_E;
  case S_CRLF_RL_E: return c == '\n' ? S_LINE0 : S_ERR_E;
  case S_CRLF_RL: return c == '\n' ? S_LINE0_E : S_ERR_E;
  case S_LINE0: case S_LINE0_E:   /* first header line (:266-311): no obs-fold yet */
    if (c == '\r') return S_END_CR;
    if (c == '\n') return S_SLOW;
    return c_tchar(c) ? S_NAME : S_ERR_E;
  case S_LINE_E:
    if (c == '\r') return S_END_CR;
    if (c == '\n' || c_ows(c)) return S_SLOW;   /* bare LF, obs-fold */
    return c_tchar(c) ? S_NAME : S_ERR_E;
  case S_NAME:      /* name bytes must be tchar up to ':' (:297-310) */
    if (c == ':') return S_COLON_E;
    return c_tchar(c) ? S_NAME : S_ERR_E;
  case S_COLON_E:   /* OWS after ':' (:312-317): exactly one SP on the fast path */
    if (c == ' ') return S_VAL0;
    return c_ctl(c) && c != '\t' && c != '\r' && c != '\n' ? S_ERR_E : S_SLOW;
  case S_VAL0:      /* first value byte, get_token_to_eol (:134-195) */
    if (c_ows(c) || c == '\n') return S_SLOW;
    if (c == '\r') return S_VCR;
    return c_ctl(c) ? S_ERR_E : S_VALUE;
  case S_VALUE:
    if (c_ows(c)) return S_VWS;
    if (c == '\r') return S_VCR;
    if (c == '\n') return S_SLOW;
    return c_ctl(c) ? S_ERR_E : S_VALUE;
  case S_VWS:       /* OWS inside a value; OWS before the EOL is trimmed (:327-336) -> exact */
    if (c_ows(c)) return S_VWS;
    if (c == '\r' || c == '\n') return S_SLOW;
    return c_ctl(c) ? S_ERR_E : S_VALUE;
  case S_VCR: return c == '\n' ? S_LINE_E : S_ERR_E;
  case S_END_CR:    /* empty line ends the headers (:268-275) */
    return c == '\n' ? S_DONE_E : S_ERR_E;
  default: return S_SLOW;
  }
}

struct Table8 {
  uint8_t b[kTable8Bytes];
};

constexpr Table8 make_table8()
{
  Table8 t{};
  for (uint32_t i = 0; i < kTable8Bytes; i++) t.b[i] = (uint8_t) idx8(S_SLOW);   /* unused rows */
  for (uint32_t s = 0; s < S_COUNT; s++)
    for (uint32_t c = 0; c < 256; c++) t.b[idx8(s) * 256u + c] = (uint8_t) idx8(step(s, c));
  return t;
}

/*
 * Pair form (what the kernel runs): two bytes per table read.  Every state's
 * transition depends on a byte only through its class (15 classes, checked by
 * classes_exact below), so a step over bytes (b0, b1) is one read at
 *   idx * 256 + class(b0) * 16 + class(b1)
 * of a u8 table whose entries are pair indices.  A pair index carries the
 * state after both bytes and, in its low two bits, whether the transition on
 * b0 / on b1 was an event; the kernel shifts those two bits into its event
 * mask (v_alignbit by 2), so the mask is the same per-byte event mask as the
 * one-byte form produces.
 *   plain state s:  idx = 4s + e   (e = 0, or 1: event on b0 only)
 *   event state s:  idx = 4(s - S_NUM_PLAIN) + e   (e = 2 or 3: event on b1)
 * The byte-class table lives in an unused row (kClassRow).
 */
enum : uint32_t {
  C_CTLX = 0, C_HT, C_LF, C_CR, C_SP, C_COLON, C_H, C_T, C_P, C_SLASH, C_DOT, C_0, C_1, C_TCHAR, C_OTHER,
  kClasses
};

constexpr uint32_t byte_class(uint32_t c)
{
  if (c == '\t') return C_HT;
  if (c == '\n') return C_LF;
  if (c == '\r') return C_CR;
  if (c_ctl(c)) return C_CTLX;
  switch (c) {
  case ' ': return C_SP;
  case ':': return C_COLON;
  case 'H': return C_H;
  case 'T': return C_T;
  case 'P': return C_P;
  case '/': return C_SLASH;
  case '.': return C_DOT;
  case '0': return C_0;
  case '1': return C_1;
  default: return c_tchar(c) ? C_TCHAR : C_OTHER;
  }
}

constexpr uint32_t class_rep(uint32_t k)   /* a byte of class k */
{
  constexpr uint8_t rep[kClasses] = {0x00, '\t', '\n', '\r', ' ', ':', 'H', 'T', 'P', '/', '.', '0', '1', '!', '"'};
  return rep[k];
}

constexpr bool ctlx_exact()
{
  for (uint32_t c = 0; c < 256; c++)
    if (byte_class_ctlx(c) != (byte_class(c) == C_CTLX)) return false;
  return byte_class(0) == C_CTLX;
}
static_assert(ctlx_exact(), "byte_class_ctlx is the class of the zeroed bytes");

/* every byte behaves like its class representative in every state */
constexpr bool classes_exact()
{
  for (uint32_t k = 0; k < kClasses; k++)
    if (byte_class(class_rep(k)) != k) return false;
  for (uint32_t s = 0; s < S_COUNT; s++)
    for (uint32_t c = 0; c < 256; c++)
      if (step(s, c) != step(s, class_rep(byte_class(c)))) return false;
  return true;
}
static_assert(classes_exact(), "byte classes must not split any transition");

/*
 * Run skipping.  In the path token (ADVANCE_TOKEN, picohttpparser.c:71-94) and
 * inside a header value (get_token_to_eol, :134-195) every byte that is not
 * SP, a CTL or DEL keeps the state and fires no event -- the cases the
 * reference's findchar_fast pre-scan skips 16 bytes at a time (:105-132).  A
 * chunk made only of such bytes therefore leaves a lane in S_PATH, or moves
 * it from S_VALUE / S_VWS to S_VALUE, with an all-zero event mask; the kernel
 * skips the table walk for a chunk when that holds for every busy lane of the
 * wave (wave-uniform: an LDS read costs the same with idle lanes masked off).
 */
constexpr bool c_run(uint32_t c) { return c > 0x20u && c != 0x7fu; }
constexpr bool runs_exact()
{
  for (uint32_t c = 0; c < 256; c++) {
    if (!c_run(c)) continue;
    if (step(S_PATH, c) != S_PATH || step(S_VALUE, c) != S_VALUE || step(S_VWS, c) != S_VALUE) return false;
  }
  return true;
}
static_assert(runs_exact(), "run bytes keep S_PATH / move S_VALUE, S_VWS to S_VALUE without an event");

RHP_DHD constexpr uint32_t idx2(uint32_t s, uint32_t e)
{
  return s < S_NUM_PLAIN ? 4u * s + e : 4u * (s - S_NUM_PLAIN) + e;
}
RHP_DHD constexpr uint32_t state2(uint32_t idx)
{
  return (idx & 2u) ? (idx >> 2) + S_NUM_PLAIN : idx >> 2;
}

/*
 * Row geometry.  The row of pair index idx starts at LDS byte idx * kStride and
 * holds entries for the codes class(b0) * 16 + class(b1) < kCodes.  With a
 * stride of 256 the walk's address is one v_perm (idx * 256 + code), and every
 * row starts in LDS bank 0: lanes in different states reading the same code
 * read the same bank at different addresses, an N-way conflict in the walk's
 * dependent read.  A stride of 256 + 4k (RHP_ROW_STRIDE; 268: k = 3) starts row
 * idx k banks further (one v_mad_u32_u24 instead of the v_perm).
 */
#ifndef RHP_ROW_STRIDE
#define RHP_ROW_STRIDE 268   /* round 5: rows 3 banks apart; 260 (1 bank) after line windows was 1-2 % faster
                                than 256 on configs 2/3/5, 268 another 2.7 % on config 5 (profiles/r05/ab/) */
#endif
enum : uint32_t {
  kStride = RHP_ROW_STRIDE,
  kCodes = (kClasses - 1u) * 16u + kClasses,      /* highest code + 1 */
  kRows2 = 4u * (S_NUM_PLAIN - 1u) + 2u           /* highest index (last plain state, e = 1) + 1 */
};
static_assert(kStride >= 256u && kStride % 4u == 0, "rows hold every code, dword aligned");
static_assert(kRows2 <= 256u, "indices are bytes");

/* the indices a state uses: plain states 4s, 4s+1; event states 4(s - S_NUM_PLAIN) + 2, + 3 */
RHP_DHD constexpr bool idx_used(uint32_t i) { return i < kRows2 && state2(i) < S_COUNT; }

/*
 * Pair codes by two lookups instead of arithmetic:
 *   r    = T[kClassRowR * 256 + b1]     the row of class(b1): code_row(class(b1))
 *   code = T[r * 256 + b0]              = class(b0) * 16 + class(b1)
 * so a pair costs two address v_perms and no packing ops.  These rows (and the
 * byte-class row kClassRow) are 256-byte aligned (a v_perm builds their
 * addresses) and placed in the holes the state rows leave: the first free
 * 256-byte rows.
 */
struct RowLayout {
  uint32_t row[3 + kClasses];   /* kClassRow, kClassRowR, kClassRow16, code_row(0..14) */
  uint32_t bytes;               /* the table's size, 16-byte multiple */
};
constexpr RowLayout make_row_layout()
{
  RowLayout l{};
  uint32_t end = 0, n = 0;
  for (uint32_t i = 0; i < kRows2; i++)
    if (idx_used(i) && i * kStride + kCodes > end) end = i * kStride + kCodes;
  for (uint32_t r = 0; r < 256u && n < 3u + kClasses; r++) {
    bool free = true;
    for (uint32_t i = 0; i < kRows2; i++)
      if (idx_used(i) && i * kStride < r * 256u + 256u && r * 256u < i * kStride + kCodes) free = false;
    if (free) {
      l.row[n++] = r;
      if (r * 256u + 256u > end) end = r * 256u + 256u;
    }
  }
  l.bytes = n == 3u + kClasses ? (end + 15u) & ~15u : 0u;
  return l;
}
constexpr RowLayout kRowLayout = make_row_layout();
static_assert(kRowLayout.bytes != 0, "the lookup rows fit");
enum : uint32_t {
  kClassRow = kRowLayout.row[0],
  kClassRowR = kRowLayout.row[1],
  kClassRow16 = kRowLayout.row[2],   /* class(b) * 16: the b0 half of a code (the kernel's code form 2) */
  kTable2Bytes = kRowLayout.bytes
};
RHP_DHD constexpr uint32_t code_row(uint32_t k) { return kRowLayout.row[3 + k]; }   /* k < kClasses */
static_assert(kClassRowR < 256u && code_row(kClasses - 1u) < 256u, "row numbers are bytes");

RHP_DHD constexpr bool is_done2(uint32_t i) { return state2(i) == S_DONE || state2(i) == S_DONE_E; }
RHP_DHD constexpr bool is_err2(uint32_t i) { return state2(i) == S_ERR || state2(i) == S_ERR_E; }
RHP_DHD constexpr bool is_slow2(uint32_t i) { return state2(i) == S_SLOW; }

struct Table2 {
  uint8_t b[kTable2Bytes];
};

constexpr Table2 make_table2()
{
  Table2 t{};
  for (uint32_t i = 0; i < kTable2Bytes; i++) t.b[i] = (uint8_t) idx2(S_SLOW, 0);   /* unused rows */
  for (uint32_t s = 0; s < S_COUNT; s++) {
    const bool ev = s >= S_NUM_PLAIN;
    for (uint32_t e = ev ? 2u : 0u; e < (ev ? 4u : 2u); e++) {
      const uint32_t row = idx2(s, e) * kStride;
      for (uint32_t k0 = 0; k0 < kClasses; k0++)
        for (uint32_t k1 = 0; k1 < kClasses; k1++) {
          const uint32_t s1 = step(s, class_rep(k0)), s2 = step(s1, class_rep(k1));
          t.b[row + k0 * 16u + k1] = (uint8_t) idx2(s2, (s1 >= S_NUM_PLAIN ? 1u : 0u) | (s2 >= S_NUM_PLAIN ? 2u : 0u));
        }
    }
  }
  for (uint32_t c = 0; c < 256; c++) t.b[kClassRow * 256u + c] = (uint8_t) byte_class(c);
  for (uint32_t c = 0; c < 256; c++) t.b[kClassRowR * 256u + c] = (uint8_t) code_row(byte_class(c));
  for (uint32_t c = 0; c < 256; c++) t.b[kClassRow16 * 256u + c] = (uint8_t) (byte_class(c) * 16u);
  for (uint32_t k = 0; k < kClasses; k++)
    for (uint32_t c = 0; c < 256; c++) t.b[code_row(k) * 256u + c] = (uint8_t) (byte_class(c) * 16u + k);
  return t;
}

/*
 * Event decoder state of one request (the emulator's form of the kernel's
 * anchor decode).  e[0..3] hold the last four event positions, e[0] newest.
 */
struct Dec {
  uint32_t e[4];
  uint32_t k;       /* events consumed: 0..2 request line, then 3,4 = CO, EOL */
  uint32_t nh;      /* header lines completed */
  uint32_t rl01;    /* method_len | path_off << 16 */
  uint32_t rl23;    /* path_len | minor << 16 */
  uint32_t ovf;     /* 0, or 1 + the position at which max_headers overflowed */
};

RHP_DHD inline void dec_reset(Dec &d)
{
  d.e[0] = d.e[1] = d.e[2] = d.e[3] = 0;
  d.k = 0;
  d.nh = 0;
  d.rl01 = d.rl23 = 0;
  d.ovf = 0;
}

/*
 * Consume one (non-terminal) event at position p.  Returns true when a header
 * record completed that is to be stored at index d.nh - 1 (< max_headers):
 * (lo, hi) = (name_off | name_len << 16, value_off | value_len << 16).
 * Sets d.ovf when the reference's max_headers check fires (picohttpparser.c:
 * 281-284: a new line starts while num_headers == max_headers).  Records are
 * u16: they are only used when the request ends below RHP_MAX_LEN.
 */
RHP_DHD inline bool dec_event(Dec &d, uint32_t p, uint32_t maxh, uint32_t &lo, uint32_t &hi)
{
  d.e[3] = d.e[2];
  d.e[2] = d.e[1];
  d.e[1] = d.e[0];
  d.e[0] = p;
  if (d.k < 2) {
    d.k++;
    return false;
  }
  if (d.k == 2) {   /* RL: history = RL, PE, ME */
    const uint32_t pe = d.e[1], me = d.e[2];
    const uint32_t minor = p - pe - 9u;   /* 0 (event at the CR) or 1 (at the LF) */
    d.rl01 = (me & 0xffffu) | ((me + 1u) << 16);
    d.rl23 = ((pe - me - 1u) & 0xffffu) | (minor << 16);
    d.e[0] = pe + 10u;   /* e0 := the LF that ends the request line */
    d.k = 3;
    return false;
  }
  if (d.k == 3) {   /* CO: history = CO, prevLF, ... */
    if (d.nh == maxh && d.ovf == 0) d.ovf = 1u + d.e[1] + 1u;
    d.k = 4;
    return false;
  }
  /* EOL: history = LF, CO, prevLF */
  const uint32_t lf = p, co = d.e[1], prev = d.e[2];
  lo = ((prev + 1u) & 0xffffu) | ((co - prev - 1u) << 16);
  hi = ((co + 2u) & 0xffffu) | ((lf - co - 3u) << 16);
  d.k = 3;
  d.nh++;
  return d.nh <= maxh;
}

}  // namespace rhp

#endif
