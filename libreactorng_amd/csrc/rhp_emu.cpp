/*
 * rhp_emu.cpp -- CPU emulation of rhp_dfa_kernel, for tests only.
 *
 * Runs the same pair transition table (rhp_dfa.h Table2), windows starting in the
 * same S_PRE state with the bytes before the request zeroed (a request whose
 * first byte is of their class goes to the exact path, as in the kernel; the
 * same window geometry: phr mode's first windows start at the 128-byte line
 * holding the request, http mode's at its dword), the same blocks with one
 * event-mask decode per block
 * (rhp_dfa.h dec_event) and the same finalize decisions as the kernel, one
 * request at a time on the host.  Lets the DFA design be checked against
 * the oracle on millions of requests without a GPU; the GPU tests then check
 * the kernel itself.
 */
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "rhp.h"
#include "rhp_host.h"
#include "rhp_dfa.h"
#include "rhp_scalar.h"

using namespace rhp;

namespace {

const Table2 &table()
{
  static const Table2 t = make_table2();
  return t;
}

struct Stats {
  uint64_t fast_ok, fast_bad, exact;
};

/* the exact path's (wide) records of request i: the batch's hdrs in its layout,
 * or the wide area behind the lengths of a compact batch (rhp.h) */
rhp_hdr_t *wide_records(const rhp_batch_t *b, uint32_t i, uint64_t &hs_hdr)
{
  if (b->layout == RHP_LAYOUT_COMPACT || b->layout == RHP_LAYOUT_DENSE || b->layout == RHP_LAYOUT_DENSE_RM) {
    hs_hdr = 1u;
    const size_t off = b->layout != RHP_LAYOUT_COMPACT ? RHP_DENSE_WIDE_OFF(b->n, b->max_headers)
                                                       : RHP_COMPACT_WIDE_OFF(b->n, b->max_headers);
    return reinterpret_cast<rhp_hdr_t *>(reinterpret_cast<uint8_t *>(b->hdrs) + off) + (uint64_t) i * b->max_headers;
  }
  const bool hmajor = b->layout == RHP_LAYOUT_HEADER_MAJOR;
  hs_hdr = hmajor ? b->n : 1u;
  return b->hdrs + (uint64_t) i * (hmajor ? 1u : b->max_headers);
}

/* compact http records (rhp.h, RHP_LAYOUT_COMPACT in http mode): as the kernel,
 * a record whose consumed follows from ret is stored compact, any other one
 * (the exact path's, a chunked body de-framed in place) in the wide area */
bool compact_http(const rhp_batch_t *b)
{
  return b->mode == RHP_MODE_HTTP && (b->layout == RHP_LAYOUT_COMPACT || b->layout == RHP_LAYOUT_DENSE);
}
rhp_http_compact_t *http_compact(const rhp_batch_t *b) { return reinterpret_cast<rhp_http_compact_t *>(b->http); }
rhp_http_t *http_wide(const rhp_batch_t *b)
{
  return reinterpret_cast<rhp_http_t *>(reinterpret_cast<uint8_t *>(b->http) + RHP_COMPACT_HTTP_WIDE_OFF(b->n));
}
void put_http(const rhp_batch_t *b, uint32_t i, const rhp_http_t &x, bool wide)
{
  if (!compact_http(b)) {
    b->http[i] = x;
    return;
  }
  rhp_http_compact_t c = {(int8_t) x.result, (uint8_t) x.body_kind, 0, 0, (uint32_t) x.body_len};
  if (wide) {
    c = rhp_http_compact_t{0, 0, (uint8_t) RHP_HTTP_WIDE, 0, 0};
    http_wide(b)[i] = x;
  }
  http_compact(b)[i] = c;
}
/* the consumed a compact record stands for (rhp.h) */
uint64_t compact_consumed(int32_t ret, const rhp_http_t &x)
{
  return x.result == 1 ? (uint64_t) ret + (x.body_kind == 1 ? x.body_len : 0u) : 0u;
}

/* the layouts whose records of an exact-path request are the wide ones */
bool dense_layout(const rhp_batch_t *b) { return b->layout == RHP_LAYOUT_DENSE || b->layout == RHP_LAYOUT_DENSE_RM; }
bool wide_layout(const rhp_batch_t *b) { return b->layout == RHP_LAYOUT_COMPACT || dense_layout(b); }

/* dense layout (rhp.h RHP_LAYOUT_DENSE): the 8-byte records and their wide area */
rhp_req_dense_t *dense_reqs(const rhp_batch_t *b) { return reinterpret_cast<rhp_req_dense_t *>(b->reqs); }
rhp_req_t *dense_wide_reqs(const rhp_batch_t *b)
{
  return reinterpret_cast<rhp_req_t *>(reinterpret_cast<uint8_t *>(b->reqs) + RHP_DENSE_REQ_WIDE_OFF(b->n));
}
/* request i's record: rhp_req_t, or (dense) the wide area and a WIDE mark */
void put_req(const rhp_batch_t *b, uint32_t i, const rhp_req_t &r)
{
  if (!dense_layout(b)) {
    b->reqs[i] = r;
    return;
  }
  dense_wide_reqs(b)[i] = r;
  dense_reqs(b)[i] = rhp_req_dense_t{0, 0, 0, 0, 0, (uint8_t) RHP_DENSE_WIDE};
}

void emu_exact(const rhp_batch_t *b, uint32_t i, uint64_t off, uint64_t len)
{
  rhp_req_t r;
  r.flags = RHP_F_EXACT | (wide_layout(b) ? RHP_F_WIDE : 0u);
  uint64_t hs_hdr = 1;
  rhp_hdr_t *h = wide_records(b, i, hs_hdr);
  if (b->mode == RHP_MODE_HTTP) {
    PlainBytes B{b->bytes_rw + off};
    rhp_http_t x;
    scalar_http_t(B, b->bytes_rw + off, len, b->max_headers, &r, h, hs_hdr, &x, !(b->flags & RHP_BATCH_SPECULATIVE));
    put_http(b, i, x, true);
  }
  else {
    const uint64_t ll = b->last_len ? b->last_len[i] : 0;
    const int pre = ll ? is_complete(b->bytes + off, len, ll) : 0;   /* picohttpparser.c:399-401 */
    if (pre != 0) {
      memset(&r, 0, sizeof r);
      r.ret = pre;
      r.minor_version = -1;
      r.flags = RHP_F_EXACT | (wide_layout(b) ? RHP_F_WIDE : 0u);
    } else {
      scalar_phr(b->bytes + off, len, b->max_headers, &r, h, hs_hdr);
    }
  }
  put_req(b, i, r);
}

}  // namespace

extern "C" int rhp_emu_parse_batch(const rhp_batch_t *b, uint64_t *stats /* [3] or NULL */)
{
  if ((b->layout == RHP_LAYOUT_COMPACT || dense_layout(b)) && (b->flags & RHP_BATCH_SPECULATIVE))
    return -22;   /* as rhp_parse_batch */
  if (b->layout == RHP_LAYOUT_DENSE_RM && b->mode != RHP_MODE_PHR) return -22;   /* dense http: header-major */
  const Table2 &T = table();
  const uint8_t *cls = T.b + kClassRow * 256u;
  Stats st_count = {0, 0, 0};
  const uint32_t maxh = b->max_headers;

  for (uint32_t i = 0; i < b->n; i++) {
    const uint64_t off = b->offsets[i], len = b->offsets[i + 1] - off;
    /* the kernel's first window: from the 128-byte line (phr mode) or the dword
     * (http mode) holding the request's first byte, offsets from the batch's
     * bytes.  The geometry decides, in rare cases, whether the DFA path or the
     * exact path answers (a max_headers overflow whose colon lies in the window
     * that also holds a SLOW, or lies past len): the flags follow it, the
     * answers do not */
    const uint32_t mis = (uint32_t) off & (b->mode == RHP_MODE_PHR ? 127u : 3u);
    const uint8_t *win = b->bytes + (off - mis);
    int32_t pos = -(int32_t) mis;
    uint32_t st = idx2(byte_class_ctlx(b->bytes[off]) ? S_SLOW : S_PRE, 0);
    Dec d;
    dec_reset(d);
    const bool compact = b->layout == RHP_LAYOUT_COMPACT, dense = dense_layout(b);
    const uint64_t hs_req = b->layout == RHP_LAYOUT_HEADER_MAJOR ? 1u : maxh;
    const uint64_t hs_hdr = b->layout == RHP_LAYOUT_HEADER_MAJOR ? b->n : 1u;
    rhp_hdr_t *hout = compact || dense ? nullptr : b->hdrs + i * hs_req;
    uint32_t *lens = compact ? reinterpret_cast<uint32_t *>(b->hdrs) + i : nullptr;   /* lens[k * n + i] */
    /* dense: the u16 lengths (k * n + i, or request-major i * m + k) and the overflow area */
    const bool drm = b->layout == RHP_LAYOUT_DENSE_RM;
    uint16_t *lens16 = dense ? reinterpret_cast<uint16_t *>(b->hdrs) + (drm ? (uint64_t) i * maxh : i) : nullptr;
    uint32_t *ovf32 = dense ? reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(b->hdrs) + RHP_DENSE_OVF_OFF(b->n, maxh)) +
                                  (drm ? (uint64_t) i * maxh : i)
                            : nullptr;
    const uint64_t dstride = drm ? 1u : b->n;
    /* header k's u32 lengths, name_len | value_len << 16, in the compact or a dense layout */
    auto len32 = [&](uint32_t k) -> uint32_t {
      if (compact) return lens[(uint64_t) k * b->n];
      const uint32_t l = lens16[k * dstride];
      return l == RHP_DENSE_OVERFLOW ? ovf32[k * dstride] : (l & 63u) | (l >> 6) << 16;
    };
    /* the kernel's window: http mode walks RHP_HTTP_BLOCK bytes per window */
    const int32_t block = b->mode == RHP_MODE_HTTP ? RHP_HTTP_BLOCK : RHP_BLOCK;
    constexpr int kMaxWords = (RHP_HTTP_BLOCK > RHP_BLOCK ? RHP_HTTP_BLOCK : RHP_BLOCK) / 32;
    const int words = block / 32;
    for (;;) {
      /* one window: steps, then the decode of its event mask (32 bytes per word) */
      const int32_t block_pos = pos;
      uint32_t evw[kMaxWords];
      for (int w = 0; w < words; w++) {
        uint32_t ev = 0;
        for (int k = 0; k < 32; k += 2) {   /* one table read per byte pair */
          const int32_t at = block_pos + 32 * w + k;   /* the bytes before the request read as 0 */
          st = T.b[st * kStride + (at < 0 ? 0u : cls[win[32 * w + k]]) * 16u + (at + 1 < 0 ? 0u : cls[win[32 * w + k + 1]])];
          ev |= (st & 3u) << k;
        }
        evw[w] = ev;
      }
      win += block;
      pos += block;
      const bool slow = is_slow2(st);
      const bool term_ev = is_done2(st) || is_err2(st);
      uint32_t term_pos = 0xffffffffu;
      if (term_ev) {   /* the terminal is the window's last event */
        for (int w = words - 1; w >= 0; w--)
          if (evw[w]) {
            const uint32_t bt = 31u - (uint32_t) __builtin_clz(evw[w]);
            term_pos = (uint32_t) (block_pos + 32 * w) + bt;
            evw[w] &= ~(1u << bt);
            break;
          }
      }
      for (int w = 0; w < words && !slow; w++) {
        uint32_t m = evw[w];
        while (m && !d.ovf) {
          const uint32_t bit = (uint32_t) __builtin_ctz(m);
          m &= m - 1;
          uint32_t lo, hi;
          if (dec_event(d, (uint32_t) (block_pos + 32 * w) + bit, maxh, lo, hi)) {
            if (compact) {   /* as the kernel: the two lengths (rhp.h RHP_LAYOUT_COMPACT) */
              lens[(uint64_t) (d.nh - 1) * b->n] = (lo >> 16) | (hi & 0xffff0000u);
            } else if (dense) {   /* name_len | value_len << 6 (rhp.h RHP_LAYOUT_DENSE), or the overflow area */
              const uint32_t nl = lo >> 16, vl = hi >> 16, at = (d.nh - 1) * dstride;
              const bool fits = std::max(nl << 4, vl) <= RHP_DENSE_VALUE_MAX;
              lens16[at] = (uint16_t) (fits ? nl | vl << 6 : RHP_DENSE_OVERFLOW);
              if (!fits) ovf32[at] = nl | vl << 16;
            } else {
              rhp_hdr_t &o = hout[(uint64_t) (d.nh - 1) * hs_hdr];
              o.name_off = (uint16_t) lo;
              o.name_len = (uint16_t) (lo >> 16);
              o.value_off = (uint16_t) hi;
              o.value_len = (uint16_t) (hi >> 16);
            }
          }
        }
      }
      const bool ovf = d.ovf != 0;
      if (!(ovf || slow || term_ev || pos >= (int32_t) len)) continue;
      /* ---- finalize (same decisions as the kernel) ---- */
      bool ok = !ovf && is_done2(st) && term_pos < len && term_pos < RHP_MAX_LEN;
      /* an ERR in the version (request line events ME, PE consumed) needs the
       * version's 9 bytes: len >= PE + 10 (picohttpparser.c:248-251) */
      bool bad = ovf ? d.ovf - 1u < len
                     : (is_err2(st) && term_pos < len && (d.k != 2 || d.e[0] + 10u <= len));
      if (b->mode == RHP_MODE_PHR && b->last_len && b->last_len[i] != 0) {   /* as the kernel's decode_end */
        ok = ok && (b->last_len[i] < 3u || b->last_len[i] <= term_pos);
        bad = false;
      }
      if (ok && dense && (d.rl01 & 0xffffu) > 255u) {
        /* as the kernel: a method longer than the dense record holds takes the exact path (wide) */
        st_count.exact++;
        emu_exact(b, i, off, len);
        break;
      }
      if (ok) {
        st_count.fast_ok++;
        rhp_req_t r;
        r.ret = (int32_t) term_pos + 1;
        r.method_off = 0;
        r.method_len = (uint16_t) d.rl01;
        r.path_off = (uint16_t) (d.rl01 >> 16);
        r.path_len = (uint16_t) d.rl23;
        r.minor_version = (int8_t) (d.rl23 >> 16);
        r.num_headers = (uint16_t) d.nh;
        r.flags = 0;
        if (dense)
          dense_reqs(b)[i] = rhp_req_dense_t{(uint16_t) r.ret, r.path_len, (uint8_t) r.method_len, (uint8_t) r.num_headers,
                                             (uint8_t) r.minor_version, 0};
        else
          b->reqs[i] = r;
        if (b->mode == RHP_MODE_HTTP && (compact || dense)) {
          /* as the kernel: with compact records a request that is not GET and
           * has three or more framing candidates (names of 14 or 17 bytes), or
           * one at header index >= 30, is framed by the exact path (its http_frame
           * has no rhp_hdr_t records to read) */
          uint32_t ncand = 0;
          bool late = false;
          for (uint32_t k = 0; k < d.nh && k < maxh; k++) {
            const uint32_t nl = len32(k) & 0xffffu;
            if (nl == 14u || nl == 17u) {
              ncand++;
              late |= k >= 30u;
            }
          }
          const bool get = len >= 4 && memcmp(b->bytes + off, "GET ", 4) == 0;
          if (!get && (ncand >= 3 || late)) {
            st_count.fast_ok--;
            st_count.exact++;
            emu_exact(b, i, off, len);
            break;
          }
        }
        if (b->mode == RHP_MODE_HTTP) {
          rhp_http_t x;
          if (compact || dense) {   /* http_frame reads rhp_hdr_t records: the lengths expanded */
            rhp_hdr_t tmp[RHP_MAX_HEADERS];
            uint32_t at = (uint32_t) r.path_off + r.path_len + 11u;
            for (uint32_t k = 0; k < d.nh && k < maxh; k++) {
              const uint32_t l = len32(k), nl = l & 0xffffu, vl = l >> 16;
              tmp[k] = rhp_hdr_t{(uint16_t) at, (uint16_t) nl, (uint16_t) (at + nl + 2u), (uint16_t) vl};
              at += nl + vl + 4u;
            }
            http_frame(b->bytes_rw + off, len, r, tmp, 1u, &x, ~0ull, !(b->flags & RHP_BATCH_SPECULATIVE));
          } else {
            http_frame(b->bytes_rw + off, len, r, hout, hs_hdr, &x, ~0ull, !(b->flags & RHP_BATCH_SPECULATIVE));
          }
          put_http(b, i, x, x.consumed != compact_consumed(r.ret, x) || x.body_len > 0xffffffffull);
        }
      } else if (bad) {
        st_count.fast_bad++;
        rhp_req_t r;
        memset(&r, 0, sizeof r);
        r.ret = -1;
        r.minor_version = -1;
        if (dense) dense_reqs(b)[i] = rhp_req_dense_t{0, 0, 0, 0, 0, (uint8_t) RHP_DENSE_BAD};
        else b->reqs[i] = r;
        if (b->mode == RHP_MODE_HTTP) {
          rhp_http_t x;
          memset(&x, 0, sizeof x);
          x.result = -1;
          put_http(b, i, x, false);
        }
      } else {
        st_count.exact++;
        emu_exact(b, i, off, len);
      }
      break;
    }
  }
  if (stats) {
    stats[0] = st_count.fast_ok;
    stats[1] = st_count.fast_bad;
    stats[2] = st_count.exact;
  }
  return 0;
}

/* test hook: one_chunk_window over the nw (<= 32) bytes at `line`
 * (tests/test_cpu_units.py compares it with one_chunk_t); returns 0 when the
 * window cannot decide */
extern "C" int rhp_test_chunk_window(const uint8_t *line, uint32_t nw, uint64_t avail, int64_t *res, uint64_t *doff,
                                     uint64_t *dlen)
{
  uint32_t W[8];
  memcpy(W, line, 32);
  return one_chunk_window(W, nw, avail, res, doff, dlen) ? 1 : 0;
}

/* test hook: one_chunk_head over the first 4 * nd bytes at `line` (nd 5: the
 * GPU replay's 20-byte window, or 8); returns 0 when it leaves the line to
 * one_chunk_window */
extern "C" int rhp_test_chunk_head(const uint8_t *line, uint32_t nw, uint64_t avail, int64_t *res, uint64_t *doff,
                                   uint64_t *dlen, uint32_t nd)
{
  uint32_t W[8];
  memcpy(W, line, 32);
  return (nd == 5 ? one_chunk_head<5>(W, nw, avail, res, doff, dlen) : one_chunk_head<8>(W, nw, avail, res, doff, dlen))
             ? 1 : 0;
}

/* test hook: the pair table the kernel copies into LDS (rhp_dfa.h make_table2)
 * and its geometry: meta = {bytes, row stride, kClassRowR, kClassRow, idx2(S_SLOW, 1), kClassRow16} */
extern "C" uint32_t rhp_test_table2(uint8_t *out, uint32_t *meta)
{
  const Table2 &t = table();
  if (out) memcpy(out, t.b, kTable2Bytes);
  if (meta) {
    meta[0] = kTable2Bytes;
    meta[1] = kStride;
    meta[2] = kClassRowR;
    meta[3] = kClassRow;
    meta[4] = idx2(S_SLOW, 1);
    meta[5] = kClassRow16;
  }
  return kTable2Bytes;
}

/* test hook: one_chunk_t over `body` (size bytes, readable to size + 64) */
extern "C" int64_t rhp_test_chunk_exact(const uint8_t *body, uint64_t at, uint64_t size, uint64_t *doff, uint64_t *dlen)
{
  PlainBytes B{body};
  return one_chunk_t(B, at, size, doff, dlen);
}

extern "C" int rhp_expand_records(const rhp_batch_t *b, const rhp_req_t *reqs, const void *hdrs, rhp_hdr_t *out)
{
  if (!b || !reqs || !out || (b->max_headers && !hdrs)) return -22;
  const uint32_t n = b->n, m = b->max_headers;
  const bool hmajor = b->layout == RHP_LAYOUT_HEADER_MAJOR, dense = dense_layout(b);
  const bool compact = b->layout == RHP_LAYOUT_COMPACT || dense, drm = b->layout == RHP_LAYOUT_DENSE_RM;
  if (!hmajor && !compact && b->layout != RHP_LAYOUT_REQUEST_MAJOR) return -22;
  const rhp_hdr_t *h = static_cast<const rhp_hdr_t *>(hdrs);
  const uint32_t *lens = static_cast<const uint32_t *>(hdrs);
  const uint16_t *lens16 = static_cast<const uint16_t *>(hdrs);
  const uint32_t *ovf32 = reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(hdrs) + RHP_DENSE_OVF_OFF(n, m));
  const rhp_hdr_t *wide = reinterpret_cast<const rhp_hdr_t *>(
      static_cast<const uint8_t *>(hdrs) + (dense ? RHP_DENSE_WIDE_OFF(n, m) : RHP_COMPACT_WIDE_OFF(n, m)));
  for (uint32_t i = 0; i < n; i++) {
    rhp_hdr_t *o = out + (uint64_t) i * m;
    memset(o, 0, sizeof(rhp_hdr_t) * m);
    const rhp_req_t &r = reqs[i];
    if (r.ret <= 0) continue;
    const uint32_t nh = r.num_headers < m ? r.num_headers : m;
    if (compact && !(r.flags & RHP_F_WIDE)) {
      uint32_t at = (uint32_t) r.path_off + r.path_len + 11u;   /* the first header line (rhp.h) */
      for (uint32_t k = 0; k < nh; k++) {
        uint32_t nl, vl;
        if (dense) {
          const uint64_t at = drm ? (uint64_t) i * m + k : (uint64_t) k * n + i;
          const uint32_t l = lens16[at], o = l == RHP_DENSE_OVERFLOW ? ovf32[at] : (l & 63u) | (l >> 6) << 16;
          nl = o & 0xffffu;
          vl = o >> 16;
        } else {
          const uint32_t l = lens[(uint64_t) k * n + i];
          nl = l & 0xffffu;
          vl = l >> 16;
        }
        o[k] = rhp_hdr_t{(uint16_t) at, (uint16_t) nl, (uint16_t) (at + nl + 2u), (uint16_t) vl};
        at += nl + vl + 4u;
      }
    } else {
      for (uint32_t k = 0; k < nh; k++)
        o[k] = compact ? wide[(uint64_t) i * m + k] : hmajor ? h[(uint64_t) k * n + i] : h[(uint64_t) i * m + k];
    }
  }
  return 0;
}

extern "C" int rhp_expand_reqs(const rhp_batch_t *b, const void *reqs, rhp_req_t *out)
{
  if (!b || !reqs || !out) return -22;
  if (!dense_layout(b)) {
    memcpy(out, reqs, sizeof(rhp_req_t) * b->n);
    return 0;
  }
  const rhp_req_dense_t *d = static_cast<const rhp_req_dense_t *>(reqs);
  const rhp_req_t *wide = reinterpret_cast<const rhp_req_t *>(static_cast<const uint8_t *>(reqs) + RHP_DENSE_REQ_WIDE_OFF(b->n));
  for (uint32_t i = 0; i < b->n; i++) {
    rhp_req_t r;
    memset(&r, 0, sizeof r);
    if (d[i].flags & RHP_DENSE_WIDE) {
      r = wide[i];
    } else if (d[i].flags & RHP_DENSE_BAD) {
      r.ret = -1;
      r.minor_version = -1;
    } else {
      r.ret = d[i].ret;
      r.method_len = d[i].method_len;
      r.path_off = (uint16_t) (d[i].method_len + 1u);
      r.path_len = d[i].path_len;
      r.minor_version = (int8_t) d[i].minor_version;
      r.num_headers = d[i].num_headers;
    }
    out[i] = r;
  }
  return 0;
}

extern "C" int rhp_expand_http(const rhp_batch_t *b, const rhp_req_t *reqs, const void *http, rhp_http_t *out)
{
  if (!b || !reqs || !http || !out) return -22;
  if (b->layout != RHP_LAYOUT_COMPACT && b->layout != RHP_LAYOUT_DENSE) {
    memcpy(out, http, sizeof(rhp_http_t) * b->n);
    return 0;
  }
  const rhp_http_compact_t *c = static_cast<const rhp_http_compact_t *>(http);
  const rhp_http_t *wide = reinterpret_cast<const rhp_http_t *>(static_cast<const uint8_t *>(http) + RHP_COMPACT_HTTP_WIDE_OFF(b->n));
  for (uint32_t i = 0; i < b->n; i++) {
    if (c[i].flags & RHP_HTTP_WIDE) {
      out[i] = wide[i];
      continue;
    }
    rhp_http_t x = {c[i].result, c[i].body_kind, 0, c[i].body_len};
    x.consumed = compact_consumed(reqs[i].ret, x);
    out[i] = x;
  }
  return 0;
}

/* rhp_pack_dense (rhp.h) on the host: the same encodings as the kernel's
 * (rhp_kernel.hip rhp_pack_dense_kernel), for the reactor's host-async parser */
extern "C" int rhp_cpu_pack_dense(const rhp_batch_t *b, rhp_req_dense_t *dreq, rhp_http_compact_t *hc, uint16_t *lens16)
{
  if (!b || b->mode != RHP_MODE_HTTP || b->layout != RHP_LAYOUT_REQUEST_MAJOR || b->max_headers > RHP_MAX_HEADERS) return -22;
  const uint32_t n = b->n, m = b->max_headers;
  for (uint32_t i = 0; i < n; i++) {
    const rhp_req_t r = b->reqs[i];
    const rhp_http_t x = b->http[i];
    const uint64_t cons = x.result == 1 ? (uint64_t) (uint32_t) r.ret + (x.body_kind == 1 ? x.body_len : 0u) : 0u;
    const bool hok = x.consumed == cons && x.body_kind <= 1u && !(x.body_len >> 32) && (x.result != 1 || r.ret > 0);
    hc[i] = hok ? rhp_http_compact_t{(int8_t) x.result, (uint8_t) x.body_kind, 0, 0, (uint32_t) x.body_len}
                : rhp_http_compact_t{0, 0, (uint8_t) RHP_HTTP_WIDE, 0, 0};
    bool reg = hok && x.result == 1 && r.ret > 0 && r.ret <= (int32_t) RHP_MAX_LEN && r.method_off == 0 && r.method_len <= 255u &&
               r.path_off == r.method_len + 1u && r.num_headers <= m;
    uint32_t at = (uint32_t) r.path_off + r.path_len + 11u;
    const uint32_t nh = reg ? r.num_headers : 0u;
    for (uint32_t k = 0; k < nh; k++) {
      const rhp_hdr_t h = b->hdrs[(uint64_t) i * m + k];
      reg = reg && h.name_off == at && h.value_off == at + h.name_len + 2u &&
            std::max((uint32_t) h.name_len << 4, (uint32_t) h.value_len) <= RHP_DENSE_VALUE_MAX;
      at += (uint32_t) h.name_len + h.value_len + 4u;
      lens16[(uint64_t) k * n + i] = (uint16_t) (h.name_len | (uint32_t) h.value_len << 6);
    }
    dreq[i] = reg ? rhp_req_dense_t{(uint16_t) r.ret, r.path_len, (uint8_t) r.method_len, (uint8_t) r.num_headers,
                                    (uint8_t) r.minor_version, 0}
                  : rhp_req_dense_t{0, 0, 0, 0, 0, (uint8_t) RHP_DENSE_WIDE};
  }
  return 0;
}

/* rhp_fixup_sessions (rhp.h) on the host: the same walk (rhp_scalar.h
 * fixup_session_t) over a speculative batch parsed by rhp_cpu_parse_batch or
 * rhp_emu_parse_batch. */
extern "C" int rhp_cpu_fixup_sessions(const rhp_batch_t *b, const rhp_session_t *sessions, uint32_t n_sessions,
                                      rhp_session_result_t *results, uint64_t *req_start)
{
  if (!b || b->mode != RHP_MODE_HTTP || !(b->flags & RHP_BATCH_SPECULATIVE)) return -22;
  const bool hmajor = b->layout == RHP_LAYOUT_HEADER_MAJOR;
  const FixupIO io{b->bytes_rw, b->offsets, b->reqs, b->hdrs, b->http, hmajor ? 1u : b->max_headers,
                   hmajor ? (uint64_t) b->n : 1u, b->max_headers};
  for (uint32_t k = 0; k < n_sessions; k++)
    fixup_session_t(io, sessions[k].piece_lo, sessions[k].piece_hi, req_start, &results[k],
                    [&](uint64_t at) { return PlainBytes{b->bytes_rw + at}; });
  return 0;
}

/* The exact scalar path alone, on the host (the product's CPU parser). */
extern "C" int rhp_cpu_parse_batch(const rhp_batch_t *b)
{
  /* as rhp_parse_batch: compact records in both modes (every record wide: the
   * exact path's), not in a speculative batch */
  if (b->layout == RHP_LAYOUT_COMPACT && (b->flags & RHP_BATCH_SPECULATIVE)) return -22;
  if (dense_layout(b) && ((b->layout == RHP_LAYOUT_DENSE_RM && b->mode != RHP_MODE_PHR) || (b->flags & RHP_BATCH_SPECULATIVE)))
    return -22;
  for (uint32_t i = 0; i < b->n; i++) emu_exact(b, i, b->offsets[i], b->offsets[i + 1] - b->offsets[i]);
  return 0;
}

/* ---- the pointer-based host parser: phr_parse_request's own outputs ---- */

namespace {

/* rhp_scalar.h output policy writing phr_parse_request's outputs (pointers
 * into buf, size_t lengths): no length limit */
struct OutPhr {
  const uint8_t *base;
  const char **method;
  size_t *method_len;
  const char **path;
  size_t *path_len;
  int *minor_version;
  rhp_phr_header_t *h;
  size_t *num_headers;
  void begin()
  {
    *method = nullptr; *method_len = 0; *path = nullptr; *path_len = 0;   /* picohttpparser.c:390-395 */
    *minor_version = -1; *num_headers = 0;
  }
  int fail(int code) { return code; }
  void header(uint32_t n, bool fold, uint64_t name, uint64_t name_len, uint64_t vs, uint64_t vlen)
  {
    h[n].name = fold ? nullptr : (const char *) base + name;
    h[n].name_len = (size_t) name_len;
    h[n].value = (const char *) base + vs;
    h[n].value_len = (size_t) vlen;
  }
  int done(uint64_t p, const uint64_t (&tok)[2][2], int minor, uint32_t n)
  {
    *method = (const char *) base + tok[0][0];
    *method_len = (size_t) (tok[0][1] - tok[0][0]);
    *path = (const char *) base + tok[1][0];
    *path_len = (size_t) (tok[1][1] - tok[1][0]);
    *minor_version = minor;
    *num_headers = n;
    return (int) p;
  }
};

/* rhp_scalar.h header view over phr_header records */
struct HdrsPhr {
  const rhp_phr_header_t *h;
  bool null(uint32_t i) const { return h[i].name == nullptr; }
  const uint8_t *name(uint32_t i) const { return (const uint8_t *) h[i].name; }
  uint64_t name_len(uint32_t i) const { return h[i].name_len; }
  const uint8_t *value(uint32_t i) const { return (const uint8_t *) h[i].value; }
  uint64_t value_len(uint32_t i) const { return h[i].value_len; }
};

}  // namespace

extern "C" int rhp_phr_parse_request(const char *buf, size_t len, const char **method, size_t *method_len,
                                     const char **path, size_t *path_len, int *minor_version,
                                     rhp_phr_header_t *headers, size_t *num_headers, size_t last_len)
{
  const uint8_t *b = (const uint8_t *) buf;
  const size_t max = *num_headers;
  OutPhr o{b, method, method_len, path, path_len, minor_version, headers, num_headers};
  if (last_len != 0) {   /* picohttpparser.c:399-401 */
    o.begin();
    const int r = is_complete(b, len, last_len);
    if (r != 0) return r;
  }
  PlainBytes B{b};
  return scalar_phr_t(B, len, (uint32_t) (max < 0xffffffffu ? max : 0xffffffffu), o);
}

extern "C" int rhp_http_read_cpu(uint8_t *buf, size_t len, rhp_http_req_t *req, rhp_phr_header_t *fields,
                                 size_t *fields_count)
{
  if (len == 0) return 0;                               /* http.c:184-186 */
  const int n = rhp_phr_parse_request((const char *) buf, len, &req->method, &req->method_len, &req->target,
                                      &req->target_len, &req->minor_version, fields, fields_count, 0);
  if (n <= 0) return n == kBad ? -1 : 0;                /* http.c:194-195 */
  const bool get = req->method_len == 3 && memcmp(req->method, "GET", 3) == 0;
  rhp_http_t x;
  http_frame_t(buf, len, n, get, HdrsPhr{fields}, (uint32_t) *fields_count, &x);
  req->body = x.body_kind ? buf + n : nullptr;
  req->body_len = x.body_kind ? (size_t) x.body_len : 0;
  req->consumed = x.consumed;
  return x.result;
}
