/*
 * rhp_emu.cpp -- CPU emulation of rhp_dfa_kernel, for tests only.
 *
 * Runs the same transition table (rhp_dfa.h), the same 4-byte window alignment
 * (SKIP states), 64-byte blocks with a header-capacity check every 16 bytes,
 * the same capture-area layout and the same finalize decisions as the kernel,
 * one request at a time on the host.  Lets the DFA design be checked against
 * the oracle on millions of requests without a GPU; the GPU tests then check
 * the kernel itself.
 */
#include <stdint.h>
#include <string.h>
#include <vector>

#include "rhp.h"
#include "rhp_dfa.h"
#include "rhp_scalar.h"

using namespace rhp;

namespace {

const Table &table()
{
  static const Table t = make_table();
  return t;
}

struct Stats {
  uint64_t fast_ok, fast_bad, exact;
};

void emu_exact(const rhp_batch_t *b, uint32_t i, uint64_t off, uint64_t len)
{
  rhp_req_t r;
  r.flags = RHP_F_EXACT;
  rhp_hdr_t *h = b->hdrs + (uint64_t) i * b->max_headers;
  if (len > RHP_MAX_LEN) {
    memset(&r, 0, sizeof r);
    r.ret = RHP_RET_TOOLONG;
    r.minor_version = -1;
    r.flags = RHP_F_EXACT;
    b->reqs[i] = r;
    if (b->mode == RHP_MODE_HTTP) memset(&b->http[i], 0, sizeof b->http[i]);
    return;
  }
  if (b->mode == RHP_MODE_HTTP) scalar_http(b->bytes_rw + off, len, b->max_headers, &r, h, &b->http[i]);
  else scalar_phr(b->bytes + off, len, b->max_headers, &r, h);
  b->reqs[i] = r;
}

}  // namespace

extern "C" int rhp_emu_parse_batch(const rhp_batch_t *b, uint64_t *stats /* [3] or NULL */)
{
  const Table &T = table();
  const uint32_t cap_lane = (cap_bytes(b->max_headers) + 15u) & ~15u;
  std::vector<uint8_t> area(cap_lane + 64);
  Stats st_count = {0, 0, 0};
  auto ld16 = [&](uint32_t a) { uint16_t v; memcpy(&v, &area[a], 2); return (uint32_t) v; };
  auto st16 = [&](uint32_t a, uint32_t v) { uint16_t x = (uint16_t) v; memcpy(&area[a], &x, 2); };
  const uint32_t cap0 = 0;
  const uint32_t cap_limit = b->max_headers ? cap0 + kRlBytes + kHdrBytes * (b->max_headers - 1) : cap0;

  for (uint32_t i = 0; i < b->n; i++) {
    uint64_t off = b->offsets[i], len = b->offsets[i + 1] - off;
    uint32_t mis = (uint32_t) off & 3u;
    const uint8_t *win = b->bytes + (off - mis);
    int32_t pos = -(int32_t) mis;
    uint32_t s0 = mis == 0 ? S_START : mis == 1 ? S_SKIP1 : mis == 2 ? S_SKIP2 : S_SKIP3;
    if (len > RHP_MAX_LEN - 256) s0 = S_SLOW;
    uint32_t st = entry(s0, C_NONE_RL);
    uint32_t cap = cap0;
    /* stale garbage everywhere except the VE slots: the kernel only re-zeroes VE */
    memset(area.data(), 0xA5, cap_lane);
    for (uint32_t a = kRlBytes + C_VE; a + 2 <= cap_lane; a += kHdrBytes) st16(a, 0);
    /* blocks until terminal or past the end (block boundary checks) */
    for (;;) {
      if (is_terminal_row(entry_next(st)) || pos >= (int32_t) len) break;
      for (int q = 0; q < 4; q++) {
        for (int k = 0; k < 16; k++) {
          uint32_t c = win[16 * q + k];
          uint32_t e = T.w[(entry_next(st) >> 2) + c];
          cap += entry_inc(e);
          if (cap + entry_slot(e) + 2 > cap_lane) return -1000 - (int) i;  /* capture overflow: design bug */
          st16(cap + entry_slot(e), (uint32_t) pos);
          pos++;
          st = e;
        }
        if (cap > cap_limit && !is_terminal_row(entry_next(st)))
          st = entry(pos <= (int32_t) len ? S_OVF : S_SLOW, C_NONE_T);
      }
      win += 64;
    }
    /* finalize (same decisions as the kernel's finalize) */
    uint32_t row = entry_next(st);
    uint32_t count = cap == cap0 ? 0u : (cap - cap0 - kRlBytes) / kHdrBytes + 1u;
    uint32_t term = ld16(cap == cap0 ? cap0 + C_TERM_RL : cap + C_TERM_H);
    bool ok = row == row_of(S_DONE) && term < len && count <= b->max_headers;
    bool bad = (row == row_of(S_DONE) && term < len && count > b->max_headers) ||
               (row == row_of(S_ERR1) && term < len) || row == row_of(S_OVF);
    if (ok) {
      st_count.fast_ok++;
      rhp_req_t r;
      uint32_t ms = ld16(C_MS), me = ld16(C_ME), ps = ld16(C_PS), pe = ld16(C_PE), vd = ld16(C_VD);
      r.ret = (int32_t) term + 1;
      r.method_off = (uint8_t) ms;
      r.method_len = (uint16_t) (me - ms);
      r.path_off = (uint16_t) ps;
      r.path_len = (uint16_t) (pe - ps);
      r.minor_version = (int8_t) (b->bytes[off + vd] - '0');
      r.num_headers = (uint16_t) count;
      r.flags = 0;
      b->reqs[i] = r;
      rhp_hdr_t *h = b->hdrs + (uint64_t) i * b->max_headers;
      for (uint32_t k = 0; k < count; k++) {
        uint32_t rec = cap0 + kRlBytes + kHdrBytes * k;
        uint32_t ls = ld16(rec + C_LS), co = ld16(rec + C_CO), vs = ld16(rec + C_VS), ve = ld16(rec + C_VE);
        h[k].name_off = (uint16_t) ls;
        h[k].name_len = (uint16_t) (co - ls);
        h[k].value_off = (uint16_t) vs;
        h[k].value_len = (uint16_t) (ve > vs ? ve - vs : 0);
      }
      if (b->mode == RHP_MODE_HTTP) http_frame(b->bytes_rw + off, len, r, h, &b->http[i]);
    } else if (bad) {
      st_count.fast_bad++;
      rhp_req_t r;
      memset(&r, 0, sizeof r);
      r.ret = -1;
      r.minor_version = -1;
      b->reqs[i] = r;
      if (b->mode == RHP_MODE_HTTP) {
        memset(&b->http[i], 0, sizeof b->http[i]);
        b->http[i].result = -1;
      }
    } else {
      st_count.exact++;
      emu_exact(b, i, off, len);
    }
  }
  if (stats) {
    stats[0] = st_count.fast_ok;
    stats[1] = st_count.fast_bad;
    stats[2] = st_count.exact;
  }
  return 0;
}

/* The exact scalar path alone, on the host (the product's CPU parser). */
extern "C" int rhp_cpu_parse_batch(const rhp_batch_t *b)
{
  for (uint32_t i = 0; i < b->n; i++) emu_exact(b, i, b->offsets[i], b->offsets[i + 1] - b->offsets[i]);
  return 0;
}
