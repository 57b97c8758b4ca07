/*
 * rhp_gen.c -- deterministic synthetic HTTP/1.1 request batches (host C).
 *
 * Shapes follow SURVEY.md §8d / BASELINE.json configs:
 *   1  TFB128 : the 128 B TechEmpower /plaintext GET whose known answer is
 *               ret=128 method=(0,3) path=(4,10) minor=1, 4 headers
 *   2  GET256 : same template, path padded to 138 B of seeded URL characters
 *   3  ZIPF   : lengths L = 64k-u, k~Zipf(1.2) on [1,64], u~U[0,63] (clamped to
 *               the 18 B minimal request), 0..32 headers, fill in path/values
 *   5  POST1K : 1 KiB POST with Content-Length body, 5 % seeded malformed
 *               (HTTP/2.0, CTL in value, SP before ':', CL+TE, missing ':')
 *   6  CHUNKED: ~1 KiB POST, Transfer-Encoding: chunked, 1-8 chunks of seeded
 *               data; chunk lines with extensions, OWS and either hex case;
 *               5 % seeded malformed framing (bad hex, bare LF, a size past
 *               the input, a coding other than chunked)
 *   100/101   : structured random edge cases for parity (every §8a hazard)
 * Every request depends only on (config, seed, index): shards are independent.
 */
#include "rhp_gen.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

uint64_t rhp_splitmix64(uint64_t *s)
{
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

typedef struct {
  uint64_t s;
} rng_t;

static rng_t rng_for(uint64_t seed, uint64_t idx, int config)
{
  rng_t r = {seed ^ (idx * 0xD1B54A32D192ED03ull) ^ ((uint64_t) config << 56)};
  rhp_splitmix64(&r.s);
  return r;
}
static uint64_t rnd(rng_t *r) { return rhp_splitmix64(&r->s); }
static uint32_t rndu(rng_t *r, uint32_t n) { return n ? (uint32_t) (rnd(r) % n) : 0; }
static int chance(rng_t *r, uint32_t pct) { return rndu(r, 100) < pct; }

/* output builder; buf == NULL sizes only */
typedef struct {
  uint8_t *buf;
  size_t len, cap;
} bld_t;

static void put(bld_t *b, const void *p, size_t n)
{
  if (b->buf && b->len + n <= b->cap)
    memcpy(b->buf + b->len, p, n);
  b->len += n;
}
static void puts_(bld_t *b, const char *s) { put(b, s, strlen(s)); }
static void putc_(bld_t *b, uint8_t c) { put(b, &c, 1); }

static const char URL_CHARS[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-._~/";
static const char VAL_CHARS[] =
    "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-._~/:;,=+*()!?@#$%&'\"<>[]{}|^`\\";
static const char TCHARS[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789!#$%&'*+-.^_`|~";

static void put_rand(bld_t *b, rng_t *r, const char *alphabet, size_t n)
{
  size_t a = strlen(alphabet);
  for (size_t i = 0; i < n; i++)
    putc_(b, (uint8_t) alphabet[rndu(r, (uint32_t) a)]);
}

/* ---------------- config 1/2: TechEmpower plaintext GET ---------------- */

static const char *TFB_HEADERS =
    "Host: tfb-server:8080\r\n"
    "Accept: text/plain\r\n"
    "Connection: keep-alive\r\n"
    "User-Agent: wrk/4.2.0 (tfb-load)\r\n"
    "\r\n";

static size_t gen_tfb(bld_t *b, rng_t *r, size_t path_len)
{
  size_t start = b->len;
  puts_(b, "GET ");
  if (path_len == 10) {
    puts_(b, "/plaintext");
  } else {
    putc_(b, '/');
    put_rand(b, r, URL_CHARS, path_len - 1);
  }
  puts_(b, " HTTP/1.1\r\n");
  puts_(b, TFB_HEADERS);
  return b->len - start;
}

/* ---------------- config 3: Zipf mixed lengths ---------------- */

static const char *NAMES[] = {"Host", "Accept", "Connection", "User-Agent", "Accept-Encoding",
                              "Accept-Language", "Cookie", "X-Request-Id", "Cache-Control", "Referer",
                              "Content-Type", "Authorization", "If-None-Match", "X-Forwarded-For",
                              "Pragma", "DNT", "TE", "Origin", "Sec-Fetch-Mode", "Upgrade-Insecure-Requests"};
#define NNAMES (sizeof NAMES / sizeof *NAMES)
static const char *METHODS[] = {"GET", "GET", "GET", "GET", "GET", "GET", "GET", "POST", "PUT", "HEAD",
                                "DELETE", "OPTIONS", "PATCH"};
#define NMETHODS (sizeof METHODS / sizeof *METHODS)

static double zipf_cdf[65];
static int zipf_ready;

static uint32_t zipf_bucket(rng_t *r)
{
  if (!zipf_ready) {
    double t = 0;
    for (int k = 1; k <= 64; k++) t += pow((double) k, -1.2);
    double c = 0;
    for (int k = 1; k <= 64; k++) {
      c += pow((double) k, -1.2) / t;
      zipf_cdf[k] = c;
    }
    zipf_cdf[64] = 1.0;
    zipf_ready = 1;
  }
  double u = (double) (rnd(r) >> 11) * (1.0 / 9007199254740992.0);
  for (uint32_t k = 1; k <= 64; k++)
    if (u < zipf_cdf[k]) return k;
  return 64;
}

#define ZIPF_MIN 18 /* "GET / HTTP/1.1\r\n\r\n" */

static size_t gen_zipf(bld_t *b, rng_t *r)
{
  size_t start = b->len;
  uint32_t k = zipf_bucket(r);
  size_t L = 64 * (size_t) k - rndu(r, 64);
  const char *method = METHODS[rndu(r, NMETHODS)];
  size_t base = strlen(method) + 1 + 1 + 1 + 8 + 2 + 2; /* "M / HTTP/1.1\r\n" ... "\r\n" */
  if (L < base) L = base;
  uint32_t want = rndu(r, 33);
  const char *names[32];
  uint32_t h = 0;
  for (uint32_t i = 0; i < want; i++) {
    const char *nm = NAMES[rndu(r, NNAMES)];
    size_t need = strlen(nm) + 2 + 1 + 2;
    if (base + need > L) break;
    names[h++] = nm;
    base += need;
  }
  size_t extra = L - base;
  /* split the extra bytes: path gets a random share, values the rest */
  size_t path_extra = h ? (size_t) rndu(r, (uint32_t) extra + 1) : extra;
  size_t left = extra - path_extra;
  puts_(b, method);
  putc_(b, ' ');
  putc_(b, '/');
  put_rand(b, r, URL_CHARS, path_extra);
  puts_(b, " HTTP/1.1\r\n");
  for (uint32_t i = 0; i < h; i++) {
    size_t v = 1 + (i + 1 == h ? left : (size_t) rndu(r, (uint32_t) left + 1));
    left -= v - 1;
    puts_(b, names[i]);
    puts_(b, ": ");
    /* printable value, interior spaces allowed, first/last byte non-space */
    for (size_t j = 0; j < v; j++) {
      uint8_t c = (uint8_t) VAL_CHARS[rndu(r, sizeof VAL_CHARS - 1)];
      if (j > 0 && j + 1 < v && chance(r, 8)) c = ' ';
      putc_(b, c);
    }
    puts_(b, "\r\n");
  }
  puts_(b, "\r\n");
  return b->len - start;
}

/* ---------------- config 5: 1 KiB POST with Content-Length ---------------- */

static size_t gen_post(bld_t *b, rng_t *r, size_t *hdr_bytes)
{
  size_t start = b->len;
  const size_t total = 1024;
  int bad = chance(r, 5) ? 1 + (int) rndu(r, 5) : 0;
  puts_(b, "POST /upload ");
  puts_(b, bad == 1 ? "HTTP/2.0\r\n" : "HTTP/1.1\r\n");
  if (bad == 3) puts_(b, "Host : tfb-server:8080\r\n");
  else if (bad == 5) puts_(b, "Host tfb-server:8080\r\n");
  else if (bad == 2) puts_(b, "Host: tfb-\x01server:8080\r\n");
  else puts_(b, "Host: tfb-server:8080\r\n");
  puts_(b, "Content-Type: application/octet-stream\r\n");
  puts_(b, "Connection: keep-alive\r\n");
  if (bad == 4) puts_(b, "Transfer-Encoding: chunked\r\n");
  /* header section length with a 3-digit Content-Length */
  size_t head = (b->len - start) + strlen("Content-Length: 000\r\n\r\n");
  char cl[32];
  size_t body = total - head;
  cl[0] = (char) ('0' + body / 100);
  cl[1] = (char) ('0' + body / 10 % 10);
  cl[2] = (char) ('0' + body % 10);
  cl[3] = 0;
  puts_(b, "Content-Length: ");
  puts_(b, cl);
  puts_(b, "\r\n\r\n");
  *hdr_bytes = b->len - start;
  for (size_t i = 0; i < body; i++) putc_(b, 'x');
  return b->len - start;
}

/* ---------------- chunked POST (Transfer-Encoding: chunked) ---------------- */

static void put_hex(bld_t *b, rng_t *r, uint32_t v)
{
  char t[16];
  int n = 0;
  const int upper_case = chance(r, 30);
  do {
    uint32_t d = v & 15u;
    t[n++] = (char) (d < 10 ? '0' + d : (upper_case ? 'A' : 'a') + d - 10);
    v >>= 4;
  } while (v);
  while (n) putc_(b, (uint8_t) t[--n]);
}

static size_t gen_chunked(bld_t *b, rng_t *r)
{
  size_t start = b->len;
  int bad = chance(r, 5) ? 1 + (int) rndu(r, 5) : 0;
  puts_(b, "POST /upload HTTP/1.1\r\n");
  puts_(b, "Host: tfb-server:8080\r\n");
  puts_(b, "Content-Type: application/octet-stream\r\n");
  puts_(b, "Connection: keep-alive\r\n");
  puts_(b, bad == 1 ? "Transfer-Encoding: gzip\r\n\r\n" : "Transfer-Encoding: chunked\r\n\r\n");
  const uint32_t k = 1 + rndu(r, 8);                 /* data chunks */
  const uint32_t payload = 640 + rndu(r, 256);       /* data bytes in all */
  const uint32_t bad_at = rndu(r, k);                /* the chunk a framing error goes in */
  uint32_t left = payload;
  uint64_t word = 0;
  for (uint32_t c = 0; c < k; c++) {
    uint32_t sz = c + 1 == k ? left : 1 + rndu(r, left - (k - 1 - c));
    left -= sz;
    if (chance(r, 4)) putc_(b, ' ');                  /* OWS before the size (isblank) */
    if (bad == 2 && c == bad_at) puts_(b, "zz");
    else put_hex(b, r, bad == 4 && c == bad_at ? sz + 4096 : sz);
    if (chance(r, 4)) putc_(b, '\t');                 /* OWS after it */
    if (chance(r, 10)) puts_(b, ";ext=1");            /* chunk extension */
    puts_(b, bad == 3 && c == bad_at ? "\n" : "\r\n");
    for (uint32_t i = 0; i < sz; i++) {
      if ((i & 7) == 0) word = rnd(r);
      putc_(b, (uint8_t) (0x21 + (word >> (8 * (i & 7))) % 94));
    }
    puts_(b, "\r\n");
  }
  puts_(b, bad == 5 ? "0;last\n\r\n" : "0\r\n\r\n");
  return b->len - start;
}

/* ---------------- edge-case fuzz ---------------- */

/* per-request noise level: clean requests inject no invalid bytes, so roughly
 * half of a fuzz batch parses successfully (ret > 0) */
static _Thread_local int fz_dirty;

static void fuzz_token(bld_t *b, rng_t *r, size_t maxlen)
{
  size_t n = rndu(r, (uint32_t) maxlen + 1);
  for (size_t i = 0; i < n; i++) {
    uint32_t p = rndu(r, 100);
    uint8_t c;
    if (!fz_dirty && p >= 94) p = rndu(r, 94);
    if (p < 80) c = (uint8_t) URL_CHARS[rndu(r, sizeof URL_CHARS - 1)];
    else if (p < 90) c = (uint8_t) (0x80 + rndu(r, 128));
    else if (p < 94) c = (uint8_t) VAL_CHARS[rndu(r, sizeof VAL_CHARS - 1)];
    else if (p < 96) c = 0x7f;
    else if (p < 98) c = (uint8_t) rndu(r, 0x20);
    else c = '\t';
    putc_(b, c);
  }
}

static void fuzz_eol(bld_t *b, rng_t *r)
{
  uint32_t p = rndu(r, fz_dirty ? 100 : 94);
  if (p < 80) puts_(b, "\r\n");
  else if (p < 94) puts_(b, "\n");
  else if (p < 97) puts_(b, "\r");
  else puts_(b, "\r\r\n");
}

static void fuzz_sps(bld_t *b, rng_t *r)
{
  uint32_t p = rndu(r, 100);
  size_t n = p < 85 ? 1 : p < 95 ? 2 + rndu(r, 3) : 0;
  for (size_t i = 0; i < n; i++) putc_(b, ' ');
}

static void fuzz_version(bld_t *b, rng_t *r)
{
  static const char *V[] = {"HTTP/1.1", "HTTP/1.1", "HTTP/1.1", "HTTP/1.0", "HTTP/1.9", "HTTP/1.10",
                            "HTTP/2.0", "HTTP/1.", "XTTP/1.1", "HTTP/1.x", "http/1.1", "HTTP/1",
                            "HTTP/11.1", "HTTP/1.1 "};
  puts_(b, V[rndu(r, fz_dirty ? sizeof V / sizeof *V : 4)]);
}

static void fuzz_value(bld_t *b, rng_t *r, size_t maxlen)
{
  size_t n = rndu(r, (uint32_t) maxlen + 1);
  for (size_t i = 0; i < n; i++) {
    uint32_t p = rndu(r, fz_dirty ? 1000 : 985);
    uint8_t c;
    if (p < 850) c = (uint8_t) VAL_CHARS[rndu(r, sizeof VAL_CHARS - 1)];
    else if (p < 920) c = ' ';
    else if (p < 950) c = '\t';
    else if (p < 985) c = (uint8_t) (0x80 + rndu(r, 128));
    else if (p < 992) c = 0x7f;
    else c = (uint8_t) rndu(r, 0x20);
    putc_(b, c);
  }
}

static void fuzz_name(bld_t *b, rng_t *r)
{
  uint32_t p = rndu(r, 100);
  if (p < 60) {
    puts_(b, NAMES[rndu(r, NNAMES)]);
  } else if (p < 70) {
    static const char *S[] = {"Content-Length", "content-length", "CONTENT-LENGTH", "Transfer-Encoding",
                              "transfer-encoding", "Content-Lengt", "Transfer-Encodings"};
    puts_(b, S[rndu(r, sizeof S / sizeof *S)]);
  } else if (p < 92 || !fz_dirty) {
    put_rand(b, r, TCHARS, 1 + rndu(r, 12));
  } else {
    fuzz_token(b, r, 8); /* may contain non-tchar / be empty */
  }
}

static void fuzz_cl_value(bld_t *b, rng_t *r, size_t body_len)
{
  static const char *S[] = {"", "0", "-1", "-0", "+5", "18446744073709551615", "18446744073709551616",
                            "99999999999999999999999", "12abc", " 7", "3 4", "0x10", "-18446744073709551615"};
  char num[32];
  uint32_t p = rndu(r, 100);
  if (p < 60) {
    size_t v = p < 50 ? body_len : rndu(r, 2000);
    int k = 0;
    char tmp[32];
    do { tmp[k++] = (char) ('0' + v % 10); v /= 10; } while (v);
    for (int i = 0; i < k; i++) num[i] = tmp[k - 1 - i];
    num[k] = 0;
    puts_(b, num);
  } else {
    puts_(b, S[rndu(r, sizeof S / sizeof *S)]);
  }
}

static void fuzz_chunked_body(bld_t *b, rng_t *r)
{
  uint32_t chunks = rndu(r, 4);
  for (uint32_t i = 0; i <= chunks; i++) {
    size_t sz = i == chunks ? 0 : 1 + rndu(r, 40);
    static const char HEX[] = "0123456789abcdefABCDEF";
    if (chance(r, 10)) puts_(b, chance(r, 50) ? " " : "\t");
    char tmp[20];
    int k = 0;
    size_t v = sz;
    int upper = chance(r, 30);
    do { tmp[k++] = HEX[(v % 16) + (upper && v % 16 >= 10 ? 6 : 0)]; v /= 16; } while (v);
    if (chance(r, 3)) puts_(b, "FFFFFFFFFFFFFFFFF");
    for (int j = k - 1; j >= 0; j--) putc_(b, (uint8_t) tmp[j]);
    uint32_t p = rndu(r, 100);
    if (p < 8) puts_(b, "; ext=1");
    else if (p < 11) puts_(b, " ");
    if (chance(r, 94)) puts_(b, "\r\n");
    else puts_(b, chance(r, 50) ? "\n" : "\r \n");
    for (size_t j = 0; j < sz; j++) putc_(b, (uint8_t) VAL_CHARS[rndu(r, sizeof VAL_CHARS - 1)]);
    if (chance(r, 95)) puts_(b, "\r\n");
    else puts_(b, "xy");
  }
}

static size_t gen_fuzz(bld_t *b, rng_t *r, int http)
{
  size_t start = b->len;
  fz_dirty = chance(r, 40);
  uint32_t shape = rndu(r, 100);

  /* tiny pathological buffers around the one-past-end hazard */
  if (shape < 6) {
    static const char *T[] = {"", "G", "GET", "GET ", "GET  ", " ", "  ", "GET /", "GET / ", "GET /  ",
                              "\r", "\n", "\r\n", "\r\nGET ", " / ", "GET / H", "GET / HTTP/1.1",
                              "GET / HTTP/1.1\r", "GET / HTTP/1.1\r\n", "GET / HTTP/1.1\r\n\r",
                              "GET / XTTP", "GET / XTTP/1.1", "GET\x01", "GET / HTTP/1.1\n\n"};
    puts_(b, T[rndu(r, sizeof T / sizeof *T)]);
    return b->len - start;
  }
  if (shape < 9) {
    /* leading spaces feed the previous request's past-end SP skip */
    size_t n = 1 + rndu(r, 3);
    for (size_t i = 0; i < n; i++) putc_(b, ' ');
  }

  if (chance(r, 6)) puts_(b, chance(r, 70) ? "\r\n" : "\n");
  int post = 0;
  uint32_t mp = rndu(r, 100);
  if (mp < 45) puts_(b, "GET");
  else if (mp < (http ? 85u : 65u)) { puts_(b, chance(r, 80) ? "POST" : "PUT"); post = 1; }
  else if (mp < 88) puts_(b, "get");
  else if (mp < 92 && fz_dirty) fuzz_token(b, r, 0);
  else fuzz_token(b, r, 10);
  fuzz_sps(b, r);
  if (chance(r, 90)) putc_(b, '/');
  fuzz_token(b, r, 40);
  fuzz_sps(b, r);
  fuzz_version(b, r);
  fuzz_eol(b, r);

  uint32_t nh = chance(r, 10) ? 10 + rndu(r, 25) : rndu(r, 8);
  size_t body_len = rndu(r, 60);
  int te = 0;
  for (uint32_t i = 0; i < nh; i++) {
    if (i > 0 && chance(r, 3)) {
      /* obs-fold continuation line */
      puts_(b, chance(r, 50) ? " " : "\t");
      fuzz_value(b, r, 20);
      fuzz_eol(b, r);
      continue;
    }
    int special = post && chance(r, http ? 45 : 15);
    if (special) {
      if (chance(r, 55)) {
        puts_(b, chance(r, 80) ? "Content-Length" : "content-length");
        puts_(b, ":");
        fuzz_sps(b, r);
        fuzz_cl_value(b, r, body_len);
      } else {
        puts_(b, chance(r, 80) ? "Transfer-Encoding" : "TRANSFER-encoding");
        puts_(b, ":");
        fuzz_sps(b, r);
        static const char *E[] = {"chunked", "Chunked", "CHUNKED", "chunked ", "gzip", "", "chunke",
                                  "chunked, gzip"};
        const char *e = E[rndu(r, sizeof E / sizeof *E)];
        puts_(b, e);
        te = 1;
      }
      if (chance(r, 10)) puts_(b, " \t");
    } else {
      fuzz_name(b, r);
      if (fz_dirty && chance(r, 6)) putc_(b, ' ');
      if (!fz_dirty || chance(r, 94)) putc_(b, ':');
      uint32_t ows = rndu(r, 100);
      if (ows < 75) putc_(b, ' ');
      else if (ows < 82) puts_(b, " \t ");
      fuzz_value(b, r, 30);
    }
    fuzz_eol(b, r);
  }
  uint32_t endp = rndu(r, 100);
  if (endp < 85) puts_(b, "\r\n");
  else if (endp < 95) puts_(b, "\n");
  if (post) {
    if (te && chance(r, 70)) fuzz_chunked_body(b, r);
    else
      for (size_t i = 0; i < body_len; i++) putc_(b, (uint8_t) VAL_CHARS[rndu(r, sizeof VAL_CHARS - 1)]);
  }
  if (chance(r, 8)) fuzz_value(b, r, 20); /* trailing pipelined garbage */
  return b->len - start;
}

/* ---------------- dispatch ---------------- */

static size_t gen_one(int config, uint64_t seed, uint64_t idx, bld_t *b, size_t *hdr_bytes)
{
  rng_t r = rng_for(seed, idx, config);
  size_t n, h = 0;
  switch (config) {
  case RHP_GEN_TFB128: n = gen_tfb(b, &r, 10); break;
  case RHP_GEN_GET256: n = gen_tfb(b, &r, 138); break;
  case RHP_GEN_ZIPF: n = gen_zipf(b, &r); break;
  case RHP_GEN_POST1K: n = gen_post(b, &r, &h); break;
  case RHP_GEN_CHUNKED: n = gen_chunked(b, &r); break;
  case RHP_GEN_FUZZ: n = gen_fuzz(b, &r, 0); break;
  case RHP_GEN_FUZZ_HTTP: n = gen_fuzz(b, &r, 1); break;
  default: return (size_t) -1;
  }
  if (hdr_bytes) *hdr_bytes = config == RHP_GEN_POST1K ? h : n;
  return n;
}

uint64_t rhp_gen_size(int config, uint64_t lo, uint64_t hi, uint64_t seed)
{
  if (config == RHP_GEN_TFB128) return (hi - lo) * 128;
  if (config == RHP_GEN_GET256) return (hi - lo) * 256;
  if (config == RHP_GEN_POST1K) return (hi - lo) * 1024;
  uint64_t total = 0;
  for (uint64_t i = lo; i < hi; i++) {
    bld_t b = {0};
    size_t n = gen_one(config, seed, i, &b, NULL);
    if (n == (size_t) -1) return 0;
    total += n;
  }
  return total;
}

uint64_t rhp_gen_header_bytes(int config, uint64_t lo, uint64_t hi, uint64_t seed)
{
  if (config == RHP_GEN_TFB128) return (hi - lo) * 128;
  if (config == RHP_GEN_GET256) return (hi - lo) * 256;
  uint64_t total = 0;
  for (uint64_t i = lo; i < hi; i++) {
    bld_t b = {0};
    size_t h = 0;
    gen_one(config, seed, i, &b, &h);
    total += h;
  }
  return total;
}

int rhp_gen_fill(int config, uint64_t lo, uint64_t hi, uint64_t seed, uint8_t *bytes, uint64_t *offsets)
{
  uint64_t pos = 0;
  for (uint64_t i = lo; i < hi; i++) {
    offsets[i - lo] = pos;
    bld_t b = {bytes + pos, 0, (size_t) -1};
    size_t n = gen_one(config, seed, i, &b, NULL);
    if (n == (size_t) -1) return -1;
    pos += n;
  }
  offsets[hi - lo] = pos;
  memset(bytes + pos, 0, RHP_GEN_PAD);
  return 0;
}
