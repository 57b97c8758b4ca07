/*
 * diff_fuzz.c -- TEST INFRASTRUCTURE ONLY: pins the restatement (rhp_oracle.c)
 * against the reference compiled from /root/reference (ref_harness.c).
 *
 * usage: diff_fuzz <batches> <requests-per-batch> [seed]
 * Every batch: generator configs 100/101 (edge cases) and 2/3/5, every
 * max_headers in {0,1,2,4,16,32} rotating, phr mode and http mode (bytes
 * compared too, since chunked bodies are rewritten in place).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "rhp_gen.h"
#include "rhp_oracle.h"

void ref_phr_batch(const uint8_t *, const uint64_t *, uint32_t, uint32_t, orc_req_t *, orc_hdr_t *);
void ref_http_batch(uint8_t *, const uint64_t *, uint32_t, uint32_t, orc_req_t *, orc_hdr_t *, orc_http_t *);

static void dump(const uint8_t *p, size_t n)
{
  fputc('"', stderr);
  for (size_t i = 0; i < n && i < 400; i++) {
    if (p[i] >= 0x20 && p[i] < 0x7f && p[i] != '"' && p[i] != '\\') fputc(p[i], stderr);
    else fprintf(stderr, "\\x%02x", p[i]);
  }
  fputs("\"\n", stderr);
}

int main(int argc, char **argv)
{
  int batches = argc > 1 ? atoi(argv[1]) : 100;
  uint32_t n = argc > 2 ? (uint32_t) atoi(argv[2]) : 1000;
  uint64_t seed0 = argc > 3 ? strtoull(argv[3], NULL, 0) : 1;
  static const uint32_t MAXH[] = {0, 1, 2, 4, 16, 32};
  static const int CONFIGS[] = {100, 101, 100, 101, 3, 5, 2};
  uint64_t stat_ok = 0, stat_m1 = 0, stat_m2 = 0, http1 = 0, http0 = 0, httpm1 = 0, total = 0;

  for (int bi = 0; bi < batches; bi++) {
    int config = CONFIGS[bi % 7];
    uint32_t maxh = MAXH[(bi / 7) % 6];
    uint64_t seed = seed0 * 1000003ull + (uint64_t) bi;
    uint64_t size = rhp_gen_size(config, 0, n, seed);
    uint8_t *bytes = malloc(size + RHP_GEN_PAD);
    uint8_t *b1 = malloc(size + RHP_GEN_PAD), *b2 = malloc(size + RHP_GEN_PAD);
    uint64_t *off = malloc(sizeof *off * (n + 1));
    rhp_gen_fill(config, 0, n, seed, bytes, off);
    size_t hcap = (size_t) n * (maxh ? maxh : 1);
    orc_req_t *ra = calloc(n, sizeof *ra), *rb = calloc(n, sizeof *rb);
    orc_hdr_t *ha = calloc(hcap, sizeof *ha), *hb = calloc(hcap, sizeof *hb);
    orc_http_t *xa = calloc(n, sizeof *xa), *xb = calloc(n, sizeof *xb);

    ref_phr_batch(bytes, off, n, maxh, ra, ha);
    orc_phr_batch(bytes, off, n, maxh, rb, hb);
    for (uint32_t i = 0; i < n; i++) {
      total++;
      if (ra[i].ret > 0) stat_ok++;
      else if (ra[i].ret == -1) stat_m1++;
      else stat_m2++;
      int bad = memcmp(&ra[i], &rb[i], sizeof ra[i]) != 0 ||
                memcmp(ha + (size_t) i * maxh, hb + (size_t) i * maxh, sizeof *ha * maxh) != 0;
      if (bad) {
        fprintf(stderr, "PHR MISMATCH batch %d cfg %d maxh %u req %u: ref ret %d nh %u orc ret %d nh %u\n",
                bi, config, maxh, i, ra[i].ret, ra[i].num_headers, rb[i].ret, rb[i].num_headers);
        dump(bytes + off[i], off[i + 1] - off[i]);
        return 1;
      }
    }

    memcpy(b1, bytes, size + RHP_GEN_PAD);
    memcpy(b2, bytes, size + RHP_GEN_PAD);
    ref_http_batch(b1, off, n, maxh, ra, ha, xa);
    orc_http_batch(b2, off, n, maxh, rb, hb, xb);
    for (uint32_t i = 0; i < n; i++) {
      if (xa[i].result == 1) http1++;
      else if (xa[i].result == 0) http0++;
      else httpm1++;
      int bad = memcmp(&ra[i], &rb[i], sizeof ra[i]) != 0 || memcmp(&xa[i], &xb[i], sizeof xa[i]) != 0 ||
                memcmp(ha + (size_t) i * maxh, hb + (size_t) i * maxh, sizeof *ha * maxh) != 0;
      if (bad) {
        fprintf(stderr,
                "HTTP MISMATCH batch %d cfg %d maxh %u req %u: ref r=%d cons=%llu body=%d(%lld,%llu) ret=%d | "
                "orc r=%d cons=%llu body=%d(%lld,%llu) ret=%d\n",
                bi, config, maxh, i, xa[i].result, (unsigned long long) xa[i].consumed, xa[i].body_kind,
                (long long) xa[i].body_off, (unsigned long long) xa[i].body_len, ra[i].ret, xb[i].result,
                (unsigned long long) xb[i].consumed, xb[i].body_kind, (long long) xb[i].body_off,
                (unsigned long long) xb[i].body_len, rb[i].ret);
        dump(bytes + off[i], off[i + 1] - off[i]);
        return 1;
      }
    }
    if (memcmp(b1, b2, size + RHP_GEN_PAD) != 0) {
      fprintf(stderr, "HTTP BYTES MISMATCH batch %d\n", bi);
      return 1;
    }
    free(bytes); free(b1); free(b2); free(off);
    free(ra); free(rb); free(ha); free(hb); free(xa); free(xb);
  }
  printf("diff_fuzz OK: %llu requests (phr ok %llu, -1 %llu, -2 %llu; http 1:%llu 0:%llu -1:%llu)\n",
         (unsigned long long) total, (unsigned long long) stat_ok, (unsigned long long) stat_m1,
         (unsigned long long) stat_m2, (unsigned long long) http1, (unsigned long long) http0,
         (unsigned long long) httpm1);
  return 0;
}
