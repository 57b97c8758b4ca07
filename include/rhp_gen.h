/*
 * rhp_gen.h -- deterministic synthetic request batches (splitmix64) for the
 * BASELINE.json configs and for edge-case fuzzing.  Host C, no GPU.
 *
 * Batch format (same as rhp.h): requests packed back to back, offsets[n+1],
 * followed by RHP_GEN_PAD zero bytes (the parity contract pins the bytes after
 * each request).
 *
 * Every request is a pure function of (config, seed, global index), so a shard
 * [lo, hi) of a batch is generated independently (multi-GPU).
 */
#ifndef RHP_GEN_H
#define RHP_GEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RHP_GEN_PAD 256u

enum rhp_gen_config {
  RHP_GEN_TFB128 = 1,     /* config 1: 128 B TechEmpower /plaintext GET (KAT shape)  */
  RHP_GEN_GET256 = 2,     /* config 2/4: 256 B GET, 4 headers, 138 B seeded path    */
  RHP_GEN_ZIPF = 3,       /* config 3: 64 B..4 KiB Zipf(1.2) lengths, 0..32 headers */
  RHP_GEN_POST1K = 5,     /* config 5: 1 KiB POST, Content-Length body, 5% malformed */
  RHP_GEN_CHUNKED = 6,    /* ~1 KiB POST, Transfer-Encoding: chunked body of 1-8 chunks
                             (extensions, OWS, hex case), 5% malformed framing; the
                             chunked path of http_read_request (http.c:73-160, 221-230) */
  RHP_GEN_FUZZ = 100,     /* structured random edge cases (parity only)             */
  RHP_GEN_FUZZ_HTTP = 101 /* edge cases biased to http_read_request framing        */
};

/* Total request bytes of requests [lo, hi) (excluding padding). */
uint64_t rhp_gen_size(int config, uint64_t lo, uint64_t hi, uint64_t seed);

/* Write requests [lo, hi) packed from bytes[0]; offsets[0..hi-lo] are local
 * (offsets[0] == 0).  `bytes` must hold rhp_gen_size(...) + RHP_GEN_PAD bytes;
 * the padding is zero-filled.  Returns 0 on success. */
int rhp_gen_fill(int config, uint64_t lo, uint64_t hi, uint64_t seed, uint8_t *bytes,
                 uint64_t *offsets);

/* Sum over [lo, hi) of the header-section bytes the reference reads (the
 * algorithmic bytes of SURVEY.md §8d): the whole request for GET configs, the
 * bytes before the body for config 5, the whole request for the chunked config
 * (http_dechunk reads every chunk line and moves every data byte). */
uint64_t rhp_gen_header_bytes(int config, uint64_t lo, uint64_t hi, uint64_t seed);

/* splitmix64 step, exposed for tests */
uint64_t rhp_splitmix64(uint64_t *state);

#ifdef __cplusplus
}
#endif
#endif
