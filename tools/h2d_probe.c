/* h2d_probe.c -- what one reactor round's H2D copy costs (VERDICT r4 item 5:
 * the round timeline shows ~1.2 ms per copy at any size).  Copies of 64 KiB
 * .. 8 MiB from hipHostMalloc'd (default and mapped/non-coherent flags) and
 * hipHostRegister'ed memory to the device with hipMemcpyAsync on a
 * non-blocking stream; per copy: the host time of the call, the event time of
 * the copy, the host time until the stream is done.
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/h2d_probe.c -o tools/h2d_probe -L/opt/rocm/lib -lamdhip64 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <stdint.h>

#define HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %d at %d\n", (int) e_, __LINE__); exit(1); } } while (0)

static double now_us(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static void run(const char *name, void *h, void *d, size_t n, hipStream_t s)
{
  hipEvent_t a, b;
  HIP(hipEventCreate(&a));
  HIP(hipEventCreate(&b));
  double call = 0, done = 0;
  float dev = 0;
  const int reps = 20;
  for (int r = -2; r < reps; r++) {
    memset(h, r & 0xff, 4096);
    const double t0 = now_us();
    HIP(hipEventRecord(a, s));
    HIP(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
    HIP(hipEventRecord(b, s));
    const double t1 = now_us();
    HIP(hipStreamSynchronize(s));
    const double t2 = now_us();
    float ms = 0;
    HIP(hipEventElapsedTime(&ms, a, b));
    if (r >= 0) {
      call += t1 - t0;
      done += t2 - t0;
      dev += ms * 1e3f;
    }
  }
  printf("%-28s %8zu KiB: call %8.1f us, copy (events) %8.1f us, call -> done %8.1f us\n", name, n >> 10, call / reps,
         dev / reps, done / reps);
  HIP(hipEventDestroy(a));
  HIP(hipEventDestroy(b));
}

/* the reactor's sequence: fresh pinned + device buffers, a tiny warm-up copy,
 * then the host fills the input and copies it (first real copy of the buffer) */
static void fresh(size_t n, hipStream_t s, int reuse)
{
  static void *h, *d;
  double call = 0, dev = 0;
  const int reps = 8;
  char *src = malloc(n);
  memset(src, 'x', n);
  for (int r = 0; r < reps; r++) {
    if (!reuse || !h) {
      if (h) { HIP(hipHostFree(h)); HIP(hipFree(d)); }
      HIP(hipHostMalloc(&h, 4u << 20, hipHostMallocDefault));
      HIP(hipMalloc(&d, 4u << 20));
      HIP(hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s));
      HIP(hipStreamSynchronize(s));
    }
    memcpy(h, src, n);
    hipEvent_t a, b;
    HIP(hipEventCreate(&a));
    HIP(hipEventCreate(&b));
    const double t0 = now_us();
    HIP(hipEventRecord(a, s));
    HIP(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
    const double t1 = now_us();
    HIP(hipEventRecord(b, s));
    HIP(hipStreamSynchronize(s));
    float ms = 0;
    HIP(hipEventElapsedTime(&ms, a, b));
    call += t1 - t0;
    dev += ms * 1e3;
    HIP(hipEventDestroy(a));
    HIP(hipEventDestroy(b));
  }
  printf("%-28s %8zu KiB: call %8.1f us, copy (events) %8.1f us\n", reuse ? "reactor sequence, reused" : "reactor sequence, fresh",
         n >> 10, call / reps, dev / reps);
  free(src);
}

/* the CPU's own reads and writes of each kind of host memory (the reactor
 * packs rounds into its slots and dispatches from them) */
static void cpu_rw(const char *name, void *h, size_t n)
{
  char *src = malloc(n);
  memset(src, 'y', n);
  double tw = 0, tr = 0;
  volatile uint64_t sink = 0;
  for (int r = 0; r < 5; r++) {
    const double t0 = now_us();
    memcpy(h, src, n);
    const double t1 = now_us();
    uint64_t acc = 0;
    for (size_t i = 0; i < n / 8; i++) acc += ((const uint64_t *) h)[i];
    const double t2 = now_us();
    sink += acc;
    if (r) { tw += t1 - t0; tr += t2 - t1; }
  }
  printf("cpu %-28s %6zu KiB: write %6.2f GB/s, read %6.2f GB/s\n", name, n >> 10, n / (tw / 4) / 1e3, n / (tr / 4) / 1e3);
  free(src);
}

int main(void)
{
  hipStream_t s;
  HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t cap = 16u << 20;
  void *d, *h0, *h1, *h2;
  HIP(hipMalloc(&d, cap));
  HIP(hipHostMalloc(&h0, cap, hipHostMallocDefault));
  HIP(hipHostMalloc(&h1, cap, hipHostMallocNonCoherent));
  h2 = aligned_alloc(4096, cap);
  memset(h2, 0, cap);
  HIP(hipHostRegister(h2, cap, hipHostRegisterDefault));
  {
    void *m = malloc(8u << 20);
    cpu_rw("malloc", m, 8u << 20);
    free(m);
    cpu_rw("hipHostMalloc default", h0, 8u << 20);
    cpu_rw("hipHostMalloc non-coherent", h1, 8u << 20);
    cpu_rw("malloc + hipHostRegister", h2, 8u << 20);
  }
  for (size_t n = 128u << 10; n <= (2u << 20); n *= 4) {
    fresh(n, s, 0);
    fresh(n, s, 1);
  }
  for (size_t n = 64u << 10; n <= (8u << 20); n *= 2) {
    run("hipHostMalloc default", h0, d, n, s);
    run("hipHostMalloc non-coherent", h1, d, n, s);
    run("malloc + hipHostRegister", h2, d, n, s);
  }
  return 0;
}
