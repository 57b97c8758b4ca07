// ubench_ceiling.hip -- what one launch of config 2's size (268 MB of request
// bytes, 48 MB of records written) can reach on gfx950 (MI355X), launched back
// to back over 4 rotated copies (1 GiB, beyond the 256 MiB Infinity Cache) as
// bench.py does.  Every kernel reads every byte once (xor-folded), some also
// write config 2's record bytes (16 B + 4 x 8 B per 256-B request).
//   coal<U,NT,W>   grid-stride, wave reads 1 KiB per global_load_dwordx4, U in flight
//   chunk<U,NT,W>  persistent: a workgroup pulls 64 KiB chunks from a global counter
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_ceiling.hip -o tools/ubench_ceiling
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x4 gq;

constexpr uint64_t kBytes = 268435456ull;   /* 1M x 256 B */
constexpr uint64_t kReqs = kBytes / 256;

/* the records of request i: 16 B at reqs[i], 4 x 8 B header-major at hdrs[k * n + i] */
__device__ __forceinline__ void write_records(uint8_t *reqs, uint8_t *hdrs, uint64_t i, uint32_t v)
{
  *reinterpret_cast<__attribute__((address_space(1))) u32x4 *>((uintptr_t) (reqs + 16 * i)) = u32x4{v, 1, 2, 3};
#pragma unroll
  for (int k = 0; k < 4; k++)
    *reinterpret_cast<__attribute__((address_space(1))) u32x2 *>((uintptr_t) (hdrs + 8 * ((uint64_t) k * kReqs + i))) =
        u32x2{v, (uint32_t) k};
}

template <int U, int NT, int W>
__global__ void coal(const uint8_t *buf, uint8_t *reqs, uint8_t *hdrs, uint32_t *out)
{
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x * 16 * U;
  uint32_t acc = 0;
  for (uint64_t at = ((uint64_t) blockIdx.x * blockDim.x * U + threadIdx.x) * 16; at < kBytes; at += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      gq *p = (gq *) (uintptr_t) (buf + at + (uint64_t) u * blockDim.x * 16);
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    if (W) {
      /* one request's records per 16 lanes' worth of bytes: lanes with
       * (threadIdx & 15) == 0 of the first load write them */
      const uint64_t b0 = at;   /* this lane's first byte */
      if ((b0 & 255) == 0) write_records(reqs, hdrs, b0 >> 8, acc);
#pragma unroll
      for (int u = 1; u < U; u++) {
        const uint64_t b = at + (uint64_t) u * blockDim.x * 16;
        if ((b & 255) == 0) write_records(reqs, hdrs, b >> 8, acc);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

/* persistent: workgroup pulls CHUNK-byte chunks from a global counter (one
 * lane, the next chunk prefetched one chunk ahead) */
template <int U, int NT, int W, uint32_t CHUNK>
__global__ void chunk(const uint8_t *buf, uint8_t *reqs, uint8_t *hdrs, uint32_t *out, uint32_t *ctr)
{
  __shared__ uint32_t next;
  const uint32_t nchunks = (uint32_t) (kBytes / CHUNK);
  uint32_t acc = 0;
  if (threadIdx.x == 0) next = atomicAdd(ctr, 1u);
  __syncthreads();
  uint32_t c = next;
  while (c < nchunks) {
    __syncthreads();
    if (threadIdx.x == 0) next = atomicAdd(ctr, 1u);   /* lands while this chunk streams */
    const uint64_t base = (uint64_t) c * CHUNK;
    for (uint32_t at = threadIdx.x * 16; at < CHUNK; at += blockDim.x * 16 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        gq *p = (gq *) (uintptr_t) (buf + base + at + (uint64_t) u * blockDim.x * 16);
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
      if (W) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t b = base + at + (uint64_t) u * blockDim.x * 16;
          if ((b & 255) == 0) write_records(reqs, hdrs, b >> 8, acc);
        }
      }
    }
    __syncthreads();
    c = next;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}


/* wave per 64 requests: 16 loads of 1 KiB (U in flight), then the 64 records
 * written coalesced: reqs 1 KiB (16 B per lane), each header k one 512-B run */
template <int U, int NT, int W>
__global__ void group(const uint8_t *buf, uint8_t *reqs, uint8_t *hdrs, uint32_t *out)
{
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t) gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t) blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < kReqs / 64; g += waves) {
    const uint8_t *b = buf + g * 16384 + 16 * lane;
    for (int j = 0; j < 16; j += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        gq *p = (gq *) (uintptr_t) (b + 1024 * (j + u));
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    if (W) write_records(reqs, hdrs, g * 64 + lane, acc);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

/* a 16- / 4-byte global store with the sc1 bit: written through to memory,
 * the line dropped from L2, so the launch leaves no dirty record lines for
 * the kernel boundary's write-back (MI355X_MICROARCH.md, store flavours) */
__device__ __forceinline__ void st16_wt(void *p, u32x4 v)
{
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st8_wt(void *p, u32x2 v)
{
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st4_wt(void *p, uint32_t v)
{
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

/* group with the records written in other forms: WM 1 = nt stores (ABI layout),
 * 2 = the wave's 3 KiB of records contiguous (tiled: reqs then the 4 header
 * runs of its 64 requests), 3 = reqs only (16 MB), 4 = headers only (32 MB),
 * 5 = the ABI layout (48 B) with write-through (sc1) stores, 6 = compact
 * records: 16-B request record + 4 x 4-B header records (u16 name_len, u16
 * value_len) header-major, 32 B, 7 = 8-B request record + 4 x 4 B, 24 B,
 * 8 / 9 = 6 / 7 with write-through stores */
template <int U, int WM>
__global__ void groupw(const uint8_t *buf, uint8_t *reqs, uint8_t *hdrs, uint32_t *out)
{
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t) gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  typedef __attribute__((address_space(1))) u32x4 gw4;
  typedef __attribute__((address_space(1))) u32x2 gw2;
  for (uint64_t g = (uint64_t) blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < kReqs / 64; g += waves) {
    const uint8_t *b = buf + g * 16384 + 16 * lane;
    for (int j = 0; j < 16; j += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load((gq *) (uintptr_t) (b + 1024 * (j + u)));
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    const uint64_t i = g * 64 + lane;
    if (WM == 1) {
      __builtin_nontemporal_store(u32x4{acc, 1, 2, 3}, (gw4 *) (uintptr_t) (reqs + 16 * i));
#pragma unroll
      for (int k = 0; k < 4; k++)
        __builtin_nontemporal_store(u32x2{acc, (uint32_t) k}, (gw2 *) (uintptr_t) (hdrs + 8 * ((uint64_t) k * kReqs + i)));
    } else if (WM == 2) {
      uint8_t *t = reqs + g * 3072;   /* reqs (16 MB) + hdrs (32 MB): one 48 MB area */
      *(gw4 *) (uintptr_t) (t + 16 * lane) = u32x4{acc, 1, 2, 3};
#pragma unroll
      for (int k = 0; k < 4; k++) *(gw2 *) (uintptr_t) (t + 1024 + 512 * k + 8 * lane) = u32x2{acc, (uint32_t) k};
    } else if (WM == 3) {
      *(gw4 *) (uintptr_t) (reqs + 16 * i) = u32x4{acc, 1, 2, 3};
    } else if (WM == 4) {
#pragma unroll
      for (int k = 0; k < 4; k++) *(gw2 *) (uintptr_t) (hdrs + 8 * ((uint64_t) k * kReqs + i)) = u32x2{acc, (uint32_t) k};
    } else if (WM == 5) {
      st16_wt(reqs + 16 * i, u32x4{acc, 1, 2, 3});
#pragma unroll
      for (int k = 0; k < 4; k++) st8_wt(hdrs + 8 * ((uint64_t) k * kReqs + i), u32x2{acc, (uint32_t) k});
    } else if (WM == 6 || WM == 8) {
      typedef __attribute__((address_space(1))) uint32_t gw1;
      if (WM == 6) *(gw4 *) (uintptr_t) (reqs + 16 * i) = u32x4{acc, 1, 2, 3};
      else st16_wt(reqs + 16 * i, u32x4{acc, 1, 2, 3});
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint8_t *q = hdrs + 4 * ((uint64_t) k * kReqs + i);
        if (WM == 6) *(gw1 *) (uintptr_t) q = acc + k;
        else st4_wt(q, acc + k);
      }
    } else if (WM == 7 || WM == 9) {
      typedef __attribute__((address_space(1))) uint32_t gw1;
      if (WM == 7) *(gw2 *) (uintptr_t) (reqs + 8 * i) = u32x2{acc, 1};
      else st8_wt(reqs + 8 * i, u32x2{acc, 1});
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint8_t *q = hdrs + 4 * ((uint64_t) k * kReqs + i);
        if (WM == 7) *(gw1 *) (uintptr_t) q = acc + k;
        else st4_wt(q, acc + k);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

/* group, with the records of group g stored after the loads of group g + 1
 * are issued: vmcnt counts loads and stores together in issue order, so in
 * `group` each group's first load wait also waits for the previous group's
 * stores; here the stores are younger than the loads waited for */
template <int U>
__global__ void groupp(const uint8_t *buf, uint8_t *reqs, uint8_t *hdrs, uint32_t *out)
{
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t) gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0, prev_acc = 0;
  uint64_t prev_i = ~0ull;
  for (uint64_t g = (uint64_t) blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < kReqs / 64; g += waves) {
    const uint8_t *b = buf + g * 16384 + 16 * lane;
    acc = 0;
    for (int j = 0; j < 16; j += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load((gq *) (uintptr_t) (b + 1024 * (j + u)));
      if (j == 0 && prev_i != ~0ull) write_records(reqs, hdrs, prev_i, prev_acc);
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    prev_i = g * 64 + lane;
    prev_acc = acc;
  }
  if (prev_i != ~0ull) write_records(reqs, hdrs, prev_i, prev_acc);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

/* writes only: 48 MB with 16 B per lane, contiguous */
__global__ void wonly(const uint8_t *, uint8_t *reqs, uint8_t *hdrs, uint32_t *out)
{
  typedef __attribute__((address_space(1))) u32x4 gw4;
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x * 16;
  for (uint64_t at = ((uint64_t) blockIdx.x * blockDim.x + threadIdx.x) * 16; at < 48 * kReqs; at += stride) {
    uint8_t *t = reqs + at;
    *(gw4 *) (uintptr_t) t = u32x4{(uint32_t) at, 1, 2, 3};
  }
}

struct Bufs {
  uint8_t *in[4];
  uint8_t *reqs, *hdrs;
  uint32_t *out, *ctr;
};

template <class L>
void run(const char *name, L launch, Bufs &b, bool counter)
{
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int steps = 50;
  for (int k = 0; k < 8; k++) {
    if (counter) CHECK(hipMemsetAsync(b.ctr + 64 * (k % 4), 0, 4));
    launch(b.in[k % 4], b.ctr + 64 * (k % 4));
  }
  CHECK(hipDeviceSynchronize());
  /* counters for the timed launches are zeroed beforehand (a memset between
   * launches would be timed too): one counter per launch */
  if (counter) CHECK(hipMemset(b.ctr, 0, 4 * 64 * steps));
  CHECK(hipEventRecord(e0));
  for (int k = 0; k < steps; k++) launch(b.in[k % 4], b.ctr + 64 * k);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / steps;
  printf("%-34s %7.1f us  %6.0f GB/s read  frac %.3f\n", name, us, kBytes / us / 1e3, kBytes / us / 1e3 / 8000.0);
  fflush(stdout);
}

int main()
{
  Bufs b;
  for (int k = 0; k < 4; k++) {
    CHECK(hipMalloc(&b.in[k], kBytes + 4096));
    CHECK(hipMemset(b.in[k], k + 1, kBytes + 4096));
  }
  /* one area: reqs (16 MB) then hdrs (32 MB), plus slack */
  CHECK(hipMalloc(&b.reqs, 48 * kReqs + 65536));
  b.hdrs = b.reqs + 16 * kReqs;
  CHECK(hipMalloc(&b.out, 4 << 20));
  CHECK(hipMalloc(&b.ctr, 4 * 64 * 64));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs %d, %llu B per launch, 4 rotated copies\n", cus, (unsigned long long) kBytes);
#define COAL(U, NT, W, GRID, BLOCK)                                                                               \
  run("coal U" #U " nt" #NT " w" #W " grid " #GRID "x" #BLOCK,                                                  \
      [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL((coal<U, NT, W>), dim3(GRID), dim3(BLOCK), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false)
#define CHUNK(U, NT, W, C, GRID, BLOCK)                                                                            \
  run("chunk" #C " U" #U " nt" #NT " w" #W " grid " #GRID "x" #BLOCK,                                            \
      [&](uint8_t *in, uint32_t *ctr) { hipLaunchKernelGGL((chunk<U, NT, W, C>), dim3(GRID), dim3(BLOCK), 0, 0, in, b.reqs, b.hdrs, b.out, ctr); }, b, true)
#define GROUP(U, NT, W, GRID, BLOCK)                                                                              \
  run("group U" #U " nt" #NT " w" #W " grid " #GRID "x" #BLOCK,                                                 \
      [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL((group<U, NT, W>), dim3(GRID), dim3(BLOCK), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false)
#define GROUPW(U, WM, GRID, BLOCK)                                                                              \
  run("groupw U" #U " wm" #WM " grid " #GRID "x" #BLOCK,                                                        \
      [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL((groupw<U, WM>), dim3(GRID), dim3(BLOCK), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false)
  if (getenv("ONLY_C")) {   /* compact and write-through record forms (round 4) */
    for (int rep = 0; rep < 2; rep++) {
      GROUP(8, 1, 0, 256, 1024);
      GROUP(8, 1, 1, 256, 1024);
      GROUPW(8, 3, 256, 1024);
      GROUPW(8, 5, 256, 1024);
      GROUPW(8, 6, 256, 1024);
      GROUPW(8, 7, 256, 1024);
      GROUPW(8, 8, 256, 1024);
      GROUPW(8, 9, 256, 1024);
    }
    return 0;
  }
  if (getenv("ONLY_W")) {
    for (int rep = 0; rep < 2; rep++) {
      GROUP(8, 1, 0, 256, 1024);
      GROUP(8, 1, 1, 256, 1024);
      GROUPW(8, 1, 256, 1024);
      GROUPW(8, 2, 256, 1024);
      GROUPW(8, 3, 256, 1024);
      GROUPW(8, 4, 256, 1024);
      run("groupp U8 (stores after the next loads)", [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL((groupp<8>), dim3(256), dim3(1024), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false);
      run("groupp U4 (stores after the next loads)", [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL((groupp<4>), dim3(256), dim3(1024), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false);
      run("wonly 48 MB", [&](uint8_t *in, uint32_t *) { hipLaunchKernelGGL(wonly, dim3(256 * 4), dim3(256), 0, 0, in, b.reqs, b.hdrs, b.out); }, b, false);
    }
    return 0;
  }
  for (int rep = 0; rep < 2; rep++) {
    COAL(4, 1, 0, 256 * 4, 256);
    COAL(4, 1, 0, 256, 1024);
    COAL(8, 1, 0, 256, 1024);
    COAL(4, 0, 0, 256, 1024);
    COAL(4, 1, 0, 256 * 16, 256);
    COAL(4, 1, 1, 256, 1024);
    COAL(4, 1, 1, 256 * 4, 256);
    CHUNK(4, 1, 0, 65536, 256, 1024);
    CHUNK(4, 1, 1, 65536, 256, 1024);
    GROUP(4, 1, 0, 256, 1024);
    GROUP(8, 1, 0, 256, 1024);
    GROUP(4, 1, 1, 256, 1024);
    GROUP(8, 1, 1, 256, 1024);
    GROUP(16, 1, 1, 256, 1024);
    GROUP(8, 1, 1, 512, 512);
  }
  return 0;
}
