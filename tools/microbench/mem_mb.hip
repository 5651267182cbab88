// Memory-system microbenchmarks that decide the pane-store design on gfx950:
//  - streaming copy bandwidth (HBM roof as this code reaches it)
//  - random 64-bit / 32-bit atomic add throughput vs table footprint
//  - random 8-byte gather throughput vs table footprint (hash probe cost)
//  - LDS 64-bit atomic add throughput
// Build: hipcc --offload-arch=gfx950 -O3 mem_mb.hip -o mem_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void k_copy(const int4* __restrict__ a, int4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}
__global__ void k_read(const int4* __restrict__ a, size_t n, int* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  int acc = 0;
  for (; i < n; i += s) { int4 v = a[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x7fffffff) out[0] = acc;
}

template <typename T>
__global__ void k_atomic_rand(T* tab, uint64_t mask, size_t n, uint64_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    uint64_t h = mix64(seed ^ i);
    atomicAdd(&tab[h & mask], (T)1);
  }
}
// 64-bit atomic where each record also reads 24B of streamed input (models fused ingest)
__global__ void k_ingest_atomic(const long long* __restrict__ key, const long long* __restrict__ val,
                                const long long* __restrict__ ts,
                                unsigned long long* tab, uint64_t mask, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    uint64_t h = mix64((uint64_t)key[i] ^ (uint64_t)(ts[i] / 1000));
    atomicAdd(&tab[h & mask], (unsigned long long)val[i]);
  }
}
__global__ void k_gather_rand(const unsigned long long* __restrict__ tab, uint64_t mask, size_t n,
                              uint64_t seed, unsigned long long* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (; i < n; i += s) acc += tab[mix64(seed ^ i) & mask];
  if (acc == 0x123456789ull) out[0] = acc;
}
// LDS: each block hammers a 16K-entry (128 KiB) u64 table with random atomic adds
__global__ void k_lds_atomic(size_t iters, uint64_t seed, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lt[];
  const int E = 16384;
  for (int j = threadIdx.x; j < E; j += blockDim.x) lt[j] = 0;
  __syncthreads();
  uint64_t base = seed ^ ((uint64_t)blockIdx.x << 40) ^ ((uint64_t)threadIdx.x << 20);
  for (size_t k = 0; k < iters; ++k) {
    uint64_t h = mix64(base + k);
    atomicAdd(&lt[h & (E - 1)], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, lt[blockIdx.x & (E - 1)]);
}
__global__ void k_lds_atomic32(size_t iters, uint64_t seed, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned lt32[];
  const int E = 32768;
  for (int j = threadIdx.x; j < E; j += blockDim.x) lt32[j] = 0;
  __syncthreads();
  uint64_t base = seed ^ ((uint64_t)blockIdx.x << 40) ^ ((uint64_t)threadIdx.x << 20);
  for (size_t k = 0; k < iters; ++k) {
    uint64_t h = mix64(base + k);
    atomicAdd(&lt32[h & (E - 1)], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, lt32[blockIdx.x & (E - 1)]);
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main() {
  const int G = 256 * 8, B = 256;
  Timer t;
  size_t nbytes = 2ull << 30;  // 2 GiB
  int4 *a, *b; CK(hipMalloc(&a, nbytes)); CK(hipMalloc(&b, nbytes));
  CK(hipMemset(a, 1, nbytes)); CK(hipMemset(b, 0, nbytes));
  int* dummy; CK(hipMalloc(&dummy, 64));
  size_t n16 = nbytes / 16;
  for (int w = 0; w < 2; ++w) k_copy<<<G, B>>>(a, b, n16);
  t.start(); for (int r = 0; r < 5; ++r) k_copy<<<G, B>>>(a, b, n16);
  float ms = t.stop() / 5;
  printf("copy   2GiB: %.3f ms  %.1f GB/s (r+w)\n", ms, 2.0 * nbytes / ms / 1e6);
  t.start(); for (int r = 0; r < 5; ++r) k_read<<<G, B>>>(a, n16, dummy);
  ms = t.stop() / 5;
  printf("read   2GiB: %.3f ms  %.1f GB/s\n", ms, 1.0 * nbytes / ms / 1e6);

  size_t nat = 1ull << 26;
  unsigned long long* tab; CK(hipMalloc(&tab, 1ull << 30)); CK(hipMemset(tab, 0, 1ull << 30));
  for (int lg : {10, 13, 16, 17, 20, 23, 27}) {  // entries (u64) 2^lg
    uint64_t mask = (1ull << lg) - 1;
    k_atomic_rand<unsigned long long><<<G, B>>>(tab, mask, nat, 7);
    t.start(); k_atomic_rand<unsigned long long><<<G, B>>>(tab, mask, nat, 9);
    ms = t.stop();
    printf("atomic u64 rand  tab=%8.2f MiB: %.3f ms  %.2f Gatom/s\n", (8.0 * (mask + 1)) / 1048576, ms, nat / ms / 1e6);
    k_atomic_rand<unsigned><<<G, B>>>((unsigned*)tab, (mask << 1) | 1, nat, 7);
    t.start(); k_atomic_rand<unsigned><<<G, B>>>((unsigned*)tab, (mask << 1) | 1, nat, 9);
    ms = t.stop();
    printf("atomic u32 rand  tab=%8.2f MiB: %.3f ms  %.2f Gatom/s\n", (8.0 * (mask + 1)) / 1048576, ms, nat / ms / 1e6);
    k_gather_rand<<<G, B>>>(tab, mask, nat, 3, tab + (1ull << 26));
    t.start(); k_gather_rand<<<G, B>>>(tab, mask, nat, 5, tab + (1ull << 26));
    ms = t.stop();
    printf("gather u64 rand  tab=%8.2f MiB: %.3f ms  %.2f Gload/s\n", (8.0 * (mask + 1)) / 1048576, ms, nat / ms / 1e6);
  }
  // fused ingest model: 2^27 records, 24 B each, keys 64K, 1 window
  size_t nr = 1ull << 26;
  long long *key = (long long*)a, *val = key + nr, *ts = val + nr;
  {
    std::vector<long long> hk(nr);
    uint64_t x = 1;
    for (size_t i = 0; i < nr; ++i) { x = x * 6364136223846793005ull + 1442695040888963407ull; hk[i] = (x >> 33) & 0xFFFF; }
    CK(hipMemcpy(key, hk.data(), nr * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(val, hk.data(), nr * 8, hipMemcpyHostToDevice));
    for (size_t i = 0; i < nr; ++i) hk[i] = (long long)(i * 1000 / (1ull << 24));
    CK(hipMemcpy(ts, hk.data(), nr * 8, hipMemcpyHostToDevice));
  }
  for (int lg : {17, 20}) {
    uint64_t mask = (1ull << lg) - 1;
    k_ingest_atomic<<<G, B>>>(key, val, ts, tab, mask, nr);
    t.start(); k_ingest_atomic<<<G, B>>>(key, val, ts, tab, mask, nr);
    ms = t.stop();
    printf("ingest+atomic tab 2^%d: %.3f ms  %.2f Gev/s  %.1f GB/s input\n", lg, ms, nr / ms / 1e6, 24.0 * nr / ms / 1e6);
  }
  // MALL absorption: stream-read 96 MiB "input", write 80 MiB "partition", read it back; repeat
  {
    size_t in_b = 96ull << 20, part_b = 80ull << 20;
    int4* inp = b; int4* part = b + (512ull << 20) / 16;
    for (int w = 0; w < 3; ++w) { k_copy<<<G, B>>>(inp, part, part_b / 16); k_read<<<G, B>>>(part, part_b / 16, dummy); }
    t.start();
    for (int r = 0; r < 20; ++r) {
      int4* inr = inp + (r % 4) * (in_b / 16);   // rotate input so it is not cache resident
      k_copy<<<G, B>>>(inr, part, part_b / 16);
      k_read<<<G, B>>>(part, part_b / 16, dummy);
    }
    ms = t.stop() / 20;
    printf("stage: read in(80MiB)+write part(80MiB)+read part: %.3f ms/iter  eff %.1f GB/s of input\n", ms, part_b / ms / 1e6);
    t.start();
    for (int r = 0; r < 20; ++r) { int4* inr = inp + (r % 4) * (in_b / 16); k_read<<<G, B>>>(inr, part_b / 16, dummy); }
    ms = t.stop() / 20;
    printf("stage: read in(80MiB) only: %.3f ms/iter  %.1f GB/s\n", ms, part_b / ms / 1e6);
  }
  // LDS atomics
  size_t iters = 4096;
  k_lds_atomic<<<G / 2, B, 131072>>>(iters, 1, tab);
  t.start(); k_lds_atomic<<<1024, B, 131072>>>(iters, 2, tab);
  ms = t.stop();
  printf("lds atomic u64: %.3f ms  %.2f Gatom/s\n", ms, 1024.0 * B * iters / ms / 1e6);
  t.start(); k_lds_atomic32<<<1024, B, 131072>>>(iters, 2, (unsigned*)tab);
  ms = t.stop();
  printf("lds atomic u32: %.3f ms  %.2f Gatom/s\n", ms, 1024.0 * B * iters / ms / 1e6);
  return 0;
}
