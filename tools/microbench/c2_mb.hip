// C2 pane-access microbenchmark (gfx950): 4 Mi records a batch over 10 M uniform keys, directory of 32 M
// slots (C2's geometry).  What bounds the direct form: the atomic rate, or the random lines each record
// touches (directory probe, sum column, first-arrival column)?
//   V0  read24 alone
//   V1  SoA (the engine's layout): dir[slot] load, atomicAdd sum[slot], load first[slot]
//   V2  V1 without the directory load
//   V3  AoS {sum, first} 16 B: dir load, atomicAdd pane.sum, load pane.first (one line for both)
//   V4  V3 with a plain load + store instead of the atomic (racy: throughput only)
//   V5  rows {key, sum, first, f1} 32 B: the directory key and the pane in one line
//   V6  SoA, plain load + store instead of the atomic (racy)
// Build: hipcc --offload-arch=gfx950 -O3 c2_mb.hip -o c2_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef unsigned long long u64;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
}

constexpr int NB = 1 << 22;
constexpr int RING = 16;
constexpr i64 KEYS = 10000000;
constexpr u64 D = 1ull << 25;
struct Cols { const i64* key; const i64* ts; const i64* val; };

__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64(base + i) % (u64)KEYS);
    ts[i] = 1700000000000ll + (i64)(((base + i) * 1000) >> 26);
    val[i] = (i64)(mix64((base + i) ^ 0xabcdef) & 0xffff);
  }
}
__global__ void k_fill(u64* t, size_t n, u64 v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) t[i] = v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_pane(Cols c, int n, i64* dir, u64* sum, i64* first, u64* rows, i64 ord_base,
                                              i64* sink) {
  i64 acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const i64 key = c.key[i], ts = c.ts[i], v = c.val[i];
    acc ^= ts;
    if (MODE == 0) { acc ^= key ^ v; continue; }
    const u64 slot = fmix64((u64)key) & (D - 1);
    const i64 ord = ord_base + i;
    if (MODE == 1 || MODE == 3 || MODE == 4 || MODE == 6) {
      const i64 dk = dir[slot];
      acc ^= dk;
    }
    if (MODE == 1 || MODE == 2) {
      atomicAdd(&sum[slot], (u64)v);
      if (ord < first[slot]) acc ^= 1;
    } else if (MODE == 6) {
      sum[slot] = sum[slot] + (u64)v;
      if (ord < first[slot]) acc ^= 1;
    } else if (MODE == 3) {
      u64* p = rows + 2 * slot;
      atomicAdd(p, (u64)v);
      if (ord < (i64)p[1]) acc ^= 1;
    } else if (MODE == 4) {
      u64* p = rows + 2 * slot;
      p[0] = p[0] + (u64)v;
      if (ord < (i64)p[1]) acc ^= 1;
    } else if (MODE == 5) {
      u64* p = rows + 4 * slot;
      acc ^= (i64)p[0];
      atomicAdd(p + 1, (u64)v);
      if (ord < (i64)p[2]) acc ^= 1;
    }
  }
  if (acc == 0x123456789) sink[0] = acc;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUS = prop.multiProcessorCount;
  printf("device %s, %d CUs; %d records per batch over %lld keys, %llu directory slots\n", prop.name, CUS, NB, KEYS, D);
  const size_t colb = (size_t)NB * 8;
  char* ring; CK(hipMalloc(&ring, (size_t)RING * 3 * colb));
  for (int r = 0; r < RING; ++r) {
    char* b = ring + (size_t)r * 3 * colb;
    k_gen<<<2048, 256>>>((i64*)b, (i64*)(b + colb), (i64*)(b + 2 * colb), NB, (size_t)r * NB);
  }
  auto batch = [&](int r) { char* b = ring + (size_t)(r % RING) * 3 * colb; return Cols{(const i64*)b, (const i64*)(b + colb), (const i64*)(b + 2 * colb)}; };
  i64 *dir, *first, *sink; u64 *sum, *rows;
  CK(hipMalloc(&dir, D * 8)); CK(hipMalloc(&sum, D * 8)); CK(hipMalloc(&first, D * 8));
  CK(hipMalloc(&rows, D * 32)); CK(hipMalloc(&sink, 64));
  k_fill<<<4096, 256>>>((u64*)dir, D, 0); k_fill<<<4096, 256>>>(sum, D, 0);
  k_fill<<<4096, 256>>>((u64*)first, D, 0); k_fill<<<4096, 256>>>(rows, D * 4, 0);
  CK(hipDeviceSynchronize());
  Timer t;
  const int IT = 32;
  const char* names[] = {"V0 read24", "V1 SoA dir + atomic sum + first load", "V2 SoA atomic sum + first load (no dir)",
                         "V3 AoS16 dir + atomic + first", "V4 AoS16 dir + plain RMW + first",
                         "V5 rows32 key+sum+first in one line", "V6 SoA dir + plain RMW + first"};
  for (int grid : {CUS * 8, CUS * 32}) {
    for (int mode = 0; mode < 7; ++mode) {
      auto launch = [&](int r) {
        switch (mode) {
#define L(M) case M: k_pane<M><<<grid, 256>>>(batch(r), NB, dir, sum, first, rows, (i64)r * NB, sink); break;
          L(0) L(1) L(2) L(3) L(4) L(5) L(6)
#undef L
        }
      };
      for (int w = 0; w < 4; ++w) launch(w);
      t.start();
      for (int r = 0; r < IT; ++r) launch(r);
      const double us = t.stop() * 1e3 / IT;
      printf("%-44s grid=%5d %8.1f us/batch %6.2f G rec/s\n", names[mode], grid, us, NB / us / 1e3);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
