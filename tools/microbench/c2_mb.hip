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
//   V7  round 6: records first partitioned by directory range (NRANGE ranges of D / NRANGE
//       slots: per-tile LDS histograms, a column scan, a scatter of (slot, value) pairs), then V1 over the ranges
//       with range r's records on XCD r % 8 (the blocks of one XCD take its ranges in turn), so a range's directory
//       and pane lines are reused while they sit in that XCD's L2 — prints the partition and the update apart
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

// ---- V7: partition by directory range, then the SoA update over each range's records ----
constexpr int NRANGE = 1024, PT = 4096, PBLK = NB / PT;   // ranges; records per partition tile; tiles
__device__ __forceinline__ int range_of(u64 slot) { return (int)(slot / (D / NRANGE)); }
__global__ __launch_bounds__(1024) void k_phist(Cols c, unsigned* hist) {   // hist[range][tile]
  __shared__ unsigned h[NRANGE];
  for (int i = threadIdx.x; i < NRANGE; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < PT; i += blockDim.x)
    atomicAdd(&h[range_of(fmix64((u64)c.key[(size_t)blockIdx.x * PT + i]) & (D - 1))], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < NRANGE; i += blockDim.x) hist[(size_t)i * PBLK + blockIdx.x] = h[i];
}
// exclusive scan of hist in (range, tile) order, one block; also each range's start
__global__ __launch_bounds__(1024) void k_pscan(unsigned* hist, unsigned* rstart) {
  __shared__ unsigned tot[NRANGE];
  for (int r = threadIdx.x; r < NRANGE; r += blockDim.x) {
    unsigned s = 0;
    for (int b = 0; b < PBLK; ++b) { const unsigned x = hist[(size_t)r * PBLK + b]; hist[(size_t)r * PBLK + b] = s; s += x; }
    tot[r] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned s = 0;
    for (int r = 0; r < NRANGE; ++r) { rstart[r] = s; s += tot[r]; }
    rstart[NRANGE] = s;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < NRANGE; r += blockDim.x)
    for (int b = 0; b < PBLK; ++b) hist[(size_t)r * PBLK + b] += rstart[r];
}
__global__ __launch_bounds__(1024) void k_pscatter(Cols c, const unsigned* hist, u64* out_slot, i64* out_val) {
  __shared__ unsigned cur[NRANGE];
  for (int i = threadIdx.x; i < NRANGE; i += blockDim.x) cur[i] = hist[(size_t)i * PBLK + blockIdx.x];
  __syncthreads();
  for (int i = threadIdx.x; i < PT; i += blockDim.x) {
    const size_t g = (size_t)blockIdx.x * PT + i;
    const u64 slot = fmix64((u64)c.key[g]) & (D - 1);
    const unsigned pos = atomicAdd(&cur[range_of(slot)], 1u);
    out_slot[pos] = slot;
    out_val[pos] = c.val[g];
  }
}
// blocks: XCD x = b % 8 takes the ranges r = x (mod 8) in turn, PER blocks per range
constexpr int PER = 4;
__global__ __launch_bounds__(256) void k_prange(const u64* slots, const i64* vals, const unsigned* rstart, i64* dir,
                                                u64* sum, i64* first, i64 ord_base, i64* sink) {
  const int x = blockIdx.x & 7, idx = blockIdx.x >> 3;
  const int r = (idx / PER) * 8 + x, part = idx % PER;
  if (r >= NRANGE) return;
  const unsigned lo = rstart[r], hi = rstart[r + 1];
  i64 acc = 0;
  for (unsigned i = lo + part * blockDim.x + threadIdx.x; i < hi; i += PER * blockDim.x) {
    const u64 slot = slots[i];
    acc ^= dir[slot];
    atomicAdd(&sum[slot], (u64)vals[i]);
    if (ord_base + (i64)i < first[slot]) acc ^= 1;
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
  {   // V7
    unsigned *hist, *rstart; u64* pslot; i64* pval;
    CK(hipMalloc(&hist, (size_t)NRANGE * PBLK * 4)); CK(hipMalloc(&rstart, (NRANGE + 1) * 4));
    CK(hipMalloc(&pslot, (size_t)NB * 8)); CK(hipMalloc(&pval, (size_t)NB * 8));
    const int ublocks = NRANGE / 8 * PER * 8;
    auto part = [&](int r) {
      k_phist<<<PBLK, 1024>>>(batch(r), hist);
      k_pscan<<<1, 1024>>>(hist, rstart);
      k_pscatter<<<PBLK, 1024>>>(batch(r), hist, pslot, pval);
    };
    auto upd = [&](int r) { k_prange<<<ublocks, 256>>>(pslot, pval, rstart, dir, sum, first, (i64)r * NB, sink); };
    for (int w = 0; w < 4; ++w) { part(w); upd(w); }
    t.start();
    for (int r = 0; r < IT; ++r) part(r);
    const double us_p = t.stop() * 1e3 / IT;
    t.start();
    for (int r = 0; r < IT; ++r) upd(r);
    const double us_u = t.stop() * 1e3 / IT;
    t.start();
    for (int r = 0; r < IT; ++r) { part(r); upd(r); }
    const double us = t.stop() * 1e3 / IT;
    printf("%-44s partition %6.1f us + update %6.1f us = %6.1f us/batch %6.2f G rec/s\n",
           "V7 range-partitioned, XCD-local update", us_p, us_u, us, NB / us / 1e3);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
