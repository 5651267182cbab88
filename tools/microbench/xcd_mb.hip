// XCD-private aggregation microbenchmark (gfx950): can one pass over (key, ts, value) aggregate into
// per-XCD copies of a 64K-pane table with atomics executed in that XCD's own L2?
//   X1  read24 alone (reference)
//   X2  read24 + agent-scope atomicAdd into ONE shared 64K table (the memory-side atomic rate)
//   X3  read24 + workgroup-scope atomicAdd into the table copy of HW_REG_XCC_ID
//   X4  X3 + guarded first-arrival atomicMin on the adjacent ordinal word
//   X5  X4 + a directory probe (random 8-B load from a 2 MiB table)
// Each run checks the summed copies against the exact wrapping sum of the values.
// Build: hipcc --offload-arch=gfx950 -O3 xcd_mb.hip -o xcd_mb
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
__device__ __forceinline__ int xcc_id() {   // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4)
  return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7);
}

constexpr int NB = 1 << 22;
constexpr int RING = 32;
constexpr int TAB = 1 << 16;
struct Cols { const i64* key; const i64* ts; const i64* val; };

__global__ __launch_bounds__(256) void k_read24(Cols c, int n, i64* sink) {
  i64 acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += gridDim.x * blockDim.x) {
    longlong2 a = ((const longlong2*)c.key)[i], b = ((const longlong2*)c.ts)[i], d = ((const longlong2*)c.val)[i];
    acc ^= a.x ^ a.y ^ b.x ^ b.y ^ d.x ^ d.y;
  }
  if (acc == 0x123456789) sink[0] = acc;
}

// MODE 0: agent atomics into copy 0; 1: workgroup scope into copy xcc; 2: + first arrival; 3: + directory probe
template <int MODE>
__global__ __launch_bounds__(256) void k_xcd(Cols c, int n, u64* tabs, const i64* dir, uint64_t dmask, i64 ord_base) {
  const int x = MODE == 0 ? 0 : xcc_id();
  u64* tab = tabs + (size_t)x * TAB * 2;   // [TAB] x {sum, first}
  for (int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x); i < n; i += 2 * gridDim.x * blockDim.x) {
    const longlong2 a = *(const longlong2*)(c.key + i), d = *(const longlong2*)(c.val + i);
    const i64 ks[2] = {a.x, a.y}, vs[2] = {d.x, d.y};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      uint32_t slot = (uint32_t)ks[e] & (TAB - 1);
      if (MODE >= 3) {
        const i64 dk = dir[fmix64((uint64_t)ks[e]) & dmask];
        slot ^= (uint32_t)(dk == 0x7fffffffffffffffll);   // keeps the probe live
      }
      u64* p = tab + 2 * (size_t)slot;
      if (MODE == 0) atomicAdd(p, (u64)vs[e]);
      else __hip_atomic_fetch_add(p, (u64)vs[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (MODE >= 2) {
        const i64 ord = ord_base + i + e;
        if (ord < (i64)p[1]) __hip_atomic_fetch_min((i64*)(p + 1), ord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
}

__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64(base + i) & 0xFFFF);
    ts[i] = 1700000000000ll + (i64)(((base + i) * 1000) >> 24);
    val[i] = (i64)mix64((base + i) ^ 0xabcdef);
  }
}
__global__ void k_init(u64* t, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    t[i] = (i & 1) ? 0x7fffffffffffffffull : 0ull;
}
__global__ void k_xcc_census(int* out) { if (threadIdx.x == 0) out[blockIdx.x] = xcc_id(); }

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUS = prop.multiProcessorCount;
  printf("device %s, %d CUs\n", prop.name, CUS);
  {
    int* d; CK(hipMalloc(&d, 4 * 64)); k_xcc_census<<<64, 64>>>(d); std::vector<int> h(64);
    CK(hipMemcpy(h.data(), d, 4 * 64, hipMemcpyDeviceToHost));
    printf("xcc id of blocks 0..23:"); for (int i = 0; i < 24; ++i) printf(" %d", h[i]); printf("\n");
  }
  const size_t colb = (size_t)NB * 8;
  char* ring; CK(hipMalloc(&ring, (size_t)RING * 3 * colb));
  for (int r = 0; r < RING; ++r) {
    char* b = ring + (size_t)r * 3 * colb;
    k_gen<<<2048, 256>>>((i64*)b, (i64*)(b + colb), (i64*)(b + 2 * colb), NB, (size_t)r * NB);
  }
  CK(hipDeviceSynchronize());
  auto batch = [&](int r) { char* b = ring + (size_t)(r % RING) * 3 * colb; return Cols{(const i64*)b, (const i64*)(b + colb), (const i64*)(b + 2 * colb)}; };
  const int IT = 32;
  std::vector<i64> hv(NB);
  u64 expect = 0;
  for (int r = 0; r < IT; ++r) {
    CK(hipMemcpy(hv.data(), batch(r).val, colb, hipMemcpyDeviceToHost));
    for (int i = 0; i < NB; ++i) expect += (u64)hv[i];
  }
  i64* sink; CK(hipMalloc(&sink, 64));
  const size_t tab_words = (size_t)8 * TAB * 2;
  u64* tabs; CK(hipMalloc(&tabs, tab_words * 8));
  i64* dir; CK(hipMalloc(&dir, 8ull << 18)); CK(hipMemset(dir, 0, 8ull << 18));
  Timer t;
  const double in_bytes = 24.0 * NB;
  auto rep = [&](const char* name, float ms_total) {
    double us = ms_total * 1e3 / IT;
    printf("%-48s %8.2f us/batch  %6.1f Gev/s  %7.1f GB/s input  (%.0f%% of 8 TB/s)\n", name, us, NB / us / 1e3,
           in_bytes / us / 1e3, 100.0 * in_bytes / us / 1e3 / 8000.0);
  };
  auto check = [&](const char* name) {
    std::vector<u64> h(tab_words);
    CK(hipMemcpy(h.data(), tabs, tab_words * 8, hipMemcpyDeviceToHost));
    u64 s = 0; for (size_t i = 0; i < tab_words; i += 2) s += h[i];
    printf("   %s: summed copies %s the value sum\n", name, s == expect ? "MATCH" : "DO NOT MATCH");
  };
  for (int grid : {CUS * 4, CUS * 8, CUS * 16}) {
    for (int w = 0; w < 4; ++w) k_read24<<<grid, 256>>>(batch(w), NB, sink);
    t.start(); for (int r = 0; r < IT; ++r) k_read24<<<grid, 256>>>(batch(r), NB, sink);
    char nm[64]; snprintf(nm, 64, "X1 read24 grid=%d", grid); rep(nm, t.stop());
  }
#define RUN(MODE, NAME, GRID)                                                                                      \
  {                                                                                                                \
    k_init<<<1024, 256>>>(tabs, tab_words); CK(hipDeviceSynchronize());                                            \
    t.start();                                                                                                     \
    for (int r = 0; r < IT; ++r) k_xcd<MODE><<<GRID, 256>>>(batch(r), NB, tabs, dir, (1ull << 18) - 1, (i64)r * NB); \
    char nm[80]; snprintf(nm, 80, "%s grid=%d", NAME, GRID); rep(nm, t.stop()); check(NAME);                        \
  }
  for (int grid : {CUS * 4, CUS * 8, CUS * 16}) {
    RUN(0, "X2 agent atomics, one table", grid);
    RUN(1, "X3 wg-scope atomics, XCD copy", grid);
    RUN(2, "X4 X3 + first-arrival min", grid);
    RUN(3, "X5 X4 + directory probe (2 MiB)", grid);
  }
  return 0;
}
