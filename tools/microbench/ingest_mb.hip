// Ingest-shape microbenchmarks (gfx950): what one 2^22-event batch of (key, ts, value) int64 columns
// costs under the candidate ingest designs.  Input batches rotate through a 3 GiB ring so they are
// never Infinity-Cache resident; intermediates are reused across batches (as the engine's are).
// Build: hipcc --offload-arch=gfx950 -O3 ingest_mb.hip -o ingest_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

constexpr int NB = 1 << 22;          // events per batch
constexpr int RING = 32;             // batches in the ring (3 GiB)

struct Cols { const i64* key; const i64* ts; const i64* val; };

// T1: read the three columns, 2 records per lane per column (16-B loads)
__global__ __launch_bounds__(256) void k_read24(Cols c, int n, i64* sink) {
  const int2* k2 = (const int2*)c.key;
  i64 acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += gridDim.x * blockDim.x) {
    longlong2 a = ((const longlong2*)c.key)[i];
    longlong2 b = ((const longlong2*)c.ts)[i];
    longlong2 d = ((const longlong2*)c.val)[i];
    acc ^= a.x ^ a.y ^ b.x ^ b.y ^ d.x ^ d.y;
  }
  (void)k2;
  if (acc == 0x123456789) sink[0] = acc;
}

// T2/T3: read24 and write W bytes/event (W = 12: 4-B tag + 8-B value; 16: key + value) to a reused
// intermediate, each record sent to one of 256 buckets' regions (bucket-major, tile chunks)
template <int W>
__global__ __launch_bounds__(256) void k_read24_write(Cols c, int n, char* inter) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += gridDim.x * blockDim.x) {
    longlong2 a = ((const longlong2*)c.key)[i];
    longlong2 b = ((const longlong2*)c.ts)[i];
    longlong2 d = ((const longlong2*)c.val)[i];
    if (W == 16) {
      ((longlong2*)inter)[i] = make_longlong2(a.x ^ b.x, a.y ^ b.y);
      ((longlong2*)(inter + 8ll * n))[i] = d;
    } else {
      ((int2*)inter)[i] = make_int2((int)(a.x ^ b.x), (int)(a.y ^ b.y));
      ((longlong2*)(inter + 4ll * n))[i] = d;
    }
  }
}
template <int W>
__global__ __launch_bounds__(256) void k_read_inter(const char* inter, int n, i64* sink) {
  i64 acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += gridDim.x * blockDim.x) {
    if (W == 16) {
      longlong2 a = ((const longlong2*)inter)[i];
      longlong2 d = ((const longlong2*)(inter + 8ll * n))[i];
      acc ^= a.x ^ a.y ^ d.x ^ d.y;
    } else {
      int2 a = ((const int2*)inter)[i];
      longlong2 d = ((const longlong2*)(inter + 4ll * n))[i];
      acc ^= a.x ^ a.y ^ d.x ^ d.y;
    }
  }
  if (acc == 0x123456789) sink[0] = acc;
}

// T4: read24 + one agent-scope 64-bit atomic add per record into a 64K table (random)
__global__ __launch_bounds__(256) void k_read24_atomic(Cols c, int n, unsigned long long* tab) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    i64 k = c.key[i], v = c.val[i], t = c.ts[i];
    atomicAdd(&tab[(k ^ (t >> 40)) & 0xFFFF], (unsigned long long)v);
  }
}
// T5: atomics whose 64 lanes hit 64 consecutive words (one 512-B run per wave-instruction)
__global__ __launch_bounds__(256) void k_atomic_coalesced(int n, unsigned long long* tab, int runs) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int run = (int)(mix64(i >> 6) % runs);
    atomicAdd(&tab[run * 64 + (i & 63)], 1ull);
  }
}
// T6: read24 + random 8-B gather from an L2-sized table (directory probe model)
__global__ __launch_bounds__(256) void k_read24_gather(Cols c, int n, const i64* tab, uint64_t mask, i64* sink) {
  i64 acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    i64 k = c.key[i], v = c.val[i], t = c.ts[i];
    acc ^= tab[mix64((uint64_t)k) & mask] ^ v ^ t;
  }
  if (acc == 0x123456789) sink[0] = acc;
}
// T6b: same with 4 independent records per lane in flight
__global__ __launch_bounds__(256) void k_read24_gather4(Cols c, int n, const i64* tab, uint64_t mask, i64* sink) {
  i64 acc = 0;
  const int stride = gridDim.x * blockDim.x;
  for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += 4 * stride) {
    i64 k[4], v[4], t[4], d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { int i = min(i0 + u * stride, n - 1); k[u] = c.key[i]; v[u] = c.val[i]; t[u] = c.ts[i]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) d[u] = tab[mix64((uint64_t)k[u]) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= d[u] ^ v[u] ^ t[u];
  }
  if (acc == 0x123456789) sink[0] = acc;
}
// T8: LDS-resident aggregation of a tile: read24 + LDS atomic add into a 16K-slot table per block
__global__ __launch_bounds__(1024) void k_read24_lds(Cols c, int n, unsigned long long* out) {
  __shared__ unsigned long long lt[16384];
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) lt[j] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    i64 k = c.key[i], v = c.val[i], t = c.ts[i];
    atomicAdd(&lt[(k ^ t) & 16383], (unsigned long long)v);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) if (lt[j] == 0x1234567) out[0] = 1;
}
// T9: pass-1 model: read24 + directory gather + write 12 B (tag, value)
__global__ __launch_bounds__(256) void k_pass1_model(Cols c, int n, const i64* tab, uint64_t mask, char* inter) {
  const int stride = gridDim.x * blockDim.x;
  for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += 4 * stride) {
    i64 k[4], v[4], t[4], d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { int i = min(i0 + u * stride, n - 1); k[u] = c.key[i]; v[u] = c.val[i]; t[u] = c.ts[i]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) d[u] = tab[mix64((uint64_t)k[u]) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int i = i0 + u * stride;
      if (i < n) { ((int*)inter)[i] = (int)(d[u] ^ t[u]); ((i64*)(inter + 4ll * n))[i] = v[u]; }
    }
  }
}
__global__ void k_empty() {}
// C1-shaped random batch: keys uniform in [0, 65536), ts increasing, full-range values
__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64(base + i) & 0xFFFF);
    ts[i] = 1700000000000ll + (i64)(((base + i) * 1000) >> 24);
    val[i] = (i64)mix64((base + i) ^ 0xabcdef);
  }
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
  printf("device %s, %d CUs\n", prop.name, CUS);
  const size_t colb = (size_t)NB * 8;
  char* ring; CK(hipMalloc(&ring, (size_t)RING * 3 * colb));
  for (int r = 0; r < RING; ++r) {
    char* b = ring + (size_t)r * 3 * colb;
    k_gen<<<2048, 256>>>((i64*)b, (i64*)(b + colb), (i64*)(b + 2 * colb), NB, (size_t)r * NB);
  }
  CK(hipDeviceSynchronize());
  auto batch = [&](int r) { char* b = ring + (size_t)(r % RING) * 3 * colb; return Cols{(const i64*)b, (const i64*)(b + colb), (const i64*)(b + 2 * colb)}; };
  char* inter; CK(hipMalloc(&inter, 16ull * NB));
  i64* sink; CK(hipMalloc(&sink, 64));
  unsigned long long* tab; CK(hipMalloc(&tab, 64ull << 20)); CK(hipMemset(tab, 0, 64ull << 20));
  Timer t;
  const int IT = 64;
  const double in_bytes = 24.0 * NB;
  auto rep = [&](const char* name, float ms_total, double extra = 0) {
    double us = ms_total * 1e3 / IT;
    printf("%-44s %8.2f us/batch  %6.1f Gev/s  %7.1f GB/s input  (%.0f%% of 8 TB/s)\n", name, us, NB / us / 1e3,
           in_bytes / us / 1e3, 100.0 * in_bytes / us / 1e3 / 8000.0);
    (void)extra;
  };
  for (int grid : {CUS * 4, CUS * 8, CUS * 16}) {
    for (int w = 0; w < 8; ++w) k_read24<<<grid, 256>>>(batch(w), NB, sink);
    t.start(); for (int r = 0; r < IT; ++r) k_read24<<<grid, 256>>>(batch(r), NB, sink);
    char nm[64]; snprintf(nm, 64, "T1 read24 grid=%d", grid); rep(nm, t.stop());
  }
  const int G = CUS * 8;
  // T2/T3
  {
    for (int w = 0; w < 8; ++w) { k_read24_write<12><<<G, 256>>>(batch(w), NB, inter); k_read_inter<12><<<G, 256>>>(inter, NB, sink); }
    t.start(); for (int r = 0; r < IT; ++r) k_read24_write<12><<<G, 256>>>(batch(r), NB, inter);
    rep("T2a read24+write12 (pass 1 alone)", t.stop());
    t.start(); for (int r = 0; r < IT; ++r) k_read_inter<12><<<G, 256>>>(inter, NB, sink);
    rep("T2b read12 (pass 2 alone, hot)", t.stop());
    t.start(); for (int r = 0; r < IT; ++r) { k_read24_write<12><<<G, 256>>>(batch(r), NB, inter); k_read_inter<12><<<G, 256>>>(inter, NB, sink); }
    rep("T2 pass1+pass2 (12 B intermediate)", t.stop());
    t.start(); for (int r = 0; r < IT; ++r) { k_read24_write<16><<<G, 256>>>(batch(r), NB, inter); k_read_inter<16><<<G, 256>>>(inter, NB, sink); }
    rep("T3 pass1+pass2 (16 B intermediate)", t.stop());
  }
  // T4
  {
    for (int w = 0; w < 4; ++w) k_read24_atomic<<<G, 256>>>(batch(w), NB, tab);
    t.start(); for (int r = 0; r < IT; ++r) k_read24_atomic<<<G, 256>>>(batch(r), NB, tab);
    rep("T4 read24 + agent atomic (64K table)", t.stop());
  }
  // T5
  for (int runs : {1024, 16384}) {
    k_atomic_coalesced<<<G, 256>>>(NB, tab, runs);
    t.start(); for (int r = 0; r < IT; ++r) k_atomic_coalesced<<<G, 256>>>(NB, tab, runs);
    char nm[64]; snprintf(nm, 64, "T5 coalesced atomics (64 x 8B), %d runs", runs); rep(nm, t.stop());
  }
  // T6
  for (int lg : {17, 18, 21}) {
    uint64_t mask = (1ull << lg) - 1;
    k_read24_gather<<<G, 256>>>(batch(0), NB, (const i64*)tab, mask, sink);
    t.start(); for (int r = 0; r < IT; ++r) k_read24_gather<<<G, 256>>>(batch(r), NB, (const i64*)tab, mask, sink);
    char nm[64]; snprintf(nm, 64, "T6 read24 + gather (%d KB table)", (int)((8ull << lg) >> 10)); rep(nm, t.stop());
    t.start(); for (int r = 0; r < IT; ++r) k_read24_gather4<<<G, 256>>>(batch(r), NB, (const i64*)tab, mask, sink);
    snprintf(nm, 64, "T6b read24 + gather x4 (%d KB table)", (int)((8ull << lg) >> 10)); rep(nm, t.stop());
  }
  // T9
  for (int lg : {17, 18}) {
    uint64_t mask = (1ull << lg) - 1;
    t.start(); for (int r = 0; r < IT; ++r) k_pass1_model<<<G, 256>>>(batch(r), NB, (const i64*)tab, mask, inter);
    char nm[64]; snprintf(nm, 64, "T9 pass1 model gather+write12 (%d KB)", (int)((8ull << lg) >> 10)); rep(nm, t.stop());
    t.start(); for (int r = 0; r < IT; ++r) { k_pass1_model<<<G, 256>>>(batch(r), NB, (const i64*)tab, mask, inter); k_read_inter<12><<<G, 256>>>(inter, NB, sink); }
    snprintf(nm, 64, "T9+pass2 read (%d KB)", (int)((8ull << lg) >> 10)); rep(nm, t.stop());
  }
  // T8
  {
    k_read24_lds<<<CUS, 1024>>>(batch(0), NB, tab);
    t.start(); for (int r = 0; r < IT; ++r) k_read24_lds<<<CUS, 1024>>>(batch(r), NB, tab);
    rep("T8 read24 + LDS atomic (1 WG/CU)", t.stop());
    t.start(); for (int r = 0; r < IT; ++r) k_read24_lds<<<CUS * 2, 1024>>>(batch(r), NB, tab);
    rep("T8 read24 + LDS atomic (2 WG/CU req)", t.stop());
  }
  // T7 launch overhead
  {
    for (int w = 0; w < 100; ++w) k_empty<<<1, 64>>>();
    t.start(); for (int r = 0; r < 1000; ++r) k_empty<<<1, 64>>>();
    printf("T7 empty kernel back-to-back: %.2f us/launch\n", t.stop());
    t.start(); for (int r = 0; r < 1000; ++r) k_empty<<<G, 256>>>();
    printf("T7 empty kernel grid %d back-to-back: %.2f us/launch\n", G, t.stop());
  }
  return 0;
}
