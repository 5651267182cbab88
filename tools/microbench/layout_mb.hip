// Partitioned-ingest intermediate layout: tile-major segments (each tile written contiguously, bin-sorted;
// pass 2 gathers one segment per tile) against bucket-major regions (each tile's bin segment written at its
// place in the bin's contiguous region; pass 2 streams the region).  C1-shaped batches, 16-B records.
// Build: hipcc --offload-arch=gfx950 -O3 layout_mb.hip -o layout_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef unsigned long long u64;
constexpr int NB = 1 << 22;
constexpr int RING = 24;
constexpr int T = 4096, NT = 512, NBIN = 256;
constexpr int NTILES = NB / T;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
}
__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64((base + i) ^ 1) & 0xFFFF);
    ts[i] = 1700000000000ll + (i64)(((base + i) * 1000) >> 24);
    val[i] = (i64)mix64((base + i) ^ 2);
  }
}
__device__ __forceinline__ int bin_of(i64 key) { return (int)((fmix64((uint64_t)key) >> 10) & (NBIN - 1)); }

// per-(tile, bin) counts -> offsets (untimed setup for the bucket-major write pattern)
__global__ void k_hist(const i64* key, int* cnt) {
  __shared__ int c[NBIN];
  for (int x = threadIdx.x; x < NBIN; x += blockDim.x) c[x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < T; i += blockDim.x) atomicAdd(&c[bin_of(key[(i64)blockIdx.x * T + i])], 1);
  __syncthreads();
  for (int x = threadIdx.x; x < NBIN; x += blockDim.x) cnt[x * NTILES + blockIdx.x] = c[x];   // bin-major
}

// pass 1: MODE 0 tile-major output; MODE 1 bucket-major with precomputed offsets; MODE 2 bucket-major with
// per-tile atomic reservation on bin cursors
template <int MODE>
__global__ __launch_bounds__(NT) void k_p1(const i64* __restrict__ key, const i64* __restrict__ ts, const i64* __restrict__ val,
                                          longlong2* out, const int* offs, int* cursor, int* segs) {
  __shared__ longlong2 st[T];
  __shared__ int cnt[NBIN + 1];
  __shared__ int base_[NBIN];
  __shared__ int wt[NT / 64];
  constexpr int R = T / NT, V = R / 2;
  const i64 base = (i64)blockIdx.x * T;
  for (int x = threadIdx.x; x <= NBIN; x += NT) cnt[x] = 0;
  i64 kk[R], vv[R], tt[R];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const i64 i = base + 2 * (j * NT + threadIdx.x);
    longlong2 a = *(const longlong2*)(key + i), b = *(const longlong2*)(ts + i), c = *(const longlong2*)(val + i);
    kk[2 * j] = a.x; kk[2 * j + 1] = a.y; tt[2 * j] = b.x; tt[2 * j + 1] = b.y; vv[2 * j] = c.x; vv[2 * j + 1] = c.y;
  }
  __syncthreads();
  int bn[R], rk[R];
#pragma unroll
  for (int k = 0; k < R; ++k) { bn[k] = bin_of(kk[k] ^ (tt[k] & 0)); rk[k] = atomicAdd(&cnt[bn[k]], 1); }
  __syncthreads();
  // exclusive scan (NBIN + 1 <= NT)
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int v = threadIdx.x <= NBIN ? cnt[threadIdx.x] : 0, x = v;
    for (int o = 1; o < 64; o <<= 1) { int y = __shfl_up(x, o); if (lane >= o) x += y; }
    if (lane == 63) wt[w] = x;
    __syncthreads();
    int wb = 0;
    for (int q = 0; q < w; ++q) wb += wt[q];
    const int ex = wb + x - v;
    if (MODE == 1 && threadIdx.x < NBIN) base_[threadIdx.x] = offs[threadIdx.x * NTILES + blockIdx.x] - ex;
    if (MODE == 2 && threadIdx.x < NBIN) base_[threadIdx.x] = (v ? atomicAdd(&cursor[threadIdx.x], v) : 0) + threadIdx.x * (NB / NBIN * 2) - ex;
    __syncthreads();
    if (threadIdx.x <= NBIN) cnt[threadIdx.x] = ex;
    if (MODE == 0 && threadIdx.x <= NBIN) segs[blockIdx.x * (NBIN + 1) + threadIdx.x] = ex;
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < R; ++k) st[cnt[bn[k]] + rk[k]] = make_longlong2((i64)fmix64((uint64_t)kk[k]), vv[k]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int p = k * NT + threadIdx.x;
    if (MODE == 0) out[base + p] = st[p];
    else {
      // bin of position p: the last bin whose start <= p (binary search in cnt)
      int lo = 0, hi = NBIN - 1;
      while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (cnt[mid] <= p) lo = mid; else hi = mid - 1; }
      out[base_[lo] + p] = st[p];
    }
  }
}

// pass 2 over a bucket-major region: stream [start, start + n) of records, LDS atomic per record
__global__ __launch_bounds__(1024) void k_p2_stream(const longlong2* in, const int* start, const int* count, u64* out) {
  __shared__ u64 acc[1024 + 64];
  for (int x = threadIdx.x; x < 1024 + 64; x += 1024) acc[x] = 0;
  __syncthreads();
  const int b = blockIdx.x, n = count[b];
  const longlong2* p = in + start[b];
  constexpr int U = 8;
  for (int i0 = 0; i0 < n; i0 += 1024 * U) {
    longlong2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { const int i = min(i0 + u * 1024 + (int)threadIdx.x, n - 1); r[u] = p[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool act = i0 + u * 1024 + (int)threadIdx.x < n;
      atomicAdd(&acc[act ? (r[u].x & 1023) : 1024 + (threadIdx.x & 63)], (u64)r[u].y);
    }
  }
  __syncthreads();
  for (int x = threadIdx.x; x < 1024; x += 1024) out[(i64)b * 1024 + x] = acc[x];
}
// pass 2 over tile-major segments (16-lane groups, as the engine)
__global__ __launch_bounds__(1024) void k_p2_seg(const longlong2* in, const int* segs, u64* out) {
  __shared__ u64 acc[1024 + 64];
  __shared__ int sst[NTILES], sln[NTILES];
  const int b = blockIdx.x;
  for (int x = threadIdx.x; x < 1024 + 64; x += 1024) acc[x] = 0;
  for (int t = threadIdx.x; t < NTILES; t += 1024) { sst[t] = segs[t * (NBIN + 1) + b]; sln[t] = segs[t * (NBIN + 1) + b + 1] - sst[t]; }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = lane >> 4, sub = lane & 15;
  constexpr int UR = 6;
  for (int tb = wave * 4 * UR; tb < NTILES; tb += 16 * 4 * UR) {
    longlong2 ra[UR], rb[UR];
    bool aa[UR], ab[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int tt = tb + u * 4 + grp, t = min(tt, NTILES - 1);
      const int ln = tt < NTILES ? sln[t] : 0;
      aa[u] = sub < ln; ab[u] = sub + 16 < ln;
      ra[u] = in[(i64)t * T + (aa[u] ? sst[t] + sub : 0)];
      rb[u] = in[(i64)t * T + (ab[u] ? sst[t] + sub + 16 : 0)];
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      atomicAdd(&acc[aa[u] ? (ra[u].x & 1023) : 1024 + lane], (u64)ra[u].y);
      atomicAdd(&acc[ab[u] ? (rb[u].x & 1023) : 1024 + lane], (u64)rb[u].y);
    }
  }
  __syncthreads();
  for (int x = threadIdx.x; x < 1024; x += 1024) out[(i64)b * 1024 + x] = acc[x];
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main() {
  const size_t colb = (size_t)NB * 8;
  char* ring; CK(hipMalloc(&ring, (size_t)RING * 3 * colb));
  for (int r = 0; r < RING; ++r) {
    char* b = ring + (size_t)r * 3 * colb;
    k_gen<<<2048, 256>>>((i64*)b, (i64*)(b + colb), (i64*)(b + 2 * colb), NB, (size_t)r * NB);
  }
  auto col = [&](int r, int c) { return (const i64*)(ring + ((size_t)(r % RING) * 3 + c) * colb); };
  longlong2* out; CK(hipMalloc(&out, 16ull * NB * 2 + (1 << 20)));
  int *cnt, *segs, *cursor, *start, *count;
  CK(hipMalloc(&cnt, 4 * NBIN * NTILES)); CK(hipMalloc(&segs, 4 * (NBIN + 1) * NTILES));
  CK(hipMalloc(&cursor, 4 * NBIN)); CK(hipMalloc(&start, 4 * NBIN)); CK(hipMalloc(&count, 4 * NBIN));
  u64* acc; CK(hipMalloc(&acc, 8 * 1024 * NBIN));
  // offsets for batch 0 (the timed loop reuses batch-0 offsets for every batch: the pattern, not the data, matters)
  k_hist<<<NTILES, 256>>>(col(0, 0), cnt);
  std::vector<int> h(NBIN * NTILES), hs(NBIN), hc(NBIN);
  CK(hipMemcpy(h.data(), cnt, h.size() * 4, hipMemcpyDeviceToHost));
  int run = 0;
  for (int b = 0; b < NBIN; ++b) {
    hs[b] = run;
    int c = 0;
    for (int t = 0; t < NTILES; ++t) { int v = h[b * NTILES + t]; h[b * NTILES + t] = run; run += v; c += v; }
    hc[b] = c;
  }
  CK(hipMemcpy(cnt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(start, hs.data(), NBIN * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(count, hc.data(), NBIN * 4, hipMemcpyHostToDevice));
  const int IT = 48;
  Timer tm;
  auto rep = [&](const char* nm, float ms) { printf("%-52s %8.2f us/batch\n", nm, ms * 1e3 / IT); };
  // warm
  for (int r = 0; r < 4; ++r) { k_p1<0><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs); k_p2_seg<<<NBIN, 1024>>>(out, segs, acc); }
  tm.start(); for (int r = 0; r < IT; ++r) k_p1<0><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs);
  rep("p1 tile-major write", tm.stop());
  tm.start(); for (int r = 0; r < IT; ++r) k_p2_seg<<<NBIN, 1024>>>(out, segs, acc);
  rep("p2 segment gather (hot)", tm.stop());
  tm.start(); for (int r = 0; r < IT; ++r) { k_p1<0><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs); k_p2_seg<<<NBIN, 1024>>>(out, segs, acc); }
  rep("p1 + p2 tile-major / segment gather", tm.stop());
  tm.start(); for (int r = 0; r < IT; ++r) k_p1<1><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs);
  rep("p1 bucket-major write (precomputed offsets)", tm.stop());
  tm.start(); for (int r = 0; r < IT; ++r) k_p2_stream<<<NBIN, 1024>>>(out, start, count, acc);
  rep("p2 region stream (hot)", tm.stop());
  tm.start(); for (int r = 0; r < IT; ++r) { k_p1<1><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs); k_p2_stream<<<NBIN, 1024>>>(out, start, count, acc); }
  rep("p1 + p2 bucket-major / stream", tm.stop());
  tm.start();
  for (int r = 0; r < IT; ++r) {
    CK(hipMemsetAsync(cursor, 0, 4 * NBIN));
    k_p1<2><<<NTILES, NT>>>(col(r, 0), col(r, 1), col(r, 2), out, cnt, cursor, segs);
  }
  rep("p1 bucket-major write (atomic reservation) + memset", tm.stop());
  return 0;
}
