// Fire-pass microbenchmark (C1 shape): what one watermark's fire + purge costs on its own, phase by phase.
// 256 Ki key ids, a quarter present in the firing slice; per key id: the presence word, then (present) f1 and
// the sum, a block-aggregated append to a 4-column output log, then the slice column reset.
// Build: hipcc --offload-arch=gfx950 -O3 -o wm_mb wm_mb.hip ; run: ./wm_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int T = 1024;
struct Args {
  int64_t n;
  int64_t *first, *f1v, *sum, *keys;
  int64_t *okey, *of1, *ots, *osum;
  unsigned long long* count;
  unsigned int* done;
  int mode;   // bit 0: skip the append atomic (per-WG slots); bit 1: skip the purge; bit 2: skip the done counter;
              // bit 3: key loaded with the presence word; bit 4: unconditional loads; bit 5: no output stores
};

__global__ __launch_bounds__(T) void k_fire(Args a) {
  __shared__ int32_t wtot[T / 64];
  __shared__ unsigned long long base;
  __shared__ int last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t gs = (int64_t)gridDim.x * T;
  for (int64_t k0 = (int64_t)blockIdx.x * T; k0 < a.n; k0 += gs) {
    const int64_t kid = k0 + threadIdx.x;
    bool any = false;
    int64_t f1 = 0, sm = 0, key = 0;
    if (kid < a.n) {
      if (a.mode & 8) key = a.keys[kid];
      const int64_t o = a.first[kid];
      if (a.mode & 16) { f1 = a.f1v[kid]; sm = a.sum[kid]; any = o != INT64_MAX; }
      else if (o != INT64_MAX) { f1 = a.f1v[kid]; sm = a.sum[kid]; any = true; }
    }
    const uint64_t bal = __ballot(any);
    const int32_t rank = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) wtot[wave] = __popcll(bal);
    __syncthreads();
    int32_t off = 0, tot = 0;
    for (int w = 0; w < T / 64; ++w) { const int32_t c = wtot[w]; off += w < wave ? c : 0; tot += c; }
    if (threadIdx.x == 0) base = (a.mode & 1) ? (unsigned long long)blockIdx.x * T : atomicAdd(a.count, (unsigned long long)tot);
    __syncthreads();
    if (any && !(a.mode & 32)) {
      if (!(a.mode & 8)) key = a.keys[kid];
      const unsigned long long pos = base + off + rank;
      a.okey[pos] = key; a.of1[pos] = f1; a.ots[pos] = 999; a.osum[pos] = sm;
    }
    __syncthreads();
  }
  if (!(a.mode & 2)) {
    for (int64_t kid = (int64_t)blockIdx.x * T + threadIdx.x; kid < a.n; kid += gs) {
      a.sum[kid] = 0; a.first[kid] = INT64_MAX;
    }
  }
  if (!(a.mode & 4)) {
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(a.done, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) *a.done = 0;
  }
}

__global__ void k_init(Args a, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    const bool pres = (h & 3) == 0;
    a.first[i] = pres ? i : INT64_MAX;
    a.f1v[i] = i;
    a.sum[i] = pres ? 7 : 0;
    a.keys[i] = i * 3 + 1;
  }
}
__global__ void k_empty() {}

int main() {
  Args a{};
  a.n = 256 * 1024 + 1;
  int64_t** cols[] = {&a.first, &a.f1v, &a.sum, &a.keys, &a.okey, &a.of1, &a.ots, &a.osum};
  for (auto c : cols) CK(hipMalloc(c, 8 * a.n + 4096));
  CK(hipMalloc(&a.count, 8));
  CK(hipMalloc(&a.done, 4));
  CK(hipMemset(a.done, 0, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int modes[] = {0, 1, 2, 4, 8, 16, 32, 1 | 2 | 4, 1 | 2 | 4 | 32, 8 | 16, 2 | 8, 2 | 8 | 16, 1 | 2 | 4 | 8 | 16 | 32};
  const int grids[] = {257, 128, 64};
  // a bare launch, for scale
  {
    float best = 1e9f;
    for (int r = 0; r < 50; ++r) {
      hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0);
      CK(hipEventRecord(e0)); hipLaunchKernelGGL(k_empty, dim3(257), dim3(T), 0, 0); CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;
    }
    printf("empty 257x1024: min %.1f us\n", best * 1e3);
  }
  for (int g : grids) {
    for (int m : modes) {
      a.mode = m;
      std::vector<float> t;
      for (int r = 0; r < 40; ++r) {
        hipLaunchKernelGGL(k_init, dim3(1024), dim3(256), 0, 0, a, (uint32_t)r);
        CK(hipMemset(a.count, 0, 8));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_fire, dim3(g), dim3(T), 0, 0, a);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms * 1e3f);
      }
      float mn = 1e9f, sum = 0; for (float x : t) { mn = x < mn ? x : mn; sum += x; }
      printf("grid %3d mode %2d: min %6.1f us  avg %6.1f us\n", g, m, mn, sum / t.size());
    }
  }
  return 0;
}
