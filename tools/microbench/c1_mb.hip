// C1 pipeline study (round 5): what the partitioned ingest can reach on one MI355X when its two passes
// are lean and overlap.  C1 geometry: 4 Mi records per batch, 64 Ki uniform keys, one tumbling slice per
// batch, long sum + first arrival (f1 = timestamp).  Pass 1 (route) bin-sorts each 4096-record tile by
// directory bucket in LDS and writes (fmix64(key), value) 16 B + the in-tile index 2 B, with the segment
// table written bucket-major; pass 2 (aggregate) gives each of the 256 buckets to one workgroup: the
// bucket's segment row (contiguous), its directory slice, LDS atomics, one fold per touched pane.
// Variants: route one tile per workgroup / persistent with the next tile's loads in flight; aggregate at
// 512 / 1024 threads; the passes serial, on two streams with a ring of routed buffers, or as one launch
// with both roles (aggregate of batch j-1 beside route of batch j).  Every variant is checked against
// device atomics (sums, first-arrival ordinal and its f1).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 c1_mb.hip -o c1_mb
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef unsigned long long u64;
constexpr i64 EMPTY = INT64_MIN;
constexpr int NB = 1 << 22;        // records per batch
constexpr int TL = 12;
constexpr int T = 1 << TL;         // records per tile
constexpr int NTILE = NB / T;
constexpr int NBK = 256;           // directory buckets
constexpr int KBL = 10;
constexpr int KB = 1 << KBL;       // slots per bucket
constexpr int DL = 18;
constexpr i64 D = 1ll << DL;
constexpr int RING = 12;           // input batches resident
constexpr int RT_NT = 512;
constexpr int PER = T / RT_NT;     // 8 records per thread
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t EMPTY_H = 0x8f780810af31a493ull;   // fmix64(Long.MIN_VALUE)
constexpr i64 T0 = 1700000000000ll;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
}

struct Panes { i64* sum; i64* first; i64* f1; };   // one slice, [D]
struct Routed { longlong2* kv; uint16_t* idx; uint32_t* seg; };   // seg[bucket][tile] = start | end << 16

__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64((base + i) ^ 1) & 0xFFFF);
    ts[i] = T0 + (i64)(((base + i) * 1000) >> 24);
    val[i] = (i64)mix64((base + i) ^ 2);
  }
}
__global__ void k_fill(i64* p, i64 v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__device__ i64 dir_insert(i64* dir, i64 key) {
  const uint64_t home = fmix64((uint64_t)key) & (D - 1);
  const uint64_t kbm = KB - 1, base = home & ~kbm;
  uint64_t off = home & kbm;
  for (int p = 0; p < KB; ++p) {
    const uint64_t h = base + off;
    const i64 cur = dir[h];
    if (cur == key) return (i64)h;
    if (cur == EMPTY) {
      const u64 prev = atomicCAS((u64*)&dir[h], (u64)EMPTY, (u64)key);
      if ((i64)prev == EMPTY || (i64)prev == key) return (i64)h;
    }
    off = (off + 1) & kbm;
  }
  return -1;
}
// reference: device atomics per record
__global__ void k_ref(i64* dir, const i64* key, const i64* ts, const i64* val, int n, i64 ord_base, Panes p) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const i64 kid = dir_insert(dir, key[i]);
    atomicAdd((u64*)&p.sum[kid], (u64)val[i]);
    atomicMin(&p.first[kid], ord_base + i);
  }
}
__global__ void k_ref_f1(Panes p, const i64* const* ts_of_batch, i64 nb_batches) {
  for (i64 x = blockIdx.x * (i64)blockDim.x + threadIdx.x; x < D; x += (i64)gridDim.x * blockDim.x) {
    const i64 f = p.first[x];
    if (f == INT64_MAX) continue;
    p.f1[x] = ts_of_batch[f / NB][f % NB];
  }
}
__global__ void k_cmp(Panes a, Panes b, int* bad) {
  for (i64 x = blockIdx.x * (i64)blockDim.x + threadIdx.x; x < D; x += (i64)gridDim.x * blockDim.x) {
    if (a.sum[x] != b.sum[x]) atomicAdd(bad, 1);
    if (a.first[x] != b.first[x]) atomicAdd(bad + 1, 1);
    if (a.first[x] != INT64_MAX && a.f1[x] != b.f1[x]) atomicAdd(bad + 2, 1);
  }
}

// ------------------------------------------------------------------------------------------------
// pass 1: route one tile (LDS counting sort by bucket)
// ------------------------------------------------------------------------------------------------
constexpr size_t RT_LDS = (size_t)T * 18 + 4 * (NBK + 1) + 4 * 16;

struct RouteIn { const i64* key; const i64* ts; const i64* val; i64 m0; double inv_size; i64 size; long long* stamps; };
#define RST(k) do { if (in.stamps && threadIdx.x == 0) in.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

__device__ __forceinline__ void route_load(const RouteIn& in, int tile, i64 (&kk)[PER], i64 (&tt)[PER], i64 (&vv)[PER]) {
  typedef long long v2 __attribute__((ext_vector_type(2)));
  const i64 base = (i64)tile * T;
#pragma unroll
  for (int j = 0; j < PER / 2; ++j) {
    const i64 i = base + 2 * (j * RT_NT + (int)threadIdx.x);
    const v2 a = __builtin_nontemporal_load((const v2*)(in.key + i));
    const v2 c = __builtin_nontemporal_load((const v2*)(in.ts + i));
    const v2 d = __builtin_nontemporal_load((const v2*)(in.val + i));
    kk[2 * j] = a.x; kk[2 * j + 1] = a.y;
    tt[2 * j] = c.x; tt[2 * j + 1] = c.y;
    vv[2 * j] = d.x; vv[2 * j + 1] = d.y;
  }
}

// bins / ranks / LDS scatter of a loaded tile; returns after the barrier that publishes st_kv
__device__ __forceinline__ void route_sort(const RouteIn& in, int tile, Routed o, unsigned char* smem, i64 (&kk)[PER],
                                           const i64 (&tt)[PER], const i64 (&vv)[PER], int* other) {
  longlong2* st_kv = (longlong2*)smem;
  uint16_t* st_idx = (uint16_t*)(st_kv + T);
  int* cnt = (int*)(st_idx + T);
  int* wtot = cnt + NBK + 1;
  int bin[PER], rank[PER];
  int oth = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    // slice of the record: floor((ts - 0) / size) by reciprocal, corrected
    const i64 x = tt[k];
    i64 q = (i64)((double)x * in.inv_size);
    const i64 r = x - q * in.size;
    q += (r < 0) ? -1 : (r >= in.size ? 1 : 0);
    const uint64_t hk = fmix64((uint64_t)kk[k]);
    bin[k] = -1;
    rank[k] = 0;
    if (q == in.m0) {
      bin[k] = (int)((hk & (D - 1)) >> KBL);
      rank[k] = atomicAdd(&cnt[bin[k]], 1);
    } else {
      ++oth;
    }
    kk[k] = (i64)hk;
  }
  if (oth) atomicAdd(other, oth);
  __syncthreads();
  RST(2);
  // exclusive scan of cnt[0..NBK) by the first NBK threads; cnt[NBK] = total
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int c = 0, incl = 0;
  if (threadIdx.x < NBK) {
    c = cnt[threadIdx.x];
    incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) { const int y = __shfl_up(incl, off); if (lane >= off) incl += y; }
    if (lane == 63) wtot[wave] = incl;
  }
  __syncthreads();
  if (threadIdx.x < NBK) {
    int run = incl - c;
    for (int w = 0; w < wave; ++w) run += wtot[w];
    cnt[threadIdx.x] = run;
    o.seg[(i64)threadIdx.x * NTILE + tile] = (uint32_t)run | ((uint32_t)(run + c) << 16);
    if (threadIdx.x == NBK - 1) cnt[NBK] = run + c;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (bin[k] >= 0) {
      const int pos = cnt[bin[k]] + rank[k];
      st_kv[pos] = make_longlong2(kk[k], vv[k]);
      st_idx[pos] = (uint16_t)(2 * ((k >> 1) * RT_NT + (int)threadIdx.x) + (k & 1));
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void route_store(int tile, Routed o, unsigned char* smem) {
  const longlong2* st_kv = (const longlong2*)smem;
  const uint16_t* st_idx = (const uint16_t*)(st_kv + T);
  const int* cnt = (const int*)(st_idx + T);
  const int total = cnt[NBK];
  const i64 base = (i64)tile * T;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int pos = k * RT_NT + (int)threadIdx.x;
    if (pos < total) o.kv[base + pos] = st_kv[pos];
  }
#pragma unroll
  for (int j = 0; j < PER / 2; ++j) {
    const int pos = 2 * (j * RT_NT + (int)threadIdx.x);
    if (pos < total) *(uint32_t*)(o.idx + base + pos) = *(const uint32_t*)(st_idx + pos);
  }
}

__device__ __forceinline__ void route_reset(unsigned char* smem) {
  int* cnt = (int*)(smem + (size_t)T * 18);
  for (int x = threadIdx.x; x <= NBK; x += RT_NT) cnt[x] = 0;
}

// PERSIST: tile loop with the next tile's loads issued before this tile's write-out
template <bool PERSIST>
__device__ __forceinline__ void route_role(const RouteIn& in, Routed o, unsigned char* smem, int wg, int nwg, int* other) {
  i64 kk[PER], tt[PER], vv[PER];
  if (!PERSIST) {
    RST(0);
    route_reset(smem);
    route_load(in, wg, kk, tt, vv);
    __syncthreads();
    RST(1);
    route_sort(in, wg, o, smem, kk, tt, vv, other);
    RST(3);
    route_store(wg, o, smem);
    RST(4);
    return;
  }
  int tile = wg;
  if (tile >= NTILE) return;
  route_reset(smem);
  route_load(in, tile, kk, tt, vv);
  __syncthreads();
  for (;;) {
    route_sort(in, tile, o, smem, kk, tt, vv, other);
    const int next = tile + nwg;
    if (next < NTILE) route_load(in, next, kk, tt, vv);   // in flight during the write-out
    route_store(tile, o, smem);
    if (next >= NTILE) break;
    __syncthreads();   // st_kv read by every thread's write-out before the next scatter
    route_reset(smem);
    __syncthreads();
    tile = next;
  }
}

template <bool PERSIST>
__global__ __launch_bounds__(RT_NT, 4) void k_route(RouteIn in, Routed o, int* other) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  route_role<PERSIST>(in, o, smem, blockIdx.x, gridDim.x, other);
}

// ------------------------------------------------------------------------------------------------
// pass 2: aggregate one bucket
// ------------------------------------------------------------------------------------------------
constexpr int AG_STEPS = 1024;   // wave steps tabulated per chunk
__host__ __device__ constexpr size_t ag_lds() {
  return (size_t)8 * KB + (size_t)8 * (KB + 64) + (size_t)4 * (KB + 64) + (size_t)4 * NTILE + (size_t)4 * (NTILE + 1 + 8) +
         4 * AG_STEPS + 4 * 32 + 16;
}

struct AggIn { const i64* dir; const i64* f1col; i64 ord_base; long long* stamps; const i64* hdr; int mode; };
#define ST(k) do { if (in.stamps && threadIdx.x == 0) in.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

template <int NT, int UR>
__device__ __forceinline__ void agg_role(const AggIn& in, Routed r, Panes p, unsigned char* smem, int vb) {
  const int bkt = (vb % 8) * (NBK / 8) + vb / 8;   // XCD x (blocks dealt round-robin) takes a contiguous bucket range
  uint64_t* lh = (uint64_t*)smem;
  i64* lsum = (i64*)(lh + KB);
  uint32_t* lfirst = (uint32_t*)(lsum + KB + 64);
  uint32_t* lseg = lfirst + KB + 64;
  int* off = (int*)(lseg + NTILE);
  int* step_tile = off + NTILE + 1 + 8;
  int* wt = step_tile + AG_STEPS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i64 dbase = (i64)bkt * KB;
  ST(0);
  // prologue: the bucket's segment row and directory slice, loads independent
  if (in.mode & 1) {   // engine-like: per-tile headers (2 slices) + 2 segment rows
    for (int t = threadIdx.x; t < NTILE; t += NT) {
      const i64 h0 = in.hdr[2 * t], h1 = in.hdr[2 * t + 1];
      const uint32_t a = r.seg[(i64)bkt * NTILE + t], b2 = r.seg[(i64)(bkt + NBK) * NTILE + t];
      lseg[t] = h0 != EMPTY ? a : (h1 != EMPTY ? b2 : 0u);
    }
  } else
  for (int t = threadIdx.x; t < NTILE; t += NT) lseg[t] = r.seg[(i64)bkt * NTILE + t];
  for (int x = threadIdx.x; x < KB; x += NT) lh[x] = fmix64((uint64_t)in.dir[dbase + x]);
  for (int x = threadIdx.x; x < KB + 64; x += NT) { lsum[x] = 0; lfirst[x] = NONE; }
  __syncthreads();
  ST(1);
  // exclusive prefix of the segment lengths: NTILE / NT per thread, contiguous
  {
    constexpr int PT = NTILE / NT;
    int loc[PT], s = 0;
#pragma unroll
    for (int i = 0; i < PT; ++i) { const uint32_t g = lseg[threadIdx.x * PT + i]; loc[i] = (int)(g >> 16) - (int)(g & 0xFFFF); s += loc[i]; }
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const int y = __shfl_up(incl, o); if (lane >= o) incl += y; }
    if (lane == 63) wt[wave] = incl;
    __syncthreads();
    int run = incl - s;
    for (int w = 0; w < wave; ++w) run += wt[w];
#pragma unroll
    for (int i = 0; i < PT; ++i) { off[threadIdx.x * PT + i] = run; run += loc[i]; }
    if (threadIdx.x == NT - 1) off[NTILE] = run;
    if (threadIdx.x < 8) off[NTILE + 1 + threadIdx.x] = 0x7fffffff;
  }
  __syncthreads();
  ST(2);
  const int R = off[NTILE];
  for (int cb = 0; cb < R; cb += AG_STEPS * 64) {
    for (int t = threadIdx.x; t < NTILE; t += NT) {
      const int o = off[t], l = off[t + 1] - o;
      if (l == 0) continue;
      const int s_lo = max(0, (o - cb + 63) >> 6), s_hi = min(AG_STEPS, (o + l - cb + 63) >> 6);
      for (int st = s_lo; st < s_hi; ++st) step_tile[st] = t;
    }
    __syncthreads();
    const int nsteps = min(AG_STEPS, (R - cb + 63) >> 6);
    auto load = [&](int s0, longlong2* rv, uint32_t* ri, bool* ra) {
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int st = s0 + u;
        const int rr = cb + 64 * st + lane;
        ra[u] = st < nsteps && rr < R;
        int t = 0;
        i64 pos = 0;
        if (ra[u]) {
          t = step_tile[st];
          if (in.mode & 2) {   // engine-like: independent broadcast reads of the next 8 segment ends
            const int t0 = t;
#pragma unroll
            for (int j = 1; j <= 8; ++j) t += off[t0 + j] <= rr ? 1 : 0;
          }
          while (off[t + 1] <= rr) ++t;
          pos = (i64)t * T + (lseg[t] & 0xFFFF) + (rr - off[t]);
        }
        rv[u] = r.kv[pos];
        ri[u] = ((uint32_t)t << TL) | (uint32_t)r.idx[pos];
      }
    };
    auto process = [&](const longlong2* rv, const uint32_t* ri, const bool* ra) {
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const uint64_t h = (uint64_t)rv[u].x;
        const uint32_t h0 = (uint32_t)h & (KB - 1);
        uint32_t kl = h0;
        bool found = false;
        if (in.mode & 4) {   // engine-like 8-slot window
#pragma unroll
          for (int j = 7; j >= 0; --j) { const uint32_t x = (h0 + j) & (KB - 1); const bool m = lh[x] == h; kl = m ? x : kl; found |= m; }
        } else {
#pragma unroll
          for (int j = 3; j >= 0; --j) { const uint32_t x = (h0 + j) & (KB - 1); const bool m = lh[x] == h; kl = m ? x : kl; found |= m; }
        }
        if (__any(ra[u] && !found) && ra[u] && !found) {
          uint32_t x = (h0 + 4) & (KB - 1);
          for (int q = 0; q < KB; ++q, x = (x + 1) & (KB - 1)) if (lh[x] == h) break;
          kl = x;
        }
        kl = ra[u] ? kl : (uint32_t)KB + (uint32_t)lane;
        atomicAdd((u64*)&lsum[kl], (u64)rv[u].y);
        atomicMin(&lfirst[kl], ri[u]);
      }
    };
    longlong2 rvA[UR], rvB[UR];
    uint32_t riA[UR], riB[UR];
    bool raA[UR], raB[UR];
    constexpr int G = (NT / 64) * UR;
    int s0 = wave * UR;
    if (s0 < nsteps) load(s0, rvA, riA, raA);
    while (s0 < nsteps) {
      if (s0 + G < nsteps) load(s0 + G, rvB, riB, raB);
      process(rvA, riA, raA);
      s0 += G;
      if (s0 >= nsteps) break;
      if (s0 + G < nsteps) load(s0 + G, rvA, riA, raA);
      process(rvB, riB, raB);
      s0 += G;
    }
    __syncthreads();
  }
  ST(3);
  // fold: this workgroup is the only writer of the bucket's panes
  for (int x = threadIdx.x; x < KB; x += NT) {
    const uint32_t lf = lfirst[x];
    if (lf == NONE) continue;
    const i64 idx = dbase + x;
    p.sum[idx] = (i64)((u64)p.sum[idx] + (u64)lsum[x]);
    const i64 o = in.ord_base + (i64)lf;
    if (o < p.first[idx]) { p.first[idx] = o; p.f1[idx] = in.f1col[lf]; }
  }
  __syncthreads();
  ST(4);
}

template <int NT, int UR>
__global__ __launch_bounds__(NT, 4) void k_agg(AggIn in, Routed r, Panes p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  agg_role<NT, UR>(in, r, p, smem, blockIdx.x);
}

// both roles in one launch: blocks [0, NBK) aggregate batch j-1 (when agg_on), the rest route batch j
template <bool PERSIST>
__global__ __launch_bounds__(RT_NT, 4) void k_dual(int agg_on, AggIn ain, Routed ar, Panes p, RouteIn rin, Routed ro,
                                                   int nroute, int* other) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int na = agg_on ? NBK : 0;
  if ((int)blockIdx.x < na) { agg_role<RT_NT, 2>(ain, ar, p, smem, blockIdx.x); return; }
  route_role<PERSIST>(rin, ro, smem, blockIdx.x - na, nroute, other);
}

// ------------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------------
struct Ctx {
  i64* cols[RING][3];
  i64* dir;
  Routed rb[3];
  Panes pane, ref;
  int* other;
  int* bad;
};

static void reset_panes(Panes p) {
  k_fill<<<1024, 256>>>(p.sum, 0, D);
  k_fill<<<1024, 256>>>(p.first, INT64_MAX, D);
  k_fill<<<1024, 256>>>(p.f1, 0, D);
}

static long long* g_rstamps = nullptr;
static RouteIn rin_of(Ctx& c, int j) {
  RouteIn in;
  in.stamps = g_rstamps;
  in.key = c.cols[j % RING][0]; in.ts = c.cols[j % RING][1]; in.val = c.cols[j % RING][2];
  in.size = 1000; in.inv_size = 1.0 / 1000; in.m0 = (T0 + ((i64)(j % 4) * NB * 1000 >> 24)) / 1000;
  // every batch of a run of 4 lies in the same second: batches 4a..4a+3 of the ring start at index (j%RING)*NB
  in.m0 = (T0 + (((i64)(j % RING) * NB) * 1000 >> 24)) / 1000;
  return in;
}
static long long* g_stamps = nullptr; static i64* g_hdr = nullptr; static int g_mode = 0;
static AggIn ain_of(Ctx& c, int j) { return AggIn{c.dir, c.cols[j % RING][1], (i64)(j % RING) * NB, g_stamps, g_hdr, g_mode}; }

enum Mode { SERIAL = 0, STREAMS = 1, DUAL = 2 };

template <bool PERSIST, int ANT, int AUR>
static float run(Ctx& c, Mode mode, int nbatch, int rgrid, hipStream_t s0, hipStream_t s1, std::vector<hipEvent_t>& ev_r,
                 std::vector<hipEvent_t>& ev_a, int nbuf) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, s0));
  for (int j = 0; j < nbatch; ++j) {
    const int q = j % nbuf;
    RouteIn rin = rin_of(c, j);
    if (mode == SERIAL) {
      k_route<PERSIST><<<rgrid, RT_NT, RT_LDS, s0>>>(rin, c.rb[q], c.other);
      k_agg<ANT, AUR><<<NBK, ANT, ag_lds(), s0>>>(ain_of(c, j), c.rb[q], c.pane);
    } else if (mode == STREAMS) {
      if (j >= nbuf) CK(hipStreamWaitEvent(s1, ev_a[(j - nbuf) % ev_a.size()], 0));   // buffer q free
      if (j == 0) CK(hipStreamWaitEvent(s1, a, 0));
      k_route<PERSIST><<<rgrid, RT_NT, RT_LDS, s1>>>(rin, c.rb[q], c.other);
      CK(hipEventRecord(ev_r[j % ev_r.size()], s1));
      CK(hipStreamWaitEvent(s0, ev_r[j % ev_r.size()], 0));
      k_agg<ANT, AUR><<<NBK, ANT, ag_lds(), s0>>>(ain_of(c, j), c.rb[q], c.pane);
      CK(hipEventRecord(ev_a[j % ev_a.size()], s0));
    } else {
      const int qp = (j + 1) % 2;   // two buffers: batch j-1 in (j-1)%2
      k_dual<PERSIST><<<(j > 0 ? NBK : 0) + rgrid, RT_NT, RT_LDS, s0>>>(j > 0, ain_of(c, j - 1), c.rb[qp], c.pane, rin,
                                                                         c.rb[j % 2], rgrid, c.other);
    }
  }
  if (mode == DUAL)
    k_agg<RT_NT, 2><<<NBK, RT_NT, ag_lds(), s0>>>(ain_of(c, nbatch - 1), c.rb[(nbatch - 1) % 2], c.pane);
  if (mode == STREAMS) {
    CK(hipEventRecord(b, s1));
    CK(hipStreamWaitEvent(s0, b, 0));
  }
  CK(hipEventRecord(b, s0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
  return ms / nbatch;
}

template <bool PERSIST, int ANT, int AUR>
static void variant(Ctx& c, const char* name, Mode mode, int rgrid, hipStream_t s0, hipStream_t s1,
                    std::vector<hipEvent_t>& ev_r, std::vector<hipEvent_t>& ev_a, int nbuf) {
  CK(hipFuncSetAttribute((const void*)k_route<PERSIST>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RT_LDS));
  CK(hipFuncSetAttribute((const void*)k_dual<PERSIST>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RT_LDS));
  CK(hipFuncSetAttribute((const void*)k_agg<ANT, AUR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ag_lds()));
  // correctness: 4 batches (one slice) from empty panes against the reference
  reset_panes(c.pane);
  CK(hipMemset(c.other, 0, 4));
  CK(hipDeviceSynchronize());
  run<PERSIST, ANT, AUR>(c, mode, 4, rgrid, s0, s1, ev_r, ev_a, nbuf);
  CK(hipMemset(c.bad, 0, 12));
  k_cmp<<<1024, 256>>>(c.pane, c.ref, c.bad);
  int hb[3], ho;
  CK(hipMemcpy(hb, c.bad, 12, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&ho, c.other, 4, hipMemcpyDeviceToHost));
  // timing: the ring's 12 batches, 4 times (checked state is discarded)
  run<PERSIST, ANT, AUR>(c, mode, 12, rgrid, s0, s1, ev_r, ev_a, nbuf);
  float best = 1e9, sum = 0;
  for (int rep = 0; rep < 4; ++rep) {
    const float ms = run<PERSIST, ANT, AUR>(c, mode, 48, rgrid, s0, s1, ev_r, ev_a, nbuf);
    best = std::min(best, ms);
    sum += ms;
  }
  printf("%-46s %7.2f us/batch (best %7.2f)  %6.1f Gev/s  frac %.3f  check %s%s\n", name, sum / 4 * 1e3, best * 1e3,
         NB / (sum / 4) / 1e6, 24.0 * NB / (sum / 4 / 1e3) / 8e12, (hb[0] | hb[1] | hb[2]) ? "BAD" : "ok",
         ho ? " (other-slice records!)" : "");
  if (hb[0] | hb[1] | hb[2]) printf("   mismatches: sum %d first %d f1 %d\n", hb[0], hb[1], hb[2]);
  fflush(stdout);
}

// floors: a 24-B read and a 24-B read + 16-B write per record
__global__ __launch_bounds__(256) void k_read24(const i64* a, const i64* b, const i64* c, i64* sink) {
  typedef long long v2 __attribute__((ext_vector_type(2)));
  i64 acc = 0;
  for (int i = 2 * (blockIdx.x * 256 + threadIdx.x); i < NB; i += 2 * 256 * gridDim.x) {
    const v2 x = __builtin_nontemporal_load((const v2*)(a + i));
    const v2 y = __builtin_nontemporal_load((const v2*)(b + i));
    const v2 z = __builtin_nontemporal_load((const v2*)(c + i));
    acc += x.x ^ y.y ^ z.x ^ x.y ^ y.x ^ z.y;
  }
  if (acc == 42) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_copy40(const i64* a, const i64* b, const i64* c, longlong2* o) {
  typedef long long v2 __attribute__((ext_vector_type(2)));
  for (int i = 2 * (blockIdx.x * 256 + threadIdx.x); i < NB; i += 2 * 256 * gridDim.x) {
    const v2 x = __builtin_nontemporal_load((const v2*)(a + i));
    const v2 y = __builtin_nontemporal_load((const v2*)(b + i));
    const v2 z = __builtin_nontemporal_load((const v2*)(c + i));
    o[i] = make_longlong2(x.x ^ y.x, z.x);
    o[i + 1] = make_longlong2(x.y ^ y.y, z.y);
  }
}
__global__ __launch_bounds__(256) void k_read16(const longlong2* o, i64* sink) {
  i64 acc = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < NB; i += 256 * gridDim.x) { const longlong2 v = o[i]; acc += v.x ^ v.y; }
  if (acc == 42) sink[0] = acc;
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  Ctx c;
  for (int r = 0; r < RING; ++r)
    for (int k = 0; k < 3; ++k) CK(hipMalloc(&c.cols[r][k], 8ull * NB));
  for (int r = 0; r < RING; ++r) k_gen<<<2048, 256>>>(c.cols[r][0], c.cols[r][1], c.cols[r][2], NB, (size_t)r * NB);
  CK(hipMalloc(&c.dir, 8 * D));
  k_fill<<<1024, 256>>>(c.dir, EMPTY, D);
  for (int q = 0; q < 3; ++q) {
    CK(hipMalloc(&c.rb[q].kv, 16ull * NB));
    CK(hipMalloc(&c.rb[q].idx, 2ull * NB));
    CK(hipMalloc(&c.rb[q].seg, 4ull * NBK * NTILE));
  }
  for (Panes* p : {&c.pane, &c.ref}) { CK(hipMalloc(&p->sum, 8 * D)); CK(hipMalloc(&p->first, 8 * D)); CK(hipMalloc(&p->f1, 8 * D)); }
  CK(hipMalloc(&c.other, 4));
  CK(hipMalloc(&c.bad, 12));
  // reference over batches 0..3 (the directory is filled by it, as the engine's would be after warm-up)
  reset_panes(c.ref);
  for (int j = 0; j < 4; ++j) k_ref<<<2048, 256>>>(c.dir, c.cols[j][0], c.cols[j][1], c.cols[j][2], NB, (i64)j * NB, c.ref);
  {
    const i64* h[RING];
    for (int r = 0; r < RING; ++r) h[r] = c.cols[r][1];
    const i64** d;
    CK(hipMalloc(&d, sizeof(h)));
    CK(hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice));
    k_ref_f1<<<1024, 256>>>(c.ref, d, RING);
  }
  CK(hipDeviceSynchronize());
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev_r(8), ev_a(8);
  for (auto& e : ev_r) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : ev_a) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  // floors
  {
    i64* sink; CK(hipMalloc(&sink, 8));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int g : {1024, 2048}) {
      CK(hipEventRecord(a));
      for (int j = 0; j < 48; ++j) k_read24<<<g, 256>>>(c.cols[j % RING][0], c.cols[j % RING][1], c.cols[j % RING][2], sink);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      printf("floor read24 grid %-5d                         %7.2f us/batch  %6.2f TB/s\n", g, ms / 48 * 1e3, 24.0 * NB / (ms / 48 / 1e3) / 1e12);
      CK(hipEventRecord(a));
      for (int j = 0; j < 48; ++j) k_copy40<<<g, 256>>>(c.cols[j % RING][0], c.cols[j % RING][1], c.cols[j % RING][2], c.rb[j % 2].kv);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      printf("floor read24+write16 grid %-5d                 %7.2f us/batch  %6.2f TB/s\n", g, ms / 48 * 1e3, 40.0 * NB / (ms / 48 / 1e3) / 1e12);
      CK(hipEventRecord(a));
      for (int j = 0; j < 48; ++j) k_read16<<<g, 256>>>(c.rb[j % 2].kv, sink);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      printf("floor read16 (two 64 MB buffers) grid %-5d     %7.2f us/batch  %6.2f TB/s\n", g, ms / 48 * 1e3, 16.0 * NB / (ms / 48 / 1e3) / 1e12);
    }
    fflush(stdout);
  }
  // route alone / aggregate alone
  {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    CK(hipFuncSetAttribute((const void*)k_route<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RT_LDS));
    CK(hipFuncSetAttribute((const void*)k_route<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RT_LDS));
    CK(hipFuncSetAttribute((const void*)k_agg<512, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ag_lds()));
    CK(hipFuncSetAttribute((const void*)k_agg<512, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ag_lds()));
    CK(hipFuncSetAttribute((const void*)k_agg<1024, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ag_lds()));
    CK(hipEventRecord(a));
    for (int j = 0; j < 48; ++j) k_route<false><<<NTILE, RT_NT, RT_LDS>>>(rin_of(c, j), c.rb[j % 2], c.other);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("route alone, one tile per WG                   %7.2f us/batch\n", ms / 48 * 1e3);
    for (int g : {256, 512}) {
      CK(hipEventRecord(a));
      for (int j = 0; j < 48; ++j) k_route<true><<<g, RT_NT, RT_LDS>>>(rin_of(c, j), c.rb[j % 2], c.other);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      printf("route alone, persistent grid %-4d              %7.2f us/batch\n", g, ms / 48 * 1e3);
    }
    reset_panes(c.pane);
    CK(hipEventRecord(a));
    for (int j = 0; j < 48; ++j) k_agg<512, 2><<<NBK, 512, ag_lds()>>>(ain_of(c, j), c.rb[j % 2], c.pane);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("aggregate alone, 512 thr UR2                   %7.2f us/batch\n", ms / 48 * 1e3);
    CK(hipEventRecord(a));
    for (int j = 0; j < 48; ++j) k_agg<512, 4><<<NBK, 512, ag_lds()>>>(ain_of(c, j), c.rb[j % 2], c.pane);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("aggregate alone, 512 thr UR4                   %7.2f us/batch\n", ms / 48 * 1e3);
    CK(hipEventRecord(a));
    for (int j = 0; j < 48; ++j) k_agg<1024, 2><<<NBK, 1024, ag_lds()>>>(ain_of(c, j), c.rb[j % 2], c.pane);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("aggregate alone, 1024 thr UR2                  %7.2f us/batch\n", ms / 48 * 1e3);
    CK(hipFuncSetAttribute((const void*)k_agg<1024, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    CK(hipEventRecord(a));
    for (int j = 0; j < 48; ++j) k_agg<1024, 2><<<NBK, 1024, 81 * 1024>>>(ain_of(c, j), c.rb[j % 2], c.pane);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("aggregate alone, 1024 thr UR2, 81 KB LDS       %7.2f us/batch\n", ms / 48 * 1e3);
    fflush(stdout);
    CK(hipMalloc(&g_stamps, 8 * 8 * NBK)); CK(hipMalloc(&g_hdr, 16 * NTILE));
    k_fill<<<64, 256>>>(g_hdr, 0, 2 * NTILE);
    CK(hipFuncSetAttribute((const void*)k_agg<1024, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    for (int mode : {0, 2, 4, 6, 8}) {
      g_mode = mode;
      const size_t lds = (mode & 8) ? 81 * 1024 : ag_lds();   // 8: one workgroup per CU as the engine forces
      for (int rep = 0; rep < 3; ++rep) {
        k_route<false><<<NTILE, RT_NT, RT_LDS>>>(rin_of(c, rep), c.rb[0], c.other);
        k_agg<1024, 2><<<NBK, 1024, lds>>>(ain_of(c, rep), c.rb[0], c.pane);
      }
      CK(hipDeviceSynchronize());
      std::vector<long long> h(8 * NBK);
      CK(hipMemcpy(h.data(), g_stamps, 8 * 8 * NBK, hipMemcpyDeviceToHost));
      long long t0 = h[0], tend = 0; double ph[4] = {0};
      for (int b = 0; b < NBK; ++b) { t0 = std::min(t0, h[8 * b]); tend = std::max(tend, h[8 * b + 4]); for (int k = 0; k < 4; ++k) ph[k] += (h[8 * b + k + 1] - h[8 * b + k]) * 10.0 / NBK; }
      printf("   agg 1024 stamps mode %d (ns): prologue %.0f scan %.0f main %.0f fold %.0f | span %.0f\n", mode, ph[0], ph[1], ph[2], ph[3], (tend - t0) * 10.0);
    }
    g_mode = 0; g_stamps = nullptr;
    CK(hipMalloc(&g_rstamps, 8 * 8 * NTILE));
    for (int rep = 0; rep < 3; ++rep) k_route<false><<<NTILE, RT_NT, RT_LDS>>>(rin_of(c, rep), c.rb[0], c.other);
    CK(hipDeviceSynchronize());
    {
      std::vector<long long> h(8 * NTILE);
      CK(hipMemcpy(h.data(), g_rstamps, 8 * 8 * NTILE, hipMemcpyDeviceToHost));
      long long t0 = h[0], tend = 0; double ph[4] = {0}, sk = 0;
      for (int b = 0; b < NTILE; ++b) { t0 = std::min(t0, h[8 * b]); tend = std::max(tend, h[8 * b + 4]); }
      for (int b = 0; b < NTILE; ++b) { sk += (h[8 * b] - t0) * 10.0 / NTILE; for (int k = 0; k < 4; ++k) ph[k] += (h[8 * b + k + 1] - h[8 * b + k]) * 10.0 / NTILE; }
      printf("   route stamps (ns): start-skew %.0f load %.0f bins %.0f scan+scatter %.0f write %.0f | span %.0f\n", sk, ph[0], ph[1], ph[2], ph[3], (tend - t0) * 10.0);
    }
    g_rstamps = nullptr;
    fflush(stdout);
  }
  auto want = [&](const char* n) { return !only || strstr(n, only); };
  if (want("serial")) {
    variant<false, 512, 2>(c, "serial: route 1 tile/WG + agg 512/UR2", SERIAL, NTILE, s0, s1, ev_r, ev_a, 2);
    variant<true, 512, 2>(c, "serial: route persist 512 + agg 512/UR2", SERIAL, 512, s0, s1, ev_r, ev_a, 2);
    variant<false, 1024, 2>(c, "serial: route 1 tile/WG + agg 1024/UR2", SERIAL, NTILE, s0, s1, ev_r, ev_a, 2);
  }
  if (want("streams")) {
    variant<false, 512, 2>(c, "streams(3 buf): route 1 tile/WG + agg 512", STREAMS, NTILE, s0, s1, ev_r, ev_a, 3);
    variant<true, 512, 2>(c, "streams(3 buf): route persist 512 + agg 512", STREAMS, 512, s0, s1, ev_r, ev_a, 3);
    variant<true, 512, 2>(c, "streams(2 buf): route persist 512 + agg 512", STREAMS, 512, s0, s1, ev_r, ev_a, 2);
    variant<true, 512, 2>(c, "streams(3 buf): route persist 256 + agg 512", STREAMS, 256, s0, s1, ev_r, ev_a, 3);
    variant<false, 1024, 2>(c, "streams(3 buf): route 1 tile/WG + agg 1024", STREAMS, NTILE, s0, s1, ev_r, ev_a, 3);
  }
  if (want("dual")) {
    variant<false, 512, 2>(c, "dual: agg(j-1) + route(j) 1 tile/WG", DUAL, NTILE, s0, s1, ev_r, ev_a, 2);
    variant<true, 512, 2>(c, "dual: agg(j-1) + route(j) persist 256", DUAL, 256, s0, s1, ev_r, ev_a, 2);
    variant<true, 512, 2>(c, "dual: agg(j-1) + route(j) persist 512", DUAL, 512, s0, s1, ev_r, ev_a, 2);
  }
  return 0;
}
