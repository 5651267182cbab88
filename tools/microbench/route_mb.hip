// Prototype of the partitioned ingest (pass 1 = tile counting sort by directory bucket, pass 2 =
// per-bucket LDS aggregation) on C1-shaped batches, with variants of tile size and block shape,
// checked against direct atomics.  Build: hipcc --offload-arch=gfx950 -O3 route_mb.hip -o route_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef long long i64;
typedef unsigned long long u64;
constexpr i64 EMPTY = INT64_MIN;
constexpr int NB = 1 << 22;
constexpr int RING = 24;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33; return k;
}
__device__ __forceinline__ int32_t murmur(int32_t in) {
  uint32_t c = (uint32_t)in;
  c *= 0xcc9e2d51u; c = (c << 15) | (c >> 17); c *= 0x1b873593u; c = (c << 13) | (c >> 19);
  c = c * 5u + 0xe6546b64u; c ^= 4u; c ^= c >> 16; c *= 0x85ebca6bu; c ^= c >> 13; c *= 0xc2b2ae35u; c ^= c >> 16;
  int32_t code = (int32_t)c;
  return code >= 0 ? code : (code != INT32_MIN ? -code : 0);
}

struct Spec {
  i64 size, offset, wm;
  double inv_size;
  int mp, kg_lo, kg_hi;
  uint64_t dmask;
  int kb, nb;
  i64* dir;
  int* err;
  u64* late;
  long long* stamps;
};

__global__ void k_gen(i64* key, i64* ts, i64* val, size_t n, size_t base) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    key[i] = (i64)(mix64((base + i) ^ 1) & 0xFFFF);
    ts[i] = 1700000000000ll + (i64)(((base + i) * 1000) >> 24);
    val[i] = (i64)mix64((base + i) ^ 2);
  }
}
__device__ i64 dir_insert(const Spec& s, i64 key) {
  uint64_t home = fmix64((uint64_t)key) & s.dmask;
  uint64_t kbm = (1ull << s.kb) - 1, base = home & ~kbm, off = home & kbm;
  for (uint64_t p = 0; p <= kbm; ++p) {
    uint64_t h = base + off;
    i64 cur = s.dir[h];
    if (cur == key) return (i64)h;
    if (cur == EMPTY) {
      u64 prev = atomicCAS((u64*)&s.dir[h], (u64)EMPTY, (u64)key);
      if ((i64)prev == EMPTY || (i64)prev == key) return (i64)h;
    }
    off = (off + 1) & kbm;
  }
  return -1;
}
__global__ void k_fill(i64* p, i64 v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void k_ref(Spec s, const i64* key, const i64* val, int n, u64* ref) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    i64 kid = dir_insert(s, key[i]);
    atomicAdd(&ref[kid], (u64)val[i]);
  }
}

__device__ __forceinline__ i64 slice_of(const Spec& s, i64 ts) {
  i64 x = ts - s.offset;
  i64 q = (i64)((double)x * s.inv_size);
  i64 r = x - q * s.size;
  if (r < 0) { --q; } else if (r >= s.size) { ++q; }
  return q;
}

// ---------------------------------------------------------------------------------------------
// pass 1: tile counting sort by bin = q * nb + bucket.  Output per tile: key, val, idx (tile-major,
// bin-sorted) and seg[tile][bin] = start of the bin's segment (uint16; the tile end closes the last).
// ---------------------------------------------------------------------------------------------
struct P1Out { i64* key; i64* val; uint16_t* idx; uint16_t* seg; int ntiles; };

template <int T, int NT>
__global__ __launch_bounds__(NT) void k_pass1(Spec s, const i64* __restrict__ key, const i64* __restrict__ ts,
                                              const i64* __restrict__ val, int n, i64 m0, P1Out o) {
  constexpr int R = T / NT;           // records per thread
  constexpr int V = R / 2;            // 16-B vectors per column per thread
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  i64* st_key = (i64*)smem;
  i64* st_val = st_key + T;
  uint16_t* st_idx = (uint16_t*)(st_val + T);
  int* cnt = (int*)(st_idx + T);      // [nbq + 1]
  int* wtot = cnt + 2 * s.nb + 1;     // [NT/64]
  const int nbq = 2 * s.nb;
  const int tile = blockIdx.x;
  const i64 base = (i64)tile * T;
  for (int x = threadIdx.x; x <= nbq; x += NT) cnt[x] = 0;
  i64 kk[R], tt[R], vv[R];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const i64 r = base + 2 * (j * NT + threadIdx.x);
    const i64 rr = r + 1 < n ? r : (n >= 2 ? n - 2 : 0);
    longlong2 a = *(const longlong2*)(key + rr);
    longlong2 b = *(const longlong2*)(ts + rr);
    longlong2 c = *(const longlong2*)(val + rr);
    kk[2 * j] = a.x; kk[2 * j + 1] = a.y; tt[2 * j] = b.x; tt[2 * j + 1] = b.y; vv[2 * j] = c.x; vv[2 * j + 1] = c.y;
  }
  __syncthreads();
  int bin[R], rank[R];
  u64 late = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const i64 r = base + 2 * ((k >> 1) * NT + threadIdx.x) + (k & 1);
    bool ok = r < n;
    const i64 key_ = kk[k];
    const int32_t h = (int32_t)(uint32_t)((uint64_t)key_ ^ ((uint64_t)key_ >> 32));
    const int kg = murmur(h) & (s.mp - 1);
    if (ok && (kg < s.kg_lo || kg > s.kg_hi)) { atomicCAS(s.err, 0, 4); ok = false; }
    const i64 m = slice_of(s, tt[k]);
    const i64 maxts = s.offset + (m + 1) * s.size - 1;
    if (ok && maxts <= s.wm) { ++late; ok = false; }
    bin[k] = -1; rank[k] = 0;
    if (ok) {
      const int q = m == m0 ? 0 : 1;
      const int bucket = (int)((fmix64((uint64_t)key_) & s.dmask) >> s.kb);
      bin[k] = q * s.nb + bucket;
      rank[k] = atomicAdd(&cnt[bin[k]], 1);
    }
  }
  if (late) atomicAdd(s.late, late);
  __syncthreads();
  // exclusive scan of cnt[0..nbq)
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    const int nsc = nbq + 1;                // bins + the total
    const int per = (nsc + NT - 1) / NT;    // bins per thread (contiguous)
    int loc[8];
    int sum = 0;
    for (int i = 0; i < per; ++i) { int b = threadIdx.x * per + i; loc[i] = b < nsc ? cnt[b] : 0; sum += loc[i]; }
    int x = sum;
    for (int o = 1; o < 64; o <<= 1) { int y = __shfl_up(x, o); if (lane >= o) x += y; }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += wtot[w];
    int run = wbase + x - sum;
    __syncthreads();
    for (int i = 0; i < per; ++i) { int b = threadIdx.x * per + i; if (b < nsc) { cnt[b] = run; run += loc[i]; } }
    (void)NW;
  }
  __syncthreads();
  for (int x = threadIdx.x; x <= nbq; x += NT) o.seg[(i64)tile * (nbq + 1) + x] = (uint16_t)cnt[x];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (bin[k] >= 0) {
      const int p = cnt[bin[k]] + rank[k];
      st_key[p] = kk[k];
      st_val[p] = vv[k];
      st_idx[p] = (uint16_t)(2 * ((k >> 1) * NT + threadIdx.x) + (k & 1));
    }
  }
  __syncthreads();
  // write out (16-B stores); unrouted tail entries are left as garbage beyond the last segment end
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int p = 2 * (j * NT + threadIdx.x);
    if (base + p < n) {
      *(longlong2*)(o.key + base + p) = *(const longlong2*)(st_key + p);
      *(longlong2*)(o.val + base + p) = *(const longlong2*)(st_val + p);
      *(uint32_t*)(o.idx + base + p) = *(const uint32_t*)(st_idx + p);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// pass 2: one block per bin: gathers the bin's segment from every tile (flattened, binary search on
// the per-tile prefix), resolves the key in the bucket's LDS directory slice, aggregates with LDS
// atomics, folds into sum[kid] (exclusive owner: plain RMW).
// ---------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void k_pass2(Spec s, P1Out o, int n, u64* sum, uint32_t* first, int dbg) {
  // one block per bucket; for each used batch slice q, every tile's segment of bin (q, bucket) is read
  // by a 16-lane group (2 records per lane per round), 4 segments per wave-instruction
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nbq = 2 * s.nb;
  const int bucket = blockIdx.x;
  const int KB = 1 << s.kb;
  const uint32_t kbm = KB - 1;
  i64* ldir = (i64*)smem;
  u64* lsum = (u64*)(ldir + KB);
  uint32_t* lfirst = (uint32_t*)(lsum + KB);
  int* sst = (int*)(lfirst + KB);           // [ntiles] segment start
  int* sln = sst + o.ntiles;                // [ntiles] segment length
  const i64 dbase = (i64)bucket * KB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane >> 4, sub = lane & 15;
  const i64 T = n / o.ntiles;
  long long* tst = s.stamps ? s.stamps + (size_t)blockIdx.x * 8 : nullptr;
  if (tst && threadIdx.x == 0) tst[0] = __builtin_amdgcn_s_memrealtime();
  for (int x = threadIdx.x; x < KB; x += NT) ldir[x] = s.dir[dbase + x];
  for (int qq = 0; qq < (dbg & 8 ? 1 : 2); ++qq) {
    const int bin = qq * s.nb + bucket;
    for (int x = threadIdx.x; x < KB; x += NT) { lsum[x] = 0; lfirst[x] = 0xFFFFFFFFu; }
    for (int t = threadIdx.x; t < o.ntiles; t += NT) {
      const int a0 = o.seg[(i64)t * (nbq + 1) + bin], a1 = o.seg[(i64)t * (nbq + 1) + bin + 1];
      sst[t] = a0;
      sln[t] = a1 - a0;
    }
    __syncthreads();
    if (tst && threadIdx.x == 0) tst[1 + 3 * qq] = __builtin_amdgcn_s_memrealtime();
    constexpr int UR = 4;                        // rounds (4 segments each) per wave-step
    auto process = [&](bool act, i64 key, i64 v, uint32_t oi) {
      uint32_t h = (uint32_t)(fmix64((uint64_t)key) & s.dmask) & kbm;
      i64 d = ldir[h];
      if (act && d != key) {
        for (;;) {
          h = (h + 1) & kbm;
          i64 cur = ldir[h];
          if (cur == key) break;
          if (cur == EMPTY) { atomicCAS(s.err, 0, 9); act = false; break; }
        }
      }
      if (act && !(dbg & 1)) {
        atomicAdd(&lsum[h], (u64)v);
        atomicMin(&lfirst[h], oi);
      }
    };
    for (int tb = wave * 4 * UR; tb < o.ntiles; tb += (NT / 64) * 4 * UR) {
      i64 ka[UR], kb2[UR], va[UR], vb[UR];
      uint32_t ia[UR], ib[UR];
      bool aa[UR], ab[UR];
#pragma unroll
      for (int r = 0; r < UR; ++r) {
        const int t = min(tb + r * 4 + grp, o.ntiles - 1);
        const int st_ = sst[t], ln = (tb + r * 4 + grp < o.ntiles) ? sln[t] : 0;
        aa[r] = sub < ln;
        ab[r] = sub + 16 < ln;
        const i64 pa = (i64)t * T + (aa[r] ? st_ + sub : 0);
        const i64 pb = (i64)t * T + (ab[r] ? st_ + sub + 16 : 0);
        ka[r] = o.key[pa]; kb2[r] = o.key[pb];
        va[r] = o.val[pa]; vb[r] = o.val[pb];
        ia[r] = ((uint32_t)t << 16) | o.idx[pa];
        ib[r] = ((uint32_t)t << 16) | o.idx[pb];
      }
#pragma unroll
      for (int r = 0; r < UR; ++r) { process(aa[r], ka[r], va[r], ia[r]); process(ab[r], kb2[r], vb[r], ib[r]); }
      // segments longer than 32 records
#pragma unroll
      for (int r = 0; r < UR; ++r) {
        const int tt = tb + r * 4 + grp;
        const int ln = tt < o.ntiles ? sln[tt] : 0;
        if (__any(ln > 32)) {
          const int t = min(tt, o.ntiles - 1);
          for (int j0 = 32; __any(j0 < ln); j0 += 16) {
            const bool act = j0 + sub < ln;
            const i64 p = (i64)t * T + (act ? sst[t] + j0 + sub : 0);
            process(act, o.key[p], o.val[p], ((uint32_t)t << 16) | o.idx[p]);
          }
        }
      }
    }
    __syncthreads();
    if (tst && threadIdx.x == 0) tst[2 + 3 * qq] = __builtin_amdgcn_s_memrealtime();
    for (int x = threadIdx.x; x < KB; x += NT) {
      if (lfirst[x] == 0xFFFFFFFFu) continue;
      sum[dbase + x] += lsum[x];
      if (first[dbase + x] == 0xFFFFFFFFu) first[dbase + x] = lfirst[x];
    }
    if (tst && threadIdx.x == 0) tst[3 + 3 * qq] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
  }
  if (tst && threadIdx.x == 0) tst[7] = __builtin_amdgcn_s_memrealtime();
}

__global__ void k_cmp(const u64* a, const u64* b, size_t n, int* bad) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (a[i] != b[i]) atomicAdd(bad, 1);
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

template <int T, int NT, int NT2>
void run(const char* name, int dbg, Spec s, char* ring, size_t colb, P1Out o, u64* sum, uint32_t* first, u64* ref, int* bad) {
  const int ntiles = NB / T;
  o.ntiles = ntiles;
  const int nbq = 2 * s.nb;
  size_t lds1 = (size_t)T * 18 + 4 * (nbq + 1) + 4 * 16;
  size_t lds2 = (size_t)(1 << s.kb) * 20 + 8 * ntiles + 64;
  if (getenv("PAD")) lds2 = std::max(lds2, (size_t)atoi(getenv("PAD")) * 1024);
  CK(hipFuncSetAttribute((const void*)k_pass1<T, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
  CK(hipFuncSetAttribute((const void*)k_pass2<NT2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
  auto col = [&](int r, int c) { return (const i64*)(ring + ((size_t)(r % RING) * 3 + c) * colb); };
  const i64 m0 = 1700000000000ll / 1000;
  // correctness on batch 0 (all in slice m0)
  CK(hipMemset(sum, 0, 8ull << 18)); CK(hipMemset(first, 0xFF, 4ull << 18)); CK(hipMemset(bad, 0, 4));
  k_pass1<T, NT><<<ntiles, NT, lds1>>>(s, col(0, 0), col(0, 1), col(0, 2), NB, m0, o);
  k_pass2<NT2><<<s.nb, NT2, lds2>>>(s, o, NB, sum, first, dbg);
  k_cmp<<<1024, 256>>>(sum, ref, 1ull << 18, bad);
  int hbad = 0; CK(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
  const int IT = 48;
  for (int r = 1; r < 5; ++r) { k_pass1<T, NT><<<ntiles, NT, lds1>>>(s, col(r, 0), col(r, 1), col(r, 2), NB, m0, o); k_pass2<NT2><<<s.nb, NT2, lds2>>>(s, o, NB, sum, first, dbg); }
  Timer t;
  t.start(); for (int r = 0; r < IT; ++r) k_pass1<T, NT><<<ntiles, NT, lds1>>>(s, col(r, 0), col(r, 1), col(r, 2), NB, m0, o);
  float ms1 = t.stop() / IT;
  t.start(); for (int r = 0; r < IT; ++r) k_pass2<NT2><<<s.nb, NT2, lds2>>>(s, o, NB, sum, first, dbg);
  float ms2 = t.stop() / IT;
  t.start(); for (int r = 0; r < IT; ++r) { k_pass1<T, NT><<<ntiles, NT, lds1>>>(s, col(r, 0), col(r, 1), col(r, 2), NB, m0, o); k_pass2<NT2><<<s.nb, NT2, lds2>>>(s, o, NB, sum, first, dbg); }
  float ms = t.stop() / IT;
  int herr = 0; CK(hipMemcpy(&herr, s.err, 4, hipMemcpyDeviceToHost));
  {
    Spec s2 = s;
    CK(hipMalloc(&s2.stamps, 8 * 8 * s.nb));
    k_pass1<T, NT><<<ntiles, NT, lds1>>>(s, col(3, 0), col(3, 1), col(3, 2), NB, m0, o);
    k_pass2<NT2><<<s.nb, NT2, lds2>>>(s2, o, NB, sum, first, dbg);
    std::vector<long long> h(8 * s.nb);
    CK(hipMemcpy(h.data(), s2.stamps, 8 * 8 * s.nb, hipMemcpyDeviceToHost));
    long long t0 = h[0], tend = h[7];
    for (int b = 0; b < s.nb; ++b) { t0 = std::min(t0, h[8 * b]); tend = std::max(tend, h[8 * b + 7]); }
    double ph[7] = {0};
    for (int b = 0; b < s.nb; ++b) for (int k = 0; k < 7; ++k) ph[k] += (h[8 * b + k + 1] - h[8 * b + k]) * 10.0 / s.nb;
    double st0 = 0; for (int b = 0; b < s.nb; ++b) st0 += (h[8 * b] - t0) * 10.0 / s.nb;
    printf("   p2 phases (ns avg over blocks): start-skew %.0f prefix0 %.0f main0 %.0f fold0 %.0f prefix1 %.0f main1 %.0f fold1 %.0f | span %.0f ns\n",
           st0, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], (tend - t0) * 10.0);
    CK(hipFree(s2.stamps));
  }
  printf("%-28s p1 %7.2f us  p2 %7.2f us  both %7.2f us  %6.1f Gev/s (%.0f%% of 8TB/s)  check %s err %d\n", name, ms1 * 1e3,
         ms2 * 1e3, ms * 1e3, NB / ms / 1e6, 100.0 * 24.0 * NB / ms / 1e6 / 8000.0, hbad ? "BAD" : "ok", herr);
}

int main(int argc, char** argv) {
  const bool quick = argc > 1;
  const size_t colb = (size_t)NB * 8;
  char* ring; CK(hipMalloc(&ring, (size_t)RING * 3 * colb));
  for (int r = 0; r < RING; ++r) {
    char* b = ring + (size_t)r * 3 * colb;
    k_gen<<<2048, 256>>>((i64*)b, (i64*)(b + colb), (i64*)(b + 2 * colb), NB, (size_t)r * NB);
  }
  Spec s{};
  s.size = 1000; s.offset = 0; s.wm = INT64_MIN; s.inv_size = 1.0 / 1000; s.mp = 128; s.kg_lo = 0; s.kg_hi = 127;
  s.dmask = (1ull << 18) - 1; s.kb = 10; s.nb = 256;
  CK(hipMalloc(&s.dir, 8ull << 18)); k_fill<<<1024, 256>>>(s.dir, EMPTY, 1ull << 18);
  CK(hipMalloc(&s.err, 4)); CK(hipMemset(s.err, 0, 4));
  CK(hipMalloc(&s.late, 8)); CK(hipMemset(s.late, 0, 8));
  u64* ref; CK(hipMalloc(&ref, 8ull << 18)); CK(hipMemset(ref, 0, 8ull << 18));
  k_ref<<<2048, 256>>>(s, (const i64*)ring, (const i64*)(ring + 2 * colb), NB, ref);
  CK(hipDeviceSynchronize());
  P1Out o{};
  CK(hipMalloc(&o.key, 8ull * NB)); CK(hipMalloc(&o.val, 8ull * NB)); CK(hipMalloc(&o.idx, 2ull * NB));
  CK(hipMalloc(&o.seg, 2ull * 513 * (NB / 1024)));
  u64* sum; CK(hipMalloc(&sum, 8ull << 18));
  uint32_t* first; CK(hipMalloc(&first, 4ull << 18));
  int* bad; CK(hipMalloc(&bad, 4));
  if (quick) { run<4096, 512, 1024>("T4096 NT512", 0, s, ring, colb, o, sum, first, ref, bad); return 0; }
  for (int d : {0, 8}) {
    printf("dbg %d\n", d);
    run<4096, 512, 1024>("T4096 NT512", d, s, ring, colb, o, sum, first, ref, bad);
    run<8192, 1024, 1024>("T8192 NT1024", d, s, ring, colb, o, sum, first, ref, bad);
    run<2048, 256, 1024>("T2048 NT256", d, s, ring, colb, o, sum, first, ref, bad);
  }
  return 0;
}
