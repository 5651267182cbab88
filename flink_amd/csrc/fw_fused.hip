// fw_fused.hip — ingest form 3: one persistent launch per batch in which the records of a
// chunk are handed from the workgroup that read them to the workgroup that owns their keys through the
// L2 of the XCD both run on, so the routed intermediate of the two-kernel form (k_route -> k_aggregate,
// ~40 B per event of HBM / Infinity-Cache traffic) never leaves the chip.  Included by fw_engine.hip.
//
// Reference path: WindowOperator.processElement (SJ/runtime/operators/windowing/WindowOperator.java:222-333)
// -> HeapReducingState.add (RT/state/heap/HeapReducingState.java:84-122), for a batch of records between two
// watermarks (StreamInputProcessor.java:147-177).  Exact for integer reduces and the first-arrival f1;
// double sums change association (the tolerance path), as in the other forms.
//
// Geometry.  FU_GRID = 256 workgroups of 1024 threads, one per CU (LDS > 80 KiB), in FU_GROUPS = 8 groups
// g = blockIdx % 8 of FU_MEMBERS = 32 members (blockIdx / 8).  The dispatcher deals workgroups to the 8
// XCDs round-robin, so a group is normally the 32 CUs of one XCD.  Placement is only ever a speed matter:
// every workgroup reads HW_REG_XCC_ID, and a group whose members do not all report the same XCD hands off
// with the agent-scope release/acquire recipe (MI355X_MICROARCH.md § visibility) instead of the same-L2
// path (plain stores drained with vmcnt(0) before a memory-side counter add; every consumer load L1-bypassing).
//
// Ownership.  Member j of each group owns directory slots [j SO, (j+1) SO), SO = D / 32: whole directory
// buckets, and linear probing never leaves a bucket, so every key lives in its owner's range.  The owner
// keeps an LDS copy of its slots' key hashes and LDS accumulators of the batch's primary slice m0 (the
// slice of the middle record: an in-order batch has one slice).
//
// Round k (chunk c = 256 k + blockIdx, FU_CH records, loaded into registers during round k - 1):
//   produce  the operator work of k_route (timestamp, key group, windows, lateness), a wave multisplit of
//            the records of slice m0 by owner, an LDS counting sort, and the chunk stored bin-sorted as
//            (fmix64(key), value) + chunk index into this workgroup's ring slot k % FU_S; one counter add
//            tells the group.  Records of any other slice and the Long.MIN_VALUE key update the dense
//            columns directly (device atomics, as k_ingest_direct; rare for in-order streams).
//   consume  round k - 1: this owner's bin of each of the group's 32 slots, resolved against the LDS
//            directory copy, reduced with LDS atomics (first arrival = least batch index).
// Then every owner publishes its partial accumulators (write-through), and the 8 owners of one directory
// range (one per group) each fold one eighth of the range over the 8 partials into the dense columns,
// plain read-modify-write: in this launch they are the only writers of those panes.
//
// Counters are monotonic across launches (targets from the launch count and the ring slots' uses), every
// wait is bounded (a launch that cannot make progress reports FW_ERR_CAPACITY site 30 and runs to its end
// instead of hanging the device), and the host serialises fused launches device-wide, so two of them
// never hold half of the CUs each.
namespace fw {

constexpr int FU_THREADS = 1024;
constexpr int FU_WAVES = FU_THREADS / 64;
constexpr int FU_CH = 2 * FU_THREADS;       // records per chunk: two per thread
constexpr int FU_GROUPS = 8;
constexpr int FU_MEMBERS = 32;
constexpr int FU_GRID = FU_GROUPS * FU_MEMBERS;
constexpr int FU_S = 2;                     // ring slots per workgroup
constexpr int FU_HDR = 128;                 // slot header: bin starts uint16[33], round tag uint64 at byte 96
constexpr size_t FU_SLOT = FU_HDR + (size_t)FU_CH * 16 + (size_t)FU_CH * 2;
// counter block (64-bit, monotonic)
constexpr int FU_C_REG = 0;                               // [g]      workgroups registered (32 per launch)
constexpr int FU_C_PROD = FU_C_REG + FU_GROUPS;           // [g][s]   chunks stored in slot s
constexpr int FU_C_DONE = FU_C_PROD + FU_GROUPS * FU_S;   // [g][s]   owners done reading slot s
constexpr int FU_C_FOLD = FU_C_DONE + FU_GROUPS * FU_S;   // [j]      partials of range j published (8 per launch)
constexpr int FU_C_FIN = FU_C_FOLD + FU_MEMBERS;          //          workgroups finished (256 per launch)
constexpr int FU_C_N = FU_C_FIN + 1;

struct FusedBuf {
  unsigned char* ring;          // [FU_GRID][FU_S] slots of FU_SLOT bytes
  unsigned long long* ctr;      // [FU_C_N]
  int32_t* xcc;                 // [FU_GRID] HW_REG_XCC_ID of each workgroup (this launch)
  int64_t *psum, *pmn, *pmx, *pcnt;   // partial accumulators [FU_MEMBERS][FU_GROUPS][SO]
  uint32_t* pfirst;             // ... least batch index (NO_FIRST: slot untouched by that group)
  unsigned long long uses[FU_S];  // rounds that used each ring slot in earlier launches
  int64_t epoch;                // fused launches before this one
  int32_t rounds;               // chunks per workgroup
  int32_t so_bits;              // log2(SO)
  int32_t owner_shift;          // log2(D) - 5: (fmix64(key) & dir_mask) >> owner_shift = owning member
  int32_t force_safe;           // diagnostics (FW_FUSED_SAFE=1): the release/acquire hand-off for every group
  long long* stamps;            // diagnostics (FW_DEBUG_AGG & 16): per-workgroup realtime stamps, 64 per workgroup
};
// stamp i of this workgroup: 0 start, 1 placement known, 2 + 4k + {0 produced, 1 published, 2 round k - 1 arrived,
// 3 consumed}, 60 partials published, 61 fold range ready, 62 end; 63 = xcc | one_l2 << 8
#define FU_STAMP(i) do { if (f.stamps && tid == 0 && (i) < 63) f.stamps[(int64_t)w * 64 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// LDS bytes of k_fused: staging of one chunk, bin counts, the owner's directory copy and accumulators
__host__ __device__ constexpr size_t fused_lds_bytes(int so_bits, int nacc) {
  return (size_t)FU_CH * 18 + 4 * (size_t)(FU_WAVES * 32 + 48 + 16) + ((size_t)8 << so_bits) +
         (((size_t)1 << so_bits) + 64) * (8 * (size_t)nacc + 4) + 64;
}

__device__ __forceinline__ int fu_xcc_id() { return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15); }

// one lane: wait until counter ci reaches target, bounded.  Returns false (and reports FW_ERR_CAPACITY
// site 30 once) when it gave up; a workgroup that gave up skips its later waits (broken)
__device__ __noinline__ bool fu_wait_at(int32_t* err, unsigned long long* stats, unsigned long long* c,
                                        unsigned long long target) {
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (spins > (1u << 21)) {
      set_error(err, FW_ERR_CAPACITY);
      atomicCAS(&stats[7], 0ull, 30ull);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
#define fu_wait(s, ctr, ci, target, broken) \
  ((broken) ? false : ((broken) = !fu_wait_at((s).err, (s).stats, (ctr) + (ci), (target)), !(broken)))

typedef long long fu_v2 __attribute__((ext_vector_type(2)));
typedef int fu_i2 __attribute__((ext_vector_type(2)));

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(FU_THREADS) void k_fused(Spec s, BatchIn b, FusedBuf f, const int64_t* f1col) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool HAS_MIN = (AGG & FW_AGG_MIN) != 0, HAS_MAX = (AGG & FW_AGG_MAX) != 0;
  constexpr bool HAS_CNT = (AGG & FW_AGG_COUNT) != 0;
  const int w = blockIdx.x, g = w & (FU_GROUPS - 1), me = w / FU_GROUPS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int SO = 1 << f.so_bits;
  const int KA = SO + 64;
  longlong2* st_kv = (longlong2*)smem;                 // [FU_CH] the chunk's routed records, bin-sorted
  uint16_t* st_idx = (uint16_t*)(st_kv + FU_CH);       // [FU_CH] ... their index in the chunk
  int32_t* wc = (int32_t*)(st_idx + FU_CH);            // [FU_WAVES][32] records of wave v in bin b, then offsets
  int32_t* bst = wc + FU_WAVES * 32;                   // [48] bin starts, [32] = routed records
  int32_t* misc = bst + 48;                            // [16] 0: same-L2 group, 2: pane slot of m0
  uint64_t* lh = (uint64_t*)(misc + 16);               // [SO] fmix64 of the owned directory slots
  int64_t* lsum = (int64_t*)(lh + SO);                 // [KA]
  int64_t* lmin = lsum + KA;
  int64_t* lmax = lmin + (HAS_MIN ? KA : 0);
  int64_t* lcnt = lmax + (HAS_MAX ? KA : 0);
  uint32_t* lfirst = (uint32_t*)(lcnt + (HAS_CNT ? KA : 0));
  const AggLds L{lsum, lmin, lmax, lcnt, lfirst, nullptr};
  const bool cmpto = s.cmpto != 0;
  const int64_t n = b.n;
  const unsigned long long ep = (unsigned long long)f.epoch;
  const int R = f.rounds;
  bool broken = false;   // (thread 0) a bounded wait gave up
  // the batch's primary slice: the middle record's
  int64_t m0 = 0;
  {
    const int64_t tm = b.ts[n >> 1];
    if (tm != INT64_MIN) m0 = uniform64(record_windows(s, tm, b.wm).m);
  }
  FU_STAMP(0);
  // registration: this workgroup's XCD, published write-through, then counted
  const int my_xcc = fu_xcc_id();
  if (tid == 0) {
    __hip_atomic_store(f.xcc + w, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(f.ctr + FU_C_REG + g, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // chunk k of this workgroup into registers (two records per thread; whole chunks with 16-B loads)
  int64_t nk[2], nt[2], nv[2];
  int32_t nh[2] = {0, 0};
  auto load_chunk = [&](int k) {
    const int64_t i = ((int64_t)k * FU_GRID + w) * FU_CH + 2 * tid;
    if (i + 1 < n) {
      const fu_v2 a = __builtin_nontemporal_load((const fu_v2*)(b.key + i));
      const fu_v2 c = __builtin_nontemporal_load((const fu_v2*)(b.ts + i));
      const fu_v2 d = __builtin_nontemporal_load((const fu_v2*)(b.val + i));
      nk[0] = a.x; nk[1] = a.y; nt[0] = c.x; nt[1] = c.y; nv[0] = d.x; nv[1] = d.y;
      if (b.key_hash) { const fu_i2 h = *(const fu_i2*)(b.key_hash + i); nh[0] = h.x; nh[1] = h.y; }
    } else {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool in = i + e < n;
        nk[e] = in ? b.key[i + e] : 0;
        nt[e] = in ? b.ts[i + e] : 0;
        nv[e] = in ? b.val[i + e] : 0;
        if (b.key_hash) nh[e] = in ? b.key_hash[i + e] : 0;
      }
    }
  };
  if (R > 0) load_chunk(0);
  // the owned directory slots and their accumulators
  const int64_t dbase = (int64_t)me * SO;
  for (int x = tid; x < SO; x += FU_THREADS) lh[x] = fmix64((uint64_t)s.dir_keys[dbase + x]);
  for (int x = tid; x < KA; x += FU_THREADS) {
    lsum[x] = sum_identity(VT);
    if (HAS_MIN) lmin[x] = INT64_MAX;
    if (HAS_MAX) lmax[x] = INT64_MIN;
    if (HAS_CNT) lcnt[x] = 0;
    lfirst[x] = NO_FIRST;
  }
  // the group's placement: one L2 (the fast hand-off) unless some member runs on another XCD
  if (tid == 0) {
    bool one_l2 = false;
    if (fu_wait(s, f.ctr, FU_C_REG + g, (ep + 1) * FU_MEMBERS, broken)) {
      one_l2 = !f.force_safe;
      for (int j = 0; j < FU_MEMBERS; ++j)
        one_l2 &= __hip_atomic_load(f.xcc + j * FU_GROUPS + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == my_xcc;
      if (!one_l2 && me == 0) atomicAdd(&s.stats[6], 1ull);   // diagnostics: group-launches on the safe path
    }
    misc[0] = one_l2 ? 1 : 0;
  }
  __syncthreads();
  const bool one_l2 = misc[0] != 0;
  FU_STAMP(1);
  if (f.stamps && tid == 0) f.stamps[(int64_t)w * 64 + 63] = my_xcc | (one_l2 ? 256 : 0);
  const bool all_kg = s.kg_start == 0 && s.kg_end == s.mp - 1;
  const uint32_t kbm = (1u << s.kb_bits) - 1u;
  unsigned long long late_pairs = 0;

  for (int k = 0; k <= R; ++k) {   // uniform
    if (k < R) {
      // ---------------- produce chunk k ----------------
      int64_t kk[2] = {nk[0], nk[1]}, tt[2] = {nt[0], nt[1]}, vv[2] = {nv[0], nv[1]};
      int32_t hh[2] = {nh[0], nh[1]};
      const int64_t cbase = ((int64_t)k * FU_GRID + w) * FU_CH;
      if (k + 1 < R) load_chunk(k + 1);   // in flight during this round
      // the wave's reference slice (first valid lane), valid for every record whose timestamp lies in it
      RecWin w0;
      w0.m = 0; w0.n_late = 0; w0.n_fire = 0; w0.n_windows = 0; w0.quirk = false; w0.lo = 1; w0.hi = 0;
      {
        const bool c0 = cbase + 2 * tid < n && tt[0] > -(1LL << 61) && tt[0] < (1LL << 61);
        const uint64_t cm = __ballot(c0);
        if (cm && s.size < (1LL << 60)) {
          const int64_t ts0 = uniform64(__shfl(tt[0], __ffsll((long long)cm) - 1));
          w0 = record_windows(s, ts0, b.wm);
          w0.m = uniform64(w0.m); w0.lo = uniform64(w0.lo); w0.hi = uniform64(w0.hi);
          w0.n_late = __builtin_amdgcn_readfirstlane(w0.n_late);
          w0.n_fire = __builtin_amdgcn_readfirstlane(w0.n_fire);
          w0.n_windows = __builtin_amdgcn_readfirstlane(w0.n_windows);
        }
      }
      uint32_t route = 0, spill = 0;
      int64_t mm[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int64_t i = cbase + 2 * tid + e;
        bool ok = i < n;
        if (ok && tt[e] == INT64_MIN) { set_error(s.err, FW_ERR_NO_TIMESTAMP); ok = false; }
        if (ok && !all_kg) {
          const int32_t h = b.key_hash ? hh[e] : long_hash_code(kk[e]);
          const int32_t kg = record_key_group(s, h);   // AbstractKeyedStateBackend.setCurrentKey :167-170
          if (kg < s.kg_start || kg > s.kg_end) { set_error(s.err, FW_ERR_KEY_GROUP); ok = false; }
        }
        RecWin rw = w0;
        if (ok && !(tt[e] >= w0.lo && tt[e] <= w0.hi)) {
          rw = record_windows(s, tt[e], b.wm);
          if (rw.quirk) quirk_record(s, b, kk[e], i, rw.qn, rw.q_late, rw.q_fire);
        }
        if (ok) late_pairs += (unsigned long long)rw.n_late;
        const bool live = ok && rw.n_windows - rw.n_late > 0;
        if (live && rw.n_fire > 0) set_error(s.err, FW_ERR_UNSUPPORTED);   // no per-element fires: lateness is 0
        const bool rt = live && rw.m == m0 && kk[e] != EMPTY_KEY;
        route |= (rt ? 1u : 0u) << e;
        spill |= (live && !rt ? 1u : 0u) << e;
        mm[e] = rw.m;
      }
      // records of another slice, and the Long.MIN_VALUE key: the dense columns directly
      if (__any(spill != 0)) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int64_t i = cbase + 2 * tid + e;
          bool fresh = false;
          int64_t idx = 0;
          if ((spill >> e) & 1u) {
            const int32_t p = slice_slot(s, mm[e]);
            const int64_t kid = p < 0 ? -1 : dir_lookup(s, kk[e]);   // (Long.MIN_VALUE: kid D)
            if (p < 0 || kid < 0) {
              cap_error(s, 31);
            } else {
              idx = (int64_t)p * s.stride + kid;
              fresh = pane_update<VT, AGG, FIRST>(s, idx, vv[e], b.ord_base + i);
            }
          }
          if (FIRST) {   // the panes this batch created: their f1 is set after every workgroup is done
            const unsigned long long pos = wave_append(b.new_count, fresh);
            if (fresh) {
              if ((int64_t)pos < b.new_capacity)
                __hip_atomic_store((unsigned long long*)b.new_list + pos, (unsigned long long)idx, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
              else cap_error(s, 5);
            }
          }
        }
      }
      // owner of each routed record, and its rank among the wave's records of that owner
      uint64_t hk[2];
      int32_t bin[2], rank[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        hk[e] = fmix64((uint64_t)kk[e]);
        bin[e] = (int32_t)((hk[e] & s.dir_mask) >> f.owner_shift);
      }
      if (tid < FU_WAVES * 32) wc[tid] = 0;
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool act = (route >> e) & 1u;
        uint64_t peers = __ballot(act);
#pragma unroll
        for (int bb = 0; bb < 5; ++bb) {
          const bool bit = (bin[e] >> bb) & 1;
          const uint64_t m = __ballot(bit);
          peers &= bit ? m : ~m;
        }
        const int32_t below = __popcll(peers & lanemask_lt());
        int32_t base = 0;
        if (e == 1 && act) base = wc[wave * 32 + bin[e]];
        rank[e] = base + below;
        if (act && below == 0) wc[wave * 32 + bin[e]] = base + __popcll(peers);
      }
      __syncthreads();
      // bin starts, and each wave's offset inside each bin (wave 0, one lane per bin)
      if (wave == 0) {
        int32_t c[FU_WAVES];
        int32_t tot = 0;
#pragma unroll
        for (int v = 0; v < FU_WAVES; ++v) { c[v] = lane < 32 ? wc[v * 32 + lane] : 0; tot += c[v]; }
        int32_t incl = tot;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const int32_t y = __shfl_up(incl, o);
          if (lane >= o) incl += y;
        }
        int32_t run = incl - tot;
        if (lane < 32) {
          bst[lane] = run;
#pragma unroll
          for (int v = 0; v < FU_WAVES; ++v) { wc[v * 32 + lane] = run; run += c[v]; }
        }
        if (lane == 31) bst[32] = incl;
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if ((route >> e) & 1u) {
          const int32_t pos = wc[wave * 32 + bin[e]] + rank[e];
          st_kv[pos] = make_longlong2((long long)hk[e], (long long)vv[e]);
          st_idx[pos] = (uint16_t)(2 * tid + e);
        }
      }
      FU_STAMP(2 + 4 * k);
      // the ring slot is free once every owner of the group read its previous use
      const int sl = k % FU_S;
      if (tid == 0) (void)fu_wait(s, f.ctr, FU_C_DONE + g * FU_S + sl, (f.uses[sl] + (unsigned long long)(k / FU_S)) * FU_MEMBERS, broken);
      __syncthreads();
      unsigned char* slot = f.ring + ((size_t)w * FU_S + sl) * FU_SLOT;
      const int32_t total = bst[32];
      longlong2* gkv = (longlong2*)(slot + FU_HDR);
      uint32_t* gidx = (uint32_t*)(slot + FU_HDR + (size_t)FU_CH * 16);
      for (int x = tid; x < total; x += FU_THREADS) gkv[x] = st_kv[x];
      for (int x = tid; 2 * x < total; x += FU_THREADS) gidx[x] = ((const uint32_t*)st_idx)[x];
      if (tid <= 32) ((uint16_t*)slot)[tid] = (uint16_t)bst[tid];
      if (tid == 64) *(unsigned long long*)(slot + 96) = (ep << 16) | (unsigned long long)(k + 1);
      // publish: every storing wave drained, then one counter add (same L2), or release + add (safe path)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (!one_l2) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(f.ctr + FU_C_PROD + g * FU_S + sl, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      FU_STAMP(3 + 4 * k);
    }
    if (k >= 1) {
      // ---------------- consume round kc = k - 1 ----------------
      const int kc = k - 1;
      const int sl = kc % FU_S;
      if (tid == 0) {
        if (fu_wait(s, f.ctr, FU_C_PROD + g * FU_S + sl, (f.uses[sl] + (unsigned long long)(kc / FU_S) + 1) * FU_MEMBERS,
                    broken) && !one_l2)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      FU_STAMP(4 + 4 * kc);
      // 32 threads per producer: its segment for this owner, 16-B L1-bypassing loads from the XCD's L2
      const int p = tid >> 5, u = tid & 31;
      const int wp = p * FU_GROUPS + g;
      const unsigned char* slot = f.ring + ((size_t)wp * FU_S + sl) * FU_SLOT;
      int32_t a = 0, z = 0;
      if (u == 0) {
        a = __builtin_nontemporal_load((const uint16_t*)slot + me);
        z = __builtin_nontemporal_load((const uint16_t*)slot + me + 1);
        const unsigned long long tag = __builtin_nontemporal_load((const unsigned long long*)(slot + 96));
        if (tag != ((ep << 16) | (unsigned long long)(kc + 1))) { cap_error(s, 33); z = a; }   // not this round's chunk
      }
      a = __shfl(a, lane & 32);
      z = __shfl(z, lane & 32);
      z = min(z, FU_CH);   // (bounds a torn header could break; the tag check reports it)
      a = min(a, z);
      const longlong2* gkv = (const longlong2*)(slot + FU_HDR);
      const uint16_t* gidx = (const uint16_t*)(slot + FU_HDR + (size_t)FU_CH * 16);
      const uint32_t cb = (uint32_t)(((int64_t)kc * FU_GRID + wp) * FU_CH);   // batch index of the chunk's record 0
      auto add = [&](const fu_v2 r, uint32_t ix) {
        const uint64_t h = (uint64_t)r.x;
        const uint32_t loc = (uint32_t)((h & s.dir_mask) - (uint64_t)dbase);   // slot relative to the owned range
        if (loc >= (uint32_t)SO) { cap_error(s, 35); return; }                 // (another owner's key: a torn slot)
        const uint32_t bb = loc & ~kbm, h0 = (uint32_t)h & kbm;
        uint32_t kl = 0;
        bool found = false;
#pragma unroll
        for (int j = 7; j >= 0; --j) {   // the nearest match wins
          const uint32_t x = bb + ((h0 + (uint32_t)j) & kbm);
          const bool m = lh[x] == h;
          kl = m ? x : kl;
          found |= m;
        }
        if (!found) {
          const int32_t x = agg_probe_insert(lh + bb, s.dir_keys + dbase + bb, kbm, h, s.stats + ST_DIR_KEYS);
          if (x < 0) { cap_error(s, 34); return; }
          kl = bb + (uint32_t)x;
        }
        acc_add<VT, AGG>(L, cmpto, false, 0, kl, (int64_t)r.y, cb + ix);
      };
      for (int x = a + u; x < z; x += 64) {
        const bool two = x + 32 < z;
        const fu_v2 r0 = __builtin_nontemporal_load((const fu_v2*)(gkv + x));
        const uint32_t i0 = __builtin_nontemporal_load(gidx + x);
        fu_v2 r1 = r0;
        uint32_t i1 = i0;
        if (two) { r1 = __builtin_nontemporal_load((const fu_v2*)(gkv + x + 32)); i1 = __builtin_nontemporal_load(gidx + x + 32); }
        add(r0, i0);
        if (two) add(r1, i1);
      }
      __syncthreads();
      FU_STAMP(5 + 4 * kc);
      if (tid == 0) __hip_atomic_fetch_add(f.ctr + FU_C_DONE + g * FU_S + sl, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (__any(late_pairs != 0)) {
    for (int off = 32; off > 0; off >>= 1) late_pairs += __shfl_xor(late_pairs, off);
    if (lane == 0) atomicAdd(&s.stats[ST_LATE], late_pairs);
  }

  // ---------------- publish the partials of the owned slots (write-through 4- and 8-B stores) ----------------
  const size_t pb = ((size_t)me * FU_GROUPS + g) << f.so_bits;
  for (int x = tid; x < SO; x += FU_THREADS) {
    const uint32_t lf = lfirst[x];
    __hip_atomic_store(f.pfirst + pb + x, lf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lf != NO_FIRST) {
      if (AGG & FW_AGG_SUM)
        __hip_atomic_store((unsigned long long*)f.psum + pb + x, (unsigned long long)lsum[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (HAS_MIN)
        __hip_atomic_store((unsigned long long*)f.pmn + pb + x, (unsigned long long)lmin[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (HAS_MAX)
        __hip_atomic_store((unsigned long long*)f.pmx + pb + x, (unsigned long long)lmax[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (HAS_CNT)
        __hip_atomic_store((unsigned long long*)f.pcnt + pb + x, (unsigned long long)lcnt[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  FU_STAMP(60);
  if (tid == 0) {
    __hip_atomic_fetch_add(f.ctr + FU_C_FOLD + me, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    (void)fu_wait(s, f.ctr, FU_C_FOLD + me, (ep + 1) * FU_GROUPS, broken);
  }
  __syncthreads();
  FU_STAMP(61);

  // ---------------- fold: slots [g SH, (g+1) SH) of range me over the 8 groups' partials ----------------
  const int SH = SO / FU_GROUPS;
  for (int x0 = 0; x0 < SH; x0 += FU_THREADS) {   // uniform
    const int x = g * SH + x0 + tid;
    bool touched = false;
    int64_t tsum = sum_identity(VT), tmin = INT64_MAX, tmax = INT64_MIN, tcnt = 0;
    uint32_t tfirst = NO_FIRST;
    if (x0 + tid < SH) {
#pragma unroll
      for (int gg = 0; gg < FU_GROUPS; ++gg) {   // group order: a fixed association for double sums
        const size_t pi = (((size_t)me * FU_GROUPS + gg) << f.so_bits) + (size_t)x;
        const uint32_t pf = __hip_atomic_load(f.pfirst + pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pf == NO_FIRST) continue;
        touched = true;
        tfirst = pf < tfirst ? pf : tfirst;
        if (AGG & FW_AGG_SUM) {
          const int64_t v = (int64_t)__hip_atomic_load((unsigned long long*)f.psum + pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (VT == FW_VALUE_I64) tsum = jadd(tsum, v);
          else tsum = __double_as_longlong(__longlong_as_double(tsum) + __longlong_as_double(v));
        }
        if (HAS_MIN) {
          const int64_t v = (int64_t)__hip_atomic_load((unsigned long long*)f.pmn + pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tmin = v < tmin ? v : tmin;
        }
        if (HAS_MAX) {
          const int64_t v = (int64_t)__hip_atomic_load((unsigned long long*)f.pmx + pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tmax = v > tmax ? v : tmax;
        }
        if (HAS_CNT) {
          const int64_t v = (int64_t)__hip_atomic_load((unsigned long long*)f.pcnt + pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tcnt = jadd(tcnt, v);
        }
      }
    }
    // the primary slice's pane slot: claimed (idempotently) once some slot of this share was touched
    // (a block-wide OR through LDS: all of this kernel's LDS stays dynamic)
    if (tid == 0) misc[4] = 0;
    __syncthreads();
    if (__any(touched) && lane == 0) misc[4] = 1;
    __syncthreads();
    if (misc[4]) {   // uniform
      if (tid == 0) misc[2] = slice_slot(s, m0);
      __syncthreads();
      const int32_t p0 = misc[2];
      if (p0 < 0) {
        if (tid == 0) cap_error(s, 32);
      } else if (touched) {
        const int64_t idx = (int64_t)p0 * s.stride + dbase + x;
        if (AGG & FW_AGG_SUM) {
          if (VT == FW_VALUE_I64) s.c.sum[idx] = jadd(s.c.sum[idx], tsum);
          else s.c.sum[idx] = __double_as_longlong(__longlong_as_double(s.c.sum[idx]) + __longlong_as_double(tsum));
        }
        if (HAS_MIN) { if (tmin < s.c.mn[idx]) s.c.mn[idx] = tmin; }
        if (HAS_MAX) { if (tmax > s.c.mx[idx]) s.c.mx[idx] = tmax; }
        if (HAS_CNT) s.c.cnt[idx] = jadd(s.c.cnt[idx], tcnt);
        if (FIRST) {
          // a pane present before this batch keeps its (earlier) first arrival
          if (s.c.first[idx] == INT64_MAX && (int64_t)tfirst < n) {
            s.c.first[idx] = b.ord_base + (int64_t)tfirst;
            s.c.f1v[idx] = f1col[tfirst];
          }
        } else {
          s.c.present[idx] = 1;
        }
      }
      __syncthreads();   // misc[2] is rewritten by the next share
    }
  }

  // ---------------- the last workgroup: f1 of the panes the direct records created ----------------
  if (FIRST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned long long done = __hip_atomic_fetch_add(f.ctr + FU_C_FIN, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      misc[3] = done + 1 == (ep + 1) * FU_GRID ? 1 : 0;
    }
    __syncthreads();
    if (misc[3]) {   // uniform
      const int64_t nl = min((int64_t)__hip_atomic_load(b.new_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), b.new_capacity);
      for (int64_t j = tid; j < nl; j += FU_THREADS) {
        const int64_t idx = (int64_t)__hip_atomic_load((unsigned long long*)b.new_list + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t o = (int64_t)__hip_atomic_fetch_add((unsigned long long*)&s.c.first[idx], 0ull, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) - b.ord_base;
        if (o >= 0 && o < n) s.c.f1v[idx] = f1col[o];
      }
      __syncthreads();
      if (tid == 0) __hip_atomic_store(b.new_count, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  FU_STAMP(62);
}

}  // namespace fw
