// fw_fused.hip — ingest form 3: one persistent launch per batch.  The records a workgroup reads
// are handed to the workgroup that owns their keys through the L2 of the XCD both run on, and each owner reduces
// its share in LDS, so no routed intermediate has to survive a kernel boundary.  Included by fw_engine.hip.
//
// Reference path: WindowOperator.processElement (SJ/runtime/operators/windowing/WindowOperator.java:222-333)
// -> HeapReducingState.add (RT/state/heap/HeapReducingState.java:84-122), for a batch of records between two
// watermarks (StreamInputProcessor.java:147-177).  Exact for integer reduces and the first-arrival f1; double
// sums change association (the tolerance path), as in the other forms.
//
// Geometry.  FU_GRID = 256 workgroups of 1024 threads, one per CU, in FU_GROUPS = 8 groups g = blockIdx % 8 of
// FU_MEMBERS = 32 members (blockIdx / 8).  The dispatcher deals workgroups to the XCDs round-robin, so a group is
// normally the 32 CUs of one XCD.  Placement is only ever a speed matter: every workgroup registers its
// HW_REG_XCC_ID, and a group whose members do not all report one XCD hands off with the agent-scope
// release / acquire recipe (MI355X_MICROARCH.md, inter-workgroup visibility) instead of the same-L2 path.
//
// Ownership.  Member j of each group owns directory slots [j SO, (j + 1) SO), SO = D / 32: whole directory
// buckets, and probing never leaves a bucket, so every key lives in its owner's range.  The owner keeps an LDS
// copy of its slots' key hashes and LDS accumulators of the batch's primary slice m0 (the slice of the middle
// record: an in-order batch has one).  A key's probe starts at the first slot of its home line of 8 slots
// (Spec::home_mask), so its candidates are one aligned 64-B line of that copy.
//
// Roles.  Waves 0..FU_PW-1 of a workgroup are producers, the others consumers; neither waits on the other
// inside the workgroup (no workgroup barrier between the prologue and the flush).
//   producer  per unit of FU_U records (four per lane, the next unit's columns in flight meanwhile): the
//             operator work (timestamp, key group, window, lateness), fmix64 of the key, the owner; a
//             counting sort of the unit by owner in the wave's LDS staging; the unit stored to its ring slot
//             as (fmix64(key), value) + the record's index in the unit, then a header of 32 words (segment
//             start, length, tag) once every store of the unit has completed.  Records of another slice and the
//             Long.MIN_VALUE key update the dense columns directly (device atomics, as k_ingest_direct).
//   consumer  round after round, the owner's segment of each of the group's FU_NP units (8 lanes per unit,
//             headers polled by tag), resolved against the LDS directory copy and reduced with LDS atomics
//             (first arrival = least batch index).  The last consumer wave of a workgroup done with a round
//             tells the group, and a producer re-fills a ring slot only after all 32 owners have read it.
// Flush.  Every owner adds its accumulators to the dense columns of slice m0 with device atomics (one lane per
// slot, consecutive slots in consecutive lanes); the last workgroup of the launch stores the f1 of the panes the
// batch created (their final first-arrival ordinal).
//
// Counters are monotonic across launches (targets from the launch count and the ring slots' uses), every wait is
// bounded (a launch that cannot make progress, e.g. because other work holds CUs so that the 256 workgroups are
// not resident together, reports FW_ERR_RESIDENCY and runs to its end instead of hanging the device), and the
// host serialises fused launches device-wide, so two of them never hold half of the CUs each.
namespace fw {

constexpr int FU_THREADS = 512;   // one workgroup per CU, two waves per SIMD (256 VGPRs a lane)
constexpr int FU_WAVES = FU_THREADS / 64;
#ifndef FW_FU_PW
#define FW_FU_PW 4
#endif
constexpr int FU_PW = FW_FU_PW;             // producer waves per workgroup
constexpr int FU_CW = FU_WAVES - FU_PW;     // consumer waves
constexpr int FU_RPL = 8;                   // records per lane of a producer unit
constexpr int FU_U = 64 * FU_RPL;           // records per producer unit
constexpr int FU_GROUPS = 8;
constexpr int FU_MEMBERS = 32;
constexpr int FU_GRID = FU_GROUPS * FU_MEMBERS;
constexpr int FU_NP = FU_MEMBERS * FU_PW;   // producer units per group and round
#ifndef FW_FU_S
#define FW_FU_S 4
#endif
constexpr int FU_S = FW_FU_S;               // ring slots (rounds in flight) per producer wave
constexpr int64_t FU_ROUND = (int64_t)FU_GROUPS * FU_NP * FU_U;   // records per round
constexpr size_t FU_HDR = 32 * 8;           // per owner: start | length << 16 | tag << 32
constexpr size_t FU_UNIT = FU_HDR + (size_t)FU_U * 18;            // header, (hash, value) pairs, unit indices (u16)
static_assert(FU_NP % (8 * FU_CW) == 0, "consumer steps of 8 units per wave");
static_assert(FU_S <= 8, "consumer round counters: misc[4, 12)");
// counter block (64-bit, monotonic)
constexpr int FU_C_REG = 0;                               // [g]     workgroups registered (32 per launch)
constexpr int FU_C_DONE = FU_C_REG + FU_GROUPS;           // [g][s]  owners done reading the units of slot s
constexpr int FU_C_PUB = FU_C_DONE + FU_GROUPS * FU_S;    // [g][s]  units of slot s published (FU_NP per use)
constexpr int FU_C_FIN = FU_C_PUB + FU_GROUPS * FU_S;     //         workgroups finished (256 per launch)
constexpr int FU_C_N = FU_C_FIN + 1;
constexpr int FU_C_PAD = 64;   // u64 words between counters: each on its own 512-B stretch (memory channel), so pollers
                               // of one counter never queue behind another's
#define FU_CTR(f, i) ((f).ctr + (size_t)(i) * FU_C_PAD)

struct FusedBuf {
  unsigned char* ring;          // [FU_GROUPS][FU_NP][FU_S] units of FU_UNIT bytes
  unsigned long long* ctr;      // [FU_C_N][FU_C_PAD]
  int32_t* xcc;                 // [FU_GRID] HW_REG_XCC_ID of each workgroup (this launch)
  unsigned long long uses[FU_S];  // rounds that used each ring slot in earlier launches
  int64_t epoch;                // fused launches before this one
  int32_t rounds;               // units per producer wave
  int32_t so_bits;              // log2(SO)
  int32_t force_safe;           // diagnostics (FW_FUSED_SAFE=1): the release/acquire hand-off for every group
  long long* stamps;            // diagnostics (FW_DEBUG_AGG & 16): per-workgroup realtime stamps, 64 per workgroup
};
// stamp i of this workgroup: 0 start, 1 prologue done, 2 producers done, 3 consumers done, 4 flushed, 5 end,
// 63 = xcc | one_l2 << 8
#define FU_STAMP(i) do { if (f.stamps && (i) < 63) f.stamps[(int64_t)w * 64 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// LDS bytes of k_fused: the producers' staging, the owner's directory copy and accumulators, counters
__host__ __device__ constexpr size_t fused_stage_bytes() { return (size_t)FU_PW * (128 + (size_t)FU_U * 18); }
__host__ __device__ constexpr size_t fused_lds_bytes(int so_bits, int nacc) {
  return fused_stage_bytes() + 64 + ((size_t)8 << so_bits) + ((size_t)1 << so_bits) * (8 * (size_t)nacc + 4);
}

__device__ __forceinline__ int fu_xcc_id() { return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15); }

// one lane: wait until counter c reaches target, bounded (~0.5 s).  Returns false (and reports
// FW_ERR_RESIDENCY once) when it gave up; a wave that gave up skips its later waits (broken)
__device__ __noinline__ bool fu_wait_at(int32_t* err, unsigned long long* c, unsigned long long target) {
  for (uint32_t spins = 0;; ++spins) {
    if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    // another wave of the launch gave up already: so does this one (the launch drains quickly)
    const bool gone = (spins & 255) == 255 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == FW_ERR_RESIDENCY;
    if (spins > (1u << 23) || gone) {
      set_error(err, FW_ERR_RESIDENCY);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

// a wave-uniform poll through the scalar unit (s_load ... glc: the scalar cache is bypassed).  Scalar loads are
// counted by lgkmcnt, not vmcnt, so waiting for one does not wait for the wave's vector loads in flight (vmcnt
// retires in issue order: a vector poll would wait for the next unit's columns).  Counters only grow, so a stale
// value can only delay a wait, never end it early
__device__ __forceinline__ unsigned long long fu_sload(const unsigned long long* p) {
  unsigned long long v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ int32_t fu_sload32(const int32_t* p) {
  int32_t v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
// the whole wave: wait until counter c reaches target, bounded like fu_wait_at
__device__ __forceinline__ bool fu_swait(int32_t* err, const unsigned long long* c, unsigned long long target) {
  for (uint32_t spins = 0;; ++spins) {
    if (fu_sload(c) >= target) return true;
    const bool gone = (spins & 255) == 255 && fu_sload32(err) == FW_ERR_RESIDENCY;
    if (spins > (1u << 23) || gone) {
      set_error(err, FW_ERR_RESIDENCY);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

typedef long long fu_v2 __attribute__((ext_vector_type(2)));
typedef unsigned long long fu_u2 __attribute__((ext_vector_type(2)));
typedef int fu_i4 __attribute__((ext_vector_type(4)));

// the owner's LDS directory copy (lh, fmix64 of its slots): slot of hash h, inserting the key (fmix64_inv(h))
// into the global directory if absent.  The probe sequence of dir_find_or_insert_at with home_mask ~7: from the
// first slot of h's home line, linearly through the bucket.  Out of line: taken by a lane only when its key is not
// on its home line
__device__ __noinline__ int32_t fu_probe_insert(uint64_t* lh, int64_t* dir_keys, uint32_t kbm, uint32_t start, uint64_t h,
                                                unsigned long long* inserted) {
  uint32_t x = start;
  for (uint32_t probe = 0; probe <= kbm; ++probe) {
    const uint64_t cur = lh[x];
    if (cur == h) return (int32_t)x;
    if (cur == EMPTY_H) {
      const int64_t key = (int64_t)fmix64_inv(h);
      const unsigned long long prev = atomicCAS((unsigned long long*)&dir_keys[x], (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)key);
      if ((int64_t)prev == EMPTY_KEY) atomicAdd(inserted, 1ull);
      const uint64_t now = (int64_t)prev == EMPTY_KEY ? h : fmix64(prev);
      lh[x] = now;   // only globally confirmed keys enter the copy
      if (now == h) return (int32_t)x;
    }
    x = (x + 1) & kbm;
  }
  return -1;
}

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(FU_THREADS, 2) void k_fused(Spec s, BatchIn b, FusedBuf f, const int64_t* f1col) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool HAS_MIN = (AGG & FW_AGG_MIN) != 0, HAS_MAX = (AGG & FW_AGG_MAX) != 0;
  constexpr bool HAS_CNT = (AGG & FW_AGG_COUNT) != 0;
  const int w = blockIdx.x, g = w & (FU_GROUPS - 1), me = w / FU_GROUPS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int SO = 1 << f.so_bits;
  unsigned char* stage = smem;                                             // [FU_PW] staging areas
  int32_t* misc = (int32_t*)(smem + fused_stage_bytes());                  // [16]
  uint64_t* lh = (uint64_t*)(misc + 16);                                   // [SO] fmix64 of the owned slots
  int64_t* lsum = (int64_t*)(lh + SO);                                     // [SO]
  int64_t* lmin = lsum + SO;
  int64_t* lmax = lmin + (HAS_MIN ? SO : 0);
  int64_t* lcnt = lmax + (HAS_MAX ? SO : 0);
  uint32_t* lfirst = (uint32_t*)(lcnt + (HAS_CNT ? SO : 0));
  const AggLds L{lsum, lmin, lmax, lcnt, lfirst, nullptr};
  const bool cmpto = s.cmpto != 0;
  const int64_t n = b.n;
  const unsigned long long ep = (unsigned long long)f.epoch;
  const int R = f.rounds;
  const int64_t dbase = (int64_t)me * SO;
  const uint32_t kbm = (1u << s.kb_bits) - 1u;
  if (tid == 0) FU_STAMP(0);
  // the batch's primary slice: the middle record's
  int64_t m0 = 0;
  {
    const int64_t tm = b.ts[n >> 1];
    if (tm != INT64_MIN) m0 = uniform64(record_windows(s, tm, b.wm).m);
  }
  // registration: this workgroup's XCD, published write-through, then counted
  const int my_xcc = fu_xcc_id();
  if (tid == 0) {
    __hip_atomic_store(f.xcc + w, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(FU_CTR(f, FU_C_REG + g), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the owned directory slots and their accumulators
  for (int x = tid; x < SO; x += FU_THREADS) {
    lh[x] = fmix64((uint64_t)s.dir_keys[dbase + x]);
    lsum[x] = sum_identity(VT);
    if (HAS_MIN) lmin[x] = INT64_MAX;
    if (HAS_MAX) lmax[x] = INT64_MIN;
    if (HAS_CNT) lcnt[x] = 0;
    lfirst[x] = NO_FIRST;
  }
  if (tid < 16) misc[tid] = 0;
  // the group's placement: one L2 (the fast hand-off) unless some member runs on another XCD
  if (tid == 0) {
    bool one_l2 = false;
    if (fu_wait_at(s.err, FU_CTR(f, FU_C_REG + g), (ep + 1) * FU_MEMBERS)) {
      one_l2 = !f.force_safe;
      for (int j = 0; j < FU_MEMBERS; ++j)
        one_l2 &= __hip_atomic_load(f.xcc + j * FU_GROUPS + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == my_xcc;
      if (!one_l2 && me == 0) atomicAdd(&s.stats[6], 1ull);   // diagnostics: group-launches on the safe path
    } else {
      misc[1] = 1;   // broken: every later wait is skipped
    }
    misc[0] = one_l2 ? 1 : 0;
  }
  __syncthreads();
  const bool one_l2 = misc[0] != 0;
  bool broken = misc[1] != 0;
  if (tid == 0) { FU_STAMP(1); if (f.stamps) f.stamps[(int64_t)w * 64 + 63] = my_xcc | (one_l2 ? 256 : 0); }
  const bool all_kg = s.kg_start == 0 && s.kg_end == s.mp - 1;
  unsigned long long late_pairs = 0;
  unsigned char* gbase = f.ring + (size_t)g * FU_NP * FU_S * FU_UNIT;

  if (wave < FU_PW) {
    // =============================== producer wave ===============================
    const int pw = wave;
    const int pu = me * FU_PW + pw;                       // this wave's unit index in the group
    int32_t* wcnt = (int32_t*)(stage + (size_t)pw * (128 + (size_t)FU_U * 18));   // [32] per owner: count, then start
    longlong2* skv = (longlong2*)(wcnt + 32);             // [FU_U]
    uint16_t* sidx = (uint16_t*)(skv + FU_U);             // [FU_U]
    // two units' columns in registers, ping-pong: unit r in X while unit r + 1 is in flight in Y; X takes unit
    // r + 2 once unit r is stored (no register copies, so no wait for Y's loads before they are used)
    int64_t ak[FU_RPL], at[FU_RPL], av[FU_RPL], bk[FU_RPL], bt[FU_RPL], bv[FU_RPL];
    bool a_vec = false, b_vec = false;   // the buffer's loads were the 12 wide loads of every lane (nothing else)
    auto unit_base = [&](int r) { return ((int64_t)(r * FU_GROUPS + g) * FU_NP + pu) * FU_U; };
    // lane: records [FU_RPL lane, FU_RPL (lane + 1)) of unit r
    auto load_unit = [&](int r, int64_t* nk, int64_t* nt, int64_t* nv) -> bool {
      const int64_t i = unit_base(r) + FU_RPL * lane;
      const bool whole = __all(i + FU_RPL - 1 < n);
      if (whole) {
#pragma unroll
        for (int q = 0; q < FU_RPL / 2; ++q) {
          const fu_v2 a = __builtin_nontemporal_load((const fu_v2*)(b.key + i + 2 * q));
          const fu_v2 c = __builtin_nontemporal_load((const fu_v2*)(b.ts + i + 2 * q));
          const fu_v2 d = __builtin_nontemporal_load((const fu_v2*)(b.val + i + 2 * q));
          nk[2 * q] = a.x; nk[2 * q + 1] = a.y; nt[2 * q] = c.x; nt[2 * q + 1] = c.y; nv[2 * q] = d.x; nv[2 * q + 1] = d.y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < FU_RPL; ++e) {
          const bool in = i + e < n;
          nk[e] = in ? b.key[i + e] : 0;
          nt[e] = in ? b.ts[i + e] : 0;
          nv[e] = in ? b.val[i + e] : 0;
        }
      }
      return whole;
    };
    if (R > 0) a_vec = load_unit(0, ak, at, av);
    if (R > 1) b_vec = load_unit(1, bk, bt, bv);
    // the previous unit's header, published once its stores have completed (one unit later, so the wait for
    // them overlaps this unit's work)
    bool pend = false;
    int pend_sl = 0;
    // unit r from buffer X (kk, tt, vv, hh); Y's loads (unit r + 1, y_vec) are the youngest memory operations
    auto unit_body = [&](int r, int64_t* kk, int64_t* tt, int64_t* vv, bool& x_vec, const bool y_vec) {
      const bool next_vec = y_vec;
      if (pw == 0 && lane == 0 && r < 8) FU_STAMP(8 + 3 * r);
      const int64_t ubase = unit_base(r);
      const int64_t lbase = ubase + FU_RPL * lane;   // batch index of this lane's first record
      // the wave's reference slice (first valid lane), valid for every record whose timestamp lies in it
      RecWin w0;
      w0.m = 0; w0.n_late = 0; w0.n_fire = 0; w0.n_windows = 0; w0.quirk = false; w0.lo = 1; w0.hi = 0;
      {
        const bool c0 = lbase < n && tt[0] > -(1LL << 61) && tt[0] < (1LL << 61);
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
      if (lane < 32) wcnt[lane] = 0;
      uint32_t route = 0, spill = 0, slow = 0;
      const bool w0_live = w0.n_windows - w0.n_late > 0;
#pragma unroll
      for (int e = 0; e < FU_RPL; ++e) {
        const int64_t i = lbase + e;
        bool ok = i < n;
        if (ok && tt[e] == INT64_MIN) { set_error(s.err, FW_ERR_NO_TIMESTAMP); ok = false; }
        if (ok && !all_kg) {
          const int32_t h = b.key_hash ? b.key_hash[i] : long_hash_code(kk[e]);   // (Java hashes: rare, loaded here)
          const int32_t kg = record_key_group(s, h);   // AbstractKeyedStateBackend.setCurrentKey :167-170
          if (kg < s.kg_start || kg > s.kg_end) { set_error(s.err, FW_ERR_KEY_GROUP); ok = false; }
        }
        const bool fast = ok && tt[e] >= w0.lo && tt[e] <= w0.hi;
        slow |= (ok && !fast ? 1u : 0u) << e;
        if (fast) late_pairs += (unsigned long long)w0.n_late;
        const bool live = fast && w0_live;
        if (live && w0.n_fire > 0) set_error(s.err, FW_ERR_UNSUPPORTED);   // no per-element fires: lateness is 0
        const bool rt = live && w0.m == m0 && kk[e] != EMPTY_KEY;
        route |= (rt ? 1u : 0u) << e;
        spill |= (live && !rt ? 1u : 0u) << e;
      }
      // records outside the wave's reference slice: the full window assignment (rare: not unrolled); a record
      // of another slice than the primary one (or the Long.MIN_VALUE key) updates the dense columns directly
      if (__any((slow | spill) != 0)) {
#pragma unroll 1
        for (int e = 0; e < FU_RPL; ++e) {
          const int64_t i = lbase + e;
          bool sp = (spill >> e) & 1u;
          int64_t m = w0.m;
          if ((slow >> e) & 1u) {
            const int64_t ts = b.ts[i], key = b.key[i];
            const RecWin rw = record_windows(s, ts, b.wm);
            if (rw.quirk) quirk_record(s, b, key, i, rw.qn, rw.q_late, rw.q_fire);
            late_pairs += (unsigned long long)rw.n_late;
            const bool live = rw.n_windows - rw.n_late > 0;
            if (live && rw.n_fire > 0) set_error(s.err, FW_ERR_UNSUPPORTED);
            const bool rt = live && rw.m == m0 && key != EMPTY_KEY;
            route |= (rt ? 1u : 0u) << e;
            sp = live && !rt;
            m = rw.m;
          }
          int64_t idx = -1;
          if (sp) {
            const int32_t p = slice_slot(s, m);
            const int64_t kid = p < 0 ? -1 : dir_lookup(s, b.key[i]);   // (Long.MIN_VALUE: kid D)
            if (p < 0 || kid < 0) {
              cap_error(s, 31);
            } else {
              const int64_t pi = (int64_t)p * s.stride + kid;
              if (pane_update<VT, AGG, FIRST>(s, pi, b.val[i], b.ord_base + i)) idx = pi;
            }
          }
          if (FIRST) {   // the panes this batch created: their f1 is set after every workgroup is done
            const bool fresh = idx >= 0;
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
      // owner of each routed record, and its rank among the unit's records of that owner (LDS counters of
      // this wave only: in-order LDS operations of one wave need no barrier)
      int32_t br[FU_RPL];   // owner << 16 | rank among the unit's records of that owner (fmix64 recomputed below:
                            // fewer registers live across the scan)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the counters are zero
#pragma unroll
      for (int e = 0; e < FU_RPL; ++e) {
        const int32_t bin = (int32_t)((fmix64((uint64_t)kk[e]) & s.dir_mask) >> f.so_bits);
        br[e] = ((route >> e) & 1u) ? (bin << 16) | atomicAdd(&wcnt[bin], 1) : 0;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // every rank taken
      // segment starts (lanes 0..31, one owner each) and the header words
      uint64_t hword = 0;
      {
        const int32_t c = lane < 32 ? __hip_atomic_load(&wcnt[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
        int32_t incl = c;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const int32_t y = __shfl_up(incl, o);
          if (lane >= o) incl += y;
        }
        const int32_t st = incl - c;
        if (lane < 32) __hip_atomic_store(&wcnt[lane], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        hword = (uint64_t)(uint32_t)st | ((uint64_t)(uint32_t)c << 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the starts are in place
      int32_t rc = __popc(route);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) rc += __shfl_xor(rc, o);
      const int32_t routed = __builtin_amdgcn_readfirstlane(rc);   // records staged by the unit
#pragma unroll
      for (int e = 0; e < FU_RPL; ++e) {
        if ((route >> e) & 1u) {
          const int32_t pos = __hip_atomic_load(&wcnt[br[e] >> 16], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + (br[e] & 0xFFFF);
          skv[pos] = make_longlong2((long long)fmix64((uint64_t)kk[e]), (long long)vv[e]);
          sidx[pos] = (uint16_t)(FU_RPL * lane + e);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the staging is written
      // publish unit r - 1 (before waiting for this unit's ring slot, which needs the consumers to progress): its stores (header included) are older than unit r + 1's loads (issued after them),
      // so waiting for all but those 12 wide loads waits for the stores only (vmcnt counts in issue order)
      if (pend) {
        if (next_vec && one_l2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!one_l2) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) __hip_atomic_fetch_add(FU_CTR(f, FU_C_PUB + g * FU_S + pend_sl), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // the ring slot is free once every owner of the group read its previous use
      const int sl = r % FU_S;
      const unsigned long long use = f.uses[sl] + (unsigned long long)(r / FU_S);
      if (use > 0 && !broken) {
        bool okw = true;
        if (lane == 0) okw = fu_wait_at(s.err, FU_CTR(f, FU_C_DONE + g * FU_S + sl), use * FU_MEMBERS);
        broken = !__builtin_amdgcn_readfirstlane(okw ? 1 : 0);
      }
      if (pw == 0 && lane == 0 && r < 8) FU_STAMP(9 + 3 * r);
      // (the slot's address made scalar here, not hoisted into vector registers for the whole loop)
      unsigned char* unit = (unsigned char*)uniform64((int64_t)(gbase + ((size_t)pu * FU_S + sl) * FU_UNIT));
      longlong2* gkv = (longlong2*)(unit + FU_HDR);
      uint16_t* gidx = (uint16_t*)(gkv + FU_U);
#pragma unroll 1
      for (int x = lane; x < routed; x += 64) gkv[x] = skv[x];
#pragma unroll 1
      for (int x = 2 * lane; x < routed; x += 128) *(uint32_t*)(gidx + x) = *(const uint32_t*)(sidx + x);
      if (lane < 32) ((unsigned long long*)unit)[lane] = hword | ((use + 1) << 32);
      pend = true;
      pend_sl = sl;
      if (pw == 0 && lane == 0 && r < 8) FU_STAMP(10 + 3 * r);
      if (r + 2 < R) x_vec = load_unit(r + 2, kk, tt, vv);   // after the stores: see the publish above
      else x_vec = false;
    };
    for (int r = 0; r < R; r += 2) {   // uniform
      unit_body(r, ak, at, av, a_vec, b_vec);
      if (r + 1 < R) unit_body(r + 1, bk, bt, bv, b_vec, a_vec);
    }
    if (pend) {   // the last unit
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!one_l2) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (lane == 0) __hip_atomic_fetch_add(FU_CTR(f, FU_C_PUB + g * FU_S + pend_sl), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) FU_STAMP(2);
  } else {
    // =============================== consumer wave ===============================
    const int cw = wave - FU_PW;
    int32_t* lcd = misc + 4;   // [FU_S <= 8] consumer waves done with the rounds of ring slot s
    constexpr int UPW = FU_NP / FU_CW;   // units per consumer wave and round (lanes 0..UPW-1 poll their headers)
    constexpr int STEPS = UPW / 8;       // 8 lanes per unit's segment
    constexpr int KPRE = 2;              // records per lane and step loaded up front (segments up to 16 records)
    static_assert(UPW <= 64, "one header per lane");
    const int sub = lane & 7;
    bool got = false;   // this lane reduced a record
    auto unit_of = [&](int r, int u) {
      return gbase + ((size_t)(cw * UPW + u) * FU_S + (size_t)(r % FU_S)) * FU_UNIT;
    };
    auto tag_of = [&](int r) { return (uint32_t)(f.uses[r % FU_S] + (unsigned long long)(r / FU_S) + 1); };
    // one record of the segment into the accumulators
    auto reduce_one = [&](const fu_v2 rv, uint32_t bi) {
      const uint64_t h = (uint64_t)rv.x;
      const uint32_t loc = (uint32_t)((h & s.dir_mask) - (uint64_t)dbase);   // slot relative to the owned range
      if (loc >= (uint32_t)SO) { cap_error(s, 35); return; }                 // (another owner's key: a torn unit)
      const uint32_t bb = loc & ~kbm, h0 = loc & kbm & s.home_mask;
      const fu_u2* wl = (const fu_u2*)(lh + bb + h0);
      const fu_u2 a0 = wl[0], a1 = wl[1], a2 = wl[2], a3 = wl[3];
      int32_t kl = -1;
      kl = a3.y == h ? 7 : kl; kl = a3.x == h ? 6 : kl; kl = a2.y == h ? 5 : kl; kl = a2.x == h ? 4 : kl;
      kl = a1.y == h ? 3 : kl; kl = a1.x == h ? 2 : kl; kl = a0.y == h ? 1 : kl; kl = a0.x == h ? 0 : kl;
      if (kl >= 0) kl += (int32_t)h0;
      else kl = fu_probe_insert(lh + bb, s.dir_keys + dbase + bb, kbm, h0, h, s.stats + ST_DIR_KEYS);
      if (kl < 0) { cap_error(s, 34); return; }
      acc_add<VT, AGG>(L, cmpto, false, 0, bb + (uint32_t)kl, (int64_t)rv.y, bi);
      got = true;
    };
    // headers: lane u < UPW holds the header word of unit cw * UPW + u of the round, read once the group's
    // publication counter of the ring slot says every unit of the round is complete (one polling lane per wave)
    for (int r = 0; r < R; ++r) {   // uniform
      const int sl = r % FU_S;
      const uint32_t tag = tag_of(r);
      const unsigned long long use = f.uses[sl] + (unsigned long long)(r / FU_S);
      if (!broken) {
        bool okw = true;
        if (lane == 0) okw = fu_wait_at(s.err, FU_CTR(f, FU_C_PUB + g * FU_S + sl), (use + 1) * FU_NP);
        broken = !__builtin_amdgcn_readfirstlane(okw ? 1 : 0);
      }
      if (!one_l2) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (cw == 0 && lane == 0 && r < 8) FU_STAMP(32 + 3 * r);
      uint64_t hw = 0;
      if (lane < UPW && !broken)
        hw = __hip_atomic_load((const unsigned long long*)unit_of(r, lane) + me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane < UPW && !broken && (uint32_t)(hw >> 32) != tag) { cap_error(s, 33); hw = 0; }   // (a torn publication)
      if (lane >= UPW) hw = 0;
      // every lane's first KPRE records of each step's segment, loaded before any is reduced
      fu_v2 rv[STEPS][KPRE];
      uint32_t bi[STEPS][KPRE];
      int32_t cnt[STEPS], st[STEPS];
#pragma unroll
      for (int q = 0; q < STEPS; ++q) {
        const int u = q * 8 + (lane >> 3);
        const uint64_t w = __shfl(hw, u);
        st[q] = (int32_t)(w & 0xFFFF);
        cnt[q] = min((int32_t)((w >> 16) & 0xFFFF), FU_U - st[q]);   // (bounds a torn header could break)
        const unsigned char* unit = unit_of(r, u);
        const fu_v2* gkv = (const fu_v2*)(unit + FU_HDR);
        const uint16_t* gidx = (const uint16_t*)(unit + FU_HDR + (size_t)FU_U * 16);
        const uint32_t ub = (uint32_t)(((int64_t)(r * FU_GROUPS + g) * FU_NP + cw * UPW + u) * FU_U);
#pragma unroll
        for (int k = 0; k < KPRE; ++k) {
          const int i = sub + 8 * k;
          if (i < cnt[q]) {
            rv[q][k] = __builtin_nontemporal_load(gkv + st[q] + i);
            bi[q][k] = ub + __builtin_nontemporal_load(gidx + st[q] + i);
          }
        }
      }
      if (cw == 0 && lane == 0 && r < 8) FU_STAMP(33 + 3 * r);
#pragma unroll
      for (int q = 0; q < STEPS; ++q) {
#pragma unroll
        for (int k = 0; k < KPRE; ++k)
          if (sub + 8 * k < cnt[q]) reduce_one(rv[q][k], bi[q][k]);
      }
      if (cw == 0 && lane == 0 && r < 8) FU_STAMP(34 + 3 * r);
      // segments longer than KPRE * 8 records (rare)
#pragma unroll 1
      for (int q = 0; q < STEPS; ++q) {
        if (!__any(cnt[q] > 8 * KPRE)) continue;
        const int u = q * 8 + (lane >> 3);
        const unsigned char* unit = unit_of(r, u);
        const fu_v2* gkv = (const fu_v2*)(unit + FU_HDR);
        const uint16_t* gidx = (const uint16_t*)(unit + FU_HDR + (size_t)FU_U * 16);
        const uint32_t ub = (uint32_t)(((int64_t)(r * FU_GROUPS + g) * FU_NP + cw * UPW + u) * FU_U);
        for (int i = sub + 8 * KPRE; i < cnt[q]; i += 8)
          reduce_one(__builtin_nontemporal_load(gkv + st[q] + i), ub + __builtin_nontemporal_load(gidx + st[q] + i));
      }
      // this wave is done with round r; the last consumer wave of the workgroup tells the group
      if (lane == 0) {
        const int old = atomicAdd(&lcd[sl], 1);
        if (old + 1 == FU_CW * (r / FU_S + 1))
          __hip_atomic_fetch_add(FU_CTR(f, FU_C_DONE + g * FU_S + sl), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (__any(got) && lane == 0) misc[12] = 1;
    if (lane == 0) FU_STAMP(3);
  }
  if (__any(late_pairs != 0)) {
    for (int off = 32; off > 0; off >>= 1) late_pairs += __shfl_xor(late_pairs, off);
    if (lane == 0) atomicAdd(&s.stats[ST_LATE], late_pairs);
  }
  __syncthreads();

  // ---------------- flush: the owned slots' accumulators into the dense columns of slice m0 ----------------
  if (tid == 0) {   // the slot of slice m0, claimed (idempotently) by every owner that reduced a record
    int32_t p0 = -1;
    if (misc[12]) {
      p0 = slice_slot(s, m0);
      if (p0 < 0) cap_error(s, 32);
    }
    misc[2] = p0;
  }
  __syncthreads();
  const int32_t p0 = misc[2];
  if (p0 >= 0) {
    for (int x = tid; x < SO; x += FU_THREADS) {   // whole waves (SO is a power of two >= 64)
      const uint32_t lf = lfirst[x];
      const int64_t idx = (int64_t)p0 * s.stride + dbase + x;
      bool fresh = false;
      if (lf != NO_FIRST) {
      if (AGG & FW_AGG_SUM) {
        if (VT == FW_VALUE_I64) atomicAdd((unsigned long long*)&s.c.sum[idx], (unsigned long long)lsum[x]);
        else unsafeAtomicAdd((double*)&s.c.sum[idx], __longlong_as_double(lsum[x]));
      }
      if (HAS_MIN) atomicMin((long long*)&s.c.mn[idx], (long long)lmin[x]);
      if (HAS_MAX) atomicMax((long long*)&s.c.mx[idx], (long long)lmax[x]);
      if (HAS_CNT) atomicAdd((unsigned long long*)&s.c.cnt[idx], (unsigned long long)lcnt[x]);
      if (FIRST) {
        // a pane present before this batch keeps its (earlier) first arrival; first only decreases within the
        // launch, so a plain load already at or below this batch's ordinal proves there is nothing to do
        const int64_t ord = b.ord_base + (int64_t)lf;
        if (ord < s.c.first[idx]) fresh = atomicMin((long long*)&s.c.first[idx], (long long)ord) == INT64_MAX;
      } else {
        s.c.present[idx] = 1;
      }
      }
      if (FIRST) {   // the panes this batch created (one creator each): their f1 once every workgroup is done
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
  if (tid == 0) FU_STAMP(4);

  // ---------------- the last workgroup: f1 of the panes this batch created ----------------
  if (FIRST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned long long done = __hip_atomic_fetch_add(FU_CTR(f, FU_C_FIN), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  if (tid == 0) FU_STAMP(5);
}

}  // namespace fw
