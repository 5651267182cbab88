// fw_engine.hip — MI355X (gfx950) keyed event-time window aggregation engine behind the C-ABI of
// include/flink_window.h.  One engine = one WindowOperator subtask = one GPU.
//
// Data layout in HBM:
//   key directory   dir_keys[D+1]            open addressing, linear probing on fmix64(key); the slot index
//                                            is the dense key id `kid` (index D holds key Long.MIN_VALUE)
//   pane slices     per slice slot p < P:    dense columns [p][kid] of the reduce accumulator
//                                            (sum/min/max/count, first-arrival ordinal, first-arrival f1)
//                   slice_tag[P]             slice number m held by slot p = floor_mod(m, P), or FREE
//   output log      fired records + watermark marks, appended on device, drained by fw_collect
//
// A pane is (key, window).  Windows are unions of K = size/g consecutive slices of width
// g = gcd(size, slide) (tumbling: one slice = one window), so a record touches exactly ONE slice
// whatever the window overlap — the reference keeps one pane per (key, window) instead
// (HeapReducingState.add, RT/state/heap/HeapReducingState.java:84-122, called once per assigned
// window from WindowOperator.java:302-333).  Fire combines the K slices of a window; this is exact
// for integer sum/min/max/count and order-changing (tolerance 1e-9) for double sums.
//
// Timers (HeapInternalTimerService, SJ/api/operators/HeapInternalTimerService.java:211-278) are not
// materialised: a pane exists iff its trigger timer is pending, so the watermark step fires every
// window whose maxTimestamp lies in (previous watermark, new watermark] and purges every slice whose
// last window's cleanup time has passed (WindowOperator.onEventTime :336-375, cleanupTime :511-514).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan_by_key.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <set>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flink_window.h"
#include "java_semantics.h"
#include "flink_kg_format.h"

#ifndef FW_NO_HOSTLOAD
#define FW_NO_HOSTLOAD 0
#endif
#ifndef FW_NO_GSLSORT
#define FW_NO_GSLSORT 0
#endif
#ifndef FW_AGG_PRECHECK
#define FW_AGG_PRECHECK 0
#endif
#ifndef FW_AGG_UR
#define FW_AGG_UR 1   // k_aggregate: wave steps whose loads are in flight together (two sets: 2 x UR; 1 measured faster than 2 in round 6)
#endif

namespace fw {

constexpr int64_t FREE_TAG = INT64_MIN;
constexpr int64_t EMPTY_KEY = INT64_MIN;
constexpr int MAX_K = 1024;        // max slices per window (k_watermark's LDS table of a window's slice slots)
constexpr int MAX_P = 4096;        // max slice slots
constexpr int LIST_MAX_K = 64;     // list state: slices per window (k_list_gather's per-thread slice table)
constexpr int BLOCK = 256;

// ST_SHARES: helper shares run; ST_DIR_KEYS: keys in the directory buckets (inserts since the last compaction + the keys it kept)
// ST_QUIRK: records that got the sliding assigner's extra window (negative remainder, window panes below)
enum Stat { ST_LATE = 0, ST_FIRED = 1, ST_LATE_FIRES = 2, ST_SHARES = 3, ST_DIR_KEYS = 4, ST_QUIRK = 5, ST_NSTATS = 8 };

// ------------------------------------------------------------------------------------------------
// device views
// ------------------------------------------------------------------------------------------------
struct Cols {  // dense pane columns, each [P][stride]
  int64_t* sum;        // int64 sum, or double bits
  int64_t* mn;         // int64 min, or Math.min code of a double
  int64_t* mx;
  int64_t* cnt;
  int64_t* first;      // first-arrival ordinal, INT64_MAX = no pane
  int64_t* f1v;        // f1 of the first arrival
  uint8_t* present;    // pane presence when first-arrival is not tracked
};

struct OutLog {
  int64_t* key;
  int64_t* f1;
  int64_t* ts;
  int64_t* sum;
  int64_t* mn;
  int64_t* mx;
  int64_t* cnt;
  unsigned long long* count;  // records appended since the last collect
  int64_t capacity;
  int64_t* mark_wm;
  int64_t* mark_pos;
  unsigned long long* mark_count;
  int64_t mark_capacity;
  int64_t* win_start;   // session windows: window.getStart() of each result
};

struct Spec {  // window specification + reduce + subtask, passed by value
  int32_t assigner, trigger;
  int64_t size, slide, offset, lateness, g;
  double inv_size, inv_g;   // reciprocals for jdivmod
  int32_t K;        // slices per window
  int32_t R;        // slices per slide
  int32_t mp, kg_start, kg_end;
  int32_t mp_mask;  // mp - 1 when mp is a power of two, else 0
  int32_t vt, agg, first;
  int32_t cmpto;    // min/max of doubles in Double.compareTo order (ComparableAggregator), else Math.min/max
  int32_t by;       // 0, FW_AGG_MAXBY or FW_AGG_MINBY: the extremal record (value, f1) is the result
  int32_t by_last;  // maxBy/minBy tie rule: the later record (first = false)
  int32_t fold;     // WindowedStream.fold: every result starts from fold_init (applied where results are emitted)
  int64_t fold_init;
  // directory
  int64_t* dir_keys;
  int32_t* dir_min_used;
  uint64_t dir_mask;
  int64_t D;
  int32_t kb_bits;  // log2(slots per directory bucket); probing stays inside the home bucket
  int32_t nb;       // directory buckets = D >> kb_bits
  // slices
  int32_t P;
  int64_t stride;   // D + 1
  int64_t* slice_tag;
  Cols c;
  // sliding windows: per-window panes [W][stride] for the one window a record below offset - slide gets
  // beyond its slice's windows (SlidingEventTimeWindows.assignWindows starting at
  // getWindowStartWithOffset, whose Java % of a negative numerator lands one slide above the record:
  // SlidingEventTimeWindows.java:64-77, TimeWindow.java:239-241); wtag[w] = window number held, FREE else
  Cols wc;
  int64_t* wtag;
  int32_t W;
  OutLog o;
  int32_t* err;
  unsigned long long* stats;
  unsigned int* dir_keys_host;   // host-mapped copy of stats[ST_DIR_KEYS], posted at each firing watermark
  // restored tumbling windows whose trigger timers fired before the checkpoint (restore at Long.MIN_VALUE,
  // fw_restore_kg_flink): disarm[p] marks such a window's slot; a pane fires at its maxTimestamp only if a
  // record re-armed its timer (armed[p * stride + kid], EventTimeTrigger.onElement :37-45).  Null otherwise
  uint8_t* disarm;
  uint8_t* armed;
  // PurgingTrigger + allowed lateness (tumbling): a fired window's purge clears its state but keeps each key's
  // cleanup timer until the cleanup time (WindowOperator.java:365-371 purges contents only; the timer goes at
  // :420-428).  gfirst[p * stride + kid] = the arrival ordinal that registered the timer of (key, window gtag[p])
  // (0 without first-arrival tracking), INT64_MAX = none; the timers' only trace, written to checkpoints.  Null else
  int64_t* gtag;
  int64_t* gfirst;
  long long* wm_stamps;   // diagnostics (FW_DEBUG_AGG & 16): k_watermark phase timestamps, 8 per workgroup; null else
};

// the Spec fields k_route's per-record work reads, passed by value (kernel arguments, in SGPRs from the wave's start;
// read through the device Spec pointer they were scalar loads issued and waited on in the middle of each tile's
// record pass, round 6).  Field names as in Spec, so the window assignment takes either
struct RouteSpec {
  int32_t assigner, K, R, mp, kg_start, kg_end, mp_mask, kb_bits, nb;
  int64_t size, slide, offset, lateness, g;
  double inv_size, inv_g;
  uint64_t dir_mask;
  int32_t* err;
  unsigned long long* stats;
};

// the Spec fields k_aggregate reads, by value (kernel arguments: in SGPRs from the wave's start, where the
// device Spec's fields were scalar loads waited on at the prologue and at each slice's claim, round 6)
struct AggSpec {
  int32_t nb, kb_bits, P, by_last, cmpto;
  int64_t stride, D;
  int64_t* dir_keys;
  int64_t* slice_tag;
  int32_t* dir_min_used;
  int32_t* err;
  unsigned long long* stats;
  Cols c;
};

__device__ __forceinline__ void set_error(int32_t* err, int32_t code) { atomicCAS(err, 0, code); }
// a capacity error, with the id of the site that raised it first (fw_debug_counters word 7: diagnostics)
#define cap_error(s, site) do { set_error((s).err, FW_ERR_CAPACITY); \
    atomicCAS(&(s).stats[7], 0ull, (unsigned long long)(site)); } while (0)

// a pointer the compiler cannot see is global (loaded from the device-resident Spec) is accessed as flat: every
// flat access waits on LDS and global traffic alike (s_waitcnt vmcnt(0) lgkmcnt(0)), which serialised k_aggregate's
// fold and prologue loads (round 6).  G() states the address space where it matters
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* G(T* p) { return (__attribute__((address_space(1))) T*)p; }

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {  // MurmurHash3 finaliser: directory hash
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// inverse of fmix64 (fmix64 is a bijection on 64-bit words): k ^= k >> 33 is an involution, and the
// multipliers are odd, so their inverses mod 2^64 exist
__device__ __forceinline__ uint64_t fmix64_inv(uint64_t h) {
  h ^= h >> 33;
  h *= 0x9cb4b2f8129337dbull;
  h ^= h >> 33;
  h *= 0x4f74430c22a54005ull;
  h ^= h >> 33;
  return h;
}
constexpr uint64_t EMPTY_H = 0x8f780810af31a493ull;   // fmix64(Long.MIN_VALUE): the hash of an empty slot

__device__ __forceinline__ uint64_t lanemask_lt() { return __lanemask_lt(); }

// wave-aggregated counter add; returns this lane's slot (only meaningful where pred)
__device__ __forceinline__ unsigned long long wave_append(unsigned long long* ctr, bool pred) {
  uint64_t mask = __ballot(pred);
  if (mask == 0) return 0;
  int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  return base + (unsigned long long)__popcll(mask & lanemask_lt());
}
__device__ __forceinline__ void wave_count(unsigned long long* ctr, bool pred) {
  uint64_t mask = __ballot(pred);
  if (mask != 0 && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)mask) - 1))
    atomicAdd(ctr, (unsigned long long)__popcll(mask));
}

// key -> kid (directory slot).  Linear probing inside the key's home bucket of 2^kb_bits slots, so
// every kid of a key lies in the bucket its hash names: the partitioned ingest (k_route / k_aggregate)
// owns whole buckets exclusively, and k_aggregate probes an LDS copy of the bucket with the same
// sequence.  Entries go EMPTY -> key once and never change until engine reset, so a plain (possibly
// stale) load can only under-report, which the CAS then corrects; a key found EMPTY at slot j cannot
// sit at a later slot.
__device__ __forceinline__ int64_t dir_find_or_insert_at(int64_t* dir_keys, int32_t* dir_min_used, uint64_t dir_mask,
                                                         int32_t kb_bits, int64_t D, int64_t key,
                                                         unsigned long long* inserted) {
  if (key == EMPTY_KEY) {
    if (dir_min_used[0] == 0) dir_min_used[0] = 1;
    return D;
  }
  const uint64_t home = fmix64((uint64_t)key) & dir_mask;
  const uint64_t kbm = (1ull << kb_bits) - 1;
  const uint64_t base = home & ~kbm;
  uint64_t off = home & kbm;
  for (uint64_t probe = 0; probe <= kbm; ++probe) {
    const uint64_t h = base + off;
    const int64_t cur = dir_keys[h];
    if (cur == key) return (int64_t)h;
    if (cur == EMPTY_KEY) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&dir_keys[h], (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)key);
      if ((int64_t)prev == EMPTY_KEY) atomicAdd(inserted, 1ull);
      if ((int64_t)prev == EMPTY_KEY || (int64_t)prev == key) return (int64_t)h;
    }
    off = (off + 1) & kbm;
  }
  return -1;
}
__device__ __noinline__ int64_t dir_find_or_insert_call(int64_t* dir_keys, int32_t* dir_min_used, uint64_t dir_mask,
                                                        int32_t kb_bits, int64_t D, int64_t key,
                                                        unsigned long long* inserted) {
  return dir_find_or_insert_at(dir_keys, dir_min_used, dir_mask, kb_bits, D, key, inserted);
}
// inline: the direct form's per-record lookup
__device__ __forceinline__ int64_t dir_find_or_insert(const Spec& s, int64_t key) {
  return dir_find_or_insert_at(s.dir_keys, s.dir_min_used, s.dir_mask, s.kb_bits, s.D, key, s.stats + ST_DIR_KEYS);
}
// out of line: the rare lookups of the partitioned form (new keys, direct-list records) and restore
__device__ __forceinline__ int64_t dir_lookup(const Spec& s, int64_t key) {
  return dir_find_or_insert_call(s.dir_keys, s.dir_min_used, s.dir_mask, s.kb_bits, s.D, key, s.stats + ST_DIR_KEYS);
}

// slice number m -> slot p, claiming a FREE slot.  Returns -1 when slot p holds another live slice.
// Out of line: one call per wave and slice change on the hot path.
__device__ __forceinline__ int32_t slice_slot_body(int64_t* slice_tag, int32_t P, int64_t m) {
  int32_t p = (int32_t)floor_mod(m, P);
  int64_t tag = slice_tag[p];
  if (tag == m) return p;
  if (tag == FREE_TAG) {
    unsigned long long prev = atomicCAS((unsigned long long*)&slice_tag[p], (unsigned long long)FREE_TAG,
                                        (unsigned long long)m);
    if ((int64_t)prev == FREE_TAG || (int64_t)prev == m) return p;
    return -1;
  }
  // the cached value may be stale (the slot was freed and re-claimed by a kernel boundary, which
  // flushes caches) — re-read atomically before giving up
  unsigned long long now = atomicCAS((unsigned long long*)&slice_tag[p], (unsigned long long)FREE_TAG,
                                     (unsigned long long)m);
  if ((int64_t)now == FREE_TAG || (int64_t)now == m) return p;
  return -1;
}
__device__ __noinline__ int32_t slice_slot_at(int64_t* slice_tag, int32_t P, int64_t m) { return slice_slot_body(slice_tag, P, m); }
__device__ __forceinline__ int32_t slice_slot(const Spec& s, int64_t m) { return slice_slot_at(s.slice_tag, s.P, m); }

// the identity of the sum: 0, or -0.0 for doubles (x + -0.0 == x for every x, -0.0 included; +0.0 would
// turn a pane whose only values are -0.0 into +0.0, where the reference keeps its first value as is)
__host__ __device__ __forceinline__ int64_t sum_identity(int32_t vt) { return vt == FW_VALUE_F64 ? INT64_MIN : 0; }

// orderable codes of a value for the min / max columns: int64 values as they are; doubles in Math.min /
// Math.max order, or Double.compareTo order for ComparableAggregator (.min/.max with FW_AGGF_COMPARABLE,
// and always for maxBy/minBy)
__host__ __device__ __forceinline__ int64_t min_code(int32_t vt, bool cmpto, int64_t v) {
  if (vt == FW_VALUE_I64) return v;
  double d;
  memcpy(&d, &v, 8);
  return cmpto ? f64_cmp_code(d) : f64_min_code(d);
}
__host__ __device__ __forceinline__ int64_t max_code(int32_t vt, bool cmpto, int64_t v) {
  if (vt == FW_VALUE_I64) return v;
  double d;
  memcpy(&d, &v, 8);
  return cmpto ? f64_cmp_code(d) : f64_max_code(d);
}

// Window bookkeeping for one record, following SlidingEventTimeWindows.assignWindows (:64-77) /
// TumblingEventTimeWindows.assignWindows (:59-68).  Produces the record's slice number m and how many
// of its windows are late (WindowOperator.isLate :470-472) or already fired (EventTimeTrigger.onElement
// FIRE branch, EventTimeTrigger.java:38-40).
struct RecWin {
  int64_t m;          // slice number
  int32_t n_windows;  // windows assigned
  int32_t n_late;     // of which late (dropped)
  int32_t n_fire;     // of which not late but maxTimestamp <= watermark (per-element fire)
  bool quirk;         // sliding: the record also gets window qn (Java % of a negative numerator)
  bool q_late, q_fire;  // ... which is late / already fired (per-element fire)
  int64_t qn;
  int64_t lo, hi;     // the slice's timestamps [lo, hi]: every ts in it gets this same RecWin (lo > hi: none)
};

struct SlideSpec { int64_t offset, size, slide, g, lateness; double inv_g; int32_t K, R; };

// sliding assignment, out of line (the tumbling case is inlined on the hot path)
template <bool INL>
__device__ __forceinline__ RecWin record_windows_sliding_body(const SlideSpec& s, int64_t ts, int64_t wm) {
  RecWin r;
  r.quirk = false;
  r.q_late = false;
  r.q_fire = false;
  r.qn = 0;
  r.n_late = 0;
  r.n_fire = 0;
  const int64_t y = jsub(ts, s.offset);
  const int64_t x = jadd(y, s.g);
  if (x >= 0) {
    int64_t q, rem;
    if (INL) jdivmod_inl(x, s.g, s.inv_g, q, rem);
    else jdivmod(x, s.g, s.inv_g, q, rem);
    r.m = q - 1;
    // ts' in [ts - rem, ts - rem + g) shares q
    r.lo = jsub(ts, rem);
    r.hi = jadd(r.lo, s.g - 1);
    if (r.hi < r.lo) { r.lo = 1; r.hi = 0; }
  } else {
    r.m = floor_div(y, s.g);   // the slice holding ts (below the first slice at or above the offset)
    r.lo = 1; r.hi = 0;
  }
  if (jadd(y, s.slide) < 0) {
    // getWindowStartWithOffset(ts, offset, slide) = ts - (y + slide) % slide: a negative Java remainder puts
    // the first window one slide above the floor start — one window more than the slice's (n_hi + 1)
    r.lo = 1; r.hi = 0;
    if (y % s.slide != 0) {
      r.quirk = true;
      r.qn = floor_div(r.m, s.R) + 1;
      const int64_t start = jadd(s.offset, (int64_t)((uint64_t)r.qn * (uint64_t)s.slide));
      const int64_t max_ts = jsub(jadd(start, s.size), 1);
      const int64_t ct = cleanup_time(max_ts, s.lateness);
      r.q_late = ct <= wm;
      r.q_fire = !r.q_late && max_ts <= wm;
    }
  }
  int64_t n_hi = floor_div(r.m, s.R);
  int64_t n_lo = floor_div(r.m - s.K, s.R) + 1;
  r.n_windows = (int32_t)(n_hi - n_lo + 1);
  for (int64_t n = n_lo; n <= n_hi; ++n) {
    int64_t start = jadd(s.offset, (int64_t)((uint64_t)n * (uint64_t)s.slide));
    int64_t max_ts = jsub(jadd(start, s.size), 1);
    int64_t ct = cleanup_time(max_ts, s.lateness);
    if (ct <= wm) r.n_late++;
    else if (max_ts <= wm) r.n_fire++;
  }
  return r;
}
__device__ __noinline__ RecWin record_windows_sliding(SlideSpec s, int64_t ts, int64_t wm) {
  return record_windows_sliding_body<false>(s, ts, wm);
}


template <bool INL = false, class SP = Spec>
__device__ __forceinline__ RecWin record_windows(const SP& s, int64_t ts, int64_t wm) {
  if (s.assigner != FW_TUMBLING) {
    const SlideSpec ss{s.offset, s.size, s.slide, s.g, s.lateness, s.inv_g, s.K, s.R};
    return INL ? record_windows_sliding_body<true>(ss, ts, wm) : record_windows_sliding(ss, ts, wm);
  }
  RecWin r;
  r.quirk = false;
  r.q_late = false;
  r.q_fire = false;
  r.qn = 0;
  r.n_late = 0;
  r.n_fire = 0;
  int64_t x = jadd(jsub(ts, s.offset), s.size);
  int64_t q, rem;
  if (INL) jdivmod_inl(x, s.size, s.inv_size, q, rem);
  else jdivmod(x, s.size, s.inv_size, q, rem);
  r.m = q - 1;                                                 // start = offset + m * size
  int64_t start = jsub(ts, rem);                               // getWindowStartWithOffset
  int64_t max_ts = jsub(jadd(start, s.size), 1);               // TimeWindow.maxTimestamp
  int64_t ct = cleanup_time(max_ts, s.lateness);
  r.n_windows = 1;
  // ts' in [start, max_ts] shares the window when x >= 0 (a negative x is Java's truncating-% regime)
  r.lo = start;
  r.hi = max_ts;
  if (x < 0 || max_ts < start) { r.lo = 1; r.hi = 0; }
  if (ct <= wm) r.n_late = 1;
  else if (max_ts <= wm) r.n_fire = 1;
  return r;
}

// key group of a record (KeyGroupRangeAssignment.assignToKeyGroup :51-64); murmurHash is >= 0, so for
// the usual power-of-two maxParallelism the remainder is a mask
template <class SP>
__device__ __forceinline__ int32_t record_key_group(const SP& s, int32_t key_hash) {
  return s.mp_mask ? (murmur_hash(key_hash) & s.mp_mask) : key_group_for_hash(key_hash, s.mp);
}

// ------------------------------------------------------------------------------------------------
// ingest, direct form: every (record, slice) update is a device-scope atomic on the dense columns.
// ------------------------------------------------------------------------------------------------
template <int VT, int AGG, bool FIRST, bool COLS_ONLY = false>
// returns true for exactly one record of a pane absent before the launch (FIRST: the min-ordinal
// atomic that found the pane empty).  COLS_ONLY: the reduce columns only (no first-arrival / presence)
__device__ __forceinline__ bool pane_update(const Spec& s, int64_t idx, int64_t vbits, int64_t ord) {
  if (AGG & FW_AGG_SUM) {
    if (VT == FW_VALUE_I64) {
      atomicAdd((unsigned long long*)&s.c.sum[idx], (unsigned long long)vbits);
    } else {
      double v; __builtin_memcpy(&v, &vbits, 8);
      unsafeAtomicAdd((double*)&s.c.sum[idx], v);
    }
  }
  if (AGG & FW_AGG_MIN) {
    atomicMin((long long*)&s.c.mn[idx], (long long)min_code(VT, s.cmpto, vbits));
  }
  if (AGG & FW_AGG_MAX) {
    atomicMax((long long*)&s.c.mx[idx], (long long)max_code(VT, s.cmpto, vbits));
  }
  if (AGG & FW_AGG_COUNT) atomicAdd((unsigned long long*)&s.c.cnt[idx], 1ull);
  if (COLS_ONLY) return false;
  if (FIRST) {
    // first arrival = min ordinal; values only decrease within a kernel, so a stale load that is
    // already below our ordinal proves we are not first
    int64_t cur = s.c.first[idx];
    if (ord < cur) return atomicMin((long long*)&s.c.first[idx], (long long)ord) == INT64_MAX;
  } else {
    if (s.c.present[idx] == 0) s.c.present[idx] = 1;
  }
  return false;
}

struct BatchIn {
  const int64_t* key;
  const int32_t* key_hash;
  const int64_t* ts;
  const int64_t* val;   // int64 or double bits
  int64_t n;
  int64_t ord_base;     // arrival ordinal of record 0
  int64_t wm;           // current watermark
  // per-element fire list (allowed lateness > 0)
  unsigned long long* late_key;   // (pane id << idx_bits) | idx
  unsigned long long* late_count;
  int64_t late_capacity;
  int32_t idx_bits;
  // direct form, maxBy / minBy: every accepted record, (pane id << idx_bits) | idx, folded per pane in arrival
  // order after the launch (the late path's sort, segmented scan and commit, without fires)
  unsigned long long* by_key;
  unsigned long long* by_count;
  int64_t by_capacity;
  // sliding windows: one fire element per (record, window in its lateness period past maxTimestamp)
  unsigned long long* fire_key;   // (window pane id << idx_bits) | idx, window pane = floor_mod(n, P) * stride + kid
  unsigned long long* fire_count;
  int64_t fire_capacity;
  // direct form with first arrival: panes created by the batch, for the f1 fix-up
  int64_t* new_list;
  unsigned long long* new_count;
  int64_t new_capacity;
  // sliding: records with the assigner's extra window (entries of QK_WORDS: key, window number, value,
  // ordinal, f1), applied to the window panes before the next firing watermark (k_quirk_apply)
  int64_t* quirk;
  unsigned long long* quirk_count;
  int64_t quirk_capacity;
  const int64_t* f1;   // the batch's f1 column (the quirk entries carry their f1; NULL = the timestamp)
};
constexpr int QK_WORDS = 5;

// a record's extra sliding window (RecWin.quirk): late -> counted; already fired -> a per-element fire of
// a window pane (not implemented: FW_ERR_UNSUPPORTED); else listed for k_quirk_apply
__device__ __forceinline__ void quirk_record(const Spec& s, const BatchIn& b, int64_t key, int64_t i, int64_t qn, bool q_late,
                                          bool q_fire) {
  if (q_late) { atomicAdd(&s.stats[ST_LATE], 1ull); return; }
  if (q_fire || s.by) { set_error(s.err, FW_ERR_UNSUPPORTED); return; }
  const unsigned long long pos = atomicAdd(b.quirk_count, 1ull);
  if ((int64_t)pos >= b.quirk_capacity) { cap_error(s, 22); return; }
  int64_t* q = b.quirk + (int64_t)pos * QK_WORDS;
  q[0] = key;
  q[1] = qn;
  q[2] = b.val[i];
  q[3] = b.ord_base + i;
  q[4] = b.f1 ? b.f1[i] : b.ts[i];
  atomicAdd(&s.stats[ST_QUIRK], 1ull);
}

__device__ __forceinline__ int64_t window_start_n(const Spec& s, int64_t n) {
  return jadd(s.offset, (int64_t)((uint64_t)n * (uint64_t)(s.assigner == FW_TUMBLING ? s.size : s.slide)));
}

// a record whose slice belongs to a window in its allowed lateness past its maxTimestamp (EventTimeTrigger
// .onElement FIRE, EventTimeTrigger.java:38-40; WindowOperator.java:317-325): its slice update joins the
// commit list (applied in arrival order by k_late_commit); for sliding windows every such window of the
// record also gets a fire element (tumbling: the slice is the window, the commit list serves as both)
__device__ __forceinline__ void late_append_at(const Spec& s, const BatchIn& b, unsigned long long pos, int32_t p, int64_t kid, int64_t m,
                               int64_t i) {
  const unsigned long long pane = (unsigned long long)p * (unsigned long long)s.stride + (unsigned long long)kid;
  if ((int64_t)pos < b.late_capacity) b.late_key[pos] = (pane << b.idx_bits) | (unsigned long long)i;
  else cap_error(s, 1);
  if (s.assigner != FW_SLIDING) return;
  const int64_t n_hi = floor_div(m, s.R), n_lo = floor_div(m - s.K, s.R) + 1;
  for (int64_t n = n_lo; n <= n_hi; ++n) {
    const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
    if (max_ts > b.wm || cleanup_time(max_ts, s.lateness) <= b.wm) continue;   // not fired yet / late (dropped)
    const unsigned long long wpane = (unsigned long long)floor_mod(n, s.P) * (unsigned long long)s.stride + (unsigned long long)kid;
    const unsigned long long fpos = atomicAdd(b.fire_count, 1ull);
    if ((int64_t)fpos < b.fire_capacity) b.fire_key[fpos] = (wpane << b.idx_bits) | (unsigned long long)i;
    else cap_error(s, 2);
  }
}
__device__ void late_append(const Spec& s, const BatchIn& b, int32_t p, int64_t kid, int64_t m, int64_t i) {
  late_append_at(s, b, atomicAdd(b.late_count, 1ull), p, kid, m, i);
}

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(BLOCK) void k_ingest_direct(Spec s, BatchIn b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t c_m = INT64_MIN;   // per-wave cache of the last slice -> slot lookup
  int32_t c_p = -1;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < b.n; i0 += stride) {
    int64_t i = i0 + threadIdx.x;
    bool valid = i < b.n;
    int64_t key = 0, ts = 0, v = 0;
    int32_t h = 0;
    if (valid) {
      key = b.key[i];
      ts = b.ts[i];
      v = b.val[i];
      h = b.key_hash ? b.key_hash[i] : long_hash_code(key);
    }
    bool ok = valid;
    if (ok && ts == INT64_MIN) { set_error(s.err, FW_ERR_NO_TIMESTAMP); ok = false; }
    if (ok) {
      int32_t kg = record_key_group(s, h);   // AbstractKeyedStateBackend.setCurrentKey :167-170
      if (kg < s.kg_start || kg > s.kg_end) { set_error(s.err, FW_ERR_KEY_GROUP); ok = false; }
    }
    RecWin w;
    w.m = 0; w.n_late = 0; w.n_fire = 0; w.n_windows = 0; w.quirk = false;
    if (ok) {
      w = record_windows(s, ts, b.wm);
      if (w.quirk) quirk_record(s, b, key, i, w.qn, w.q_late, w.q_fire);
    }
    // late statistics: (record, window) pairs dropped (wave-uniform reduction)
    {
      unsigned long long late = ok ? (unsigned long long)w.n_late : 0ull;
      if (__any(late != 0)) {
        for (int off = 32; off > 0; off >>= 1) late += __shfl_xor(late, off);
        if ((threadIdx.x & 63) == 0) atomicAdd(&s.stats[ST_LATE], late);
      }
    }
    bool live = ok && (w.n_windows - w.n_late) > 0;
    bool late_fire = live && w.n_fire > 0;          // tumbling only (sliding + lateness rejected at create)
    // slice slot: wave-uniform fast path (in-order streams keep a wave inside one slice)
    const uint64_t lm = __ballot(live);
    const int leader = lm ? __ffsll((long long)lm) - 1 : 0;
    const int64_t m0 = __shfl(w.m, leader);
    const bool uniform = __all(!live || w.m == m0);
    int32_t p = -1;
    if (uniform) {
      if (lm != 0 && m0 != c_m) {   // wave-uniform: resolve once per slice change
        int32_t p0 = -1;
        if ((int)(threadIdx.x & 63) == leader) p0 = slice_slot(s, m0);
        c_p = __shfl(p0, leader);
        c_m = c_p >= 0 ? m0 : INT64_MIN;
      }
      p = live ? c_p : -1;
    } else if (live) {
      p = slice_slot(s, w.m);
    }
    if (live && p < 0) { cap_error(s, 3); live = false; }
    int64_t kid = -1;
    if (live) {
      kid = dir_find_or_insert(s, key);
      if (kid < 0) { cap_error(s, 4); live = false; }
    }
    if (b.late_key && live && late_fire) {
      late_append(s, b, p, kid, w.m, i);
      live = false;
    }
    int64_t idx = 0;
    constexpr bool BY = (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;
    if (BY && live) {
      // maxBy / minBy: the extremal record, a tie to the earlier (or later) arrival — an order atomics do not
      // give; the record is listed and folded in arrival order per pane after the launch
      idx = (int64_t)p * s.stride + kid;
      const unsigned long long pos = atomicAdd(b.by_count, 1ull);
      if ((int64_t)pos < b.by_capacity) b.by_key[pos] = ((unsigned long long)idx << b.idx_bits) | (unsigned long long)i;
      else cap_error(s, 23);
      b.new_list[i] = -1;
    } else if (live) {
      idx = (int64_t)p * s.stride + kid;
      if (FIRST) {
        (void)pane_update<VT, AGG, false, true>(s, idx, v, 0);   // the reduce columns
        // first arrival = min ordinal (values only decrease within a kernel, so a stale load already below
        // this record's ordinal proves it is not first).  The record that creates the pane stores its f1 at
        // once; a record that lowers an existing ordinal is listed by record index (the slot list[i], no
        // shared counter) and k_fix_first_f1 stores the f1 of the pane's final first arrival after the launch
        const int64_t ord = b.ord_base + i;
        int64_t fi = -1;
        if (ord < s.c.first[idx]) {
          const int64_t old = (int64_t)atomicMin((long long*)&s.c.first[idx], (long long)ord);
          if (old == INT64_MAX) s.c.f1v[idx] = b.f1 ? b.f1[i] : ts;
          else if (old > ord) fi = idx;
        }
        b.new_list[i] = fi;
      } else {
        (void)pane_update<VT, AGG, false>(s, idx, v, b.ord_base + i);
      }
    } else if (FIRST && valid) {
      b.new_list[i] = -1;
    }
  }
}

// after the direct ingest: the panes whose first-arrival ordinal a record lowered after another record of
// the batch created them (list[j] = the pane, or -1): the record that is the pane's first arrival now
// stores its f1 (one writer per pane, ordered after the creator's store by the launch boundary)
__global__ __launch_bounds__(BLOCK) void k_fix_first_f1(Spec s, const int64_t* list, const int64_t* f1col,
                                                       int64_t ord_base, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = list[j];
    if (idx < 0) continue;
    if (s.c.first[idx] == ord_base + j) s.c.f1v[idx] = f1col[j];
  }
}

// after a batch's ingest, while restored windows are disarmed and ahead of the watermark: each record of such a
// window re-arms its pane's trigger timer (EventTimeTrigger.onElement registers maxTimestamp while the
// watermark is below it; the window then fires at its maxTimestamp with everything the pane holds)
// (sliding: each of the record's windows whose own pane is disarmed, by window-pane slot)
__global__ __launch_bounds__(BLOCK) void k_arm(Spec s, BatchIn b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ts = b.ts[i];
    if (ts == INT64_MIN) continue;
    if (s.assigner == FW_SLIDING) {
      const int64_t m = record_windows(s, ts, b.wm).m;
      const int64_t n_hi = floor_div(m, s.R), n_lo = floor_div(m - s.K, s.R) + 1;
      int64_t kid = -2;
      for (int64_t n = n_lo; n <= n_hi; ++n) {
        const int32_t w = (int32_t)floor_mod(n, s.W);
        if (!s.disarm[w] || s.wtag[w] != n) continue;
        if (jsub(jadd(window_start_n(s, n), s.size), 1) <= b.wm) continue;
        if (kid == -2) kid = dir_lookup(s, b.key[i]);
        if (kid >= 0) s.armed[(int64_t)w * s.stride + kid] = 1;
      }
      continue;
    }
    const int64_t m = floor_div(jsub(ts, s.offset), s.size);   // tumbling: the slice is the window
    const int32_t p = (int32_t)floor_mod(m, s.P);
    if (!s.disarm[p] || s.slice_tag[p] != m) continue;
    const int64_t max_ts = jsub(jadd(window_start_n(s, m), s.size), 1);
    if (max_ts <= b.wm) continue;
    const int64_t kid = dir_lookup(s, b.key[i]);
    if (kid >= 0) s.armed[(int64_t)p * s.stride + kid] = 1;
  }
}

// a wave-uniform 64-bit value moved to scalar registers
__device__ __forceinline__ int64_t uniform64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// ------------------------------------------------------------------------------------------------
// ingest, partitioned form.  Two kernels per batch:
//  k_route      one workgroup per tile of RT_TILE records: streams the tile's columns in with 16-B
//               loads, does the per-record operator work (key group check, window/slice, lateness),
//               counting-sorts the routable records through LDS by bin = (tile slice q, directory
//               bucket) and writes the tile back bin-sorted as (fmix64(key), value) + the 2-B index of
//               the record in its tile, with a per-tile table of segment starts.  Records that cannot be
//               routed by slice (slices beyond the tile's RT_Q, the Long.MIN_VALUE key) and per-element
//               fires go to two more bin groups per bucket, so each bucket's workgroup finds its own.
//  k_aggregate  one workgroup per directory bucket: owns every pane of that bucket for this batch,
//               gathers the bucket's segment from every tile (the segments concatenated, one record
//               per lane), resolves keys in an LDS copy of the bucket's directory slice, reduces with
//               LDS atomics, adds the bucket's direct records the same way and folds each touched pane
//               into the dense columns once, with plain loads and stores (it is their only writer).
// No device-scope atomic per record.  (A variant that resolved the directory slot in k_route and routed
// 12-B records measured slower: the per-record probe of the global directory cost k_route more than the
// 6 B/event it saved)
// ------------------------------------------------------------------------------------------------
#ifndef FW_NBUF
#define FW_NBUF 3   // routed-batch buffer sets (fw_engine::NBUF)
#endif
#ifndef FW_AGG_UNCOND
#define FW_AGG_UNCOND 1   // k_aggregate: the next group's loads issued without a branch (A/B switch)
#endif
#ifndef FW_RT_TILE_LOG
#define FW_RT_TILE_LOG 12
#endif
constexpr int RT_TILE = 1 << FW_RT_TILE_LOG;  // records per k_route tile
constexpr int RT_THREADS = RT_TILE / 8;      // eight records per thread
constexpr int RT_Q = 2;                 // slices per tile routed through LDS (more go to the direct list)
constexpr int RT_GS = 64;               // distinct slices per batch (k_aggregate rounds)
constexpr int RT_MAXNB = 256;           // directory buckets the route table holds
constexpr int FLAG_RING = 16;           // direct-record flags, one per batch in flight
constexpr int RT_GROUPS = RT_Q + 2;     // bin groups per bucket: RT_Q routed slices, then the direct records
                                        // (any other slice, the Long.MIN_VALUE key) and the per-element fires
constexpr int AG_THREADS = 1024;
#ifndef FW_AG_WIN
#define FW_AG_WIN 8
#endif
constexpr int AG_WIN = FW_AG_WIN;       // k_aggregate: directory slots probed without a branch
constexpr int AG_CHS = 1024;            // k_aggregate wave steps (64 records each) tabulated per chunk
constexpr int AG_LOOK = 8;              // k_aggregate: segment ends a lane compares per step (independent reads)
constexpr int AG_MAXPER = 17;           // k_aggregate segment-offset scan: ntiles + 1 <= 17 * AG_THREADS
constexpr int AG_SPLIT_MAX = 31;        // k_aggregate: shares a hot bucket is split into, at most 
#ifndef FW_AGG_SPLIT_INT
#define FW_AGG_SPLIT_INT 31
#endif
constexpr int AG_SPLIT_CHAIN = 16;      // ... when its shares fold one after another (double sums, maxBy / minBy)
constexpr uint32_t AG_SPLIT_MIN = 16384; // ... and routed records per share, at least
constexpr int RT_MAX_KB_BITS = 12;      // directory slots per bucket that k_aggregate holds in LDS
constexpr int IDX_BITS = FW_RT_TILE_LOG; // record index within a tile
constexpr uint32_t NO_FIRST = 0xFFFFFFFFu;

struct RouteBuf {
  longlong2* kv;         // [ntiles][RT_TILE] routed records (fmix64(key), value), each tile sorted by bin
  uint16_t* idx;         // [ntiles][RT_TILE] record index within its tile (first arrival)
  uint32_t* seg;         // [RT_GROUPS * nb][seg_stride] bucket-major: row (group, bucket), one word per tile: the
                         // segment's start | end << 16 in the tile (written for the tile's live groups only)
  int64_t seg_stride;    // tiles per row (max_tiles)
  int64_t* hdr;          // [ntiles][RT_Q] slice number of the tile's routed bin group q (FREE_TAG = unused)
  uint32_t* tdir;        // [ntiles] the tile has direct-group records (its direct / fire rows are written)
  // hot buckets split over helper workgroups (k_aggregate): per-bucket routed records of the previous /
  // this / a retired batch (ring), the serialised-fold flags, the helpers launched, the batch tag
  unsigned int* bload_prev;
  unsigned int* bload_cur;
  unsigned int* bload_zero;
  unsigned int* fold_flag;        // [RT_MAXNB][RT_GS] (tag << 5) | shares folded
  unsigned int* fold_cnt;         // [RT_MAXNB][RT_GS] shares folded concurrently (integer variants): this batch's
  unsigned int* fold_cnt_zero;    // ring entry, and the one of the batch after next that the owners clear
  unsigned int* bload_host;       // host-mapped [RT_MAXNB]: each owner's estimate of its bucket's routed records
  int32_t helpers;
  int32_t split_max;     // shares per hot bucket, at most (<= AG_SPLIT_MAX)
  int32_t chunk_pct;     // a share's records: at least this percentage of the mean bucket load
  uint32_t tag;
  int64_t* dm;           // [tiles x RT_TILE] slice number of each direct-group record (at its routed position)
  unsigned int* dflag;   // set by a tile with direct-group records (a ring of FLAG_RING words, one per batch)
  unsigned int* dflag_reset;   // the word of batch j + FLAG_RING/2: zeroed by k_aggregate of batch j
  long long* stamps;     // diagnostics (FW_DEBUG_AGG & 16): per-workgroup phase timestamps, 8 per workgroup
  int32_t ntiles;
  int32_t dbg;
};

// Non-temporal access of the streamed columns, a bit mask: 1 = k_route's input loads (on: k_route 43 ->
// 41 us per 4 Mi-event batch), 2 = k_aggregate's gathers of the routed records, 4 = k_route's stores of
// them (both measured slower: the intermediate is re-read from the cache)
#ifndef FW_ROUTE_NT
#define FW_ROUTE_NT 1
#endif
#define FW_STAMP(r, base, k) do { if ((r).stamps && threadIdx.x == 0) (r).stamps[(base) + (int64_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define RT_STAMP(k) do { if (r.stamps && threadIdx.x == 0) r.stamps[(int64_t)tile * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// tile-local slice set in LDS (RT_Q entries): index of slice m, inserting it if new; -1 when full
__device__ __forceinline__ int32_t tile_slice(int64_t* lset, int64_t m) {
  for (int q = 0; q < RT_Q; ++q) {
    const int64_t cur = lset[q];
    if (cur == m) return q;
    if (cur == FREE_TAG) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&lset[q], (unsigned long long)FREE_TAG,
                                                (unsigned long long)m);
      if ((int64_t)prev == FREE_TAG || (int64_t)prev == m) return q;
    }
  }
  return -1;
}

// exclusive scan of a[0..n) in place (n <= MAXPER * blockDim.x), contiguous chunks per thread
template <int NT, int MAXPER = 8>
__device__ __forceinline__ void block_scan_excl(int32_t* a, int n, int32_t* wtot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = (n + NT - 1) / NT;
  int32_t loc[MAXPER];
  int32_t sum = 0;
  for (int i = 0; i < per; ++i) {
    const int x = threadIdx.x * per + i;
    loc[i] = x < n ? a[x] : 0;
    sum += loc[i];
  }
  int32_t incl = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wtot[wave] = incl;
  __syncthreads();
  int32_t run = incl - sum;
  for (int w = 0; w < wave; ++w) run += wtot[w];
  for (int i = 0; i < per; ++i) {
    const int x = threadIdx.x * per + i;
    if (x < n) a[x] = run;
    run += loc[i];
  }
  __syncthreads();
}

// LDS layout of k_route (bytes): [0, 64K) staging of the bin-sorted records (fmix64(key), value); before
// the scatter the same bytes hold, entry by entry of the thread owning the record (no barrier needed):
// the key hashes int32[RT_TILE] at 0 (optional column), and for records outside their wave's reference
// slice their slice numbers int64[RT_TILE] at 4 RT_TILE and flags int32[RT_TILE] at 12 RT_TILE.  Then the
// sorted records' index in the tile (uint16[RT_TILE]), the bin counters, the scan scratch and the tile's
// slice set.
constexpr size_t RT_LDS = (size_t)RT_TILE * (16 + 2) + 4 * (size_t)(RT_GROUPS * RT_MAXNB + 8) + 4 * 16 + 8 * RT_Q + 8;

// TAIL: the batch's last, partial tile.  A separate instantiation (round 6): with one code path for both, the whole
// tiles' 16-B loads followed a join with the tail's loads, and the compiler's waits for the join made each whole tile
// wait for its first loads before issuing the rest
template <int VT, int AGG, bool FIRST, bool TAIL>
__device__ __forceinline__ void route_tile(const Spec& s, const RouteSpec& rq, const BatchIn& b, const RouteBuf& r,
                                           unsigned char* smem, const int tile) {
  constexpr bool tail = TAIL;
  constexpr int NT = RT_THREADS;
  constexpr int PER = RT_TILE / NT;     // records per thread
  constexpr int V = PER / 2;            // 16-B vectors per column per thread
  const int nbq = RT_GROUPS * rq.nb;
  longlong2* st_kv = (longlong2*)smem;
  uint16_t* st_idx = (uint16_t*)(st_kv + RT_TILE);
  int32_t* cnt = (int32_t*)(st_idx + RT_TILE);     // [nbq + 1]
  int32_t* wtot = cnt + (RT_GROUPS * RT_MAXNB + 8); // [NT / 64]
  int64_t* lset = (int64_t*)(wtot + 16);           // [RT_Q] the tile's routed slices
  int32_t* any_direct = (int32_t*)(lset + RT_Q);   // the tile has direct-group records
  int32_t* lhash = (int32_t*)smem;                 // Java key hashes (optional column)
  const int64_t base = (int64_t)tile * RT_TILE;
  RT_STAMP(0);
  for (int x = threadIdx.x; x <= nbq; x += NT) cnt[x] = 0;
  if (threadIdx.x < RT_Q) lset[threadIdx.x] = FREE_TAG;
  if (threadIdx.x == 0) *any_direct = 0;
  // phase A: every load of the tile in flight before any dependent work; record (j, e) of this thread
  // is tile index 2 * (j * NT + tid) + e
  // (the tail test is hoisted out of the loads and the optional key-hash column is loaded after them: a branch
  // between two vectors' loads made the compiler wait for most earlier loads before issuing the next, round 6)
  int64_t kk[PER], tt[PER], vv[PER];
  if (!tail) {   // uniform
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int64_t i = base + 2 * (j * NT + (int)threadIdx.x);
#if FW_ROUTE_NT & 1
      // streamed once per batch: non-temporal, so the routed intermediate k_aggregate reads next keeps the cache
      typedef long long v2i64 __attribute__((ext_vector_type(2)));
      const v2i64 a = __builtin_nontemporal_load((const v2i64*)(b.key + i));
      const v2i64 c = __builtin_nontemporal_load((const v2i64*)(b.ts + i));
      const v2i64 d = __builtin_nontemporal_load((const v2i64*)(b.val + i));
#else
      const longlong2 a = *(const longlong2*)(b.key + i);
      const longlong2 c = *(const longlong2*)(b.ts + i);
      const longlong2 d = *(const longlong2*)(b.val + i);
#endif
      kk[2 * j] = a.x; kk[2 * j + 1] = a.y;
      tt[2 * j] = c.x; tt[2 * j + 1] = c.y;
      vv[2 * j] = d.x; vv[2 * j + 1] = d.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int64_t i = base + 2 * (j * NT + (int)threadIdx.x);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int64_t ie = min(i + e, b.n - 1);
        kk[2 * j + e] = b.key[ie];
        tt[2 * j + e] = b.ts[ie];
        vv[2 * j + e] = b.val[ie];
      }
    }
  }
  if (b.key_hash) {   // uniform: the Java key hashes (optional column)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int64_t i = base + 2 * (j * NT + (int)threadIdx.x);
      if (!tail) *(int2*)(lhash + (i - base)) = *(const int2*)(b.key_hash + i);
      else
        for (int e = 0; e < 2; ++e) lhash[i + e - base] = b.key_hash[min(i + e, b.n - 1)];
    }
  }
  __syncthreads();   // cnt and lset initialised
  RT_STAMP(1);
  // phase B1: per record operator work (timestamp, key group, windows, lateness) — pure ALU; the slice
  // number replaces the timestamp in tt[]
  unsigned long long late_pairs = 0;
  uint32_t route_mask = 0, direct_mask = 0, fire_mask = 0;
  // the wave's reference slice: assignment of its first record, valid for every record whose timestamp
  // lies in the same slice (a wave of an in-order stream nearly always does); the others take the
  // full per-record path.  Bounded away from the int64 edges so no wrap happens inside the range.
  // a subtask owning every key group cannot see a foreign key: skip the murmur range check
  const bool all_kg = rq.kg_start == 0 && rq.kg_end == rq.mp - 1;
  uint32_t slow_mask = 0;   // records outside the wave's reference slice
  bool e_ts = false, e_kg = false;   // errors, reported once after the loop (no atomics inside it)
  {
  RecWin w0;
  w0.m = 0; w0.n_late = 0; w0.n_fire = 0; w0.n_windows = 0; w0.quirk = false; w0.lo = 1; w0.hi = 0;
  {
    const int64_t i0 = base + 2 * (int)threadIdx.x;
    const bool c0 = (!tail || i0 < b.n) && tt[0] > -(1LL << 61) && tt[0] < (1LL << 61);
    const uint64_t cm = __ballot(c0);
    if (cm && rq.size < (1LL << 60)) {
      const int64_t ts0 = uniform64(__shfl(tt[0], __ffsll((long long)cm) - 1));
      w0 = record_windows<true>(rq, ts0, b.wm);   // (inline: a call here made the whole kernel keep the calling convention)
      w0.m = uniform64(w0.m); w0.lo = uniform64(w0.lo); w0.hi = uniform64(w0.hi);
      w0.n_late = __builtin_amdgcn_readfirstlane(w0.n_late);
      w0.n_fire = __builtin_amdgcn_readfirstlane(w0.n_fire);
      w0.n_windows = __builtin_amdgcn_readfirstlane(w0.n_windows);
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int64_t i = base + 2 * ((k >> 1) * NT + (int)threadIdx.x) + (k & 1);
    const bool valid = !tail || i < b.n;
    const int64_t key = kk[k], ts = tt[k];
    bool ok = valid;
    if (ok && ts == INT64_MIN) { e_ts = true; ok = false; }
    if (ok && !all_kg) {
      const int32_t h = b.key_hash ? lhash[i - base] : long_hash_code(key);
      const int32_t kg = record_key_group(rq, h);   // AbstractKeyedStateBackend.setCurrentKey :167-170
      if (kg < rq.kg_start || kg > rq.kg_end) { e_kg = true; ok = false; }
    }
    const bool fast = ok && ts >= w0.lo && ts <= w0.hi;
    slow_mask |= (ok && !fast ? 1u : 0u) << k;
    if (fast) late_pairs += (unsigned long long)w0.n_late;
    const bool live = fast && (w0.n_windows - w0.n_late) > 0;
    const bool late_fire = live && w0.n_fire > 0;
    // routable: its windows neither late nor fired yet, so no watermark up to b.wm fires or purges its slice
    const bool routable = live && !late_fire && key != EMPTY_KEY;
    route_mask |= (routable ? 1u : 0u) << k;
    direct_mask |= (live && !routable ? 1u : 0u) << k;
    fire_mask |= (late_fire ? 1u : 0u) << k;
    tt[k] = w0.m;
  }
  }
  if (__any(e_ts || e_kg)) {
    if (e_ts) set_error(rq.err, FW_ERR_NO_TIMESTAMP);
    if (e_kg) set_error(rq.err, FW_ERR_KEY_GROUP);
  }
  // the full assignment for the rest: one call-free copy of the code (a call would make the register
  // allocator spill the tile around it), timestamps re-read from the input, results through LDS
  RT_STAMP(5);
  if (__any(slow_mask != 0)) {
    int64_t* sm = (int64_t*)(smem + (size_t)RT_TILE * 4);        // [RT_TILE] slice numbers
    int32_t* sf = (int32_t*)(smem + (size_t)RT_TILE * 12);       // [RT_TILE] flags: live | late_fire << 1 | n_late << 2
#pragma unroll 1
    for (int k = 0; k < PER; ++k) {
      if ((slow_mask >> k) & 1u) {
        const int32_t t = 2 * ((k >> 1) * NT + (int)threadIdx.x) + (k & 1);
        const int64_t ts = b.ts[base + t];
        const RecWin w = record_windows<true>(rq, ts, b.wm);
        if (w.quirk) quirk_record(s, b, kk[k], base + t, w.qn, w.q_late, w.q_fire);
        const bool live = (w.n_windows - w.n_late) > 0;
        const int32_t f = (live ? 1 : 0) | (live && w.n_fire > 0 ? 2 : 0) | (w.n_late << 2);
        sm[t] = w.m;
        sf[t] = f;
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if ((slow_mask >> k) & 1u) {
        const int32_t t = 2 * ((k >> 1) * NT + (int)threadIdx.x) + (k & 1);
        const int32_t f = sf[t];
        late_pairs += (unsigned long long)(f >> 2);
        const bool live = f & 1, late_fire = (f & 2) != 0;
        const bool routable = live && !late_fire && kk[k] != EMPTY_KEY;
        route_mask |= (routable ? 1u : 0u) << k;
        direct_mask |= (live && !routable ? 1u : 0u) << k;
        fire_mask |= (late_fire ? 1u : 0u) << k;
        tt[k] = sm[t];
      }
    }
  }
  // phase B2: the routed records' index in the tile's slice set — resolved once per wave when all its
  // routed records share one slice (an in-order stream), per record otherwise — then their bin and
  // counting-sort rank.  The rest (rare: per-element fires, slices beyond the tile's RT_Q, the
  // Long.MIN_VALUE key, bucket 0) take the bucket's direct or fire bin group, which the k_aggregate
  // workgroup owning the bucket applies.
  RT_STAMP(6);
  int64_t m_ref = INT64_MIN;
  {
    const uint64_t lm = __ballot(route_mask != 0);
    if (lm) {
      const int leader = __ffsll((long long)lm) - 1;
      int64_t mine = INT64_MIN;
#pragma unroll
      for (int k = PER - 1; k >= 0; --k) if ((route_mask >> k) & 1u) mine = tt[k];
      m_ref = __shfl(mine, leader);
    }
  }
  bool same = true;
#pragma unroll
  for (int k = 0; k < PER; ++k) same &= !((route_mask >> k) & 1u) || tt[k] == m_ref;
  int32_t q_ref = -1;
  if (__all(same)) {
    if (m_ref != INT64_MIN && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)__ballot(route_mask != 0)) - 1))
      q_ref = tile_slice(lset, m_ref);
    q_ref = __shfl(q_ref, __ffsll((long long)__ballot(route_mask != 0)) - 1);
  }
  const bool wave_uniform = __all(same);
  int32_t bin[PER];       // routed bin, or -1
  int32_t rank[PER];
  // (tt[k] keeps the slice number of a direct record for the store below: k_aggregate reads it from
  // r.dm instead of re-running the window assignment)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    bin[k] = -1;
    rank[k] = 0;
    const bool routable = (route_mask >> k) & 1u;
    int32_t q = -1;
    if (wave_uniform) q = routable ? q_ref : -1;
    else if (routable) q = tile_slice(lset, tt[k]);
    if (routable && q < 0) direct_mask |= 1u << k;   // the tile's slice set is full
    const bool direct = (direct_mask >> k) & 1u;
    if (q >= 0 || direct) {
      // routed and direct records carry the directory hash (a bijection of the key; EMPTY_H is the
      // Long.MIN_VALUE key's, which lives in bucket 0)
      const bool kmin = kk[k] == EMPTY_KEY;
      const uint64_t hk = fmix64((uint64_t)kk[k]);
      const int32_t bkt = kmin ? 0 : (int32_t)((hk & rq.dir_mask) >> rq.kb_bits);
      const int32_t g = q >= 0 ? q : RT_Q + (int32_t)((fire_mask >> k) & 1u);
      bin[k] = g * rq.nb + bkt;
      rank[k] = atomicAdd(&cnt[bin[k]], 1);
      kk[k] = (int64_t)hk;
    }
  }
  RT_STAMP(7);
  if (__any(late_pairs != 0)) {
    for (int off = 32; off > 0; off >>= 1) late_pairs += __shfl_xor(late_pairs, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(&rq.stats[ST_LATE], late_pairs);
  }
  if (direct_mask != 0) *any_direct = 1;
  __syncthreads();   // every wave's slice claims are in lset, every staging read is done
  const bool tile_direct = *any_direct != 0;
  if (threadIdx.x == 0) {
    if (tile_direct) atomicOr(r.dflag, 1u);
    r.tdir[tile] = tile_direct ? 1u : 0u;
  }
  if (threadIdx.x < RT_Q) r.hdr[(int64_t)tile * RT_Q + threadIdx.x] = lset[threadIdx.x];   // routed slices
  RT_STAMP(2);
  // bins past the tile's last live group hold nothing, so the scan covers the live groups only (an in-order stream:
  // one group of nb bins); the tile's routed slices claimed lset's entries in order (a prefix)
  int nlive = tile_direct ? RT_GROUPS : 0;
  if (!tile_direct)
    for (int q = 0; q < RT_Q; ++q) nlive = lset[q] != FREE_TAG ? q + 1 : nlive;
  const int nlb = nlive * rq.nb;
  block_scan_excl<NT>(cnt, nlb + 1, wtot);   // cnt[nlb] = routed records of the tile
  // the segment table, bucket-major (row (group, bucket) holds one word per tile: start | end << 16), so that the
  // k_aggregate workgroup owning a bucket reads its rows contiguously; only the tile's live groups are written
  // (its routed slices, and the direct / fire groups when it has direct records), k_aggregate reads no other
  for (int x = threadIdx.x; x < nlb; x += NT) {
    const int g = x / rq.nb;
    const bool live = g < RT_Q ? lset[g] != FREE_TAG : tile_direct;
    if (live) r.seg[(int64_t)x * r.seg_stride + tile] = (uint32_t)cnt[x] | ((uint32_t)cnt[x + 1] << 16);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (bin[k] >= 0) {
      const int32_t pos = cnt[bin[k]] + rank[k];
      st_kv[pos] = make_longlong2(kk[k], vv[k]);
      if ((direct_mask >> k) & 1u) r.dm[base + pos] = tt[k];
      st_idx[pos] = (uint16_t)(2 * ((k >> 1) * NT + (int)threadIdx.x) + (k & 1));
    }
  }
  __syncthreads();
  RT_STAMP(3);
  const int32_t total = cnt[nlb];
#pragma unroll 2
  for (int k = 0; k < PER; ++k) {
    const int32_t pos = k * NT + (int)threadIdx.x;
    if (pos < total) r.kv[base + pos] = st_kv[pos];
  }
  // the record indices: first arrival (FIRST), and the batch index of every direct record
  if (FIRST || *any_direct) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int32_t pos = 2 * (j * NT + (int)threadIdx.x);
      if (pos < total) *(uint32_t*)(r.idx + base + pos) = *(const uint32_t*)(st_idx + pos);
    }
  }
  RT_STAMP(4);
}

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(RT_THREADS, 4) void k_route(const Spec* __restrict__ sd, RouteSpec rq, BatchIn b, RouteBuf r) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Spec& s = *sd;   // device copy (kernel arguments by value are held in scalar registers from entry)
  // every tile but the last is whole, so its 16-B loads need no bounds (uniform branch)
  // one tile per workgroup (a persistent form, two workgroups per CU looping over the tiles with the second half
  // started late so that one's compute phase falls beside the other's memory phases, measured no faster and
  // spilled: round 5)
  const int tile = (int)blockIdx.x;
  if ((int64_t)(tile + 1) * RT_TILE > b.n) route_tile<VT, AGG, FIRST, true>(s, rq, b, r, smem, tile);   // uniform
  else route_tile<VT, AGG, FIRST, false>(s, rq, b, r, smem, tile);
}

// the bucket's LDS directory-hash table: slot of h, inserting its key (fmix64_inv(h)) into the global
// directory if absent (the same linear probe sequence as dir_find_or_insert).  Out of line: taken by a
// wave only when a lane misses the probed windows.
__device__ __forceinline__ int32_t agg_probe_insert_body(uint64_t* lh, int64_t* dir_keys, uint32_t kbm, uint64_t h,
                                                        unsigned long long* inserted) {
  uint32_t x = (uint32_t)h & kbm;
  for (uint32_t probe = 0; probe <= kbm; ++probe) {
    const uint64_t cur = lh[x];
    if (cur == h) return (int32_t)x;
    if (cur == EMPTY_H) {
      const int64_t key = (int64_t)fmix64_inv(h);
      const unsigned long long prev = atomicCAS((unsigned long long*)&dir_keys[x], (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)key);
      if ((int64_t)prev == EMPTY_KEY) atomicAdd(inserted, 1ull);
      const uint64_t now = (int64_t)prev == EMPTY_KEY ? h : fmix64(prev);
      lh[x] = now;   // only globally confirmed keys enter the cache
      if (now == h) return (int32_t)x;
    }
    x = (x + 1) & kbm;
  }
  return -1;
}
__device__ __noinline__ int32_t agg_probe_insert(uint64_t* lh, int64_t* dir_keys, uint32_t kbm, uint64_t h,
                                                 unsigned long long* inserted) {
  return agg_probe_insert_body(lh, dir_keys, kbm, h, inserted);
}

// the bucket's LDS accumulators
struct AggLds {
  int64_t *sum, *mn, *mx, *cnt;
  uint32_t* first;   // earliest record of the batch (batch index): the first arrival, and the "touched" mark
  uint32_t* ord;     // maxBy / minBy: batch index of the extremal record
};

// one record into the bucket's LDS accumulators at slot kl.  maxBy / minBy take two passes over the
// records (no lock: a (value, ordinal) pair cannot be updated by one atomic): pass 0 the extremal value
// in Double.compareTo (Long) order, pass 1 among the records holding it the earliest (first) or latest
// (last) batch index — ComparableAggregator MAXBY/MINBY with the tie rule (ComparableAggregator.java:74-81)
template <int VT, int AGG>
__device__ __forceinline__ void acc_add(const AggLds& L, bool cmpto, bool by_last, int pass, uint32_t kl, int64_t v,
                                        uint32_t oi) {
  constexpr bool MAXBY = (AGG & FW_AGG_MAXBY) != 0, MINBY = (AGG & FW_AGG_MINBY) != 0;
  if (MAXBY || MINBY) {
    const int64_t code = VT == FW_VALUE_I64 ? v : f64_cmp_code(__longlong_as_double(v));
    int64_t* ext = MAXBY ? L.mx : L.mn;
    if (pass == 0) {
      if (MAXBY) atomicMax((long long*)&ext[kl], (long long)code);
      else atomicMin((long long*)&ext[kl], (long long)code);
      atomicMin(&L.first[kl], oi);
    } else if (ext[kl] == code) {
      if (by_last) atomicMax(&L.ord[kl], oi);
      else atomicMin(&L.ord[kl], oi);
    }
    return;
  }
  if (AGG & FW_AGG_SUM) {
    if (VT == FW_VALUE_I64) atomicAdd((unsigned long long*)&L.sum[kl], (unsigned long long)v);
    else unsafeAtomicAdd((double*)&L.sum[kl], __longlong_as_double(v));
  }
#if FW_AGG_PRECHECK
  // min / max / first only ever decrease (increase): a plain LDS read that already beats this record
  // proves it changes nothing, and the atomic is skipped
  if (AGG & FW_AGG_MIN) { const int64_t c = min_code(VT, cmpto, v); if (c < L.mn[kl]) atomicMin((long long*)&L.mn[kl], (long long)c); }
  if (AGG & FW_AGG_MAX) { const int64_t c = max_code(VT, cmpto, v); if (c > L.mx[kl]) atomicMax((long long*)&L.mx[kl], (long long)c); }
  if (AGG & FW_AGG_COUNT) atomicAdd((unsigned long long*)&L.cnt[kl], 1ull);
  if (oi < L.first[kl]) atomicMin(&L.first[kl], oi);   // earliest record of the batch: first arrival + "touched"
#else
  if (AGG & FW_AGG_MIN) atomicMin((long long*)&L.mn[kl], (long long)min_code(VT, cmpto, v));
  if (AGG & FW_AGG_MAX) atomicMax((long long*)&L.mx[kl], (long long)max_code(VT, cmpto, v));
  if (AGG & FW_AGG_COUNT) atomicAdd((unsigned long long*)&L.cnt[kl], 1ull);
  atomicMin(&L.first[kl], oi);   // earliest record of the batch: the first arrival, and the "touched" mark
#endif
}

// Hot keys (Zipf): when 8 or more lanes of a wave carry the slot of the wave's first active lane, they are
// reduced in registers (butterfly over the wave) and the leader makes one LDS update for all of them —
// the same-address LDS atomics of a hot key would otherwise serialise up to 64 ways.  A bucket can hold
// several hot keys (the first lane is not always the hottest), so up to HC_ROUNDS leaders are tried in
// turn, each over the lanes left.  Returns whether this lane still has its own update to make.  (Double
// sums change association: the tolerance path.)
#ifndef FW_HC_ROUNDS
#define FW_HC_ROUNDS 3
#endif
template <int VT, int AGG>
__device__ __forceinline__ bool hot_combine(const AggLds& L, bool cmpto, bool act, uint32_t kl, int64_t v, uint32_t oi,
                                            int lane) {
#pragma unroll 1
  for (int round = 0; round < FW_HC_ROUNDS; ++round) {
    const uint64_t am = __ballot(act);
    if (am == 0) return act;
    const int leader = __ffsll((long long)am) - 1;
    const uint32_t lk = __shfl(kl, leader);
    const bool same = act && kl == lk;
    const uint64_t sm = __ballot(same);
    if (__popcll(sm) < 8) return act;   // wave-uniform
    int64_t sv = same ? v : sum_identity(VT);
    int64_t mn = same ? min_code(VT, cmpto, v) : INT64_MAX;
    int64_t mx = same ? max_code(VT, cmpto, v) : INT64_MIN;
    uint32_t fo = same ? oi : NO_FIRST;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      if (AGG & FW_AGG_SUM) {
        const int64_t y = __shfl_xor(sv, o);
        if (VT == FW_VALUE_I64) sv = jadd(sv, y);
        else sv = __double_as_longlong(__longlong_as_double(sv) + __longlong_as_double(y));
      }
      if (AGG & FW_AGG_MIN) { const int64_t y = __shfl_xor(mn, o); mn = y < mn ? y : mn; }
      if (AGG & FW_AGG_MAX) { const int64_t y = __shfl_xor(mx, o); mx = y > mx ? y : mx; }
      const uint32_t y = __shfl_xor(fo, o);
      fo = y < fo ? y : fo;
    }
    if (lane == leader) {
      if (AGG & FW_AGG_SUM) {
        if (VT == FW_VALUE_I64) atomicAdd((unsigned long long*)&L.sum[lk], (unsigned long long)sv);
        else unsafeAtomicAdd((double*)&L.sum[lk], __longlong_as_double(sv));
      }
      if (AGG & FW_AGG_MIN) atomicMin((long long*)&L.mn[lk], (long long)mn);
      if (AGG & FW_AGG_MAX) atomicMax((long long*)&L.mx[lk], (long long)mx);
      if (AGG & FW_AGG_COUNT) atomicAdd((unsigned long long*)&L.cnt[lk], (unsigned long long)__popcll(sm));
      atomicMin(&L.first[lk], fo);
    }
    act = act && !same;
  }
  return act;
}

// LDS bytes k_aggregate needs for buckets of 2^kb_bits slots and ntiles tiles
__host__ __device__ constexpr size_t agg_lds_bytes(int kb_bits, int nacc, int64_t ntiles, bool by) {
  return (size_t)8 * ((size_t)1 << kb_bits) + ((size_t)(1 << kb_bits) + 65) * (8 * nacc + (by ? 4 : 0)) +
         ((((size_t)(1 << kb_bits) + 65) + 3) & ~(size_t)3) * 4 + (size_t)(8 * RT_Q + 4 * RT_GROUPS) * ntiles +
         8 * (size_t)ntiles + 4 +
         4 * (size_t)AG_CHS + 4 * (size_t)AG_LOOK + 64 + 8 + 8 * RT_GS + 8 + 4 * (size_t)(RT_MAXNB + 4);
}

// SKEW: the variant for skewed key distributions (the host launches it when the posted bucket loads ask
// for helpers): hot buckets split over helper workgroups, and the in-wave hot-key combine.  The uniform
// variant carries neither (registers: the 1024-thread workgroup has 128 VGPRs per lane)
template <int VT, int AGG, bool FIRST, bool SKEW>
__global__ __launch_bounds__(AG_THREADS) void k_aggregate(const Spec* __restrict__ sd, AggSpec sa, BatchIn b, RouteBuf r, const int64_t* f1col) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Spec& s = *sd;   // device copy (kernel arguments by value are held in scalar registers from entry)
  constexpr int NT = AG_THREADS;
  // XCD-aware bucket order: workgroups are dealt to the 8 XCDs round-robin, so XCD x runs the
  // contiguous bucket range [x * nb/8, (x + 1) * nb/8).  Neighbouring buckets' segments share the
  // 128-B lines at their boundaries; with both readers on one XCD the second read hits that XCD's L2
  // Integer variants fold a split bucket's shares without waiting on each other, so their helpers (the
  // hot buckets' shares, the longest work items) take the first block indices and start at once instead
  // of waiting for an owner's CU; vb is the block's index in the owners-then-helpers numbering
  constexpr bool HELPERS_FIRST = SKEW && VT == FW_VALUE_I64 && !(AGG & (FW_AGG_MAXBY | FW_AGG_MINBY));
  const int H = HELPERS_FIRST ? r.helpers : 0;
  const int vb = (int)blockIdx.x < H ? sa.nb + (int)blockIdx.x : (int)blockIdx.x - H;
  int owner_bkt = vb >= sa.nb ? -1
                        : (sa.nb % 8 == 0 && !(r.dbg & 32)) ? (vb % 8) * (sa.nb / 8) + vb / 8
                                                          : vb;
  const int KB = 1 << sa.kb_bits;
  const uint32_t kbm = (uint32_t)KB - 1;
  const int KA = KB + 65;                               // accumulators: KB slots, one dummy per lane, the MIN key
  const uint32_t KMIN = (uint32_t)KB + 64;              // slot of the Long.MIN_VALUE key (kid D, bucket 0)
  uint64_t* lh = (uint64_t*)smem;                       // [KB] fmix64 of this bucket's directory slice (EMPTY_H = free)
  constexpr bool MAXBY = (AGG & FW_AGG_MAXBY) != 0, MINBY = (AGG & FW_AGG_MINBY) != 0, BY = MAXBY || MINBY;
  constexpr bool HAS_MIN = (AGG & FW_AGG_MIN) || MINBY, HAS_MAX = (AGG & FW_AGG_MAX) || MAXBY;
  int64_t* lsum = (int64_t*)(lh + KB);                  // [KA]
  int64_t* lmin = lsum + KA;
  int64_t* lmax = lmin + (HAS_MIN ? KA : 0);
  int64_t* lcnt = lmax + (HAS_MAX ? KA : 0);
  uint32_t* lfirst = (uint32_t*)(lcnt + ((AGG & FW_AGG_COUNT) ? KA : 0));  // [KA] earliest record (batch index)
  uint32_t* lord = lfirst + ((KA + 3) & ~3);            // [KA] maxBy/minBy: the extremal record (batch index)
  int64_t* lhdr = (int64_t*)(lord + (BY ? ((KA + 3) & ~3) : 0)); // [ntiles][RT_Q] the tiles' routed slices
  uint32_t* lseg = (uint32_t*)(lhdr + (int64_t)r.ntiles * RT_Q);   // [ntiles][RT_GROUPS] this bucket's segment start | end << 16
  int32_t* sst = (int32_t*)(lseg + (int64_t)r.ntiles * RT_GROUPS); // [ntiles] segment start within the tile
  int32_t* off = sst + r.ntiles;                        // [ntiles + 1] segment lengths, then their exclusive prefix;
                                                        // then AG_LOOK entries of INT32_MAX (the step lookup's reads)
  int32_t* step_tile = off + r.ntiles + 1 + AG_LOOK;    // [AG_CHS] tile holding the first record of each step
  int32_t* awtot = step_tile + AG_CHS;                  // [16] scan scratch
  // (aligned by an offset from smem, not through an integer: a pointer rebuilt from an integer loses the LDS
  // address space, and every access through it became a flat access that waited on all outstanding global loads)
  int64_t* gsl = (int64_t*)(smem + ((((unsigned char*)(awtot + 16) - smem) + 7) & ~(ptrdiff_t)7));   // [RT_GS] the batch's slices
  int32_t& lclaim = *(int32_t*)(gsl + RT_GS);
  int32_t* plan = (int32_t*)(gsl + RT_GS) + 2;          // [RT_MAXNB + 1] helper prefix; then bucket, share, shares
  const int64_t SB = (int64_t)8 << 16;
  FW_STAMP(r, SB, 0);
  // Hot buckets (skewed keys) are split over helper workgroups launched after the nb owners: bucket b
  // with L_b routed records last batch gets S_b = clamp(ceil(L_b / chunk), 1, AG_SPLIT_MAX) shares, share
  // s taking tiles [s T / S_b, (s + 1) T / S_b) (tiles are in arrival order, so share order is arrival
  // order).  Every workgroup derives the same plan from the same loads; helpers are assigned to shares in
  // bucket order, so a share's predecessor always has the lower block index (dispatched earlier).  The
  // shares of a bucket fold one after another (fold_flag), share 0 first: the fold stays a plain
  // read-modify-write, first arrival included.
  int bkt = owner_bkt, share = 0, nshare = 1;
  if (SKEW && r.helpers > 0) {   // uniform
    uint32_t tot = 0;
    for (int x = threadIdx.x; x < sa.nb; x += NT) tot += r.bload_prev[x];
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if ((threadIdx.x & 63) == 0) awtot[threadIdx.x >> 6] = (int32_t)tot;
    __syncthreads();
    uint32_t all = 0;
    for (int w = 0; w < NT / 64; ++w) all += (uint32_t)awtot[w];
    // (FW_DEBUG_AGG & 64: a share of 256 records, so that tests split buckets at small sizes)
    const uint32_t chunk = max((r.dbg & 64) ? 256u : AG_SPLIT_MIN,
                               (uint32_t)(((uint64_t)(all / (uint32_t)sa.nb + 1u) * (uint32_t)r.chunk_pct) / 100u));
    for (int x = threadIdx.x; x < sa.nb; x += NT) {
      const uint32_t sh = min((r.bload_prev[x] + chunk - 1) / chunk, (uint32_t)r.split_max);
      plan[x] = sh > 1 ? (int32_t)sh - 1 : 0;    // helpers bucket x asks for
    }
    if (threadIdx.x == 0) plan[sa.nb] = 0;
    __syncthreads();
    block_scan_excl<NT, AG_MAXPER>(plan, sa.nb + 1, awtot);   // plan[x] = first helper of bucket x; plan[nb] = total
    // integer shares: owners are dispatched longest share first (owner vb takes the bucket whose share holds
    // the vb-th most records, ties by bucket), so the workgroups that wait for a CU to free up are the
    // shortest ones.  Every workgroup ranks the same loads: a permutation of the buckets.  (FW_DEBUG_AGG &
    // 128: the plain order.)
    if (HELPERS_FIRST && owner_bkt >= 0 && !(r.dbg & 128)) {   // uniform
      for (int x = threadIdx.x; x < sa.nb; x += NT)
        step_tile[x] = (int32_t)(r.bload_prev[x] / (uint32_t)(1 + max(min(plan[x + 1], r.helpers) - plan[x], 0)));
      __syncthreads();
      for (int x = threadIdx.x; x < sa.nb; x += NT) {
        const int32_t wx = step_tile[x];
        int rk = 0;
        for (int y = 0; y < sa.nb; ++y) {
          const int32_t wy = step_tile[y];
          rk += (wy > wx || (wy == wx && y < x)) ? 1 : 0;
        }
        if (rk == vb) plan[RT_MAXNB + 1] = x;
      }
      __syncthreads();
      owner_bkt = plan[RT_MAXNB + 1];
      __syncthreads();
    }
    const int32_t h = owner_bkt < 0 ? (int32_t)vb - sa.nb : -1;
    if (threadIdx.x == 0) plan[RT_MAXNB + 1] = owner_bkt < 0 ? -1 : owner_bkt;
    __syncthreads();
    for (int x = threadIdx.x; x < sa.nb; x += NT) {
      const int32_t lo = plan[x], n = max(min(plan[x + 1], r.helpers) - lo, 0);   // helpers bucket x gets
      if (h >= lo && h < lo + n) { plan[RT_MAXNB + 1] = x; plan[RT_MAXNB + 2] = h - lo + 1; plan[RT_MAXNB + 3] = 1 + n; }
      if (x == owner_bkt) { plan[RT_MAXNB + 2] = 0; plan[RT_MAXNB + 3] = 1 + n; }
    }
    __syncthreads();
    bkt = plan[RT_MAXNB + 1];
    if (bkt < 0) return;   // uniform: a helper no bucket needs
    share = plan[RT_MAXNB + 2];
    nshare = plan[RT_MAXNB + 3];
    __syncthreads();   // plan[] is reused below only after every thread has read it
  }
  const int t_lo = SKEW ? (int)((int64_t)share * r.ntiles / nshare) : 0;
  const int t_hi = SKEW ? (int)((int64_t)(share + 1) * r.ntiles / nshare) : r.ntiles;
  const int64_t dbase = (int64_t)bkt * KB;
  if (share == 0 && r.fold_cnt_zero)
    for (int g = threadIdx.x; g < RT_GS; g += NT) r.fold_cnt_zero[(int64_t)bkt * RT_GS + g] = 0u;
  // the bucket's directory slice, every tile's header and this bucket's segment bounds in each of its routed bin
  // groups, the tiles' direct marks and the batch's direct flag: all loads independent, issued before any is
  // used (one round trip; the flag read first and waited on cost a round trip of its own, round 6).  The
  // bucket's rows of the bucket-major segment table are contiguous; a row's word is used only where the tile
  // wrote it (a live routed group; the direct / fire groups of a tile with direct records, read in a second
  // round trip by those tiles only)
  const int64_t dk0 = (int)threadIdx.x < KB ? G(sa.dir_keys)[dbase + threadIdx.x] : EMPTY_KEY;
  const unsigned int dfl = *r.dflag;
  // one-slice batches (the usual in-order batch: every tile routed one slice, the same, into group 0, and no tile
  // has direct records) need no slice set and no separate segment scan: with at most one tile per thread, each
  // thread keeps its tile's group-0 segment, the waves scan their lengths and post their slice here, and the
  // checks after the first barrier decide (every thread alike) whether the batch is such a batch
  const bool one_pass = !SKEW && r.ntiles <= NT;   // uniform
  int64_t my_m = FREE_TAG;
  bool my_ok = true;
  int32_t my_len = 0, my_st = 0;
  for (int t = threadIdx.x; t < r.ntiles; t += NT) {
    int64_t h[RT_Q];
    uint32_t sg[RT_GROUPS];
#pragma unroll
    for (int q = 0; q < RT_Q; ++q) h[q] = r.hdr[(int64_t)t * RT_Q + q];
#pragma unroll
    for (int q = 0; q < RT_Q; ++q) sg[q] = r.seg[(int64_t)(q * sa.nb + bkt) * r.seg_stride + t];
    const uint32_t td = r.tdir[t];
#pragma unroll
    for (int q = RT_Q; q < RT_GROUPS; ++q) sg[q] = 0u;
    if (td != 0u) {
#pragma unroll
      for (int q = RT_Q; q < RT_GROUPS; ++q) sg[q] = r.seg[(int64_t)(q * sa.nb + bkt) * r.seg_stride + t];
    }
#pragma unroll
    for (int q = 0; q < RT_Q; ++q)
      if (h[q] == FREE_TAG) sg[q] = 0u;
#pragma unroll
    for (int q = 0; q < RT_Q; ++q) lhdr[t * RT_Q + q] = h[q];
#pragma unroll
    for (int q = 0; q < RT_GROUPS; ++q) lseg[t * RT_GROUPS + q] = sg[q];
    my_m = h[0];
    my_ok = h[1] == FREE_TAG;
    my_st = (int32_t)(sg[0] & 0xFFFFu);
    my_len = (int32_t)(sg[0] >> 16) - my_st;
  }
  // does any tile hold direct-group records (the batch's flag; no: skip all direct work)
  const bool has_direct = __builtin_amdgcn_readfirstlane(dfl) != 0;
  int64_t* wsl = (int64_t*)plan;                  // [NT / 64] one-slice check: each wave's slice (plan is SKEW's)
  int32_t* wok = (int32_t*)(wsl + NT / 64);       // [NT / 64] ... and whether its tiles agree
  int32_t my_incl = 0;
  if (one_pass) {   // uniform
    const uint64_t lm = __ballot(my_m != FREE_TAG);
    const int64_t wm = lm ? __shfl(my_m, __ffsll((long long)lm) - 1) : FREE_TAG;
    const bool ok = __all(my_ok && (my_m == FREE_TAG || my_m == wm));
    my_incl = my_len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(my_incl, o);
      if ((threadIdx.x & 63) >= (unsigned)o) my_incl += y;
    }
    if ((threadIdx.x & 63) == 63) awtot[threadIdx.x >> 6] = my_incl;
    if ((threadIdx.x & 63) == 0) { wsl[threadIdx.x >> 6] = wm; wok[threadIdx.x >> 6] = ok ? 1 : 0; }
  }
  if ((int)threadIdx.x < KB) lh[threadIdx.x] = fmix64((uint64_t)dk0);
  for (int x = threadIdx.x + NT; x < KB; x += NT) lh[x] = fmix64((uint64_t)G(sa.dir_keys)[dbase + x]);
  if (threadIdx.x < AG_LOOK) off[r.ntiles + 1 + threadIdx.x] = INT32_MAX;
  for (int x = threadIdx.x; x < KA; x += NT) {
    lsum[x] = sum_identity(VT);
    if (HAS_MIN) lmin[x] = INT64_MAX;
    if (HAS_MAX) lmax[x] = INT64_MIN;
    if (AGG & FW_AGG_COUNT) lcnt[x] = 0;
    lfirst[x] = NO_FIRST;
    if (BY) lord[x] = sa.by_last ? 0u : NO_FIRST;
  }
  const AggLds L{lsum, lmin, lmax, lcnt, lfirst, lord};
  const bool cmpto = sa.cmpto != 0, by_last = sa.by_last != 0;
  if (threadIdx.x < RT_GS) gsl[threadIdx.x] = FREE_TAG;
  __syncthreads();
  FW_STAMP(r, SB, 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ord_base = b.ord_base;
  // a one-slice batch: the slice set is {m0} and this bucket's segment offsets are the waves' scans (every thread
  // reads the same NT / 64 posts, so `uni` is uniform)
  bool uni = false;
  if (one_pass && !has_direct) {   // uniform
    // lane w < NT / 64 reads wave w's post (one LDS read per lane, no loop of dependent reads and branches)
    constexpr int NW = NT / 64;
    const bool in = lane < NW;
    const int64_t x = in ? wsl[lane] : FREE_TAG;
    const bool okw = !in || wok[lane] != 0;
    const int32_t c = in ? awtot[lane] : 0;
    const uint64_t nz = __ballot(x != FREE_TAG);
    const int64_t m0 = nz ? __shfl(x, __ffsll((long long)nz) - 1) : FREE_TAG;
    const bool ok = __all(okw && (x == FREE_TAG || x == m0));
    int32_t total = c, before = lane < wave ? c : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {   // (over the whole wave: every lane needs the sums)
      total += __shfl_xor(total, o);
      before += __shfl_xor(before, o);
    }
    uni = ok;
    FW_STAMP(r, SB, 5);
    if (uni) {
      if ((int)threadIdx.x < r.ntiles) {
        sst[threadIdx.x] = my_st;
        off[threadIdx.x] = before + my_incl - my_len;
      }
      if (threadIdx.x == 0) {
        off[r.ntiles] = total;
        gsl[0] = m0;   // (FREE_TAG: nothing routed)
      }
    }
  }
  auto gsl_insert = [&](int64_t m) {
    int g = 0;
    for (; g < RT_GS; ++g) {
      const int64_t cur = gsl[g];
      if (cur == m) break;
      if (cur == FREE_TAG) {
        const unsigned long long prev = atomicCAS((unsigned long long*)&gsl[g], (unsigned long long)FREE_TAG, (unsigned long long)m);
        if ((int64_t)prev == FREE_TAG || (int64_t)prev == m) break;
      }
    }
    if (g == RT_GS) cap_error(sa, 6);   // more distinct slices in one batch than RT_GS
  };
  // this bucket's direct-group records (one tile per thread): per-element fires join the late list
  // (k_late_* apply them after this kernel, in arrival order); the others are added in the round of
  // their slice below.  A direct record carries its directory hash (EMPTY_H: the Long.MIN_VALUE key) and
  // its index in the tile, i.e. its batch index
  // no memset between batches: batch j's flag was zeroed by k_aggregate of batch j - FLAG_RING/2, whose
  // flag is no longer read and whose successor k_route starts only after this kernel (event order)
  if (blockIdx.x == 0 && threadIdx.x == 0) *r.dflag_reset = 0u;
  for (int t = threadIdx.x; has_direct && t < r.ntiles; t += NT) {
    const uint32_t sd = lseg[t * RT_GROUPS + RT_Q];
    for (uint32_t x = sd & 0xFFFFu; x < (sd >> 16); ++x) gsl_insert(r.dm[(int64_t)t * RT_TILE + x]);
  }
  // the per-element fire records of this share's tiles, flattened over the workgroup in tile order (after a
  // window boundary most of a hot key's tile can be fire records: one thread per tile walked them
  // serially), under one reservation of the late list
  if (has_direct && b.late_key != nullptr) {   // uniform
    for (int t = threadIdx.x; t < r.ntiles; t += NT) {
      const uint32_t sf = lseg[t * RT_GROUPS + RT_Q + 1];
      const uint32_t f_lo = sf & 0xFFFFu, f_hi = sf >> 16;
      off[t] = (t >= t_lo && t < t_hi && f_hi > f_lo) ? (int32_t)(f_hi - f_lo) : 0;
    }
    if (threadIdx.x == 0) off[r.ntiles] = 0;
    __syncthreads();
    block_scan_excl<NT, AG_MAXPER>(off, r.ntiles + 1, awtot);
    const int32_t nf = off[r.ntiles];
    if (nf > 0) {   // uniform
      if (threadIdx.x == 0) lclaim = (int32_t)atomicAdd(b.late_count, (unsigned long long)nf);
      __syncthreads();
      const unsigned long long lbase = (uint32_t)lclaim;
      for (int32_t j = threadIdx.x; j < nf; j += NT) {
        int t = 0, hi = r.ntiles;   // the last tile t with off[t] <= j holds record j
        while (hi - t > 1) { const int mid = (t + hi) >> 1; if (off[mid] <= j) t = mid; else hi = mid; }
        const uint32_t x = (lseg[t * RT_GROUPS + RT_Q + 1] & 0xFFFFu) + (uint32_t)(j - off[t]);
        const int64_t pos = (int64_t)t * RT_TILE + x;
        const int64_t i = (int64_t)t * RT_TILE + r.idx[pos];
        const uint64_t h = (uint64_t)r.kv[pos].x;
        const int64_t m = r.dm[pos];
        int32_t p = slice_slot_body(sa.slice_tag, sa.P, m);
        int64_t kid = sa.D;
        if (h == EMPTY_H) {   // marks the Long.MIN_VALUE key's column in use
          if (sa.dir_min_used[0] == 0) sa.dir_min_used[0] = 1;
        } else {
          const int32_t x2 = agg_probe_insert_body(lh, sa.dir_keys + dbase, kbm, h, sa.stats + ST_DIR_KEYS);
          kid = x2 < 0 ? -1 : dbase + x2;
        }
        if (p < 0 || kid < 0) { cap_error(sa, 7); p = 0; kid = 0; }   // (a failed batch: a harmless entry keeps the slot)
        late_append_at(s, b, lbase + (unsigned long long)j, p, kid, m, i);
      }
    }
  }
  // the batch's routed slices: distinct entries of the tile headers (every workgroup builds the same
  // set).  A lane whose slice equals its left neighbour's leaves the insert to it, so a wave of an
  // in-order stream inserts once, not 64 times (same-address LDS atomics serialise)
  for (int t0 = 0; !uni && t0 < r.ntiles; t0 += NT) {   // uniform
    const int t = t0 + (int)threadIdx.x;
    for (int q = 0; q < RT_Q; ++q) {
      const int64_t m = t < r.ntiles ? lhdr[t * RT_Q + q] : FREE_TAG;
      const int64_t left = __shfl_up(m, 1);
      const bool dup = lane != 0 && left == m;
      if (m != FREE_TAG && !dup) gsl_insert(m);
    }
  }
  __syncthreads();
  FW_STAMP(r, SB, 6);
  if (SKEW) {   // uniform
    if (threadIdx.x == 0) {   // ascending: every share of a bucket takes the slices in the same rounds
      for (int i = 1; i < RT_GS && gsl[i] != FREE_TAG; ++i)
        for (int j = i; j > 0 && gsl[j - 1] > gsl[j]; --j) { const int64_t t = gsl[j]; gsl[j] = gsl[j - 1]; gsl[j - 1] = t; }
    }
    __syncthreads();
  }

  // directory hash -> slot in this bucket.  Linear probing keeps a key within the run that starts at
  // its home slot, so the first AG_WIN slots are compared without branching (the directory's load factor
  // <= 1/4 keeps nearly every key there); a second inline window takes the few displaced further, the
  // out-of-line probe the rest and new keys (a global CAS on the key, fmix64_inv(h), confirms every slot
  // before it enters the LDS copy)
  auto probe = [&](bool& act, uint64_t h) -> uint32_t {
    const uint32_t h0 = (uint32_t)h & kbm;
    uint32_t kl = h0;
    bool found = false;
#pragma unroll
    for (int j = AG_WIN - 1; j >= 0; --j) {   // the nearest match wins
      const uint32_t x = (h0 + j) & kbm;
      const bool m = lh[x] == h;
      kl = m ? x : kl;
      found |= m;
    }
    const bool miss = act && !found;
    if (__any(miss)) {
      bool found2 = false;
#pragma unroll
      for (int j = 2 * AG_WIN - 1; j >= AG_WIN; --j) {
        const uint32_t x = (h0 + j) & kbm;
        const bool m = lh[x] == h;
        kl = (miss && m) ? x : kl;
        found2 |= m;
      }
      const bool miss2 = miss && !found2;
      if (__any(miss2) && miss2) {
        const int32_t x = agg_probe_insert_body(lh, sa.dir_keys + dbase, kbm, h, sa.stats + ST_DIR_KEYS);
        if (x < 0) { cap_error(sa, 8); act = false; }
        else kl = (uint32_t)x;
      }
    }
    return kl;
  };

  int32_t routed = 0;   // this share's routed records (thread 0's copy is used)
  for (int g = 0; g < RT_GS; ++g) {
    const int64_t m = gsl[g];
    if (m == FREE_TAG) break;                            // uniform
    // pane-slot claim: authoritative here, after every earlier watermark (engine stream order); slot
    // p = floor_mod(m, P) is claimed by whichever workgroup comes first, the rest find it taken by m.  The
    // slot's tag is read now, its value used (and the slot claimed if free) at the fold: the load's latency
    // lies under the main loop instead of in front of it
    int64_t tagv = FREE_TAG;
    if (threadIdx.x == 0) tagv = G(sa.slice_tag)[floor_mod(m, sa.P)];
    if (g == 0) FW_STAMP(r, SB, 7);
    for (int t = threadIdx.x; !uni && t < r.ntiles; t += NT) {   // (uni: offsets already in place)
      int32_t a0 = 0, a1 = 0;
#pragma unroll
      for (int q = 0; q < RT_Q; ++q) {
        if (lhdr[t * RT_Q + q] == m && t >= t_lo && t < t_hi) {
          const uint32_t sg = lseg[t * RT_GROUPS + q];
          a0 = (int32_t)(sg & 0xFFFFu);
          a1 = (int32_t)(sg >> 16);
        }
      }
      sst[t] = a0;
      off[t] = a1 - a0;
    }
    if (!uni) {   // uniform
      if (threadIdx.x == 0) off[r.ntiles] = 0;
      __syncthreads();
      block_scan_excl<NT, AG_MAXPER>(off, r.ntiles + 1, awtot);   // off[ntiles] = the bucket's records of slice m
    }
    const int32_t R = off[r.ntiles];
    routed += R;
    FW_STAMP(r, SB, 2 + 3 * min(g, 1));
    // dense assignment: the bucket's records of slice m, concatenated over the tiles in order (record
    // rr lies in the tile t with off[t] <= rr < off[t + 1]), are taken 64 at a time, one per lane, in
    // wave steps; the tile of each step's first record is tabulated per chunk of AG_CHS steps, a lane
    // walks forward from it (a step spans ~4 segments at 256 buckets), and every load of a wave's UR
    // steps is issued before any of them is processed
    constexpr int UR = FW_AGG_UR;
    constexpr int NPASS = BY ? 2 : 1;
    for (int pass = 0; pass < NPASS; ++pass) {
    for (int32_t cb = 0; cb < R; cb += AG_CHS * 64) {   // uniform
      for (int t = threadIdx.x; t < r.ntiles; t += NT) {
        const int32_t o = off[t], l = off[t + 1] - o;
        if (l == 0) continue;
        const int32_t s_lo = max(0, (o - cb + 63) >> 6), s_hi = min(AG_CHS, (o + l - cb + 63) >> 6);
        for (int32_t st = s_lo; st < s_hi; ++st) step_tile[st] = t;
      }
      __syncthreads();
      const int32_t nsteps = min(AG_CHS, (R - cb + 63) >> 6);
      // one group = UR steps of this wave: addresses from the step table, loads issued, nothing waited on
      // (the record's tile and its in-tile index stay apart until the group is processed: OR-ing the loaded index in
      // here made every group wait for its own loads at once, so no loads were in flight across a group, round 6)
      auto load_group = [&](int32_t s0, longlong2* rv, uint32_t* ri, uint16_t* rx, bool* ra) {
#pragma unroll
        for (int u = 0; u < UR; ++u) {
          const int32_t st = s0 + u;
          const int32_t rr = cb + 64 * st + lane;
          ra[u] = st < nsteps && rr < R;
          int32_t t = 0;
          int64_t pos = 0;   // inactive lanes read tile 0's first slot
          if (ra[u]) {
            // the step's tiles start at t0 (wave-uniform): the segment ends at or below rr among the next
            // AG_LOOK are counted with independent (broadcast) LDS reads, not walked one dependent read at a time
            const int32_t t0 = step_tile[st];
            t = t0;
#pragma unroll
            for (int j = 1; j <= AG_LOOK; ++j) t += off[t0 + j] <= rr ? 1 : 0;
            while (off[t + 1] <= rr) ++t;   // a step over more than AG_LOOK segments (short or empty ones)
            pos = (int64_t)t * RT_TILE + sst[t] + (rr - off[t]);
          }
          rv[u] = r.kv[pos];
          ri[u] = (uint32_t)t << IDX_BITS;
          rx[u] = FIRST ? r.idx[pos] : (uint16_t)0;
        }
      };
      auto process_group = [&](const longlong2* rv, const uint32_t* ri, const uint16_t* rx, const bool* ra) {
#pragma unroll
        for (int u = 0; u < UR; ++u) {
          bool act = ra[u];
          uint32_t kl = probe(act, (uint64_t)rv[u].x);
          const uint32_t oi = ri[u] | (uint32_t)rx[u];
          if (SKEW && !BY) act = hot_combine<VT, AGG>(L, cmpto, act, kl, rv[u].y, oi, lane);
          kl = act ? kl : (uint32_t)KB + (uint32_t)lane;   // inactive lanes update a private dummy slot
          acc_add<VT, AGG>(L, cmpto, by_last, pass, kl, rv[u].y, oi);
        }
      };
      // software pipelined: the next group's loads are in flight while this group updates LDS (two
      // register sets, the loop unrolled by two so that both stay in registers)
      longlong2 rvA[UR], rvB[UR];
      uint32_t riA[UR], riB[UR];
      uint16_t rxA[UR], rxB[UR];
      bool raA[UR], raB[UR];
      constexpr int32_t G = (NT / 64) * UR;
      int32_t s0 = wave * UR;
      if (s0 < nsteps) load_group(s0, rvA, riA, rxA, raA);
      // (the next group's loads are issued unconditionally — past the end a group's lanes are inactive and read tile
      // 0's first slot — so no branch joins paths with different loads in flight: at such a join the compiler waited
      // for every load, the next group's included, round 6)
      while (s0 < nsteps) {   // wave-uniform
        if (FW_AGG_UNCOND || s0 + G < nsteps) load_group(s0 + G, rvB, riB, rxB, raB);
        process_group(rvA, riA, rxA, raA);
        s0 += G;
        if (s0 >= nsteps) break;
        if (FW_AGG_UNCOND || s0 + G < nsteps) load_group(s0 + G, rvA, riA, rxA, raA);
        process_group(rvB, riB, rxB, raB);
        s0 += G;
      }
      __syncthreads();   // the next chunk rewrites step_tile
    }
    // this bucket's direct records of slice m (rare; one tile per thread): the same accumulators, their
    // batch index as the arrival order
    for (int t = t_lo + (int)threadIdx.x; has_direct && t < t_hi; t += NT) {
      const uint32_t sd = lseg[t * RT_GROUPS + RT_Q];
      for (uint32_t x = sd & 0xFFFFu; x < (sd >> 16); ++x) {
        const int64_t pos = (int64_t)t * RT_TILE + x;
        if (r.dm[pos] != m) continue;
        const int64_t i = (int64_t)t * RT_TILE + r.idx[pos];
        const longlong2 rec = r.kv[pos];
        uint32_t kl = KMIN;
        if ((uint64_t)rec.x == EMPTY_H) {
          if (sa.dir_min_used[0] == 0) sa.dir_min_used[0] = 1;   // marks the Long.MIN_VALUE key's column in use
        } else {
          const int32_t x2 = agg_probe_insert_body(lh, sa.dir_keys + dbase, kbm, (uint64_t)rec.x, sa.stats + ST_DIR_KEYS);
          if (x2 < 0) { cap_error(sa, 10); continue; }
          kl = (uint32_t)x2;
        }
        acc_add<VT, AGG>(L, cmpto, by_last, pass, kl, rec.y, (uint32_t)i);
      }
    }
    __syncthreads();
    }   // passes
    FW_STAMP(r, SB, 3 + 3 * min(g, 1));
    if (threadIdx.x == 0) lclaim = tagv == m ? (int32_t)floor_mod(m, sa.P) : slice_slot_body(sa.slice_tag, sa.P, m);
    __syncthreads();
    const int32_t p = lclaim;
    __syncthreads();   // every thread has read lclaim (the next round rewrites it)
    if (p < 0) { if (threadIdx.x == 0) cap_error(sa, 9); continue; }   // slice pool exhausted (uniform)
    unsigned int* flag = r.fold_flag + (int64_t)bkt * RT_GS + g;
    // integer shares of a split bucket fold concurrently with device atomics (sum / count / min / max
    // are exact in any order, and the first arrival is the least batch index over the shares: the last
    // share to fold resolves its f1); double sums and maxBy / minBy fold one share after another
    constexpr bool AFOLD = SKEW && VT == FW_VALUE_I64 && !BY;
    const bool afold = AFOLD && nshare > 1;   // uniform
    if (SKEW && share > 0 && !afold) {   // uniform: wait for the previous share's fold of this slice
      if (threadIdx.x == 0) {
        const unsigned want = (r.tag << 5) | (unsigned)share;
        int64_t spins = 0;
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want) {
          __builtin_amdgcn_s_sleep(8);
          if (++spins > ((int64_t)1 << 21)) { cap_error(sa, 16); break; }   // never hang: report and go on
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // this CU's L1 invalidated once, for the workgroup
      }
      __syncthreads();
    }
    // fold into the dense columns: this workgroup (this share, in share order) is the only writer of
    // (p, bucket) panes while it folds
    for (int x = threadIdx.x; x <= KB; x += NT) {
      if (x == KB && bkt != 0) continue;
      const uint32_t xl = x < KB ? (uint32_t)x : KMIN;
      const uint32_t lf = lfirst[xl];
      if (lf == NO_FIRST) continue;
      const int64_t idx = (int64_t)p * sa.stride + (x < KB ? dbase + x : sa.D);
      if (AFOLD && afold) {
        if (AGG & FW_AGG_SUM) atomicAdd((unsigned long long*)&sa.c.sum[idx], (unsigned long long)lsum[xl]);
        if (AGG & FW_AGG_MIN) atomicMin((long long*)&sa.c.mn[idx], (long long)lmin[xl]);
        if (AGG & FW_AGG_MAX) atomicMax((long long*)&sa.c.mx[idx], (long long)lmax[xl]);
        if (AGG & FW_AGG_COUNT) atomicAdd((unsigned long long*)&sa.c.cnt[idx], (unsigned long long)lcnt[xl]);
        if (FIRST) atomicMin((long long*)&sa.c.first[idx], (long long)(ord_base + (int64_t)lf));
        else sa.c.present[idx] = 1;
      } else if (!BY) {
      // every column of the pane (and the f1 of the batch's earliest record, used if the pane is new) loaded
      // before any store: one round trip (as far as the compiler knows the columns may alias, so a store between
      // two loads made the second wait for it: three round trips per pane, round 6)
      const int64_t o_sum = (AGG & FW_AGG_SUM) ? G(sa.c.sum)[idx] : 0;
      const int64_t o_mn = (AGG & FW_AGG_MIN) ? G(sa.c.mn)[idx] : 0;
      const int64_t o_mx = (AGG & FW_AGG_MAX) ? G(sa.c.mx)[idx] : 0;
      const int64_t o_cnt = (AGG & FW_AGG_COUNT) ? G(sa.c.cnt)[idx] : 0;
      const int64_t o_first = FIRST ? G(sa.c.first)[idx] : 0;
      const int64_t f1n = FIRST ? f1col[lf] : 0;
      if (AGG & FW_AGG_SUM) {
        if (VT == FW_VALUE_I64) G(sa.c.sum)[idx] = jadd(o_sum, lsum[xl]);
        else G(sa.c.sum)[idx] = __double_as_longlong(__longlong_as_double(o_sum) + __longlong_as_double(lsum[xl]));
      }
      if (AGG & FW_AGG_MIN) { if (lmin[xl] < o_mn) G(sa.c.mn)[idx] = lmin[xl]; }
      if (AGG & FW_AGG_MAX) { if (lmax[xl] > o_mx) G(sa.c.mx)[idx] = lmax[xl]; }
      if (AGG & FW_AGG_COUNT) G(sa.c.cnt)[idx] = jadd(o_cnt, lcnt[xl]);
      if (FIRST) {
        // first arrival: the pane's earliest record of the batch, if the pane is new
        if (ord_base + (int64_t)lf < o_first) {
          G(sa.c.first)[idx] = ord_base + (int64_t)lf;
          G(sa.c.f1v)[idx] = f1n;
        }
      } else {
        G(sa.c.present)[idx] = 1;
      }
      } else {
      if (AGG & FW_AGG_SUM) {
        if (VT == FW_VALUE_I64) G(sa.c.sum)[idx] = jadd(G(sa.c.sum)[idx], lsum[xl]);
        else G(sa.c.sum)[idx] = __double_as_longlong(__longlong_as_double(G(sa.c.sum)[idx]) + __longlong_as_double(lsum[xl]));
      }
      if (AGG & FW_AGG_MIN) { const int64_t o = G(sa.c.mn)[idx]; if (lmin[xl] < o) G(sa.c.mn)[idx] = lmin[xl]; }
      if (AGG & FW_AGG_MAX) { const int64_t o = G(sa.c.mx)[idx]; if (lmax[xl] > o) G(sa.c.mx)[idx] = lmax[xl]; }
      if (AGG & FW_AGG_COUNT) G(sa.c.cnt)[idx] = jadd(G(sa.c.cnt)[idx], lcnt[xl]);
      {   // BY
        // the batch's extremal record against the pane's (an earlier arrival: a tie keeps it under
        // "first", takes the batch's under "last"); its ordinal in the count column, its f1 in f1v
        auto col = G(MAXBY ? sa.c.mx : sa.c.mn);
        const int64_t code = MAXBY ? lmax[xl] : lmin[xl];
        const uint32_t lo = lord[xl];
        const int64_t cur = col[idx];
        const bool present = G(sa.c.first)[idx] != INT64_MAX;
        if (!present || (MAXBY ? code > cur : code < cur) || (code == cur && by_last)) {
          col[idx] = code;
          G(sa.c.cnt)[idx] = ord_base + (int64_t)lo;
          G(sa.c.f1v)[idx] = f1col[lo];
        }
        if (ord_base + (int64_t)lf < G(sa.c.first)[idx]) G(sa.c.first)[idx] = ord_base + (int64_t)lf;
        lord[xl] = by_last ? 0u : NO_FIRST;
      }
      }   // !afold
      // cleared for the next round (untouched entries still are; the per-lane dummies are never read)
      lsum[xl] = sum_identity(VT);
      if (HAS_MIN) lmin[xl] = INT64_MAX;
      if (HAS_MAX) lmax[xl] = INT64_MIN;
      if (AGG & FW_AGG_COUNT) lcnt[xl] = 0;
      lfirst[xl] = NO_FIRST;
    }
    if (AFOLD && afold) {
      // count this share's fold in; the last one reads the first arrivals back (agent atomics: coherent
      // across the XCDs' L2s) and stores the f1 of each pane the batch opened.  Atomics on both sides, so
      // no L2 write-back: each wave waits for its own atomics, then one add counts the share in (a
      // __threadfence() per thread here wrote back the XCD's whole L2 sixteen times: ~50 us per share)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {   // (one add: a compare-and-swap loop here serialised the shares for ~50 us)
        const unsigned done = __hip_atomic_fetch_add(r.fold_cnt + (int64_t)bkt * RT_GS + g, 1u, __ATOMIC_ACQ_REL,
                                                     __HIP_MEMORY_SCOPE_AGENT) + 1u;
        lclaim = (int32_t)done == nshare ? 1 : 0;
      }
      __syncthreads();
      if (FIRST && lclaim) {   // uniform
        for (int x = threadIdx.x; x <= KB; x += NT) {
          if (x == KB && bkt != 0) continue;
          const int64_t idx = (int64_t)p * sa.stride + (x < KB ? dbase + x : sa.D);
          const int64_t f = (int64_t)__hip_atomic_fetch_add((unsigned long long*)&sa.c.first[idx], 0ull,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (f >= ord_base && f != INT64_MAX) sa.c.f1v[idx] = f1col[f - ord_base];
        }
      }
    } else {
      // this share's fold visible before the next one's starts: every wave's stores complete, then one
      // release (one L2 write-back) and the flag
      if (SKEW && share + 1 < nshare) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (SKEW && share + 1 < nshare && threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(flag, (r.tag << 5) | (unsigned)(share + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    FW_STAMP(r, SB, 4 + 3 * min(g, 1));
  }
  // this batch's routed records of the bucket (the next batch's split plan); the owner clears the ring
  // entry of the batch after next
  if (threadIdx.x == 0 && r.bload_cur) {
    atomicAdd(&r.bload_cur[bkt], (unsigned)routed);
    if (share == 0) {
      r.bload_zero[bkt] = 0u;
      // for the host's sizing of the next launches: the bucket's load, extrapolated from this share
#if !FW_NO_HOSTLOAD
      if (r.bload_host)
        __hip_atomic_store(&r.bload_host[bkt], (unsigned)routed * (unsigned)nshare, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    } else {
      atomicAdd(&sa.stats[ST_SHARES], 1ull);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// per-element fires (allowed lateness > 0, tumbling): ordered per-pane scan over this batch's records
// whose window already fired.  WindowOperator.java:317-325 + EventTimeTrigger.java:38-40.
// ------------------------------------------------------------------------------------------------
struct LateAcc {
  int64_t sum;    // int64 or double bits
  int64_t mn, mx, cnt;
  int64_t ord, f1;  // maxBy / minBy: the extremal record's arrival ordinal and f1
  int32_t vt;
  int32_t by;       // 0, or FW_AGG_MAXBY / FW_AGG_MINBY, | 1 for the last-tie rule
  __host__ __device__ LateAcc() : sum(0), mn(INT64_MAX), mx(INT64_MIN), cnt(0), ord(INT64_MAX), f1(0), vt(0), by(0) {}
};
// ComparableAggregator.reduce for MAXBY / MINBY (ComparableAggregator.java:74-81): the extremal record;
// on a tie the earlier one (first) or the later one — decided by arrival ordinal, not argument order
__device__ __forceinline__ const LateAcc& by_select(const LateAcc& a, const LateAcc& b) {
  const bool maxby = (a.by & FW_AGG_MAXBY) != 0, last = (a.by & 1) != 0;
  const int64_t ca = maxby ? a.mx : a.mn, cb = maxby ? b.mx : b.mn;
  bool take_b;
  if (ca != cb) take_b = maxby ? cb > ca : cb < ca;
  else take_b = last ? b.ord > a.ord : b.ord < a.ord;
  return take_b ? b : a;
}
struct LateCombine {
  __device__ LateAcc operator()(const LateAcc& a, const LateAcc& b) const {
    if (a.by) return by_select(a, b);
    LateAcc r;
    r.vt = a.vt;
    if (a.vt == FW_VALUE_I64) {
      r.sum = jadd(a.sum, b.sum);
    } else {
      r.sum = __double_as_longlong(__longlong_as_double(a.sum) + __longlong_as_double(b.sum));
    }
    r.mn = a.mn < b.mn ? a.mn : b.mn;
    r.mx = a.mx > b.mx ? a.mx : b.mx;
    r.cnt = jadd(a.cnt, b.cnt);
    return r;
  }
};

// (emit_n > 0: also reserves the emit kernel's emit_n output slots at once, *out_base = the first —
// one device atomic instead of one per wave of emitters on the shared output cursor)
__global__ void k_late_prepare(Spec s, const unsigned long long* sorted_key, int64_t nl, int32_t idx_bits,
                               const int64_t* val, unsigned long long* seg, LateAcc* acc, int64_t* headpos,
                               const int64_t* f1col, int64_t ord_base, int64_t emit_n, unsigned long long* out_base) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0 && emit_n > 0) *out_base = atomicAdd(s.o.count, (unsigned long long)emit_n);
  if (j >= nl) return;
  unsigned long long k = sorted_key[j];
  int64_t i = (int64_t)(k & ((1ull << idx_bits) - 1));
  seg[j] = k >> idx_bits;
  headpos[j] = (j == 0 || (sorted_key[j - 1] >> idx_bits) != (k >> idx_bits)) ? j : 0;
  int64_t v = val[i];
  LateAcc a;
  a.vt = s.vt;
  a.sum = v;
  a.mn = min_code(s.vt, s.cmpto, v);
  a.mx = max_code(s.vt, s.cmpto, v);
  a.cnt = 1;
  a.by = s.by ? (s.by | (s.by_last ? 1 : 0)) : 0;
  a.ord = ord_base + i;
  a.f1 = f1col[i];
  acc[j] = a;
}

// Ordered segmented scan of the late records' accumulators (segments = runs of one pane in the sorted
// list, combined in arrival order) and of each record's segment head position: a tile of LS_T x LS_I
// records per workgroup, serial per thread, Hillis-Steele over the threads in LDS; the tiles' carries by
// one workgroup; then the records of each tile ahead of its first head take their carry.  A fixed
// combine tree: double sums are reproducible run to run (replaces a rocPRIM scan-by-key of the 56-B
// accumulator, ~0.57 ms per 1.6 M records)
#ifndef FW_LS_I
#define FW_LS_I 1
#endif
constexpr int LS_T = 256, LS_I = FW_LS_I, LS_TILE = LS_T * LS_I, LS_CT = 512;
struct SegPart {
  LateAcc v;
  int64_t hp;      // the last segment head at or before this point (-1: none)
  int32_t head;    // a segment starts inside
  int32_t empty;   // no records
};
__device__ __forceinline__ SegPart seg_join(const SegPart& x, const SegPart& y) {
  if (y.empty) return x;
  if (x.empty) return y;
  SegPart r;
  r.v = y.head ? y.v : LateCombine()(x.v, y.v);
  r.hp = x.hp > y.hp ? x.hp : y.hp;
  r.head = x.head | y.head;
  r.empty = 0;
  return r;
}
__global__ __launch_bounds__(LS_T) void k_segscan_tile(const unsigned long long* __restrict__ seg,
                                                        const LateAcc* __restrict__ acc, int64_t n,
                                                        LateAcc* __restrict__ out, int64_t* __restrict__ hp_out,
                                                        SegPart* tile_agg,
                                                        int32_t* tile_first_head) {
  __shared__ __attribute__((aligned(16))) unsigned char sp_raw[LS_T * sizeof(SegPart)];   // (LateAcc has a constructor)
  SegPart* sp = (SegPart*)sp_raw;
  __shared__ int32_t first_head;
  if (threadIdx.x == 0) first_head = LS_TILE;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * LS_TILE;
  const int64_t base = t0 + (int64_t)threadIdx.x * LS_I;
  SegPart a;
  a.empty = 1; a.head = 0; a.hp = -1;
  int32_t lead = LS_I;   // this thread's records before its first head
  for (int i = 0; i < LS_I; ++i) {
    const int64_t j = base + i;
    if (j >= n) break;
    const bool h = j == 0 || seg[j] != seg[j - 1];
    const LateAcc x = acc[j];
    if (h || a.empty) a.v = x;
    else a.v = LateCombine()(a.v, x);
    if (h) { a.hp = j; if (!a.head) lead = i; a.head = 1; }
    a.empty = 0;
    out[j] = a.v;
    hp_out[j] = a.hp;
  }
  if (a.head) atomicMin(&first_head, (int32_t)(threadIdx.x * LS_I + lead));
  sp[threadIdx.x] = a;
  __syncthreads();
  for (int o = 1; o < LS_T; o <<= 1) {   // inclusive over the threads
    SegPart y = a;
    if ((int)threadIdx.x >= o) y = seg_join(sp[threadIdx.x - o], a);
    __syncthreads();
    sp[threadIdx.x] = y;
    a = y;
    __syncthreads();
  }
  if (threadIdx.x == LS_T - 1) { tile_agg[blockIdx.x] = a; tile_first_head[blockIdx.x] = first_head; }
  if (threadIdx.x == 0) return;
  const SegPart pre = sp[threadIdx.x - 1];   // exclusive prefix within the tile
  if (pre.empty) return;
  for (int i = 0; i < lead; ++i) {   // the records ahead of this thread's first head continue pre's segment
    const int64_t j = base + i;
    if (j >= n) break;
    out[j] = LateCombine()(pre.v, out[j]);
    hp_out[j] = pre.hp;
  }
}
// the tiles' exclusive carries (one workgroup; chunks of consecutive tiles per thread)
__global__ __launch_bounds__(LS_CT) void k_segscan_carry(SegPart* tile_agg, int32_t ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned char sp_raw[LS_CT * sizeof(SegPart)];   // (LateAcc has a constructor)
  SegPart* sp = (SegPart*)sp_raw;
  const int per = (ntiles + LS_CT - 1) / LS_CT;
  const int lo = (int)threadIdx.x * per, hi = min(ntiles, lo + per);
  SegPart a;
  a.empty = 1; a.head = 0; a.hp = -1;
  for (int t = lo; t < hi; ++t) a = seg_join(a, tile_agg[t]);
  sp[threadIdx.x] = a;
  __syncthreads();
  for (int o = 1; o < LS_CT; o <<= 1) {
    SegPart y = a;
    if ((int)threadIdx.x >= o) y = seg_join(sp[threadIdx.x - o], a);
    __syncthreads();
    sp[threadIdx.x] = y;
    a = y;
    __syncthreads();
  }
  SegPart run;
  if (threadIdx.x > 0) run = sp[threadIdx.x - 1];
  else { run.empty = 1; run.head = 0; run.hp = -1; }
  for (int t = lo; t < hi; ++t) {   // in place: tile t's aggregate becomes its carry
    const SegPart own = tile_agg[t];
    tile_agg[t] = run;
    run = seg_join(run, own);
  }
}
// the carries in two levels when the tiles outnumber the one workgroup's threads: each workgroup of LS_CT
// tiles turns their aggregates into carries within the group (in place) and posts the group's aggregate;
// k_segscan_carry then turns the groups' aggregates into their carries, and k_segscan_apply joins the two
__global__ __launch_bounds__(LS_CT) void k_segscan_carry_grp(SegPart* tile_agg, int32_t ntiles, SegPart* grp) {
  __shared__ __attribute__((aligned(16))) unsigned char sp_raw[LS_CT * sizeof(SegPart)];   // (LateAcc has a constructor)
  SegPart* sp = (SegPart*)sp_raw;
  const int t = (int)blockIdx.x * LS_CT + (int)threadIdx.x;
  SegPart a;
  a.empty = 1; a.head = 0; a.hp = -1;
  if (t < ntiles) a = tile_agg[t];
  sp[threadIdx.x] = a;
  __syncthreads();
  for (int o = 1; o < LS_CT; o <<= 1) {
    SegPart y = a;
    if ((int)threadIdx.x >= o) y = seg_join(sp[threadIdx.x - o], a);
    __syncthreads();
    sp[threadIdx.x] = y;
    a = y;
    __syncthreads();
  }
  if (threadIdx.x == LS_CT - 1) grp[blockIdx.x] = a;
  SegPart ex;
  if (threadIdx.x > 0) ex = sp[threadIdx.x - 1];
  else { ex.empty = 1; ex.head = 0; ex.hp = -1; }
  if (t < ntiles) tile_agg[t] = ex;
}
__global__ __launch_bounds__(LS_T) void k_segscan_apply(const SegPart* carry, const SegPart* grp_carry,
                                                         const int32_t* tile_first_head, int64_t n,
                                                         LateAcc* out, int64_t* hp_out) {
  const SegPart c = grp_carry ? seg_join(grp_carry[blockIdx.x / LS_CT], carry[blockIdx.x]) : carry[blockIdx.x];
  if (c.empty) return;
  const int32_t lead = tile_first_head[blockIdx.x];
  const int64_t t0 = (int64_t)blockIdx.x * LS_TILE;
  for (int i = threadIdx.x; i < lead; i += LS_T) {
    const int64_t j = t0 + i;
    if (j >= n) break;
    out[j] = LateCombine()(c.v, out[j]);
    hp_out[j] = c.hp;
  }
}

__device__ __forceinline__ bool cols_present(const Spec& s, const Cols& c, int64_t idx) {
  return s.first ? c.first[idx] != INT64_MAX : c.present[idx] != 0;
}
__device__ __forceinline__ bool pane_present(const Spec& s, int64_t idx) { return cols_present(s, s.c, idx); }

__device__ __forceinline__ LateAcc cols_load(const Spec& s, const Cols& c, int64_t idx) {
  LateAcc a;
  a.vt = s.vt;
  a.sum = c.sum ? c.sum[idx] : 0;
  a.mn = c.mn ? c.mn[idx] : INT64_MAX;
  a.mx = c.mx ? c.mx[idx] : INT64_MIN;
  a.cnt = c.cnt ? c.cnt[idx] : 0;
  if (s.by) {   // the extremal record: ordinal in the count column, its f1 in f1v
    a.by = s.by | (s.by_last ? 1 : 0);
    a.ord = a.cnt;
    a.cnt = 0;
    a.f1 = c.f1v[idx];
  }
  return a;
}
__device__ __forceinline__ LateAcc pane_load(const Spec& s, int64_t idx) { return cols_load(s, s.c, idx); }

// slot of window n's window pane (sliding, -1: none)
__device__ __forceinline__ int32_t wpane_slot(const Spec& s, int64_t n) {
  if (s.W == 0) return -1;
  const int32_t w = (int32_t)floor_mod(n, s.W);
  return s.wtag[w] == n ? w : -1;
}

__device__ __forceinline__ void emit_record(const Spec& s, unsigned long long pos, int64_t key, int64_t f1, int64_t ts,
                                            const LateAcc& a) {
  if ((int64_t)pos >= s.o.capacity) { cap_error(s, 11); return; }
  if (s.fold) {   // HeapFoldingState: the first record folded into the initial value (every fold here associates)
    LateAcc f = a;
    const int64_t x = s.fold_init;
    if (s.vt == FW_VALUE_I64) f.sum = jadd(x, a.sum);
    else f.sum = __double_as_longlong(__longlong_as_double(x) + __longlong_as_double(a.sum));
    const int64_t cn = min_code(s.vt, s.cmpto, x), cx = max_code(s.vt, s.cmpto, x);
    f.mn = cn < a.mn ? cn : a.mn;
    f.mx = cx > a.mx ? cx : a.mx;
    f.cnt = jadd(x, a.cnt);
    s.o.key[pos] = key;
    if (s.o.f1) s.o.f1[pos] = f1;
    s.o.ts[pos] = ts;
    if (s.o.sum) s.o.sum[pos] = f.sum;
    if (s.o.mn) s.o.mn[pos] = s.vt == FW_VALUE_I64 ? f.mn : __double_as_longlong(f64_from_code(f.mn));
    if (s.o.mx) s.o.mx[pos] = s.vt == FW_VALUE_I64 ? f.mx : __double_as_longlong(f64_from_code(f.mx));
    if (s.o.cnt) s.o.cnt[pos] = f.cnt;
    return;
  }
  s.o.key[pos] = key;
  if (s.o.f1) s.o.f1[pos] = f1;
  s.o.ts[pos] = ts;
  if (s.o.sum) s.o.sum[pos] = a.sum;
  if (s.o.mn) s.o.mn[pos] = s.vt == FW_VALUE_I64 ? a.mn : __double_as_longlong(f64_from_code(a.mn));
  if (s.o.mx) s.o.mx[pos] = s.vt == FW_VALUE_I64 ? a.mx : __double_as_longlong(f64_from_code(a.mx));
  if (s.o.cnt) s.o.cnt[pos] = a.cnt;
}

__device__ __forceinline__ int64_t kid_key(const Spec& s, int64_t kid) { return kid == s.D ? EMPTY_KEY : s.dir_keys[kid]; }

__device__ __forceinline__ int64_t slot_max_ts(const Spec& s, int32_t p) {
  int64_t m = s.slice_tag[p];
  int64_t start = jadd(s.offset, (int64_t)((uint64_t)m * (uint64_t)s.size));  // tumbling: slice = window
  return jsub(jadd(start, s.size), 1);
}

// emit one result per late record: state(base) (+) prefix
__global__ void k_late_emit(Spec s, const unsigned long long* sorted_key, int64_t nl, int32_t idx_bits,
                            const unsigned long long* seg, const LateAcc* acc, const LateAcc* scanned,
                            const int64_t* f1col, int64_t ord_base, const int64_t* headpos,
                            const unsigned long long* out_base) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nl) return;
  const unsigned long long pos = *out_base + (unsigned long long)j;   // one result per late record, in place
  unsigned long long pane = seg[j];
  int64_t idx = (int64_t)pane;
  int32_t p = (int32_t)(pane / (unsigned long long)s.stride);
  int64_t kid = (int64_t)(pane % (unsigned long long)s.stride);
  bool head = j == 0 || seg[j - 1] != pane;
  bool base_present = pane_present(s, idx);
  LateCombine op;
  LateAcc out;
  if (s.trigger == FW_TRIGGER_PURGING_EVENT_TIME && !head) out = acc[j];   // state was purged by the previous fire
  else if (s.trigger == FW_TRIGGER_PURGING_EVENT_TIME) out = base_present ? op(pane_load(s, idx), acc[j]) : acc[j];
  else out = base_present ? op(pane_load(s, idx), scanned[j]) : scanned[j];
  int64_t f1 = 0;
  if (s.by) {
    f1 = out.f1;   // maxBy / minBy: the extremal record's
  } else if (s.first) {
    // first arrival: the pane's if it existed, else the segment head (purging: the record itself
    // unless it is the head of a segment over an existing pane)
    int64_t i_self = (int64_t)(sorted_key[j] & ((1ull << idx_bits) - 1));
    if (s.trigger == FW_TRIGGER_PURGING_EVENT_TIME) {
      f1 = (head && base_present) ? s.c.f1v[idx] : f1col[i_self];
    } else if (base_present) {
      f1 = s.c.f1v[idx];
    } else {
      f1 = f1col[(int64_t)(sorted_key[headpos[j]] & ((1ull << idx_bits) - 1))];
    }
  }
  emit_record(s, pos, kid_key(s, kid), f1, slot_max_ts(s, p), out);
}

// write the pane state after the batch's per-element fires (segment tails)
__global__ void k_late_commit(Spec s, const unsigned long long* sorted_key, int64_t nl, int32_t idx_bits,
                              const unsigned long long* seg, const LateAcc* scanned, const int64_t* f1col,
                              int64_t ord_base, const int64_t* headpos, bool fired = true) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nl) return;
  unsigned long long pane = seg[j];
  bool tail = j == nl - 1 || seg[j + 1] != pane;
  if (!tail) return;
  int64_t idx = (int64_t)pane;
  int32_t p = (int32_t)(pane / (unsigned long long)s.stride);
  if (fired && s.trigger == FW_TRIGGER_PURGING_EVENT_TIME && s.assigner == FW_TUMBLING) {
    // FIRE_AND_PURGE after the last element: pane cleared (AbstractHeapState.clear).  (Sliding: the slice
    // also feeds windows that have not fired; a purged window's later per-element fires emit the record
    // alone, k_fire_emit).  The cleanup timer the segment's first record registered stays (s.gfirst)
    if (s.gfirst) {
      int64_t o = s.first ? ord_base + (int64_t)(sorted_key[headpos[j]] & ((1ull << idx_bits) - 1)) : 0;
      if (s.first && s.c.first[idx] < o) o = s.c.first[idx];
      if (o < s.gfirst[idx]) s.gfirst[idx] = o;
    }
    if (s.c.sum) s.c.sum[idx] = sum_identity(s.vt);
    if (s.c.mn) s.c.mn[idx] = INT64_MAX;
    if (s.c.mx) s.c.mx[idx] = INT64_MIN;
    if (s.c.cnt) s.c.cnt[idx] = 0;
    if (s.first) s.c.first[idx] = INT64_MAX; else s.c.present[idx] = 0;
    return;
  }
  bool base_present = pane_present(s, idx);
  LateCombine op;
  LateAcc st = base_present ? op(pane_load(s, idx), scanned[j]) : scanned[j];
  if (s.c.sum) s.c.sum[idx] = st.sum;
  if (s.c.mn) s.c.mn[idx] = st.mn;
  if (s.c.mx) s.c.mx[idx] = st.mx;
  if (s.c.cnt) s.c.cnt[idx] = s.by ? st.ord : st.cnt;
  if (s.by) s.c.f1v[idx] = st.f1;
  if (!base_present) {
    int64_t ih = (int64_t)(sorted_key[headpos[j]] & ((1ull << idx_bits) - 1));
    if (s.first) { s.c.first[idx] = ord_base + ih; if (!s.by) s.c.f1v[idx] = f1col[ih]; }
    else s.c.present[idx] = 1;
  }
  (void)p;
}

// sliding windows: one result per fire element (record, window) in (window, arrival) order — the window's
// contents when the record was added: its slices' states before this batch's per-element records (+) the
// prefix of the window's late records up to this one.  PurgingTrigger: the window was purged by its
// watermark fire and by every per-element fire since (FIRE_AND_PURGE), so the result is the record alone.
__global__ void k_fire_emit(Spec s, const unsigned long long* sorted_key, int64_t nf, int32_t idx_bits,
                            const unsigned long long* seg, const LateAcc* acc, const LateAcc* scanned,
                            const int64_t* f1col, const int64_t* tscol, int64_t wm, const int64_t* headpos,
                            const unsigned long long* out_base) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nf) return;
  const unsigned long long pos = *out_base + (unsigned long long)j;   // one result per fire element, in place
  const unsigned long long wpane = seg[j];
  const int32_t wp = (int32_t)(wpane / (unsigned long long)s.stride);
  const int64_t kid = (int64_t)(wpane % (unsigned long long)s.stride);
  const int64_t i_self = (int64_t)(sorted_key[j] & ((1ull << idx_bits) - 1));
  // the window: the one of the record's windows with slot wp (its windows span fewer than P numbers)
  const int64_t m = record_windows(s, tscol[i_self], wm).m;
  const int64_t n_hi = floor_div(m, s.R), n_lo = floor_div(m - s.K, s.R) + 1;
  int64_t n = n_lo;
  for (int64_t x = n_lo; x <= n_hi; ++x) if (floor_mod(x, s.P) == wp) n = x;
  const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
  LateAcc out;
  int64_t f1 = f1col[i_self];
  if (s.trigger == FW_TRIGGER_PURGING_EVENT_TIME) {
    out = acc[j];
  } else {
    LateCombine op;
    bool any = false;
    LateAcc base;
    int64_t best = INT64_MAX, bf1 = 0;
    for (int k = 0; k < s.K; ++k) {
      const int64_t mm = n * s.R + k;
      const int32_t pp = (int32_t)floor_mod(mm, s.P);
      if (s.slice_tag[pp] != mm) continue;
      const int64_t idx = (int64_t)pp * s.stride + kid;
      if (!pane_present(s, idx)) continue;
      if (s.first && s.c.first[idx] < best) { best = s.c.first[idx]; bf1 = s.c.f1v[idx]; }
      const LateAcc bb = pane_load(s, idx);
      base = any ? op(base, bb) : bb;
      any = true;
    }
    const int32_t wq = wpane_slot(s, n);   // the window's own pane (records with the assigner's extra window)
    if (wq >= 0) {
      const int64_t idx = (int64_t)wq * s.stride + kid;
      if (cols_present(s, s.wc, idx)) {
        if (s.first && s.wc.first[idx] < best) { best = s.wc.first[idx]; bf1 = s.wc.f1v[idx]; }
        const LateAcc bb = cols_load(s, s.wc, idx);
        base = any ? op(base, bb) : bb;
        any = true;
      }
    }
    out = any ? op(base, scanned[j]) : scanned[j];
    // first arrival: the window's earliest slice record, else the head of this window's late records
    f1 = any ? bf1 : f1col[(int64_t)(sorted_key[headpos[j]] & ((1ull << idx_bits) - 1))];
  }
  if (s.by) f1 = out.f1;
  emit_record(s, pos, kid_key(s, kid), f1, max_ts, out);
}

// ------------------------------------------------------------------------------------------------
// watermark: plan fires/purges from the live slices, fire, purge, mark
// ------------------------------------------------------------------------------------------------

// ------------------------------------------------------------------------------------------------
// watermark (AbstractStreamOperator.processWatermark :803-808 -> HeapInternalTimerService.advanceWatermark
// :264-278 -> WindowOperator.onEventTime :336-375), one launch per watermark.  Every workgroup derives
// the same plan from the live slices (windows with maxTimestamp in (old, new], each owned by its first
// live slice; slices whose last window's cleanup time <= new), fires those windows over its share of
// the key ids, then purges its share of the expired slices; the last workgroup to finish frees the
// slots and records the watermark's position in the output log.
// ------------------------------------------------------------------------------------------------
constexpr int WM_THREADS = 1024;
constexpr int WM_MAXT = MAX_P + MAX_K;   // windows firing at one watermark: every live slot's windows (a flush to
                                         // Long.MAX_VALUE fires up to P + K - 1 of them at K slices per window)
constexpr int WM_MAXP = MAX_P;     // slices purged at one watermark (>= P)
constexpr int32_t PURGE_GHOST = 1 << 30;   // purge list flag: keep the panes' cleanup timers (Spec::gfirst)

constexpr int WM_C = 8;                    // slices whose panes one thread loads at once (one round trip each)

// a pane's state for the fire pass: the columns the reduce shape keeps (AGG 15: the runtime set)
template <int VT, int AGG>
__device__ __forceinline__ LateAcc wm_load(const Spec& s, int64_t idx) {
  constexpr bool BY = (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;   // maxBy / minBy come alone (fw_create)
  LateAcc a;
  a.vt = VT;
  if (AGG == 15) {   // the runtime column set, never maxBy / minBy
    if (s.c.sum) a.sum = s.c.sum[idx];
    if (s.c.mn) a.mn = s.c.mn[idx];
    if (s.c.mx) a.mx = s.c.mx[idx];
    if (s.c.cnt) a.cnt = s.c.cnt[idx];
    return a;
  }
  if (BY) {   // the extremal record: its code, its ordinal (count column) and its f1
    a.by = s.by | (s.by_last ? 1 : 0);
    if (AGG & FW_AGG_MAXBY) a.mx = s.c.mx[idx]; else a.mn = s.c.mn[idx];
    a.ord = s.c.cnt[idx];
    a.f1 = s.c.f1v[idx];
    return a;
  }
  if (AGG & FW_AGG_SUM) a.sum = s.c.sum[idx];
  if (AGG & FW_AGG_MIN) a.mn = s.c.mn[idx];
  if (AGG & FW_AGG_MAX) a.mx = s.c.mx[idx];
  if (AGG & FW_AGG_COUNT) a.cnt = s.c.cnt[idx];
  return a;
}
template <int VT, int AGG>
__device__ __forceinline__ LateAcc wm_combine(const LateAcc& a, const LateAcc& b) {
  if (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) return by_select(a, b);
  LateAcc r = a;   // (absent columns hold their identities on both sides)
  if (AGG & FW_AGG_SUM)
    r.sum = VT == FW_VALUE_I64 ? jadd(a.sum, b.sum)
                               : __double_as_longlong(__longlong_as_double(a.sum) + __longlong_as_double(b.sum));
  if (AGG & FW_AGG_MIN) r.mn = a.mn < b.mn ? a.mn : b.mn;
  if (AGG & FW_AGG_MAX) r.mx = a.mx > b.mx ? a.mx : b.mx;
  if (AGG & FW_AGG_COUNT) r.cnt = jadd(a.cnt, b.cnt);
  return r;
}
// a slice pane back to the empty state (WindowOperator.clearAllState -> windowState.clear())
__device__ __forceinline__ void pane_clear(const Spec& s, int64_t idx) {
  if (s.c.sum) s.c.sum[idx] = sum_identity(s.vt);
  if (s.c.mn) s.c.mn[idx] = INT64_MAX;
  if (s.c.mx) s.c.mx[idx] = INT64_MIN;
  if (s.c.cnt) s.c.cnt[idx] = 0;
  if (s.first) s.c.first[idx] = INT64_MAX; else s.c.present[idx] = 0;
}

// ------------------------------------------------------------------------------------------------
// per-element fires of tumbling windows in one pass (WindowOperator.processElement :317-325 for each late
// record in arrival order, EventTimeTrigger.onElement FIRE): over the (pane, arrival)-sorted late list, an
// ordered segmented scan whose segment head folds in the pane's state before the batch, so every record's
// result is its running window content; each record emits it, each segment tail writes the pane back.
// Tiles take tickets in launch order and chain their carries by decoupled look-back (a tile holding a
// segment head publishes its inclusive carry at once), so the list is read once and the pane state
// columns once per segment.  Replaces prepare / tile scan / carries / apply / emit / commit (six kernels
// and ~270 B of accumulator traffic per record).
// ------------------------------------------------------------------------------------------------
constexpr int LF_T = 256;                   // records per tile, one per thread
struct LfPart {
  LateAcc v;        // the segment's running content (its head folded in the pane's state before the batch)
  int64_t sf1;      // the segment's first-arrival f1 (the pane's, else its head record's)
  int64_t sfirst;   // the head record's arrival ordinal
  int32_t head;     // a segment starts inside
  int32_t bpres;    // the pane existed before the batch (of the last head inside)
  int32_t empty;
};
template <int VT, int AGG>
__device__ __forceinline__ LfPart lf_join(const LfPart& x, const LfPart& y) {
  if (y.empty) return x;
  if (x.empty) return y;
  LfPart r = y;
  if (!y.head) {   // y continues x's segment
    r.v = wm_combine<VT, AGG>(x.v, y.v);
    r.sf1 = x.sf1; r.sfirst = x.sfirst; r.bpres = x.bpres;
    r.head = x.head;
  }
  return r;
}
// a tile's carry crosses XCDs: written and read with agent-scope atomics (they bypass the XCD's L2), the
// writer waiting for its stores before it raises the flag — no release fence, whose L2 write-back cost
// ~20-50 us per tile behind the batch's output stores
__device__ __forceinline__ void lf_put(LfPart* dst, const LfPart& v) {
  static_assert(sizeof(LfPart) % 8 == 0, "LfPart moves in qwords");
  const unsigned long long* a = (const unsigned long long*)&v;
  unsigned long long* b = (unsigned long long*)dst;
#pragma unroll
  for (int w = 0; w < (int)(sizeof(LfPart) / 8); ++w) __hip_atomic_store(b + w, a[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ LfPart lf_get(const LfPart* src) {
  LfPart r;
  unsigned long long* b = (unsigned long long*)&r;
  const unsigned long long* a = (const unsigned long long*)src;
#pragma unroll
  for (int w = 0; w < (int)(sizeof(LfPart) / 8); ++w)
    b[w] = __hip_atomic_load((unsigned long long*)(a + w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}
// Ordering of the carries (target-dependent, gfx94x / gfx950 only): a tile's data is written with
// agent-scope relaxed atomic stores (write-through past the XCD's non-coherent L2), lf_raise waits for their
// acknowledgement (s_waitcnt vmcnt(0)) before the agent-scope flag store, and a reader issues its agent-scope
// relaxed atomic data loads only after its flag load returned the new value (control dependency, loads issued in
// order and served at the coherence point).  The C++ model would want acquire on the flag load; on these targets an
// agent-scope acquire adds a cache invalidate per look-back step and buys nothing the atomics do not already give.
// Porting this kernel to another target means making the flag load an acquire.
__device__ __forceinline__ void lf_raise(unsigned int* flag, unsigned int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the data's stores acknowledged first
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the scan's LDS traffic and shuffles carry only the accumulator fields the reduce shape keeps (a whole LfPart
// per step held ~150 VGPRs: three tiles per CU)
template <int AGG>
__device__ __forceinline__ void lf_fields(LfPart& d, const LfPart& x) {
  constexpr bool BY = (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;
  if (AGG & FW_AGG_SUM) d.v.sum = x.v.sum;
  if (AGG & (FW_AGG_MIN | FW_AGG_MINBY)) d.v.mn = x.v.mn;
  if (AGG & (FW_AGG_MAX | FW_AGG_MAXBY)) d.v.mx = x.v.mx;
  if (AGG & FW_AGG_COUNT) d.v.cnt = x.v.cnt;
  if (BY) { d.v.ord = x.v.ord; d.v.f1 = x.v.f1; d.v.by = x.v.by; }
  d.sf1 = x.sf1; d.sfirst = x.sfirst; d.head = x.head; d.bpres = x.bpres; d.empty = x.empty;
}
template <int VT, int AGG>
__device__ __forceinline__ LfPart lf_ld(const LfPart* p) {
  LfPart r;
  r.v.vt = VT;
  lf_fields<AGG>(r, *p);
  return r;
}
template <int AGG>
__device__ __forceinline__ void lf_st(LfPart* p, const LfPart& x) { lf_fields<AGG>(*p, x); }
template <int VT, int AGG>
__device__ __forceinline__ LfPart lf_shfl_t(const LfPart& x, int src) {
  constexpr bool BY = (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;
  LfPart r;
  r.v.vt = VT;
  if (AGG & FW_AGG_SUM) r.v.sum = __shfl(x.v.sum, src);
  if (AGG & (FW_AGG_MIN | FW_AGG_MINBY)) r.v.mn = __shfl(x.v.mn, src);
  if (AGG & (FW_AGG_MAX | FW_AGG_MAXBY)) r.v.mx = __shfl(x.v.mx, src);
  if (AGG & FW_AGG_COUNT) r.v.cnt = __shfl(x.v.cnt, src);
  if (BY) { r.v.ord = __shfl(x.v.ord, src); r.v.f1 = __shfl(x.v.f1, src); r.v.by = __shfl(x.v.by, src); }
  r.sf1 = __shfl(x.sf1, src); r.sfirst = __shfl(x.sfirst, src);
  r.head = __shfl(x.head, src); r.bpres = __shfl(x.bpres, src); r.empty = __shfl(x.empty, src);
  return r;
}
struct LfLink {            // one tile's published carry: epoch << 2 | 1 (tile aggregate), | 2 (inclusive prefix)
  unsigned int* flag;
  LfPart* agg;
  LfPart* incl;
  unsigned long long* base;   // [0] the launch's first output slot, [1] its epoch
  unsigned int* ticket;
  unsigned int ticket0, epoch;
};

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(LF_T) void k_late_fused(Spec s, const unsigned long long* __restrict__ sorted_key, int64_t nl,
                                                     int32_t idx_bits, const int64_t* __restrict__ val,
                                                     const int64_t* __restrict__ f1col, int64_t ord_base, LfLink L) {
  __shared__ __attribute__((aligned(16))) unsigned char sp_raw[LF_T * sizeof(LfPart)];
  LfPart* sp = (LfPart*)sp_raw;
  __shared__ __attribute__((aligned(16))) unsigned char carry_raw[sizeof(LfPart)];
  LfPart& carry_s = *(LfPart*)carry_raw;
  __shared__ unsigned int tile_s;
  __shared__ unsigned long long base_s;
  constexpr bool BY = (AGG & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;
  const bool purging = s.trigger == FW_TRIGGER_PURGING_EVENT_TIME;
  if (threadIdx.x == 0) tile_s = atomicAdd(L.ticket, 1u) - L.ticket0;
  __syncthreads();
  const int64_t tile = tile_s;
  const int64_t j = tile * LF_T + threadIdx.x;
  const unsigned long long imask = (1ull << idx_bits) - 1;
  // this record: its pane, its accumulator; a segment head folds in the pane's state before the batch
  LfPart a;
  a.empty = 1; a.head = 0; a.bpres = 0; a.sf1 = 0; a.sfirst = 0;
  unsigned long long pane = 0;
  int64_t i_self = 0;
  bool tail = false;
  if (j < nl) {
    const unsigned long long k = sorted_key[j];
    pane = k >> idx_bits;
    i_self = (int64_t)(k & imask);
    const bool head = j == 0 || (sorted_key[j - 1] >> idx_bits) != pane;
    tail = j == nl - 1 || (sorted_key[j + 1] >> idx_bits) != pane;
    const int64_t v = val[i_self];
    a.v.vt = VT;
    a.v.sum = v;
    a.v.mn = min_code(VT, s.cmpto, v);
    a.v.mx = max_code(VT, s.cmpto, v);
    a.v.cnt = 1;
    if (BY) { a.v.by = s.by | (s.by_last ? 1 : 0); a.v.ord = ord_base + i_self; a.v.f1 = f1col[i_self]; }
    a.empty = 0;
    a.head = head;
    a.sfirst = ord_base + i_self;
    // f1 by batch index (a random line per record): a segment takes its head's, so only heads need it, and
    // under PurgingTrigger, where every record's result carries its own
    if (FIRST && !BY && (head || purging)) a.sf1 = f1col[i_self];
    if (head) {
      const int64_t idx = (int64_t)pane;
      const bool pres = pane_present(s, idx);
      a.bpres = pres;
      if (pres) {
        a.v = wm_combine<VT, AGG>(wm_load<VT, AGG>(s, idx), a.v);
        if (FIRST && !BY) a.sf1 = s.c.f1v[idx];
      }
    }
  }
  // inclusive segmented scan over the tile (Hillis-Steele in LDS)
  lf_st<AGG>(&sp[threadIdx.x], a);
  __syncthreads();
  LfPart x = a;
  for (int o = 1; o < LF_T; o <<= 1) {
    LfPart y = x;
    if ((int)threadIdx.x >= o) y = lf_join<VT, AGG>(lf_ld<VT, AGG>(&sp[threadIdx.x - o]), x);
    __syncthreads();
    lf_st<AGG>(&sp[threadIdx.x], y);
    x = y;
    __syncthreads();
  }
  // the tile's carry from its predecessors (decoupled look-back), and the launch's output base
  if (threadIdx.x < 64) {   // wave 0
    const int lane = threadIdx.x;
    const LfPart agg = lf_ld<VT, AGG>(&sp[LF_T - 1]);
    const unsigned int ep = L.epoch << 2;
    if (lane == 0) {
      if (tile == 0) {
        __hip_atomic_store(&L.base[0], atomicAdd(s.o.count, (unsigned long long)nl), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&L.base[1], (unsigned long long)L.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (agg.head || tile == 0) {   // the inclusive prefix needs nothing before the tile's last head
        lf_put(&L.incl[tile], agg);
        lf_raise(&L.flag[tile], ep | 2u);
      } else {
        lf_put(&L.agg[tile], agg);
        lf_raise(&L.flag[tile], ep | 1u);
      }
    }
    LfPart c;
    c.empty = 1; c.head = 0; c.bpres = 0; c.sf1 = 0; c.sfirst = 0;
    // look back 64 tiles a step, one per lane, to the nearest inclusive prefix or segment head (none needed
    // when the tile's first record starts a segment)
    if (tile > 0 && !sp[0].head) {
      int64_t hi = tile - 1;
      while (true) {
        const int64_t t = hi - lane;
        LfPart e;
        e.empty = 1; e.head = 0; e.bpres = 0; e.sf1 = 0; e.sfirst = 0;
        bool stop = false;
        if (t >= 0) {
          unsigned int f;
          do { f = __hip_atomic_load(&L.flag[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); } while ((f & ~3u) != ep || (f & 3u) == 0);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          e = lf_get((f & 2u) ? L.incl + t : L.agg + t);
          stop = (f & 2u) || e.head;
        }
        const uint64_t sb = __ballot(stop);
        const int first_stop = sb ? __builtin_ctzll(sb) : 64;
        if (lane > first_stop) e.empty = 1;
        for (int off = 1; off < 64; off <<= 1) {   // lane 0: the lanes' parts joined, farthest first
          const LfPart o = lf_shfl_t<VT, AGG>(e, lane + off < 64 ? lane + off : lane);
          if (lane + off < 64) e = lf_join<VT, AGG>(o, e);
        }
        c = lf_join<VT, AGG>(lf_shfl_t<VT, AGG>(e, 0), c);
        if (sb || hi < 64) break;
        hi -= 64;
      }
    }
    if (lane == 0) {
      if (tile > 0 && !agg.head) {
        lf_put(&L.incl[tile], lf_join<VT, AGG>(c, agg));
        lf_raise(&L.flag[tile], ep | 2u);
      }
      while (__hip_atomic_load(&L.base[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)L.epoch) {
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      base_s = __hip_atomic_load(&L.base[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      carry_s = c;
    }
  }
  __syncthreads();
  if (j >= nl) return;
  const LfPart r = lf_join<VT, AGG>(carry_s, x);   // the record's running window content
  // PurgingTrigger: every fire purged the pane, so a record's result is itself (its segment's head: with the
  // pane's state before the batch; its f1 the pane's, else its own, as a.sf1 holds)
  const LateAcc out = purging ? a.v : r.v;
  const int64_t idx = (int64_t)pane;
  const int32_t p = (int32_t)(pane / (unsigned long long)s.stride);
  const int64_t kid = (int64_t)(pane % (unsigned long long)s.stride);
  int64_t f1 = 0;
  if (BY) f1 = out.f1;
  else if (FIRST) f1 = purging ? a.sf1 : r.sf1;
  emit_record(s, base_s + (unsigned long long)j, kid_key(s, kid), f1, slot_max_ts(s, p), out);
  if (!tail) return;
  // segment tail: the pane after the batch's per-element fires
  if (purging) {   // FIRE_AND_PURGE after the last element: the pane cleared, its cleanup timer kept (s.gfirst)
    if (s.gfirst) {
      int64_t o = s.first ? r.sfirst : 0;
      if (s.first && s.c.first[idx] < o) o = s.c.first[idx];
      if (o < s.gfirst[idx]) s.gfirst[idx] = o;
    }
    pane_clear(s, idx);
    return;
  }
  if (s.c.sum) s.c.sum[idx] = r.v.sum;
  if (s.c.mn) s.c.mn[idx] = r.v.mn;
  if (s.c.mx) s.c.mx[idx] = r.v.mx;
  if (s.c.cnt) s.c.cnt[idx] = BY ? r.v.ord : r.v.cnt;
  if (BY) s.c.f1v[idx] = r.v.f1;
  if (!r.bpres) {
    if (s.first) { s.c.first[idx] = r.sfirst; if (!BY) s.c.f1v[idx] = r.sf1; }
    else s.c.present[idx] = 1;
  }
}

// k_watermark's LDS, sized per engine (a small plan leaves the CU's LDS to the route and aggregate
// workgroups it runs beside): windows firing at one watermark are those holding a live slice (each slice
// lies in ceil(K / R) windows) or a window pane, at most WM_MAXT
__host__ __device__ inline int32_t wm_max_tasks(int32_t P, int32_t K, int32_t R, int32_t W) {
  const int64_t t = (int64_t)P * ((K + R - 1) / R) + W;
  return (int32_t)(t < WM_MAXT ? t : WM_MAXT);
}
__host__ __device__ inline size_t wm_lds_bytes(int32_t P, int32_t K, int32_t R, int32_t W) {
  return 8 * ((size_t)wm_max_tasks(P, K, R, W) + P) + 4 * ((size_t)P + K + (W > 0 ? W : 1)) + 16;
}

template <int VT, int AGG, bool FIRST>
__global__ __launch_bounds__(WM_THREADS) void k_watermark(Spec s, int64_t wm_old, int64_t wm_new, unsigned int* done) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int32_t maxt = wm_max_tasks(s.P, s.K, s.R, s.W);
  int64_t* task_n = (int64_t*)smem;                // [maxt]
  int64_t* tags = task_n + maxt;                   // [P] the slice tags, read once
  int32_t* purge = (int32_t*)(tags + s.P);         // [P]
  int32_t* slots = purge + s.P;                    // [K]
  int32_t* wpurge = slots + s.K;                   // [max(W, 1)]
  __shared__ int32_t n_tasks, n_purge, n_wpurge, wslot_t, last;
  __shared__ int64_t nkid_s;
  __shared__ int32_t wtot[WM_THREADS / 64];
  __shared__ unsigned long long base;
  __shared__ unsigned long long fired;
#define WM_STAMP(k) do { if (s.wm_stamps && threadIdx.x == 0) s.wm_stamps[(int64_t)blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
  WM_STAMP(0);
  if (threadIdx.x == 0) { n_tasks = 0; n_purge = 0; n_wpurge = 0; last = 0; fired = 0; }
  for (int32_t p = threadIdx.x; p < s.P; p += WM_THREADS) tags[p] = s.slice_tag[p];
  // key ids scanned: the null key's id D only while it is in use (D = 2^k ids fill 2^k / 1024 workgroups
  // exactly; id D would give workgroup 0 a second round of loads, ~4 us per fire)
  if (threadIdx.x == 0) nkid_s = s.dir_min_used[0] ? s.stride : s.D;
  __syncthreads();
  const int64_t nkid = nkid_s;
  // one thread per (slot, window of its slice) pair, not one per slot looping over its windows (a serial chain of
  // K windows x up to K owner checks per thread: the plan took 7-8 us per fire at C3's K = 10, round 6)
  // (tumbling, K = 1: a slot's one window in the purge loop below, no pair loop)
  const int32_t nw = (s.K + s.R - 1) / s.R + 1;   // windows of one slice, at most
  for (int32_t x = threadIdx.x; s.K > 1 && x < s.P * nw; x += WM_THREADS) {
    const int32_t p = x / nw, j = x - p * nw;
    const int64_t m = tags[p];
    if (m == FREE_TAG) continue;
    const int64_t n_hi = s.R == 1 ? m : floor_div(m, s.R);   // (64-bit divides: ~100 instructions each)
    const int64_t n_lo = s.R == 1 ? m - s.K + 1 : floor_div(m - s.K, s.R) + 1;
    const int64_t n = n_hi - j;
    if (n < n_lo) continue;
    const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
    const bool fires = max_ts > wm_old && max_ts <= wm_new;
    if (!fires) continue;
    bool owner = true;                                                    // first live slice of window n
    int32_t pp = (int32_t)floor_mod(n * s.R, s.P);
    for (int64_t mm = n * s.R; mm < m; ++mm) {
      if (tags[pp] == mm) { owner = false; break; }
      pp = pp + 1 == s.P ? 0 : pp + 1;
    }
    if (!owner) continue;
    const int32_t t = atomicAdd(&n_tasks, 1);
    if (t < maxt) task_n[t] = n;
    else cap_error(s, 12);
  }
  for (int32_t p = threadIdx.x; p < s.P; p += WM_THREADS) {
    const int64_t m = tags[p];
    if (m == FREE_TAG) continue;
    const int64_t n_hi = s.R == 1 ? m : floor_div(m, s.R);
    bool purge_now = false, fire_purge = false;
    if (s.K == 1 && n_hi * s.R == m) {   // tumbling (and K = 1 sliding): the slice is the window, its task here
      const int64_t max_ts = jsub(jadd(window_start_n(s, n_hi), s.size), 1);
      if (max_ts > wm_old && max_ts <= wm_new) {
        if (s.trigger == FW_TRIGGER_PURGING_EVENT_TIME && s.assigner == FW_TUMBLING) purge_now = fire_purge = true;
        const int32_t t = atomicAdd(&n_tasks, 1);
        if (t < maxt) task_n[t] = n_hi;
        else cap_error(s, 12);
      }
    }
    const int64_t ct = cleanup_time(jsub(jadd(window_start_n(s, n_hi), s.size), 1), s.lateness);
    if (ct <= wm_new) purge_now = true;
    if (purge_now) {
      const int32_t q = atomicAdd(&n_purge, 1);
      // a fire's purge keeps the panes' cleanup timers (as ghost ordinals) until the cleanup time
      const bool ghost = s.gfirst && fire_purge && ct > wm_new;
      if (q < s.P) purge[q] = p | (ghost ? PURGE_GHOST : 0);
    }
  }
  // window panes (sliding: the assigner's extra windows): a firing window without any live slice is a task
  // of its own; a pane whose window's cleanup time passed is purged
  for (int32_t w = threadIdx.x; w < s.W; w += WM_THREADS) {
    const int64_t n = s.wtag[w];
    if (n == FREE_TAG) continue;
    const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
    if (max_ts > wm_old && max_ts <= wm_new) {
      bool slice_live = false;
      for (int64_t mm = n * s.R; mm < n * s.R + s.K && !slice_live; ++mm) slice_live = tags[floor_mod(mm, s.P)] == mm;
      if (!slice_live) {
        const int32_t t = atomicAdd(&n_tasks, 1);
        if (t < maxt) task_n[t] = n;
        else cap_error(s, 12);
      }
    }
    if (cleanup_time(max_ts, s.lateness) <= wm_new) {
      const int32_t q = atomicAdd(&n_wpurge, 1);
      if (q < s.W) wpurge[q] = w;
    }
  }
  __syncthreads();
  WM_STAMP(1);
  const int32_t nt = min(n_tasks, maxt), np = min(n_purge, s.P), nwp = min(n_wpurge, s.W);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t gstride = (int64_t)gridDim.x * WM_THREADS;
  // windows of many slices: a key id without a key holds no pane, so its key is read first and gates the
  // slice loads (a quarter of the directory is live at the default load)
  const bool gate = s.K > 2;
  for (int32_t t = 0; t < nt; ++t) {
    const int64_t n = task_n[t];
    if (threadIdx.x < s.K) {
      const int64_t mm = n * s.R + threadIdx.x;
      const int32_t pp = (int32_t)floor_mod(mm, s.P);
      slots[threadIdx.x] = tags[pp] == mm ? pp : -1;
    }
    if (threadIdx.x == 0) wslot_t = wpane_slot(s, n);
    __syncthreads();
    const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
    // a restored window whose trigger timers fired before the checkpoint: only re-armed panes fire
    const int32_t p_dis =
        (s.disarm && s.assigner != FW_SLIDING && s.K == 1 && slots[0] >= 0 && s.disarm[slots[0]]) ? slots[0] : -1;
    // (sliding: a restored window's own pane disarmed — the window fires only for the keys re-armed since)
    const int32_t w_dis = (s.disarm && s.assigner == FW_SLIDING && wslot_t >= 0 && s.disarm[wslot_t]) ? wslot_t : -1;
    for (int64_t k0 = (int64_t)blockIdx.x * WM_THREADS; k0 < nkid; k0 += gstride) {
      const int64_t kid = k0 + threadIdx.x;
      bool any = false;
      LateAcc a;
      a.vt = VT;
      int64_t best_ord = INT64_MAX, f1 = 0;
      const int64_t key = kid < nkid ? kid_key(s, kid) : EMPTY_KEY;
      const bool live = kid < nkid && !(gate && kid != s.D && key == EMPTY_KEY) &&
                        (w_dis < 0 || s.armed[(int64_t)w_dis * s.stride + kid]);
      if (live) {
        for (int kb = 0; kb < s.K; kb += WM_C) {
          // the chunk's presence words in one round trip, then the present panes' columns in one more
          int64_t fo[WM_C];
#pragma unroll
          for (int j = 0; j < WM_C; ++j) {
            const int32_t v = kb + j < s.K ? slots[kb + j] : -1;
            fo[j] = INT64_MAX;
            if (v >= 0) {
              const int64_t idx = (int64_t)v * s.stride + kid;
              fo[j] = FIRST ? s.c.first[idx] : (s.c.present[idx] ? 0 : INT64_MAX);
            }
          }
          if (FIRST) {
            int jb = -1;
#pragma unroll
            for (int j = 0; j < WM_C; ++j) if (fo[j] < best_ord) { best_ord = fo[j]; jb = j; }
            if (jb >= 0) f1 = s.c.f1v[(int64_t)slots[kb + jb] * s.stride + kid];
          }
          LateAcc b[WM_C];
#pragma unroll
          for (int j = 0; j < WM_C; ++j) {
            if (fo[j] == INT64_MAX) continue;
            b[j] = wm_load<VT, AGG>(s, (int64_t)slots[kb + j] * s.stride + kid);
          }
#pragma unroll
          for (int j = 0; j < WM_C; ++j) {
            if (fo[j] == INT64_MAX) continue;
            if (p_dis < 0 || s.armed[(int64_t)slots[kb + j] * s.stride + kid]) {
              a = any ? wm_combine<VT, AGG>(a, b[j]) : b[j];
              any = true;
            }
          }
        }
        if (wslot_t >= 0) {   // the window's own pane
          const int64_t idx = (int64_t)wslot_t * s.stride + kid;
          if (cols_present(s, s.wc, idx)) {
            if (FIRST) {
              const int64_t o = s.wc.first[idx];
              if (o < best_ord) { best_ord = o; f1 = s.wc.f1v[idx]; }
            }
            const LateAcc b = cols_load(s, s.wc, idx);
            a = any ? LateCombine()(a, b) : b;
            any = true;
          }
        }
      }
      // block-aggregated append: one device atomic per workgroup and chunk
      const uint64_t bal = __ballot(any);
      const int32_t rank = __popcll(bal & lanemask_lt());
      if (lane == 0) wtot[wave] = __popcll(bal);
      __syncthreads();
      int32_t off = 0, tot = 0;
      for (int w = 0; w < WM_THREADS / 64; ++w) { const int32_t c = wtot[w]; off += w < wave ? c : 0; tot += c; }
      if (threadIdx.x == 0 && tot > 0) { base = atomicAdd(s.o.count, (unsigned long long)tot); fired += tot; }
      __syncthreads();
      if (any) emit_record(s, base + off + rank, key, s.by ? a.f1 : f1, max_ts, a);
    }
    __syncthreads();
  }
  WM_STAMP(2);
  // purge this workgroup's share of the expired slices (it fired that share above; clearing each pane as the
  // fire reads it writes partial column lines and measured slower beside the next batch's kernels)
  for (int32_t q = 0; q < np; ++q) {
    const bool ghost = (purge[q] & PURGE_GHOST) != 0;
    const int32_t p = purge[q] & ~PURGE_GHOST;
    const int64_t pbase = (int64_t)p * s.stride;
    for (int64_t kid = (int64_t)blockIdx.x * WM_THREADS + threadIdx.x; kid < nkid; kid += gstride) {
      const int64_t idx = pbase + kid;
      if (ghost) {
        const int64_t o = s.first ? s.c.first[idx] : (s.c.present[idx] ? 0 : INT64_MAX);
        if (o < s.gfirst[idx]) s.gfirst[idx] = o;
      }
      pane_clear(s, idx);
    }
  }
  for (int32_t q = 0; q < nwp; ++q) {
    const int64_t pbase = (int64_t)wpurge[q] * s.stride;
    for (int64_t kid = (int64_t)blockIdx.x * WM_THREADS + threadIdx.x; kid < nkid; kid += gstride) {
      const int64_t idx = pbase + kid;
      if (s.wc.sum) s.wc.sum[idx] = sum_identity(s.vt);
      if (s.wc.mn) s.wc.mn[idx] = INT64_MAX;
      if (s.wc.mx) s.wc.mx[idx] = INT64_MIN;
      if (s.wc.cnt) s.wc.cnt[idx] = 0;
      if (s.first) s.wc.first[idx] = INT64_MAX; else s.wc.present[idx] = 0;
    }
  }
  __syncthreads();
  WM_STAMP(3);
  if (threadIdx.x == 0) {
    if (fired) atomicAdd(&s.stats[ST_FIRED], fired);
    last = atomicAdd(done, 1u) == gridDim.x - 1;   // issued after this workgroup's appends returned
  }
  __syncthreads();
  if (!last) return;
  // last workgroup: free the purged slots, then record the watermark's position in the log
  for (int32_t q = threadIdx.x; q < np; q += WM_THREADS) s.slice_tag[purge[q] & ~PURGE_GHOST] = FREE_TAG;
  for (int32_t q = threadIdx.x; q < nwp; q += WM_THREADS) s.wtag[wpurge[q]] = FREE_TAG;
  if (threadIdx.x == 0) {
    *done = 0u;
    const unsigned long long cnt = atomicAdd(s.o.count, 0ull);
    const unsigned long long mc = *s.o.mark_count;
    if ((int64_t)mc < s.o.mark_capacity) {
      s.o.mark_wm[mc] = wm_new;
      s.o.mark_pos[mc] = (int64_t)(cnt < (unsigned long long)s.o.capacity ? cnt : (unsigned long long)s.o.capacity);
      *s.o.mark_count = mc + 1;
    } else {
      cap_error(s, 13);
    }
    // the directory's key count, for the host's compaction trigger (fw_advance_watermark)
    if (s.dir_keys_host)
      __hip_atomic_store(s.dir_keys_host, (unsigned)s.stats[ST_DIR_KEYS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------------------------------------------
// key directory compaction (unbounded key spaces).  The reference keeps no entry for a key once its
// last pane is cleared (AbstractHeapState.clear, AbstractHeapState.java:90-119, removes the key from the
// namespace's map and the namespace when empty): here a key leaves the directory once no live slice
// holds a pane of it.  One workgroup per directory bucket (probing never leaves a bucket): the bucket's
// live keys are re-inserted into a fresh linear-probe layout in LDS and their pane columns moved in every
// live slice; the evicted keys' key groups are remembered (their state tables stay "present" for a
// checkpoint, HeapKeyedStateBackend.java:228-233).  Launched after a firing watermark when the directory
// is more than half full; buckets of <= 4096 slots (LDS).
// ------------------------------------------------------------------------------------------------
constexpr int CP_THREADS = 1024;
__host__ __device__ constexpr size_t compact_lds_bytes(int kb_bits, int P) {
  return (size_t)(1 << kb_bits) * (8 + 8 + 8 + 2) + 8 * (size_t)P + 64;
}

__global__ __launch_bounds__(CP_THREADS) void k_compact(Spec s, unsigned char* kg_evicted) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int KB = 1 << s.kb_bits;
  const uint32_t kbm = (uint32_t)KB - 1;
  int64_t* okey = (int64_t*)smem;                 // [KB] the bucket's keys before
  int64_t* nkey = okey + KB;                      // [KB] after
  int64_t* tmp = nkey + KB;                       // [KB] one column of one slice
  int64_t* tags = tmp + KB;                       // [P] slice tags
  int16_t* inv = (int16_t*)(tags + s.P);          // [KB] new slot -> old slot (-1: empty)
  const int64_t dbase = (int64_t)blockIdx.x * KB;
  for (int p = threadIdx.x; p < s.P; p += CP_THREADS) tags[p] = s.slice_tag[p];
  for (int x = threadIdx.x; x < KB; x += CP_THREADS) {
    okey[x] = s.dir_keys[dbase + x];
    nkey[x] = EMPTY_KEY;
    inv[x] = -1;
  }
  __syncthreads();
  unsigned long long kept = 0;
  for (int x = threadIdx.x; x < KB; x += CP_THREADS) {
    const int64_t key = okey[x];
    if (key == EMPTY_KEY) continue;
    bool live = false;
    for (int p = 0; p < s.P && !live; ++p)
      if (tags[p] != FREE_TAG) live = pane_present(s, (int64_t)p * s.stride + dbase + x);
    for (int w = 0; w < s.W && !live; ++w)   // window panes (sliding extra windows)
      if (s.wtag[w] != FREE_TAG) live = cols_present(s, s.wc, (int64_t)w * s.stride + dbase + x);
    for (int p = 0; s.gtag && p < s.P && !live; ++p)   // cleanup timers of purged windows
      if (s.gtag[p] != FREE_TAG) live = s.gfirst[(int64_t)p * s.stride + dbase + x] != INT64_MAX;
    if (!live) {
      kg_evicted[key_group_for_hash(long_hash_code(key), s.mp)] = 1;
      continue;
    }
    // re-insert: the same probe sequence as dir_find_or_insert, in the fresh LDS layout
    uint32_t y = (uint32_t)fmix64((uint64_t)key) & kbm;
    for (;;) {
      const unsigned long long prev =
          atomicCAS((unsigned long long*)&nkey[y], (unsigned long long)EMPTY_KEY, (unsigned long long)key);
      if ((int64_t)prev == EMPTY_KEY) break;
      y = (y + 1) & kbm;
    }
    inv[y] = (int16_t)x;
    ++kept;
  }
  for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
  if ((threadIdx.x & 63) == 0 && kept) atomicAdd(&s.stats[ST_DIR_KEYS], kept);
  __syncthreads();
  // move the live slices' columns of this bucket: new slot y takes old slot inv[y]
  auto move = [&](int64_t* col, int64_t ident) {
    for (int p = 0; p < s.P; ++p) {   // uniform
      if (tags[p] == FREE_TAG) continue;
      int64_t* c = col + (int64_t)p * s.stride + dbase;
      for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
      __syncthreads();
      for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? tmp[inv[y]] : ident;
      __syncthreads();
    }
  };
  auto wmove = [&](int64_t* col, int64_t ident) {   // the window panes' columns likewise
    for (int w = 0; w < s.W; ++w) {   // uniform
      if (s.wtag[w] == FREE_TAG) continue;
      int64_t* c = col + (int64_t)w * s.stride + dbase;
      for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
      __syncthreads();
      for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? tmp[inv[y]] : ident;
      __syncthreads();
    }
  };
  if (s.W > 0) {
    if (s.wc.sum) wmove(s.wc.sum, sum_identity(s.vt));
    if (s.wc.mn) wmove(s.wc.mn, INT64_MAX);
    if (s.wc.mx) wmove(s.wc.mx, INT64_MIN);
    if (s.wc.cnt) wmove(s.wc.cnt, 0);
    if (s.first) { wmove(s.wc.first, INT64_MAX); wmove(s.wc.f1v, 0); }
    else {
      for (int w = 0; w < s.W; ++w) {
        if (s.wtag[w] == FREE_TAG) continue;
        unsigned char* c = s.wc.present + (int64_t)w * s.stride + dbase;
        for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
        __syncthreads();
        for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? (unsigned char)tmp[inv[y]] : 0;
        __syncthreads();
      }
    }
  }
  if (s.gtag)
    for (int p = 0; p < s.P; ++p) {   // uniform
      if (s.gtag[p] == FREE_TAG) continue;
      int64_t* c = s.gfirst + (int64_t)p * s.stride + dbase;
      for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
      __syncthreads();
      for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? tmp[inv[y]] : INT64_MAX;
      __syncthreads();
    }
  // re-arm marks of restored disarmed windows (tumbling: by slice slot, sliding: by window-pane slot; W = P): a
  // key's mark moves with its key id, or the window would fire for whichever key took the old id
  if (s.armed && s.disarm)
    for (int p = 0; p < s.P; ++p) {   // uniform
      if (!s.disarm[p]) continue;
      uint8_t* c = s.armed + (int64_t)p * s.stride + dbase;
      for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
      __syncthreads();
      for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? (uint8_t)tmp[inv[y]] : 0;
      __syncthreads();
    }
  if (s.c.sum) move(s.c.sum, sum_identity(s.vt));
  if (s.c.mn) move(s.c.mn, INT64_MAX);
  if (s.c.mx) move(s.c.mx, INT64_MIN);
  if (s.c.cnt) move(s.c.cnt, 0);
  if (s.first) {
    move(s.c.first, INT64_MAX);
    move(s.c.f1v, 0);
  } else {
    for (int p = 0; p < s.P; ++p) {
      if (tags[p] == FREE_TAG) continue;
      unsigned char* c = s.c.present + (int64_t)p * s.stride + dbase;
      for (int x = threadIdx.x; x < KB; x += CP_THREADS) tmp[x] = c[x];
      __syncthreads();
      for (int y = threadIdx.x; y < KB; y += CP_THREADS) c[y] = inv[y] >= 0 ? (unsigned char)tmp[inv[y]] : 0;
      __syncthreads();
    }
  }
  for (int y = threadIdx.x; y < KB; y += CP_THREADS) s.dir_keys[dbase + y] = nkey[y];
}

// the listed extra-window records into their window panes (one workgroup; the list is short): key id, the
// pane's slot for window qn, device-scope atomics on the window-pane columns, then f1 of each pane's first
// arrival.  Launched before every firing watermark of a sliding engine, so the panes are complete before
// their window fires (a record whose extra window had already fired is rejected at ingest).
__global__ __launch_bounds__(1024) void k_quirk_apply(Spec s, int64_t* list, unsigned long long* count, int64_t cap) {
  const int64_t n = min((int64_t)*count, cap);
  if (n == 0) return;   // the usual batch (timestamps past the offset by a slide have no extra window)
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    int64_t* q = list + e * QK_WORDS;
    const int64_t kid = dir_lookup(s, q[0]);
    const int32_t w = kid < 0 ? -1 : slice_slot_at(s.wtag, s.W, q[1]);
    if (kid < 0 || w < 0) { cap_error(s, 23); q[0] = -1; continue; }
    const int64_t idx = (int64_t)w * s.stride + kid;
    const int64_t v = q[2];
    if (s.wc.sum) {
      if (s.vt == FW_VALUE_I64) atomicAdd((unsigned long long*)&s.wc.sum[idx], (unsigned long long)v);
      else unsafeAtomicAdd((double*)&s.wc.sum[idx], __longlong_as_double(v));
    }
    if (s.wc.mn) atomicMin((long long*)&s.wc.mn[idx], (long long)min_code(s.vt, s.cmpto, v));
    if (s.wc.mx) atomicMax((long long*)&s.wc.mx[idx], (long long)max_code(s.vt, s.cmpto, v));
    if (s.wc.cnt) atomicAdd((unsigned long long*)&s.wc.cnt[idx], 1ull);
    if (s.first) atomicMin((long long*)&s.wc.first[idx], (long long)q[3]);
    else s.wc.present[idx] = 1;
    q[0] = idx;   // the pane, for the f1 pass
  }
  __threadfence();
  __syncthreads();
  if (s.first) {
    for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
      const int64_t* q = list + e * QK_WORDS;
      if (q[0] < 0) continue;
      if (__hip_atomic_load(&s.wc.first[q[0]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == q[3]) s.wc.f1v[q[0]] = q[4];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) *count = 0;
}

// asynchronous drain (fw_collect_begin), step 1 on the engine stream: the output log's rows and device marks since
// the last collect copied into device staging (column-major, `rows` per column; HBM to HBM), with hdr[0..3] = rows,
// device marks, fits, the engine's error word.  A log larger than the staging is left in place (fits = 0)
constexpr int DR_COLS = 8;   // key, f1, ts, sum, min, max, count, window start (those the log has, packed in this order)
__host__ __device__ __forceinline__ int dr_slot(uint32_t colmask, int c) { return __builtin_popcount(colmask & ((1u << c) - 1u)); }
__global__ __launch_bounds__(BLOCK) void k_drain(OutLog L, const int32_t* err, int64_t rows, int64_t* stage, int64_t* marks,
                                                 int64_t* hdr, unsigned int* done, uint32_t colmask) {
  __shared__ int64_t cnt_s[2];
  if (threadIdx.x == 0) { cnt_s[0] = (int64_t)*L.count; cnt_s[1] = (int64_t)*L.mark_count; }
  __syncthreads();
  const int64_t n = cnt_s[0], nm = cnt_s[1];
  const bool fits = n <= rows && n <= L.capacity && nm <= L.mark_capacity;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    hdr[0] = n;
    hdr[1] = nm;
    hdr[2] = fits ? 1 : 0;
    hdr[3] = *err;
  }
  // the log restarts once every block has read the counts: the last block to arrive resets them
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    *done = 0u;
    if (fits) { *L.count = 0; *L.mark_count = 0; }
  }
  if (!fits) return;
  const int64_t* src[DR_COLS] = {L.key, L.f1, L.ts, L.sum, L.mn, L.mx, L.cnt, L.win_start};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int c = 0; c < DR_COLS; ++c)
      if (src[c]) stage[(int64_t)dr_slot(colmask, c) * rows + i] = src[c][i];
  }
  if (blockIdx.x == 0)
    for (int64_t i = threadIdx.x; i < nm; i += blockDim.x) marks[i] = L.mark_pos[i];
}
// step 2 on the drain stream (beside the next batch's kernels): the staged rows, marks and header into the pinned
// host buffer (zero-copy stores over PCIe), only the columns present and only the rows staged
__global__ __launch_bounds__(BLOCK) void k_drain_host(const int64_t* stage, const int64_t* dmarks, const int64_t* dhdr,
                                                      int64_t rows, int64_t mark_cap, uint32_t colmask, int64_t* host) {
  const int64_t n = dhdr[2] ? dhdr[0] : 0, nm = dhdr[2] ? dhdr[1] : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
#pragma unroll
    for (int c = 0; c < DR_COLS; ++c)
      if ((colmask >> c) & 1u) {
        const int64_t o = (int64_t)dr_slot(colmask, c) * rows + i;
        host[o] = stage[o];
      }
  }
  int64_t* hmarks = host + (size_t)__builtin_popcount(colmask) * rows;
  if (blockIdx.x == 0) {
    for (int64_t i = threadIdx.x; i < nm; i += blockDim.x) hmarks[i] = dmarks[i];
    if (threadIdx.x < 4) hmarks[mark_cap + threadIdx.x] = dhdr[threadIdx.x];
  }
}

__global__ void k_mark_only(Spec s, int64_t wm) {
  unsigned long long mc = *s.o.mark_count;
  if ((int64_t)mc < s.o.mark_capacity) {
    unsigned long long cnt = *s.o.count;
    s.o.mark_wm[mc] = wm;
    s.o.mark_pos[mc] = (int64_t)(cnt < (unsigned long long)s.o.capacity ? cnt : (unsigned long long)s.o.capacity);
    *s.o.mark_count = mc + 1;
  } else {
    cap_error(s, 14);
  }
}

// fill helpers
__global__ void k_fill_i64(int64_t* p, int64_t v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// ------------------------------------------------------------------------------------------------
// checkpoint restore: one thread per snapshot entry (FW_SNAP_ENTRY_WORDS int64 words) inserts the key
// into the directory, claims the slice's slot and writes the pane — readStateTableForKeyGroup
// (HeapKeyedStateBackend.java:318-349) putting (namespace, key) -> state into the state table
// ------------------------------------------------------------------------------------------------
// wpane = 0: entries of slices (x[0] = slice number); 1: sliding windows' own panes (x[0] = window number, the
// reference layout's per-window state restored as it is)
__global__ void k_restore(Spec s, const int64_t* ent, int64_t n, int32_t wpane) {
  const Cols& c = wpane ? s.wc : s.c;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* x = ent + j * FW_SNAP_ENTRY_WORDS;
    const int64_t kid = dir_lookup(s, x[1]);
    if (wpane == 2) {   // a cleanup timer without state (purged window): its ghost ordinal (slot tag set by the host)
      if (kid < 0) { cap_error(s, 15); continue; }
      s.gfirst[floor_mod(x[0], s.P) * s.stride + kid] = x[6];
      continue;
    }
    const int32_t p = wpane ? slice_slot_at(s.wtag, s.W, x[0]) : slice_slot(s, x[0]);
    if (kid < 0 || p < 0) { cap_error(s, 15); continue; }
    const int64_t idx = (int64_t)p * s.stride + kid;
    if (c.sum) c.sum[idx] = x[2];
    if (c.mn) c.mn[idx] = x[3];
    if (c.mx) c.mx[idx] = x[4];
    if (c.cnt) c.cnt[idx] = x[5];
    if (s.first) { c.first[idx] = x[6]; c.f1v[idx] = x[7]; }
    else c.present[idx] = 1;
  }
}

// ------------------------------------------------------------------------------------------------
// keyBy routing (multi-GPU exchange): stable counting sort of records by operator index
// KeyGroupStreamPartitioner.selectChannels (SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:52-65)
// ------------------------------------------------------------------------------------------------
constexpr int PART_MAX = 64;
constexpr int PART_CHUNK = 4096;   // records per block (contiguous)

__device__ __forceinline__ int32_t route(const int64_t* key, const int32_t* kh, int64_t i, int32_t mp, int32_t par) {
  int32_t h = kh ? kh[i] : long_hash_code(key[i]);
  return operator_index_for_key_group(mp, par, key_group_for_hash(h, mp));
}

__global__ __launch_bounds__(BLOCK) void k_part_count(const int64_t* key, const int32_t* kh, int64_t n, int32_t mp,
                                                      int32_t par, int64_t* block_counts) {
  __shared__ int64_t cnt[PART_MAX];
  for (int d = threadIdx.x; d < par; d += blockDim.x) cnt[d] = 0;
  __syncthreads();
  int64_t lo = (int64_t)blockIdx.x * PART_CHUNK, hi = lo + PART_CHUNK < n ? lo + PART_CHUNK : n;
  // per-thread private counts of its records' destinations (few destinations: a thread's records are
  // counted in registers when par <= 8, then one LDS atomic per thread and destination)
  if (par <= 8) {
    int32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      const int32_t d = route(key, kh, i, mp, par);
#pragma unroll
      for (int q = 0; q < 8; ++q) c[q] += d == q ? 1 : 0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int32_t x = c[q];
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);   // wave total
      if ((threadIdx.x & 63) == 0 && x != 0) atomicAdd((unsigned long long*)&cnt[q], (unsigned long long)x);
    }
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd((unsigned long long*)&cnt[route(key, kh, i, mp, par)], 1ull);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < par; d += blockDim.x) block_counts[(int64_t)blockIdx.x * par + d] = cnt[d];
}

// one workgroup: per destination d (in output order), an exclusive scan of the blocks' counts (column d of
// [nblocks][par]) into per-block write offsets, after the totals of the destinations before d; totals and
// destination offsets out.  Output order: 0 .. par-1, or, with last >= 0, last + 1 .. par-1, 0 .. last (the
// records of operator `last` at the end: a receiver appends what its peers send right behind its own share)
constexpr int PART_SCAN_THREADS = 1024;
__global__ __launch_bounds__(PART_SCAN_THREADS) void k_part_scan(int64_t* block_counts, int64_t nblocks, int32_t par,
                                                                  int64_t* counts, int64_t* offsets, int32_t last) {
  __shared__ int64_t wtot[PART_SCAN_THREADS / 64];
  __shared__ int64_t base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t per = (nblocks + PART_SCAN_THREADS - 1) / PART_SCAN_THREADS;
  const int64_t b0 = (int64_t)threadIdx.x * per, b1 = min(b0 + per, nblocks);
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int32_t di = 0; di < par; ++di) {
    const int32_t d = last >= 0 ? (last + 1 + di) % par : di;
    int64_t sum = 0;
    for (int64_t b = b0; b < b1; ++b) sum += block_counts[b * par + d];
    int64_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int64_t run = base + incl - sum, total = 0;
    for (int w = 0; w < PART_SCAN_THREADS / 64; ++w) {
      run += w < wave ? wtot[w] : 0;
      total += wtot[w];
    }
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t c = block_counts[b * par + d];
      block_counts[b * par + d] = run;
      run += c;
    }
    __syncthreads();   // every thread has read base and wtot
    if (threadIdx.x == 0) {
      counts[d] = total;
      offsets[d] = base;
      base += total;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(BLOCK) void k_part_scatter(const int64_t* key, const int32_t* kh, const int64_t* f1,
                                                        const int64_t* ts, const int64_t* val, int64_t n, int32_t mp,
                                                        int32_t par, const int64_t* block_offsets, int64_t* okey,
                                                        int32_t* okh, int64_t* of1, int64_t* ots, int64_t* oval) {
  __shared__ int64_t base[PART_MAX];
  __shared__ int32_t wave_cnt[BLOCK / 64][PART_MAX];
  for (int d = threadIdx.x; d < par; d += blockDim.x) base[d] = block_offsets[(int64_t)blockIdx.x * par + d];
  __syncthreads();
  int64_t lo = (int64_t)blockIdx.x * PART_CHUNK, hi = lo + PART_CHUNK < n ? lo + PART_CHUNK : n;
  const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
  for (int64_t c0 = lo; c0 < hi; c0 += blockDim.x) {
    int64_t i = c0 + threadIdx.x;
    bool act = i < hi;
    int32_t dst = act ? route(key, kh, i, mp, par) : -1;
    int32_t rank = 0;
    for (int d = 0; d < par; ++d) {
      uint64_t m = __ballot(dst == d);
      if (dst == d) rank = __popcll(m & lanemask_lt());
      if (lane == 0) wave_cnt[wave][d] = __popcll(m);
    }
    __syncthreads();
    if (act) {
      int64_t pos = base[dst] + rank;
      for (int w = 0; w < wave; ++w) pos += wave_cnt[w][dst];
      okey[pos] = key[i];
      if (okh) okh[pos] = kh ? kh[i] : long_hash_code(key[i]);
      if (of1) of1[pos] = f1 ? f1[i] : ts[i];
      ots[pos] = ts[i];
      oval[pos] = val[i];
    }
    __syncthreads();
    for (int d = threadIdx.x; d < par; d += blockDim.x) {
      int32_t tot = 0;
      for (int w = 0; w < BLOCK / 64; ++w) tot += wave_cnt[w][d];
      base[d] += tot;
    }
    __syncthreads();
  }
}

}  // namespace fw


#include <mutex>
struct fw_engine;

// ==================================================================================================
// host side
// ==================================================================================================
using namespace fw;

namespace {

int64_t gcd64(int64_t a, int64_t b) { while (b) { int64_t t = a % b; a = b; b = t; } return a; }
int64_t next_pow2(int64_t x) { int64_t p = 1; while (p < x) p <<= 1; return p; }
int bits_for(uint64_t x) { int b = 0; while (b < 64 && (x >> b) != 0) ++b; return b; }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// list state (fw_list.hip): per pane slice slot a buffer of elements (kid, ordinal, value, f1)
constexpr int LST_WORDS = 4;   // a buffered list element: kid, arrival ordinal, value, f1
struct ListDev {
  int64_t cap;                  // elements per slice slot
  unsigned long long* cnt;      // [P] elements buffered
  int64_t* buf;                 // [P][cap][4]
  // allowed lateness: the batch's per-element re-fires (kid, window number, arrival ordinal)
  int64_t* fire;
  unsigned long long* fcnt;
  int64_t fcap;
};

// session windows (fw_session.hip): per key id `sw` window slots, key-major [D + 1][sw]
constexpr int SESS_SW_DEFAULT = 32, SESS_SW_MAX = 256;   // in-flight session windows per key
struct SessDev {
  int64_t gap;
  int32_t sw;
  int32_t nw;       // 64-bit words of a key's slot masks (1, 2 or 4)
  int64_t* start;   // window [start, end)
  int64_t* end;
  int64_t* sum;     // accumulator: sum (long / double bits), min / max codes, count
  int64_t* mn;
  int64_t* mx;
  int64_t* cnt;
  int64_t* f1;      // first-arrival f1 (keep_first_f1) / the extremal record's f1 (maxBy / minBy), or null
  unsigned long long* live;   // [D + 1] slots in flight
  unsigned long long* trig;   // [D + 1] slots whose trigger timer (at maxTimestamp) is pending
  // checkpoint bookkeeping (fw_snapshot_kg_flink; arrival ordinals, restored entries below zero in blob order):
  // per slot the state window's start (its end: start + gap — a state window is the window a session began as),
  // when that state window's "window-contents" entry was created, when the window was last put into
  // MergingWindowSet.windows, when its cleanup timer and its trigger timer were registered; per key when its
  // MergingWindowSet was first fetched (-1: not since the operator opened) with the first fired timer's time as
  // the tie-break of a watermark's fetches, and whether any of its records was accepted into a window
  int64_t *sws, *swc, *put, *cre, *tre;
  int64_t *ktouch, *ktts;
  int32_t* kacc;
  // a "window-contents" namespace (key group, state window) is shared by every key whose session began at that
  // instant; it lives while any of their entries does.  nscnt counts live entries per hashed (key group, state
  // window); an entry removed while its counter stays positive (possibly shared) is logged — key, state-window
  // start, creation and removal ordinals — so a snapshot can tell when the namespace's current instance began
  int32_t* nscnt;
  uint64_t nsmask;
  int64_t* nslog;
  unsigned long long* nslog_n;
  int64_t nslog_cap;
  // PurgingTrigger with allowed lateness: a purged session's cleanup timer outlives it (WindowOperator.cleanup
  // clears the state and the trigger timer only); logged as (key, start, end, registration ordinal)
  int64_t* olog;
  unsigned long long* olog_n;
  int64_t olog_cap;
  int32_t ckpt;     // checkpoint bookkeeping on (FW_SESS_CKPT=0: off; fw_snapshot_kg_flink / restore then fail)
  int64_t* rlist;   // slots a watermark retired (k_sess_wm -> k_sess_ns_retire)
  unsigned long long* rlist_n;
  int64_t rlist_cap;
  // list state (FW_AGG_LIST): per slot the window's elements as a linked list through an element pool of pcap
  // entries, handed out from a ring of free entry indices (freeq; pool[0] head, pool[1] end of the free ones,
  // pool[2] entries freed during the current launch, listed in fpend)
  int32_t list;
  int64_t* head;
  int64_t* tail;
  int64_t* len;
  int64_t *pv, *pf1, *pnext;
  int64_t *freeq, *fpend;
  unsigned long long* pool;
  int64_t pcap;
  // hot keys (a batch run of >= hot records, reducing state): walked by one wave each (k_sess_walk_hot)
  int32_t hot;
  int64_t* hot_list;                 // run heads (sorted positions)
  unsigned long long* hot_count;
};

// "window-contents" namespace bookkeeping (SessDev::nscnt / nslog): an entry created, an entry removed at ordinal r
__device__ __forceinline__ uint64_t sess_ns_slot(const SessDev& d, int32_t kg, int64_t sws) {
  return fmix64(((uint64_t)(uint32_t)kg << 48) ^ fmix64((uint64_t)sws)) & d.nsmask;
}
__device__ __forceinline__ void sess_ns_add(const SessDev& d, int32_t kg, int64_t sws) {
  atomicAdd(&d.nscnt[sess_ns_slot(d, kg, sws)], 1);
}
__device__ __forceinline__ void sess_ns_remove(const SessDev& d, int32_t kg, int64_t key, int64_t x, int64_t r) {
  const int64_t sws = d.sws[x];
  if (atomicSub(&d.nscnt[sess_ns_slot(d, kg, sws)], 1) <= 1) return;   // the namespace's last entry: it ends here
  const unsigned long long pos = atomicAdd(d.nslog_n, 1ull);
  if ((int64_t)pos >= d.nslog_cap) return;   // (overflow: the snapshot falls back to the oldest live entry)
  int64_t* l = d.nslog + 4 * pos;
  l[0] = key;
  l[1] = sws;
  l[2] = d.swc[x];
  l[3] = r;
}
__device__ __forceinline__ void sess_orphan(const SessDev& d, int64_t key, int64_t start, int64_t end, int64_t seq) {
  const unsigned long long pos = atomicAdd(d.olog_n, 1ull);
  if ((int64_t)pos >= d.olog_cap) return;   // (overflow: the snapshot reports FW_ERR_CAPACITY)
  int64_t* l = d.olog + 4 * pos;
  l[0] = key;
  l[1] = start;
  l[2] = end;
  l[3] = seq;
}


}  // namespace

struct fw_engine {
  fw_config cfg{};
  std::string err;
  int32_t sticky = FW_OK;
  hipStream_t stream = nullptr;       // engine stream: aggregation, watermarks, late path, output
  hipStream_t rstream = nullptr;      // route stream: k_route of batch j+1 overlaps k_aggregate/k_watermark of j
  void* client = nullptr;             // producer/consumer stream of the caller (fw_set_stream)
  bool has_client = false;            // set by fw_set_stream; the handle itself may be 0 (the null stream)
  bool serial = false;                // diagnostics (FW_SERIAL=1): k_route on the engine stream too
  bool no_consumed = false;           // diagnostics (FW_NO_CONSUMED=1): no per-push consumption event
  bool debug_late = false;            // FW_DEBUG_LATE=1: check every skipped late-count read-back (fires_possible)
  bool debug_sync = false;            // FW_DEBUG_SYNC=1: synchronise after each list / session launch, naming it
  bool event_query = true;            // skip stream waits on events already complete (FW_EVENT_QUERY=0: off)
  hipEvent_t ev_in = nullptr;         // client work up to a push (input columns ready)
  static constexpr int NCONS = 8;
  hipEvent_t ev_consumed[NCONS] = {};  // per push (ring): every read of that push's input columns done
  int64_t cons_push[NCONS] = {-1, -1, -1, -1, -1, -1, -1, -1};   // the push each ring event was recorded for
  // consumption events are recorded only once a caller has asked for one (fw_stream_wait_input): each is a
  // packet the command processor handles between the engine stream's kernels
  bool track_consumed = false;
  hipEvent_t ev_now = nullptr;
  hipEvent_t ev_hcopy = nullptr;      // host-column copies of a push done (system-scope fence kept)
  // routed batches rotate over NBUF buffer sets: k_route of batch j waits only for k_aggregate of batch
  // j - NBUF, long finished, so neither stream waits on the other's latest kernel (a cross-stream wait costs
  // ~13 us of signal latency on MI355X, measured: profiles/r02_v13_timeline.txt)
  static constexpr int NBUF = FW_NBUF;
  hipEvent_t ev_route[NBUF] = {};     // k_route of the batch using that buffer set done
  hipEvent_t ev_agg[NBUF] = {};       // k_aggregate of the batch using that buffer set done
  Spec s{};
  int64_t cur_wm = INT64_MIN;
  int64_t ordinal = 0;
  bool used_key_hash = false;         // a push carried Java key hashes: key groups are not derivable from keys
  bool restored = false;              // fw_restore_kg was called (fixes the watermark of every later restore)
  // restored tumbling windows (slice numbers) whose trigger timers fired before the checkpoint, still ahead of
  // the watermark (Spec::disarm / armed); and the restored windows that did carry their trigger timers
  std::set<int64_t> disarmed, armed_windows;
  // PurgingTrigger + allowed lateness: windows whose cleanup timers may outlive their state (Spec::gtag), each
  // held until the watermark reaches its cleanup time
  std::set<int64_t> ghost_windows;
  std::vector<std::vector<int64_t>> snap_gkg;   // per key group: (window, key, ordinal) of such timers
  std::set<std::pair<int64_t, int64_t>> snap_unarmed;   // build_snapshot: (slice, key) panes not re-armed
  // fw_snapshot_kg: entries of every key group, built once per engine state (state_epoch)
  int64_t state_epoch = 0, snap_epoch = -1;
  std::vector<std::vector<int64_t>> snap_kg;
  std::vector<std::vector<int64_t>> snap_wkg;   // sliding: the windows' own panes (entry word 0 = window number)
  std::vector<uint8_t> snap_has_key;   // per key group: a key of it is in the directory (it held window state)
  // list state (tumbling): each (window, key)'s elements as (arrival ordinal, value bits, f1), in arrival order
  std::map<std::pair<int64_t, int64_t>, std::vector<std::array<int64_t, 3>>> snap_list;
  bool snap_any_key = false;
  std::vector<uint8_t> kg_touched;     // per key group: restored with present = 1 (fw_restore_kg_flink)
  int64_t restore_ord = -((int64_t)1 << 62);   // arrival ordinals of restored panes, in blob order
  // fw_restore_kg_flink: each restored timer's position in the timer sections (restoreTimersForKeyGroup adds
  // them to the set in that order, so later snapshots list them in it within a hash bucket)
  std::map<std::array<int64_t, 4>, int64_t> restored_timer_rank;
  // sliding-window list state restored in the reference layout: each (window start, key) entry's place in its
  // namespace's insertion order (blob order; the elements' ordinals follow the merged arrival order instead)
  std::map<std::pair<int64_t, int64_t>, int64_t> list_entry_rank;
  // sliding windows under PurgingTrigger with allowed lateness: a fired window's state is purged (its slices stay
  // for the windows sharing them) while each key whose first element preceded the fire keeps its cleanup timer.
  // adv_log: (watermark, arrival ordinal) of each advance (and of the restore), to tell when a window fired;
  // sl_ghost: restored cleanup timers without state, (window start, key)
  std::vector<std::pair<int64_t, int64_t>> adv_log;
  std::set<std::pair<int64_t, int64_t>> sl_ghost;
  // session windows' checkpoints: the state tables a restore brought, per key group whether its
  // "merging-window-set" map exists (a snapshot wrote an entry or a restore read it present), the restored
  // merging-window-set entries (key -> rank in blob order), and the device state read back for snapshots
  bool sess_wc_table = false, sess_mws_table = false;
  std::vector<uint8_t> mws_created;
  std::map<int64_t, int64_t> sess_mws_rank;
  // PurgingTrigger with allowed lateness: purged sessions' cleanup timers — drained from the device log
  // (key, start, end, registration ordinal) and restored ones (key, start, end); the (watermark, ordinal) of each
  // advance; keys whose set a restored timer fetched when it fired (key -> (ordinal, timer time))
  std::vector<std::array<int64_t, 4>> sess_orphans;
  std::set<std::array<int64_t, 3>> sess_rorphans;
  std::vector<std::pair<int64_t, int64_t>> sess_adv;
  std::map<int64_t, std::pair<int64_t, int64_t>> sess_touch_adj;
  int64_t sess_pool_used = 0;   // session list state: pool entries a restore laid elements in
  struct SessHost {
    int64_t epoch = -1, wm = 0;
    std::vector<int64_t> keys, st, en, sws, swc, put, cre, tre, sum, mn, mx, cnt, f1, ktouch, ktts, nslog;
    std::vector<int64_t> lhead, llen, pv, pf1, pnext;   // list state: per slot its element chain; the pool
    bool nslog_over = false;
    std::vector<int32_t> kacc;
    std::vector<unsigned long long> live, trig;
  } sess_host;
  int64_t records_in = 0;
  int64_t pushes = 0;                 // non-empty pushes (ev_consumed ring position)
  int grid = 0;
  std::vector<void*> allocs;
  // staging for host-memory (and misaligned device) pushes, one set per batch parity
  int64_t *stg_key[NBUF] = {}, *stg_ts[NBUF] = {}, *stg_val[NBUF] = {}, *stg_f1[NBUF] = {};
  int32_t* stg_hash[NBUF] = {};
  // late path
  unsigned long long *late_key = nullptr, *late_key_sorted = nullptr, *late_count = nullptr, *seg = nullptr;
  bool by_direct = false;                      // maxBy / minBy on the direct form (by_key folded after each launch)
  unsigned long long *by_key = nullptr, *by_count = nullptr;
  unsigned long long* out_base = nullptr;   // first output slot reserved for a per-element emit kernel
  unsigned long long *fire_key = nullptr, *fire_count = nullptr;   // sliding: per-element fire elements
  int64_t fire_cap = 0;
  unsigned long long *late_idx_in = nullptr, *late_idx_out = nullptr;
  LateAcc *late_acc = nullptr, *late_scan = nullptr;
  int64_t *headpos = nullptr, *headpos_scan = nullptr;
  SegPart* seg_tiles = nullptr;   // the late scan's per-tile aggregates, then carries
  SegPart* seg_groups = nullptr;  // ... and per group of LS_CT tiles (two-level carries)
  int32_t* seg_first = nullptr;   // ... and first segment head per tile
  // tumbling per-element fires in one pass (k_late_fused): per-tile look-back links, launch epochs, tickets
  bool late_fused = true;
  unsigned int* lf_flag = nullptr;
  LfPart *lf_agg = nullptr, *lf_incl = nullptr;
  unsigned long long* lf_base = nullptr;
  unsigned int* lf_ticket = nullptr;
  unsigned int lf_ticket0 = 0, lf_epoch = 0;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  int32_t idx_bits = 0;
  int64_t late_fires_host = 0;
  // device-time accounting (fw_set_profiling)
  bool profiling = false;
  struct Timed { int phase; hipEvent_t a, b; int64_t records; };
  std::vector<Timed> timed;
  std::vector<hipEvent_t> event_pool;
  double prof_ms[FW_NPHASES] = {};
  int64_t prof_launches[FW_NPHASES] = {};
  int64_t prof_records[FW_NPHASES] = {};
  hipEvent_t take_event() {
    hipEvent_t ev = nullptr;
    if (!event_pool.empty()) { ev = event_pool.back(); event_pool.pop_back(); }
    else (void)hipEventCreate(&ev);
    return ev;
  }
  int open_phase = -1;
  hipEvent_t open_ev = nullptr;
  void phase_begin(int ph, hipStream_t st = nullptr) {
    if (!profiling) return;
    open_phase = ph;
    open_ev = take_event();
    (void)hipEventRecord(open_ev, st ? st : stream);
  }
  void phase_end(int64_t records, hipStream_t st = nullptr) {
    if (!profiling || open_phase < 0) return;
    hipEvent_t b = take_event();
    (void)hipEventRecord(b, st ? st : stream);
    timed.push_back({open_phase, open_ev, b, records});
    open_phase = -1;
  }
  unsigned int* wm_done = nullptr;   // k_watermark's workgroup completion counter
  // partitioned ingest (ingest_mode 2)
  bool routed = false;
  RouteBuf rb{};                            // fields shared by both parities (dbg, stamps)
  RouteBuf rbs[NBUF] = {};                  // routed-batch buffers, one set per buffer slot
  unsigned int* dflags = nullptr;           // direct-record flags, a ring of FLAG_RING
  unsigned int* bload = nullptr;            // [4][RT_MAXNB] routed records per bucket and batch (k_aggregate split plan)
  unsigned int* fold_flag = nullptr;        // [5][RT_MAXNB][RT_GS]: chained-fold flags, concurrent-fold count ring
  unsigned int* bload_host = nullptr;       // host-mapped [RT_MAXNB], written by k_aggregate's owners
  // key directory compaction
  unsigned char* kg_evicted = nullptr;      // [max_parallelism] a key of the key group was evicted
  unsigned int* dir_keys_host = nullptr;    // host-mapped: keys in the directory at the last firing watermark
  bool compact_ok = false;
  size_t compact_lds = 0;
  double compact_fill = 0.5;                // FW_COMPACT_FILL
  int64_t compactions = 0;
  // fw_decode scratch (grow-only)
  // fw_decode scratch: one slot per decode in flight (fw_decode_begin / fw_decode_end)
  struct DecSlot {
    void *small = nullptr, *bytes = nullptr;   // chunk tables; a host input's device copy
    size_t small_cap = 0, bytes_cap = 0;
    int64_t* pin = nullptr;                    // pinned, mapped: the totals and the error word (k_dec_emit posts them)
    int64_t* pin_dev = nullptr;                // the same words as the device sees them
    hipEvent_t done = nullptr;
    bool pending = false, empty = false;
    int32_t ticket = -1;
    int64_t record_cap = 0, marker_cap = 0;
  };
  static constexpr int NDEC = 2;
  DecSlot dec[NDEC];
  int64_t dec_seq = 0;
  int agg_helpers_max = RT_MAXNB;           // FW_AGG_HELPERS (0: never split a bucket)
  int agg_split = AG_SPLIT_CHAIN;           // shares per hot bucket, at most (FW_AGG_SPLIT)
  int agg_chunk_pct = 200;                  // records per share: at least this % of the mean load (FW_AGG_CHUNK_PCT)
  // sliding: the assigner's extra-window records, one list per routed buffer set (fw_push_batch applies
  // a batch's list right after its ingest, on the engine stream)
  int64_t* quirk_list[NBUF] = {};
  unsigned long long* quirk_count = nullptr;
  // list state (FW_AGG_LIST, fw_list.hip)
  bool list = false;
  ListDev lst{};
  int64_t* list_plan = nullptr;            // k_list_plan's output (device), copied to list_plan_h
  std::vector<int64_t> list_plan_h;
  unsigned long long *list_k1 = nullptr, *list_k2 = nullptr;   // sort keys (ordinal, then kid)
  int64_t *list_v1 = nullptr, *list_v2 = nullptr;              // element indices
  void* list_temp = nullptr;
  size_t list_temp_bytes = 0;
  int64_t list_tmp_cap = 0;
  int64_t* list_fire_dp = nullptr;   // list re-fires: (kid, arrival) pairs, counts, offsets (grow-only)
  int64_t list_fire_cap = 0;
  int64_t list_out = 0;                    // results appended since the last collect
  // session windows (FW_SESSION, fw_session.hip)
  bool session = false;
  SessDev sess{};
  unsigned long long *sess_key = nullptr, *sess_sorted = nullptr;
  void* sess_temp = nullptr;
  size_t sess_temp_bytes = 0;
  int32_t sess_idx_bits = 0, sess_key_bits = 0;
  int64_t batches = 0;
  int32_t max_tiles = 0;
  size_t route_lds = 0, agg_lds = 0;
  int agg_min_lds = 81 * 1024;
  hipError_t attr_err = hipSuccess;         // routed_attrs_t: a failed hipFuncSetAttribute
  Spec* s_dev = nullptr;                    // routed form: device copy of s (k_route), re-uploaded when s changes
  // partition scratch
  int64_t* new_list = nullptr;                // direct form with first arrival: panes created per batch
  unsigned long long* new_counts = nullptr;   // one list length per batch parity
  int64_t* part_block_counts = nullptr;
  int64_t part_blocks_cap = 0;
  // host output copies
  std::vector<int64_t> h_key, h_f1, h_ts, h_sum, h_mn, h_mx, h_cnt, h_mark_wm, h_mark_pos, h_dev_pos, h_start;
  // fw_collect(FW_MEM_HOST): pinned staging of the result columns (DMA copies, one wait), grown on demand up
  // to COLLECT_PIN_MAX rows (larger drains use pageable vectors); two pinned words for the counts
  static constexpr int64_t COLLECT_PIN_MAX = 1 << 22;
  static constexpr int64_t DRAIN_ROWS_MAX = 1 << 25;   // results one asynchronous drain holds at most
  int64_t* h_pin = nullptr;
  int64_t h_pin_rows = 0;
  unsigned long long* h_pin_cnt = nullptr;
  // watermark marks since the last collect, in emission order.  A firing watermark's kernel (and a
  // k_mark_only) writes a device mark; a quiet watermark with no output appended since the previous
  // device mark launches nothing: its position is that mark's (dev < 0: the start of the log)
  struct HostMark { int64_t wm; int64_t dev; bool own; };
  std::vector<HostMark> hmarks;
  int64_t dev_marks = 0;        // device marks enqueued since the last collect
  bool out_dirty = false;       // output appended (per-element fires) after the last device mark
  std::vector<double> h_sum_d, h_mn_d, h_mx_d;
  // asynchronous drains (fw_collect_begin / fw_collect_end): NDRAIN pinned host staging buffers, in turn
  struct Drain {
    int64_t* host = nullptr;        // [log columns][rows], then [mark_capacity] device mark positions, then hdr[4]
    int64_t* dptr = nullptr;        // the same memory as the device sees it
    int64_t* dev = nullptr;         // device staging of the same layout (k_drain's copy)
    hipEvent_t staged = nullptr;    // the engine stream's copy done (the drain stream waits for it)
    hipEvent_t done = nullptr;
    bool pending = false;           // begun, not yet ended
    int32_t ticket = -1;            // the ticket fw_collect_begin handed out for it
    bool host_ready = false;        // the device arrival counter initialised
    std::vector<HostMark> marks;    // the host marks of the drain
    int64_t dev_marks = 0;
    std::vector<int64_t> mark_wm, mark_pos;
  };
  static constexpr int NDRAIN = 3;   // drains outstanding at once
  Drain drains[NDRAIN];
  hipStream_t dstream = nullptr;     // drain stream: staged results to pinned host memory beside the next batches
  int64_t drain_rows = 0;
  int64_t drain_seq = 0;
  int dev = 0;

  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) > 0 ? n * sizeof(T) : 1) != hipSuccess) return nullptr;
    allocs.push_back(p);
    return (T*)p;
  }
  ~fw_engine() {
    if (rstream) (void)hipStreamSynchronize(rstream);
    if (stream) (void)hipStreamSynchronize(stream);
    if (rstream) (void)hipStreamDestroy(rstream);
    if (stream) (void)hipStreamDestroy(stream);
    if (ev_in) (void)hipEventDestroy(ev_in);
    for (int q = 0; q < NBUF; ++q) for (hipEvent_t ev : {ev_route[q], ev_agg[q]}) if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : ev_consumed) if (ev) (void)hipEventDestroy(ev);
    if (ev_now) (void)hipEventDestroy(ev_now);
    if (ev_hcopy) (void)hipEventDestroy(ev_hcopy);
    for (auto& t : timed) { (void)hipEventDestroy(t.a); (void)hipEventDestroy(t.b); }
    for (auto ev : event_pool) (void)hipEventDestroy(ev);
    for (void* p : allocs) (void)hipFree(p);
    if (bload_host) (void)hipHostFree(bload_host);
    if (dir_keys_host) (void)hipHostFree(dir_keys_host);
    for (auto& ds : dec) {
      for (void* p : {ds.small, ds.bytes}) if (p) (void)hipFree(p);
      if (ds.pin) (void)hipHostFree(ds.pin);
      if (ds.done) (void)hipEventDestroy(ds.done);
    }
    if (h_pin) (void)hipHostFree(h_pin);
    if (dstream) { (void)hipStreamSynchronize(dstream); (void)hipStreamDestroy(dstream); }
    for (auto& d : drains) {
      if (d.host) (void)hipHostFree(d.host);
      if (d.dev) (void)hipFree(d.dev);
      if (d.done) (void)hipEventDestroy(d.done);
      if (d.staged) (void)hipEventDestroy(d.staged);
    }
    if (h_pin_cnt) (void)hipHostFree(h_pin_cnt);
    for (void* p : {(void*)list_k1, (void*)list_k2, (void*)list_v1, (void*)list_v2, list_temp, (void*)list_fire_dp})
      if (p) (void)hipFree(p);
  }
};

static thread_local std::string g_create_error;

// session windows (fw_session.hip)
int session_create(fw_engine* e);
int session_push(fw_engine* e, const fw::BatchIn& b);
int session_watermark(fw_engine* e, int64_t wm);
// list state (fw_list.hip)
int list_create(fw_engine* e);
int list_push(fw_engine* e, const fw::BatchIn& b);
int list_watermark(fw_engine* e, int64_t wm);

static int fail(fw_engine* e, int code, const std::string& msg) {
  if (e) { e->err = msg; if (e->sticky == FW_OK) e->sticky = code; }
  return code;
}
#define HIPCHK(e, x) do { hipError_t _r = (x); if (_r != hipSuccess) \
  return fail(e, FW_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(_r)); } while (0)
// diagnostics (FW_DEBUG_SYNC=1): the launch just made, waited for and named when it failed
#define DBGSYNC(e, what) do { if ((e)->debug_sync) { hipError_t _r = hipGetLastError(); \
  if (_r == hipSuccess) _r = hipStreamSynchronize((e)->stream); \
  if (_r != hipSuccess) return fail(e, FW_ERR_DEVICE, std::string("after ") + (what) + ": " + hipGetErrorString(_r)); } } while (0)

// the engine stream orders the copy before every later kernel; the host copy is the engine's own (stable)
static int upload_spec(fw_engine* e) {
  if (!e->s_dev) return FW_OK;
  HIPCHK(e, hipMemcpyAsync(e->s_dev, &e->s, sizeof(Spec), hipMemcpyHostToDevice, e->stream));
  return FW_OK;
}

static int launch_fill(fw_engine* e, int64_t* p, int64_t v, int64_t n) {
  if (!p || n <= 0) return FW_OK;
  int blocks = (int)std::min<int64_t>((n + BLOCK - 1) / BLOCK, 4096);
  hipLaunchKernelGGL(k_fill_i64, dim3(blocks), dim3(BLOCK), 0, e->stream, p, v, n);
  return FW_OK;
}

template <int VT, int AGG, bool FIRST>
static void launch_ingest_t(fw_engine* e, const BatchIn& b) {
  int blocks = (int)std::min<int64_t>((b.n + BLOCK - 1) / BLOCK, e->grid);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((k_ingest_direct<VT, AGG, FIRST>), dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, b);
}
// the routed kernels use dynamic LDS only, so the whole 160 KiB is grantable: the largest any engine may ask for,
// set once per device and instantiation (engines may be created from several threads), from fw_create, which
// fails with the HIP error when the attribute cannot be set
template <int VT, int AGG, bool FIRST>
static void routed_attrs_t(fw_engine* e) {
  static std::mutex mu;
  static std::set<int> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count(e->dev)) return;
  const void* fns[] = {(const void*)k_route<VT, AGG, FIRST>, (const void*)k_aggregate<VT, AGG, FIRST, false>,
                       (const void*)k_aggregate<VT, AGG, FIRST, true>};
  for (const void* f : fns) {
    const hipError_t rc = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (rc != hipSuccess) { e->attr_err = rc; return; }
  }
  done.insert(e->dev);
}

// k_watermark's plan grows to ~112 KiB of LDS at the largest P and K (dynamic LDS past 64 KiB needs the attribute)
template <int VT, int AGG, bool FIRST>
static void wm_attrs_t(fw_engine* e) {
  static std::mutex mu;
  static std::set<int> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count(e->dev)) return;
  const hipError_t rc = hipFuncSetAttribute((const void*)k_watermark<VT, AGG, FIRST>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)wm_lds_bytes(MAX_P, MAX_K, 1, MAX_P));
  if (rc != hipSuccess) { e->attr_err = rc; return; }
  done.insert(e->dev);
}

template <int VT, int AGG, bool FIRST>
static void launch_routed_t(fw_engine* e, const BatchIn& b, const int64_t* f1col, int par) {
  RouteBuf r = e->rbs[par];
  r.ntiles = (int32_t)((b.n + RT_TILE - 1) / RT_TILE);
  r.dflag = e->dflags + (e->batches % FLAG_RING);
  r.dflag_reset = e->dflags + ((e->batches + FLAG_RING / 2) % FLAG_RING);
  // helpers for hot buckets: as many as the same plan asks for on the loads the owners posted (read
  // without a sync: a batch or two stale at most; each launch's device plan caps itself at the helpers
  // it got)
  int wanted = 0;
  if (e->bload_host && e->agg_helpers_max > 0) {
    uint64_t all = 0;
    for (int x = 0; x < e->s.nb; ++x) all += __atomic_load_n(&e->bload_host[x], __ATOMIC_RELAXED);
    const uint32_t cmin = (e->rb.dbg & 64) ? 256u : AG_SPLIT_MIN;
    const uint64_t chunk = std::max<uint64_t>(cmin, ((all / (uint64_t)e->s.nb + 1) * (uint64_t)e->agg_chunk_pct) / 100);
    for (int x = 0; x < e->s.nb; ++x) {
      const uint64_t sh = std::min<uint64_t>((__atomic_load_n(&e->bload_host[x], __ATOMIC_RELAXED) + chunk - 1) / chunk,
                                             (uint64_t)e->agg_split);
      wanted += sh > 1 ? (int)sh - 1 : 0;
    }
  }
  r.helpers = std::min(e->agg_helpers_max, wanted);
  r.split_max = e->agg_split;
  r.chunk_pct = e->agg_chunk_pct;
  r.bload_prev = e->bload + ((e->batches + 3) % 4) * RT_MAXNB;
  r.bload_cur = e->bload + (e->batches % 4) * RT_MAXNB;
  r.bload_zero = e->bload + ((e->batches + 2) % 4) * RT_MAXNB;
  r.fold_flag = e->fold_flag;
  r.fold_cnt = e->fold_flag + (size_t)(1 + e->batches % 4) * RT_MAXNB * RT_GS;
  r.fold_cnt_zero = e->fold_flag + (size_t)(1 + (e->batches + 2) % 4) * RT_MAXNB * RT_GS;
  r.bload_host = e->bload_host;
  r.tag = (uint32_t)((e->batches + 1) & 0x7FFFFFF);
  // at least 81 KiB of LDS: one k_aggregate workgroup per CU (the dispatcher would otherwise pair two
  // of the nb = CU-count workgroups on one CU and leave another idle)
  const size_t agg_lds = std::max<size_t>(e->agg_lds - (size_t)(e->max_tiles - r.ntiles) * 8, (size_t)e->agg_min_lds);
  hipStream_t rs = e->serial ? e->stream : e->rstream;
  const AggSpec sa{e->s.nb, e->s.kb_bits, e->s.P, e->s.by_last, e->s.cmpto, e->s.stride, e->s.D, e->s.dir_keys, e->s.slice_tag,
                   e->s.dir_min_used, e->s.err, e->s.stats, e->s.c};
  e->phase_begin(FW_PHASE_INGEST, rs);
  const Spec& sp = e->s;
  const RouteSpec q{sp.assigner, sp.K, sp.R, sp.mp, sp.kg_start, sp.kg_end, sp.mp_mask, sp.kb_bits, sp.nb,
                    sp.size, sp.slide, sp.offset, sp.lateness, sp.g, sp.inv_size, sp.inv_g, sp.dir_mask, sp.err, sp.stats};
  hipLaunchKernelGGL((k_route<VT, AGG, FIRST>), dim3(r.ntiles), dim3(RT_THREADS), e->route_lds, rs, e->s_dev, q, b, r);
  e->phase_end(b.n, rs);
  (void)hipEventRecord(e->ev_route[par], rs);
  (void)hipStreamWaitEvent(e->stream, e->ev_route[par], 0);
  e->phase_begin(FW_PHASE_AGGREGATE);
  if (r.helpers > 0)
    hipLaunchKernelGGL((k_aggregate<VT, AGG, FIRST, true>), dim3(e->s.nb + r.helpers), dim3(AG_THREADS), agg_lds, e->stream,
                       e->s_dev, sa, b, r, f1col);
  else
    hipLaunchKernelGGL((k_aggregate<VT, AGG, FIRST, false>), dim3(e->s.nb), dim3(AG_THREADS), agg_lds, e->stream,
                       e->s_dev, sa, b, r,
                       f1col);
  e->phase_end(b.n);
  // (ev_agg[par] is recorded by fw_push_batch once the batch's extra-window list is applied too)
}

// no window of the assigner has its maxTimestamp or its cleanup time in (old, new]: the advance fires
// and purges nothing (a live slice's fire and cleanup times lie above the watermark it was created
// under), only the watermark's mark is due.  Conservative near the int64 edges.
static bool wm_quiet(const Spec& s, int64_t old_wm, int64_t new_wm) {
  const int64_t lim = (int64_t)1 << 61;
  if (old_wm <= -lim || new_wm >= lim || s.lateness >= lim || s.size >= lim || s.offset <= -lim || s.offset >= lim)
    return false;
  const __int128 d = s.assigner == FW_TUMBLING ? s.size : s.slide;
  auto fdiv = [](__int128 x, __int128 y) { __int128 q = x / y; if (x % y != 0 && x < 0) --q; return q; };
  auto crosses = [&](__int128 a) { return fdiv((__int128)new_wm - a, d) != fdiv((__int128)old_wm - a, d); };
  const __int128 a = (__int128)s.offset + s.size - 1;   // maxTimestamp of window n is a + n * d
  return !crosses(a) && !crosses(a + s.lateness);
}

// can a record pushed under watermark wm be a per-element fire (a window of it with maxTimestamp <= wm <
// cleanup time, WindowOperator.java:302-325)?  Window maxTimestamps are a + n d, so only if the latest one
// at or below wm lies within the allowed lateness of wm.  If not, the push needs no late-record count
// read-back (a host sync per batch that kept the next k_route from overlapping).  Conservative near the
// int64 edges.
static bool fires_possible(const Spec& s, int64_t wm) {
  const int64_t lim = (int64_t)1 << 61;
  if (wm <= -lim || wm >= lim || s.lateness >= lim || s.size >= lim || s.offset <= -lim || s.offset >= lim)
    return true;
  const __int128 d = s.assigner == FW_TUMBLING ? s.size : s.slide;
  const __int128 a = (__int128)s.offset + s.size - 1;
  __int128 r = ((__int128)wm - a) % d;   // wm minus the latest maxTimestamp <= wm
  if (r < 0) r += d;
  return r < (__int128)s.lateness;
}

template <int VT, int AGG, bool FIRST>
static void launch_late_fused_t(fw_engine* e, int64_t nl, const int64_t* dv, const int64_t* df1) {
  const unsigned int ntiles = (unsigned int)((nl + LF_T - 1) / LF_T);
  const LfLink L{e->lf_flag, e->lf_agg, e->lf_incl, e->lf_base, e->lf_ticket, e->lf_ticket0, ++e->lf_epoch};
  hipLaunchKernelGGL((k_late_fused<VT, AGG, FIRST>), dim3(ntiles), dim3(LF_T), 0, e->stream, e->s, e->late_key_sorted, nl,
                     e->idx_bits, dv, df1, e->ordinal, L);
  e->lf_ticket0 += ntiles;   // (the ticket counter wraps with it)
}

template <int VT, int AGG, bool FIRST>
static void launch_watermark_t(fw_engine* e, int64_t wm_old, int64_t wm_new) {
  // (one workgroup per CU: a 257th for the null key's id D = 2^k measured ~4 us slower per fire than workgroup 0
  // taking that id's chunk too)
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((e->s.stride + WM_THREADS - 1) / WM_THREADS, e->grid / 8));
  hipLaunchKernelGGL((k_watermark<VT, AGG, FIRST>), dim3(blocks), dim3(WM_THREADS),
                     wm_lds_bytes(e->s.P, e->s.K, e->s.R, e->s.W), e->stream, e->s, wm_old, wm_new, e->wm_done);
}

// dispatch over (value type, aggregate mask, first-arrival) — the instantiated reduce shapes
#ifdef FW_DISPATCH_C1_ONLY   // register / spill experiments: the C1 shape only (a library that serves nothing else)
#define FW_DISPATCH(FN, e, ...) FN<0, 1, true>(e, ##__VA_ARGS__)
#else
#define FW_DISPATCH(FN, e, ...)                                                                  \
  do {                                                                                           \
    const Spec& _s = (e)->s;                                                                     \
    const bool _f = _s.first != 0;                                                               \
    if (_s.vt == FW_VALUE_I64) {                                                                 \
      switch (_s.agg) {                                                                          \
        case 1: if (_f) FN<0, 1, true>(e, ##__VA_ARGS__); else FN<0, 1, false>(e, ##__VA_ARGS__); break;   \
        case 16: FN<0, 16, true>(e, ##__VA_ARGS__); break;                                       \
        case 32: FN<0, 32, true>(e, ##__VA_ARGS__); break;                                       \
        case 9: if (_f) FN<0, 9, true>(e, ##__VA_ARGS__); else FN<0, 9, false>(e, ##__VA_ARGS__); break;   \
        default: if (_f) FN<0, 15, true>(e, ##__VA_ARGS__); else FN<0, 15, false>(e, ##__VA_ARGS__); break; \
      }                                                                                          \
    } else {                                                                                     \
      switch (_s.agg) {                                                                          \
        case 1: if (_f) FN<1, 1, true>(e, ##__VA_ARGS__); else FN<1, 1, false>(e, ##__VA_ARGS__); break;   \
        case 16: FN<1, 16, true>(e, ##__VA_ARGS__); break;                                       \
        case 32: FN<1, 32, true>(e, ##__VA_ARGS__); break;                                       \
        case 9: if (_f) FN<1, 9, true>(e, ##__VA_ARGS__); else FN<1, 9, false>(e, ##__VA_ARGS__); break;   \
        default: if (_f) FN<1, 15, true>(e, ##__VA_ARGS__); else FN<1, 15, false>(e, ##__VA_ARGS__); break; \
      }                                                                                          \
    }                                                                                            \
  } while (0)
#endif

extern "C" {

const char* fw_version(void) { return "flink_amd fw 0.1 (gfx950)"; }

int fw_create(const fw_config* cfg_in, fw_engine** out) {
  if (!cfg_in || !out) return FW_ERR_INVALID_ARG;
  *out = nullptr;
  fw_config c = *cfg_in;
  auto* e = new fw_engine();
  e->cfg = c;
  auto bad = [&](const char* m) { g_create_error = m; delete e; return FW_ERR_INVALID_ARG; };
  auto unsupported = [&](const char* m) { g_create_error = m; delete e; return FW_ERR_UNSUPPORTED; };
  if (c.size <= 0) return bad("window size must be > 0");
  if (c.assigner != FW_TUMBLING && c.assigner != FW_SLIDING && c.assigner != FW_SESSION) return bad("unknown assigner");
  e->session = c.assigner == FW_SESSION;
  e->list = c.agg_mask == FW_AGG_LIST;
  if ((c.agg_mask & FW_AGG_LIST) && !e->list) return bad("list state (FW_AGG_LIST) is used alone");
  if (e->list && (c.agg_flags & FW_AGGF_FOLD)) return unsupported("list state: no fold");
  if (e->list) { c.ingest_mode = 1; c.keep_first_f1 = 1; e->cfg = c; }
  if (e->session) {
    if (c.max_open_slices > SESS_SW_MAX) return bad("session windows: at most 256 in-flight sessions per key (max_open_slices)");
    e->sess.sw = c.max_open_slices > 0 ? c.max_open_slices : SESS_SW_DEFAULT;
    c.slide = c.size; c.offset = 0; c.max_open_slices = 1; c.ingest_mode = 1; e->cfg = c;
  }
  if (c.assigner == FW_SLIDING && c.slide <= 0) return bad("slide must be > 0");
  if (c.allowed_lateness < 0) return bad("allowed lateness must be >= 0");
  if (c.max_parallelism <= 0 || c.max_parallelism > (1 << 15) || c.kg_start < 0 || c.kg_end < c.kg_start ||
      c.kg_end >= c.max_parallelism)
    return bad("bad key-group range");
  if (c.value_type != FW_VALUE_I64 && c.value_type != FW_VALUE_F64) return bad("bad value type");
  const bool by = (c.agg_mask & (FW_AGG_MAXBY | FW_AGG_MINBY)) != 0;
  if ((c.agg_mask & ~127) != 0 || c.agg_mask == 0 || (by && c.agg_mask != FW_AGG_MAXBY && c.agg_mask != FW_AGG_MINBY))
    return bad("bad aggregate mask (maxBy / minBy return the whole record and combine with nothing else)");
  if ((c.agg_flags & ~(FW_AGGF_COMPARABLE | FW_AGGF_BY_LAST | FW_AGGF_FOLD)) != 0) return bad("bad aggregate flags");
  if ((c.agg_flags & FW_AGGF_FOLD) && (c.assigner == FW_SESSION))
    return unsupported("Fold cannot be used with a merging WindowAssigner.");
  if ((c.agg_flags & FW_AGGF_FOLD) && (c.keep_first_f1 || !(c.agg_mask == FW_AGG_SUM || c.agg_mask == FW_AGG_MIN ||
                                                              c.agg_mask == FW_AGG_MAX || c.agg_mask == FW_AGG_COUNT)))
    return unsupported("fold: one aggregate (sum, count, min or max) from the initial value, no first-arrival f1");
  if (c.key_capacity <= 0 || c.max_batch <= 0 || c.out_capacity <= 0) return bad("capacities must be > 0");
  if (c.ingest_mode < 0 || c.ingest_mode > 3) return bad("bad ingest mode");
  HIPCHK(e, hipSetDevice(c.device));
  e->dev = c.device;
  HIPCHK(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  {
    // FW_STREAM_PRIO (diagnostics): 1 = route stream high priority, 2 = engine stream high priority
    const char* sp = getenv("FW_STREAM_PRIO");
    const int which = sp ? atoi(sp) : 0;
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    HIPCHK(e, hipStreamCreateWithPriority(&e->rstream, hipStreamNonBlocking, which == 1 ? hi : lo));
    if (which == 2) {
      HIPCHK(e, hipStreamDestroy(e->stream));
      HIPCHK(e, hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, hi));
    }
  }
  e->serial = getenv("FW_SERIAL") && atoi(getenv("FW_SERIAL")) != 0;
  e->event_query = !(getenv("FW_EVENT_QUERY") && atoi(getenv("FW_EVENT_QUERY")) == 0);
  e->no_consumed = getenv("FW_NO_CONSUMED") && atoi(getenv("FW_NO_CONSUMED")) != 0;
  e->debug_late = getenv("FW_DEBUG_LATE") && atoi(getenv("FW_DEBUG_LATE")) != 0;
  e->debug_sync = getenv("FW_DEBUG_SYNC") && atoi(getenv("FW_DEBUG_SYNC")) != 0;
  HIPCHK(e, hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
  for (auto& ev : e->ev_consumed) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCHK(e, hipEventCreateWithFlags(&e->ev_now, hipEventDisableTiming));
  HIPCHK(e, hipEventCreateWithFlags(&e->ev_hcopy, hipEventDisableTiming));
  // ev_route / ev_agg order two device streams of one GPU: no system-scope fence needed (FW_EVENT_FENCE=1: with)
  const unsigned pf = hipEventDisableTiming |
      ((getenv("FW_EVENT_FENCE") && atoi(getenv("FW_EVENT_FENCE")) != 0) ? 0u : (unsigned)hipEventDisableSystemFence);
  for (int q = 0; q < fw_engine::NBUF; ++q) {
    HIPCHK(e, hipEventCreateWithFlags(&e->ev_route[q], pf));
    HIPCHK(e, hipEventCreateWithFlags(&e->ev_agg[q], pf));
  }
  hipDeviceProp_t prop;
  HIPCHK(e, hipGetDeviceProperties(&prop, c.device));
  e->grid = prop.multiProcessorCount * 8;

  Spec& s = e->s;
  s.assigner = c.assigner;
  s.trigger = c.trigger;
  s.size = c.size;
  s.slide = c.assigner == FW_TUMBLING ? c.size : c.slide;
  s.offset = c.offset;
  s.lateness = c.allowed_lateness;
  s.g = c.assigner == FW_TUMBLING ? c.size : gcd64(c.size, s.slide);
  s.K = (int32_t)(c.size / s.g);
  s.inv_size = 1.0 / (double)s.size;
  s.inv_g = 1.0 / (double)s.g;
  s.R = (int32_t)(s.slide / s.g);
  if (s.K > MAX_K) return unsupported("more than 1024 slices per window (size / gcd(size, slide))");
  s.mp = c.max_parallelism;
  s.mp_mask = (c.max_parallelism & (c.max_parallelism - 1)) == 0 ? c.max_parallelism - 1 : 0;
  s.kg_start = c.kg_start;
  s.kg_end = c.kg_end;
  s.vt = c.value_type;
  s.agg = by ? c.agg_mask
             : (c.agg_mask == FW_AGG_SUM || e->list) ? FW_AGG_SUM
             : c.agg_mask == (FW_AGG_SUM | FW_AGG_COUNT) ? c.agg_mask   // the average shape: no min/max columns
             : 15;   // instantiated reduce shapes
  // (list state: the sum column carries each element's value, f1 its f1)
  s.by = by ? c.agg_mask : 0;
  s.by_last = (c.agg_flags & FW_AGGF_BY_LAST) ? 1 : 0;
  s.cmpto = by || (c.agg_flags & FW_AGGF_COMPARABLE) ? 1 : 0;
  s.fold = (c.agg_flags & FW_AGGF_FOLD) ? 1 : 0;
  s.fold_init = c.fold_initial;
  // maxBy/minBy: the pane's presence and the extremal f1; fold: first arrivals order the reference layout's
  // entries (HashMap chains in insertion order) though no f1 is kept
  s.first = c.keep_first_f1 || by || (c.agg_flags & FW_AGGF_FOLD) ? 1 : 0;

  // ingest_mode 3 was the fused form (one persistent launch per batch, XCD-local hand-off of the routed records):
  // measured slower than the partitioned form in rounds 3 and 4 (23 / 14 G vs 51-56 G events/s on C1), removed
  if (c.ingest_mode == 3) return unsupported("ingest_mode 3 (fused) was removed: the partitioned form (2) is faster; DESIGN.md section 4");
  // key directory at load factor <= 1/4 (<= 1/2 above 2^20 keys, <= 0.625 above 2^22): short linear-probe sequences.
  // Above 2^22 keys the direct form is bound by random lines of the directory and the pane columns (D + 1 rows
  // each), so a denser table pays: C2 (10 M keys) 16 M slots instead of 32 M, 9.3 -> 10.0 G events/s (same-box
  // A/B).  FW_DIR_SLOTS (slots per key x 100, experiments) overrides the factor
  {
    int64_t f100 = c.key_capacity <= (1 << 20) ? 400 : c.key_capacity <= (1 << 22) ? 200 : 160;
    if (const char* v = getenv("FW_DIR_SLOTS")) f100 = std::max(100, atoi(v));
    s.D = next_pow2(std::max<int64_t>((f100 * c.key_capacity + 99) / 100, 64));
  }
  s.dir_mask = (uint64_t)s.D - 1;
  {
    int dbits = bits_for((uint64_t)s.D) - 1;                  // D = 2^dbits
    int kb = std::max(std::min(dbits, 9), dbits - 8);          // <= 256 buckets of >= 512 slots
    s.kb_bits = kb;
    s.nb = (int32_t)(s.D >> kb);
  }
  s.stride = s.D + 1;
  int32_t P = c.max_open_slices;
  if (P <= 0) {
    int64_t late_slices = (c.allowed_lateness + s.g - 1) / s.g;
    P = (int32_t)std::min<int64_t>(2 * s.K + late_slices + 8, MAX_P);
  }
  if (P > MAX_P) P = MAX_P;
  s.P = P;

  s.dir_keys = e->alloc<int64_t>((size_t)s.D);
  s.dir_min_used = e->alloc<int32_t>(1);
  s.slice_tag = e->alloc<int64_t>((size_t)P);
  const size_t cells = (size_t)P * (size_t)s.stride;
  s.c.sum = (s.agg & FW_AGG_SUM) ? e->alloc<int64_t>(cells) : nullptr;
  s.c.mn = (s.agg & (FW_AGG_MIN | FW_AGG_MINBY)) ? e->alloc<int64_t>(cells) : nullptr;
  s.c.mx = (s.agg & (FW_AGG_MAX | FW_AGG_MAXBY)) ? e->alloc<int64_t>(cells) : nullptr;
  s.c.cnt = (s.agg & FW_AGG_COUNT) || by ? e->alloc<int64_t>(cells) : nullptr;   // maxBy/minBy: the extremal ordinal
  if (s.first) {
    s.c.first = e->alloc<int64_t>(cells);
    s.c.f1v = e->alloc<int64_t>(cells);
    s.c.present = nullptr;
  } else {
    s.c.first = nullptr;
    s.c.f1v = nullptr;
    s.c.present = e->alloc<uint8_t>(cells);
  }
  if (c.trigger == FW_TRIGGER_PURGING_EVENT_TIME && c.allowed_lateness > 0 && c.assigner == FW_TUMBLING) {
    s.gtag = e->alloc<int64_t>((size_t)P);   // purged windows' cleanup timers (Spec::gfirst)
    s.gfirst = e->alloc<int64_t>(cells);
  }
  if (c.assigner == FW_SLIDING) {   // window panes for the assigner's extra windows
    s.W = P;
    s.wtag = e->alloc<int64_t>((size_t)P);
    s.wc.sum = s.c.sum ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.mn = s.c.mn ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.mx = s.c.mx ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.cnt = s.c.cnt ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.first = s.c.first ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.f1v = s.c.f1v ? e->alloc<int64_t>(cells) : nullptr;
    s.wc.present = s.c.present ? e->alloc<uint8_t>(cells) : nullptr;
    for (int q = 0; q < fw_engine::NBUF; ++q) e->quirk_list[q] = e->alloc<int64_t>((size_t)c.max_batch * QK_WORDS);
    e->quirk_count = e->alloc<unsigned long long>(fw_engine::NBUF);
  }
  OutLog& o = s.o;
  o.capacity = c.out_capacity;
  o.key = e->alloc<int64_t>((size_t)o.capacity);
  o.f1 = c.keep_first_f1 || s.by ? e->alloc<int64_t>((size_t)o.capacity) : nullptr;
  o.ts = e->alloc<int64_t>((size_t)o.capacity);
  o.sum = (s.agg & FW_AGG_SUM) ? e->alloc<int64_t>((size_t)o.capacity) : nullptr;
  o.mn = (s.agg & (FW_AGG_MIN | FW_AGG_MINBY)) ? e->alloc<int64_t>((size_t)o.capacity) : nullptr;
  o.mx = (s.agg & (FW_AGG_MAX | FW_AGG_MAXBY)) ? e->alloc<int64_t>((size_t)o.capacity) : nullptr;
  o.cnt = (s.agg & FW_AGG_COUNT) ? e->alloc<int64_t>((size_t)o.capacity) : nullptr;
  o.count = e->alloc<unsigned long long>(1);
  o.mark_capacity = 1 << 16;
  o.mark_wm = e->alloc<int64_t>((size_t)o.mark_capacity);
  o.mark_pos = e->alloc<int64_t>((size_t)o.mark_capacity);
  o.mark_count = e->alloc<unsigned long long>(1);
  s.err = e->alloc<int32_t>(1);
  s.stats = e->alloc<unsigned long long>(ST_NSTATS);
  // key directory compaction (k_compact): buckets that fit LDS
  e->kg_evicted = e->alloc<unsigned char>((size_t)c.max_parallelism);
  e->compact_lds = compact_lds_bytes(s.kb_bits, s.P);
  e->compact_ok = s.kb_bits <= 12 && e->compact_lds <= 160 * 1024 && !e->session;
  if (e->compact_ok) {
    if (hipHostMalloc((void**)&e->dir_keys_host, 4, hipHostMallocMapped) != hipSuccess) e->dir_keys_host = nullptr;
    if (e->dir_keys_host) *e->dir_keys_host = 0;
    s.dir_keys_host = e->dir_keys_host;
    (void)hipFuncSetAttribute((const void*)k_compact, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const char* cf = getenv("FW_COMPACT_FILL");   // percent of the directory's slots (0: never compact)
    if (cf && atoi(cf) <= 0) e->compact_ok = false;
    else if (cf) e->compact_fill = std::min(atoi(cf), 95) / 100.0;
  }

  for (int q = 0; q < fw_engine::NBUF; ++q) {
    e->stg_key[q] = e->alloc<int64_t>((size_t)c.max_batch);
    e->stg_ts[q] = e->alloc<int64_t>((size_t)c.max_batch);
    e->stg_val[q] = e->alloc<int64_t>((size_t)c.max_batch);
    e->stg_f1[q] = e->alloc<int64_t>((size_t)c.max_batch);
    e->stg_hash[q] = e->alloc<int32_t>((size_t)c.max_batch);
  }

  // ingest form: partitioned (LDS pre-aggregation) when a directory bucket's accumulators fit in LDS
  // and batches are large; direct atomics otherwise
  {
    const int32_t max_tiles = (int32_t)((c.max_batch + RT_TILE - 1) / RT_TILE);
    const int nacc = 1 + ((s.agg & (FW_AGG_MIN | FW_AGG_MINBY)) ? 1 : 0) + ((s.agg & (FW_AGG_MAX | FW_AGG_MAXBY)) ? 1 : 0) +
                     ((s.agg & FW_AGG_COUNT) ? 1 : 0);
    const size_t agg_need = agg_lds_bytes(s.kb_bits, nacc, max_tiles, by);
    const bool fits = s.kb_bits <= RT_MAX_KB_BITS && s.nb <= RT_MAXNB && agg_need <= 160 * 1024 &&
                      c.max_batch <= (1ll << 26);
    if (c.ingest_mode == 2 && !fits)
      return unsupported("partitioned ingest needs <= 4096 directory slots per bucket (key_capacity <= 256 Ki)");
    e->routed = !e->session && (c.ingest_mode == 2 || (c.ingest_mode == 0 && fits && (c.max_batch >= (1 << 16) || by)));
    e->by_direct = by && !e->routed && !e->session;
    if (e->routed) {
      e->max_tiles = max_tiles;
      const size_t cap = (size_t)max_tiles * RT_TILE;
      const char* dbg = getenv("FW_DEBUG_AGG");
      e->rb.dbg = dbg ? atoi(dbg) : 0;
      e->rb.stamps = (e->rb.dbg & 16) ? e->alloc<long long>((size_t)16 << 16) : nullptr;
      e->s.wm_stamps = e->rb.stamps ? e->rb.stamps + ((size_t)12 << 16) : nullptr;
      e->dflags = e->alloc<unsigned int>(FLAG_RING);
      e->bload = e->alloc<unsigned int>(4 * RT_MAXNB);
      e->fold_flag = e->alloc<unsigned int>((size_t)5 * RT_MAXNB * RT_GS);   // flags, then the 4-entry count ring
      if (hipHostMalloc((void**)&e->bload_host, 4 * RT_MAXNB, hipHostMallocMapped) != hipSuccess) e->bload_host = nullptr;
      if (e->bload_host) memset(e->bload_host, 0, 4 * RT_MAXNB);
      const char* hv = getenv("FW_AGG_HELPERS");
      if (hv) e->agg_helpers_max = std::max(0, std::min(atoi(hv), (int)RT_MAXNB));
      // integer reduces fold a split bucket's shares concurrently, so they take more of them
      const bool afold = e->s.vt == FW_VALUE_I64 && !e->s.by;
      e->agg_split = afold ? FW_AGG_SPLIT_INT : AG_SPLIT_CHAIN;
      const char* sv = getenv("FW_AGG_SPLIT");
      if (sv) e->agg_split = std::max(1, std::min(atoi(sv), afold ? AG_SPLIT_MAX : AG_SPLIT_CHAIN));
      const char* cv = getenv("FW_AGG_CHUNK_PCT");
      if (cv) e->agg_chunk_pct = std::max(50, std::min(atoi(cv), 1000));
      for (int q = 0; q < fw_engine::NBUF; ++q) {
        RouteBuf& r = e->rbs[q];
        r = e->rb;
        r.kv = e->alloc<longlong2>(cap);
        r.idx = e->alloc<uint16_t>(cap);
        r.seg = e->alloc<uint32_t>((size_t)RT_GROUPS * s.nb * max_tiles);
        r.seg_stride = max_tiles;
        r.hdr = e->alloc<int64_t>((size_t)max_tiles * RT_Q);
        r.tdir = e->alloc<uint32_t>((size_t)max_tiles);
        r.dm = e->alloc<int64_t>(cap);
      }
      e->route_lds = RT_LDS;
      const char* ml = getenv("FW_AGG_MIN_LDS_KB");
      e->agg_min_lds = (ml ? atoi(ml) : 81) * 1024;
      e->agg_lds = agg_need;   // at launch: less the unused tiles, at least agg_min_lds
      FW_DISPATCH(routed_attrs_t, e);
      if (e->attr_err != hipSuccess) {
        g_create_error = std::string("hipFuncSetAttribute(MaxDynamicSharedMemorySize): ") + hipGetErrorString(e->attr_err);
        delete e;
        return FW_ERR_DEVICE;
      }
    }
  }
  if (wm_lds_bytes(s.P, s.K, s.R, s.W) > 64 * 1024) {
    FW_DISPATCH(wm_attrs_t, e);
    if (e->attr_err != hipSuccess) {
      g_create_error = std::string("hipFuncSetAttribute(MaxDynamicSharedMemorySize): ") + hipGetErrorString(e->attr_err);
      delete e;
      return FW_ERR_DEVICE;
    }
  }
  e->wm_done = e->alloc<unsigned int>(1);
  if (e->routed) e->s_dev = e->alloc<Spec>(1);
  if (s.first && !e->routed) {
    e->new_list = e->alloc<int64_t>((size_t)c.max_batch);
    e->new_counts = e->alloc<unsigned long long>(2);
  }

  for (void* p : e->allocs) if (!p) { delete e; return FW_ERR_DEVICE; }

  if (e->by_direct) {
    e->by_key = e->alloc<unsigned long long>((size_t)c.max_batch);
    e->by_count = e->alloc<unsigned long long>(1);
    for (void* p : e->allocs) if (!p) { delete e; return FW_ERR_DEVICE; }
    if (hipMemset(e->by_count, 0, 8) != hipSuccess) { delete e; return FW_ERR_DEVICE; }
  }
  // late path (allowed lateness > 0; its sort and segmented scan also fold the direct form's maxBy / minBy)
  if (c.allowed_lateness > 0 || e->by_direct) {
    e->idx_bits = bits_for((uint64_t)c.max_batch);
    int pane_bits = bits_for((uint64_t)P * (uint64_t)s.stride);
    if (e->idx_bits + pane_bits > 64) { delete e; return FW_ERR_UNSUPPORTED; }
    // sliding: a late record fires once per window of its slice in its lateness period
    // (bounded: a batch of late records whose windows' per-element fires exceed it reports FW_ERR_CAPACITY)
    if (c.assigner == FW_SLIDING) e->fire_cap = std::min<int64_t>(c.max_batch * (int64_t)((s.K + s.R - 1) / s.R), (int64_t)1 << 27);
    const size_t nb = (size_t)std::max<int64_t>(c.max_batch, e->fire_cap);
    if (e->fire_cap) {
      e->fire_key = e->alloc<unsigned long long>((size_t)e->fire_cap);
      e->fire_count = e->alloc<unsigned long long>(1);
    }
    e->late_key = e->alloc<unsigned long long>((size_t)c.max_batch);
    e->late_key_sorted = e->alloc<unsigned long long>(nb);
    e->late_count = e->alloc<unsigned long long>(1);
    e->out_base = e->alloc<unsigned long long>(1);
    e->seg = e->alloc<unsigned long long>(nb);
    e->late_acc = e->alloc<LateAcc>(nb);
    e->late_scan = e->alloc<LateAcc>(nb);
    e->headpos = e->alloc<int64_t>(nb);
    e->headpos_scan = e->alloc<int64_t>(nb);
    e->seg_tiles = e->alloc<SegPart>(nb / LS_TILE + 1);
    e->seg_groups = e->alloc<SegPart>((nb / LS_TILE + 1) / LS_CT + 2);
    e->seg_first = e->alloc<int32_t>(nb / LS_TILE + 1);
    if (c.assigner != FW_SLIDING) {
      const char* lf = getenv("FW_LATE_FUSED");   // 0: the six-kernel scan (A/B)
      e->late_fused = !(lf && atoi(lf) == 0);
      const size_t nt = (size_t)c.max_batch / LF_T + 1;
      e->lf_flag = e->alloc<unsigned int>(nt);
      e->lf_agg = e->alloc<LfPart>(nt);
      e->lf_incl = e->alloc<LfPart>(nt);
      e->lf_base = e->alloc<unsigned long long>(2);
      e->lf_ticket = e->alloc<unsigned int>(1);
      if (!e->lf_flag || !e->lf_base || !e->lf_ticket || hipMemset(e->lf_flag, 0, 4 * nt) != hipSuccess ||
          hipMemset(e->lf_base, 0, 16) != hipSuccess || hipMemset(e->lf_ticket, 0, 4) != hipSuccess) {
        delete e;
        return FW_ERR_DEVICE;
      }
    }
    size_t t1 = 0;
    (void)rocprim::radix_sort_keys(nullptr, t1, e->late_key, e->late_key_sorted, nb, 0, 64, e->stream);
    e->temp_bytes = t1;
    e->temp = e->alloc<char>(e->temp_bytes);
    for (void* p : e->allocs) if (!p) { delete e; return FW_ERR_DEVICE; }
  } else {
    e->late_count = e->alloc<unsigned long long>(1);
  }

  if (e->session) {
    if (int rc = session_create(e)) { g_create_error = "session window state allocation failed"; delete e; return rc; }
  }
  if (e->list && !e->session) {
    if (s.K > LIST_MAX_K) return unsupported("list state: more than 64 slices per window (size / gcd(size, slide))");
    if (int rc = list_create(e)) { g_create_error = "list state allocation failed"; delete e; return rc; }
  }
  // initial state
  launch_fill(e, s.dir_keys, EMPTY_KEY, s.D);
  launch_fill(e, s.slice_tag, FREE_TAG, P);
  launch_fill(e, s.c.sum, sum_identity(s.vt), (int64_t)cells);
  launch_fill(e, s.c.mn, INT64_MAX, (int64_t)cells);
  launch_fill(e, s.c.mx, INT64_MIN, (int64_t)cells);
  launch_fill(e, s.c.cnt, 0, (int64_t)cells);
  launch_fill(e, s.c.first, INT64_MAX, (int64_t)cells);
  launch_fill(e, s.gtag, FREE_TAG, P);
  launch_fill(e, s.gfirst, INT64_MAX, (int64_t)cells);
  if (s.c.present) HIPCHK(e, hipMemsetAsync(s.c.present, 0, cells, e->stream));
  if (s.W > 0) {
    launch_fill(e, s.wtag, FREE_TAG, s.W);
    launch_fill(e, s.wc.sum, sum_identity(s.vt), (int64_t)cells);
    launch_fill(e, s.wc.mn, INT64_MAX, (int64_t)cells);
    launch_fill(e, s.wc.mx, INT64_MIN, (int64_t)cells);
    launch_fill(e, s.wc.cnt, 0, (int64_t)cells);
    launch_fill(e, s.wc.first, INT64_MAX, (int64_t)cells);
    if (s.wc.present) HIPCHK(e, hipMemsetAsync(s.wc.present, 0, cells, e->stream));
    HIPCHK(e, hipMemsetAsync(e->quirk_count, 0, 8 * fw_engine::NBUF, e->stream));
  }
  HIPCHK(e, hipMemsetAsync(s.dir_min_used, 0, 4, e->stream));
  HIPCHK(e, hipMemsetAsync(o.count, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(o.mark_count, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(s.err, 0, 4, e->stream));
  HIPCHK(e, hipMemsetAsync(s.stats, 0, 8 * ST_NSTATS, e->stream));
  HIPCHK(e, hipMemsetAsync(e->kg_evicted, 0, (size_t)c.max_parallelism, e->stream));
  HIPCHK(e, hipMemsetAsync(e->late_count, 0, 8, e->stream));
  if (e->fire_count) HIPCHK(e, hipMemsetAsync(e->fire_count, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(e->wm_done, 0, 4, e->stream));
  if (e->new_counts) HIPCHK(e, hipMemsetAsync(e->new_counts, 0, 16, e->stream));
  if (e->dflags) HIPCHK(e, hipMemsetAsync(e->dflags, 0, 4 * FLAG_RING, e->stream));
  if (e->bload) HIPCHK(e, hipMemsetAsync(e->bload, 0, 4 * 4 * RT_MAXNB, e->stream));
  if (e->fold_flag) HIPCHK(e, hipMemsetAsync(e->fold_flag, 0, 4 * (size_t)5 * RT_MAXNB * RT_GS, e->stream));
  if (e->routed) {   // k_route reads the Spec from a device copy
    if (int rc = upload_spec(e)) return rc;
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipGetLastError());
  if (e->debug_sync && (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess)) {
    g_create_error = "FW_DEBUG_SYNC: initial fills failed";
    delete e;
    return FW_ERR_DEVICE;
  }
  *out = e;
  return FW_OK;
}

static int device_error(fw_engine* e, int32_t derr);
static int check_device_error(fw_engine* e) {
  int32_t derr = 0;
  HIPCHK(e, hipMemcpyAsync(&derr, e->s.err, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return device_error(e, derr);
}
// the device error word as the engine's sticky error, with the reference's message where it has one
static int device_error(fw_engine* e, int32_t derr) {
  if (derr != 0 && e->sticky == FW_OK) {
    const char* msg = "device error";
    switch (derr) {
      case FW_ERR_NO_TIMESTAMP:
        msg = "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time characteristic set to "
              "'ProcessingTime', or did you forget to call 'DataStream.assignTimestampsAndWatermarks(...)'?";
        break;
      case FW_ERR_KEY_GROUP: msg = "Unexpected key group index. This indicates a bug."; break;
      case FW_ERR_CAPACITY: msg = "capacity exceeded (key directory, slice pool, per-element fire list or output log)"; break;
      case FW_ERR_UNSUPPORTED: msg = "a record's extra sliding window (timestamp below offset - slide, Java % of a negative "
                                     "numerator) is already behind the watermark, or maxBy/minBy with such a record: "
                                     "per-element fire of a window pane not supported"; break;
    }
    return fail(e, derr, msg);
  }
  return e->sticky;
}

static int64_t host_window_start(const fw_config& c, int64_t n);   // (below, with the checkpoint code)

// sort (pane << idx_bits | batch index) keys, then the per-pane inclusive scan of the records' accumulators in
// arrival order (k_late_prepare, k_segscan_*); emit_n > 0 reserves that many output rows for per-element fires
static int late_sorted_scan(fw_engine* e, unsigned long long* keys, unsigned long long n, int64_t emit_n,
                            const int64_t* dv, const int64_t* df1) {
  const int key_bits = std::min(64, e->idx_bits + bits_for((uint64_t)e->s.P * (uint64_t)e->s.stride));
  size_t tb = e->temp_bytes;
  HIPCHK(e, rocprim::radix_sort_keys(e->temp, tb, keys, e->late_key_sorted, (size_t)n, 0, key_bits, e->stream));
  const int blocks = (int)((n + BLOCK - 1) / BLOCK);
  hipLaunchKernelGGL(k_late_prepare, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->late_key_sorted, (int64_t)n,
                     e->idx_bits, dv, e->seg, e->late_acc, e->headpos, df1, e->ordinal, emit_n, e->out_base);
  const int32_t ntl = (int32_t)((n + LS_TILE - 1) / LS_TILE);
  hipLaunchKernelGGL(k_segscan_tile, dim3(ntl), dim3(LS_T), 0, e->stream, e->seg, e->late_acc, (int64_t)n,
                     e->late_scan, e->headpos_scan, e->seg_tiles, e->seg_first);
  const SegPart* grp = nullptr;
  if (ntl > LS_CT) {   // two levels (one workgroup's serial chunks took ~90 us at 4 K tiles)
    const int32_t ng = (ntl + LS_CT - 1) / LS_CT;
    hipLaunchKernelGGL(k_segscan_carry_grp, dim3(ng), dim3(LS_CT), 0, e->stream, e->seg_tiles, ntl, e->seg_groups);
    hipLaunchKernelGGL(k_segscan_carry, dim3(1), dim3(LS_CT), 0, e->stream, e->seg_groups, ng);
    grp = e->seg_groups;
  } else {
    hipLaunchKernelGGL(k_segscan_carry, dim3(1), dim3(LS_CT), 0, e->stream, e->seg_tiles, ntl);
  }
  hipLaunchKernelGGL(k_segscan_apply, dim3(ntl), dim3(LS_T), 0, e->stream, e->seg_tiles, grp, e->seg_first, (int64_t)n,
                     e->late_scan, e->headpos_scan);
  return FW_OK;
}

int fw_push_batch(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1, const int64_t* ts,
                  const void* value, int64_t n, int32_t mem) {
  if (!e) return FW_ERR_INVALID_ARG;
  if (e->sticky) return e->sticky;
  if (n < 0 || (n > 0 && (!key || !ts || !value))) return fail(e, FW_ERR_INVALID_ARG, "null column");
  if (n > e->cfg.max_batch) return fail(e, FW_ERR_CAPACITY, "batch larger than max_batch");
  if (n == 0) return FW_OK;
  HIPCHK(e, hipSetDevice(e->dev));
  if (key_hash) e->used_key_hash = true;
  e->state_epoch++;
  // routed form: the batch's copies and k_route run on the route stream, k_aggregate on the engine
  // stream; buffer set par is reused only after k_aggregate of batch j - NBUF finished
  const int par = (int)(e->batches % fw_engine::NBUF);
  // host columns are copied on the route stream (a copy queue beside the engine stream's kernels)
  hipStream_t in_stream = (e->routed || mem == FW_MEM_HOST) && !e->serial ? e->rstream : e->stream;
  // a wait whose event has already completed is skipped: each one costs the command processor a barrier
  // packet on the stream (FW_EVENT_QUERY=0 enqueues them all, for A/B)
  auto wait_on = [&](hipStream_t st, hipEvent_t ev) -> hipError_t {
    if (e->event_query && hipEventQuery(ev) == hipSuccess) return hipSuccess;
    return hipStreamWaitEvent(st, ev, 0);
  };
  // buffer set par (routed buffers, host staging) is rewritten only after the push that used it NBUF pushes ago
  if (e->routed || mem == FW_MEM_HOST) HIPCHK(e, wait_on(in_stream, e->ev_agg[par]));
  // input columns are produced on the caller's stream: order the push after it (nothing to order when that
  // stream has no work pending)
  if (e->has_client && !(e->event_query && hipStreamQuery((hipStream_t)e->client) == hipSuccess)) {
    HIPCHK(e, hipEventRecord(e->ev_in, (hipStream_t)e->client));
    HIPCHK(e, wait_on(in_stream, e->ev_in));
  }
  const int64_t *dk = key, *dts = ts, *dv = (const int64_t*)value, *df1 = f1;
  const int32_t* dh = key_hash;
  if (mem == FW_MEM_HOST) {
    HIPCHK(e, hipMemcpyAsync(e->stg_key[par], key, 8 * n, hipMemcpyHostToDevice, in_stream));
    HIPCHK(e, hipMemcpyAsync(e->stg_ts[par], ts, 8 * n, hipMemcpyHostToDevice, in_stream));
    HIPCHK(e, hipMemcpyAsync(e->stg_val[par], value, 8 * n, hipMemcpyHostToDevice, in_stream));
    dk = e->stg_key[par]; dts = e->stg_ts[par]; dv = e->stg_val[par];
    if (key_hash) { HIPCHK(e, hipMemcpyAsync(e->stg_hash[par], key_hash, 4 * n, hipMemcpyHostToDevice, in_stream)); dh = e->stg_hash[par]; }
    if (f1) { HIPCHK(e, hipMemcpyAsync(e->stg_f1[par], f1, 8 * n, hipMemcpyHostToDevice, in_stream)); df1 = e->stg_f1[par]; }
    // the caller may reuse its arrays once fw_push_batch returns (flink_window.h): wait for the copies here
    // (pinned host memory would otherwise still be read by the DMA engine afterwards); the earlier batches'
    // kernels keep running on the engine stream meanwhile
    HIPCHK(e, hipEventRecord(e->ev_hcopy, in_stream));
    HIPCHK(e, hipEventSynchronize(e->ev_hcopy));
    if (in_stream != e->stream && !e->routed) HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_hcopy, 0));
  }
  if (e->routed && mem == FW_MEM_DEVICE) {
    // k_route streams the columns with 16-B loads (key hashes with 8-B loads): realign odd pointers
    auto mis = [](const void* ptr, uintptr_t a) { return ((uintptr_t)ptr & (a - 1)) != 0; };
    if (mis(dk, 16)) { HIPCHK(e, hipMemcpyAsync(e->stg_key[par], dk, 8 * n, hipMemcpyDeviceToDevice, in_stream)); dk = e->stg_key[par]; }
    if (mis(dts, 16)) { HIPCHK(e, hipMemcpyAsync(e->stg_ts[par], dts, 8 * n, hipMemcpyDeviceToDevice, in_stream)); dts = e->stg_ts[par]; }
    if (mis(dv, 16)) { HIPCHK(e, hipMemcpyAsync(e->stg_val[par], dv, 8 * n, hipMemcpyDeviceToDevice, in_stream)); dv = e->stg_val[par]; }
    if (dh && mis(dh, 8)) { HIPCHK(e, hipMemcpyAsync(e->stg_hash[par], dh, 4 * n, hipMemcpyDeviceToDevice, in_stream)); dh = e->stg_hash[par]; }
  }
  if (!df1) df1 = dts;
  BatchIn b;
  b.key = dk; b.key_hash = dh; b.ts = dts; b.val = dv; b.n = n;
  b.ord_base = e->ordinal;
  b.wm = e->cur_wm;
  b.late_key = e->late_key;
  b.late_count = e->late_count;
  b.late_capacity = e->late_key ? e->cfg.max_batch : 0;
  b.idx_bits = e->idx_bits;
  b.by_key = e->by_key;
  b.by_count = e->by_count;
  b.by_capacity = e->by_key ? e->cfg.max_batch : 0;
  b.fire_key = e->fire_key;
  b.fire_count = e->fire_count;
  b.fire_capacity = e->fire_cap;
  b.quirk = e->s.W > 0 ? e->quirk_list[par] : nullptr;
  b.quirk_count = e->s.W > 0 ? e->quirk_count + par : nullptr;
  b.quirk_capacity = e->s.W > 0 ? e->cfg.max_batch : 0;
  b.f1 = df1;
  b.new_list = e->new_list;
  b.new_count = e->new_counts;   // (the direct form's list is indexed by record; the count stays unused)
  b.new_capacity = e->new_list ? e->cfg.max_batch : 0;
  if (e->session) {
    if (int rc = session_push(e, b)) return rc;
  } else if (e->list) {
    if (int rc = list_push(e, b)) return rc;
  } else if (e->routed) {
    FW_DISPATCH(launch_routed_t, e, b, df1, par);
  } else {
    e->phase_begin(FW_PHASE_INGEST);
    FW_DISPATCH(launch_ingest_t, e, b);
    if (e->by_direct) {
      // maxBy / minBy: the listed records folded per pane in arrival order into the panes (the late path's
      // commit, no fires); the list length read back sizes the sort
      unsigned long long nb = 0;
      HIPCHK(e, hipMemcpyAsync(&nb, e->by_count, 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      nb = std::min<unsigned long long>(nb, (unsigned long long)e->cfg.max_batch);
      if (nb > 0) {
        if (int rc = late_sorted_scan(e, e->by_key, nb, 0, dv, df1)) return rc;
        hipLaunchKernelGGL(k_late_commit, dim3((unsigned)((nb + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, e->stream, e->s,
                           e->late_key_sorted, (int64_t)nb, e->idx_bits, e->seg, e->late_scan, df1, e->ordinal,
                           e->headpos_scan, false);
      }
      HIPCHK(e, hipMemsetAsync(e->by_count, 0, 8, e->stream));
    }
    e->phase_end(n);
  }
  // sliding: this batch's extra-window records into the window panes.  A record gets an extra window only
  // when ts < offset - slide, and every window of such a record ends before offset + size: once the watermark
  // is past that plus the allowed lateness, they are all late and none is listed, so nothing is launched
  // (C3: ~5 us per push on the engine stream)
  if (e->s.W > 0 && (__int128)e->cur_wm < (__int128)e->s.offset + e->s.size + e->s.slide + e->s.lateness)
    hipLaunchKernelGGL(k_quirk_apply, dim3(1), dim3(1024), 0, e->stream, e->s, e->quirk_list[par], e->quirk_count + par,
                       e->cfg.max_batch);
  e->batches++;
  HIPCHK(e, hipGetLastError());
  if (!e->disarmed.empty() && jsub(jadd(host_window_start(e->cfg, *e->disarmed.rbegin()), e->s.size), 1) > e->cur_wm)
    hipLaunchKernelGGL(k_arm, dim3(std::min<int64_t>((n + BLOCK - 1) / BLOCK, e->grid)), dim3(BLOCK), 0, e->stream, e->s, b);
  // (the direct form's record-indexed list of f1 fix-ups; the partitioned form sets f1 in k_aggregate, and session /
  // list state keep theirs themselves — new_list holds nothing of theirs)
  if (e->s.first && !e->routed && !e->session && !e->list) {
    e->phase_begin(FW_PHASE_FIXUP);
    hipLaunchKernelGGL(k_fix_first_f1, dim3(std::min<int64_t>((n + BLOCK - 1) / BLOCK, e->grid)), dim3(BLOCK), 0,
                       e->stream, e->s, e->new_list, df1, e->ordinal, n);
    e->phase_end(n);
  }
  if (e->debug_late && e->cfg.allowed_lateness > 0 && !e->session && !e->list && !fires_possible(e->s, e->cur_wm)) {
    // diagnostics: the read-back skipped below must have had nothing to read
    unsigned long long nl = 0, nf = 0;
    HIPCHK(e, hipMemcpyAsync(&nl, e->late_count, 8, hipMemcpyDeviceToHost, e->stream));
    if (e->fire_count) HIPCHK(e, hipMemcpyAsync(&nf, e->fire_count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (nl || nf) return fail(e, FW_ERR_INVALID_ARG, "internal: per-element fires at a watermark fires_possible() ruled out");
  }
  if (e->cfg.allowed_lateness > 0 && !e->session && !e->list && fires_possible(e->s, e->cur_wm)) {
    // per-element fires: the list lengths on the host size the sorts
    unsigned long long nl = 0, nf = 0;
    HIPCHK(e, hipMemcpyAsync(&nl, e->late_count, 8, hipMemcpyDeviceToHost, e->stream));
    if (e->fire_count) HIPCHK(e, hipMemcpyAsync(&nf, e->fire_count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (nl > (unsigned long long)e->cfg.max_batch) nl = e->cfg.max_batch;
    if (nf > (unsigned long long)e->fire_cap) nf = e->fire_cap;
    const bool sliding = e->cfg.assigner == FW_SLIDING;
    if (nl > 0 || nf > 0) e->phase_begin(FW_PHASE_LATE);
    // sort by (pane, arrival), per-pane inclusive scan of the records' accumulators in arrival order
    // keys are (pane << idx_bits) | batch index, pane < P * stride: only their low bits are sorted
    const int key_bits = std::min(64, e->idx_bits + bits_for((uint64_t)e->s.P * (uint64_t)e->s.stride));
    auto sorted_scan = [&](unsigned long long* keys, unsigned long long n, int64_t emit_n) -> int {
      return late_sorted_scan(e, keys, n, emit_n, dv, df1);
    };
    if (nf > 0) {   // sliding: the fires first, against the slices before this batch's late records
      if (int rc = sorted_scan(e->fire_key, nf, (int64_t)nf)) return rc;
      hipLaunchKernelGGL(k_fire_emit, dim3((unsigned)((nf + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, e->stream, e->s,
                         e->late_key_sorted, (int64_t)nf, e->idx_bits, e->seg, e->late_acc, e->late_scan, df1, dts,
                         e->cur_wm, e->headpos_scan, e->out_base);
      e->late_fires_host += (int64_t)nf;
      HIPCHK(e, hipMemsetAsync(e->fire_count, 0, 8, e->stream));
    }
    if (nl > 0 && !sliding && e->late_fused) {
      size_t tb = e->temp_bytes;
      HIPCHK(e, rocprim::radix_sort_keys(e->temp, tb, e->late_key, e->late_key_sorted, (size_t)nl, 0, key_bits, e->stream));
      FW_DISPATCH(launch_late_fused_t, e, (int64_t)nl, dv, df1);
      e->late_fires_host += (int64_t)nl;
      HIPCHK(e, hipMemsetAsync(e->late_count, 0, 8, e->stream));
    } else if (nl > 0) {
      if (int rc = sorted_scan(e->late_key, nl, sliding ? 0 : (int64_t)nl)) return rc;
      const int blocks = (int)((nl + BLOCK - 1) / BLOCK);
      if (!sliding) {
        hipLaunchKernelGGL(k_late_emit, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->late_key_sorted, (int64_t)nl,
                           e->idx_bits, e->seg, e->late_acc, e->late_scan, df1, e->ordinal, e->headpos_scan, e->out_base);
        e->late_fires_host += (int64_t)nl;
      }
      hipLaunchKernelGGL(k_late_commit, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->late_key_sorted, (int64_t)nl,
                         e->idx_bits, e->seg, e->late_scan, df1, e->ordinal, e->headpos_scan);
      HIPCHK(e, hipMemsetAsync(e->late_count, 0, 8, e->stream));
    }
    if (nl > 0 || nf > 0) e->phase_end((int64_t)(nl + nf));
    if (nf > 0 || (nl > 0 && !sliding)) e->out_dirty = true;
  }
  HIPCHK(e, hipGetLastError());
  // every reader of this push's columns (k_route, k_aggregate's direct records, the f1 fix-up, the late
  // path) is ordered before this point of the engine stream: buffer set par (routed buffers, host staging)
  // may be rewritten after it
  HIPCHK(e, hipEventRecord(e->ev_agg[par], e->stream));
  if (e->track_consumed && !e->no_consumed) {
    HIPCHK(e, hipEventRecord(e->ev_consumed[e->pushes % fw_engine::NCONS], e->stream));
    e->cons_push[e->pushes % fw_engine::NCONS] = e->pushes;
  }
  e->pushes++;
  e->ordinal += n;
  e->records_in += n;
  return FW_OK;
}

int fw_stream_wait_input(fw_engine* e, void* stream, int32_t back) {
  if (!e || back < 0 || back >= fw_engine::NCONS) return FW_ERR_INVALID_ARG;
  if (back >= e->pushes) return FW_OK;   // no such push
  HIPCHK(e, hipSetDevice(e->dev));
  const int64_t target = e->pushes - 1 - back;
  const int slot = (int)(target % fw_engine::NCONS);
  if (e->cons_push[slot] == target) {
    HIPCHK(e, hipStreamWaitEvent((hipStream_t)stream, e->ev_consumed[slot], 0));
  } else {   // not tracked yet: wait for everything the engine stream holds now (a later point, never a cycle)
    HIPCHK(e, hipEventRecord(e->ev_now, e->stream));
    HIPCHK(e, hipStreamWaitEvent((hipStream_t)stream, e->ev_now, 0));
  }
  e->track_consumed = true;
  return FW_OK;
}

// PurgingTrigger + allowed lateness: window m's cleanup timers outlive its purged state until its cleanup time;
// its slot's ghost column holds them (Spec::gfirst), tagged with m
static int64_t host_max_ts(const fw::Spec& s, int64_t m) {
  return fw::jsub(fw::jadd(fw::jadd(s.offset, (int64_t)((uint64_t)m * (uint64_t)s.size)), s.size), 1);
}
static int ghost_track(fw_engine* e, int64_t m) {
  if (e->ghost_windows.count(m)) return FW_OK;
  const int32_t p = (int32_t)floor_mod(m, e->s.P);
  for (int64_t o : e->ghost_windows)
    if (floor_mod(o, e->s.P) == p)
      return fail(e, FW_ERR_CAPACITY, "purged windows' cleanup timers: two windows in one slice slot (raise max_open_slices)");
  e->ghost_windows.insert(m);
  // the slot's column starts empty: a window that held slot p before left no ordinals behind to be inherited
  if (int rc = launch_fill(e, e->s.gfirst + (size_t)p * (size_t)e->s.stride, INT64_MAX, e->s.stride)) return rc;
  return launch_fill(e, e->s.gtag + p, m, 1);
}
// the watermark moves from wm_old to wm_new: windows whose cleanup time it reaches drop their timers; windows it
// fires (maxTimestamp in (wm_old, wm_new]) that stay within their lateness get a ghost column
static int ghost_advance(fw_engine* e, int64_t wm_old, int64_t wm_new) {
  const fw::Spec& s = e->s;
  for (auto it = e->ghost_windows.begin(); it != e->ghost_windows.end();) {
    const int64_t m = *it;
    if (fw::cleanup_time(host_max_ts(s, m), s.lateness) > wm_new) { ++it; continue; }
    const int32_t p = (int32_t)floor_mod(m, s.P);
    int rc = launch_fill(e, s.gfirst + (size_t)p * (size_t)s.stride, INT64_MAX, s.stride);
    if (!rc) rc = launch_fill(e, s.gtag + p, FREE_TAG, 1);
    if (rc) return rc;
    it = e->ghost_windows.erase(it);
  }
  // m with maxTimestamp in (max(wm_old, wm_new - lateness), wm_new]: maxTimestamp = offset + (m + 1) size - 1
  const __int128 lo = std::max<__int128>((__int128)wm_old, (__int128)wm_new - (__int128)s.lateness);
  const __int128 base = (__int128)s.offset - 1;
  auto m_at_or_below = [&](__int128 t) {   // largest m with maxTimestamp <= t
    const __int128 x = t - base;
    __int128 q = x / s.size;
    if (x % s.size != 0 && x < 0) --q;
    return q - 1;
  };
  const __int128 m_hi = m_at_or_below(wm_new), m_lo = m_at_or_below(lo) + 1;
  if (m_hi - m_lo > (__int128)s.P) return fail(e, FW_ERR_CAPACITY, "purged windows' cleanup timers: more windows within their lateness than slice slots");
  for (__int128 m = m_lo; m <= m_hi; ++m) {
    if (m < (__int128)INT64_MIN / 2 || m > (__int128)INT64_MAX / 2) continue;
    if (fw::cleanup_time(host_max_ts(s, (int64_t)m), s.lateness) <= wm_new) continue;
    int rc = ghost_track(e, (int64_t)m);
    if (rc) return rc;
  }
  return FW_OK;
}

// restored disarmed windows whose maxTimestamp the watermark passed: their re-armed panes (list state: keys)
// fired with it; the rest never fires again (cleanup at the cleanup time, as any window)
static int disarm_advance(fw_engine* e, int64_t wm) {
  for (auto it = e->disarmed.begin(); it != e->disarmed.end();) {
    const int64_t m = *it;   // (tumbling: a slice number; sliding: a window number, its own pane's slot)
    const int64_t max_ts = jsub(jadd(host_window_start(e->cfg, m), e->s.size), 1);
    if (max_ts > wm) { ++it; continue; }
    const int32_t p = (int32_t)floor_mod(m, e->s.P);
    HIPCHK(e, hipMemsetAsync(e->s.disarm + p, 0, 1, e->stream));
    HIPCHK(e, hipMemsetAsync(e->s.armed + (size_t)p * (size_t)e->s.stride, 0, (size_t)e->s.stride, e->stream));
    it = e->disarmed.erase(it);
  }
  return FW_OK;
}

int fw_advance_watermark(fw_engine* e, int64_t wm) {
  if (!e) return FW_ERR_INVALID_ARG;
  if (e->sticky) return e->sticky;
  HIPCHK(e, hipSetDevice(e->dev));
  e->state_epoch++;
  if (e->session) return session_watermark(e, wm);
  if (e->list) return list_watermark(e, wm);
  if (wm > e->cur_wm && e->cfg.trigger == FW_TRIGGER_PURGING_EVENT_TIME && e->cfg.allowed_lateness > 0 &&
      e->cfg.assigner == FW_SLIDING)
    e->adv_log.push_back({wm, e->ordinal});
  if (e->s.gtag && wm > e->cur_wm) {
    int rc = ghost_advance(e, e->cur_wm, wm);
    if (rc) return rc;
  }
  if (wm <= e->cur_wm || wm_quiet(e->s, e->cur_wm, wm)) {   // nothing fires or purges: the mark only
    if (e->out_dirty) {   // per-element fires appended since the last device mark: the mark needs the count
      hipLaunchKernelGGL(k_mark_only, dim3(1), dim3(1), 0, e->stream, e->s, wm);
      HIPCHK(e, hipGetLastError());
      e->hmarks.push_back({wm, e->dev_marks++, true});
      e->out_dirty = false;
    } else {              // no launch: the position of the previous device mark
      e->hmarks.push_back({wm, e->dev_marks - 1, false});
    }
    if (wm > e->cur_wm) e->cur_wm = wm;
    return FW_OK;
  }
  e->phase_begin(FW_PHASE_FIRE);
  FW_DISPATCH(launch_watermark_t, e, e->cur_wm, wm);
  e->phase_end(e->s.stride);
  HIPCHK(e, hipGetLastError());
  if (int rc = disarm_advance(e, wm)) return rc;
  e->hmarks.push_back({wm, e->dev_marks++, true});
  e->out_dirty = false;
  e->cur_wm = wm;
  // evict dead keys once the directory is more than compact_fill full (the count posted by an earlier
  // firing watermark: read without a sync)
  if (e->compact_ok && e->dir_keys_host &&
      (double)__atomic_load_n(e->dir_keys_host, __ATOMIC_RELAXED) > e->compact_fill * (double)e->s.D) {
    HIPCHK(e, hipMemsetAsync(e->s.stats + ST_DIR_KEYS, 0, 8, e->stream));
    hipLaunchKernelGGL(k_compact, dim3((unsigned)(e->s.D >> e->s.kb_bits)), dim3(CP_THREADS), e->compact_lds, e->stream,
                       e->s, e->kg_evicted);
    HIPCHK(e, hipGetLastError());
    __atomic_store_n(e->dir_keys_host, 0u, __ATOMIC_RELAXED);
    e->compactions++;
    e->state_epoch++;
  }
  return FW_OK;
}

int fw_sync(fw_engine* e) {
  if (!e) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipSetDevice(e->dev));
  HIPCHK(e, hipStreamSynchronize(e->rstream));
  return check_device_error(e);
}

int fw_collect(fw_engine* e, fw_out* o, int32_t mem) {
  if (!e || !o) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipSetDevice(e->dev));
  int rc = check_device_error(e);
  if (rc) return rc;
  unsigned long long cnt = 0, mc = 0;
  if (!e->h_pin_cnt && hipHostMalloc((void**)&e->h_pin_cnt, 16, hipHostMallocDefault) != hipSuccess) e->h_pin_cnt = nullptr;
  if (e->h_pin_cnt) {
    HIPCHK(e, hipMemcpyAsync(e->h_pin_cnt, e->s.o.count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->h_pin_cnt + 1, e->s.o.mark_count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    cnt = e->h_pin_cnt[0];
    mc = e->h_pin_cnt[1];
  } else {
    HIPCHK(e, hipMemcpyAsync(&cnt, e->s.o.count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(&mc, e->s.o.mark_count, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  if ((int64_t)cnt > e->s.o.capacity) return fail(e, FW_ERR_CAPACITY, "output log capacity exceeded");
  const OutLog& L = e->s.o;
  // the marks in emission order: device marks as written, the others at the position of the device mark
  // before them
  const int64_t nm = (int64_t)e->hmarks.size();
  if (nm > L.mark_capacity || (int64_t)mc != e->dev_marks) return fail(e, FW_ERR_CAPACITY, "watermark mark log capacity exceeded");
  e->h_dev_pos.resize((size_t)std::max<int64_t>(e->dev_marks, 1));
  if (e->dev_marks > 0)
    HIPCHK(e, hipMemcpy(e->h_dev_pos.data(), L.mark_pos, 8 * (size_t)e->dev_marks, hipMemcpyDeviceToHost));
  e->h_mark_wm.resize((size_t)std::max<int64_t>(nm, 1));
  e->h_mark_pos.resize((size_t)std::max<int64_t>(nm, 1));
  for (int64_t i = 0; i < nm; ++i) {
    const auto& m = e->hmarks[(size_t)i];
    e->h_mark_wm[(size_t)i] = m.wm;
    e->h_mark_pos[(size_t)i] = m.dev >= 0 ? e->h_dev_pos[(size_t)m.dev] : 0;
  }
  e->hmarks.clear();
  e->dev_marks = 0;
  e->out_dirty = false;
  e->list_out = 0;
  const int64_t n = (int64_t)cnt;
  std::memset(o, 0, sizeof(*o));
  o->n = n;
  o->n_marks = nm;
  const bool f64 = e->s.vt == FW_VALUE_F64;
  if (mem == FW_MEM_DEVICE) {
    o->key = L.key; o->f1 = L.f1; o->ts = L.ts;
    if (f64) { o->sum_f64 = (const double*)L.sum; o->min_f64 = (const double*)L.mn; o->max_f64 = (const double*)L.mx; }
    else { o->sum_i64 = L.sum; o->min_i64 = L.mn; o->max_i64 = L.mx; }
    o->count = L.cnt;
    if (nm > 0) {   // the merged marks back into the device arrays
      HIPCHK(e, hipMemcpy(L.mark_wm, e->h_mark_wm.data(), 8 * (size_t)nm, hipMemcpyHostToDevice));
      HIPCHK(e, hipMemcpy(L.mark_pos, e->h_mark_pos.data(), 8 * (size_t)nm, hipMemcpyHostToDevice));
    }
    o->mark_wm = L.mark_wm; o->mark_pos = L.mark_pos;
    o->win_start = L.win_start;
  } else {
    if (n > e->h_pin_rows && n <= fw_engine::COLLECT_PIN_MAX) {
      if (e->h_pin) (void)hipHostFree(e->h_pin);
      const int64_t rows = std::min<int64_t>(std::max<int64_t>(2 * n, 4096), fw_engine::COLLECT_PIN_MAX);
      if (hipHostMalloc((void**)&e->h_pin, 8 * 8 * (size_t)rows, hipHostMallocDefault) != hipSuccess) {
        e->h_pin = nullptr;
        e->h_pin_rows = 0;
      } else {
        e->h_pin_rows = rows;
      }
    }
    const bool pinned = e->h_pin && n <= e->h_pin_rows;
    int col = 0;
    auto cp = [&](std::vector<int64_t>& h, const int64_t* d, int64_t cnt_) -> const int64_t* {
      if (!d) return nullptr;
      if (pinned) {   // column `col` of the pinned staging
        int64_t* dst = e->h_pin + (size_t)(col++) * (size_t)e->h_pin_rows;
        if (cnt_ > 0) (void)hipMemcpyAsync(dst, d, 8 * cnt_, hipMemcpyDeviceToHost, e->stream);
        return dst;
      }
      h.resize((size_t)std::max<int64_t>(cnt_, 1));
      if (cnt_ > 0) (void)hipMemcpyAsync(h.data(), d, 8 * cnt_, hipMemcpyDeviceToHost, e->stream);
      return h.data();
    };
    o->key = cp(e->h_key, L.key, n);
    o->f1 = cp(e->h_f1, L.f1, n);
    o->ts = cp(e->h_ts, L.ts, n);
    const int64_t* su = cp(e->h_sum, L.sum, n);
    const int64_t* mn = cp(e->h_mn, L.mn, n);
    const int64_t* mx = cp(e->h_mx, L.mx, n);
    o->count = cp(e->h_cnt, L.cnt, n);
    o->win_start = cp(e->h_start, L.win_start, n);
    if (f64) { o->sum_f64 = (const double*)su; o->min_f64 = (const double*)mn; o->max_f64 = (const double*)mx; }
    else { o->sum_i64 = su; o->min_i64 = mn; o->max_i64 = mx; }
    o->mark_wm = e->h_mark_wm.data();
    o->mark_pos = e->h_mark_pos.data();
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  // only the fields the reduce function asked for
  const int32_t um = e->list ? FW_AGG_SUM : e->cfg.agg_mask;   // list state: the elements' values
  if (!(um & FW_AGG_SUM)) { o->sum_i64 = nullptr; o->sum_f64 = nullptr; }
  if (!(um & (FW_AGG_MIN | FW_AGG_MINBY))) { o->min_i64 = nullptr; o->min_f64 = nullptr; }
  if (!(um & (FW_AGG_MAX | FW_AGG_MAXBY))) { o->max_i64 = nullptr; o->max_f64 = nullptr; }
  if (!(um & FW_AGG_COUNT)) o->count = nullptr;
  // the log restarts; device pointers handed out above stay valid until the next enqueue
  HIPCHK(e, hipMemsetAsync(L.count, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(L.mark_count, 0, 8, e->stream));
  if (mem == FW_MEM_HOST) HIPCHK(e, hipStreamSynchronize(e->stream));
  return FW_OK;
}

static uint32_t drain_colmask(const OutLog& L) {
  return (L.key ? 1u : 0u) | (L.f1 ? 2u : 0u) | (L.ts ? 4u : 0u) | (L.sum ? 8u : 0u) | (L.mn ? 16u : 0u) | (L.mx ? 32u : 0u) |
         (L.cnt ? 64u : 0u) | (L.win_start ? 128u : 0u);
}

int fw_collect_begin(fw_engine* e, int32_t* ticket) {
  if (!e || !ticket) return FW_ERR_INVALID_ARG;
  if (e->sticky) return e->sticky;
  HIPCHK(e, hipSetDevice(e->dev));
  const int b = (int)(e->drain_seq % fw_engine::NDRAIN);
  fw_engine::Drain& d = e->drains[b];
  if (d.pending) { e->err = "fw_collect_begin: three drains outstanding (fw_collect_end the oldest first)"; return FW_ERR_INVALID_ARG; }
  const OutLog& L = e->s.o;
  const uint32_t colmask = drain_colmask(L);
  const int ncols = __builtin_popcount(colmask);
  const size_t words = (size_t)ncols * (size_t)std::min<int64_t>(L.capacity, fw_engine::DRAIN_ROWS_MAX) +
                       (size_t)L.mark_capacity + 8;   // + hdr[4], the blocks' arrival counter
  if (!d.host) {
    e->drain_rows = std::min<int64_t>(L.capacity, fw_engine::DRAIN_ROWS_MAX);
    if (hipHostMalloc((void**)&d.host, 8 * words, hipHostMallocMapped) != hipSuccess) {
      d.host = nullptr;
      return fail(e, FW_ERR_DEVICE, "fw_collect_begin: pinned staging allocation failed");
    }
    HIPCHK(e, hipHostGetDevicePointer((void**)&d.dptr, d.host, 0));
    HIPCHK(e, hipMalloc((void**)&d.dev, 8 * words));
    HIPCHK(e, hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    HIPCHK(e, hipEventCreateWithFlags(&d.staged, hipEventDisableTiming));
    if (!e->dstream) HIPCHK(e, hipStreamCreateWithFlags(&e->dstream, hipStreamNonBlocking));
  }
  int64_t* marks = d.dev + (size_t)ncols * (size_t)e->drain_rows;
  int64_t* hdr = marks + L.mark_capacity;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((e->drain_rows + BLOCK - 1) / BLOCK, 512));
  if (!d.host_ready) {   // the arrival counter starts at zero (k_drain returns it there)
    HIPCHK(e, hipMemsetAsync(hdr + 4, 0, 8, e->stream));
    d.host_ready = true;
  }
  hipLaunchKernelGGL(k_drain, dim3(blocks), dim3(BLOCK), 0, e->stream, L, (const int32_t*)e->s.err, e->drain_rows, d.dev,
                     marks, hdr, (unsigned int*)(hdr + 4), colmask);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipEventRecord(d.staged, e->stream));
  // to the host on the drain stream, beside whatever the engine stream runs next
  HIPCHK(e, hipStreamWaitEvent(e->dstream, d.staged, 0));
  hipLaunchKernelGGL(k_drain_host, dim3(64), dim3(BLOCK), 0, e->dstream, d.dev, marks, hdr, e->drain_rows, L.mark_capacity,
                     colmask, d.dptr);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipEventRecord(d.done, e->dstream));
  // the marks since the last collect belong to this drain; the log restarts on the device
  d.marks.swap(e->hmarks);
  e->hmarks.clear();
  d.dev_marks = e->dev_marks;
  e->dev_marks = 0;
  e->out_dirty = false;
  e->list_out = 0;
  d.pending = true;
  d.ticket = (int32_t)(e->drain_seq++ & 0x7FFFFFFF);
  *ticket = d.ticket;
  return FW_OK;
}

int fw_collect_end(fw_engine* e, int32_t ticket, fw_out* o) {
  if (!e || !o || ticket < 0) return FW_ERR_INVALID_ARG;
  fw_engine::Drain* dp = nullptr;
  for (fw_engine::Drain& x : e->drains)
    if (x.pending && x.ticket == ticket) dp = &x;
  if (!dp) {
    e->err = "fw_collect_end: no such drain outstanding";
    return FW_ERR_INVALID_ARG;
  }
  fw_engine::Drain& d = *dp;
  HIPCHK(e, hipSetDevice(e->dev));
  HIPCHK(e, hipEventSynchronize(d.done));
  d.pending = false;
  const OutLog& L = e->s.o;
  const uint32_t colmask = drain_colmask(L);
  const int64_t* marks = d.host + (size_t)__builtin_popcount(colmask) * (size_t)e->drain_rows;
  const int64_t* hdr = marks + L.mark_capacity;
  if (int rc = device_error(e, (int32_t)hdr[3])) return rc;
  if (!hdr[2]) return fail(e, FW_ERR_CAPACITY, "fw_collect_end: more results than an asynchronous drain holds (collect more often)");
  if (hdr[1] != d.dev_marks) return fail(e, FW_ERR_CAPACITY, "watermark mark log capacity exceeded");
  const int64_t n = hdr[0], nm = (int64_t)d.marks.size();
  d.mark_wm.resize((size_t)std::max<int64_t>(nm, 1));
  d.mark_pos.resize((size_t)std::max<int64_t>(nm, 1));
  for (int64_t i = 0; i < nm; ++i) {
    d.mark_wm[(size_t)i] = d.marks[(size_t)i].wm;
    d.mark_pos[(size_t)i] = d.marks[(size_t)i].dev >= 0 ? marks[d.marks[(size_t)i].dev] : 0;
  }
  std::memset(o, 0, sizeof(*o));
  o->n = n;
  o->n_marks = nm;
  auto col = [&](int c, const void* present) -> const int64_t* {
    return present ? d.host + (size_t)dr_slot(colmask, c) * (size_t)e->drain_rows : nullptr;
  };
  o->key = col(0, L.key);
  o->f1 = col(1, L.f1);
  o->ts = col(2, L.ts);
  const int64_t* su = col(3, L.sum);
  const int64_t* mn = col(4, L.mn);
  const int64_t* mx = col(5, L.mx);
  o->count = col(6, L.cnt);
  o->win_start = col(7, L.win_start);
  if (e->s.vt == FW_VALUE_F64) { o->sum_f64 = (const double*)su; o->min_f64 = (const double*)mn; o->max_f64 = (const double*)mx; }
  else { o->sum_i64 = su; o->min_i64 = mn; o->max_i64 = mx; }
  o->mark_wm = d.mark_wm.data();
  o->mark_pos = d.mark_pos.data();
  const int32_t um = e->list ? FW_AGG_SUM : e->cfg.agg_mask;   // only the fields the reduce function asked for
  if (!(um & FW_AGG_SUM)) { o->sum_i64 = nullptr; o->sum_f64 = nullptr; }
  if (!(um & (FW_AGG_MIN | FW_AGG_MINBY))) { o->min_i64 = nullptr; o->min_f64 = nullptr; }
  if (!(um & (FW_AGG_MAX | FW_AGG_MAXBY))) { o->max_i64 = nullptr; o->max_f64 = nullptr; }
  if (!(um & FW_AGG_COUNT)) o->count = nullptr;
  return FW_OK;
}

int fw_get_stats(fw_engine* e, fw_stats* st) {
  if (!e || !st) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipSetDevice(e->dev));
  unsigned long long d[ST_NSTATS];
  HIPCHK(e, hipMemcpyAsync(d, e->s.stats, sizeof(d), hipMemcpyDeviceToHost, e->stream));
  std::vector<int64_t> tags((size_t)e->s.P);
  HIPCHK(e, hipMemcpyAsync(tags.data(), e->s.slice_tag, 8 * (size_t)e->s.P, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::memset(st, 0, sizeof(*st));
  st->records_in = e->records_in;
  st->records_late = (int64_t)d[ST_LATE];
  st->panes_fired = (int64_t)d[ST_FIRED] + e->late_fires_host;
  st->late_fires = e->late_fires_host + (int64_t)d[ST_LATE_FIRES];   // (device-counted: session windows)
  int64_t live = 0;
  for (int64_t t : tags) live += t != FREE_TAG;
  st->slices_live = live;
  st->keys_resident = (int64_t)d[ST_DIR_KEYS];   // the Long.MIN_VALUE key's own column not counted
  st->ingest_form = e->routed ? 2 : 1;
  st->compactions = e->compactions;
  return FW_OK;
}

int fw_debug_stamps(fw_engine* e, int64_t* out, int64_t n) {
  if (!e || !out) return FW_ERR_INVALID_ARG;
  if (!e->rb.stamps) return FW_ERR_UNSUPPORTED;
  HIPCHK(e, hipMemcpyAsync(out, e->rb.stamps, 8 * (size_t)std::min<int64_t>(n, (int64_t)16 << 16), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return FW_OK;
}

int fw_debug_counters(fw_engine* e, int64_t* out8) {
  if (!e || !out8) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipMemcpyAsync(out8, e->s.stats, 8 * ST_NSTATS, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return FW_OK;
}

int fw_set_stream(fw_engine* e, void* stream) {
  if (!e) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipSetDevice(e->dev));
  HIPCHK(e, hipStreamSynchronize(e->rstream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->client = stream;
  e->has_client = true;
  return FW_OK;
}

int fw_set_profiling(fw_engine* e, int32_t enable) {
  if (!e) return FW_ERR_INVALID_ARG;
  e->profiling = enable != 0;
  return FW_OK;
}

int fw_get_profile(fw_engine* e, fw_profile* out) {
  if (!e || !out) return FW_ERR_INVALID_ARG;
  HIPCHK(e, hipSetDevice(e->dev));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (auto& t : e->timed) {
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, t.a, t.b));
    e->prof_ms[t.phase] += ms;
    e->prof_launches[t.phase] += 1;
    e->prof_records[t.phase] += t.records;
    e->event_pool.push_back(t.a);
    e->event_pool.push_back(t.b);
  }
  e->timed.clear();
  for (int i = 0; i < FW_NPHASES; ++i) {
    out->ms[i] = e->prof_ms[i];
    out->launches[i] = e->prof_launches[i];
    out->records[i] = e->prof_records[i];
    e->prof_ms[i] = 0; e->prof_launches[i] = 0; e->prof_records[i] = 0;
  }
  return FW_OK;
}

const char* fw_last_error(const fw_engine* e) { return e ? e->err.c_str() : g_create_error.c_str(); }

void fw_destroy(fw_engine* e) { delete e; }

// key group of a Long key (KeyGroupRangeAssignment.assignToKeyGroup :51-64 over Long.hashCode)
static int32_t host_key_group(const fw::Spec& s, int64_t key) {
  return fw::key_group_for_hash(fw::long_hash_code(key), s.mp);
}

// an argument the call rejects: reported like a failure but, unlike one, leaves the engine usable
static int reject(fw_engine* e, int code, const std::string& msg) {
  e->err = msg;
  return code;
}

// window panes hold state a checkpoint blob does not carry (the sliding assigner's extra windows)
static bool window_panes_used(fw_engine* e) {
  if (e->s.W == 0) return false;
  unsigned long long n = 0;
  if (hipMemcpy(&n, e->s.stats + ST_QUIRK, 8, hipMemcpyDeviceToHost) != hipSuccess) return true;
  return n > 0;
}

static void snap_header(const fw_engine* e, int32_t kg, int64_t n, int64_t* h) {
  const fw_config& c = e->cfg;
  const int64_t w[FW_SNAP_HEADER_WORDS] = {FW_SNAP_MAGIC, 2, kg, n, e->cur_wm, c.assigner, c.size,
                                          c.assigner == FW_SLIDING ? c.slide : c.size, c.offset, c.value_type,
                                          c.agg_mask, c.keep_first_f1 ? 1 : 0, c.allowed_lateness,
                                          (int64_t)c.trigger | ((int64_t)c.agg_flags << 8)};
  memcpy(h, w, sizeof(w));
}

// every key group's entries, from one copy of the directory and the live slices' columns.  The heap
// backend walks its per-key-group maps instead (HeapKeyedStateBackend.java:196-212); here the panes of
// all key groups sit in one dense table, so one pass sorts them into key groups
static int build_snapshot(fw_engine* e) {
  if (e->snap_epoch == e->state_epoch) return FW_OK;
  const fw::Spec& s = e->s;
  HIPCHK(e, hipStreamSynchronize(e->rstream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int rc = check_device_error(e);
  if (rc) return rc;
  std::vector<int64_t> keys((size_t)s.D), tags((size_t)s.P);
  int32_t min_used = 0;
  HIPCHK(e, hipMemcpy(keys.data(), s.dir_keys, 8 * (size_t)s.D, hipMemcpyDeviceToHost));
  HIPCHK(e, hipMemcpy(tags.data(), s.slice_tag, 8 * (size_t)s.P, hipMemcpyDeviceToHost));
  HIPCHK(e, hipMemcpy(&min_used, s.dir_min_used, 4, hipMemcpyDeviceToHost));
  const int32_t mp = s.mp;
  std::vector<int32_t> kid_kg((size_t)s.stride, -1);
  for (int64_t k = 0; k < s.D; ++k)
    if (keys[k] != fw::EMPTY_KEY) kid_kg[k] = host_key_group(s, keys[k]);
  if (min_used) kid_kg[s.D] = host_key_group(s, fw::EMPTY_KEY);
  e->snap_kg.assign((size_t)mp, {});
  e->snap_wkg.assign((size_t)mp, {});
  e->snap_unarmed.clear();
  e->snap_has_key.assign((size_t)mp, 0);
  e->snap_any_key = false;
  for (size_t k = 0; k < kid_kg.size(); ++k)
    if (kid_kg[k] >= 0) { e->snap_has_key[(size_t)kid_kg[k]] = 1; e->snap_any_key = true; }
  if (e->kg_evicted) {   // key groups whose keys were all evicted still had state (StateTable.get(kg) != null)
    std::vector<uint8_t> ev((size_t)mp);
    HIPCHK(e, hipMemcpy(ev.data(), e->kg_evicted, (size_t)mp, hipMemcpyDeviceToHost));
    for (int32_t k = 0; k < mp; ++k) if (ev[(size_t)k]) { e->snap_has_key[(size_t)k] = 1; e->snap_any_key = true; }
  }
  if (e->list) {   // list state (tumbling): the slices' element buffers, grouped by (window, key) in arrival order
    e->snap_list.clear();
    std::vector<unsigned long long> lc((size_t)s.P);
    HIPCHK(e, hipMemcpy(lc.data(), e->lst.cnt, 8 * (size_t)s.P, hipMemcpyDeviceToHost));
    std::vector<int64_t> rows;
    for (int32_t p = 0; p < s.P; ++p) {
      const int64_t m = tags[(size_t)p];
      if (m == fw::FREE_TAG) continue;
      const int64_t ne = std::min<int64_t>((int64_t)lc[(size_t)p], e->lst.cap);
      rows.resize((size_t)ne * LST_WORDS);
      if (ne > 0)
        HIPCHK(e, hipMemcpy(rows.data(), e->lst.buf + (size_t)p * (size_t)e->lst.cap * LST_WORDS, 8 * rows.size(),
                            hipMemcpyDeviceToHost));
      std::vector<uint8_t> armed;
      if (e->disarmed.count(m)) {   // a restored window that fired before: the keys no record re-armed since
        armed.resize((size_t)s.stride);
        HIPCHK(e, hipMemcpy(armed.data(), s.armed + (size_t)p * (size_t)s.stride, (size_t)s.stride, hipMemcpyDeviceToHost));
      }
      for (int64_t j = 0; j < ne; ++j) {
        const int64_t* x = &rows[(size_t)j * LST_WORDS];   // kid, ordinal, value, f1
        if (x[0] < 0 || x[0] >= s.stride || kid_kg[(size_t)x[0]] < 0) continue;
        const int64_t key = x[0] == s.D ? fw::EMPTY_KEY : keys[(size_t)x[0]];
        e->snap_list[{m, key}].push_back({x[1], x[2], x[3]});
        if (!armed.empty() && !armed[(size_t)x[0]]) e->snap_unarmed.insert({m, key});
      }
    }
    for (auto& kv : e->snap_list) {
      std::sort(kv.second.begin(), kv.second.end());
      const int64_t key = kv.first.second;
      const int64_t ent[FW_SNAP_ENTRY_WORDS] = {kv.first.first, key, 0, INT64_MAX, INT64_MIN, 0,
                                                kv.second[0][0] - e->ordinal, 0};
      auto& v = e->snap_kg[(size_t)host_key_group(s, key)];
      v.insert(v.end(), ent, ent + FW_SNAP_ENTRY_WORDS);
    }
    e->snap_gkg.assign((size_t)mp, {});
    e->snap_epoch = e->state_epoch;
    return FW_OK;
  }
  const size_t st = (size_t)s.stride;
  std::vector<int64_t> sum(st), mn, mx, cnt, first, f1v;
  std::vector<uint8_t> present;
  for (int32_t p = 0; p < s.P; ++p) {
    const int64_t m = tags[p];
    if (m == fw::FREE_TAG) continue;
    const size_t off = (size_t)p * st;
    auto get = [&](std::vector<int64_t>& v, const int64_t* col) -> hipError_t {
      if (!col) return hipSuccess;
      v.resize(st);
      return hipMemcpy(v.data(), col + off, 8 * st, hipMemcpyDeviceToHost);
    };
    HIPCHK(e, get(sum, s.c.sum));
    HIPCHK(e, get(mn, s.c.mn));
    HIPCHK(e, get(mx, s.c.mx));
    HIPCHK(e, get(cnt, s.c.cnt));
    if (s.first) {
      HIPCHK(e, get(first, s.c.first));
      HIPCHK(e, get(f1v, s.c.f1v));
    } else {
      present.resize(st);
      HIPCHK(e, hipMemcpy(present.data(), s.c.present + off, st, hipMemcpyDeviceToHost));
    }
    std::vector<uint8_t> armed;
    const bool dis = s.assigner != FW_SLIDING && e->disarmed.count(m) != 0;
    if (dis) {
      armed.resize(st);
      HIPCHK(e, hipMemcpy(armed.data(), s.armed + off, st, hipMemcpyDeviceToHost));
    }
    for (size_t k = 0; k < st; ++k) {
      const bool pres = s.first ? first[k] != INT64_MAX : present[k] != 0;
      if (!pres || kid_kg[k] < 0) continue;
      const int64_t key = (int64_t)k == s.D ? fw::EMPTY_KEY : keys[k];
      if (dis && !armed[k]) e->snap_unarmed.insert({m, key});
      const int64_t ent[FW_SNAP_ENTRY_WORDS] = {
          m, key, sum[k], s.c.mn ? mn[k] : INT64_MAX, s.c.mx ? mx[k] : INT64_MIN,
          s.c.cnt ? (s.by ? cnt[k] - e->ordinal : cnt[k]) : 0,
          s.first ? first[k] - e->ordinal : -1, s.first ? f1v[k] : 0};
      auto& v = e->snap_kg[(size_t)kid_kg[k]];
      v.insert(v.end(), ent, ent + FW_SNAP_ENTRY_WORDS);
    }
  }
  // sliding: the windows' own panes (restored window state, records below offset - slide)
  if (s.W > 0) {
    std::vector<int64_t> wtags((size_t)s.W);
    HIPCHK(e, hipMemcpy(wtags.data(), s.wtag, 8 * (size_t)s.W, hipMemcpyDeviceToHost));
    for (int32_t w = 0; w < s.W; ++w) {
      const int64_t n = wtags[(size_t)w];
      if (n == fw::FREE_TAG) continue;
      const size_t off = (size_t)w * st;
      auto get = [&](std::vector<int64_t>& v, const int64_t* col) -> hipError_t {
        if (!col) return hipSuccess;
        v.resize(st);
        return hipMemcpy(v.data(), col + off, 8 * st, hipMemcpyDeviceToHost);
      };
      HIPCHK(e, get(sum, s.wc.sum));
      HIPCHK(e, get(mn, s.wc.mn));
      HIPCHK(e, get(mx, s.wc.mx));
      HIPCHK(e, get(cnt, s.wc.cnt));
      if (s.first) {
        HIPCHK(e, get(first, s.wc.first));
        HIPCHK(e, get(f1v, s.wc.f1v));
      } else {
        present.resize(st);
        HIPCHK(e, hipMemcpy(present.data(), s.wc.present + off, st, hipMemcpyDeviceToHost));
      }
      if (e->disarmed.count(n)) {   // a restored window that fired before: the keys no record re-armed since
        std::vector<uint8_t> armed(st);
        HIPCHK(e, hipMemcpy(armed.data(), s.armed + off, st, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < st; ++k)
          if (!armed[k] && kid_kg[k] >= 0) e->snap_unarmed.insert({n, (int64_t)k == s.D ? fw::EMPTY_KEY : keys[k]});
      }
      for (size_t k = 0; k < st; ++k) {
        const bool pres = s.first ? first[k] != INT64_MAX : present[k] != 0;
        if (!pres || kid_kg[k] < 0) continue;
        const int64_t key = (int64_t)k == s.D ? fw::EMPTY_KEY : keys[k];
        const int64_t ent[FW_SNAP_ENTRY_WORDS] = {
            n, key, sum[k], s.wc.mn ? mn[k] : INT64_MAX, s.wc.mx ? mx[k] : INT64_MIN,
            s.wc.cnt ? (s.by ? cnt[k] - e->ordinal : cnt[k]) : 0,
            s.first ? first[k] - e->ordinal : -1, s.first ? f1v[k] : 0};
        auto& v = e->snap_wkg[(size_t)kid_kg[k]];
        v.insert(v.end(), ent, ent + FW_SNAP_ENTRY_WORDS);
      }
    }
  }
  // purged windows' cleanup timers (PurgingTrigger + allowed lateness)
  e->snap_gkg.assign((size_t)mp, {});
  for (int64_t m : e->ghost_windows) {
    const size_t off = (size_t)floor_mod(m, s.P) * st;
    std::vector<int64_t> g(st);
    HIPCHK(e, hipMemcpy(g.data(), s.gfirst + off, 8 * st, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < st; ++k) {
      if (g[k] == INT64_MAX || kid_kg[k] < 0) continue;
      const int64_t key = (int64_t)k == s.D ? fw::EMPTY_KEY : keys[k];
      auto& v = e->snap_gkg[(size_t)kid_kg[k]];
      v.insert(v.end(), {m, key, s.first ? g[k] - e->ordinal : -1});
    }
  }
  e->snap_epoch = e->state_epoch;
  return FW_OK;
}

int fw_snapshot_kg(fw_engine* e, int32_t kg, void* buf, int64_t cap, int64_t* len) {
  if (!e || !len) return FW_ERR_INVALID_ARG;
  if (e->session) return reject(e, FW_ERR_UNSUPPORTED, "session windows: the merging-window set is keyed list state of its own (no checkpoint)");
  if (e->list) return reject(e, FW_ERR_UNSUPPORTED, "list state: buffered elements have no checkpoint layout here");
  if (window_panes_used(e)) return reject(e, FW_ERR_UNSUPPORTED, "sliding windows: records below offset - slide put state in window panes, which no checkpoint layout carries");
  if (!e->disarmed.empty())
    return reject(e, FW_ERR_UNSUPPORTED, "restored windows without trigger timers: only the reference layout (explicit "
                                         "timers, fw_snapshot_kg_flink) carries them");
  if (e->s.gtag && !e->ghost_windows.empty())
    return reject(e, FW_ERR_UNSUPPORTED, "PurgingTrigger with allowed lateness: purged windows within their lateness keep "
                                         "cleanup timers without state, which only the reference layout "
                                         "(fw_snapshot_kg_flink) carries");
  if (e->sticky) return e->sticky;
  if (kg < e->s.kg_start || kg > e->s.kg_end)   // HeapInternalTimerService.restoreTimersForKeyGroup's check
    return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
  if (e->used_key_hash)
    return reject(e, FW_ERR_UNSUPPORTED, "snapshot needs Long keys (a push carried Java key hashes)");
  HIPCHK(e, hipSetDevice(e->dev));
  int rc = build_snapshot(e);
  if (rc) return rc;
  const std::vector<int64_t>& v = e->snap_kg[(size_t)kg];
  const int64_t n = (int64_t)v.size() / FW_SNAP_ENTRY_WORDS;
  *len = 8 * (FW_SNAP_HEADER_WORDS + (int64_t)v.size());
  if (!buf) return FW_OK;
  if (cap < *len) return reject(e, FW_ERR_CAPACITY, "snapshot buffer too small");
  snap_header(e, kg, n, (int64_t*)buf);
  if (!v.empty()) memcpy((int64_t*)buf + FW_SNAP_HEADER_WORDS, v.data(), 8 * v.size());
  return FW_OK;
}

static int restore_entries(fw_engine* e, int64_t wm, const int64_t* ent, int64_t n, int32_t wpane = 0);

int fw_restore_kg(fw_engine* e, int32_t kg, const void* buf, int64_t len) {
  if (!e || !buf) return FW_ERR_INVALID_ARG;
  if (e->session) return reject(e, FW_ERR_UNSUPPORTED, "session windows: the merging-window set is keyed list state of its own (no checkpoint)");
  if (e->list) return reject(e, FW_ERR_UNSUPPORTED, "list state: buffered elements have no checkpoint layout here");
  if (e->sticky) return e->sticky;
  if (e->pushes > 0 || e->records_in > 0) return reject(e, FW_ERR_INVALID_ARG, "restore after the first push");
  if (len < 8 * FW_SNAP_HEADER_WORDS) return reject(e, FW_ERR_INVALID_ARG, "snapshot blob too short");
  const int64_t* h = (const int64_t*)buf;
  int64_t ref[FW_SNAP_HEADER_WORDS];
  snap_header(e, kg, h[3], ref);
  if (h[0] != FW_SNAP_MAGIC || h[1] != 2) return reject(e, FW_ERR_INVALID_ARG, "not a key-group snapshot (magic/version)");
  if (h[2] != kg) return reject(e, FW_ERR_INVALID_ARG, "snapshot holds key group " + std::to_string(h[2]));
  for (int w = 5; w < FW_SNAP_HEADER_WORDS; ++w)
    if (h[w] != ref[w]) return reject(e, FW_ERR_INVALID_ARG, "snapshot of a different window/reduce configuration");
  if (kg < e->s.kg_start || kg > e->s.kg_end)
    return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
  const int64_t n = h[3];
  if (n < 0 || len != 8 * (FW_SNAP_HEADER_WORDS + n * FW_SNAP_ENTRY_WORDS))
    return reject(e, FW_ERR_INVALID_ARG, "snapshot blob length does not match its entry count");
  if (e->restored && h[4] != e->cur_wm)
    return reject(e, FW_ERR_INVALID_ARG, "key groups checkpointed at different watermarks");
  const int64_t* ent = h + FW_SNAP_HEADER_WORDS;
  for (int64_t j = 0; j < n; ++j)
    if (host_key_group(e->s, ent[j * FW_SNAP_ENTRY_WORDS + 1]) != kg)
      return reject(e, FW_ERR_KEY_GROUP, "snapshot entry key outside its key group");
  if (int rc = restore_entries(e, h[4], ent, n)) return rc;
  // PurgingTrigger + allowed lateness: the windows within their lateness at the restored watermark are tracked
  // for their cleanup timers as after any watermark (fw_snapshot_kg took none with such timers pending)
  if (e->s.gtag) return ghost_advance(e, INT64_MIN, e->cur_wm);
  return FW_OK;
}

// load n validated snapshot entries (FW_SNAP_ENTRY_WORDS each) and set the watermark
static int restore_entries(fw_engine* e, int64_t wm, const int64_t* ent, int64_t n, int32_t wpane) {
  HIPCHK(e, hipSetDevice(e->dev));
  e->restored = true;
  e->cur_wm = wm;
  e->state_epoch++;
  if (n == 0) return FW_OK;
  int64_t* d = nullptr;
  HIPCHK(e, hipMalloc(&d, 8 * (size_t)n * FW_SNAP_ENTRY_WORDS));
  hipError_t r = hipMemcpyAsync(d, ent, 8 * (size_t)n * FW_SNAP_ENTRY_WORDS, hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) {
    const int blocks = (int)std::min<int64_t>((n + BLOCK - 1) / BLOCK, 1024);
    hipLaunchKernelGGL(fw::k_restore, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, d, n, wpane);
    r = hipGetLastError();
  }
  const hipError_t r2 = hipStreamSynchronize(e->stream);
  (void)hipFree(d);
  HIPCHK(e, r);
  HIPCHK(e, r2);
  return check_device_error(e);
}

// ------------------------------------------------------------------------------------------------
// checkpoint state in the reference's key-group layout (flink_kg_format.h; flink_window.h)
// ------------------------------------------------------------------------------------------------

// one (window, key) entry of a key group's state table, engine encodings (double bits, min/max codes)
struct KgPane {
  int64_t start, end, key;
  int64_t sum, mn, mx, cnt;
  int64_t first;    // first-arrival ordinal (0 when the config does not track first arrival)
  int64_t f1;
  bool unarmed;     // a restored window's pane whose trigger timer fired before the checkpoint (none pending)
  int64_t m = 0;    // tumbling: the slice (= window) number
};

static int check_state_layout(fw_engine* e, const fw_state_layout* L) {
  if (!L || L->n_fields < 0 || L->n_fields > FW_SF_MAX_FIELDS)
    return reject(e, FW_ERR_INVALID_ARG, "bad state layout");
  int seen[FW_SF_VALUE + 1] = {0};
  for (int i = 0; i < L->n_fields; ++i) {
    const int f = L->field[i];
    if (f < FW_SF_KEY || f > FW_SF_VALUE) return reject(e, FW_ERR_INVALID_ARG, "bad state layout field");
    seen[f]++;
  }
  const fw_config& c = e->cfg;
  const bool by = e->s.by;
  if (e->list) {   // ListSerializer's element: the window's input tuple — its key, f1 and value fields, in order
    if (seen[FW_SF_KEY] > 1 || seen[FW_SF_F1] > 1 || seen[FW_SF_VALUE] != 1 || seen[FW_SF_SUM] || seen[FW_SF_MIN] ||
        seen[FW_SF_MAX] || seen[FW_SF_COUNT])
      return reject(e, FW_ERR_INVALID_ARG, "list state layout: the element tuple's fields, FW_SF_VALUE once and "
                                           "FW_SF_KEY / FW_SF_F1 at most once");
    return FW_OK;
  }
  const int want[FW_SF_VALUE + 1] = {0, -1, c.keep_first_f1 || by ? 1 : 0, !by && (c.agg_mask & FW_AGG_SUM) ? 1 : 0,
                                     !by && (c.agg_mask & FW_AGG_MIN) ? 1 : 0, !by && (c.agg_mask & FW_AGG_MAX) ? 1 : 0,
                                     !by && (c.agg_mask & FW_AGG_COUNT) ? 1 : 0, by ? 1 : 0};
  if (seen[FW_SF_KEY] > 1) return reject(e, FW_ERR_INVALID_ARG, "state layout names the key twice");
  for (int f = FW_SF_F1; f <= FW_SF_VALUE; ++f)
    if (seen[f] != want[f])
      return reject(e, FW_ERR_INVALID_ARG, "state layout must name each computed aggregate (and f1 iff "
                                           "keep_first_f1) exactly once");
  return FW_OK;
}

static int64_t host_window_start(const fw_config& c, int64_t n) {
  return fw::jadd(c.offset, (int64_t)((uint64_t)n * (uint64_t)(c.assigner == FW_TUMBLING ? c.size : c.slide)));
}

// HeapFoldingState holds the accumulator: the fold's initial value folded with the pane (as emit_record
// applies it), and back (sum and count subtract it: exact for Long, to the last bit for doubles only when
// the initial value is 0; min and max hold it already: the accumulator is at or beyond it)
static KgPane fold_pane(const fw_engine* e, KgPane p) {
  const fw::Spec& s = e->s;
  const int64_t x = s.fold_init;
  if (s.vt == FW_VALUE_I64) p.sum = fw::jadd(x, p.sum);
  else { double a, b; memcpy(&a, &x, 8); memcpy(&b, &p.sum, 8); b = a + b; memcpy(&p.sum, &b, 8); }
  p.mn = std::min(p.mn, fw::min_code(s.vt, s.cmpto, x));
  p.mx = std::max(p.mx, fw::max_code(s.vt, s.cmpto, x));
  p.cnt = fw::jadd(x, p.cnt);
  return p;
}
static KgPane unfold_pane(const fw_engine* e, KgPane p) {
  const fw::Spec& s = e->s;
  const int64_t x = s.fold_init;
  if (s.vt == FW_VALUE_I64) p.sum = fw::jsub(p.sum, x);
  else { double a, b; memcpy(&a, &x, 8); memcpy(&b, &p.sum, 8); b = b - a; memcpy(&p.sum, &b, 8); }
  p.cnt = fw::jsub(p.cnt, x);
  return p;
}

// the pane value of field f, written as the field's Java type
static void put_field(const fw_engine* e, fwkg::BeOut& o, int f, const KgPane& p_in) {
  const KgPane p = e->s.fold ? fold_pane(e, p_in) : p_in;
  const bool f64 = e->s.vt == FW_VALUE_F64;
  auto val = [&](int64_t bits) { if (f64) { double d; memcpy(&d, &bits, 8); o.f64(d); } else o.i64(bits); };
  auto code = [&](int64_t c) { if (f64) o.f64(fw::f64_from_code(c)); else o.i64(c); };
  switch (f) {
    case FW_SF_KEY: o.i64(p.key); break;
    case FW_SF_F1: o.i64(p.f1); break;
    case FW_SF_SUM: val(p.sum); break;
    case FW_SF_MIN: code(p.mn); break;
    case FW_SF_MAX: code(p.mx); break;
    case FW_SF_COUNT: o.i64(p.cnt); break;
    case FW_SF_VALUE: code(e->cfg.agg_mask == FW_AGG_MAXBY ? p.mx : p.mn); break;
  }
}

// The panes of key group kg as the reference holds them: one per (window, key).  Tumbling: a slice is a
// window.  Sliding: every window still in its lifetime (cleanup time > watermark) that a slice of the key
// overlaps, combined from its slices in slice order (double sums: the slice-sum order, not arrival order)
static void kg_panes(const fw_engine* e, int32_t kg, std::vector<KgPane>& out) {
  const fw_config& c = e->cfg;
  const fw::Spec& s = e->s;
  const std::vector<int64_t>& v = e->snap_kg[(size_t)kg];
  const size_t n = v.size() / FW_SNAP_ENTRY_WORDS;
  const bool tumbling = c.assigner == FW_TUMBLING;
  auto pane_of = [&](const int64_t* x, int64_t start) {
    KgPane p;
    p.start = start;
    p.end = fw::jadd(start, c.size);
    p.key = x[1];
    p.sum = x[2]; p.mn = x[3]; p.mx = x[4];
    p.cnt = x[5];               // maxBy/minBy: the extremal record's ordinal
    p.first = s.first ? x[6] : 0;
    p.f1 = x[7];
    p.unarmed = e->snap_unarmed.count({x[0], x[1]}) != 0 && tumbling;
    p.m = x[0];
    return p;
  };
  out.clear();
  if (tumbling) {
    for (size_t j = 0; j < n; ++j) {
      const int64_t* x = &v[j * FW_SNAP_ENTRY_WORDS];
      KgPane p = pane_of(x, host_window_start(c, x[0]));
      if (fw::cleanup_time(fw::jsub(p.end, 1), c.allowed_lateness) > e->cur_wm) out.push_back(p);
    }
    return;
  }
  std::vector<size_t> ord(n);
  for (size_t j = 0; j < n; ++j) ord[j] = j;
  std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
    const int64_t* x = &v[a * FW_SNAP_ENTRY_WORDS];
    const int64_t* y = &v[b * FW_SNAP_ENTRY_WORDS];
    return x[1] != y[1] ? x[1] < y[1] : x[0] < y[0];
  });
  std::map<std::pair<int64_t, int64_t>, KgPane> win;   // (window number, key)
  const bool f64 = s.vt == FW_VALUE_F64;
  // the windows' own panes first (restored window state: the earlier arrivals), then each slice into every
  // window it makes up
  const std::vector<int64_t>& wv = e->snap_wkg[(size_t)kg];
  std::vector<std::pair<int64_t, const int64_t*>> items;   // (window number or -1 for a slice, entry)
  for (size_t j = 0; j < wv.size() / FW_SNAP_ENTRY_WORDS; ++j) items.push_back({1, &wv[j * FW_SNAP_ENTRY_WORDS]});
  for (size_t j : ord) items.push_back({0, &v[j * FW_SNAP_ENTRY_WORDS]});
  for (const auto& item : items) {
    const int64_t* x = item.second;
    const int64_t m = x[0];
    const int64_t w_lo = item.first ? m : fw::floor_div(m - s.K, s.R) + 1, w_hi = item.first ? m : fw::floor_div(m, s.R);
    for (int64_t w = w_lo; w <= w_hi; ++w) {
      const int64_t start = host_window_start(c, w);
      if (fw::cleanup_time(fw::jsub(fw::jadd(start, c.size), 1), c.allowed_lateness) <= e->cur_wm) continue;
      KgPane b = pane_of(x, start);
      auto it = win.find({w, b.key});
      if (it == win.end()) { win.emplace(std::make_pair(w, b.key), b); continue; }
      KgPane& a = it->second;
      if (s.by) {   // the extremal record; a tie keeps the earlier one (maxBy/minBy(first = false): the later)
        const bool maxby = c.agg_mask == FW_AGG_MAXBY;
        const int64_t ca = maxby ? a.mx : a.mn, cb = maxby ? b.mx : b.mn;
        const bool better = maxby ? cb > ca : cb < ca;
        const bool tie_later = (c.agg_flags & FW_AGGF_BY_LAST) != 0;
        if (better || (cb == ca && (tie_later ? b.cnt > a.cnt : b.cnt < a.cnt))) {
          a.mx = b.mx; a.mn = b.mn; a.cnt = b.cnt; a.f1 = b.f1;
        }
        a.first = std::min(a.first, b.first);
        continue;
      }
      if (f64) {
        double da, db;
        memcpy(&da, &a.sum, 8); memcpy(&db, &b.sum, 8);
        da += db;
        memcpy(&a.sum, &da, 8);
      } else {
        a.sum = fw::jadd(a.sum, b.sum);
      }
      a.mn = std::min(a.mn, b.mn);
      a.mx = std::max(a.mx, b.mx);
      a.cnt = fw::jadd(a.cnt, b.cnt);
      if (s.first && b.first < a.first) { a.first = b.first; a.f1 = b.f1; }
    }
  }
  for (auto& kv : win) {   // (sliding: a window restored disarmed and not re-armed for the key)
    kv.second.unarmed = e->snap_unarmed.count({kv.first.first, kv.first.second}) != 0;
    if (!e->list_entry_rank.empty()) {   // a restored list entry keeps its place in the namespace's insertion order
      auto it = e->list_entry_rank.find({kv.second.start, kv.second.key});
      if (it != e->list_entry_rank.end()) kv.second.first = it->second - e->ordinal;
    }
    out.push_back(kv.second);
  }
}


// ------------------------------------------------------------------------------------------------
// session windows in the reference's key-group layout: WindowOperator keeps two keyed states for a merging
// assigner (WindowOperator.java:445-460, 724-736) — "window-contents" (the reducing state, namespace = each
// in-flight window's STATE window) and "merging-window-set" (ListState<Tuple2<W, W>> in VoidNamespace: per
// key its in-flight windows and their state windows, MergingWindowSet.persist, MergingWindowSet.java:91-95).
// stateTables iterates "window-contents" (HashMap bucket 12 of 16) before "merging-window-set" (bucket 15): ids
// 0 and 1.  Engine side: k_sess_walk / k_sess_walk_hot / k_sess_wm keep per slot the state window and the
// arrival ordinals that place each entry in its HashMap's insertion order (SessDev).
// ------------------------------------------------------------------------------------------------
namespace fw {
// restored sessions: one row per in-flight window (key, slot, start, end, state-window start, its entry's rank,
// trigger pending, sum, min / max codes, count, f1); key ids by the directory's insert
constexpr int SESS_ROW = 15;
__global__ __launch_bounds__(BLOCK) void k_sess_restore(Spec s, SessDev d, const int64_t* rows, int64_t n, int64_t put0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* r = rows + i * SESS_ROW;
  const int64_t kid = dir_find_or_insert(s, r[0]);
  if (kid < 0) { cap_error(s, 20); return; }
  const int q = (int)r[1];
  const int64_t x = kid * d.sw + q;
  d.start[x] = r[2];
  d.end[x] = r[3];
  d.sws[x] = r[4];
  d.swc[x] = r[5];
  d.put[x] = put0 + q;             // MergingWindowSet(assigner, state): puts in list order
  d.cre[x] = d.tre[x] = put0;      // (restored timers are ordered by their blob rank)
  if (d.sum) d.sum[x] = r[7];
  if (d.mn) d.mn[x] = r[8];
  if (d.mx) d.mx[x] = r[9];
  if (d.cnt) d.cnt[x] = r[10];
  if (d.f1) d.f1[x] = r[11];
  if (d.list) {   // list state: the window's elements, chained in pool entries the host laid out
    d.head[x] = r[12];
    d.tail[x] = r[13];
    d.len[x] = r[14];
  }
  sess_ns_add(d, record_key_group(s, long_hash_code(r[0])), r[4]);
  atomicOr(&d.live[kid * d.nw + (q >> 6)], 1ull << (q & 63));
  if (r[6]) atomicOr(&d.trig[kid * d.nw + (q >> 6)], 1ull << (q & 63));
}
}  // namespace fw

static int session_download(fw_engine* e) {
  fw_engine::SessHost& h = e->sess_host;
  if (h.epoch == e->state_epoch && h.wm == e->cur_wm) return FW_OK;
  const fw::Spec& s = e->s;
  const SessDev& d = e->sess;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (int rc = check_device_error(e)) return rc;
  const size_t cells = (size_t)d.sw * (size_t)s.stride, rows = (size_t)s.stride;
  auto get = [&](std::vector<int64_t>& v, const int64_t* p, size_t n) -> hipError_t {
    v.assign(p ? n : 0, 0);
    return p ? hipMemcpy(v.data(), p, 8 * n, hipMemcpyDeviceToHost) : hipSuccess;
  };
  HIPCHK(e, get(h.keys, s.dir_keys, (size_t)s.D));
  HIPCHK(e, get(h.st, d.start, cells));
  HIPCHK(e, get(h.en, d.end, cells));
  HIPCHK(e, get(h.sws, d.sws, cells));
  HIPCHK(e, get(h.swc, d.swc, cells));
  HIPCHK(e, get(h.put, d.put, cells));
  HIPCHK(e, get(h.cre, d.cre, cells));
  HIPCHK(e, get(h.tre, d.tre, cells));
  HIPCHK(e, get(h.sum, d.sum, cells));
  HIPCHK(e, get(h.mn, d.mn, cells));
  HIPCHK(e, get(h.mx, d.mx, cells));
  HIPCHK(e, get(h.cnt, d.cnt, cells));
  HIPCHK(e, get(h.f1, d.f1, cells));
  HIPCHK(e, get(h.ktouch, d.ktouch, rows));
  HIPCHK(e, get(h.lhead, d.list ? d.head : nullptr, cells));
  HIPCHK(e, get(h.llen, d.list ? d.len : nullptr, cells));
  HIPCHK(e, get(h.pv, d.list ? d.pv : nullptr, (size_t)d.pcap));
  HIPCHK(e, get(h.pf1, d.list ? d.pf1 : nullptr, (size_t)d.pcap));
  HIPCHK(e, get(h.pnext, d.list ? d.pnext : nullptr, (size_t)d.pcap));
  HIPCHK(e, get(h.ktts, d.ktts, rows));
  h.kacc.assign(rows, 0);
  HIPCHK(e, hipMemcpy(h.kacc.data(), d.kacc, 4 * rows, hipMemcpyDeviceToHost));
  unsigned long long nl = 0;
  HIPCHK(e, hipMemcpy(&nl, d.nslog_n, 8, hipMemcpyDeviceToHost));
  h.nslog_over = (int64_t)nl > d.nslog_cap;
  HIPCHK(e, get(h.nslog, d.nslog, 4 * (size_t)std::min<int64_t>((int64_t)nl, d.nslog_cap)));
  h.live.assign(rows * (size_t)d.nw, 0);
  h.trig.assign(rows * (size_t)d.nw, 0);
  HIPCHK(e, hipMemcpy(h.live.data(), d.live, 8 * h.live.size(), hipMemcpyDeviceToHost));
  HIPCHK(e, hipMemcpy(h.trig.data(), d.trig, 8 * h.trig.size(), hipMemcpyDeviceToHost));
  h.epoch = e->state_epoch;
  h.wm = e->cur_wm;
  return FW_OK;
}

static int session_reject_config(fw_engine* e) {
  const fw_config& c = e->cfg;
  (void)c;
  if (!e->sess.ckpt)
    return reject(e, FW_ERR_UNSUPPORTED, "session checkpoint bookkeeping is off (FW_SESS_CKPT=0)");
  if (e->mws_created.empty()) e->mws_created.assign((size_t)(e->s.kg_end - e->s.kg_start + 1), 0);
  if (e->kg_touched.empty()) e->kg_touched.assign((size_t)(e->s.kg_end - e->s.kg_start + 1), 0);
  return FW_OK;
}

static int session_snapshot_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, void* state,
                                     int64_t state_cap, int64_t* state_len, void* timers, int64_t timers_cap,
                                     int64_t* timers_len) {
  if (int rc = session_reject_config(e)) return rc;
  HIPCHK(e, hipSetDevice(e->dev));
  if (int rc = session_download(e)) return rc;
  const fw_engine::SessHost& h = e->sess_host;
  const fw::Spec& s = e->s;
  const SessDev& d = e->sess;
  const fw_config& c = e->cfg;
  const size_t kgi = (size_t)(kg - s.kg_start);
  const bool orphans = c.trigger == FW_TRIGGER_PURGING_EVENT_TIME && c.allowed_lateness > 0;
  if (orphans) {   // purged sessions' cleanup timers logged since the last snapshot
    unsigned long long no = 0;
    HIPCHK(e, hipMemcpy(&no, d.olog_n, 8, hipMemcpyDeviceToHost));
    if ((int64_t)no > d.olog_cap)
      return reject(e, FW_ERR_CAPACITY, "more purged sessions since the last snapshot than the orphan timer log holds");
    std::vector<int64_t> ol(4 * (size_t)no);
    if (no) HIPCHK(e, hipMemcpy(ol.data(), d.olog, 8 * ol.size(), hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemset(d.olog_n, 0, 8));
    for (size_t j = 0; j < (size_t)no; ++j) e->sess_orphans.push_back({ol[4 * j], ol[4 * j + 1], ol[4 * j + 2], ol[4 * j + 3]});
    auto ct_of = [&](int64_t end) { return fw::cleanup_time(fw::jsub(end, 1), c.allowed_lateness); };
    std::vector<std::array<int64_t, 4>> keep;
    for (const auto& o : e->sess_orphans) if (ct_of(o[2]) > e->cur_wm) keep.push_back(o);
    e->sess_orphans.swap(keep);
    // a restored timer that fired fetched its key's set (onEventTime -> getMergingWindowSet)
    for (auto it = e->sess_rorphans.begin(); it != e->sess_rorphans.end();) {
      const int64_t ct = ct_of((*it)[2]);
      if (ct > e->cur_wm) { ++it; continue; }
      int64_t ord = 0;
      for (const auto& a : e->sess_adv) if (a.first >= ct) { ord = a.second; break; }
      auto adj = e->sess_touch_adj.find((*it)[0]);
      if (adj == e->sess_touch_adj.end() || std::make_pair(ord, ct) < adj->second) e->sess_touch_adj[(*it)[0]] = {ord, ct};
      it = e->sess_rorphans.erase(it);
    }
  }
  struct Pane { int64_t kid, key, start, end, sws, swc, put, cre, tre; bool trig; KgPane acc; int64_t lhead, llen; };
  std::vector<Pane> panes;
  std::vector<int64_t> kids;   // the key group's keys
  int64_t n_touched = 0;
  bool any_acc = false, kg_acc = false;
  // when a key's set was first fetched: the device's record or watermark, or a restored timer's firing (host)
  auto touch_of = [&](int64_t kid, int64_t key) -> std::pair<int64_t, int64_t> {
    std::pair<int64_t, int64_t> t{h.ktouch[(size_t)kid], h.ktts[(size_t)kid]};
    auto adj = e->sess_touch_adj.find(key);
    if (adj != e->sess_touch_adj.end() && (t.first < 0 || adj->second < t)) t = adj->second;
    return t;
  };
  std::set<int64_t> dir_keys_touched;
  for (int64_t k = 0; k < s.stride; ++k) {
    const int64_t key = k == s.D ? fw::EMPTY_KEY : h.keys[(size_t)k];
    if (k < s.D && key == fw::EMPTY_KEY) continue;
    if (touch_of(k, key).first >= 0) { ++n_touched; dir_keys_touched.insert(key); }
    any_acc = any_acc || h.kacc[(size_t)k];
    if (host_key_group(s, key) != kg) continue;
    kids.push_back(k);
    kg_acc = kg_acc || h.kacc[(size_t)k];
    for (int q = 0; q < d.sw; ++q) {
      const size_t w = (size_t)k * (size_t)d.nw + (size_t)(q >> 6);
      if (!((h.live[w] >> (q & 63)) & 1ull)) continue;
      const size_t x = (size_t)k * (size_t)d.sw + (size_t)q;
      Pane p{k, key, h.st[x], h.en[x], h.sws[x], h.swc[x], h.put[x], h.cre[x], h.tre[x], ((h.trig[w] >> (q & 63)) & 1ull) != 0, {},
             h.lhead.empty() ? -1 : h.lhead[x], h.llen.empty() ? 0 : h.llen[x]};
      p.acc = KgPane{p.sws, fw::jadd(p.sws, d.gap), key, h.sum.empty() ? 0 : h.sum[x], h.mn.empty() ? INT64_MAX : h.mn[x],
                     h.mx.empty() ? INT64_MIN : h.mx[x], h.cnt.empty() ? 0 : h.cnt[x], 0, h.f1.empty() ? 0 : h.f1[x], false};
      panes.push_back(p);
    }
  }
  for (const auto& a : e->sess_touch_adj) if (!dir_keys_touched.count(a.first)) ++n_touched;   // (keys not in the directory)
  const bool wc_table = e->sess_wc_table || any_acc;
  const bool mws_table = e->sess_mws_table || n_touched > 0;
  fwkg::BeOut st, tm;
  if (wc_table || mws_table) st.i32(kg);
  int id = 0;
  if (wc_table) {   // "window-contents": namespaces = state windows, created by their first record
    const bool present = kg_acc || e->kg_touched[kgi];
    st.i16(id++);
    st.u8(present ? 1 : 0);
    if (present) {
      std::map<int64_t, std::vector<size_t>> ns;
      for (size_t i = 0; i < panes.size(); ++i) ns[panes[i].sws].push_back(i);
      std::vector<std::pair<int64_t, std::vector<size_t>>> nsv(ns.begin(), ns.end());
      // when each namespace's current instance was put into the namespace map: its entries' lifetimes — the live
      // ones and the logged entries of other keys removed while it stayed shared — chained without a gap
      std::map<int64_t, std::vector<std::pair<int64_t, int64_t>>> life;
      for (size_t j = 0; j + 4 <= h.nslog.size(); j += 4)
        if (ns.count(h.nslog[j + 1]) && host_key_group(s, h.nslog[j]) == kg) life[h.nslog[j + 1]].push_back({h.nslog[j + 2], h.nslog[j + 3]});
      std::vector<int64_t> ns_first(nsv.size(), INT64_MAX);
      for (size_t w = 0; w < nsv.size(); ++w) {
        auto& iv = life[nsv[w].first];
        for (size_t i : nsv[w].second) iv.push_back({panes[i].swc, INT64_MAX});
        std::sort(iv.begin(), iv.end());
        int64_t from = iv[0].first, reach = iv[0].second;
        for (const auto& x : iv) {
          if (x.first >= reach) from = x.first;   // a gap: the namespace was removed and put again
          reach = x.first >= reach ? x.second : std::max(reach, x.second);
        }
        ns_first[w] = from;
      }
      std::vector<size_t> wo(nsv.size());
      for (size_t w = 0; w < wo.size(); ++w) wo[w] = w;
      fwkg::hashmap_order(
          wo, [&](size_t w) { return fwkg::window_hash(nsv[w].first, fw::jadd(nsv[w].first, d.gap)); },
          [&](size_t a, size_t b) { return ns_first[a] != ns_first[b] ? ns_first[a] < ns_first[b] : nsv[a].first < nsv[b].first; });
      st.i32((int32_t)nsv.size());
      for (size_t w : wo) {
        st.i64(nsv[w].first);
        st.i64(fw::jadd(nsv[w].first, d.gap));
        std::vector<size_t>& ent = nsv[w].second;
        fwkg::hashmap_order(
            ent, [&](size_t i) { return fw::long_hash_code(panes[i].key); },
            [&](size_t a, size_t b) { return panes[a].swc != panes[b].swc ? panes[a].swc < panes[b].swc : panes[a].key < panes[b].key; });
        st.i32((int32_t)ent.size());
        for (size_t i : ent) {
          st.i64(panes[i].key);
          if (d.list) {   // ListSerializer: int size, then the window's elements in list order
            st.i32((int32_t)panes[i].llen);
            int64_t el = panes[i].lhead;
            for (int64_t j = 0; j < panes[i].llen && el >= 0 && el < d.pcap; ++j, el = h.pnext[(size_t)el])
              for (int f = 0; f < layout->n_fields; ++f) {
                const int fld = layout->field[f];
                if (fld == FW_SF_KEY) st.i64(panes[i].key);
                else if (fld == FW_SF_F1) st.i64(h.pf1[(size_t)el]);
                else if (s.vt == FW_VALUE_F64) { double dv; memcpy(&dv, &h.pv[(size_t)el], 8); st.f64(dv); }
                else st.i64(h.pv[(size_t)el]);
              }
            continue;
          }
          for (int f = 0; f < layout->n_fields; ++f) put_field(e, st, layout->field[f], panes[i].acc);
        }
      }
    }
  }
  if (mws_table) {   // "merging-window-set", as WindowOperator.snapshotState rewrites it
    // entries: the restored ones of keys not touched since (inserted at the restore, in blob order), then every
    // other key with sessions in flight, re-added in mergingWindowsByKey's order (HashMap<K, MergingWindowSet>
    // over every key fetched since the operator opened: bucket, then first fetch)
    struct Ent { int64_t kid, key, rank; bool touched; std::vector<size_t> slots; };
    std::vector<Ent> ents;
    std::map<int64_t, size_t> at;
    for (size_t i = 0; i < panes.size(); ++i) {
      auto it = at.find(panes[i].kid);
      if (it == at.end()) {
        const int64_t k = panes[i].kid;
        auto r = e->sess_mws_rank.find(panes[i].key);
        const bool touched = touch_of(k, panes[i].key).first >= 0 || r == e->sess_mws_rank.end();
        it = at.emplace(k, ents.size()).first;
        ents.push_back({k, panes[i].key, touched ? INT64_MAX : r->second, touched, {}});
      }
      ents[it->second].slots.push_back(i);
    }
    if (!ents.empty()) e->mws_created[kgi] = 1;
    const bool present = e->mws_created[kgi] != 0;
    st.i16(id++);
    st.u8(present ? 1 : 0);
    if (present) {
      st.i32(ents.empty() ? 0 : 1);
      if (!ents.empty()) {
        st.u8(0);   // VoidNamespaceSerializer: one byte
        const uint32_t gmask = fwkg::capacity_for((size_t)n_touched) - 1;
        std::vector<size_t> eo(ents.size());
        for (size_t i = 0; i < eo.size(); ++i) eo[i] = i;
        fwkg::hashmap_order(
            eo, [&](size_t i) { return fw::long_hash_code(ents[i].key); },
            [&](size_t a, size_t b) {
              const Ent &x = ents[a], &y = ents[b];
              if (x.touched != y.touched) return !x.touched;
              if (!x.touched) return x.rank < y.rank;
              const uint32_t gx = (uint32_t)fwkg::spread(fw::long_hash_code(x.key)) & gmask;
              const uint32_t gy = (uint32_t)fwkg::spread(fw::long_hash_code(y.key)) & gmask;
              if (gx != gy) return gx < gy;
              const auto tx = touch_of(x.kid, x.key), ty = touch_of(y.kid, y.key);
              return tx != ty ? tx < ty : x.key < y.key;
            });
        st.i32((int32_t)ents.size());
        for (size_t i : eo) {
          std::vector<size_t>& sl = ents[i].slots;   // MergingWindowSet.windows (HashMap<W, W>): bucket, then put order
          fwkg::hashmap_order(
              sl, [&](size_t j) { return fwkg::window_hash(panes[j].start, panes[j].end); },
              [&](size_t a, size_t b) { return panes[a].put < panes[b].put; });
          st.i64(ents[i].key);
          st.i32((int32_t)sl.size());
          for (size_t j : sl) {
            st.i64(panes[j].start);
            st.i64(panes[j].end);
            st.i64(panes[j].sws);
            st.i64(fw::jadd(panes[j].sws, d.gap));
          }
        }
      }
    }
  }
  // timers: per in-flight window its trigger timer while pending (registered by onElement / onMerge) and its
  // cleanup timer (registerCleanupTimer right after; one timer when the lateness is 0); restored ones keep their
  // blob order ahead of every later one
  struct Tm { int64_t key, start, end, ts, seq; int kind; int64_t rank; };
  std::vector<Tm> tv;
  for (const Pane& p : panes) {
    const int64_t max_ts = fw::jsub(p.end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
    if (p.trig) tv.push_back({p.key, p.start, p.end, max_ts, p.tre, 0, INT64_MAX});
    if (ct != max_ts) tv.push_back({p.key, p.start, p.end, ct, p.cre, 1, INT64_MAX});
  }
  if (orphans) {   // purged sessions' cleanup timers (the same timer as a later in-flight window's keeps its place)
    std::map<std::array<int64_t, 3>, size_t> at;
    for (size_t i = 0; i < tv.size(); ++i) if (tv[i].kind == 1) at[{tv[i].key, tv[i].start, tv[i].end}] = i;
    auto add = [&](int64_t key, int64_t start, int64_t end, int64_t seq) {
      if (host_key_group(s, key) != kg) return;
      auto it = at.find({key, start, end});
      if (it != at.end()) { tv[it->second].seq = std::min(tv[it->second].seq, seq); return; }
      at[{key, start, end}] = tv.size();
      tv.push_back({key, start, end, fw::cleanup_time(fw::jsub(end, 1), c.allowed_lateness), seq, 1, INT64_MAX});
    };
    for (const auto& o : e->sess_rorphans) add(o[0], o[1], o[2], INT64_MIN);
    for (const auto& o : e->sess_orphans) add(o[0], o[1], o[2], o[3]);
  }
  if (!e->restored_timer_rank.empty())
    for (Tm& t : tv) {
      auto it = e->restored_timer_rank.find({t.key, t.start, t.end, t.ts});
      if (it != e->restored_timer_rank.end()) t.rank = it->second;
    }
  std::vector<size_t> to(tv.size());
  for (size_t i = 0; i < to.size(); ++i) to[i] = i;
  fwkg::hashmap_order(
      to, [&](size_t i) { return fwkg::timer_hash(tv[i].ts, tv[i].key, tv[i].start, tv[i].end); },
      [&](size_t a, size_t b) {
        const Tm &x = tv[a], &y = tv[b];
        if (x.rank != y.rank) return x.rank < y.rank;
        if (x.seq != y.seq) return x.seq < y.seq;
        return x.kind < y.kind;
      });
  tm.i32((int32_t)tv.size());
  for (size_t i : to) {
    tm.i64(tv[i].key);
    tm.i64(tv[i].start);
    tm.i64(tv[i].end);
    tm.i64(tv[i].ts);
  }
  tm.i32(0);
  *state_len = (int64_t)st.b.size();
  *timers_len = (int64_t)tm.b.size();
  if (!state && !timers) return FW_OK;
  if (!state || !timers || state_cap < *state_len || timers_cap < *timers_len)
    return reject(e, FW_ERR_CAPACITY, "snapshot buffer too small");
  if (!st.b.empty()) memcpy(state, st.b.data(), st.b.size());
  memcpy(timers, tm.b.data(), tm.b.size());
  return FW_OK;
}

static int session_restore_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, int64_t watermark,
                                    const void* state, int64_t state_len, const void* timers, int64_t timers_len) {
  if (int rc = session_reject_config(e)) return rc;
  const fw::Spec& s = e->s;
  const SessDev& d = e->sess;
  const fw_config& c = e->cfg;
  const bool f64 = s.vt == FW_VALUE_F64;
  const size_t kgi = (size_t)(kg - s.kg_start);
  struct WcEnt { KgPane p; int64_t rank; std::vector<std::array<int64_t, 2>> el; };   // (list state: value, f1)
  std::map<std::pair<int64_t, int64_t>, WcEnt> wc;   // (state-window start, key) -> its state
  std::vector<std::pair<int64_t, std::vector<std::array<int64_t, 4>>>> mws;
  bool wc_seen = false, mws_seen = false, wc_present = false, mws_present = false;
  if (state_len > 0) {
    fwkg::BeIn in(state, state_len);
    if (in.i32() != kg) return reject(e, FW_ERR_INVALID_ARG, "state section of another key group");
    for (int table = 0; in.ok && (table == 0 || in.pos < in.n); ++table) {   // (at least one table)
      if (in.i16() != table || table > 1) return reject(e, FW_ERR_UNSUPPORTED, "keyed state other than window-contents and merging-window-set");
      const bool present = in.u8() != 0;
      if (table == 0) {
        wc_seen = true;
        wc_present = present;
        const int32_t nns = present ? in.i32() : 0;
        if (nns < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt state section");
        for (int32_t w = 0; w < nns && in.ok; ++w) {
          const int64_t start = in.i64(), end = in.i64();
          if (in.ok && end != fw::jadd(start, d.gap))
            return reject(e, FW_ERR_INVALID_ARG, "namespace is not a state window [ts, ts + gap) of this assigner");
          const int32_t ne = in.i32();
          if (ne < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt state section");
          for (int32_t j = 0; j < ne && in.ok; ++j) {
            KgPane p{start, end, in.i64(), 0, INT64_MAX, INT64_MIN, 0, 0, 0, false};
            std::vector<std::array<int64_t, 2>> el;
            if (e->list) {   // ListSerializer: int size, then the elements (the layout's fields of the input tuple)
              const int32_t nel = in.i32();
              if (nel <= 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt or empty list state entry");
              for (int32_t q = 0; q < nel && in.ok; ++q) {
                std::array<int64_t, 2> x{0, 0};
                for (int f = 0; f < layout->n_fields; ++f) {
                  const int64_t v = in.i64();
                  if (layout->field[f] == FW_SF_KEY && in.ok && v != p.key)
                    return reject(e, FW_ERR_UNSUPPORTED, "element key field differs from the key");
                  if (layout->field[f] == FW_SF_F1) x[1] = v;
                  if (layout->field[f] == FW_SF_VALUE) x[0] = v;
                }
                el.push_back(x);
              }
            }
            for (int f = 0; f < layout->n_fields && !e->list; ++f) {
              const int64_t x = in.i64();
              double dv;
              memcpy(&dv, &x, 8);
              switch (layout->field[f]) {
                case FW_SF_KEY:
                  if (in.ok && x != p.key) return reject(e, FW_ERR_UNSUPPORTED, "state key field differs from the key");
                  break;
                case FW_SF_F1: p.f1 = x; break;
                case FW_SF_SUM: p.sum = x; break;
                case FW_SF_MIN: p.mn = f64 ? (s.cmpto ? fw::f64_cmp_code(dv) : fw::f64_min_code(dv)) : x; break;
                case FW_SF_MAX: p.mx = f64 ? (s.cmpto ? fw::f64_cmp_code(dv) : fw::f64_max_code(dv)) : x; break;
                case FW_SF_COUNT: p.cnt = x; break;
                case FW_SF_VALUE: p.mn = p.mx = f64 ? fw::f64_cmp_code(dv) : x; break;
              }
            }
            if (!in.ok) break;
            if (host_key_group(s, p.key) != kg) return reject(e, FW_ERR_KEY_GROUP, "state entry key outside its key group");
            if (!wc.emplace(std::make_pair(start, p.key), WcEnt{p, e->restore_ord++, std::move(el)}).second)
              return reject(e, FW_ERR_INVALID_ARG, "duplicate (window, key) entry");
          }
        }
      } else {
        mws_seen = true;
        mws_present = present;
        const int32_t nns = present ? in.i32() : 0;
        if (nns < 0 || nns > 1) return reject(e, FW_ERR_INVALID_ARG, "corrupt merging-window-set section");
        if (nns == 1 && in.u8() != 0) return reject(e, FW_ERR_INVALID_ARG, "merging-window-set namespace is not VoidNamespace");
        const int32_t ne = nns ? in.i32() : 0;
        if (ne < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt merging-window-set section");
        for (int32_t j = 0; j < ne && in.ok; ++j) {
          const int64_t key = in.i64();
          const int32_t m = in.i32();
          if (m < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt merging-window-set entry");
          if (m > d.sw) return reject(e, FW_ERR_CAPACITY, "more in-flight sessions for a key than max_open_slices");
          std::vector<std::array<int64_t, 4>> l;
          for (int32_t q = 0; q < m && in.ok; ++q) l.push_back({in.i64(), in.i64(), in.i64(), in.i64()});
          if (!in.ok) break;
          if (host_key_group(s, key) != kg) return reject(e, FW_ERR_KEY_GROUP, "merging-window-set key outside its key group");
          mws.push_back({key, std::move(l)});
        }
      }
    }
    if (!in.done()) return reject(e, FW_ERR_INVALID_ARG, "state section truncated or with trailing bytes");
  }
  std::vector<std::array<int64_t, 4>> got;
  {
    fwkg::BeIn in(timers, timers_len);
    const int32_t nt = in.i32();
    if (nt < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt timer section");
    for (int32_t i = 0; i < nt && in.ok; ++i) {
      const int64_t key = in.i64(), start = in.i64(), end = in.i64(), ts = in.i64();
      got.push_back({key, start, end, ts});
    }
    const int32_t np = in.i32();
    if (!in.done()) return reject(e, FW_ERR_INVALID_ARG, "timer section truncated or with trailing bytes");
    if (np != 0) return reject(e, FW_ERR_UNSUPPORTED, "processing-time timers");
  }
  // the in-flight windows: each with its state window's contents; timers exactly the ones they imply
  std::set<std::array<int64_t, 4>> tset(got.begin(), got.end()), want;
  std::vector<int64_t> rows;
  std::vector<std::array<int64_t, 4>> pool;   // list state: (entry, value, f1, next)
  std::set<std::pair<int64_t, int64_t>> used, keys_seen;
  for (const auto& kv : mws) {
    if (!keys_seen.insert({kv.first, 0}).second) return reject(e, FW_ERR_INVALID_ARG, "duplicate merging-window-set key");
    for (size_t q = 0; q < kv.second.size(); ++q) {
      const auto& w = kv.second[q];   // window start, end, state window start, end
      if (w[3] != fw::jadd(w[2], d.gap) || w[0] > w[2] || w[1] < w[3])
        return reject(e, FW_ERR_INVALID_ARG, "a state window is not a session's first window inside the window");
      auto it = wc.find({w[2], kv.first});
      if (it == wc.end()) return reject(e, FW_ERR_INVALID_ARG, "in-flight session without window-contents state");
      used.insert({w[2], kv.first});
      const int64_t max_ts = fw::jsub(w[1], 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
      const std::array<int64_t, 4> trig_t{kv.first, w[0], w[1], max_ts};
      const bool trig = tset.count(trig_t) != 0;
      if (trig) want.insert(trig_t);
      if (ct != max_ts) want.insert({kv.first, w[0], w[1], ct});
      const KgPane& p = it->second.p;
      int64_t lh = -1, lt = -1, ln = 0;
      if (e->list) {   // the elements into pool entries, chained in list order
        const auto& el = it->second.el;
        if (e->sess_pool_used + (int64_t)el.size() > d.pcap)
          return reject(e, FW_ERR_CAPACITY, "restored session elements exceed list_capacity");
        lh = e->sess_pool_used;
        for (size_t j = 0; j < el.size(); ++j) {
          const int64_t at = e->sess_pool_used++;
          pool.push_back({at, el[j][0], el[j][1], j + 1 < el.size() ? at + 1 : -1});
        }
        lt = e->sess_pool_used - 1;
        ln = (int64_t)el.size();
      }
      const int64_t row[fw::SESS_ROW] = {kv.first, (int64_t)q, w[0], w[1], w[2], it->second.rank,
                                         trig ? 1 : 0, p.sum, p.mn, p.mx, p.cnt, p.f1, lh, lt, ln};
      rows.insert(rows.end(), row, row + fw::SESS_ROW);
    }
  }
  if (used.size() != wc.size()) return reject(e, FW_ERR_INVALID_ARG, "window-contents state of no in-flight session");
  if (!std::includes(tset.begin(), tset.end(), want.begin(), want.end()))
    return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the sessions imply");
  std::vector<std::array<int64_t, 3>> rorph;   // PurgingTrigger + lateness: cleanup timers of purged sessions
  for (const auto& t : tset) {
    if (want.count(t)) continue;
    const int64_t max_ts = fw::jsub(t[2], 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
    if (c.trigger != FW_TRIGGER_PURGING_EVENT_TIME || ct == max_ts || t[3] != ct || t[2] <= t[1] ||
        host_key_group(s, t[0]) != kg)
      return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the sessions imply");
    rorph.push_back({t[0], t[1], t[2]});
  }
  HIPCHK(e, hipSetDevice(e->dev));
  for (const auto& kv : mws) e->sess_mws_rank[kv.first] = (int64_t)e->sess_mws_rank.size();
  e->sess_rorphans.insert(rorph.begin(), rorph.end());
  if (e->sess_adv.empty()) e->sess_adv.push_back({watermark, 0});
  for (const auto& t : got) e->restored_timer_rank[t] = (int64_t)e->restored_timer_rank.size();
  if (wc_seen) e->sess_wc_table = true;
  if (mws_seen) e->sess_mws_table = true;
  if (wc_present) e->kg_touched[kgi] = 1;
  if (mws_present) e->mws_created[kgi] = 1;
  e->restored = true;
  e->cur_wm = watermark;
  e->state_epoch++;
  if (!pool.empty()) {   // the entries the restored elements took (the pool's free ring hands out the rest)
    std::vector<int64_t> pv(pool.size()), pf(pool.size()), pn(pool.size());
    const int64_t first = pool[0][0];
    for (size_t j = 0; j < pool.size(); ++j) { pv[j] = pool[j][1]; pf[j] = pool[j][2]; pn[j] = pool[j][3]; }
    HIPCHK(e, hipMemcpy(d.pv + first, pv.data(), 8 * pv.size(), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(d.pf1 + first, pf.data(), 8 * pf.size(), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(d.pnext + first, pn.data(), 8 * pn.size(), hipMemcpyHostToDevice));
    const unsigned long long taken = (unsigned long long)e->sess_pool_used;
    HIPCHK(e, hipMemcpy(d.pool, &taken, 8, hipMemcpyHostToDevice));
  }
  const int64_t n = (int64_t)(rows.size() / fw::SESS_ROW);
  if (n == 0) return FW_OK;
  int64_t* dr = nullptr;
  HIPCHK(e, hipMalloc(&dr, 8 * rows.size()));
  hipError_t r = hipMemcpyAsync(dr, rows.data(), 8 * rows.size(), hipMemcpyHostToDevice, e->stream);
  if (r == hipSuccess) {
    hipLaunchKernelGGL(fw::k_sess_restore, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, e->stream, e->s,
                       e->sess, dr, n, -((int64_t)1 << 61));
    r = hipGetLastError();
  }
  const hipError_t r2 = hipStreamSynchronize(e->stream);
  (void)hipFree(dr);
  HIPCHK(e, r);
  HIPCHK(e, r2);
  return check_device_error(e);
}

int fw_snapshot_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, void* state, int64_t state_cap,
                         int64_t* state_len, void* timers, int64_t timers_cap, int64_t* timers_len) {
  if (!e || !state_len || !timers_len) return FW_ERR_INVALID_ARG;
  if (e->session) {
    if (e->sticky) return e->sticky;
    if (kg < e->s.kg_start || kg > e->s.kg_end)
      return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
    if (e->used_key_hash) return reject(e, FW_ERR_UNSUPPORTED, "snapshot needs Long keys (a push carried Java key hashes)");
    if (int rc = check_state_layout(e, layout)) return rc;
    return session_snapshot_kg_flink(e, kg, layout, state, state_cap, state_len, timers, timers_cap, timers_len);
  }
  if (e->sticky) return e->sticky;
  if (kg < e->s.kg_start || kg > e->s.kg_end)
    return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
  if (e->used_key_hash) return reject(e, FW_ERR_UNSUPPORTED, "snapshot needs Long keys (a push carried Java key hashes)");
  int rc = check_state_layout(e, layout);
  if (rc) return rc;
  const fw_config& c = e->cfg;
  const bool sl_purge = c.trigger == FW_TRIGGER_PURGING_EVENT_TIME && c.allowed_lateness > 0 && c.assigner == FW_SLIDING;
  if (sl_purge && !e->s.first)
    return reject(e, FW_ERR_UNSUPPORTED, "sliding windows under PurgingTrigger with allowed lateness need first-arrival "
                                         "tracking (keep_first_f1) to tell which keys' cleanup timers outlive a purge");
  HIPCHK(e, hipSetDevice(e->dev));
  rc = build_snapshot(e);
  if (rc) return rc;
  std::vector<KgPane> panes;
  kg_panes(e, kg, panes);
  struct Ghost { int64_t key, start, end, first; };
  std::vector<Ghost> sl_ghosts;
  if (sl_purge) {   // fired windows: no state (FIRE_AND_PURGE); cleanup timers of the keys that had an element before
    std::vector<KgPane> kept;
    std::set<std::pair<int64_t, int64_t>> seen;
    for (const KgPane& p : panes) {
      const int64_t max_ts = fw::jsub(p.end, 1);
      if (max_ts > e->cur_wm) { kept.push_back(p); continue; }
      int64_t fire_ord = 0;   // the arrival ordinal at the advance that fired the window (or the restore)
      for (const auto& a : e->adv_log) if (a.first >= max_ts) { fire_ord = a.second; break; }
      if (p.first + e->ordinal < fire_ord && seen.insert({p.start, p.key}).second) sl_ghosts.push_back({p.key, p.start, p.end, p.first});
    }
    for (const auto& g : e->sl_ghost) {   // restored ones
      const int64_t end = fw::jadd(g.first, c.size);
      if (fw::cleanup_time(fw::jsub(end, 1), c.allowed_lateness) <= e->cur_wm || host_key_group(e->s, g.second) != kg) continue;
      if (seen.insert({g.first, g.second}).second) sl_ghosts.push_back({g.second, g.first, end, INT64_MIN});
    }
    panes.swap(kept);
  }
  const bool first = e->s.first;
  bool any_state = e->snap_any_key;
  for (uint8_t t : e->kg_touched) any_state = any_state || t;
  fwkg::BeOut st, tm;
  if (any_state) {
    const bool present = !panes.empty() || e->snap_has_key[(size_t)kg] ||
                         (!e->kg_touched.empty() && e->kg_touched[(size_t)(kg - e->s.kg_start)]);
    st.i32(kg);
    st.i16(0);
    st.u8(present ? 1 : 0);
    if (present) {
      // namespaces: HashMap<TimeWindow, HashMap<K, S>>, created by the first arrival into the window
      std::map<std::pair<int64_t, int64_t>, std::vector<size_t>> ns;
      for (size_t i = 0; i < panes.size(); ++i) ns[{panes[i].start, panes[i].end}].push_back(i);
      std::vector<std::pair<std::pair<int64_t, int64_t>, std::vector<size_t>>> nsv(ns.begin(), ns.end());
      std::vector<int64_t> ns_first(nsv.size(), INT64_MAX);
      for (size_t w = 0; w < nsv.size(); ++w)
        for (size_t i : nsv[w].second) ns_first[w] = std::min(ns_first[w], panes[i].first);
      std::vector<size_t> wo(nsv.size());
      for (size_t w = 0; w < wo.size(); ++w) wo[w] = w;
      fwkg::hashmap_order(
          wo, [&](size_t w) { return fwkg::window_hash(nsv[w].first.first, nsv[w].first.second); },
          [&](size_t a, size_t b) {
            return first && ns_first[a] != ns_first[b] ? ns_first[a] < ns_first[b] : nsv[a].first < nsv[b].first;
          });
      st.i32((int32_t)nsv.size());
      for (size_t w : wo) {
        st.i64(nsv[w].first.first);
        st.i64(nsv[w].first.second);
        std::vector<size_t>& ent = nsv[w].second;
        fwkg::hashmap_order(
            ent, [&](size_t i) { return fw::long_hash_code(panes[i].key); },
            [&](size_t a, size_t b) {
              return first && panes[a].first != panes[b].first ? panes[a].first < panes[b].first : panes[a].key < panes[b].key;
            });
        st.i32((int32_t)ent.size());
        for (size_t i : ent) {
          st.i64(panes[i].key);
          if (e->list) {   // ListSerializer.serialize: int size, then every element in insertion order
            // (sliding: the window's list holds its slices' elements of the key, merged in arrival order)
            std::vector<std::array<int64_t, 3>> merged;
            if (c.assigner == FW_SLIDING) {
              const int64_t n = fw::floor_div(fw::jsub(panes[i].start, c.offset), c.slide);
              for (int64_t mm = n * e->s.R; mm < n * e->s.R + e->s.K; ++mm) {
                auto it = e->snap_list.find({mm, panes[i].key});
                if (it != e->snap_list.end()) merged.insert(merged.end(), it->second.begin(), it->second.end());
              }
              std::sort(merged.begin(), merged.end());
            }
            const auto& el = c.assigner == FW_SLIDING ? merged : e->snap_list.at({panes[i].m, panes[i].key});
            st.i32((int32_t)el.size());
            for (const auto& x : el)
              for (int f = 0; f < layout->n_fields; ++f) {
                const int fld = layout->field[f];
                if (fld == FW_SF_KEY) st.i64(panes[i].key);
                else if (fld == FW_SF_F1) st.i64(x[2]);
                else if (e->s.vt == FW_VALUE_F64) { double d; memcpy(&d, &x[1], 8); st.f64(d); }
                else st.i64(x[1]);
              }
            continue;
          }
          for (int f = 0; f < layout->n_fields; ++f) put_field(e, st, layout->field[f], panes[i]);
        }
      }
    }
  }
  // timers: per pane the trigger timer at maxTimestamp while it has not fired, and the cleanup timer (the
  // same timer when the lateness is 0), registered in that order by the pane's first arrival
  // (WindowOperator.java:314-330; EventTimeTrigger.onElement :37-45); a record's sliding windows register
  // theirs latest window first (SlidingEventTimeWindows.assignWindows :64-77)
  // (restored timers: added at restore, before any later one, in the order of the restored sections)
  struct Tm { int64_t key, start, end, ts, first; int kind; int64_t rank; };
  std::vector<Tm> tv;
  for (const KgPane& p : panes) {
    const int64_t max_ts = fw::jsub(p.end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
    if (max_ts > e->cur_wm && !p.unarmed) tv.push_back({p.key, p.start, p.end, max_ts, p.first, 0, INT64_MAX});
    if (ct != max_ts || max_ts <= e->cur_wm) tv.push_back({p.key, p.start, p.end, ct, p.first, 1, INT64_MAX});
  }
  for (const Ghost& g : sl_ghosts)
    tv.push_back({g.key, g.start, g.end, fw::cleanup_time(fw::jsub(g.end, 1), c.allowed_lateness), g.first, 1, INT64_MAX});
  // purged windows' cleanup timers (no state; a key whose window holds state again has the timer above)
  if (!e->snap_gkg.empty()) {
    std::set<std::pair<int64_t, int64_t>> has;
    for (const KgPane& p : panes) has.insert({p.start, p.key});
    const std::vector<int64_t>& g = e->snap_gkg[(size_t)kg];
    for (size_t j = 0; j + 3 <= g.size(); j += 3) {
      const int64_t start = host_window_start(c, g[j]), end = fw::jadd(start, c.size);
      if (has.count({start, g[j + 1]})) continue;
      tv.push_back({g[j + 1], start, end, fw::cleanup_time(fw::jsub(end, 1), c.allowed_lateness), g[j + 2], 1, INT64_MAX});
    }
  }
  if (!e->restored_timer_rank.empty())
    for (Tm& t : tv) {
      auto it = e->restored_timer_rank.find({t.key, t.start, t.end, t.ts});
      if (it != e->restored_timer_rank.end()) t.rank = it->second;
    }
  std::vector<size_t> to(tv.size());
  for (size_t i = 0; i < to.size(); ++i) to[i] = i;
  fwkg::hashmap_order(
      to, [&](size_t i) { return fwkg::timer_hash(tv[i].ts, tv[i].key, tv[i].start, tv[i].end); },
      [&](size_t a, size_t b) {
        const Tm &x = tv[a], &y = tv[b];
        if (x.rank != y.rank) return x.rank < y.rank;
        if (first && x.first != y.first) return x.first < y.first;
        if (!first && x.key != y.key) return x.key < y.key;
        if (x.start != y.start) return x.start > y.start;
        return x.kind < y.kind;
      });
  tm.i32((int32_t)tv.size());
  for (size_t i : to) {
    tm.i64(tv[i].key);
    tm.i64(tv[i].start);
    tm.i64(tv[i].end);
    tm.i64(tv[i].ts);
  }
  tm.i32(0);
  *state_len = (int64_t)st.b.size();
  *timers_len = (int64_t)tm.b.size();
  if (!state && !timers) return FW_OK;
  if (!state || !timers || state_cap < *state_len || timers_cap < *timers_len)
    return reject(e, FW_ERR_CAPACITY, "snapshot buffer too small");
  if (!st.b.empty()) memcpy(state, st.b.data(), st.b.size());
  memcpy(timers, tm.b.data(), tm.b.size());
  return FW_OK;
}

// list state (tumbling): the restored entries' elements appended to their slices' buffers (the directory and
// the slots were set by restore_entries), each with its ordinal in blob order
static int restore_list_elements(fw_engine* e, const std::vector<KgPane>& panes, const std::vector<int64_t>& slice_of,
                                 const std::vector<std::vector<std::array<int64_t, 2>>>& lists,
                                 const std::vector<int64_t>& ord0) {
  const fw::Spec& s = e->s;
  std::vector<int64_t> keys((size_t)s.D);
  HIPCHK(e, hipMemcpy(keys.data(), s.dir_keys, 8 * (size_t)s.D, hipMemcpyDeviceToHost));
  std::unordered_map<int64_t, int64_t> kid_of;
  for (int64_t k = 0; k < s.D; ++k) if (keys[(size_t)k] != fw::EMPTY_KEY) kid_of[keys[(size_t)k]] = k;
  std::vector<unsigned long long> lc((size_t)s.P);
  HIPCHK(e, hipMemcpy(lc.data(), e->lst.cnt, 8 * (size_t)s.P, hipMemcpyDeviceToHost));
  std::map<int32_t, std::vector<int64_t>> rows;   // slot -> elements (kid, ordinal, value, f1)
  for (size_t i = 0; i < panes.size(); ++i) {
    const int64_t kid = panes[i].key == fw::EMPTY_KEY ? s.D : (kid_of.count(panes[i].key) ? kid_of[panes[i].key] : -1);
    if (kid < 0) return reject(e, FW_ERR_CAPACITY, "restored key not in the key directory");
    auto& r = rows[(int32_t)fw::floor_mod(slice_of[i], s.P)];
    for (size_t q = 0; q < lists[i].size(); ++q) r.insert(r.end(), {kid, ord0[i] + (int64_t)q, lists[i][q][0], lists[i][q][1]});
  }
  for (auto& kv : rows) {
    const int32_t p = kv.first;
    const int64_t n = (int64_t)(kv.second.size() / LST_WORDS);
    if ((int64_t)lc[(size_t)p] + n > e->lst.cap)
      return reject(e, FW_ERR_CAPACITY, "restored list state exceeds list_capacity for its slice");
    HIPCHK(e, hipMemcpy(e->lst.buf + ((size_t)p * (size_t)e->lst.cap + lc[(size_t)p]) * LST_WORDS, kv.second.data(),
                        8 * kv.second.size(), hipMemcpyHostToDevice));
    lc[(size_t)p] += (unsigned long long)n;
  }
  HIPCHK(e, hipMemcpy(e->lst.cnt, lc.data(), 8 * (size_t)s.P, hipMemcpyHostToDevice));
  e->state_epoch++;
  return FW_OK;
}

// Sliding-window list state (slide dividing the size: a slice per slide, window n = slices n .. n + K - 1): the
// reference holds each window's list; the engine holds each record once, in its slice.  Per key, the windows are
// peeled newest first: window n's list, less the elements of slices n + 1 .. n + K - 1 (known from the newer
// windows, matched in order as a subsequence), is slice n; its elements join the key's arrival order right after
// the element they follow in the list.  Every window's list is then rebuilt from the slices and checked; the
// elements get ordinals in that arrival order, ahead of every later record
static int restore_sliding_lists(fw_engine* e, int64_t wm, const std::vector<KgPane>& panes, const std::vector<int64_t>& win,
                                 const std::vector<std::vector<std::array<int64_t, 2>>>& lists) {
  const fw::Spec& s = e->s;
  const int64_t K = s.K;
  std::map<int64_t, std::map<int64_t, size_t>> by_key;   // key -> window -> entry
  for (size_t i = 0; i < panes.size(); ++i) {
    by_key[panes[i].key][win[i]] = i;
    e->list_entry_rank[{panes[i].start, panes[i].key}] = e->restore_ord++;
  }
  struct El { int64_t v, f1, m; };
  std::map<std::pair<int64_t, int64_t>, std::vector<std::array<int64_t, 3>>> slices;   // (slice, key) -> (ord, v, f1)
  const int64_t R = s.R;
  // the oldest window still in its lifetime at wm (every newer one exists once a record of its slices arrived)
  int64_t n_alive = INT64_MIN / 4;
  if (wm != INT64_MIN) {
    const __int128 x = (__int128)wm - e->cfg.allowed_lateness - e->cfg.offset - e->cfg.size + 1;
    const __int128 sl = e->cfg.slide;
    __int128 q = x / sl;
    if (x % sl != 0 && x < 0) --q;
    n_alive = (int64_t)std::max<__int128>(q + 1, (__int128)(INT64_MIN / 4));
  }
  for (const auto& kw : by_key) {
    const int64_t key = kw.first;
    const auto& wins = kw.second;
    std::vector<El> order;
    if (R != 1) {
      // a slide that does not divide the size: each element (distinct within a window) is identified across the
      // windows' lists; its live windows [lo, hi] pick a slice m with floor(m / R) = hi whose oldest live window is
      // lo; the arrival order is any order every list agrees with (a topological order of their successions)
      std::map<std::pair<int64_t, int64_t>, int64_t> id;
      std::vector<El> el;
      std::vector<std::pair<int64_t, int64_t>> span;   // (lo, hi) of windows holding the element
      std::vector<int64_t> nwin;
      std::vector<std::vector<int64_t>> seqs;
      for (const auto& w : wins) {
        std::set<int64_t> seen;
        std::vector<int64_t> seq;
        for (const auto& x : lists[w.second]) {
          auto it = id.find({x[0], x[1]});
          int64_t k;
          if (it == id.end()) {
            k = (int64_t)el.size();
            id[{x[0], x[1]}] = k;
            el.push_back({x[0], x[1], 0});
            span.push_back({w.first, w.first});
            nwin.push_back(0);
          } else {
            k = it->second;
          }
          if (!seen.insert(k).second)
            return reject(e, FW_ERR_UNSUPPORTED, "sliding-window lists with equal elements (slide not dividing the size)");
          span[(size_t)k].first = std::min(span[(size_t)k].first, w.first);
          span[(size_t)k].second = std::max(span[(size_t)k].second, w.first);
          nwin[(size_t)k]++;
          seq.push_back(k);
        }
        seqs.push_back(std::move(seq));
      }
      for (size_t k = 0; k < el.size(); ++k) {
        const int64_t lo = span[k].first, hi = span[k].second;
        if (nwin[k] != hi - lo + 1) return reject(e, FW_ERR_INVALID_ARG, "an element missing from a window between its windows");
        bool found = false;
        for (int64_t m = hi * R; m < hi * R + R && !found; ++m) {
          const int64_t first_w = fw::floor_div(m - K + 1 + R - 1, R);
          if (std::max(first_w, n_alive) == lo) { el[k].m = m; found = true; }
        }
        if (!found) return reject(e, FW_ERR_INVALID_ARG, "an element's windows are not those of any slice");
      }
      std::vector<std::vector<int64_t>> succ(el.size());
      std::vector<int64_t> indeg(el.size(), 0);
      for (const auto& seq : seqs)
        for (size_t j = 1; j < seq.size(); ++j) { succ[(size_t)seq[j - 1]].push_back(seq[j]); indeg[(size_t)seq[j]]++; }
      std::set<int64_t> ready;
      for (size_t k = 0; k < el.size(); ++k) if (!indeg[k]) ready.insert((int64_t)k);
      while (!ready.empty()) {
        const int64_t k = *ready.begin();
        ready.erase(ready.begin());
        order.push_back(el[(size_t)k]);
        for (int64_t nx : succ[(size_t)k]) if (--indeg[(size_t)nx] == 0) ready.insert(nx);
      }
      if (order.size() != el.size()) return reject(e, FW_ERR_INVALID_ARG, "the windows' lists disagree on the arrival order");
    }
    for (int64_t n = wins.rbegin()->first; R == 1 && n >= wins.begin()->first; --n) {
      std::vector<size_t> T;   // the key's known elements of window n's newer slices, in arrival order
      for (size_t q = 0; q < order.size(); ++q)
        if (order[q].m > n && order[q].m < n + K) T.push_back(q);
      auto it = wins.find(n);
      if (it == wins.end()) {
        if (!T.empty()) return reject(e, FW_ERR_INVALID_ARG, "a window of the key is missing between its windows");
        continue;
      }
      std::vector<std::pair<size_t, El>> ins;   // (insert after this order index, or SIZE_MAX: at the front)
      size_t t = 0, pred = SIZE_MAX;
      for (const auto& x : lists[it->second]) {
        if (t < T.size() && order[T[t]].v == x[0] && order[T[t]].f1 == x[1]) { pred = T[t++]; continue; }
        ins.push_back({pred, El{x[0], x[1], n}});
      }
      if (t != T.size()) return reject(e, FW_ERR_INVALID_ARG, "the windows' lists of a key do not share their slices");
      std::vector<El> next;
      next.reserve(order.size() + ins.size());
      size_t k = 0;
      while (k < ins.size() && ins[k].first == SIZE_MAX) next.push_back(ins[k++].second);
      for (size_t q = 0; q < order.size(); ++q) {
        next.push_back(order[q]);
        while (k < ins.size() && ins[k].first == q) next.push_back(ins[k++].second);
      }
      order.swap(next);
    }
    for (const auto& w : wins) {   // every window's list rebuilt from the slices
      const auto& want = lists[w.second];
      size_t j = 0;
      for (const El& x : order) {
        if (x.m < w.first * R || x.m >= w.first * R + K) continue;
        if (j >= want.size() || want[j][0] != x.v || want[j][1] != x.f1)
          return reject(e, FW_ERR_UNSUPPORTED, "sliding-window lists with equal elements in an order no slice split gives");
        ++j;
      }
      if (j != want.size()) return reject(e, FW_ERR_UNSUPPORTED, "sliding-window lists with equal elements in an order no slice split gives");
    }
    for (const El& x : order) slices[{x.m, key}].push_back({e->restore_ord++, x.v, x.f1});
  }
  // the slices and keys into the directory and the slice table, then their elements into the slices' buffers
  std::vector<int64_t> ent;
  for (const auto& kv : slices) {
    const int64_t w[FW_SNAP_ENTRY_WORDS] = {kv.first.first, kv.first.second, 0, INT64_MAX, INT64_MIN, 0, kv.second[0][0], 0};
    ent.insert(ent.end(), w, w + FW_SNAP_ENTRY_WORDS);
  }
  int rc = restore_entries(e, wm, ent.data(), (int64_t)slices.size(), 0);
  if (rc) return rc;
  std::vector<int64_t> keys((size_t)s.D);
  HIPCHK(e, hipMemcpy(keys.data(), s.dir_keys, 8 * (size_t)s.D, hipMemcpyDeviceToHost));
  std::map<int64_t, int64_t> kid_of;
  for (int64_t k = 0; k < s.D; ++k) if (keys[(size_t)k] != fw::EMPTY_KEY) kid_of[keys[(size_t)k]] = k;
  std::vector<unsigned long long> lc((size_t)s.P);
  HIPCHK(e, hipMemcpy(lc.data(), e->lst.cnt, 8 * (size_t)s.P, hipMemcpyDeviceToHost));
  std::map<int32_t, std::vector<int64_t>> rows;   // slot -> elements (kid, ordinal, value, f1)
  for (const auto& kv : slices) {
    const int64_t key = kv.first.second;
    const int64_t kid = key == fw::EMPTY_KEY ? s.D : (kid_of.count(key) ? kid_of[key] : -1);
    if (kid < 0) return reject(e, FW_ERR_CAPACITY, "restored key not in the key directory");
    auto& r = rows[(int32_t)fw::floor_mod(kv.first.first, s.P)];
    for (const auto& x : kv.second) r.insert(r.end(), {kid, x[0], x[1], x[2]});
  }
  for (auto& kv : rows) {
    const int32_t p = kv.first;
    const int64_t n = (int64_t)(kv.second.size() / LST_WORDS);
    if ((int64_t)lc[(size_t)p] + n > e->lst.cap)
      return reject(e, FW_ERR_CAPACITY, "restored list state exceeds list_capacity for its slice");
    HIPCHK(e, hipMemcpy(e->lst.buf + ((size_t)p * (size_t)e->lst.cap + lc[(size_t)p]) * LST_WORDS, kv.second.data(),
                        8 * kv.second.size(), hipMemcpyHostToDevice));
    lc[(size_t)p] += (unsigned long long)n;
  }
  HIPCHK(e, hipMemcpy(e->lst.cnt, lc.data(), 8 * (size_t)s.P, hipMemcpyHostToDevice));
  e->state_epoch++;
  return FW_OK;
}

int fw_restore_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, int64_t watermark,
                        const void* state, int64_t state_len, const void* timers, int64_t timers_len) {
  if (!e || (!state && state_len) || !timers || state_len < 0) return FW_ERR_INVALID_ARG;
  if (e->session) {
    if (e->sticky) return e->sticky;
    if (e->pushes > 0 || e->records_in > 0) return reject(e, FW_ERR_INVALID_ARG, "restore after the first push");
    if (kg < e->s.kg_start || kg > e->s.kg_end)
      return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
    if (e->restored && watermark != e->cur_wm) return reject(e, FW_ERR_INVALID_ARG, "key groups restored at different watermarks");
    if (int rc = check_state_layout(e, layout)) return rc;
    return session_restore_kg_flink(e, kg, layout, watermark, state, state_len, timers, timers_len);
  }
  if (e->sticky) return e->sticky;
  if (e->pushes > 0 || e->records_in > 0) return reject(e, FW_ERR_INVALID_ARG, "restore after the first push");
  if (kg < e->s.kg_start || kg > e->s.kg_end)
    return reject(e, FW_ERR_INVALID_ARG, "Key Group " + std::to_string(kg) + " does not belong to the local range.");
  int rc = check_state_layout(e, layout);
  if (rc) return rc;
  const fw_config& c = e->cfg;
  const fw::Spec& s = e->s;
  const bool sliding = c.assigner == FW_SLIDING;
  if (e->restored && watermark != e->cur_wm)
    return reject(e, FW_ERR_INVALID_ARG, "key groups restored at different watermarks");
  const bool sl_purge = sliding && c.trigger == FW_TRIGGER_PURGING_EVENT_TIME && c.allowed_lateness > 0;
  if (sl_purge && !s.first)
    return reject(e, FW_ERR_UNSUPPORTED, "sliding windows under PurgingTrigger with allowed lateness need first-arrival "
                                         "tracking (keep_first_f1)");
  if (sl_purge && e->adv_log.empty()) e->adv_log.push_back({watermark, 0});   // windows fired before: at the restore
  const bool f64 = s.vt == FW_VALUE_F64;
  std::vector<KgPane> panes;
  std::vector<int64_t> slice_of;
  std::vector<std::vector<std::array<int64_t, 2>>> lists;   // list state: each entry's elements (value bits, f1)
  bool present = false;
  if (state_len > 0) {
    fwkg::BeIn in(state, state_len);
    if (in.i32() != kg) return reject(e, FW_ERR_INVALID_ARG, "state section of another key group");
    if (in.i16() != 0) return reject(e, FW_ERR_UNSUPPORTED, "keyed state other than window-contents");
    present = in.u8() != 0;
    const int32_t nns = present ? in.i32() : 0;
    if (nns < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt state section");
    std::set<std::pair<int64_t, int64_t>> seen;
    for (int32_t w = 0; w < nns && in.ok; ++w) {
      const int64_t start = in.i64(), end = in.i64();
      // tumbling: the window's slice; sliding: the window number (its own pane holds the window's state)
      const int64_t step = sliding ? c.slide : c.size;
      const int64_t m = fw::floor_div(fw::jsub(start, c.offset), step);
      if (in.ok && (end != fw::jadd(start, c.size) || host_window_start(c, m) != start ||
                    fw::window_start_with_offset(start, c.offset, step) != start))
        return reject(e, FW_ERR_INVALID_ARG, "namespace is not a window of this assigner");
      const int32_t ne = in.i32();
      if (ne < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt state section");
      for (int32_t j = 0; j < ne && in.ok; ++j) {
        KgPane p{start, end, in.i64(), 0, INT64_MAX, INT64_MIN, 0, 0, 0, false};
        if (e->list) {   // ListSerializer.deserialize: int size, then the elements
          const int32_t nel = in.i32();
          if (nel < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt list state");
          std::vector<std::array<int64_t, 2>> el;
          for (int32_t q = 0; q < nel && in.ok; ++q) {
            std::array<int64_t, 2> x{0, 0};
            for (int f = 0; f < layout->n_fields; ++f) {
              const int64_t v = in.i64();
              if (layout->field[f] == FW_SF_KEY && in.ok && v != p.key)
                return reject(e, FW_ERR_UNSUPPORTED, "element key field differs from the key");
              if (layout->field[f] == FW_SF_F1) x[1] = v;
              if (layout->field[f] == FW_SF_VALUE) x[0] = v;
            }
            el.push_back(x);
          }
          if (!in.ok) break;
          if (el.empty()) return reject(e, FW_ERR_INVALID_ARG, "empty list state entry");
          lists.push_back(std::move(el));
        }
        for (int f = 0; f < layout->n_fields && !e->list; ++f) {
          const int64_t x = in.i64();
          double d;
          memcpy(&d, &x, 8);
          switch (layout->field[f]) {
            case FW_SF_KEY:
              if (in.ok && x != p.key) return reject(e, FW_ERR_UNSUPPORTED, "state key field differs from the key");
              break;
            case FW_SF_F1: p.f1 = x; break;
            case FW_SF_SUM: p.sum = x; break;
            case FW_SF_MIN: p.mn = f64 ? (s.cmpto ? fw::f64_cmp_code(d) : fw::f64_min_code(d)) : x; break;
            case FW_SF_MAX: p.mx = f64 ? (s.cmpto ? fw::f64_cmp_code(d) : fw::f64_max_code(d)) : x; break;
            case FW_SF_COUNT: p.cnt = x; break;
            case FW_SF_VALUE: p.mn = p.mx = f64 ? fw::f64_cmp_code(d) : x; break;
          }
        }
        if (!in.ok) break;
        if (s.fold) p = unfold_pane(e, p);
        if (host_key_group(s, p.key) != kg) return reject(e, FW_ERR_KEY_GROUP, "state entry key outside its key group");
        if (!seen.insert({m, p.key}).second) return reject(e, FW_ERR_INVALID_ARG, "duplicate (window, key) entry");
        panes.push_back(p);
        slice_of.push_back(m);
      }
    }
    if (!in.done()) return reject(e, FW_ERR_INVALID_ARG, "state section truncated or with trailing bytes");
  }
  // timers: exactly the ones the panes imply at `watermark` (the engine's timers are implicit)
  std::vector<std::array<int64_t, 4>> got, want, got_in_order;
  {
    fwkg::BeIn in(timers, timers_len);
    const int32_t nt = in.i32();
    if (nt < 0) return reject(e, FW_ERR_INVALID_ARG, "corrupt timer section");
    for (int32_t i = 0; i < nt && in.ok; ++i) {
      const int64_t key = in.i64(), start = in.i64(), end = in.i64(), ts = in.i64();
      got.push_back({key, start, end, ts});
    }
    got_in_order = got;
    const int32_t np = in.i32();
    if (!in.done()) return reject(e, FW_ERR_INVALID_ARG, "timer section truncated or with trailing bytes");
    if (np != 0) return reject(e, FW_ERR_UNSUPPORTED, "processing-time timers");
  }
  // a window ahead of `watermark` whose panes carry no trigger timer fired before the checkpoint (the
  // reference restarts its timer service at Long.MIN_VALUE): it is restored disarmed — it fires again only for
  // keys a later record re-arms before the watermark passes it.  The panes of one window agree, in every key
  // group (an aligned checkpoint fired a window's timers for all its keys at one watermark)
  std::sort(got.begin(), got.end());
  std::set<int64_t> dis_now, armed_now;
  for (size_t i = 0; i < panes.size(); ++i) {
    const KgPane& p = panes[i];
    const int64_t max_ts = fw::jsub(p.end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
    if (ct <= watermark) return reject(e, FW_ERR_UNSUPPORTED, "pane past its cleanup time at the restore watermark");
    if (max_ts <= watermark) continue;
    const bool has = std::binary_search(got.begin(), got.end(), std::array<int64_t, 4>{p.key, p.start, p.end, max_ts});
    (has ? armed_now : dis_now).insert(slice_of[i]);
  }
  for (int64_t m : dis_now)
    if (armed_now.count(m) || e->armed_windows.count(m) || c.allowed_lateness == 0)
      return reject(e, FW_ERR_UNSUPPORTED, "a window with and without trigger timers (not an aligned checkpoint)");
  for (int64_t m : armed_now)
    if (e->disarmed.count(m)) return reject(e, FW_ERR_UNSUPPORTED, "a window with and without trigger timers (not an aligned checkpoint)");
  for (size_t i = 0; i < panes.size(); ++i) {
    const KgPane& p = panes[i];
    const int64_t max_ts = fw::jsub(p.end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
    if (max_ts > watermark && !dis_now.count(slice_of[i])) want.push_back({p.key, p.start, p.end, max_ts});
    if (ct != max_ts) want.push_back({p.key, p.start, p.end, ct});
  }
  std::sort(want.begin(), want.end());
  // PurgingTrigger + allowed lateness: a window purged by its fire keeps its keys' cleanup timers without state
  std::vector<int64_t> ghosts;   // restore entries (window, key, .., ordinal)
  if (s.gtag && got != want) {
    std::vector<std::array<int64_t, 4>> extra;
    if (!std::includes(got.begin(), got.end(), want.begin(), want.end()))
      return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the panes imply at the restore watermark");
    std::set_difference(got.begin(), got.end(), want.begin(), want.end(), std::back_inserter(extra));
    std::set<std::pair<int64_t, int64_t>> has;
    for (const KgPane& p : panes) has.insert({p.start, p.key});
    for (const auto& t : extra) {
      const int64_t key = t[0], start = t[1], end = t[2], ts = t[3];
      const int64_t m = fw::floor_div(fw::jsub(start, c.offset), c.size);
      const int64_t max_ts = fw::jsub(end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
      if (host_window_start(c, m) != start || end != fw::jadd(start, c.size) || ts != ct || ct == max_ts || ct <= watermark ||
          has.count({start, key}) || host_key_group(s, key) != kg)
        return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the panes imply at the restore watermark");
      const int64_t w[FW_SNAP_ENTRY_WORDS] = {m, key, 0, 0, 0, 0, 0, 0};
      ghosts.insert(ghosts.end(), w, w + FW_SNAP_ENTRY_WORDS);
    }
  } else if (sl_purge && got != want) {
    // sliding + PurgingTrigger + lateness: cleanup timers without state of fired, purged windows (each key
    // whose first element preceded the fire)
    if (!std::includes(got.begin(), got.end(), want.begin(), want.end()))
      return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the panes imply at the restore watermark");
    std::vector<std::array<int64_t, 4>> extra;
    std::set_difference(got.begin(), got.end(), want.begin(), want.end(), std::back_inserter(extra));
    std::set<std::pair<int64_t, int64_t>> has;
    for (const KgPane& p : panes) has.insert({p.start, p.key});
    for (const auto& t : extra) {
      const int64_t key = t[0], start = t[1], end = t[2], ts = t[3];
      const int64_t n = fw::floor_div(fw::jsub(start, c.offset), c.slide);
      const int64_t max_ts = fw::jsub(end, 1), ct = fw::cleanup_time(max_ts, c.allowed_lateness);
      if (host_window_start(c, n) != start || end != fw::jadd(start, c.size) || ts != ct || ct == max_ts ||
          has.count({start, key}) || host_key_group(s, key) != kg)
        return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the panes imply at the restore watermark");
      e->sl_ghost.insert({start, key});
    }
  } else if (got != want) {
    return reject(e, FW_ERR_UNSUPPORTED, "timers differ from the ones the panes imply at the restore watermark");
  }
  if (e->list && sliding) {
    if (!dis_now.empty())
      return reject(e, FW_ERR_UNSUPPORTED, "sliding-window list state restored below a window that fired before the "
                                           "checkpoint");
    for (const auto& t : got_in_order) e->restored_timer_rank[t] = (int64_t)e->restored_timer_rank.size();
    if (e->kg_touched.empty()) e->kg_touched.assign((size_t)(s.kg_end - s.kg_start + 1), 0);
    if (present) e->kg_touched[(size_t)(kg - s.kg_start)] = 1;
    return restore_sliding_lists(e, watermark, panes, slice_of, lists);
  }
  if (!dis_now.empty() && !e->s.disarm) {   // per-slot flags and per-pane re-arm marks, first needed here
    e->s.disarm = e->alloc<uint8_t>((size_t)s.P);
    e->s.armed = e->alloc<uint8_t>((size_t)s.P * (size_t)s.stride);
    if (int rc = upload_spec(e)) return rc;
    if (!e->s.disarm || !e->s.armed) return reject(e, FW_ERR_DEVICE, "out of device memory");
    HIPCHK(e, hipMemset(e->s.disarm, 0, (size_t)s.P));
    HIPCHK(e, hipMemset(e->s.armed, 0, (size_t)s.P * (size_t)s.stride));
  }
  for (int64_t m : dis_now) {
    e->disarmed.insert(m);
    const uint8_t one = 1;
    HIPCHK(e, hipMemcpy(e->s.disarm + floor_mod(m, s.P), &one, 1, hipMemcpyHostToDevice));
  }
  e->armed_windows.insert(armed_now.begin(), armed_now.end());
  // arrival ordinals in blob order: restored panes precede every later record, and keep the blob's
  // (HashMap iteration) order as their insertion order, as readStateTableForKeyGroup's puts do
  std::vector<int64_t> ent(panes.size() * FW_SNAP_ENTRY_WORDS);
  std::vector<int64_t> list_ord(panes.size());
  for (size_t i = 0; i < panes.size(); ++i) {
    const KgPane& p = panes[i];
    const int64_t ord = e->restore_ord;
    e->restore_ord += e->list ? (int64_t)lists[i].size() : 1;   // list state: one ordinal per element
    list_ord[i] = ord;
    const int64_t w[FW_SNAP_ENTRY_WORDS] = {slice_of[i], p.key, p.sum, p.mn, p.mx, s.by ? ord : p.cnt, ord, p.f1};
    memcpy(&ent[i * FW_SNAP_ENTRY_WORDS], w, sizeof(w));
  }
  for (const auto& t : got_in_order) e->restored_timer_rank[t] = (int64_t)e->restored_timer_rank.size();
  if (e->kg_touched.empty()) e->kg_touched.assign((size_t)(s.kg_end - s.kg_start + 1), 0);
  if (present) e->kg_touched[(size_t)(kg - s.kg_start)] = 1;
  rc = restore_entries(e, watermark, ent.data(), (int64_t)panes.size(), sliding ? 1 : 0);
  if (rc) return rc;
  if (e->list) return restore_list_elements(e, panes, slice_of, lists, list_ord);
  if (!s.gtag) return rc;
  // windows within their lateness at the restore watermark (later per-element fires purge them again), and the
  // restored cleanup timers without state, each with its arrival ordinal (after the panes', in blob order)
  rc = ghost_advance(e, INT64_MIN, watermark);
  const int64_t ng = (int64_t)(ghosts.size() / FW_SNAP_ENTRY_WORDS);
  for (int64_t j = 0; j < ng && !rc; ++j) {
    ghosts[(size_t)j * FW_SNAP_ENTRY_WORDS + 6] = s.first ? e->restore_ord++ : 0;
    rc = ghost_track(e, ghosts[(size_t)j * FW_SNAP_ENTRY_WORDS]);
  }
  if (rc) return rc;
  return restore_entries(e, watermark, ghosts.data(), ng, 2);
}

int fw_partition_by_operator(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1,
                             const int64_t* ts, const void* value, int64_t n, int32_t max_parallelism,
                             int32_t parallelism, int64_t* out_key, int32_t* out_key_hash, int64_t* out_f1,
                             int64_t* out_ts, void* out_value, int64_t* counts, int64_t* offsets) {
  return fw_partition_by_operator_last(e, key, key_hash, f1, ts, value, n, max_parallelism, parallelism, out_key,
                                       out_key_hash, out_f1, out_ts, out_value, counts, offsets, -1);
}

int fw_partition_by_operator_last(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1,
                                  const int64_t* ts, const void* value, int64_t n, int32_t max_parallelism,
                                  int32_t parallelism, int64_t* out_key, int32_t* out_key_hash, int64_t* out_f1,
                                  int64_t* out_ts, void* out_value, int64_t* counts, int64_t* offsets,
                                  int32_t last_operator) {
  if (!e) return FW_ERR_INVALID_ARG;
  if (parallelism <= 0 || parallelism > PART_MAX || max_parallelism < parallelism) return fail(e, FW_ERR_INVALID_ARG, "bad parallelism");
  if (last_operator >= parallelism) return fail(e, FW_ERR_INVALID_ARG, "last_operator >= parallelism");
  HIPCHK(e, hipSetDevice(e->dev));
  int64_t nblocks = std::max<int64_t>((n + PART_CHUNK - 1) / PART_CHUNK, 1);
  if (nblocks * parallelism > e->part_blocks_cap) {
    e->part_block_counts = e->alloc<int64_t>((size_t)(nblocks * parallelism));
    if (!e->part_block_counts) return fail(e, FW_ERR_DEVICE, "alloc");
    e->part_blocks_cap = nblocks * parallelism;
  }
  // with a caller stream set (fw_set_stream) the partition runs on it, ordered after the producer of the
  // batch and before whatever consumes the packed output there (the exchange); otherwise on the engine's
  hipStream_t ps = e->has_client ? (hipStream_t)e->client : e->stream;
  hipLaunchKernelGGL(k_part_count, dim3((unsigned)nblocks), dim3(BLOCK), 0, ps, key, key_hash, n, max_parallelism,
                     parallelism, e->part_block_counts);
  hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(PART_SCAN_THREADS), 0, ps, e->part_block_counts, nblocks, parallelism, counts, offsets,
                     last_operator < 0 ? -1 : last_operator);
  hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nblocks), dim3(BLOCK), 0, ps, key, key_hash, f1, ts,
                     (const int64_t*)value, n, max_parallelism, parallelism, e->part_block_counts, out_key, out_key_hash,
                     out_f1, out_ts, (int64_t*)out_value);
  HIPCHK(e, hipGetLastError());
  return FW_OK;
}

}  // extern "C"

#include "fw_decode.hip"
#include "fw_session.hip"
#include "fw_list.hip"
