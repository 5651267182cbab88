// fw_session.hip — event-time session windows on the GPU (included by fw_engine.hip).
//
// Replaces the merging branch of WindowOperator.processElement (SJ/runtime/operators/windowing/
// WindowOperator.java:228-301) over MergingWindowSet (MergingWindowSet.java:142-214, TimeWindow.mergeWindows
// TimeWindow.java:186-230) and its timers (EventTimeTrigger.onMerge :70-74, onEventTime :344-375), for
// EventTimeSessionWindows.withGap (EventTimeSessionWindows.java:53-56) with a reducing state (sum / min / max /
// count, first-arrival f1, maxBy / minBy) or a list state (WindowedStream.apply: the window's elements).
//
// Layout in HBM: per key id (the engine's key directory) `sw` window slots (max_open_slices, default 32, up to
// 256), key-major ([D + 1][sw]) so one key's windows share cache lines: window start / end and the accumulator
// (sum, min / max codes, count, f1); per key two bit masks of 1, 2 or 4 words: slots in flight, slots whose
// trigger timer is pending.
//
// A batch (every record of it sees the same watermark): k_sess_prep resolves each record's key id,
// rocPRIM sorts (key id, arrival index), and k_sess_walk runs one thread per key over that key's records in
// arrival order — the reference's per-record state machine, exactly: a new window [ts, ts + gap) merges
// with every in-flight window it intersects (start <= other.end && end >= other.start), the merged window's
// trigger timer is registered and the merged windows' timers dropped; the late check applies to the
// resulting window; the record is reduced into it; onElement fires it at once when its maxTimestamp is
// already behind the watermark (allowed lateness), purging it under PurgingTrigger.  Keys are independent,
// so keys run in parallel.  Cleanup timers are implicit: every in-flight window has one, at
// cleanupTime = maxTimestamp + lateness (clamped).
//
// A merge follows MergingWindowSet.addWindow exactly: the merged in-flight windows in the iteration order of
// the JDK HashSet TimeWindow.mergeWindows put them in (bucket of the spread TimeWindow.hashCode in a table
// of the capacity the adds grew, then insertion order = start order); the state window is the first one's,
// the others' states are reduced in that order and the result added to it
// (AbstractKeyedStateBackend.mergePartitionedStates :294-333).  So first-arrival f1, maxBy / minBy (ties by
// argument order, ComparableAggregator.java:74-81) and double sums come out as the reference's.  List state
// keeps each window's elements as a linked list through an element pool (a ring indexed by arrival
// ordinal, list_capacity entries): a merge concatenates the target's list and the sources' in that order.
// (Not modelled: HashMap treeification / early resize of a bucket holding 8+ of one group's windows.)
//
// A watermark: k_sess_wm, one thread per key: each live window's timers — the trigger timer at maxTimestamp
// (FIRE; PurgingTrigger: FIRE_AND_PURGE; cleanup when maxTimestamp is also the cleanup time), then the
// cleanup timer (retire).  Results are appended wave-aggregated; their order within one watermark's mark is
// unspecified (the reference's timer queue orders by timestamp, ties between keys in heap order; the
// operator contract compares a mark's records as a set, TestHarnessUtil.java:80-117).

namespace fw {

__device__ __forceinline__ void sess_emit(const Spec& s, unsigned long long pos, int64_t key, int64_t start, int64_t max_ts,
                                          const LateAcc& a) {
  emit_record(s, pos, key, a.f1, max_ts, a);
  if ((int64_t)pos < s.o.capacity) s.o.win_start[pos] = start;
}

__device__ __forceinline__ LateAcc sess_load(const Spec& s, const SessDev& d, int64_t x) {
  LateAcc a;
  a.vt = s.vt;
  a.sum = d.sum ? d.sum[x] : 0;
  a.mn = d.mn ? d.mn[x] : INT64_MAX;
  a.mx = d.mx ? d.mx[x] : INT64_MIN;
  a.cnt = d.cnt ? d.cnt[x] : 0;
  a.f1 = d.f1 ? d.f1[x] : 0;
  a.by = s.by;
  return a;
}
__device__ __forceinline__ void sess_store(const SessDev& d, int64_t x, const LateAcc& a) {
  if (d.sum) d.sum[x] = a.sum;
  if (d.mn) d.mn[x] = a.mn;
  if (d.mx) d.mx[x] = a.mx;
  if (d.cnt) d.cnt[x] = a.cnt;
  if (d.f1) d.f1[x] = a.f1;
}

// ReduceFunction.reduce(v1 = a, v2 = b) of the operator's reduce: the aggregates combined, f1 of v1 (the
// Tuple3.of(a.f0, a.f1, ...) shape); maxBy / minBy the extremal record, a tie to v1 (first) or v2 (last) —
// by argument order, as ComparableAggregator.reduce decides it (ComparableAggregator.java:74-81)
__device__ __forceinline__ LateAcc sess_combine(const Spec& s, const LateAcc& a, const LateAcc& b) {
  if (s.by) {
    const bool maxby = (s.by & FW_AGG_MAXBY) != 0;
    const int64_t ca = maxby ? a.mx : a.mn, cb = maxby ? b.mx : b.mn;
    if (ca == cb) return s.by_last ? b : a;
    return (maxby ? ca > cb : ca < cb) ? a : b;
  }
  LateAcc r = LateCombine()(a, b);
  r.f1 = a.f1;
  return r;
}

// java.util.HashSet<TimeWindow> iteration rank of a window: the bucket of its spread hash (HashMap.hash) in a
// table of `cap` buckets (TimeWindow.hashCode, TimeWindow.java:79-83)
__device__ __forceinline__ uint32_t sess_bucket(int64_t start, int64_t end, uint32_t cap) {
  const int32_t hs = (int32_t)(start ^ (int64_t)((uint64_t)start >> 32));
  const int32_t he = (int32_t)(end ^ (int64_t)((uint64_t)end >> 32));
  const uint32_t h = (uint32_t)hs * 31u + (uint32_t)he;
  return (h ^ (h >> 16)) & (cap - 1u);
}
// HashMap capacity after n adds to a default HashSet (16 buckets, load factor 0.75)
__device__ __forceinline__ uint32_t sess_set_cap(int n) {
  uint32_t cap = 16;
  while ((uint32_t)n * 4u > cap * 3u) cap <<= 1;
  return cap;
}

// list state: free a window's elements (their pool entries may be reused)
// (pool entries are handed out from a ring of free entry indices: freeq[(head, ftail)] mod pcap, pool[0] = head,
// pool[1] = ftail; an entry freed during a launch is listed in fpend (pool[2] entries) and joins the ring at
// k_sess_pool_recycle after it, so a launch only ever takes entries that were free when it started)
__device__ __forceinline__ void sess_list_free(const SessDev& d, int64_t x) {
  for (int64_t e = d.head[x], n = d.len[x]; n > 0 && e >= 0; --n) {
    const int64_t nx = d.pnext[e];
    const unsigned long long pos = atomicAdd(&d.pool[2], 1ull);
    if ((int64_t)pos < d.pcap) d.fpend[pos] = e;
    e = nx;
  }
  d.len[x] = 0;
}
// a pool entry for a new element, or -1 when every entry free at the launch's start is taken
__device__ __forceinline__ int64_t sess_pool_take(const SessDev& d) {
  const unsigned long long h = atomicAdd(&d.pool[0], 1ull);
  if (h >= d.pool[1]) { atomicAdd(&d.pool[0], ~0ull); return -1; }   // (pool[1] does not change during the launch)
  return d.freeq[h % (unsigned long long)d.pcap];
}
// list state: one output row per element of the window, in list order (InternalIterableWindowFunction)
__device__ __forceinline__ void sess_list_emit(const Spec& s, const SessDev& d, int64_t x, int64_t key, int64_t start,
                                               int64_t max_ts) {
  const int64_t n = d.len[x];
  if (n <= 0) return;
  unsigned long long pos = atomicAdd(s.o.count, (unsigned long long)n);
  int64_t e = d.head[x];
  for (int64_t j = 0; j < n && e >= 0; ++j, ++pos) {
    LateAcc a;
    a.vt = s.vt;
    a.sum = d.pv[e];
    sess_emit(s, pos, key, start, max_ts, a);
    if ((int64_t)pos < s.o.capacity && s.o.f1) s.o.f1[pos] = d.pf1[e];
    e = d.pnext[e];
  }
}

// per record: key group check (AbstractKeyedStateBackend.setCurrentKey :167-170), key id, and the sort key
// (key id << idx_bits) | arrival index (invalid records sort last)
__global__ __launch_bounds__(BLOCK) void k_sess_prep(Spec s, BatchIn b, unsigned long long* skey, int32_t idx_bits) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t key = b.key[i];
    const int32_t h = b.key_hash ? b.key_hash[i] : long_hash_code(key);
    unsigned long long k = ~0ull;
    const int32_t kg = record_key_group(s, h);
    if (kg < s.kg_start || kg > s.kg_end) {
      set_error(s.err, FW_ERR_KEY_GROUP);
    } else {
      const int64_t kid = dir_find_or_insert(s, key);
      if (kid < 0) cap_error(s, 20);
      else k = ((unsigned long long)kid << idx_bits) | (unsigned long long)i;
    }
    skey[i] = k;
  }
}

// a key's window slots as a bit set of NW 64-bit words (sw <= 64 NW slots)
template <int NW>
struct SBits {
  uint64_t w[NW];
  __device__ __forceinline__ static SBits none() { SBits b; for (int i = 0; i < NW; ++i) b.w[i] = 0; return b; }
  __device__ __forceinline__ static SBits low(int n) {   // slots [0, n)
    SBits b;
    for (int i = 0; i < NW; ++i) b.w[i] = n >= 64 * (i + 1) ? ~0ull : (n <= 64 * i ? 0ull : (1ull << (n - 64 * i)) - 1);
    return b;
  }
  __device__ __forceinline__ static SBits load(const unsigned long long* p) { SBits b; for (int i = 0; i < NW; ++i) b.w[i] = p[i]; return b; }
  __device__ __forceinline__ void store(unsigned long long* p) const { for (int i = 0; i < NW; ++i) p[i] = w[i]; }
  __device__ __forceinline__ bool any() const { uint64_t x = 0; for (int i = 0; i < NW; ++i) x |= w[i]; return x != 0; }
  __device__ __forceinline__ int count() const { int c = 0; for (int i = 0; i < NW; ++i) c += __popcll(w[i]); return c; }
  __device__ __forceinline__ bool test(int q) const { return (w[q >> 6] >> (q & 63)) & 1ull; }
  __device__ __forceinline__ void set(int q) { w[q >> 6] |= 1ull << (q & 63); }
  __device__ __forceinline__ void clr(int q) { w[q >> 6] &= ~(1ull << (q & 63)); }
  __device__ __forceinline__ SBits andnot(const SBits& o) const { SBits b; for (int i = 0; i < NW; ++i) b.w[i] = w[i] & ~o.w[i]; return b; }
  __device__ __forceinline__ SBits operator|(const SBits& o) const { SBits b; for (int i = 0; i < NW; ++i) b.w[i] = w[i] | o.w[i]; return b; }
  __device__ __forceinline__ bool operator!=(const SBits& o) const { bool d = false; for (int i = 0; i < NW; ++i) d |= w[i] != o.w[i]; return d; }
  __device__ __forceinline__ int first() const {   // lowest slot, -1 if none
    for (int i = 0; i < NW; ++i) if (w[i]) return 64 * i + __ffsll((long long)w[i]) - 1;
    return -1;
  }
  __device__ __forceinline__ int pop() { const int q = first(); if (q >= 0) clr(q); return q; }
  __device__ __forceinline__ uint32_t group(int g) const { return (uint32_t)(w[g >> 3] >> ((g & 7) * 8)) & 0xffu; }
};

// slots [8g, 8g + 8) of one key's column, loaded together: one memory round trip per group of slots instead of
// one per slot (the columns carry 8 slots of padding past the last key)
__device__ __forceinline__ void sess_load8(const int64_t* col, int g, int64_t* v) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = col[8 * g + k];
}

// one thread per key (the head of its run in the sorted keys): the key's records in arrival order
template <int NW>
__global__ __launch_bounds__(BLOCK) void k_sess_walk(Spec s, SessDev d, BatchIn b, const unsigned long long* sorted,
                                                     int64_t n, int32_t idx_bits) {
  typedef SBits<NW> B;
  const int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j0 >= n) return;
  const unsigned long long k0 = sorted[j0];
  if (k0 == ~0ull) return;
  const int64_t kid = (int64_t)(k0 >> idx_bits);
  if (j0 > 0 && (sorted[j0 - 1] >> idx_bits) == (unsigned long long)kid) return;   // not the head of its run
  if (d.hot > 0 && j0 + d.hot - 1 < n && (sorted[j0 + d.hot - 1] >> idx_bits) == (unsigned long long)kid) {
    d.hot_list[atomicAdd(d.hot_count, 1ull)] = j0;   // a hot key: one wave walks it (k_sess_walk_hot)
    return;
  }
  const int64_t key = kid_key(s, kid);
  const int32_t kkg = record_key_group(s, long_hash_code(key));
  const bool purging = s.trigger == FW_TRIGGER_PURGING_EVENT_TIME;
  const int64_t wm = b.wm;
  const int64_t base = kid * d.sw;
  const int64_t* st = d.start + base;
  const int64_t* en = d.end + base;
  B live = B::load(d.live + kid * NW), trig = B::load(d.trig + kid * NW);
  const B all = B::low(d.sw);
  unsigned long long late = 0, fires = 0;
  // retire a slot: its trigger and cleanup timers gone; list state frees its elements (a reducing state is
  // overwritten by the slot's next window)
  auto retire = [&](int q) {
    live.clr(q);
    trig.clr(q);
    if (d.list) sess_list_free(d, base + q);
  };
  // the accumulator of the slot last written, kept in registers (only this thread writes its key's slots):
  // a hot key's consecutive records into one session read it back without a memory round trip
  int cq = -1;
  LateAcc cacc;
  auto acc_load = [&](int q) -> LateAcc { return q == cq ? cacc : sess_load(s, d, base + q); };
  auto acc_store = [&](int q, const LateAcc& a) { sess_store(d, base + q, a); cq = q; cacc = a; };
  // the next record's columns are loaded while the current one is processed
  const unsigned long long imask = (1ull << idx_bits) - 1;
  int64_t ni = (int64_t)(k0 & imask);
  int64_t nts = b.ts[ni], nv = b.val[ni], nf1 = b.f1 ? b.f1[ni] : nts;
  const bool ck = d.ckpt != 0;   // checkpoint bookkeeping (FW_SESS_CKPT=0: off)
  if (ck && d.ktouch[kid] < 0) { d.ktouch[kid] = b.ord_base + ni; d.ktts[kid] = INT64_MAX; }   // getMergingWindowSet
  bool accepted = false;
  bool more = true;
  for (int64_t j = j0; more; ++j) {
    const int64_t ts = nts, v = nv, f1 = nf1;
    const int64_t ord = b.ord_base + ni;   // this record's arrival ordinal
    more = false;
    if (j + 1 < n) {
      const unsigned long long kn = sorted[j + 1];
      if ((kn >> idx_bits) == (unsigned long long)kid) {
        more = true;
        ni = (int64_t)(kn & imask);
        nts = b.ts[ni];
        nv = b.val[ni];
        nf1 = b.f1 ? b.f1[ni] : nts;
      }
    }
    LateAcc a;
    a.vt = s.vt;
    a.sum = v;
    a.mn = min_code(s.vt, s.cmpto, v);
    a.mx = max_code(s.vt, s.cmpto, v);
    a.cnt = 1;
    a.f1 = f1;
    a.by = s.by;
    // MergingWindowSet.addWindow: the new window's connected group of intersecting in-flight windows
    int64_t cs = ts, ce = jadd(ts, d.gap);
    B mask = B::none();
    for (;;) {   // (the fixed point — the connected group — does not depend on the order slots are tested in)
      B grew = B::none();
      const B cand = live.andnot(mask);
      for (int g = 0; g < 8 * NW; ++g) {
        const uint32_t bits = cand.group(g);
        if (!bits) continue;
        int64_t s8[8], e8[8];
        sess_load8(st, g, s8);
        sess_load8(en, g, e8);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (((bits >> k) & 1u) && cs <= e8[k] && ce >= s8[k]) { cs = min(cs, s8[k]); ce = max(ce, e8[k]); grew.set(8 * g + k); }
      }
      if (!grew.any()) break;
      mask = mask | grew;
    }
    int r = -1;          // slot of the resulting window
    bool fresh = false, contained = false;
    if (!mask.any()) {
      fresh = true;
    } else {
      r = mask.first();
      contained = mask.count() == 1 && st[r] == cs && en[r] == ce;   // new window inside an existing one
      if (!contained) {
        // merge: the group's HashSet holds the merged in-flight windows and the new one (distinct from all of
        // them here); iterated by (bucket, insertion = start order), the first window's state is the target,
        // the others' states reduce in that order into one result added to it.  EventTimeTrigger.onMerge
        // registers the merged window's timer, the merged windows' timers go.
        const uint32_t cap = sess_set_cap(mask.count() + 1);
        auto before = [&](int c, uint32_t bc, int q, uint32_t bq) { return q < 0 || bc < bq || (bc == bq && st[c] < st[q]); };
        int t = -1;
        uint32_t tb = 0;
        for (B m = mask; m.any();) {   // the target: least (bucket, start)
          const int c = m.pop();
          const uint32_t bc = sess_bucket(st[c], en[c], cap);
          if (before(c, bc, t, tb)) { t = c; tb = bc; }
        }
        LateAcc res;
        bool have = false;
        int64_t lh = -1, lt = -1, ll = 0;
        if (d.list) { lh = d.head[base + t]; lt = d.tail[base + t]; ll = d.len[base + t]; }
        B todo = mask;
        todo.clr(t);
        while (todo.any()) {   // the sources in iteration order
          int q = -1;
          uint32_t bq = 0;
          for (B m = todo; m.any();) {
            const int c = m.pop();
            const uint32_t bc = sess_bucket(st[c], en[c], cap);
            if (before(c, bc, q, bq)) { q = c; bq = bc; }
          }
          todo.clr(q);
          const int64_t x = base + q;
          if (ck) sess_ns_remove(d, kkg, key, x, ord);   // the source's state window entry cleared
          if (d.list) {   // the source's elements appended (mergePartitionedStates, list branch :315-333)
            if (d.len[x] > 0) {
              if (ll == 0) lh = d.head[x];
              else d.pnext[lt] = d.head[x];
              lt = d.tail[x];
              ll += d.len[x];
              d.len[x] = 0;
            }
          } else {
            const LateAcc sv = acc_load(q);
            res = have ? sess_combine(s, res, sv) : sv;
            have = true;
          }
        }
        if (d.list) {
          d.head[base + t] = lh;
          d.tail[base + t] = lt;
          d.len[base + t] = ll;
        } else if (have) {
          acc_store(t, sess_combine(s, acc_load(t), res));   // HeapReducingState.add
        }
        B others = mask;
        others.clr(t);
        live = live.andnot(others);
        trig = trig.andnot(mask);
        trig.set(t);
        r = t;
        d.start[base + r] = cs;
        d.end[base + r] = ce;
        if (ck) d.cre[base + r] = d.tre[base + r] = ord;   // onMerge's trigger timer, then the cleanup timer
      }
    }
    const int64_t max_ts = jsub(ce, 1);
    if (cleanup_time(max_ts, s.lateness) <= wm) {   // isLate(actualWindow): retireWindow, the record dropped
      ++late;
      if (r >= 0) retire(r);
      continue;
    }
    if (fresh) {
      r = all.andnot(live).first();
      if (r < 0) { cap_error(s, 21); continue; }   // more in-flight sessions for the key than slots
      live.set(r);
      trig.clr(r);
      d.start[base + r] = cs;
      d.end[base + r] = ce;
      if (ck) {
        d.sws[base + r] = cs;
        d.swc[base + r] = d.cre[base + r] = d.tre[base + r] = ord;
        sess_ns_add(d, kkg, cs);
      }
      if (d.list) d.len[base + r] = 0;
    }
    const int64_t x = base + r;
    if (ck) d.put[x] = ord;   // MergingWindowSet.addWindow re-puts the window the record lands in
    accepted = true;
    LateAcc cur;
    if (d.list) {
      // HeapListState.add: the element appended in a free pool entry
      const int64_t e = sess_pool_take(d);
      if (e < 0) {   // more elements buffered at once than list_capacity
        cap_error(s, 26);
        if (fresh) live.clr(r);
        continue;
      }
      d.pv[e] = v;
      d.pf1[e] = a.f1;
      d.pnext[e] = -1;
      if (d.len[x] == 0) d.head[x] = e;
      else d.pnext[d.tail[x]] = e;
      d.tail[x] = e;
      d.len[x] += 1;
    } else {
      cur = fresh ? a : sess_combine(s, acc_load(r), a);
      acc_store(r, cur);
    }
    // EventTimeTrigger.onElement on the (possibly merged) window
    if (max_ts <= wm) {
      if (d.list) {
        sess_list_emit(s, d, x, key, cs, max_ts);
      } else {
        const unsigned long long pos = atomicAdd(s.o.count, 1ull);
        sess_emit(s, pos, key, cs, max_ts, cur);
      }
      ++fires;
      if (purging) {   // FIRE_AND_PURGE: cleanup(actualWindow); an unchanged window's cleanup timer stays
        if (ck && contained && s.lateness > 0) sess_orphan(d, key, cs, ce, d.cre[x]);
        if (ck) sess_ns_remove(d, kkg, key, x, ord);
        retire(r);
      }
    } else {
      if (ck && !trig.test(r)) d.tre[x] = ord;   // (re-armed: a window restored below its fire)
      trig.set(r);
    }
  }
  live.store(d.live + kid * NW);
  trig.store(d.trig + kid * NW);
  if (ck && accepted) d.kacc[kid] = 1;
  if (late) atomicAdd(&s.stats[ST_LATE], late);
  if (fires) { atomicAdd(&s.stats[ST_FIRED], fires); atomicAdd(&s.stats[ST_LATE_FIRES], fires); }
}

// a hot key's run (>= d.hot records of the batch, reducing state): the same per-record state machine as
// k_sess_walk, one wave per key.  Lane l holds slots l + 64 w (window bounds and accumulator in registers);
// the record columns are loaded 64 at a time, one per lane, and processed in arrival order from registers
// (wave-uniform control flow: every lane takes every decision with the same values)
template <int NW>
struct SLane {   // one wave's copy of a key's slots, slot q at lane q & 63, word q >> 6
  int64_t st[NW], en[NW], sum[NW], mn[NW], mx[NW], cnt[NW], f1[NW];
};
template <int NW>
__device__ __forceinline__ int64_t slane_get(const int64_t (&v)[NW], int q) {
  int64_t x = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) if (w == (q >> 6)) x = v[w];
  return __shfl(x, q & 63);
}
template <int NW>
__device__ __forceinline__ void slane_set(int64_t (&v)[NW], int q, int64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int w = 0; w < NW; ++w) if (w == (q >> 6) && lane == (q & 63)) v[w] = x;
}
template <int NW>
__device__ __forceinline__ LateAcc slane_acc(const Spec& s, const SLane<NW>& L, int q) {
  LateAcc a;
  a.vt = s.vt;
  a.sum = slane_get<NW>(L.sum, q);
  a.mn = slane_get<NW>(L.mn, q);
  a.mx = slane_get<NW>(L.mx, q);
  a.cnt = slane_get<NW>(L.cnt, q);
  a.f1 = slane_get<NW>(L.f1, q);
  a.by = s.by;
  return a;
}
template <int NW>
__device__ __forceinline__ void slane_put(SLane<NW>& L, int q, const LateAcc& a) {
  slane_set<NW>(L.sum, q, a.sum);
  slane_set<NW>(L.mn, q, a.mn);
  slane_set<NW>(L.mx, q, a.mx);
  slane_set<NW>(L.cnt, q, a.cnt);
  slane_set<NW>(L.f1, q, a.f1);
}
// a wave-uniform value made visibly uniform to the compiler (scalar registers, scalar branches)
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t wave_min64(int64_t x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, (int64_t)__shfl_xor((long long)x, o));
  return x;
}
__device__ __forceinline__ int64_t wave_max64(int64_t x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, (int64_t)__shfl_xor((long long)x, o));
  return x;
}

template <int NW>
__global__ __launch_bounds__(64) void k_sess_walk_hot(Spec s, SessDev d, BatchIn b, const unsigned long long* sorted,
                                                      int64_t n, int32_t idx_bits) {
  typedef SBits<NW> B;
  if ((unsigned long long)blockIdx.x >= *d.hot_count) return;
  const int lane = threadIdx.x & 63;
  const int64_t j0 = d.hot_list[blockIdx.x];
  const int64_t kid = (int64_t)(sorted[j0] >> idx_bits);
  const int64_t key = kid_key(s, kid);
  const int32_t kkg = record_key_group(s, long_hash_code(key));
  const bool purging = s.trigger == FW_TRIGGER_PURGING_EVENT_TIME;
  const int64_t wm = b.wm;
  const int64_t base = kid * d.sw;
  const unsigned long long imask = (1ull << idx_bits) - 1;
  const bool ck = d.ckpt != 0;
  if (ck && lane == 0 && d.ktouch[kid] < 0) { d.ktouch[kid] = b.ord_base + (int64_t)(sorted[j0] & imask); d.ktts[kid] = INT64_MAX; }
  bool accepted = false;
  SLane<NW> L;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int q = lane + 64 * w;
    const bool in = q < d.sw;
    const int64_t x = base + q;
    L.st[w] = in ? d.start[x] : 0;
    L.en[w] = in ? d.end[x] : 0;
    L.sum[w] = in && d.sum ? d.sum[x] : 0;
    L.mn[w] = in && d.mn ? d.mn[x] : INT64_MAX;
    L.mx[w] = in && d.mx ? d.mx[x] : INT64_MIN;
    L.cnt[w] = in && d.cnt ? d.cnt[x] : 0;
    L.f1[w] = in && d.f1 ? d.f1[x] : 0;
  }
  B live = B::load(d.live + kid * NW), trig = B::load(d.trig + kid * NW);
#pragma unroll
  for (int w = 0; w < NW; ++w) { live.w[w] = (uint64_t)uni64((int64_t)live.w[w]); trig.w[w] = (uint64_t)uni64((int64_t)trig.w[w]); }
  const B all = B::low(d.sw);
  unsigned long long late = 0, fires = 0;
  // the slot the previous record went to, replicated in every lane (a hot key's records mostly extend one
  // session: its bounds and accumulator are then read without cross-lane reads)
  int cr = -1;
  int64_t c_st = 0, c_en = 0;
  LateAcc c_acc;
  auto gst = [&](int q) -> int64_t { return q == cr ? c_st : slane_get<NW>(L.st, q); };
  auto gen = [&](int q) -> int64_t { return q == cr ? c_en : slane_get<NW>(L.en, q); };
  auto gacc = [&](int q) -> LateAcc { return q == cr ? c_acc : slane_acc<NW>(s, L, q); };
  bool done = false;
  for (int64_t jc = j0; !done; jc += 64) {
    // 64 records of the run, one per lane
    const int64_t j = jc + lane;
    bool mine = false;
    int64_t rts = 0, rv = 0, rf1 = 0, ri = 0;
    if (j < n) {
      const unsigned long long kj = sorted[j];
      if ((kj >> idx_bits) == (unsigned long long)kid) {
        const int64_t i = (int64_t)(kj & imask);
        ri = i;
        mine = true;
        rts = b.ts[i];
        rv = b.val[i];
        rf1 = b.f1 ? b.f1[i] : rts;
      }
    }
    const uint64_t have = __ballot(mine);
    const int cnt_here = __popcll(have);   // the run's records are a prefix of the 64
    if (cnt_here < 64) done = true;
    for (int t = 0; t < cnt_here; ++t) {
      const int64_t ts = uni64(__shfl(rts, t)), v = uni64(__shfl(rv, t)), f1 = uni64(__shfl(rf1, t));
      const int64_t ord = b.ord_base + uni64(__shfl(ri, t));
      LateAcc a;
      a.vt = s.vt;
      a.sum = v;
      a.mn = min_code(s.vt, s.cmpto, v);
      a.mx = max_code(s.vt, s.cmpto, v);
      a.cnt = 1;
      a.f1 = f1;
      a.by = s.by;
      // the connected group of intersecting in-flight windows (a fixed point, as k_sess_walk's)
      int64_t cs = ts, ce = jadd(ts, d.gap);
      B mask = B::none();
      for (;;) {
        B grew = B::none();
        int64_t lo = INT64_MAX, hi = INT64_MIN;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const int q = lane + 64 * w;
          const bool c = live.test(q) && !mask.test(q) && cs <= L.en[w] && ce >= L.st[w];
          grew.w[w] = __ballot(c);
          if (c) { lo = min(lo, L.st[w]); hi = max(hi, L.en[w]); }
        }
        if (!grew.any()) break;
        mask = mask | grew;
        if (grew.count() == 1) {   // (the usual case: one window grows the group)
          const int q = grew.first();
          cs = uni64(min(cs, gst(q)));
          ce = uni64(max(ce, gen(q)));
        } else {
          cs = uni64(min(cs, wave_min64(lo)));
          ce = uni64(max(ce, wave_max64(hi)));
        }
      }
      int r = -1;
      bool fresh = false, contained = false;
      if (!mask.any()) {
        fresh = true;
      } else {
        r = mask.first();
        contained = mask.count() == 1 && gst(r) == cs && gen(r) == ce;
        if (!contained) {   // merge, in the JDK HashSet order (see k_sess_walk)
          const uint32_t cap = sess_set_cap(mask.count() + 1);
          int tq = -1;
          uint32_t tb = 0;
          int64_t tst = 0;
          for (B m = mask; m.any();) {
            const int c = m.pop();
            const int64_t sc = gst(c);
            const uint32_t bc = sess_bucket(sc, gen(c), cap);
            if (tq < 0 || bc < tb || (bc == tb && sc < tst)) { tq = c; tb = bc; tst = sc; }
          }
          LateAcc res;
          bool hv = false;
          B todo = mask;
          todo.clr(tq);
          while (todo.any()) {
            int q = -1;
            uint32_t bq = 0;
            int64_t sq = 0;
            for (B m = todo; m.any();) {
              const int c = m.pop();
              const int64_t sc = gst(c);
              const uint32_t bc = sess_bucket(sc, gen(c), cap);
              if (q < 0 || bc < bq || (bc == bq && sc < sq)) { q = c; bq = bc; sq = sc; }
            }
            todo.clr(q);
            if (ck && lane == 0) sess_ns_remove(d, kkg, key, base + q, ord);
            const LateAcc sv = gacc(q);
            res = hv ? sess_combine(s, res, sv) : sv;
            hv = true;
          }
          if (hv) {
            const LateAcc m2 = sess_combine(s, gacc(tq), res);
            slane_put<NW>(L, tq, m2);
            if (tq == cr) c_acc = m2;
          }
          B others = mask;
          others.clr(tq);
          live = live.andnot(others);
          trig = trig.andnot(mask);
          trig.set(tq);
          r = tq;
          slane_set<NW>(L.st, r, cs);
          slane_set<NW>(L.en, r, ce);
          if (r == cr) { c_st = cs; c_en = ce; }
          if (ck && lane == 0) d.cre[base + r] = d.tre[base + r] = ord;
        }
      }
      const int64_t max_ts = jsub(ce, 1);
      if (cleanup_time(max_ts, s.lateness) <= wm) {   // isLate(actualWindow)
        ++late;
        if (r >= 0) { live.clr(r); trig.clr(r); }
        continue;
      }
      if (fresh) {
        r = all.andnot(live).first();
        if (r < 0) { if (lane == 0) cap_error(s, 21); continue; }
        live.set(r);
        trig.clr(r);
        slane_set<NW>(L.st, r, cs);
        slane_set<NW>(L.en, r, ce);
        if (ck && lane == 0) { d.sws[base + r] = cs; d.swc[base + r] = d.cre[base + r] = d.tre[base + r] = ord; sess_ns_add(d, kkg, cs); }
      }
      if (ck && lane == 0) d.put[base + r] = ord;
      accepted = true;
      const LateAcc cur = fresh ? a : sess_combine(s, gacc(r), a);
      slane_put<NW>(L, r, cur);
      cr = __builtin_amdgcn_readfirstlane(r);   // slot r now holds [cs, ce) and cur in every lane's copy
      c_st = cs;
      c_en = ce;
      c_acc = cur;
      if (max_ts <= wm) {   // EventTimeTrigger.onElement: FIRE
        if (lane == 0) sess_emit(s, atomicAdd(s.o.count, 1ull), key, cs, max_ts, cur);
        ++fires;
        if (purging) {
          if (ck && lane == 0) {
            if (contained && s.lateness > 0) sess_orphan(d, key, cs, ce, d.cre[base + r]);
            sess_ns_remove(d, kkg, key, base + r, ord);
          }
          live.clr(r);
          trig.clr(r);
        }
      } else {
        if (ck && lane == 0 && !trig.test(r)) d.tre[base + r] = ord;
        trig.set(r);
      }
    }
  }
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int q = lane + 64 * w;
    if (q >= d.sw) continue;
    const int64_t x = base + q;
    d.start[x] = L.st[w];
    d.end[x] = L.en[w];
    if (d.sum) d.sum[x] = L.sum[w];
    if (d.mn) d.mn[x] = L.mn[w];
    if (d.mx) d.mx[x] = L.mx[w];
    if (d.cnt) d.cnt[x] = L.cnt[w];
    if (d.f1) d.f1[x] = L.f1[w];
  }
  if (lane == 0) {
    live.store(d.live + kid * NW);
    trig.store(d.trig + kid * NW);
    if (ck && accepted) d.kacc[kid] = 1;
    if (late) atomicAdd(&s.stats[ST_LATE], late);
    if (fires) { atomicAdd(&s.stats[ST_FIRED], fires); atomicAdd(&s.stats[ST_LATE_FIRES], fires); }
  }
}

// a watermark: every in-flight window's timers up to wm_new.  One thread per key; lane by lane the it-th window of
// each key, so the wave's appends stay aggregated (list state: one append per window, its element count)
template <int NW>
__global__ __launch_bounds__(BLOCK) void k_sess_wm(Spec s, SessDev d, int64_t wm_new, int64_t touch_ord) {
  typedef SBits<NW> B;
  const bool purging = s.trigger == FW_TRIGGER_PURGING_EVENT_TIME;
  const int64_t gstride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k0 = (int64_t)blockIdx.x * blockDim.x; k0 < s.stride; k0 += gstride) {   // uniform per wave
    const int64_t kid = k0 + threadIdx.x;
    B live = kid < s.stride ? B::load(d.live + kid * NW) : B::none(), trig = kid < s.stride ? B::load(d.trig + kid * NW) : B::none();
    const B live0 = live, trig0 = trig;
    // the slots' timers decided from their ends, 8 slots per memory round trip
    B fire_m = B::none(), ret_m = B::none();
    int64_t tmin = INT64_MAX;   // the key's first timer to fire (its set is fetched then)
    if (live.any()) {
      const int64_t* en = d.end + kid * d.sw;
      for (int g = 0; g < 8 * NW; ++g) {
        const uint32_t bits = live.group(g);
        if (!bits) continue;
        int64_t e8[8];
        sess_load8(en, g, e8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (!((bits >> k) & 1u)) continue;
          const int q = 8 * g + k;
          const int64_t max_ts = jsub(e8[k], 1);
          const int64_t ct = cleanup_time(max_ts, s.lateness);
          bool fire = false, retire = false;
          if (trig.test(q) && max_ts <= wm_new) {   // onEventTime(maxTimestamp): FIRE
            fire = true;
            trig.clr(q);
            if (purging || ct == max_ts) retire = true;       // FIRE_AND_PURGE, or isCleanupTime
            if (d.ckpt && purging && ct != max_ts && ct > wm_new)   // the purged window's cleanup timer stays
              sess_orphan(d, kid_key(s, kid), d.start[kid * d.sw + q], e8[k], d.cre[kid * d.sw + q]);
          }
          if (!retire && ct <= wm_new) {                    // onEventTime(cleanupTime): cleanup
            if (!fire && ct == max_ts) fire = true;         // (one timer at maxTimestamp == cleanupTime)
            retire = true;
          }
          if (fire) fire_m.set(q);
          if (retire) ret_m.set(q);
          if (fire || retire) tmin = min(tmin, fire ? max_ts : ct);
        }
      }
      live = live.andnot(ret_m);
      trig = trig.andnot(ret_m);
      if (d.ckpt && tmin != INT64_MAX && d.ktouch[kid] < 0) { d.ktouch[kid] = touch_ord; d.ktts[kid] = tmin; }
    }
    if (d.ckpt) {   // the retired windows' state entries cleared: listed (one reservation per wave) for k_sess_ns_retire, whose
        // thread per entry keeps the namespace counts off this kernel's per-key chain
      const int c = ret_m.count();
      int incl = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if ((int)(threadIdx.x & 63) >= o) incl += y;
      }
      const int total = __shfl(incl, 63);
      unsigned long long base = 0;
      if ((threadIdx.x & 63) == 63 && total) base = atomicAdd(d.rlist_n, (unsigned long long)total);
      base = __shfl(base, 63);
      unsigned long long pos = base + (unsigned long long)(incl - c);
      for (B m = ret_m; m.any(); ++pos)
        if ((int64_t)pos < d.rlist_cap) d.rlist[pos] = kid * d.sw + m.pop(); else m.pop();
    }
    // the fires (list state: and the retired windows' elements freed), the wave's appends aggregated
    B todo = d.list ? (fire_m | ret_m) : fire_m;
    int nl = todo.count();
    for (int o = 32; o > 0; o >>= 1) nl = max(nl, __shfl_xor(nl, o));
    for (int it = 0; it < nl; ++it) {
      bool fire = false;
      int q = -1;
      int64_t start = 0, max_ts = 0;
      if (todo.any()) {
        q = todo.pop();
        const int64_t x = kid * d.sw + q;
        fire = fire_m.test(q);
        start = d.start[x];
        max_ts = jsub(d.end[x], 1);
        if (d.list) {   // list state: every element of the window, then (retired) its pool entries freed
          if (fire) sess_list_emit(s, d, x, kid_key(s, kid), start, max_ts);
          if (ret_m.test(q)) sess_list_free(d, x);
        }
      }
      if (!d.list) {
        const unsigned long long pos = wave_append(s.o.count, fire);
        if (fire) sess_emit(s, pos, kid_key(s, kid), start, max_ts, sess_load(s, d, kid * d.sw + q));
      }
      wave_count(&s.stats[ST_FIRED], fire);
    }
    if (live != live0) live.store(d.live + kid * NW);
    if (trig != trig0) trig.store(d.trig + kid * NW);
  }
}

// the state entries k_sess_wm retired: namespace counts (and the shared-namespace log), a thread per entry
__global__ __launch_bounds__(BLOCK) void k_sess_ns_retire(Spec s, SessDev d, int64_t touch_ord) {
  const int64_t n = min((int64_t)*d.rlist_n, d.rlist_cap);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = d.rlist[i], kid = x / d.sw;
    const int64_t key = kid_key(s, kid);
    sess_ns_remove(d, record_key_group(s, long_hash_code(key)), key, x, touch_ord);
  }
}

// after a launch that freed pool entries: they join the free ring (one workgroup; a batch frees at most pcap)
__global__ __launch_bounds__(1024) void k_sess_pool_recycle(SessDev d) {
  const unsigned long long nf = min(d.pool[2], (unsigned long long)d.pcap), t = d.pool[1];
  for (unsigned long long i = threadIdx.x; i < nf; i += blockDim.x) d.freeq[(t + i) % (unsigned long long)d.pcap] = d.fpend[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    d.pool[1] = t + nf;
    d.pool[2] = 0;
  }
}
__global__ void k_sess_pool_init(SessDev d) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.pcap; i += (int64_t)gridDim.x * blockDim.x)
    d.freeq[i] = i;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    d.pool[0] = 0;
    d.pool[1] = (unsigned long long)d.pcap;
    d.pool[2] = 0;
  }
}

}  // namespace fw

using namespace fw;

static void session_pool_recycle(fw_engine* e) {
  if (e->sess.list) hipLaunchKernelGGL(k_sess_pool_recycle, dim3(1), dim3(1024), 0, e->stream, e->sess);
}

int session_create(fw_engine* e) {
  const Spec& s = e->s;
  SessDev& d = e->sess;
  d.gap = e->cfg.size;
  const size_t cells = (size_t)d.sw * (size_t)s.stride;
  d.start = e->alloc<int64_t>(cells + 8);   // (+ 8: sess_load8's groups past the last key's slots)
  d.end = e->alloc<int64_t>(cells + 8);
  d.sum = (s.agg & FW_AGG_SUM) ? e->alloc<int64_t>(cells) : nullptr;
  d.mn = (s.agg & FW_AGG_MIN) ? e->alloc<int64_t>(cells) : nullptr;
  d.mx = (s.agg & FW_AGG_MAX) ? e->alloc<int64_t>(cells) : nullptr;
  d.cnt = (s.agg & FW_AGG_COUNT) ? e->alloc<int64_t>(cells) : nullptr;
  if (s.by) {   // maxBy / minBy: the extremal value's code in its min / max column
    d.mn = (s.by & FW_AGG_MINBY) ? e->alloc<int64_t>(cells) : nullptr;
    d.mx = (s.by & FW_AGG_MAXBY) ? e->alloc<int64_t>(cells) : nullptr;
  }
  d.f1 = s.first && !e->list ? e->alloc<int64_t>(cells) : nullptr;
  d.list = e->list ? 1 : 0;
  if (e->list) {
    d.head = e->alloc<int64_t>(cells);
    d.tail = e->alloc<int64_t>(cells);
    d.len = e->alloc<int64_t>(cells);
    d.pcap = e->cfg.list_capacity > 0 ? e->cfg.list_capacity : 4 * e->cfg.max_batch;
    d.pv = e->alloc<int64_t>((size_t)d.pcap);
    d.pf1 = e->alloc<int64_t>((size_t)d.pcap);
    d.pnext = e->alloc<int64_t>((size_t)d.pcap);
    d.freeq = e->alloc<int64_t>((size_t)d.pcap);
    d.fpend = e->alloc<int64_t>((size_t)d.pcap);
    d.pool = e->alloc<unsigned long long>(4);
  }
  d.nw = (d.sw + 63) / 64 <= 1 ? 1 : (d.sw + 63) / 64 <= 2 ? 2 : 4;   // words of a key's slot masks
  // hot keys: runs of >= FW_SESS_HOT records (default 256; 0 = off) walked a wave each; reducing state only
  {
    const char* hv = getenv("FW_SESS_HOT");
    d.hot = e->list ? 0 : hv ? std::max(0, atoi(hv)) : 256;
    if (d.hot == 1) d.hot = 2;
  }
  if (d.hot > 0) {
    d.hot_list = e->alloc<int64_t>((size_t)(e->cfg.max_batch / d.hot + 1));
    d.hot_count = e->alloc<unsigned long long>(1);
  }
  d.live = e->alloc<unsigned long long>((size_t)s.stride * d.nw);
  d.trig = e->alloc<unsigned long long>((size_t)s.stride * d.nw);
  d.sws = e->alloc<int64_t>(cells);
  d.swc = e->alloc<int64_t>(cells);
  d.put = e->alloc<int64_t>(cells);
  d.cre = e->alloc<int64_t>(cells);
  d.tre = e->alloc<int64_t>(cells);
  d.ktouch = e->alloc<int64_t>((size_t)s.stride);
  d.ktts = e->alloc<int64_t>((size_t)s.stride);
  d.kacc = e->alloc<int32_t>((size_t)s.stride);
  {   // FW_SESS_CKPT=0: no checkpoint bookkeeping (the reference-layout snapshot then fails; ~13-16 % faster)
    const char* cv = getenv("FW_SESS_CKPT");
    d.ckpt = (cv && atoi(cv) == 0) ? 0 : 1;
  }
  {
    uint64_t m = 1024;
    while (m < 2 * (uint64_t)cells) m <<= 1;
    d.nsmask = m - 1;
    d.nscnt = e->alloc<int32_t>((size_t)m);
    d.nslog_cap = std::max<int64_t>(1 << 16, 2 * e->cfg.max_batch);
    d.nslog = e->alloc<int64_t>(4 * (size_t)d.nslog_cap);
    d.nslog_n = e->alloc<unsigned long long>(1);
    d.olog_cap = std::max<int64_t>(1 << 16, 2 * e->cfg.max_batch);
    d.olog = e->alloc<int64_t>(4 * (size_t)d.olog_cap);
    d.olog_n = e->alloc<unsigned long long>(1);
    d.rlist_cap = (int64_t)cells;   // (a watermark retires at most every slot)
    d.rlist = e->alloc<int64_t>(cells);
    d.rlist_n = e->alloc<unsigned long long>(1);
  }
  e->s.o.win_start = e->alloc<int64_t>((size_t)e->cfg.out_capacity);
  const size_t nb = (size_t)e->cfg.max_batch;
  e->sess_key = e->alloc<unsigned long long>(nb);
  e->sess_sorted = e->alloc<unsigned long long>(nb);
  e->sess_idx_bits = bits_for((uint64_t)e->cfg.max_batch);
  if (e->sess_idx_bits + bits_for((uint64_t)s.stride) > 63) return FW_ERR_UNSUPPORTED;
  e->sess_key_bits = e->sess_idx_bits + bits_for((uint64_t)s.stride);
  size_t tb = 0;
  (void)rocprim::radix_sort_keys(nullptr, tb, e->sess_key, e->sess_sorted, nb, 0, e->sess_key_bits, e->stream);
  e->sess_temp_bytes = tb;
  e->sess_temp = e->alloc<char>(tb);
  for (void* p : e->allocs) if (!p) return FW_ERR_DEVICE;
  HIPCHK(e, hipMemsetAsync(d.live, 0, 8 * (size_t)s.stride * d.nw, e->stream));
  if (d.list) {
    hipLaunchKernelGGL(k_sess_pool_init, dim3(64), dim3(BLOCK), 0, e->stream, d);   // every pool entry free
    HIPCHK(e, hipMemsetAsync(d.len, 0, 8 * cells, e->stream));
  }
  HIPCHK(e, hipMemsetAsync(d.trig, 0, 8 * (size_t)s.stride * d.nw, e->stream));
  HIPCHK(e, hipMemsetAsync(d.ktouch, 0xff, 8 * (size_t)s.stride, e->stream));   // -1: no key's set fetched yet
  HIPCHK(e, hipMemsetAsync(d.kacc, 0, 4 * (size_t)s.stride, e->stream));
  HIPCHK(e, hipMemsetAsync(d.nscnt, 0, 4 * (size_t)(d.nsmask + 1), e->stream));
  HIPCHK(e, hipMemsetAsync(d.nslog_n, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(d.olog_n, 0, 8, e->stream));
  HIPCHK(e, hipMemsetAsync(d.rlist_n, 0, 8, e->stream));
  return FW_OK;
}

int session_push(fw_engine* e, const BatchIn& b) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((b.n + BLOCK - 1) / BLOCK, e->grid));
  e->phase_begin(FW_PHASE_INGEST);
  hipLaunchKernelGGL(k_sess_prep, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, b, e->sess_key, e->sess_idx_bits);
  size_t tb = e->sess_temp_bytes;
  HIPCHK(e, rocprim::radix_sort_keys(e->sess_temp, tb, e->sess_key, e->sess_sorted, (size_t)b.n, 0, e->sess_key_bits,
                                     e->stream));
  const dim3 g((unsigned)((b.n + BLOCK - 1) / BLOCK));
  if (e->sess.hot > 0) HIPCHK(e, hipMemsetAsync(e->sess.hot_count, 0, 8, e->stream));
  if (e->sess.nw == 1) hipLaunchKernelGGL(k_sess_walk<1>, g, dim3(BLOCK), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
  else if (e->sess.nw == 2) hipLaunchKernelGGL(k_sess_walk<2>, g, dim3(BLOCK), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
  else hipLaunchKernelGGL(k_sess_walk<4>, g, dim3(BLOCK), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
  if (e->sess.hot > 0 && b.n >= e->sess.hot) {   // the hot keys' runs: one wave each (at most n / hot of them)
    const dim3 gh((unsigned)(b.n / e->sess.hot));
    if (e->sess.nw == 1) hipLaunchKernelGGL(k_sess_walk_hot<1>, gh, dim3(64), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
    else if (e->sess.nw == 2) hipLaunchKernelGGL(k_sess_walk_hot<2>, gh, dim3(64), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
    else hipLaunchKernelGGL(k_sess_walk_hot<4>, gh, dim3(64), 0, e->stream, e->s, e->sess, b, e->sess_sorted, b.n, e->sess_idx_bits);
  }
  e->phase_end(b.n);
  session_pool_recycle(e);   // the entries this batch's merges and retirements freed
  HIPCHK(e, hipGetLastError());
  if (e->cfg.allowed_lateness > 0) e->out_dirty = true;   // per-element fires may have appended
  return FW_OK;
}

int session_watermark(fw_engine* e, int64_t wm) {
  if (wm > e->cur_wm) {
    e->sess_adv.push_back({wm, e->ordinal});   // (checkpoints: when a restored orphan timer fired)
    e->phase_begin(FW_PHASE_FIRE);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((e->s.stride + BLOCK - 1) / BLOCK, e->grid));
    if (e->sess.nw == 1) hipLaunchKernelGGL(k_sess_wm<1>, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->sess, wm, e->ordinal);
    else if (e->sess.nw == 2) hipLaunchKernelGGL(k_sess_wm<2>, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->sess, wm, e->ordinal);
    else hipLaunchKernelGGL(k_sess_wm<4>, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->sess, wm, e->ordinal);
    if (e->sess.ckpt) {
      hipLaunchKernelGGL(k_sess_ns_retire, dim3(e->grid), dim3(BLOCK), 0, e->stream, e->s, e->sess, e->ordinal);
      HIPCHK(e, hipMemsetAsync(e->sess.rlist_n, 0, 8, e->stream));
    }
    e->phase_end(e->s.stride);
    session_pool_recycle(e);   // the entries of the windows purged
    e->cur_wm = wm;
    hipLaunchKernelGGL(k_mark_only, dim3(1), dim3(1), 0, e->stream, e->s, wm);
    e->hmarks.push_back({wm, e->dev_marks++, true});
    e->out_dirty = false;
  } else if (e->out_dirty) {
    hipLaunchKernelGGL(k_mark_only, dim3(1), dim3(1), 0, e->stream, e->s, wm);
    e->hmarks.push_back({wm, e->dev_marks++, true});
    e->out_dirty = false;
  } else {
    e->hmarks.push_back({wm, e->dev_marks - 1, false});
  }
  HIPCHK(e, hipGetLastError());
  return FW_OK;
}
