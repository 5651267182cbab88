// fw_oracle.cpp — CPU restatement of the reference's event-time WindowOperator path.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it, and only as the checker or the timed CPU column.
// The product path (flink_amd/, libflink_window.so) never links or calls it.
//
// It restates, literally and single-threaded, the Java code of the reference (kalmanchapman/flink
// 1.2-SNAPSHOT, paths relative to /root/reference; SJ = flink-streaming-java/src/main/java/org/
// apache/flink/streaming/, RT = flink-runtime/src/main/java/org/apache/flink/runtime/):
//   murmurHash                  flink-core/.../util/MathUtils.java:134-158
//   Long.hashCode / Tuple1      JDK Long.hashCode; flink-core/.../api/java/tuple/Tuple1.java:137-139
//   key groups                  RT/state/KeyGroupRangeAssignment.java:40-107
//   TimeWindow                  SJ/api/windowing/windows/TimeWindow.java:41-62,239-241
//   Tumbling assigner           SJ/api/windowing/assigners/TumblingEventTimeWindows.java:59-68
//   Sliding assigner            SJ/api/windowing/assigners/SlidingEventTimeWindows.java:64-77
//   processElement              SJ/runtime/operators/windowing/WindowOperator.java:222-226,302-333
//   onEventTime                 WindowOperator.java:336-375; fire :435-438; cleanup :420-428
//   isLate/cleanupTime          WindowOperator.java:470-472,479-486,511-514,527-530
//   EventTimeTrigger            SJ/api/windowing/triggers/EventTimeTrigger.java:37-62
//   PurgingTrigger              SJ/api/windowing/triggers/PurgingTrigger.java:47-53,68-76
//   session windows             SJ/api/windowing/assigners/EventTimeSessionWindows.java:53-56; TimeWindow
//                               .intersects/cover/mergeWindows TimeWindow.java:96-105,186-230; MergingWindowSet
//                               .addWindow/getStateWindow/retireWindow MergingWindowSet.java:97-214; the merging
//                               branch WindowOperator.java:228-301, onEventTime :344-353, cleanup :420-428;
//                               AbstractKeyedStateBackend.mergePartitionedStates (reducing) :294-314;
//                               EventTimeTrigger.onMerge :70-74; TriggerResult.merge
//   HeapReducingState.add       RT/state/heap/HeapReducingState.java:84-122
//   AbstractHeapState.clear     RT/state/heap/AbstractHeapState.java:90-119
//   StateTable                  RT/state/heap/StateTable.java:27-77
//   timer service               SJ/api/operators/HeapInternalTimerService.java:211-236,264-278
//   InternalTimer               SJ/api/operators/InternalTimer.java:59-86
//   processWatermark            SJ/api/operators/AbstractStreamOperator.java:803-808
//   wire format (decode)        SpanningRecordSerializer.java:69-92 (int32 BE length prefix; the receiver
//                               reads a length, then that many bytes), StreamElementSerializer.deserialize
//                               SJ/runtime/streamrecord/StreamElementSerializer.java:183-198, TupleSerializer
//                               .deserialize flink-core/.../typeutils/runtime/TupleSerializer.java:132-139
//   checkpoint, per key group   RT/state/heap/HeapKeyedStateBackend.java:196-248 (writeStateTableForKeyGroup),
//                               :251-349 (readStateTableForKeyGroup); HeapInternalTimerService.java:285-345;
//                               TimeWindow.Serializer TimeWindow.java:141-158; InternalTimer.TimerSerializer
//                               InternalTimer.java:145-157; JDK HashMap/HashSet iteration order (see below)
//   fold                        RT/state/heap/HeapFoldingState.java:84-122 (first add folds into the default value)
//   list state                  RT/state/heap/HeapListState.java:84-112 (add appends; get iterates in insertion order),
//                               InternalIterableWindowFunction (every element to the window function)
//   reduce functions            SJ/api/functions/aggregation/SumAggregator.java:64-72, SumFunction.java:60-77,
//                               JDK Math.min/Math.max (double), Long arithmetic (wrapping),
//                               ComparableAggregator.java:66-90 + Comparator.java:45-105 (min/max/minBy/maxBy
//                               over Comparable fields: Long.compareTo, Double.compareTo)
//
// Java semantics kept: wrapping int32/int64 arithmetic (done in unsigned), logical >>>, truncating %,
// Long.MIN_VALUE-timestamp error, cleanup-time overflow clamp, arrival-order left fold.
//
// C API (fwo_*) mirrors include/flink_window.h so tests can drive oracle and engine identically.
#include "../include/flink_window.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace {

// ---------------- Java integer helpers ----------------
inline int32_t jint_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
inline int32_t jint_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t rotl32(int32_t v, int r) { uint32_t u = (uint32_t)v; return (int32_t)((u << r) | (u >> (32 - r))); }
inline int32_t ushr32(int32_t v, int r) { return (int32_t)((uint32_t)v >> r); }
inline int64_t jlong_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t jlong_sub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

// MathUtils.murmurHash(int) — MathUtils.java:134-158
int32_t murmurHash(int32_t code) {
  code = jint_mul(code, (int32_t)0xcc9e2d51);
  code = rotl32(code, 15);
  code = jint_mul(code, (int32_t)0x1b873593);
  code = rotl32(code, 13);
  code = jint_add(jint_mul(code, 5), (int32_t)0xe6546b64);
  code ^= 4;
  code ^= ushr32(code, 16);
  code = jint_mul(code, (int32_t)0x85ebca6b);
  code ^= ushr32(code, 13);
  code = jint_mul(code, (int32_t)0xc2b2ae35);
  code ^= ushr32(code, 16);
  if (code >= 0) return code;
  else if (code != INT32_MIN) return -code;
  else return 0;
}
// JDK Long.hashCode(long) = (int)(value ^ (value >>> 32))
int32_t longHashCode(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32)); }
// java.util.HashMap's spread of a key's hashCode and the capacity a HashSet grew to by n adds
int32_t hmSpread(int32_t h) { return h ^ ushr32(h, 16); }
uint32_t hmCapacitySet(size_t n) {
  uint32_t cap = 16;
  while ((double)n > cap * 0.75) cap <<= 1;
  return cap;
}
// KeyGroupRangeAssignment.computeKeyGroupForKeyHash — :62-64
int32_t computeKeyGroupForKeyHash(int32_t keyHash, int32_t maxParallelism) {
  return murmurHash(keyHash) % maxParallelism;
}
// KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup — :105-107
int32_t computeOperatorIndexForKeyGroup(int32_t maxParallelism, int32_t parallelism, int32_t keyGroupId) {
  return keyGroupId * parallelism / maxParallelism;
}

// ---------------- windows ----------------
struct TimeWindow {  // TimeWindow.java:41-62
  int64_t start, end;
  int64_t maxTimestamp() const { return jlong_sub(end, 1); }
  bool operator==(const TimeWindow& o) const { return start == o.start && end == o.end; }
  bool operator<(const TimeWindow& o) const { return start != o.start ? start < o.start : end < o.end; }
};
// TimeWindow.hashCode (TimeWindow.java:79-83): 31 * Long.hashCode(start) + Long.hashCode(end)
int32_t timeWindowHash(const TimeWindow& w) {
  return (int32_t)((uint32_t)longHashCode(w.start) * 31u + (uint32_t)longHashCode(w.end));
}
struct TimeWindowHash {
  size_t operator()(const TimeWindow& w) const { return std::hash<int64_t>()(w.start) * 31 + std::hash<int64_t>()(w.end); }
};
// TimeWindow.getWindowStartWithOffset — :239-241
int64_t getWindowStartWithOffset(int64_t timestamp, int64_t offset, int64_t windowSize) {
  int64_t num = jlong_add(jlong_sub(timestamp, offset), windowSize);
  return jlong_sub(timestamp, num % windowSize);
}

// ---------------- accumulator = the reduced record ----------------
struct ListElem { int64_t vi; double vd; int64_t f1; };
struct Acc {
  int64_t seq;   // when this (namespace, key) entry was put into its HashMap (iteration order), not state
  std::shared_ptr<std::vector<ListElem>> list;   // FW_AGG_LIST: HeapListState's elements, insertion order
  int64_t key;
  int64_t f1;
  int64_t sum_i, min_i, max_i, count;
  double sum_d, min_d, max_d;
};

// JDK Math.min(double,double) / Math.max(double,double)
double javaMin(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;
  return (a <= b) ? a : b;
}
double javaMax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
  return (a >= b) ? a : b;
}

// JDK Double.compare(a, b): doubleToLongBits order (every NaN equal, above +inf; -0.0 < +0.0)
int64_t doubleOrderKey(double x) {
  int64_t b;
  if (x != x) b = 0x7ff8000000000000ll;   // doubleToLongBits canonicalises NaN
  else std::memcpy(&b, &x, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
int javaDoubleCompare(double a, double b) {
  const int64_t x = doubleOrderKey(a), y = doubleOrderKey(b);
  return x < y ? -1 : (x == y ? 0 : 1);
}
int javaLongCompare(int64_t a, int64_t b) { return a < b ? -1 : (a == b ? 0 : 1); }

struct Config {
  fw_config c;
  int64_t size() const { return c.size; }
};

// ReduceFunction.reduce(value1 = stored, value2 = incoming); non-aggregated fields from value1
// (SumAggregator.java:64-72 copies value1; user lambdas of the form Tuple.of(a.f0, a.f1, ...) likewise).
Acc reduceFn(const fw_config& c, const Acc& v1, const Acc& v2) {
  if (c.agg_mask == FW_AGG_MAXBY || c.agg_mask == FW_AGG_MINBY) {
    // ComparableAggregator.reduce, byAggregate (ComparableAggregator.java:74-81): the field is the record's
    // value; Comparator MaxBy/MinBy.isExtremal (Comparator.java:60-93) -> 1 / 0 / -1
    const int cmp = c.value_type == FW_VALUE_I64 ? javaLongCompare(v1.max_i, v2.max_i) : javaDoubleCompare(v1.max_d, v2.max_d);
    const int ext = c.agg_mask == FW_AGG_MAXBY ? (cmp > 0 ? 1 : (cmp == 0 ? 0 : -1)) : (cmp < 0 ? 1 : (cmp == 0 ? 0 : -1));
    const bool first = (c.agg_flags & FW_AGGF_BY_LAST) == 0;
    if (ext == 0) return first ? v1 : v2;
    return ext == 1 ? v1 : v2;
  }
  Acc r = v1;
  if (c.value_type == FW_VALUE_I64) {
    r.sum_i = jlong_add(v1.sum_i, v2.sum_i);                 // SumFunction.LongSum :60-66
    r.min_i = v1.min_i <= v2.min_i ? v1.min_i : v2.min_i;     // Math.min(long,long)
    r.max_i = v1.max_i >= v2.max_i ? v1.max_i : v2.max_i;     // Math.max(long,long)
  } else {
    r.sum_d = v1.sum_d + v2.sum_d;                            // SumFunction.DoubleSum :68-77
    if (c.agg_flags & FW_AGGF_COMPARABLE) {
      // ComparableAggregator MIN / MAX (not byAggregate): value1's field becomes o2 unless o1 is
      // extremal (MinComparator / MaxComparator.isExtremal, Comparator.java:45-56,95-105)
      r.min_d = javaDoubleCompare(v1.min_d, v2.min_d) < 0 ? v1.min_d : v2.min_d;
      r.max_d = javaDoubleCompare(v1.max_d, v2.max_d) > 0 ? v1.max_d : v2.max_d;
    } else {
      r.min_d = javaMin(v1.min_d, v2.min_d);
      r.max_d = javaMax(v1.max_d, v2.max_d);
    }
  }
  r.count = jlong_add(v1.count, v2.count);
  return r;
}

// ---------------- timers ----------------
struct InternalTimer {  // InternalTimer.java:59-86 — equality on (timestamp, key, namespace)
  int64_t timestamp;
  int64_t key;
  TimeWindow ns;
  bool operator<(const InternalTimer& o) const {
    if (timestamp != o.timestamp) return timestamp < o.timestamp;  // queue order: timestamp (ties arbitrary)
    if (key != o.key) return key < o.key;
    return ns < o.ns;
  }
};

enum TriggerResult { CONTINUE = 0, FIRE_AND_PURGE = 1, FIRE = 2, PURGE = 3 };
inline bool isFire(TriggerResult r) { return r == FIRE || r == FIRE_AND_PURGE; }
inline bool isPurge(TriggerResult r) { return r == PURGE || r == FIRE_AND_PURGE; }

struct OutRec {
  Acc acc;
  int64_t ts;
  int64_t start;   // window.getStart() (the window function's view of the window)
};

struct Operator {
  fw_config cfg;
  std::string err;
  int64_t currentWatermark = INT64_MIN;   // HeapInternalTimerService.currentWatermark initial value
  // StateTable: per key group -> namespace -> key -> value   (StateTable.java:36)
  std::vector<std::unordered_map<TimeWindow, std::unordered_map<int64_t, Acc>, TimeWindowHash>> state;
  // event-time timers: set gives both the HashSet dedupe and the PriorityQueue order
  std::set<InternalTimer> timers;
  // insertion order of the JVM's hash tables (checkpoint iteration order): per key group when each
  // namespace was put into the namespace map, when each timer was added to the timer set; whether the
  // key group's namespace map exists at all (StateTable.get(kg) != null)
  int64_t seqCounter = 0;
  std::vector<std::unordered_map<TimeWindow, int64_t, TimeWindowHash>> nsSeq;
  std::vector<uint8_t> kgCreated;
  std::map<InternalTimer, int64_t> timerSeq;
  bool anyState = false;   // HeapKeyedStateBackend.stateTables non-empty (created by the first state access)
  // current key context
  int64_t curKey = 0;
  int32_t curKeyGroup = 0;
  // outputs
  std::vector<OutRec> out;
  std::vector<int64_t> mark_wm, mark_pos;
  fw_stats stats{};
  // materialised output columns for fwo_collect
  std::vector<int64_t> c_key, c_f1, c_ts, c_sum_i, c_min_i, c_max_i, c_count, c_start;
  // session windows: per key the in-flight windows -> their state window (MergingWindowSet.windows, a
  // HashMap<W, W>; ordered here by (start, end), which mergeWindows' stable sort by start makes equivalent)
  std::unordered_map<int64_t, std::map<TimeWindow, TimeWindow>> mergingWindowsByKey;
  // checkpoint bookkeeping of session windows (WindowOperator.java:445-460 getMergingWindowSet, :724-736
  // snapshotState; MergingWindowSet.java:77-95): when each in-flight window was last put into its key's
  // MergingWindowSet.windows (a HashMap: remove + put moves it to the end of its bucket), when each key's set
  // entered mergingWindowsByKey, and the "merging-window-set" list state (VoidNamespace) per key group: an
  // entry per key written by a snapshot or read by a restore, cleared when the key's set is first fetched
  std::unordered_map<int64_t, std::map<TimeWindow, int64_t>> putSeq;
  std::unordered_map<int64_t, int64_t> mwsSeq;
  struct MwsEntry { int64_t seq; std::vector<std::pair<TimeWindow, TimeWindow>> list; };
  std::vector<std::unordered_map<int64_t, MwsEntry>> mwsHeap;
  std::vector<uint8_t> mwsKgCreated;
  bool mwsTable = false;   // the "merging-window-set" state table exists (first getMergingWindowSet or a restore)
  std::vector<double> c_sum_d, c_min_d, c_max_d;

  explicit Operator(const fw_config& c) : cfg(c) {
    state.resize((size_t)(cfg.kg_end - cfg.kg_start + 1));
    nsSeq.resize(state.size());
    kgCreated.assign(state.size(), 0);
    mwsHeap.resize(state.size());
    mwsKgCreated.assign(state.size(), 0);
  }

  // ---- WindowAssigner.assignWindows ----
  int assignWindows(int64_t timestamp, std::vector<TimeWindow>& ws) {
    ws.clear();
    if (!(timestamp > INT64_MIN)) {
      err = "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Is the time characteristic set to "
            "'ProcessingTime', or did you forget to call 'DataStream.assignTimestampsAndWatermarks(...)'?";
      return FW_ERR_NO_TIMESTAMP;
    }
    if (cfg.assigner == FW_TUMBLING) {  // TumblingEventTimeWindows.java:59-68
      int64_t start = getWindowStartWithOffset(timestamp, cfg.offset, cfg.size);
      ws.push_back({start, jlong_add(start, cfg.size)});
    } else {  // SlidingEventTimeWindows.java:64-77
      int64_t lastStart = getWindowStartWithOffset(timestamp, cfg.offset, cfg.slide);
      int64_t bound = jlong_sub(timestamp, cfg.size);
      int64_t guard = cfg.size / cfg.slide + 2;
      for (int64_t start = lastStart; start > bound; start = jlong_sub(start, cfg.slide)) {
        ws.push_back({start, jlong_add(start, cfg.size)});
        if ((int64_t)ws.size() > guard) { err = "sliding window enumeration wrapped around"; return FW_ERR_INVALID_ARG; }
      }
    }
    return FW_OK;
  }

  // ---- WindowOperator helpers ----
  int64_t cleanupTime(const TimeWindow& w) const {  // :511-514
    int64_t ct = jlong_add(w.maxTimestamp(), cfg.allowed_lateness);
    return ct >= w.maxTimestamp() ? ct : INT64_MAX;
  }
  bool isLate(const TimeWindow& w) const { return cleanupTime(w) <= currentWatermark; }  // :470-472
  bool isCleanupTime(const TimeWindow& w, int64_t time) const { return cleanupTime(w) == time; }  // :527-530

  // ---- keyed state: HeapReducingState ----
  std::unordered_map<TimeWindow, std::unordered_map<int64_t, Acc>, TimeWindowHash>* nsMap() {
    if (curKeyGroup < cfg.kg_start || curKeyGroup > cfg.kg_end) return nullptr;  // StateTable.get :55-57
    return &state[(size_t)(curKeyGroup - cfg.kg_start)];
  }
  int stateAdd(const TimeWindow& ns, const Acc& value) {  // HeapReducingState.add :84-122
    auto* m = nsMap();
    if (!m) { err = "Unexpected key group index. This indicates a bug."; return FW_ERR_KEY_GROUP; }  // StateTable.set :59-63
    const size_t kgi = (size_t)(curKeyGroup - cfg.kg_start);
    kgCreated[kgi] = 1;
    anyState = true;
    auto nit = m->find(ns);
    if (nit == m->end()) {
      nit = m->emplace(ns, std::unordered_map<int64_t, Acc>()).first;
      nsSeq[kgi][ns] = value.seq;
    }
    auto& keyed = nit->second;
    auto it = keyed.find(curKey);
    if (cfg.agg_mask == FW_AGG_LIST) {   // HeapListState.add: append (a new list on the first element)
      if (it == keyed.end()) {
        Acc a = value;
        a.list = std::make_shared<std::vector<ListElem>>();
        a.list->push_back({value.sum_i, value.sum_d, value.f1});
        keyed.emplace(curKey, a);
      } else {
        it->second.list->push_back({value.sum_i, value.sum_d, value.f1});
      }
      return FW_OK;
    }
    if (it == keyed.end()) {
      if (cfg.agg_flags & FW_AGGF_FOLD) {
        // HeapFoldingState.add (HeapFoldingState.java:111-118): no value yet -> fold(defaultValue, value); the
        // folds offered (acc + v, acc + 1, Math.min/max(acc, v)) then continue exactly as reduce(acc, value)
        Acc init = value;
        const int64_t x = cfg.fold_initial;
        double xd;
        std::memcpy(&xd, &x, 8);
        init.sum_i = jlong_add(x, value.sum_i);
        init.min_i = x <= value.min_i ? x : value.min_i;
        init.max_i = x >= value.max_i ? x : value.max_i;
        init.sum_d = xd + value.sum_d;
        init.min_d = javaMin(xd, value.min_d);
        init.max_d = javaMax(xd, value.max_d);
        init.count = jlong_add(x, value.count);
        keyed.emplace(curKey, init);
      } else {
        keyed.emplace(curKey, value);
      }
    } else {
      const int64_t sq = it->second.seq;   // HashMap.put of an existing key keeps its place
      it->second = reduceFn(cfg, it->second, value);
      it->second.seq = sq;
    }
    return FW_OK;
  }
  const Acc* stateGet(const TimeWindow& ns) {  // HeapReducingState.get :72-82
    auto* m = nsMap();
    if (!m) return nullptr;
    auto nit = m->find(ns);
    if (nit == m->end()) return nullptr;
    auto kit = nit->second.find(curKey);
    return kit == nit->second.end() ? nullptr : &kit->second;
  }
  void stateClear(const TimeWindow& ns) {  // AbstractHeapState.clear :90-119
    auto* m = nsMap();
    if (!m) return;
    auto nit = m->find(ns);
    if (nit == m->end()) return;
    if (nit->second.erase(curKey) == 0) return;
    if (!nit->second.empty()) return;
    nsSeq[(size_t)(curKeyGroup - cfg.kg_start)].erase(ns);
    m->erase(nit);
  }

  // ---- timer service ----
  void registerEventTimeTimer(const TimeWindow& ns, int64_t time) {  // :211-218
    const InternalTimer t{time, curKey, ns};
    if (timers.insert(t).second) timerSeq[t] = ++seqCounter;
  }
  void deleteEventTimeTimer(const TimeWindow& ns, int64_t time) {  // :229-236
    const InternalTimer t{time, curKey, ns};
    timers.erase(t);
    timerSeq.erase(t);
  }

  // ---- trigger ----
  TriggerResult triggerOnElement(const TimeWindow& w) {  // EventTimeTrigger.java:37-45
    TriggerResult r;
    if (w.maxTimestamp() <= currentWatermark) {
      r = FIRE;
    } else {
      registerEventTimeTimer(w, w.maxTimestamp());
      r = CONTINUE;
    }
    if (cfg.trigger == FW_TRIGGER_PURGING_EVENT_TIME) return isFire(r) ? FIRE_AND_PURGE : r;  // PurgingTrigger :47-50
    return r;
  }
  TriggerResult triggerOnEventTime(const TimeWindow& w, int64_t time) {  // EventTimeTrigger.java:48-52
    TriggerResult r = (time == w.maxTimestamp()) ? FIRE : CONTINUE;
    if (cfg.trigger == FW_TRIGGER_PURGING_EVENT_TIME) return isFire(r) ? FIRE_AND_PURGE : r;  // PurgingTrigger :52-55
    return r;
  }
  void triggerClear(const TimeWindow& w) { deleteEventTimeTimer(w, w.maxTimestamp()); }  // EventTimeTrigger.java:59-62

  // ---- WindowOperator.fire / cleanup / registerCleanupTimer ----
  void fire(const TimeWindow& w, const Acc& contents) {  // :435-438, InternalSingleValueWindowFunction + PassThrough
    if (cfg.agg_mask == FW_AGG_LIST) {   // InternalIterableWindowFunction: every element, in insertion order
      for (const ListElem& x : *contents.list) {
        Acc a{};
        a.key = contents.key;
        a.f1 = x.f1;
        a.sum_i = x.vi;
        a.sum_d = x.vd;
        out.push_back({a, w.maxTimestamp(), w.start});
      }
      stats.panes_fired++;
      return;
    }
    out.push_back({contents, w.maxTimestamp(), w.start});
    stats.panes_fired++;
  }
  void cleanup(const TimeWindow& w) {  // :420-428
    stateClear(w);
    triggerClear(w);
  }
  void registerCleanupTimer(const TimeWindow& w) { registerEventTimeTimer(w, cleanupTime(w)); }  // :479-486

  // ---- session windows: MergingWindowSet.addWindow (MergingWindowSet.java:142-214) with the merge function
  // of WindowOperator.processElement (:239-263); returns the window the element belongs to ----
  TimeWindow addWindow(std::map<TimeWindow, TimeWindow>& windows, const TimeWindow& newWindow) {
    // TimeWindow.mergeWindows (:186-230): sort by start, chain windows that intersect; the callback gets
    // every group whose HashSet has more than one window
    std::vector<TimeWindow> sorted;
    for (const auto& kv : windows) sorted.push_back(kv.first);
    sorted.push_back(newWindow);
    std::stable_sort(sorted.begin(), sorted.end(), [](const TimeWindow& a, const TimeWindow& b) { return a.start < b.start; });
    struct Group { TimeWindow cover; std::vector<TimeWindow> set; };   // set: HashSet, insertion order
    std::vector<Group> groups;
    auto intersects = [](const TimeWindow& a, const TimeWindow& b) { return a.start <= b.end && a.end >= b.start; };
    for (const TimeWindow& c : sorted) {
      if (!groups.empty() && intersects(groups.back().cover, c)) {
        Group& g = groups.back();
        g.cover = {std::min(g.cover.start, c.start), std::max(g.cover.end, c.end)};   // TimeWindow.cover
        if (std::find(g.set.begin(), g.set.end(), c) == g.set.end()) g.set.push_back(c);
      } else {
        groups.push_back({c, {c}});
      }
    }
    TimeWindow resultWindow = newWindow;
    bool anyMerge = false;
    for (Group& g : groups) {
      if (g.set.size() <= 1) continue;
      anyMerge = true;
      const TimeWindow mergeResult = g.cover;
      // HashSet<TimeWindow> iteration order: bucket of the spread hash in the table the adds grew, then
      // insertion order (java.util.HashMap)
      const size_t grown = g.set.size();
      std::vector<TimeWindow> merged = g.set;
      auto it = std::find(merged.begin(), merged.end(), newWindow);
      if (it != merged.end()) { merged.erase(it); resultWindow = mergeResult; }
      {
        const uint32_t mask = hmCapacitySet(grown) - 1;
        std::vector<std::pair<TimeWindow, size_t>> order;
        for (size_t i = 0; i < merged.size(); ++i) order.push_back({merged[i], i});
        std::stable_sort(order.begin(), order.end(), [&](const auto& a, const auto& b) {
          const uint32_t ia = (uint32_t)hmSpread(timeWindowHash(a.first)) & mask, ib = (uint32_t)hmSpread(timeWindowHash(b.first)) & mask;
          return ia != ib ? ia < ib : a.second < b.second;
        });
        for (size_t i = 0; i < merged.size(); ++i) merged[i] = order[i].first;
      }
      const TimeWindow mergedStateWindow = windows.at(merged.front());
      std::vector<TimeWindow> mergedStateWindows;
      for (const TimeWindow& m : merged) {
        auto f = windows.find(m);
        if (f != windows.end()) { mergedStateWindows.push_back(f->second); mwsErase(windows, f->first); }
      }
      mwsPut(windows, mergeResult, mergedStateWindow);
      {
        auto f = std::find(mergedStateWindows.begin(), mergedStateWindows.end(), mergedStateWindow);
        if (f != mergedStateWindows.end()) mergedStateWindows.erase(f);
      }
      const bool selfOnly = merged.size() == 1 && merged.front() == mergeResult;
      if (!selfOnly) {
        // the merge function: onMerge registers the merged window's timer (EventTimeTrigger.onMerge :70-74;
        // PurgingTrigger passes CONTINUE through), the merged windows' trigger and cleanup timers go
        registerEventTimeTimer(mergeResult, mergeResult.maxTimestamp());
        for (const TimeWindow& m : merged) {
          triggerClear(m);
          deleteEventTimeTimer(m, cleanupTime(m));
        }
        // AbstractKeyedStateBackend.mergePartitionedStates (:294-314): the sources reduced in list order
        // and cleared, the result added to the target state window
        const TimeWindow target = windows.at(mergeResult);
        if (cfg.agg_mask == FW_AGG_LIST) {
          // list state (:315-333): the sources' elements concatenated in list order, each source cleared,
          // then every element added to the target (HeapListState.add appends)
          std::vector<ListElem> elems;
          for (const TimeWindow& src : mergedStateWindows) {
            const Acc* sv = stateGet(src);
            if (sv && sv->list) elems.insert(elems.end(), sv->list->begin(), sv->list->end());
            stateClear(src);
          }
          for (const ListElem& x : elems) {
            Acc a{};
            a.key = curKey;
            a.sum_i = x.vi;
            a.sum_d = x.vd;
            a.f1 = x.f1;
            a.seq = ++seqCounter;
            stateAdd(target, a);
          }
          continue;
        }
        bool have = false;
        Acc result{};
        for (const TimeWindow& src : mergedStateWindows) {
          const Acc* sv = stateGet(src);
          if (!have) { if (sv) { result = *sv; have = true; } }
          else if (sv) result = reduceFn(cfg, result, *sv);
          stateClear(src);
        }
        if (have) {
          result.seq = ++seqCounter;
          stateAdd(target, result);
        }
      }
    }
    if (resultWindow == newWindow && !anyMerge) mwsPut(windows, resultWindow, resultWindow);
    return resultWindow;
  }
  // MergingWindowSet.windows.put / remove, with the put's position in the HashMap's insertion order
  void mwsPut(std::map<TimeWindow, TimeWindow>& windows, const TimeWindow& w, const TimeWindow& sw) {
    windows.erase(w);
    windows[w] = sw;
    putSeq[curKey][w] = ++seqCounter;
  }
  void mwsErase(std::map<TimeWindow, TimeWindow>& windows, const TimeWindow w) {
    windows.erase(w);
    auto it = putSeq.find(curKey);
    if (it != putSeq.end()) it->second.erase(w);
  }
  // WindowOperator.getMergingWindowSet (:445-460): the key's set, created on first use from its
  // "merging-window-set" list state (puts in list order), which is then cleared
  std::map<TimeWindow, TimeWindow>& getMergingWindowSet() {
    auto it = mergingWindowsByKey.find(curKey);
    if (it != mergingWindowsByKey.end()) return it->second;
    mwsTable = true;
    auto& windows = mergingWindowsByKey[curKey];
    mwsSeq[curKey] = ++seqCounter;
    if (curKeyGroup >= cfg.kg_start && curKeyGroup <= cfg.kg_end) {
      auto& heap = mwsHeap[(size_t)(curKeyGroup - cfg.kg_start)];
      auto h = heap.find(curKey);
      if (h != heap.end()) {
        for (const auto& p : h->second.list) mwsPut(windows, p.first, p.second);
        heap.erase(h);
      }
    }
    return windows;
  }

  int processElementMerging(const Acc& value, int64_t ts) {  // WindowOperator.java:228-301
    const TimeWindow window{ts, jlong_add(ts, cfg.size)};   // EventTimeSessionWindows.assignWindows :53-56
    auto& windows = getMergingWindowSet();
    const TimeWindow actualWindow = addWindow(windows, window);
    if (isLate(actualWindow)) {   // :265-269
      mwsErase(windows, actualWindow);
      stats.records_late++;
      return FW_OK;
    }
    auto sw = windows.find(actualWindow);
    if (sw == windows.end()) { err = "Window is not in in-flight window set."; return FW_ERR_INVALID_ARG; }
    const TimeWindow stateWindow = sw->second;
    int rc = stateAdd(stateWindow, value);
    if (rc) return rc;
    // onElement on the (possibly merged) window, merged with the merge's CONTINUE
    TriggerResult triggerResult = triggerOnElement(actualWindow);
    if (isFire(triggerResult)) {
      const Acc* contents = stateGet(stateWindow);
      if (contents == nullptr) return FW_OK;
      Acc copy = *contents;
      fire(actualWindow, copy);
      stats.late_fires++;
    }
    if (isPurge(triggerResult)) cleanupMerging(actualWindow, stateWindow, windows);
    else registerCleanupTimer(actualWindow);
    return FW_OK;
  }
  void cleanupMerging(const TimeWindow& w, const TimeWindow& stateWindow, std::map<TimeWindow, TimeWindow>& windows) {
    stateClear(stateWindow);   // :420-428
    mwsErase(windows, w);      // MergingWindowSet.retireWindow
    triggerClear(w);
  }

  // ---- OneInputStreamOperator.processElement ----
  int processElement(int64_t key, int32_t keyHash, int64_t f1, int64_t ts, int64_t vi, double vd) {
    if (cfg.assigner == FW_SESSION) {   // (EventTimeSessionWindows has no Long.MIN_VALUE check: [ts, ts + gap))
      curKey = key;
      curKeyGroup = computeKeyGroupForKeyHash(keyHash, cfg.max_parallelism);
      stats.records_in++;
      Acc value{};
      value.key = key;
      value.f1 = f1;
      value.sum_i = value.min_i = value.max_i = vi;
      value.sum_d = value.min_d = value.max_d = vd;
      value.count = 1;
      value.seq = ++seqCounter;
      return processElementMerging(value, ts);
    }
    std::vector<TimeWindow> elementWindows;
    int rc = assignWindows(ts, elementWindows);
    if (rc) return rc;
    // setKeyContextElement1 -> AbstractKeyedStateBackend.setCurrentKey :167-170
    curKey = key;
    curKeyGroup = computeKeyGroupForKeyHash(keyHash, cfg.max_parallelism);
    stats.records_in++;
    Acc value{};
    value.key = key;
    value.f1 = f1;
    value.sum_i = value.min_i = value.max_i = vi;
    value.sum_d = value.min_d = value.max_d = vd;
    value.count = 1;
    value.seq = ++seqCounter;
    for (const TimeWindow& window : elementWindows) {  // :302-333
      if (isLate(window)) { stats.records_late++; continue; }
      rc = stateAdd(window, value);
      if (rc) return rc;
      TriggerResult triggerResult = triggerOnElement(window);
      if (isFire(triggerResult)) {
        const Acc* contents = stateGet(window);
        if (contents == nullptr) continue;
        Acc copy = *contents;
        fire(window, copy);
        stats.late_fires++;
      }
      if (isPurge(triggerResult)) cleanup(window);
      else registerCleanupTimer(window);
    }
    return FW_OK;
  }

  // ---- WindowOperator.onEventTime :336-375 ----
  void onEventTime(const InternalTimer& timer) {
    curKey = timer.key;
    const TimeWindow& window = timer.ns;
    if (cfg.assigner == FW_SESSION) {   // :344-353: the state lives in the window's state window
      auto& windows = getMergingWindowSet();
      auto sw = windows.find(window);
      if (sw == windows.end()) return;   // already purged: a leftover cleanup timer
      const TimeWindow stateWindow = sw->second;
      const Acc* c = stateGet(stateWindow);
      if (c == nullptr) return;
      Acc contents = *c;
      TriggerResult triggerResult = triggerOnEventTime(window, timer.timestamp);
      if (isFire(triggerResult)) fire(window, contents);
      if (isPurge(triggerResult) || isCleanupTime(window, timer.timestamp)) cleanupMerging(window, stateWindow, windows);
      return;
    }
    const Acc* c = stateGet(window);
    if (c == nullptr) return;
    Acc contents = *c;
    TriggerResult triggerResult = triggerOnEventTime(window, timer.timestamp);
    if (isFire(triggerResult)) fire(window, contents);
    if (isPurge(triggerResult) || isCleanupTime(window, timer.timestamp)) cleanup(window);
  }

  // ---- AbstractStreamOperator.processWatermark :803-808 -> advanceWatermark :264-278 ----
  void processWatermark(int64_t time) {
    currentWatermark = time;
    while (!timers.empty() && timers.begin()->timestamp <= time) {
      InternalTimer timer = *timers.begin();
      timers.erase(timers.begin());
      timerSeq.erase(timer);
      curKeyGroup = computeKeyGroupForKeyHash(keyHashOf(timer.key), cfg.max_parallelism);
      onEventTime(timer);
    }
    mark_wm.push_back(time);
    mark_pos.push_back((int64_t)out.size());
  }

  // key -> key.hashCode(), remembered from processElement for keys that came with an explicit hash
  std::unordered_map<int64_t, int32_t> explicitHash;
  int32_t keyHashOf(int64_t key) const {
    auto it = explicitHash.find(key);
    return it == explicitHash.end() ? longHashCode(key) : it->second;
  }
};


// ---------------- checkpoint of one key group, in the reference's byte layout ----------------
// DataOutputStream big-endian primitives (writeByte/Short/Int/Long, writeDouble = doubleToLongBits)
struct JavaOut {
  std::vector<uint8_t> b;
  void writeByte(int v) { b.push_back((uint8_t)v); }
  void writeShort(int v) { writeByte((v >> 8) & 0xff); writeByte(v & 0xff); }
  void writeInt(int32_t v) { for (int s = 24; s >= 0; s -= 8) writeByte((int)(((uint32_t)v >> s) & 0xff)); }
  void writeLong(int64_t v) { for (int s = 56; s >= 0; s -= 8) writeByte((int)(((uint64_t)v >> s) & 0xff)); }
  void writeDouble(double d) {
    int64_t bits;
    if (d != d) bits = 0x7ff8000000000000ll;   // Double.doubleToLongBits: the canonical NaN
    else std::memcpy(&bits, &d, 8);
    writeLong(bits);
  }
};
struct JavaIn {
  const uint8_t* p;
  int64_t n, pos = 0;
  bool eof = false;
  uint64_t read(int k) {
    if (pos + k > n) { eof = true; pos = n; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) v = (v << 8) | p[pos + i];
    pos += k;
    return v;
  }
  int readByte() { return (int)(int8_t)read(1); }
  int readShort() { return (int)(int16_t)read(2); }
  int32_t readInt() { return (int32_t)read(4); }
  int64_t readLong() { return (int64_t)read(8); }
};

// java.util.HashMap iteration: bucket (h ^ h >>> 16) & (capacity - 1) in index order, each bucket's chain
// in insertion order.  Capacity: 16, doubled on a put that makes size > 0.75 capacity.  The JVM table
// never shrinks; this restatement sizes it by the current entry count (parity unpinned where a table
// once held more entries — no JVM here to run the reference).
int32_t hmHash(int32_t h) { return h ^ ushr32(h, 16); }
uint32_t hmCapacity(size_t n) {
  uint32_t cap = 16;
  while ((double)n > cap * 0.75) cap <<= 1;
  return cap;
}
template <class T>
void hmOrder(std::vector<T>& v, int32_t (*hashOf)(const T&), int64_t (*seqOf)(const T&)) {
  const uint32_t mask = hmCapacity(v.size()) - 1;
  std::sort(v.begin(), v.end(), [&](const T& a, const T& b) {
    const uint32_t ia = (uint32_t)hmHash(hashOf(a)) & mask, ib = (uint32_t)hmHash(hashOf(b)) & mask;
    return ia != ib ? ia < ib : seqOf(a) < seqOf(b);
  });
}
int32_t timeWindowHashCode(const TimeWindow& w) {  // TimeWindow.hashCode :79-83
  return jint_add(jint_mul(longHashCode(w.start), 31), longHashCode(w.end));
}
int32_t timerHashCode(const InternalTimer& t) {    // InternalTimer.hashCode :81-86
  int32_t r = longHashCode(t.timestamp);
  r = jint_add(jint_mul(r, 31), longHashCode(t.key));
  return jint_add(jint_mul(r, 31), timeWindowHashCode(t.ns));
}

// the state tuple's fields (the ReduceFunction's value type) from / into the accumulator
void writeField(const fw_config& c, JavaOut& o, int f, const Acc& a) {
  const bool d = c.value_type == FW_VALUE_F64;
  switch (f) {
    case FW_SF_KEY: o.writeLong(a.key); break;
    case FW_SF_F1: o.writeLong(a.f1); break;
    case FW_SF_SUM: if (d) o.writeDouble(a.sum_d); else o.writeLong(a.sum_i); break;
    case FW_SF_MIN: if (d) o.writeDouble(a.min_d); else o.writeLong(a.min_i); break;
    case FW_SF_MAX: case FW_SF_VALUE: if (d) o.writeDouble(a.max_d); else o.writeLong(a.max_i); break;
    case FW_SF_COUNT: o.writeLong(a.count); break;
  }
}
void readField(const fw_config& c, JavaIn& in, int f, Acc& a) {
  const int64_t x = in.readLong();
  double d;
  std::memcpy(&d, &x, 8);
  switch (f) {
    case FW_SF_KEY: a.key = x; break;
    case FW_SF_F1: a.f1 = x; break;
    case FW_SF_SUM: a.sum_i = x; a.sum_d = d; break;
    case FW_SF_MIN: a.min_i = x; a.min_d = d; break;
    case FW_SF_MAX: a.max_i = x; a.max_d = d; break;
    case FW_SF_COUNT: a.count = x; break;
    case FW_SF_VALUE: a.sum_i = a.min_i = a.max_i = x; a.sum_d = a.min_d = a.max_d = d; break;
  }
  (void)c;
}

// a list-state element (the window's input record: key, f1, value fields in the element tuple's order)
void writeListField(const fw_config& c, JavaOut& o, int f, int64_t key, const ListElem& x) {
  switch (f) {
    case FW_SF_KEY: o.writeLong(key); break;
    case FW_SF_F1: o.writeLong(x.f1); break;
    case FW_SF_VALUE: if (c.value_type == FW_VALUE_F64) o.writeDouble(x.vd); else o.writeLong(x.vi); break;
  }
}

struct NsRef { TimeWindow w; int64_t seq; const std::unordered_map<int64_t, Acc>* entries; };
struct EntRef { int64_t key; const Acc* acc; };
struct TimerRef { InternalTimer t; int64_t seq; };
int32_t nsHash(const NsRef& r) { return timeWindowHashCode(r.w); }
int64_t nsSeqOf(const NsRef& r) { return r.seq; }
int32_t entHash(const EntRef& r) { return longHashCode(r.key); }
int64_t entSeqOf(const EntRef& r) { return r.acc->seq; }
int32_t tmHash(const TimerRef& r) { return timerHashCode(r.t); }
int64_t tmSeqOf(const TimerRef& r) { return r.seq; }

// WindowOperator.snapshotState (:724-736) for the keys of key group kg: in mergingWindowsByKey's iteration
// order (a HashMap<K, MergingWindowSet>), each key's "merging-window-set" entry cleared and rewritten by
// MergingWindowSet.persist (:91-95: the windows HashMap's entries in its iteration order; an empty set
// writes none)
void persistMergingWindows(Operator& op, int32_t kg) {
  const size_t kgi = (size_t)(kg - op.cfg.kg_start);
  std::vector<int64_t> keys;
  for (const auto& kv : op.mergingWindowsByKey) keys.push_back(kv.first);
  const uint32_t gmask = hmCapacity(keys.size()) - 1;
  std::sort(keys.begin(), keys.end(), [&](int64_t a, int64_t b) {
    const uint32_t ia = (uint32_t)hmHash(longHashCode(a)) & gmask, ib = (uint32_t)hmHash(longHashCode(b)) & gmask;
    return ia != ib ? ia < ib : op.mwsSeq.at(a) < op.mwsSeq.at(b);
  });
  auto& heap = op.mwsHeap[kgi];
  for (int64_t k : keys) {
    if (computeKeyGroupForKeyHash(op.keyHashOf(k), op.cfg.max_parallelism) != kg) continue;
    heap.erase(k);   // mergeState.clear()
    const auto& windows = op.mergingWindowsByKey.at(k);
    if (windows.empty()) continue;
    const auto& ps = op.putSeq.at(k);
    std::vector<std::pair<TimeWindow, TimeWindow>> v(windows.begin(), windows.end());
    const uint32_t wmask = hmCapacity(v.size()) - 1;
    std::sort(v.begin(), v.end(), [&](const auto& a, const auto& b) {
      const uint32_t ia = (uint32_t)hmHash(timeWindowHashCode(a.first)) & wmask;
      const uint32_t ib = (uint32_t)hmHash(timeWindowHashCode(b.first)) & wmask;
      return ia != ib ? ia < ib : ps.at(a.first) < ps.at(b.first);
    });
    heap[k] = Operator::MwsEntry{++op.seqCounter, v};   // mergeState.add per entry (HeapListState.add)
    op.mwsKgCreated[kgi] = 1;
  }
}

// the "merging-window-set" table of key group kg: ListState<Tuple2<W, W>> in VoidNamespace
// (writeStateTableForKeyGroup; VoidNamespaceSerializer: one byte; ArrayListSerializer: int size, then the
// elements; TupleSerializer of two TimeWindow.Serializer: start, end of the window, then of its state window)
void writeMergingWindowTable(const Operator& op, size_t kgi, JavaOut& st) {
  if (!op.mwsKgCreated[kgi]) { st.writeByte(0); return; }
  st.writeByte(1);
  const auto& heap = op.mwsHeap[kgi];
  st.writeInt(heap.empty() ? 0 : 1);
  if (heap.empty()) return;
  st.writeByte(0);
  std::vector<std::pair<int64_t, const Operator::MwsEntry*>> ent;
  for (const auto& kv : heap) ent.push_back({kv.first, &kv.second});
  const uint32_t mask = hmCapacity(ent.size()) - 1;
  std::sort(ent.begin(), ent.end(), [&](const auto& a, const auto& b) {
    const uint32_t ia = (uint32_t)hmHash(longHashCode(a.first)) & mask, ib = (uint32_t)hmHash(longHashCode(b.first)) & mask;
    return ia != ib ? ia < ib : a.second->seq < b.second->seq;
  });
  st.writeInt((int32_t)ent.size());
  for (const auto& x : ent) {
    st.writeLong(x.first);
    st.writeInt((int32_t)x.second->list.size());
    for (const auto& w : x.second->list) {
      st.writeLong(w.first.start);
      st.writeLong(w.first.end);
      st.writeLong(w.second.start);
      st.writeLong(w.second.end);
    }
  }
}

// HeapKeyedStateBackend.snapshot's key-group section (:196-212) + writeStateTableForKeyGroup (:217-248), and
// HeapInternalTimerService.snapshotTimersForKeyGroup (:285-310) after its serializer records.  The state
// tables in stateTables' HashMap order: "window-contents" (bucket 12 of 16), then session windows'
// "merging-window-set" (bucket 15); each key group lists every table, under its kVStateToId
void snapshotKeyGroup(Operator& op, int32_t kg, const fw_state_layout& L, JavaOut& st, JavaOut& tm) {
  const size_t kgi = (size_t)(kg - op.cfg.kg_start);
  const bool session = op.cfg.assigner == FW_SESSION;
  if (session) persistMergingWindows(op, kg);
  if (op.anyState || (session && op.mwsTable)) st.writeInt(kg);
  int nextId = 0;
  if (op.anyState) {
    st.writeShort(nextId++);   // kVStateToId of "window-contents"
    if (!op.kgCreated[kgi]) {
      st.writeByte(0);
    } else {
      st.writeByte(1);
      const auto& nsMap = op.state[kgi];
      std::vector<NsRef> ns;
      for (const auto& kv : nsMap) ns.push_back({kv.first, op.nsSeq[kgi].at(kv.first), &kv.second});
      hmOrder(ns, nsHash, nsSeqOf);
      st.writeInt((int32_t)ns.size());
      for (const NsRef& n : ns) {
        st.writeLong(n.w.start);   // TimeWindow.Serializer.serialize :141-144
        st.writeLong(n.w.end);
        std::vector<EntRef> ent;
        for (const auto& kv : *n.entries) ent.push_back({kv.first, &kv.second});
        hmOrder(ent, entHash, entSeqOf);
        st.writeInt((int32_t)ent.size());
        for (const EntRef& x : ent) {
          st.writeLong(x.key);     // LongSerializer (Tuple1<Long>: TupleSerializer over it, the same 8 bytes)
          if (op.cfg.agg_mask == FW_AGG_LIST) {   // ListSerializer.serialize: int size, then every element
            st.writeInt((int32_t)x.acc->list->size());
            for (const ListElem& el : *x.acc->list)
              for (int f = 0; f < L.n_fields; ++f) writeListField(op.cfg, st, L.field[f], x.key, el);
            continue;
          }
          for (int f = 0; f < L.n_fields; ++f) writeField(op.cfg, st, L.field[f], *x.acc);
        }
      }
    }
  }
  if (session && op.mwsTable) {
    st.writeShort(nextId++);
    writeMergingWindowTable(op, kgi, st);
  }
  std::vector<TimerRef> ts;
  for (const auto& kv : op.timerSeq)
    if (computeKeyGroupForKeyHash(op.keyHashOf(kv.first.key), op.cfg.max_parallelism) == kg) ts.push_back({kv.first, kv.second});
  hmOrder(ts, tmHash, tmSeqOf);
  tm.writeInt((int32_t)ts.size());
  for (const TimerRef& t : ts) {   // TimerSerializer.serialize: key, namespace, timestamp
    tm.writeLong(t.t.key);
    tm.writeLong(t.t.ns.start);
    tm.writeLong(t.t.ns.end);
    tm.writeLong(t.t.timestamp);
  }
  tm.writeInt(0);   // processing-time timers
}

// readStateTableForKeyGroup (:318-349) + restoreTimersForKeyGroup (:319-345); the timer service restarts at
// `wm` (the reference: Long.MIN_VALUE, its initial currentWatermark)
int restoreKeyGroup(Operator& op, int32_t kg, const fw_state_layout& L, int64_t wm, const uint8_t* st, int64_t sn,
                    const uint8_t* tb, int64_t tn) {
  if (kg < op.cfg.kg_start || kg > op.cfg.kg_end) {
    op.err = "Key Group " + std::to_string(kg) + " does not belong to the local range.";
    return FW_ERR_INVALID_ARG;
  }
  const size_t kgi = (size_t)(kg - op.cfg.kg_start);
  if (sn > 0) {
    JavaIn in{st, sn};
    const bool session = op.cfg.assigner == FW_SESSION;
    const int32_t written = in.readInt();
    if (written != kg) { op.err = "bad key-group section"; return FW_ERR_INVALID_ARG; }
    int tables = 0;
    for (int table = 0; !in.eof && (table == 0 || in.pos < sn); ++table, ++tables) {
    const int stateId = in.readShort();
    const int present = in.readByte();
    if (stateId != table || table > (session ? 1 : 0)) { op.err = "bad key-group section"; return FW_ERR_INVALID_ARG; }
    if (table == 1) {   // session windows' "merging-window-set": per key its (window, state window) list
      op.mwsTable = true;
      if (!present) continue;
      op.mwsKgCreated[kgi] = 1;
      const int32_t nns = in.readInt();
      if (nns < 0 || nns > 1) { op.err = "bad merging-window-set section"; return FW_ERR_INVALID_ARG; }
      if (nns == 0) continue;
      if (in.readByte() != 0) { op.err = "bad merging-window-set namespace"; return FW_ERR_INVALID_ARG; }
      const int32_t ne = in.readInt();
      for (int32_t j = 0; j < ne && !in.eof; ++j) {
        const int64_t key = in.readLong();
        const int32_t m = in.readInt();
        if (m < 0) { op.err = "corrupt merging-window-set entry"; return FW_ERR_INVALID_ARG; }
        Operator::MwsEntry me{++op.seqCounter, {}};
        for (int32_t q = 0; q < m && !in.eof; ++q) {
          TimeWindow w, sw;
          w.start = in.readLong();
          w.end = in.readLong();
          sw.start = in.readLong();
          sw.end = in.readLong();
          me.list.push_back({w, sw});
        }
        op.mwsHeap[kgi][key] = me;
      }
      continue;
    }
    if (session) op.anyState = true;   // (the table exists: a session checkpoint lists both)
    if (present) {
      op.kgCreated[kgi] = 1;
      op.anyState = true;
      auto& nsMap = op.state[kgi];
      const int32_t numNamespaces = in.readInt();
      for (int32_t k = 0; k < numNamespaces && !in.eof; ++k) {
        TimeWindow w;
        w.start = in.readLong();
        w.end = in.readLong();
        auto& entries = nsMap[w];
        op.nsSeq[kgi][w] = ++op.seqCounter;
        const int32_t numEntries = in.readInt();
        for (int32_t l = 0; l < numEntries && !in.eof; ++l) {
          Acc a{};
          a.key = in.readLong();
          const int64_t mapKey = a.key;
          if (op.cfg.agg_mask == FW_AGG_LIST) {   // ListSerializer.deserialize
            const int32_t ne = in.readInt();
            if (ne < 0) { op.err = "corrupt list state"; return FW_ERR_INVALID_ARG; }
            a.list = std::make_shared<std::vector<ListElem>>();
            for (int32_t q = 0; q < ne && !in.eof; ++q) {
              ListElem el{0, 0.0, 0};
              for (int f = 0; f < L.n_fields; ++f) {
                const int64_t x = in.readLong();
                if (L.field[f] == FW_SF_F1) el.f1 = x;
                if (L.field[f] == FW_SF_VALUE) { el.vi = x; std::memcpy(&el.vd, &x, 8); }
              }
              a.list->push_back(el);
            }
          } else {
            for (int f = 0; f < L.n_fields; ++f) readField(op.cfg, in, L.field[f], a);
          }
          a.seq = ++op.seqCounter;
          entries[mapKey] = a;
        }
      }
    }
    }
    if (in.eof || in.pos != sn || tables == 0) { op.err = "state section truncated or with trailing bytes"; return FW_ERR_INVALID_ARG; }
  }
  JavaIn in{tb, tn};
  const int32_t n = in.readInt();
  for (int32_t i = 0; i < n && !in.eof; ++i) {
    InternalTimer t;
    t.key = in.readLong();
    t.ns.start = in.readLong();
    t.ns.end = in.readLong();
    t.timestamp = in.readLong();
    if (op.timers.insert(t).second) op.timerSeq[t] = ++op.seqCounter;
  }
  const int32_t np = in.readInt();
  if (in.eof || in.pos != tn || np != 0) { op.err = "bad timer section"; return FW_ERR_INVALID_ARG; }
  op.currentWatermark = wm;
  return FW_OK;
}

}  // namespace

struct fw_engine {
  Operator op;
  explicit fw_engine(const fw_config& c) : op(c) {}
};

extern "C" {

int fwo_create(const fw_config* cfg, fw_engine** out) {
  if (!cfg || !out) return FW_ERR_INVALID_ARG;
  if (cfg->assigner != FW_TUMBLING && cfg->assigner != FW_SLIDING && cfg->assigner != FW_SESSION) return FW_ERR_INVALID_ARG;
  if ((cfg->agg_flags & FW_AGGF_FOLD) && cfg->assigner == FW_SESSION) return FW_ERR_UNSUPPORTED;   // WindowedStream.java:466-467
  if ((cfg->agg_mask & FW_AGG_LIST) && (cfg->agg_mask != FW_AGG_LIST || (cfg->agg_flags & FW_AGGF_FOLD)))
    return FW_ERR_UNSUPPORTED;   // list state: alone
  if (cfg->size <= 0 || (cfg->assigner == FW_SLIDING && cfg->slide <= 0) || cfg->allowed_lateness < 0 ||
      cfg->max_parallelism <= 0 || cfg->kg_start < 0 || cfg->kg_end < cfg->kg_start || cfg->kg_end >= cfg->max_parallelism)
    return FW_ERR_INVALID_ARG;
  *out = new fw_engine(*cfg);
  return FW_OK;
}

// processElement for each record, in order (one StreamInputProcessor pass)
int fwo_push_batch(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1, const int64_t* ts,
                   const void* value, int64_t n) {
  Operator& op = e->op;
  for (int64_t i = 0; i < n; ++i) {
    int32_t h = key_hash ? key_hash[i] : longHashCode(key[i]);
    if (key_hash) op.explicitHash[key[i]] = h;
    int64_t vi = 0;
    double vd = 0.0;
    if (op.cfg.value_type == FW_VALUE_I64) vi = ((const int64_t*)value)[i];
    else vd = ((const double*)value)[i];
    int rc = op.processElement(key[i], h, f1 ? f1[i] : ts[i], ts[i], vi, vd);
    if (rc) return rc;
  }
  return FW_OK;
}

int fwo_advance_watermark(fw_engine* e, int64_t wm) {
  e->op.processWatermark(wm);
  return FW_OK;
}

int fwo_collect(fw_engine* e, fw_out* o) {
  Operator& op = e->op;
  size_t n = op.out.size();
  op.c_key.resize(n); op.c_f1.resize(n); op.c_ts.resize(n);
  op.c_sum_i.resize(n); op.c_min_i.resize(n); op.c_max_i.resize(n); op.c_count.resize(n);
  op.c_sum_d.resize(n); op.c_min_d.resize(n); op.c_max_d.resize(n); op.c_start.resize(n);
  for (size_t i = 0; i < n; ++i) {
    const Acc& a = op.out[i].acc;
    op.c_start[i] = op.out[i].start;
    op.c_key[i] = a.key; op.c_f1[i] = a.f1; op.c_ts[i] = op.out[i].ts;
    op.c_sum_i[i] = a.sum_i; op.c_min_i[i] = a.min_i; op.c_max_i[i] = a.max_i; op.c_count[i] = a.count;
    op.c_sum_d[i] = a.sum_d; op.c_min_d[i] = a.min_d; op.c_max_d[i] = a.max_d;
  }
  std::memset(o, 0, sizeof(*o));
  o->n = (int64_t)n;
  o->key = op.c_key.data();
  o->f1 = op.c_f1.data();
  o->ts = op.c_ts.data();
  o->sum_i64 = op.c_sum_i.data(); o->min_i64 = op.c_min_i.data(); o->max_i64 = op.c_max_i.data();
  o->count = op.c_count.data();
  o->sum_f64 = op.c_sum_d.data(); o->min_f64 = op.c_min_d.data(); o->max_f64 = op.c_max_d.data();
  o->n_marks = (int64_t)op.mark_wm.size();
  o->mark_wm = op.mark_wm.data();
  o->mark_pos = op.mark_pos.data();
  o->win_start = op.cfg.assigner == FW_SESSION ? op.c_start.data() : nullptr;
  return FW_OK;
}

// drop collected output (keeps operator state)
int fwo_clear_output(fw_engine* e) {
  e->op.out.clear();
  e->op.mark_wm.clear();
  e->op.mark_pos.clear();
  return FW_OK;
}

int fwo_get_stats(fw_engine* e, fw_stats* st) {
  *st = e->op.stats;
  size_t keys = 0;
  for (auto& m : e->op.state) for (auto& kv : m) keys += kv.second.size();
  st->keys_resident = (int64_t)keys;
  st->ingest_form = 0;
  return FW_OK;
}

int fwo_snapshot_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, void* state, int64_t state_cap,
                          int64_t* state_len, void* timers, int64_t timers_cap, int64_t* timers_len) {
  if (!e || !layout || !state_len || !timers_len) return FW_ERR_INVALID_ARG;
  if (kg < e->op.cfg.kg_start || kg > e->op.cfg.kg_end) return FW_ERR_INVALID_ARG;
  JavaOut st, tm;
  snapshotKeyGroup(e->op, kg, *layout, st, tm);
  *state_len = (int64_t)st.b.size();
  *timers_len = (int64_t)tm.b.size();
  if (!state && !timers) return FW_OK;
  if (!state || !timers || state_cap < *state_len || timers_cap < *timers_len) return FW_ERR_CAPACITY;
  if (!st.b.empty()) std::memcpy(state, st.b.data(), st.b.size());
  std::memcpy(timers, tm.b.data(), tm.b.size());
  return FW_OK;
}

int fwo_restore_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, int64_t watermark, const void* state,
                         int64_t state_len, const void* timers, int64_t timers_len) {
  if (!e || !layout || !timers) return FW_ERR_INVALID_ARG;
  return restoreKeyGroup(e->op, kg, *layout, watermark, (const uint8_t*)state, state_len, (const uint8_t*)timers,
                         timers_len);
}

// the receiving side of one channel, element after element: length, tag, then the element's fields
// (DataInputDeserializer reads big-endian).  Outputs are host arrays here.
int fwo_decode(fw_engine* e, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes, int32_t mem, int64_t* key,
               int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap, int64_t* wm,
               int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap, fw_decode_counts* out) {
  (void)e; (void)mem;
  std::memset(out, 0, sizeof(*out));
  std::vector<int> off(sc->n_fields + 1, 0);
  for (int i = 0; i < sc->n_fields; ++i) off[i + 1] = off[i] + (sc->field_type[i] == FW_FT_INT ? 4 : 8);
  const int tupleBytes = off[sc->n_fields];
  JavaIn in{(const uint8_t*)bytes, nbytes};
  int64_t nr = 0, nw = 0, nl = 0;
  auto field = [&](const uint8_t* t, int i) -> int64_t {
    JavaIn f{t + off[i], 8};
    return sc->field_type[i] == FW_FT_INT ? (int64_t)f.readInt() : f.readLong();
  };
  while (in.pos + 4 <= nbytes) {
    const int64_t at = in.pos;
    const int32_t len = in.readInt();
    if (len < 1 || at + 4 + len > nbytes) { in.pos = at; break; }   // the rest spans into the next buffer
    const uint8_t* el = (const uint8_t*)bytes + at + 4;
    const int tag = (int)(int8_t)el[0];
    if (tag == 0 || tag == 1) {   // StreamRecord with / without timestamp
      if (len != (tag == 0 ? 9 : 1) + tupleBytes) return FW_ERR_INVALID_ARG;
      if (nr >= record_cap) return FW_ERR_CAPACITY;
      JavaIn r{el + 1, 8};
      const int64_t t = tag == 0 ? r.readLong() : INT64_MIN;
      const uint8_t* tuple = el + (tag == 0 ? 9 : 1);
      key[nr] = field(tuple, sc->key_field);
      if (key_hash) key_hash[nr] = (int32_t)key[nr];   // Integer.hashCode
      ts[nr] = t;
      f1[nr] = sc->f1_field < 0 ? t : field(tuple, sc->f1_field);
      ((int64_t*)value)[nr] = field(tuple, sc->value_field);   // long, or the double's bits
      ++nr;
    } else if (tag == 2) {        // Watermark
      if (len != 9) return FW_ERR_INVALID_ARG;
      if (nw >= marker_cap) return FW_ERR_CAPACITY;
      JavaIn r{el + 1, 8};
      wm[nw] = r.readLong();
      wm_pos[nw] = nr;
      ++nw;
    } else if (tag == 3) {        // LatencyMarker(markedTime, vertexId, subtaskIndex)
      if (len != 17) return FW_ERR_INVALID_ARG;
      if (nl >= marker_cap) return FW_ERR_CAPACITY;
      JavaIn r{el + 1, 16};
      lm[2 * nl] = r.readLong();
      const uint32_t v = (uint32_t)r.readInt(), sidx = (uint32_t)r.readInt();
      lm[2 * nl + 1] = (int64_t)(((uint64_t)v << 32) | sidx);
      lm_pos[nl] = nr;
      ++nl;
    } else {
      return FW_ERR_INVALID_ARG;  // "Corrupt stream, found tag: " (StreamElementSerializer.java:196)
    }
    in.pos = at + 4 + len;
  }
  out->n_records = nr;
  out->n_watermarks = nw;
  out->n_latency_markers = nl;
  out->consumed = in.pos;
  return FW_OK;
}

const char* fwo_last_error(const fw_engine* e) { return e ? e->op.err.c_str() : "null engine"; }
void fwo_destroy(fw_engine* e) { delete e; }

// pure functions exported for golden-vector tests
int32_t fwo_murmur_hash(int32_t code) { return murmurHash(code); }
int32_t fwo_long_hash_code(int64_t v) { return longHashCode(v); }
int32_t fwo_key_group(int32_t key_hash, int32_t max_parallelism) { return computeKeyGroupForKeyHash(key_hash, max_parallelism); }
int32_t fwo_operator_index(int32_t max_parallelism, int32_t parallelism, int32_t kg) {
  return computeOperatorIndexForKeyGroup(max_parallelism, parallelism, kg);
}
// KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex :78-89
void fwo_key_group_range(int32_t max_parallelism, int32_t parallelism, int32_t op_index, int32_t* start, int32_t* end) {
  *start = op_index == 0 ? 0 : ((op_index * max_parallelism - 1) / parallelism) + 1;
  *end = ((op_index + 1) * max_parallelism - 1) / parallelism;
}
int64_t fwo_window_start(int64_t ts, int64_t offset, int64_t size) { return getWindowStartWithOffset(ts, offset, size); }

// ---- parallel CPU job: p operator subtasks (one thread each) behind a KeyGroupStreamPartitioner.
// Each subtask owns computeKeyGroupRangeForOperatorIndex(mp, p, i) and sees the records routed to it
// (assignKeyToParallelOperator) in input order, plus every watermark (RecordWriter.broadcastEmit).
// Watermarks: after every `wm_every` records, wm = max ts seen so far - wm_lag; a final wm at the end.
// Returns total fired records; the per-subtask sum of f2 (or f64 sum) for a checksum.
int64_t fwo_run_parallel(const fw_config* cfg, int32_t parallelism, const int64_t* key, const int64_t* ts,
                         const void* value, int64_t n, int64_t wm_every, int64_t wm_lag, int64_t final_wm,
                         int64_t* checksum_out) {
  std::vector<int64_t> fired(parallelism, 0), csum(parallelism, 0);
  auto worker = [&](int32_t idx) {
    fw_config c = *cfg;
    fwo_key_group_range(cfg->max_parallelism, parallelism, idx, &c.kg_start, &c.kg_end);
    Operator op(c);
    int64_t maxTs = INT64_MIN;
    for (int64_t i = 0; i < n; ++i) {
      if (ts[i] > maxTs) maxTs = ts[i];
      int32_t h = longHashCode(key[i]);
      int32_t kg = computeKeyGroupForKeyHash(h, c.max_parallelism);
      if (computeOperatorIndexForKeyGroup(c.max_parallelism, parallelism, kg) == idx) {
        int64_t vi = 0; double vd = 0.0;
        if (c.value_type == FW_VALUE_I64) vi = ((const int64_t*)value)[i]; else vd = ((const double*)value)[i];
        op.processElement(key[i], h, ts[i], ts[i], vi, vd);
      }
      if (wm_every > 0 && (i + 1) % wm_every == 0) {
        op.processWatermark(jlong_sub(maxTs, wm_lag));
        for (auto& r : op.out) csum[idx] = jlong_add(csum[idx], c.value_type == FW_VALUE_I64 ? r.acc.sum_i : (int64_t)r.acc.count);
        fired[idx] += (int64_t)op.out.size();
        op.out.clear();
      }
    }
    op.processWatermark(final_wm);
    for (auto& r : op.out) csum[idx] = jlong_add(csum[idx], c.value_type == FW_VALUE_I64 ? r.acc.sum_i : (int64_t)r.acc.count);
    fired[idx] += (int64_t)op.out.size();
  };
  std::vector<std::thread> th;
  for (int32_t i = 0; i < parallelism; ++i) th.emplace_back(worker, i);
  for (auto& t : th) t.join();
  int64_t total = 0, cs = 0;
  for (int32_t i = 0; i < parallelism; ++i) { total += fired[i]; cs = jlong_add(cs, csum[i]); }
  if (checksum_out) *checksum_out = cs;
  return total;
}

}  // extern "C"
