// flink_kg_format.h — host-side codec of one key group of a Flink 1.2 WindowOperator checkpoint
// (SURVEY.md §8f.1), used by fw_snapshot_kg_flink / fw_restore_kg_flink.
//
//   state   what HeapKeyedStateBackend.snapshot writes at KeyGroupRangeOffsets[kg]
//           (flink-runtime/.../state/heap/HeapKeyedStateBackend.java:196-212, writeStateTableForKeyGroup
//           :217-248): int kg | short state id (0: "window-contents" is the operator's only keyed state,
//           WindowOperator.java:310-311) | byte present | int numNamespaces |
//           (TimeWindow: long start, long end (TimeWindow.Serializer, TimeWindow.java:141-144) |
//            int numEntries | (key, state tuple)*)*
//   timers  HeapInternalTimerService.snapshotTimersForKeyGroup (SJ/api/operators/HeapInternalTimerService.java
//           :285-310) after its two serializeObject records: int n | (key | start | end | long timestamp)*
//           (InternalTimer.TimerSerializer.serialize, InternalTimer.java:145-149) | int 0 processing timers
//
// Everything is big-endian (DataOutputStream).  Keys are Long / Tuple1<Long> (LongSerializer, 8 bytes);
// state tuple fields are LongSerializer / DoubleSerializer values (writeDouble = doubleToLongBits: one
// canonical NaN), in TupleSerializer field order (TupleSerializer.java:120-129).
//
// Iteration order.  The namespaces of a key group, the entries of a namespace and the timers of a key
// group live in java.util.HashMap / HashSet: iteration goes bucket by bucket, bucket = spread(hashCode) &
// (capacity - 1) with spread(h) = h ^ (h >>> 16), and within a bucket in insertion order (puts append to
// the bin's chain; a resize splits a chain without reordering it).  The capacity is 16, doubled while
// size > 3/4 capacity.  A JVM table never shrinks, so its capacity reflects the largest size it ever had;
// the codec sizes it by the current size (the two agree unless the table once held more entries, e.g. a
// timer set right before a watermark fired part of it).  Chains longer than 8 in a table of >= 64
// buckets become red-black trees in the JVM with a different order; not emulated.
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "java_semantics.h"

namespace fwkg {

struct BeOut {
  std::vector<uint8_t> b;
  void u8(uint32_t v) { b.push_back((uint8_t)v); }
  void i16(int32_t v) { u8((uint32_t)v >> 8); u8((uint32_t)v); }
  void i32(int32_t v) { for (int s = 24; s >= 0; s -= 8) u8((uint32_t)v >> s); }
  void i64(int64_t v) { for (int s = 56; s >= 0; s -= 8) u8((uint32_t)((uint64_t)v >> s)); }
  void f64(double d) {   // DataOutputStream.writeDouble: writeLong(Double.doubleToLongBits(d))
    int64_t x;
    if (d != d) x = 0x7ff8000000000000ll;
    else memcpy(&x, &d, 8);
    i64(x);
  }
};

struct BeIn {
  const uint8_t* p;
  int64_t n, pos = 0;
  bool ok = true;
  BeIn(const void* d, int64_t len) : p((const uint8_t*)d), n(len) {}
  uint64_t take(int k) {
    if (!ok || pos + k > n) { ok = false; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) v = (v << 8) | p[pos + i];
    pos += k;
    return v;
  }
  int32_t u8() { return (int32_t)take(1); }
  int32_t i16() { return (int32_t)(int16_t)take(2); }
  int32_t i32() { return (int32_t)take(4); }
  int64_t i64() { return (int64_t)take(8); }
  bool done() const { return ok && pos == n; }
};

// java.util.HashMap.hash(key) and the table capacity for `n` entries put into a new HashMap()
inline int32_t spread(int32_t h) { return (int32_t)((uint32_t)h ^ ((uint32_t)h >> 16)); }
inline uint32_t capacity_for(size_t n) {
  uint64_t c = 16;
  while (n > c / 4 * 3) c <<= 1;
  return (uint32_t)c;
}
inline int32_t jmul31(int32_t a) { return (int32_t)((uint32_t)a * 31u); }
inline int32_t jaddi(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
// TimeWindow.hashCode (TimeWindow.java:79-83)
inline int32_t window_hash(int64_t start, int64_t end) {
  return jaddi(jmul31(fw::long_hash_code(start)), fw::long_hash_code(end));
}
// InternalTimer.hashCode (InternalTimer.java:81-86) with key.hashCode = Long.hashCode
inline int32_t timer_hash(int64_t ts, int64_t key, int64_t start, int64_t end) {
  int32_t r = fw::long_hash_code(ts);
  r = jaddi(jmul31(r), fw::long_hash_code(key));
  return jaddi(jmul31(r), window_hash(start, end));
}

// Sort `idx` into HashMap iteration order: bucket of hash(i), then insertion rank(i) (a strict order).
template <class Hash, class Less>
void hashmap_order(std::vector<size_t>& idx, Hash hash, Less earlier) {
  const uint32_t mask = capacity_for(idx.size()) - 1;
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
    const uint32_t ba = (uint32_t)spread(hash(a)) & mask, bb = (uint32_t)spread(hash(b)) & mask;
    if (ba != bb) return ba < bb;
    return earlier(a, b);
  });
}

}  // namespace fwkg
