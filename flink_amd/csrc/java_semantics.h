// java_semantics.h — Java arithmetic the window path must reproduce bit for bit, on host and device.
//
// Each function cites the reference code it follows (paths relative to the reference root).
// Wrapping int32/int64 arithmetic is done in unsigned types; `>>>` is a logical shift; `%` truncates
// toward zero in both Java and C++.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fw {

#define FW_HD __host__ __device__ __forceinline__

FW_HD int32_t rotl32(uint32_t v, int r) { return (int32_t)((v << r) | (v >> (32 - r))); }

// MathUtils.murmurHash(int) — flink-core/src/main/java/org/apache/flink/util/MathUtils.java:134-158
FW_HD int32_t murmur_hash(int32_t code_in) {
  uint32_t c = (uint32_t)code_in;
  c *= 0xcc9e2d51u;
  c = (uint32_t)rotl32(c, 15);
  c *= 0x1b873593u;
  c = (uint32_t)rotl32(c, 13);
  c = c * 5u + 0xe6546b64u;
  c ^= 4u;
  c ^= c >> 16;
  c *= 0x85ebca6bu;
  c ^= c >> 13;
  c *= 0xc2b2ae35u;
  c ^= c >> 16;
  int32_t code = (int32_t)c;
  if (code >= 0) return code;
  if (code != INT32_MIN) return -code;
  return 0;
}

// JDK Long.hashCode(long) = (int)(value ^ (value >>> 32)); Tuple1.hashCode = f0.hashCode()
// (flink-core/src/main/java/org/apache/flink/api/java/tuple/Tuple1.java:137-139)
FW_HD int32_t long_hash_code(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32)); }

// KeyGroupRangeAssignment.computeKeyGroupForKeyHash — flink-runtime/.../state/KeyGroupRangeAssignment.java:62-64
FW_HD int32_t key_group_for_hash(int32_t key_hash, int32_t max_parallelism) {
  return murmur_hash(key_hash) % max_parallelism;
}
// KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup — :105-107
FW_HD int32_t operator_index_for_key_group(int32_t max_parallelism, int32_t parallelism, int32_t kg) {
  return kg * parallelism / max_parallelism;
}

FW_HD int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
FW_HD int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

// TimeWindow.getWindowStartWithOffset — flink-streaming-java/.../api/windowing/windows/TimeWindow.java:239-241
FW_HD int64_t window_start_with_offset(int64_t ts, int64_t offset, int64_t size) {
  int64_t num = jadd(jsub(ts, offset), size);
  return jsub(ts, num % size);
}

// WindowOperator.cleanupTime — flink-streaming-java/.../runtime/operators/windowing/WindowOperator.java:511-514
FW_HD int64_t cleanup_time(int64_t max_ts, int64_t allowed_lateness) {
  int64_t ct = jadd(max_ts, allowed_lateness);
  return ct >= max_ts ? ct : INT64_MAX;
}

// Java truncating division and remainder of x by a positive divisor d (x = q*d + r, r has x's sign).
// Exact; fast path through a double reciprocal when |x| < 2^52 (the 64-bit integer divide is a long
// instruction sequence on the GPU, kept out of line), fixed up by at most a couple of correction steps.
struct QR { int64_t q, r; };
__host__ __device__ __attribute__((noinline)) inline QR jdivmod_wide(int64_t x, int64_t d) { return QR{x / d, x % d}; }

FW_HD void jdivmod(int64_t x, int64_t d, double inv_d, int64_t& q, int64_t& r) {
  const int64_t lim = (int64_t)1 << 52;
  if (x > -lim && x < lim && d < lim) {
    int64_t qq = (int64_t)((double)x * inv_d);
    int64_t rr = x - qq * d;
    if (x >= 0) {
      while (rr < 0) { --qq; rr += d; }
      while (rr >= d) { ++qq; rr -= d; }
    } else {
      while (rr > 0) { ++qq; rr -= d; }
      while (rr <= -d) { --qq; rr += d; }
    }
    q = qq; r = rr;
    return;
  }
  const QR w = jdivmod_wide(x, d);
  q = w.q;
  r = w.r;
}

// jdivmod with the wide case inline (no call): for kernels whose register budget a call would spill
FW_HD void jdivmod_inl(int64_t x, int64_t d, double inv_d, int64_t& q, int64_t& r) {
  const int64_t lim = (int64_t)1 << 52;
  if (x > -lim && x < lim && d < lim) {
    jdivmod(x, d, inv_d, q, r);
    return;
  }
  q = x / d;
  r = x - q * d;
}

// floor division / modulo on int64 (slice numbering; not Java semantics, internal indexing)
FW_HD int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b, r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? q - 1 : q;
}
FW_HD int64_t floor_mod(int64_t a, int64_t b) {
  int64_t r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? r + b : r;
}

// Orderable 64-bit encoding of a double for JDK Math.min / Math.max (NaN wins, -0.0 < +0.0):
// integer order of the code equals the Math.min/max order; NaN maps to the extreme that wins.
FW_HD int64_t f64_min_code(double x) {
  if (x != x) return INT64_MIN;  // Math.min: NaN wins
  int64_t b; __builtin_memcpy(&b, &x, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
FW_HD int64_t f64_max_code(double x) {
  if (x != x) return INT64_MAX;  // Math.max: NaN wins
  int64_t b; __builtin_memcpy(&b, &x, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
// Orderable encoding for Double.compareTo (JDK: doubleToLongBits order — every NaN equal and above
// +inf, -0.0 < +0.0), the order of ComparableAggregator's Comparator (Comparator.java:45-105).  The NaN
// is canonicalised as doubleToLongBits does, so it decodes as the canonical quiet NaN.
FW_HD int64_t f64_cmp_code(double x) {
  int64_t b;
  if (x != x) b = 0x7ff8000000000000ll;
  else __builtin_memcpy(&b, &x, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
FW_HD double f64_from_code(int64_t c) {
  if (c == INT64_MIN || c == INT64_MAX) {  // a NaN won (canonical quiet NaN)
    uint64_t nan = 0x7ff8000000000000ull; double d; __builtin_memcpy(&d, &nan, 8); return d;
  }
  int64_t b = c >= 0 ? c : (c ^ INT64_MAX);
  double d; __builtin_memcpy(&d, &b, 8);
  return d;
}

}  // namespace fw
