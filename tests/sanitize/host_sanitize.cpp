// Host-code sanitizer driver (-fsanitize=address,undefined on host code; GPU sanitizers are not
// available on the pool).  Built by tests/test_host_sanitizers.py with g++ -fsanitize=address,undefined
// -fno-sanitize-recover=all together with oracle/fw_oracle.cpp (the CPU parity oracle: test infrastructure)
// and run as a plain process.  It drives
//   - the oracle through every window shape the engine offers: tumbling / sliding / session, reduce (sum,
//     min, max, count, doubles), allowed lateness with both triggers, fold, list state, maxBy, the
//     checkpoint writer and reader of the reference's byte layout (every key group snapshotted, restored
//     into a fresh oracle, snapshotted again: identical bytes), and the wire-format decoder (whole and cut
//     streams, a corrupt tag);
//   - flink_kg_format.h, the engine's host-side checkpoint codec: big-endian writer / reader round trips,
//     reads past the end (ok = false), HashMap iteration order over random tables.
// Any sanitizer report aborts with a non-zero status; the test asserts status 0.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/flink_window.h"
#include "../../flink_amd/csrc/flink_kg_format.h"

extern "C" {
int fwo_create(const fw_config* cfg, fw_engine** out);
int fwo_push_batch(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1, const int64_t* ts,
                   const void* value, int64_t n);
int fwo_advance_watermark(fw_engine* e, int64_t wm);
int fwo_collect(fw_engine* e, fw_out* o);
int fwo_get_stats(fw_engine* e, fw_stats* st);
int fwo_snapshot_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, void* state, int64_t state_cap,
                          int64_t* state_len, void* timers, int64_t timers_cap, int64_t* timers_len);
int fwo_restore_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, int64_t watermark, const void* state,
                         int64_t state_len, const void* timers, int64_t timers_len);
int fwo_decode(fw_engine* e, const fw_tuple_schema* sc, const void* bytes, int64_t nbytes, int32_t mem, int64_t* key,
               int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap, int64_t* wm,
               int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap, fw_decode_counts* out);
const char* fwo_last_error(const fw_engine* e);
void fwo_destroy(fw_engine* e);
}

static int failures = 0;
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); ++failures; } } while (0)

static uint64_t splitmix(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static fw_config base_config() {
  fw_config c;
  memset(&c, 0, sizeof(c));
  c.assigner = FW_TUMBLING;
  c.size = 1000;
  c.trigger = FW_TRIGGER_EVENT_TIME;
  c.value_type = FW_VALUE_I64;
  c.agg_mask = FW_AGG_SUM;
  c.keep_first_f1 = 1;
  c.max_parallelism = 128;
  c.kg_start = 0;
  c.kg_end = 127;
  c.key_capacity = 1 << 12;
  c.max_batch = 1 << 12;
  c.out_capacity = 1 << 18;
  return c;
}

// drive n records (keys < nk, ts advancing at rate per ms with out-of-order jitter) in batches, a watermark
// after each; returns fired records
static int64_t drive(fw_engine* e, int64_t n, int nk, int64_t t0, int ooo, bool f64, int64_t lag, uint64_t seed) {
  std::vector<int64_t> k(1024), t(1024), f1(1024), v(1024);
  int64_t fired = 0, max_ts = INT64_MIN;
  for (int64_t s = 0; s < n; s += 1024) {
    const int m = (int)std::min<int64_t>(1024, n - s);
    for (int i = 0; i < m; ++i) {
      const uint64_t r = splitmix(seed ^ (uint64_t)(s + i));
      k[i] = (int64_t)(r % (uint64_t)nk);
      t[i] = t0 + (s + i) / 8 - (ooo ? (int64_t)(splitmix(r) % (uint64_t)(ooo + 1)) : 0);
      f1[i] = (int64_t)r;
      if (f64) { double d = (double)(r >> 11) / 9007199254740992.0 - 0.25; memcpy(&v[i], &d, 8); }
      else v[i] = (int64_t)splitmix(r ^ 7);
      if (t[i] > max_ts) max_ts = t[i];
    }
    CHECK(fwo_push_batch(e, k.data(), nullptr, f1.data(), t.data(), v.data(), m) == FW_OK);
    CHECK(fwo_advance_watermark(e, max_ts - lag) == FW_OK);
    fw_out o;
    CHECK(fwo_collect(e, &o) == FW_OK);
    fired += o.n;
    for (int64_t i = 0; i < o.n; ++i) CHECK(o.key[i] >= 0 && o.key[i] < nk);
  }
  CHECK(fwo_advance_watermark(e, INT64_MAX) == FW_OK);
  fw_out o;
  CHECK(fwo_collect(e, &o) == FW_OK);
  return fired + o.n;
}

static void snapshot_restore_roundtrip(const fw_config& c, int64_t n, const fw_state_layout& L) {
  fw_engine* e = nullptr;
  CHECK(fwo_create(&c, &e) == FW_OK);
  // a run that leaves windows open: no final watermark
  std::vector<int64_t> k(n), t(n), v(n);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t r = splitmix(0xabc ^ (uint64_t)i);
    k[i] = (int64_t)(r % 500);
    t[i] = i / 4;
    v[i] = (int64_t)(r >> 3);
  }
  CHECK(fwo_push_batch(e, k.data(), nullptr, nullptr, t.data(), v.data(), n) == FW_OK);
  fw_engine* r = nullptr;
  CHECK(fwo_create(&c, &r) == FW_OK);
  for (int kg = 0; kg < c.max_parallelism; ++kg) {
    int64_t ns = 0, nt = 0;
    CHECK(fwo_snapshot_kg_flink(e, kg, &L, nullptr, 0, &ns, nullptr, 0, &nt) == FW_OK);
    std::vector<uint8_t> st((size_t)ns + 1), tm((size_t)nt + 1);
    CHECK(fwo_snapshot_kg_flink(e, kg, &L, st.data(), ns, &ns, tm.data(), nt, &nt) == FW_OK);
    if (ns == 0) continue;
    CHECK(fwo_restore_kg_flink(r, kg, &L, INT64_MIN, st.data(), ns, tm.data(), nt) == FW_OK);
    int64_t ns2 = 0, nt2 = 0;
    std::vector<uint8_t> st2((size_t)ns + 1), tm2((size_t)nt + 1);
    CHECK(fwo_snapshot_kg_flink(r, kg, &L, st2.data(), ns, &ns2, tm2.data(), nt, &nt2) == FW_OK);
    CHECK(ns2 == ns && nt2 == nt && memcmp(st.data(), st2.data(), (size_t)ns) == 0 &&
          memcmp(tm.data(), tm2.data(), (size_t)nt) == 0);
    // truncated blobs are rejected, never read past their end
    if (ns > 3) CHECK(fwo_restore_kg_flink(r, kg, &L, INT64_MIN, st.data(), ns - 3, tm.data(), nt) != FW_OK);
  }
  fwo_destroy(e);
  fwo_destroy(r);
}

static void decode_streams() {
  // Tuple3<Long, Long, Long> records with timestamps, a watermark, a latency marker
  std::vector<uint8_t> b;
  auto be = [&](uint64_t x, int nb) { for (int s = 8 * (nb - 1); s >= 0; s -= 8) b.push_back((uint8_t)(x >> s)); };
  for (int i = 0; i < 300; ++i) {
    be(33, 4); b.push_back(0); be((uint64_t)(1000 + i), 8);
    be((uint64_t)(i % 17), 8); be((uint64_t)(1000 + i), 8); be(splitmix((uint64_t)i), 8);
    if (i % 50 == 49) { be(9, 4); b.push_back(2); be((uint64_t)(1000 + i), 8); }
    if (i % 70 == 3) { be(17, 4); b.push_back(3); be(77, 8); be(5, 4); be(1, 4); }
  }
  fw_tuple_schema sc;
  memset(&sc, 0, sizeof(sc));
  sc.n_fields = 3;
  sc.key_field = 0;
  sc.f1_field = 1;
  sc.value_field = 2;
  std::vector<int64_t> key(400), f1(400), ts(400), val(400), wm(64), wmp(64), lm(128), lmp(64);
  fw_decode_counts cnt;
  for (int64_t cut : {(int64_t)b.size(), (int64_t)b.size() - 5, (int64_t)17, (int64_t)3}) {
    CHECK(fwo_decode(nullptr, &sc, b.data(), cut, FW_MEM_HOST, key.data(), nullptr, f1.data(), ts.data(), val.data(), 400,
                     wm.data(), wmp.data(), lm.data(), lmp.data(), 64, &cnt) == FW_OK);
    CHECK(cnt.consumed <= cut);
  }
  std::vector<uint8_t> bad = b;
  bad[4] = 9;   // a corrupt tag
  CHECK(fwo_decode(nullptr, &sc, bad.data(), (int64_t)bad.size(), FW_MEM_HOST, key.data(), nullptr, f1.data(), ts.data(),
                   val.data(), 400, wm.data(), wmp.data(), lm.data(), lmp.data(), 64, &cnt) == FW_ERR_INVALID_ARG);
  // too small a record capacity
  CHECK(fwo_decode(nullptr, &sc, b.data(), (int64_t)b.size(), FW_MEM_HOST, key.data(), nullptr, f1.data(), ts.data(),
                   val.data(), 10, wm.data(), wmp.data(), lm.data(), lmp.data(), 64, &cnt) == FW_ERR_CAPACITY);
}

static void kg_codec() {
  for (uint64_t round = 0; round < 200; ++round) {
    fwkg::BeOut o;
    std::vector<int64_t> xs;
    const int n = (int)(splitmix(round) % 64);
    for (int i = 0; i < n; ++i) {
      const int64_t x = (int64_t)splitmix(round * 977 + (uint64_t)i);
      xs.push_back(x);
      o.i64(x); o.i32((int32_t)x); o.i16((int32_t)(int16_t)x); o.u8((uint32_t)x & 0xff);
      double d; memcpy(&d, &x, 8); o.f64(d);
    }
    fwkg::BeIn in(o.b.data(), (int64_t)o.b.size());
    for (int i = 0; i < n; ++i) {
      CHECK(in.i64() == xs[(size_t)i]);
      CHECK(in.i32() == (int32_t)xs[(size_t)i]);
      CHECK(in.i16() == (int32_t)(int16_t)xs[(size_t)i]);
      CHECK(in.u8() == (int32_t)(xs[(size_t)i] & 0xff));
      (void)in.i64();
    }
    CHECK(in.done());
    (void)in.i64();            // past the end: flagged, nothing read
    CHECK(!in.ok);
    std::vector<size_t> idx((size_t)(splitmix(round + 5) % 300));
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    fwkg::hashmap_order(idx, [&](size_t i) { return fwkg::timer_hash((int64_t)i * 1000 + 999, (int64_t)(i % 37), (int64_t)i * 1000,
                                                                     (int64_t)i * 1000 + 1000); },
                        [](size_t a, size_t b) { return a < b; });
    std::vector<char> seen(idx.size(), 0);
    for (size_t i : idx) { CHECK(i < seen.size() && !seen[i]); if (i < seen.size()) seen[i] = 1; }
  }
}

int main() {
  kg_codec();
  decode_streams();
  // the window shapes
  struct Case { int assigner; int64_t size, slide, lateness; int trigger, agg, flags, vt, first; };
  const Case cases[] = {
      {FW_TUMBLING, 1000, 0, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM, 0, FW_VALUE_I64, 1},
      {FW_TUMBLING, 500, 0, 300, FW_TRIGGER_PURGING_EVENT_TIME, FW_AGG_SUM | FW_AGG_MAX, 0, FW_VALUE_I64, 1},
      {FW_TUMBLING, 1000, 0, 100, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM | FW_AGG_COUNT, 0, FW_VALUE_I64, 1},
      {FW_SLIDING, 3000, 1000, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM | FW_AGG_MIN | FW_AGG_MAX | FW_AGG_COUNT, 0, FW_VALUE_F64, 1},
      {FW_SLIDING, 2500, 1000, 1200, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM | FW_AGG_COUNT, 0, FW_VALUE_I64, 1},
      {FW_SESSION, 40, 0, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM | FW_AGG_COUNT, 0, FW_VALUE_I64, 0},
      {FW_SESSION, 40, 0, 500, FW_TRIGGER_PURGING_EVENT_TIME, FW_AGG_SUM, 0, FW_VALUE_F64, 0},
      {FW_TUMBLING, 1000, 0, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_SUM, FW_AGGF_FOLD, FW_VALUE_I64, 0},
      {FW_TUMBLING, 1000, 0, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_MAXBY, FW_AGGF_COMPARABLE, FW_VALUE_F64, 1},
      {FW_SLIDING, 2000, 1000, 0, FW_TRIGGER_EVENT_TIME, FW_AGG_LIST, 0, FW_VALUE_I64, 1},
  };
  for (const Case& k : cases) {
    fw_config c = base_config();
    c.assigner = k.assigner; c.size = k.size; c.slide = k.slide; c.allowed_lateness = k.lateness;
    c.trigger = k.trigger; c.agg_mask = k.agg; c.agg_flags = k.flags; c.value_type = k.vt; c.keep_first_f1 = k.first;
    if (k.flags & FW_AGGF_FOLD) c.fold_initial = 100;
    fw_engine* e = nullptr;
    const int rc = fwo_create(&c, &e);
    CHECK(rc == FW_OK);
    if (rc != FW_OK) { fprintf(stderr, "create: %s\n", fwo_last_error(nullptr)); continue; }
    const int64_t fired = drive(e, 40000, 300, -3000, k.lateness ? 900 : 0, k.vt == FW_VALUE_F64, k.lateness ? 200 : 1, 42);
    CHECK(fired > 0);
    fw_stats st;
    CHECK(fwo_get_stats(e, &st) == FW_OK);
    fwo_destroy(e);
  }
  // checkpoint layout: tumbling sum with first arrival, all int fields with the key
  {
    fw_config c = base_config();
    fw_state_layout L;
    memset(&L, 0, sizeof(L));
    L.n_fields = 3; L.field[0] = FW_SF_KEY; L.field[1] = FW_SF_F1; L.field[2] = FW_SF_SUM;
    snapshot_restore_roundtrip(c, 20000, L);
    c.agg_mask = FW_AGG_SUM | FW_AGG_MIN | FW_AGG_MAX | FW_AGG_COUNT;
    c.keep_first_f1 = 0;
    fw_state_layout M;
    memset(&M, 0, sizeof(M));
    M.n_fields = 5; M.field[0] = FW_SF_KEY; M.field[1] = FW_SF_SUM; M.field[2] = FW_SF_MIN; M.field[3] = FW_SF_MAX;
    M.field[4] = FW_SF_COUNT;
    snapshot_restore_roundtrip(c, 20000, M);
  }
  if (failures) { fprintf(stderr, "%d checks failed\n", failures); return 1; }
  printf("host sanitize driver: ok\n");
  return 0;
}
