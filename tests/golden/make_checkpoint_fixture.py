"""Generates tests/golden/checkpoint_flink.json: key-group checkpoint sections in the reference's byte layout,
built by hand from the layout's definition — independently of the oracle and of the engine — for
small seeded streams.

The model below restates, in plain Python, what the reference's heap backend holds for the event-time
WindowOperator (paths relative to the reference root):
  state tables    RT/state/heap/HeapReducingState.java:84-122 (add: namespace map per key group created
                  on first use, namespace entry, key entry, reduce(stored, incoming)),
                  AbstractHeapState.java:90-119 (clear: remove the key, then an empty namespace)
  operator        SJ/runtime/operators/windowing/WindowOperator.java:302-333 (processElement),
                  :336-375 (onEventTime), :479-486 / :511-514 (cleanup timer / time)
  trigger         SJ/api/windowing/triggers/EventTimeTrigger.java:37-62
  timer service   SJ/api/operators/HeapInternalTimerService.java:211-236, 264-278 (a HashSet per key group
                  plus a priority queue)
and encodes one key group as the reference writes it:
  state   HeapKeyedStateBackend.snapshot / writeStateTableForKeyGroup
          (RT/state/heap/HeapKeyedStateBackend.java:196-212, 217-248):
          int kg | short 0 | byte present | int numNamespaces | (long start | long end | int n | (long key | tuple)*)*
  timers  HeapInternalTimerService.snapshotTimersForKeyGroup (:285-310) after the serializer records:
          int n | (long key | long start | long end | long ts)* | int 0
Iteration order is java.util.HashMap's: bucket (h ^ h >>> 16) & (capacity - 1), capacity 16 doubled while
size > 3/4 capacity (sized by the current size, the rule DESIGN.md documents), chains in insertion order
(a Python dict keeps insertion order; deleting and re-adding appends, as a HashMap chain does).

Run from the repo root:  python tests/golden/make_checkpoint_fixture.py
"""
import json
import math
import os
import random
import struct

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checkpoint_flink.json")
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


def s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def s64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= 1 << 63 else x


def long_hash(v):                      # Long.hashCode
    u = v & ((1 << 64) - 1)
    return s32(u ^ (u >> 32))


def murmur(code):                      # MathUtils.murmurHash (flink-core/.../util/MathUtils.java:134-158)
    def rotl(v, r):
        return ((v << r) | (v >> (32 - r))) & 0xFFFFFFFF
    c = code & 0xFFFFFFFF
    c = (c * 0xCC9E2D51) & 0xFFFFFFFF
    c = rotl(c, 15)
    c = (c * 0x1B873593) & 0xFFFFFFFF
    c = rotl(c, 13)
    c = (c * 5 + 0xE6546B64) & 0xFFFFFFFF
    c ^= 4
    c ^= c >> 16
    c = (c * 0x85EBCA6B) & 0xFFFFFFFF
    c ^= c >> 13
    c = (c * 0xC2B2AE35) & 0xFFFFFFFF
    c ^= c >> 16
    c = s32(c)
    return c if c >= 0 else (-c if c != -(1 << 31) else 0)


def key_group(key, mp):                # KeyGroupRangeAssignment.assignToKeyGroup
    return murmur(long_hash(key)) % mp


def window_hash(start, end):           # TimeWindow.hashCode
    return s32(31 * long_hash(start) + long_hash(end))


def timer_hash(ts, key, start, end):   # InternalTimer.hashCode
    r = long_hash(ts)
    r = s32(31 * r + long_hash(key))
    return s32(31 * r + window_hash(start, end))


def hashmap_iter(items, hash_of):
    """items: list in insertion order -> java.util.HashMap iteration order."""
    cap = 16
    while len(items) > cap * 3 // 4:
        cap *= 2
    buckets = {}
    for it in items:
        h = hash_of(it)
        b = ((h ^ ((h & 0xFFFFFFFF) >> 16)) & 0xFFFFFFFF) & (cap - 1)
        buckets.setdefault(b, []).append(it)
    return [it for b in sorted(buckets) for it in buckets[b]]


def java_min(a, b):                    # Math.min(double, double)
    if a != a:
        return a
    if a == 0.0 and b == 0.0 and math.copysign(1.0, b) < 0:
        return b
    return a if a <= b else b


def java_max(a, b):                    # Math.max(double, double)
    if a != a:
        return a
    if a == 0.0 and b == 0.0 and math.copysign(1.0, a) < 0:
        return b
    return a if a >= b else b


class Operator:
    def __init__(self, cfg):
        self.c = cfg
        self.wm = LONG_MIN
        self.tables = {}      # kg -> {(start, end): {key: state}}  (dicts = insertion order)
        self.timers = {}      # kg -> {(key, start, end, ts): None}
        self.out = []

    def windows(self, ts):
        c = self.c
        if c["assigner"] == "tumbling":
            start = ts - (ts - c["offset"] + c["size"]) % c["size"]
            return [(start, start + c["size"])]
        last = ts - (ts - c["offset"] + c["slide"]) % c["slide"]
        ws, start = [], last
        while start > ts - c["size"]:
            ws.append((start, start + c["size"]))
            start -= c["slide"]
        return ws

    def cleanup(self, w):
        mt = w[1] - 1
        ct = mt + self.c["lateness"]
        return ct if ct <= LONG_MAX else LONG_MAX

    def reduce(self, a, b):
        vt, r = self.c["value_type"], dict(a)
        if "sum" in a:
            r["sum"] = a["sum"] + b["sum"] if vt == "f64" else s64(a["sum"] + b["sum"])
        if "min" in a:
            r["min"] = java_min(a["min"], b["min"]) if vt == "f64" else min(a["min"], b["min"])
        if "max" in a:
            r["max"] = java_max(a["max"], b["max"]) if vt == "f64" else max(a["max"], b["max"])
        if "count" in a:
            r["count"] = a["count"] + b["count"]
        return r

    def element(self, key, f1, ts, value):
        kg = key_group(key, self.c["mp"])
        rec = {"key": key, "f1": f1}
        for agg in self.c["aggs"]:
            rec[agg] = 1 if agg == "count" else value
        for w in self.windows(ts):
            if self.cleanup(w) <= self.wm:          # isLate: dropped
                continue
            ns = self.tables.setdefault(kg, {}).setdefault(w, {})
            ns[key] = self.reduce(ns[key], rec) if key in ns else dict(rec)
            if w[1] - 1 <= self.wm:                 # EventTimeTrigger.onElement: FIRE
                self.out.append((w[1] - 1, dict(ns[key])))
            else:
                self.timers.setdefault(kg, {}).setdefault((key, w[0], w[1], w[1] - 1), None)
            self.timers.setdefault(kg, {}).setdefault((key, w[0], w[1], self.cleanup(w)), None)

    def watermark(self, wm):
        self.wm = wm
        due = sorted((t[3], kg, t) for kg, ts in self.timers.items() for t in ts if t[3] <= wm)
        for _, kg, t in due:
            if t not in self.timers[kg]:
                continue
            del self.timers[kg][t]
            key, start, end, ts = t
            ns = self.tables.get(kg, {}).get((start, end))
            if ns is None or key not in ns:
                continue
            if ts == end - 1:                       # onEventTime: FIRE
                self.out.append((end - 1, dict(ns[key])))
            if self.cleanup((start, end)) == ts:    # cleanup: clear state, delete the trigger timer
                del ns[key]
                if not ns:
                    del self.tables[kg][(start, end)]
                self.timers[kg].pop((key, start, end, end - 1), None)

    def snapshot(self, kg, layout):
        vt = self.c["value_type"]

        def field(st, f, s):
            if f in ("key", "f1", "count") or vt == "i64":
                return struct.pack(">q", s[f])
            if s[f] != s[f]:
                return struct.pack(">Q", 0x7FF8000000000000)   # doubleToLongBits
            return struct.pack(">d", s[f])

        st = b""
        if self.tables:
            st = struct.pack(">ih", kg, 0)
            if kg not in self.tables:
                st += struct.pack(">b", 0)
            else:
                nss = hashmap_iter(list(self.tables[kg].items()), lambda it: window_hash(*it[0]))
                st += struct.pack(">bi", 1, len(nss))
                for (start, end), ents in nss:
                    st += struct.pack(">qqi", start, end, len(ents))
                    for key, s in hashmap_iter(list(ents.items()), lambda it: long_hash(it[0])):
                        st += struct.pack(">q", key) + b"".join(field(st, f, s) for f in layout)
        tl = hashmap_iter(list(self.timers.get(kg, {})), lambda t: timer_hash(t[3], t[0], t[1], t[2]))
        tm = struct.pack(">i", len(tl)) + b"".join(struct.pack(">qqqq", *t) for t in tl) + struct.pack(">i", 0)
        return st, tm


def stream(seed, n, keys, t0, spread, lag, wm_every, vt, specials=()):
    rng = random.Random(seed)
    recs, wms, mx = [], [], LONG_MIN
    for i in range(n):
        key = keys[rng.randrange(len(keys))]
        ts = t0 + int(i * spread) - rng.randrange(lag)
        if i in specials:
            ts -= 2500                               # far behind: dropped as late
        if vt == "i64":
            v = rng.randrange(-1000, 1000)
        else:
            v = rng.choice([0.0, -0.0, 1.5, -2.25, float("nan"), float("inf"), 3.0, 7.125, -0.5])
        recs.append([key, 1000 + i, ts, v])
        mx = max(mx, ts)
        if (i + 1) % wm_every == 0:
            wms.append([i + 1, mx - 200])
    return recs, wms


SCENARIOS = [
    dict(name="tumbling_lateness_i64",
         config=dict(assigner="tumbling", size=1000, slide=1000, offset=0, lateness=500, value_type="i64",
                     aggs=["sum"], mp=8, trigger="event_time"),
         layout=["key", "f1", "sum"], seed=11, n=1600, spread=2.5, lag=400, wm_every=80, cut="fired_kept",
         restore_wm="checkpoint"),
    dict(name="tumbling_f64_min_max",
         config=dict(assigner="tumbling", size=1000, slide=1000, offset=250, lateness=0, value_type="f64",
                     aggs=["sum", "min", "max", "count"], mp=8, trigger="event_time"),
         layout=["key", "f1", "sum", "min", "max", "count"], seed=12, n=1400, spread=3.0, lag=300,
         wm_every=70, cut=910, restore_wm="min"),
    dict(name="sliding_i64",
         config=dict(assigner="sliding", size=3000, slide=1000, offset=0, lateness=0, value_type="i64",
                     aggs=["sum", "count"], mp=8, trigger="event_time"),
         layout=["key", "f1", "sum", "count"], seed=13, n=1200, spread=4.0, lag=300, wm_every=60, cut=780,
         restore_wm=None),
]


def keyset():
    ks = list(range(0, 48))                                     # small keys: chains k, k+16, k+32 in one bucket
    ks += [s64(i * 0x9E3779B97F4A7C15) for i in range(1, 41)]   # high bits matter to Long.hashCode
    ks += [-7, -123456789012345, LONG_MAX, LONG_MIN + 1, LONG_MIN]
    return ks


def main():
    out = {"generator": "tests/golden/make_checkpoint_fixture.py", "scenarios": []}
    t0 = 1_000_000
    for sc in SCENARIOS:
        c = sc["config"]
        recs, wms = stream(sc["seed"], sc["n"], keyset(), t0, sc["spread"], sc["lag"], sc["wm_every"],
                           c["value_type"], specials={sc["n"] // 2, sc["n"] // 2 + 7})
        if sc["cut"] == "fired_kept":
            # the first watermark past 60% of the stream that lies inside a window's lateness period, so
            # the checkpoint holds fired-but-kept panes (cleanup timer only)
            sc["cut"] = next(i for i, w in wms if i >= sc["n"] * 3 // 5 and 150 <= w % c["size"] < c["lateness"] - 100)
        assert any(w[0] == sc["cut"] for w in wms)
        op = Operator(c)
        wi = 0
        for i, r in enumerate(recs[:sc["cut"]]):
            op.element(*r)
            while wi < len(wms) and wms[wi][0] == i + 1:
                op.watermark(wms[wi][1])
                wi += 1
        kgs = {}
        for kg in range(c["mp"]):
            st, tm = op.snapshot(kg, sc["layout"])
            kgs[str(kg)] = [st.hex(), tm.hex()]
        enc = [[k, f, t, (v if c["value_type"] == "i64" else struct.unpack(">q", struct.pack(">d", v))[0])]
               for k, f, t, v in recs]
        out["scenarios"].append(dict(name=sc["name"], config=c, layout=sc["layout"], records=enc,
                                     value_encoding="int64" if c["value_type"] == "i64" else "double bits as int64",
                                     watermarks=wms, cut=sc["cut"], checkpoint_wm=op.wm,
                                     restore_wm=sc["restore_wm"], kgs=kgs))
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
