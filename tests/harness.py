"""Shared test machinery: fixture replay, synthetic streams, and the reference's output contract.

Output contract (TestHarnessUtil.assertOutputEqualsSorted, flink-streaming-java/src/test/java/org/
apache/flink/streaming/util/TestHarnessUtil.java:80-117): watermark positions must match exactly;
records between two watermarks are compared as a sorted multiset.
"""
import json
import os

import numpy as np

from flink_amd import _abi
from flink_amd.windowing import (EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, ReduceFunction,
                                 SlidingEventTimeWindows, TumblingEventTimeWindows, make_config)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


WINDOW_FIXTURES = ["sliding_reduce", "tumbling_reduce", "lateness_purging", "cleanup_time_overflow",
                   "drop_late_tumbling", "drop_late_sliding", "cleanup_timer_empty_state", "tumbling_offset",
                   "sliding_offset", "itcase_tumbling_closed_form", "itcase_sliding_closed_form",
                   "sliding_lateness", "sliding_lateness_purging"]
SESSION_FIXTURES = ["session_reduce", "session_windows", "session_late_zero_purging", "session_late_zero",
                    "session_late_small_purging", "session_late_small", "session_late_huge_purging",
                    "session_late_huge", "session_cleanup_timer"]
FOLD_FIXTURES = ["fold_cleanup_timer"]
LIST_FIXTURES = ["list_sliding_apply", "list_tumbling_apply", "list_cleanup_timer"]


def hip_engine(cfg):
    """WindowEngine(cfg) (the HIP engine the GPU parity tests drive)."""
    from flink_amd.windowing import WindowEngine
    return WindowEngine(cfg)


def fixture_config(c, **kw):
    if c["assigner"] == "tumbling":
        assigner = TumblingEventTimeWindows(c["size"], c["offset"])
    elif c["assigner"] == "session":
        assigner = EventTimeSessionWindows.withGap(c["size"])
    else:
        assigner = SlidingEventTimeWindows(c["size"], c["slide"], c["offset"])
    trig = EventTimeTrigger.create() if c["trigger"] == "event_time" else PurgingTrigger.of(EventTimeTrigger.create())
    if c.get("list"):
        from flink_amd.windowing import ListStateDescriptor
        red = ListStateDescriptor(c["value_type"])
    elif "fold" in c:
        from flink_amd.windowing import FoldFunction
        red = FoldFunction(c["fold"]["kind"], c["fold"]["initial"], c["value_type"])
    else:
        red = ReduceFunction(tuple(c["agg"]), c["value_type"], c["keep_first_f1"])
    mp = c["max_parallelism"]
    args = dict(max_parallelism=mp, key_capacity=1024, max_batch=1 << 12, out_capacity=1 << 16)
    args.update(kw)
    return make_config(assigner, red, trig, c["allowed_lateness"], **args), red


def fixture_events(fx):
    if "events" in fx:
        return fx["events"]
    g = fx["generator"]
    ev = []
    for nxt in range(g["n_elements"]):
        for k in range(g["n_keys"]):
            ev.append(["rec", k, nxt, nxt])
        ev.append(["wm", nxt])
    return ev


def replay(fx, engine_factory, **kw):
    """Run a fixture's event list through an engine; returns [(wm, sorted [(key, value, ts)])]."""
    cfg, red = fixture_config(fx["config"], **kw)
    eng = engine_factory(cfg)
    kh = {int(k): v for k, v in fx.get("key_hash", {}).items()}
    epochs = []
    pend = []

    def flush():
        if not pend:
            return
        keys = np.array([p[0] for p in pend], dtype=np.int64)
        vals = np.array([p[1] for p in pend], dtype=np.int64)
        ts = np.array([p[2] for p in pend], dtype=np.int64)
        hashes = np.array([kh[int(k)] for k in keys], dtype=np.int32) if kh else None
        eng.push(keys, ts, vals, key_hash=hashes)
        pend.clear()

    for e in fixture_events(fx):
        if e[0] == "rec":
            pend.append(e[1:])
        else:
            flush()
            eng.advance_watermark(e[1])
            res = eng.collect()
            assert len(res["mark_wm"]) == 1 and res["mark_wm"][0] == e[1]
            assert res["mark_pos"][0] == res["n"], "records emitted after the watermark mark"
            if fx["config"].get("list"):   # the window function of the reference test: the sum per (key, window)
                session = fx["config"]["assigner"] == "session"
                groups = {}
                for i in range(res["n"]):
                    g = (int(res["key"][i]), int(res["ts"][i])) + ((int(res["win_start"][i]),) if session else ())
                    groups[g] = groups.get(g, 0) + int(res["sum_i64"][i])
                recs = sorted((g[0], v) + g[1:] for g, v in groups.items())
            elif fx["config"]["assigner"] == "session":   # the window's start too (end = ts + 1)
                recs = sorted((int(res["key"][i]), int(res["sum_i64"][i]), int(res["ts"][i]), int(res["win_start"][i]))
                              for i in range(res["n"]))
            else:
                recs = sorted((int(res["key"][i]), int(res["sum_i64"][i]), int(res["ts"][i])) for i in range(res["n"]))
            epochs.append((e[1], recs))
    eng.close()
    return epochs


def expected_epochs(fx):
    return [(x["wm"], sorted(tuple(r) for r in x["records"])) for x in fx["expected"]]


# ------------------------------------------------------------------ synthetic streams
M64 = (1 << 64) - 1


def splitmix64(x):
    """splitmix64 over a numpy uint64 array (counter-based generator of SURVEY.md §8d)."""
    z = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def gen_stream(n, n_keys, rate, t0=0, seed=1, zipf=None, ooo=0, value_type="i64", start=0):
    """Records start..start+n of the synthetic stream: keys, ts, values (numpy)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    if zipf is None:
        keys = (splitmix64(np.uint64(seed) ^ i) % np.uint64(n_keys)).astype(np.int64)
    else:
        ranks = np.arange(1, n_keys + 1, dtype=np.float64)
        cdf = np.cumsum(ranks ** -zipf)
        cdf /= cdf[-1]
        u = (splitmix64(np.uint64(seed) ^ i) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
        keys = np.minimum(np.searchsorted(cdf, u), n_keys - 1).astype(np.int64)
    ts = (t0 + (i.astype(np.int64) * 1000) // rate).astype(np.int64)
    if ooo:
        ts = ts - (splitmix64(np.uint64(3) ^ i) % np.uint64(ooo + 1)).astype(np.int64)
    raw = splitmix64(np.uint64(2) ^ i)
    if value_type == "i64":
        vals = raw.view(np.int64).copy()
    else:
        vals = (raw >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    return keys, ts, vals


def drive(eng, keys, ts, vals, batch, wm_lag=1, final_wm=None, f1=None):
    """Push in batches; after each batch advance wm = max ts seen - wm_lag; collect everything."""
    out = []
    max_ts = -(1 << 63)
    n = len(keys)
    for s in range(0, n, batch):
        e = min(n, s + batch)
        eng.push(keys[s:e], ts[s:e], vals[s:e], f1=None if f1 is None else f1[s:e])
        max_ts = max(max_ts, int(ts[s:e].max()))
        eng.advance_watermark(max_ts - wm_lag)
        out.append(eng.collect())
    if final_wm is not None:
        eng.advance_watermark(final_wm)
        out.append(eng.collect())
    return out


def epochs_of(results, fields, f1=False):
    """Per watermark: sorted list of (key, ts, [f1], fields...) from a list of collect() results."""
    ep = []
    for res in results:
        pos = 0
        cols = [res["key"], res["ts"]] + ([res["f1"]] if f1 else []) + [res[f] for f in fields]
        marks = list(zip(res["mark_wm"], res["mark_pos"])) + [(None, res["n"])]
        for wm, mp in marks:
            recs = [tuple(c[j].item() for c in cols) for j in range(pos, mp)]
            if wm is None:
                if recs:
                    ep.append(("tail", sorted(recs)))
            else:
                ep.append((int(wm), sorted(recs)))
            pos = mp
    return ep
