"""ComparableAggregator semantics (SJ/api/functions/aggregation/ComparableAggregator.java:66-90,
Comparator.java:45-105), behind WindowedStream.min/max/minBy/maxBy (WindowedStream.java:560-713):

  min/max   value1 with the field set to the extremum in the field's compareTo order: Long natural order;
            Double.compareTo — every NaN equal and above +inf, -0.0 < +0.0 (so .min() skips a NaN that
            Math.min would return)
  minBy/    the extremal record itself (its f1 too); on a compareTo tie the earlier record (first=true,
  maxBy     the WindowedStream default) or the later one (first=false)

Known answers are worked out by hand below from those two files (no reference run exists: no JDK
here); they pin the oracle on CPU, and the HIP engine is compared with both on the GPU.
"""
import math

import numpy as np
import pytest

from harness import drive, epochs_of, gen_stream
from flink_amd.windowing import Aggregations, SlidingEventTimeWindows, TumblingEventTimeWindows, make_config

NAN = float("nan")
LONG_MAX = (1 << 63) - 1


def _cfg(reduce_fn, assigner=None, lateness=0, **kw):
    args = dict(key_capacity=1 << 12, max_batch=1 << 16, out_capacity=1 << 18)
    args.update(kw)
    return make_config(assigner or TumblingEventTimeWindows.of(1000), reduce_fn, None, lateness, **args)


def _run(factory, cfg, keys, f1, ts, vals):
    e = factory(cfg)
    e.push(np.asarray(keys, np.int64), np.asarray(ts, np.int64), np.asarray(vals), f1=np.asarray(f1, np.int64))
    e.advance_watermark(LONG_MAX)
    r = e.collect()
    e.close()
    return r


def _tok(x):
    x = float(x)
    return b"nan" if math.isnan(x) else np.float64(x).tobytes()


# (aggregation, value type, records of key 1 as (f1, value), expected (f1, value))
CASES = [
    ("maxBy_first", "i64", [(10, 5), (11, 7), (12, 7), (13, 3)], (11, 7)),
    ("maxBy_last", "i64", [(10, 5), (11, 7), (12, 7), (13, 3)], (12, 7)),
    ("minBy_first", "i64", [(10, 5), (11, 3), (12, 7), (13, 3)], (11, 3)),
    ("minBy_last", "i64", [(10, 5), (11, 3), (12, 7), (13, 3)], (13, 3)),
    ("maxBy_first", "f64", [(1, 0.0), (2, NAN), (3, 1.0), (4, NAN)], (2, NAN)),       # NaN tops compareTo
    ("maxBy_last", "f64", [(1, 0.0), (2, NAN), (3, 1.0), (4, NAN)], (4, NAN)),
    ("minBy_first", "f64", [(1, 0.0), (2, -0.0), (3, 0.5), (4, -0.0)], (2, -0.0)),   # -0.0 < +0.0
    ("minBy_last", "f64", [(1, NAN), (2, 2.0), (3, 2.0), (4, NAN)], (3, 2.0)),
    ("maxBy_first", "f64", [(1, -0.0), (2, 0.0), (3, -1.0)], (2, 0.0)),
    ("min", "f64", [(1, NAN), (2, 1.0), (3, -0.0), (4, 0.0)], (1, -0.0)),            # f1 of value1 (first)
    ("max", "f64", [(1, 1.0), (2, NAN), (3, 5.0)], (1, NAN)),
    ("min", "i64", [(7, 4), (8, -9), (9, 3)], (7, -9)),
]


def _agg(name, vt):
    base, _, rule = name.partition("_")
    if base in ("maxBy", "minBy"):
        return getattr(Aggregations, base)(vt, first=(rule != "last")), "max" if base == "maxBy" else "min"
    return getattr(Aggregations, base)(vt), base


@pytest.mark.parametrize("name,vt,recs,exp", CASES, ids=[f"{c[0]}-{c[1]}-{i}" for i, c in enumerate(CASES)])
def test_known_answers_oracle(name, vt, recs, exp):
    from oracle.oracle import OracleEngine
    red, col = _agg(name, vt)
    n = len(recs)
    r = _run(OracleEngine, _cfg(red), [1] * n, [f for f, _ in recs], [100 + i for i in range(n)],
             np.array([v for _, v in recs], np.int64 if vt == "i64" else np.float64))
    assert r["n"] == 1 and r["ts"][0] == 999
    got = r[f"{col}_{vt}"][0]
    assert int(r["f1"][0]) == exp[0]
    if vt == "f64":
        assert _tok(got) == _tok(exp[1])
    else:
        assert int(got) == exp[1]


@pytest.mark.gpu
@pytest.mark.parametrize("name,vt,recs,exp", CASES, ids=[f"{c[0]}-{c[1]}-{i}" for i, c in enumerate(CASES)])
def test_known_answers_hip(name, vt, recs, exp):
    from flink_amd.windowing import WindowEngine
    red, col = _agg(name, vt)
    n = len(recs)
    r = _run(WindowEngine, _cfg(red), [1] * n, [f for f, _ in recs], [100 + i for i in range(n)],
             np.array([v for _, v in recs], np.int64 if vt == "i64" else np.float64))
    assert r["n"] == 1 and r["ts"][0] == 999
    assert int(r["f1"][0]) == exp[0]
    got = r[f"{col}_{vt}"][0]
    assert (_tok(got) == _tok(exp[1])) if vt == "f64" else int(got) == exp[1]


def _tie_stream(n, n_keys, vt, seed=5):
    """Few distinct values so ties are everywhere; doubles with NaN, +-0.0 and infinities mixed in."""
    keys, ts, _ = gen_stream(n, n_keys, rate=1 << 14, ooo=300)
    rng = np.random.default_rng(seed)
    if vt == "i64":
        vals = rng.integers(-3, 4, n).astype(np.int64)
    else:
        pool = np.array([0.0, -0.0, 1.5, -2.0, NAN, np.inf, -np.inf, 3.0], np.float64)
        vals = pool[rng.integers(0, len(pool), n)]
    f1 = np.arange(n, dtype=np.int64) * 7 + 3
    return keys, ts, vals, f1


def _rows(results, col, vt):
    ep = []
    for w, recs in epochs_of(results, [col], f1=True):
        ep.append((w, sorted((k, t, f, _tok(v) if vt == "f64" else v) for k, t, f, v in recs)))
    return ep


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", ["maxBy_first", "maxBy_last", "minBy_first", "minBy_last", "min", "max"])
@pytest.mark.parametrize("vt", ["i64", "f64"])
@pytest.mark.parametrize("window", ["tumbling", "sliding", "late"])
def test_parity_with_ties(name, vt, window, mode):
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    red, col = _agg(name, vt)
    # (mode 1, the direct form: maxBy / minBy records are listed and folded per pane in arrival order after each
    # launch — the late path's sort, segmented scan and commit)
    if window == "sliding":
        cfg = _cfg(red, SlidingEventTimeWindows.of(3000, 1000), ingest_mode=mode)
    elif window == "late":
        cfg = _cfg(red, TumblingEventTimeWindows.of(500), lateness=400, ingest_mode=mode)
    else:
        cfg = _cfg(red, TumblingEventTimeWindows.of(1000, 100), ingest_mode=mode)
    keys, ts, vals, f1 = _tie_stream(60_000, 700, vt)
    lag = 150 if window == "late" else 1
    rg = drive(WindowEngine(cfg), keys, ts, vals, 4000, lag, LONG_MAX, f1=f1)
    ro = drive(OracleEngine(cfg), keys, ts, vals, 4000, lag, LONG_MAX, f1=f1)
    assert _rows(rg, f"{col}_{vt}", vt) == _rows(ro, f"{col}_{vt}", vt)
