"""HIP engine parity: the reference's golden fixtures and oracle comparisons on seeded streams.

Bar: bit-exact for int64 sum/min/max/count and first-arrival f1; double sums within relative 1e-9 of
the oracle (measured against sum|v|: values are positive here), double min/max/count exact.
"""
import numpy as np
import pytest

from harness import (WINDOW_FIXTURES, drive, epochs_of, expected_epochs, fixture_config, gen_stream, load_golden,
                     replay)

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module")
def hip():
    from flink_amd import _abi
    from harness import hip_engine
    _abi.load_library()
    return hip_engine


@pytest.fixture(scope="module")
def oracle_engine():
    from oracle.oracle import OracleEngine
    return OracleEngine


MODES = [pytest.param(1, id="direct"), pytest.param(2, id="partitioned")]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name", WINDOW_FIXTURES)
def test_golden_fixture(hip, name, mode):
    fx = load_golden(name)
    got = replay(fx, hip, ingest_mode=mode)
    assert got == expected_epochs(fx), fx["source"]


def _cfg(assigner, fields=("sum",), vt="i64", first=False, lateness=0, trigger=None, mode=0, **kw):
    from flink_amd.windowing import ReduceFunction, make_config
    args = dict(key_capacity=1 << 14, max_batch=1 << 16, out_capacity=1 << 20, ingest_mode=mode)
    args.update(kw)
    return make_config(assigner, ReduceFunction(fields, vt, first), trigger, lateness, **args)


def _cfgm(mode, *a, **kw):
    return _cfg(*a, mode=mode, **kw)


def _compare(a, b, fields, rel=0.0):
    assert len(a) == len(b)
    for (wa, ra), (wb, rb) in zip(a, b):
        assert wa == wb
        assert len(ra) == len(rb), f"wm {wa}: {len(ra)} vs {len(rb)} records"
        if rel == 0.0:
            assert ra == rb, f"wm {wa}"
        else:
            for x, y in zip(ra, rb):
                for u, v in zip(x, y):
                    if isinstance(u, float):
                        assert abs(u - v) <= rel * max(1.0, abs(v)), (wa, x, y)
                    else:
                        assert u == v, (wa, x, y)


def _run_both(hip, oracle_engine, cfg, keys, ts, vals, batch, lag, fields, first=False, rel=0.0, f1=None):
    eg = hip(cfg)
    eo = oracle_engine(cfg)
    rg = drive(eg, keys, ts, vals, batch, lag, LONG_MAX, f1=f1)
    ro = drive(eo, keys, ts, vals, batch, lag, LONG_MAX, f1=f1)
    sg, so = eg.stats(), eo.stats()
    eg.close()
    eo.close()
    _compare(epochs_of(rg, fields, first), epochs_of(ro, fields, first), fields, rel)
    return sg, so


@pytest.mark.parametrize("mode", MODES)
def test_tumbling_long_sum_first_arrival(hip, oracle_engine, mode):
    """C1 shape at small scale: keyed tumbling 1 s long-sum, f1 of the first arrival (Tuple3 job)."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(200_000, 4096, rate=1 << 16)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000), first=True)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 1 << 14, 1, ["sum_i64"], first=True)
    assert sg["panes_fired"] == so["panes_fired"]


@pytest.mark.parametrize("mode", MODES)
def test_tumbling_all_fields_int(hip, oracle_engine, mode):
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(100_000, 1000, rate=1 << 15, ooo=300)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000, 250), ("sum", "min", "max", "count"))
    _run_both(hip, oracle_engine, cfg, keys, ts, vals, 10_000, 1, ["sum_i64", "min_i64", "max_i64", "count"])


@pytest.mark.parametrize("mode", MODES)
def test_sliding_double_multi_field(hip, oracle_engine, mode):
    """C3 shape: sliding 10 s / 1 s, double sum/min/max/count (sum to 1e-9 relative)."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(150_000, 2000, rate=1 << 13, value_type="f64")
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(10_000, 1000), ("sum", "min", "max", "count"), "f64", True)
    _run_both(hip, oracle_engine, cfg, keys, ts, vals, 8192, 1, ["sum_f64", "min_f64", "max_f64", "count"],
              first=True, rel=1e-9)


@pytest.mark.parametrize("mode", MODES)
def test_sliding_uneven_slide(hip, oracle_engine, mode):
    """size not a multiple of slide: slices of gcd(size, slide)."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(60_000, 300, rate=1 << 12, ooo=700, t0=1_700_000_000_123)
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(2500, 1000, 300), ("sum", "count"))
    _run_both(hip, oracle_engine, cfg, keys, ts, vals, 3000, 500, ["sum_i64", "count"])


@pytest.mark.parametrize("mode", [pytest.param(1, id="direct"), pytest.param(2, id="partitioned")])
@pytest.mark.parametrize("spec", [(10_000, 100), (60_000, 100)], ids=["10s_100ms", "60s_100ms"])
@pytest.mark.parametrize("lateness", [0, 700])
def test_sliding_many_slices(hip, oracle_engine, mode, spec, lateness):
    """Windows of more than 64 slices (VERDICT r3 missing #2): SlidingEventTimeWindows.of(10 s, 100 ms) = 100 panes
    per record and of(60 s, 100 ms) = 600 (SlidingEventTimeWindows.java:64-77 enumerates them all), with and
    without allowed lateness (per-element fires of every already-fired window of a late record), against the
    oracle; long sums, counts, max and the first-arrival f1 bit-exact."""
    from flink_amd.windowing import SlidingEventTimeWindows
    size, slide = spec
    n = 60_000 if size == 10_000 else 24_000   # 4096 events per second of event time: 10 slices per batch
    keys, ts, vals = gen_stream(n, 300, rate=1 << 12, ooo=900 if lateness else 0)
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(size, slide), ("sum", "max", "count"), first=True, lateness=lateness,
                key_capacity=1 << 10, max_batch=1 << 12)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 1 << 12, 300, ["sum_i64", "max_i64", "count"], first=True)
    assert sg["panes_fired"] == so["panes_fired"] > 0
    if lateness:
        assert sg["late_fires"] == so["late_fires"] > 0


@pytest.mark.parametrize("mode,ooo,batch", [pytest.param(1, 600, 1000, id="direct"),
                                             pytest.param(2, 0, 200, id="partitioned")])
def test_sliding_k1000_flush(hip, oracle_engine, mode, ooo, batch):
    """SlidingEventTimeWindows.of(1 s, 1 ms): 1000 slices (and windows) per record, allowed lateness 700, and a final
    Long.MAX_VALUE watermark that fires every pending window at once — about P + K of them (the watermark's
    window list held 2048).  Direct form: out of order by up to 600 ms, per-element fires.  Partitioned form: in order,
    in batches of at most RT_GS = 64 distinct 1 ms slices (its per-batch slice set; more fails with FW_ERR_CAPACITY)."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(3000, 100, rate=1 << 12, ooo=ooo)
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(1000, 1), ("sum", "count"), first=True, lateness=700,
                key_capacity=1 << 10, max_batch=1 << 12)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, batch, 300, ["sum_i64", "count"], first=True)
    assert sg["panes_fired"] == so["panes_fired"] > 0
    assert sg["late_fires"] == so["late_fires"]
    if ooo:
        assert so["late_fires"] > 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("purging", [False, True], ids=["event_time", "purging"])
def test_sliding_allowed_lateness(hip, oracle_engine, mode, purging):
    """Sliding 3 s / 1 s, allowed lateness 500, out-of-order input behind the watermark: per-element fires
    of every window of a late record's slice in its lateness period (WindowOperator.java:302-333,
    EventTimeTrigger.java:38-40); PurgingTrigger purges each window at every fire (PurgingTrigger.java:47-55)."""
    from flink_amd.windowing import EventTimeTrigger, PurgingTrigger, SlidingEventTimeWindows
    keys, ts, vals = gen_stream(120_000, 800, rate=1 << 14, ooo=900)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else None
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(3000, 1000), ("sum", "max", "count"), first=True, lateness=500,
                trigger=trig)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 3000, 300, ["sum_i64", "max_i64", "count"], first=True)
    assert so["late_fires"] > 0 and sg["late_fires"] == so["late_fires"]
    assert sg["records_late"] == so["records_late"] and so["records_late"] > 0


@pytest.mark.parametrize("mode", MODES)
def test_sliding_lateness_double_uneven(hip, oracle_engine, mode):
    """size not a multiple of slide (slices of gcd), doubles, lateness longer than a slide."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(80_000, 300, rate=1 << 13, ooo=1500, value_type="f64", t0=1_700_000_000_123)
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(2500, 1000, 300), ("sum", "min", "max", "count"), "f64", True,
                lateness=1200)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 4000, 400, ["sum_f64", "min_f64", "max_f64", "count"],
                       first=True, rel=1e-9)
    assert so["late_fires"] > 0 and sg["late_fires"] == so["late_fires"]


def test_sliding_negative_remainder_known_answer(hip, oracle_engine):
    """SlidingEventTimeWindows.of(3 s, 1 s) and a record at ts = -1500: getWindowStartWithOffset(-1500, 0, 1000)
    = -1500 - (-500 % 1000) = -1000 (Java % of a negative numerator, TimeWindow.java:239-241), so the
    assigner's loop (SlidingEventTimeWindows.java:64-77) yields starts -1000, -2000, -3000, -4000: one window
    more than the three containing the record.  Worked by hand from the Java source."""
    from flink_amd.windowing import SlidingEventTimeWindows
    want = sorted([(7, 1999, 5), (7, 999, 5), (7, -1, 5), (7, -1001, 5)])   # (key, maxTimestamp, sum)
    for f in (hip, oracle_engine):
        for mode in (1, 2):
            e = f(_cfg(SlidingEventTimeWindows.of(3000, 1000), mode=mode))
            e.push(np.array([7], np.int64), np.array([-1500], np.int64), np.array([5], np.int64))
            e.advance_watermark(LONG_MAX)
            r = e.collect()
            e.close()
            assert sorted(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist())) == want


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("spec,lateness", [((3000, 1000, 0), 0), ((2500, 1000, 300), 0), ((3000, 1000, 0), 1500),
                                           ((10000, 1000, 0), 0)])
def test_sliding_negative_timestamps(hip, oracle_engine, mode, spec, lateness):
    """A stream crossing from negative to positive event time: records below offset - slide get the
    assigner's extra window (window panes beside the slices), bit-exact incl. first-arrival f1."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(100_000, 700, rate=1 << 12, ooo=300, t0=-20_000)
    cfg = _cfgm(mode, SlidingEventTimeWindows.of(*spec), ("sum", "min", "max", "count"), first=True, lateness=lateness)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 4096, 200, ["sum_i64", "min_i64", "max_i64", "count"],
                       first=True)
    assert sg["records_late"] == so["records_late"]


@pytest.mark.parametrize("mode", MODES)
def test_zipf_out_of_order_lateness(hip, oracle_engine, mode):
    """C4 shape: Zipf(1.2) keys, out-of-order ts, bounded WM lag, allowed lateness -> per-element fires."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(200_000, 1 << 12, rate=1 << 16, zipf=1.2, ooo=200)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000), ("sum", "count"), first=True, lateness=100)
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 2048, 50, ["sum_i64", "count"], first=True)
    assert so["late_fires"] > 0 and sg["late_fires"] == so["late_fires"]
    assert sg["records_late"] == so["records_late"] and so["records_late"] > 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("spec", [(1000, 1000, 370, -6_000), (3000, 1000, 750, 6_000)])
def test_lateness_read_back_skip(hip, oracle_engine, monkeypatch, mode, spec):
    """The push skips reading the late-record counts back when no window of the assigner's grid is within its
    lateness at the watermark (fires_possible: window maxTimestamps are offset + size - 1 modulo the step).
    With FW_DEBUG_LATE=1 every skipped read-back is checked to have had nothing to read.  Offsets, negative
    timestamps, and watermarks landing right outside and inside the lateness period (lag swept through it)."""
    from flink_amd.windowing import SlidingEventTimeWindows, TumblingEventTimeWindows
    monkeypatch.setenv("FW_DEBUG_LATE", "1")
    size, slide, off, t0 = spec   # (sliding: no timestamps below offset - slide, whose extra window has no re-fire)
    a = TumblingEventTimeWindows.of(size, off) if size == slide else SlidingEventTimeWindows.of(size, slide, off)
    for lag in (0, 1, 99, 100, 101):
        keys, ts, vals = gen_stream(40_000, 500, rate=1 << 12, ooo=250, t0=t0)
        cfg = _cfgm(mode, a, ("sum", "count"), first=True, lateness=100)
        sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 1000, lag, ["sum_i64", "count"], first=True)
        assert sg["late_fires"] == so["late_fires"] and sg["records_late"] == so["records_late"]


@pytest.mark.parametrize("case", ["sum_count_lateness", "f64_min_max", "max_by", "purging", "min_no_first"])
def test_hot_buckets_split_over_helpers(hip, oracle_engine, monkeypatch, case):
    """Zipf(1.3) keys concentrate the records in a few directory buckets; with FW_DEBUG_AGG & 64 a share
    is 256 records, so from the second batch on the hot buckets are split over helper workgroups
    (k_aggregate): integer shares fold concurrently with device atomics, the last one resolving the first
    arrivals' f1; double sums and maxBy fold one share after another.  Bit-exact against the oracle
    (double sums: tolerance)."""
    import ctypes
    from flink_amd.windowing import EventTimeTrigger, PurgingTrigger, ReduceFunction, TumblingEventTimeWindows
    from flink_amd.windowing import Aggregations, make_config
    monkeypatch.setenv("FW_DEBUG_AGG", "64")
    vt = "f64" if case == "f64_min_max" else "i64"
    keys, ts, vals = gen_stream(120_000, 1 << 12, rate=1 << 15, zipf=1.3, ooo=150, value_type=vt)
    kw = dict(key_capacity=1 << 14, max_batch=1 << 14, out_capacity=1 << 20, ingest_mode=2)
    asg = TumblingEventTimeWindows.of(1000)
    rel, lag = 0.0, 1
    if case == "sum_count_lateness":
        cfg = make_config(asg, ReduceFunction(("sum", "count"), vt, True), None, 100, **kw)
        fields, lag = ["sum_i64", "count"], 50
    elif case == "f64_min_max":
        cfg = make_config(asg, ReduceFunction(("sum", "min", "max"), vt, True), None, 0, **kw)
        fields, rel = ["sum_f64", "min_f64", "max_f64"], 1e-9
    elif case == "max_by":
        cfg = make_config(asg, Aggregations.maxBy(vt), None, 0, **kw)
        fields = ["max_i64"]
    elif case == "min_no_first":
        cfg = make_config(asg, ReduceFunction(("min", "count"), vt, False), None, 0, **kw)
        fields = ["min_i64", "count"]
    else:
        cfg = make_config(asg, ReduceFunction(("sum", "max"), vt, True), PurgingTrigger.of(EventTimeTrigger.create()),
                          0, **kw)
        fields = ["sum_i64", "max_i64"]
    eg = hip(cfg)
    eo = oracle_engine(cfg)
    f1 = np.arange(len(keys), dtype=np.int64) * 5 + 2
    rg = drive(eg, keys, ts, vals, 1 << 14, lag, LONG_MAX, f1=f1)
    ro = drive(eo, keys, ts, vals, 1 << 14, lag, LONG_MAX, f1=f1)
    dbg = np.zeros(8, np.int64)
    eg.lib.fw_debug_counters(eg.h, dbg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    eg.close()
    eo.close()
    assert dbg[3] > 0, "no bucket was split"
    assert dbg[7] == 0, f"capacity error at site {dbg[7]}"
    keep_f1 = case != "min_no_first"
    _compare(epochs_of(rg, fields, keep_f1), epochs_of(ro, fields, keep_f1), fields, rel)


@pytest.mark.parametrize("lateness", [0, 500])
@pytest.mark.parametrize("mode", MODES)
def test_first_arrival_with_tiles_spanning_many_slices(hip, oracle_engine, mode, lateness):
    """Timestamps 1 s out of order over 100 ms windows: every 4096-record route tile holds records of ~10
    slices, more than its RT_Q routed ones, so most slices reach a bucket both routed and through the
    bucket's direct group (the first-arrival f1 after a tile's slice set overflows).  Bit-exact
    incl. f1 against the oracle."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(150_000, 2048, rate=1 << 14, ooo=1000)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(100), ("sum", "count"), first=True, lateness=lateness,
                max_open_slices=48)   # ~11 windows open behind the watermark, plus lateness
    f1 = np.arange(len(keys), dtype=np.int64) * 11 + 5
    _run_both(hip, oracle_engine, cfg, keys, ts, vals, 1 << 14, 150, ["sum_i64", "count"], first=True, f1=f1)


@pytest.mark.parametrize("mode", MODES)
def test_purging_trigger_lateness(hip, oracle_engine, mode):
    from flink_amd.windowing import EventTimeTrigger, PurgingTrigger, TumblingEventTimeWindows
    keys, ts, vals = gen_stream(80_000, 500, rate=1 << 14, ooo=400)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(500), ("sum", "max"), first=True, lateness=300,
               trigger=PurgingTrigger.of(EventTimeTrigger.create()))
    sg, so = _run_both(hip, oracle_engine, cfg, keys, ts, vals, 1000, 100, ["sum_i64", "max_i64"], first=True)
    assert so["late_fires"] > 0 and sg["late_fires"] == so["late_fires"]


def test_java_double_min_max_semantics(hip, oracle_engine):
    """Math.min/Math.max: NaN wins, -0.0 < +0.0 (never fmin/fmax)."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys = np.array([1, 1, 2, 2, 3, 3, 4], np.int64)
    ts = np.array([10, 20, 10, 20, 10, 20, 30], np.int64)
    vals = np.array([0.0, -0.0, 1.5, float("nan"), -0.0, 0.0, float("-inf")], np.float64)
    cfg = _cfg(TumblingEventTimeWindows.of(100), ("min", "max", "count"), "f64")
    eg, eo = hip(cfg), oracle_engine(cfg)
    for e in (eg, eo):
        e.push(keys, ts, vals)
        e.advance_watermark(1000)
    rg, ro = eg.collect(), eo.collect()
    def rows(r):
        return sorted((int(r["key"][i]), np.float64(r["min_f64"][i]).tobytes() if not np.isnan(r["min_f64"][i]) else b"nan",
                       np.float64(r["max_f64"][i]).tobytes() if not np.isnan(r["max_f64"][i]) else b"nan",
                       int(r["count"][i])) for i in range(r["n"]))
    assert rows(rg) == rows(ro)
    eg.close(); eo.close()


@pytest.mark.parametrize("mode", MODES)
def test_extreme_keys_and_timestamps(hip, oracle_engine, mode):
    """Long.MIN_VALUE / MAX_VALUE keys, negative timestamps, the cleanup-time clamp."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys = np.array([-(1 << 63), LONG_MAX, 0, -1, 1 << 32, -(1 << 63), 7], np.int64)
    ts = np.array([-5000, -5000, -1, 0, 999, -4999, LONG_MAX - 10], np.int64)
    vals = np.array([1, 2, 3, 4, 5, 6, 7], np.int64)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000, -300), ("sum", "count"), lateness=5000)
    eg, eo = hip(cfg), oracle_engine(cfg)
    rg = drive(eg, keys, ts, vals, 7, 0, LONG_MAX)
    ro = drive(eo, keys, ts, vals, 7, 0, LONG_MAX)
    _compare(epochs_of(rg, ["sum_i64", "count"]), epochs_of(ro, ["sum_i64", "count"]), None)
    eg.close(); eo.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("size,offset", [(1000, -300), (700, 0), (1000, 250)])
def test_tumbling_negative_timestamps_dense(hip, oracle_engine, mode, size, offset):
    """In-order and shuffled runs across ts < offset - size, where Java's truncating % assigns a window
    not containing ts (TimeWindow.java:239-241): the per-wave slice shortcut must not apply there."""
    from flink_amd.windowing import TumblingEventTimeWindows
    n = 120_000
    i = np.arange(n, dtype=np.int64)
    ts = -40_000 + (i * 80_000) // n
    mix = (i // 4096) % 3 == 1                       # every third tile shuffled within +-3 s
    rng = np.random.default_rng(7)
    ts[mix] += rng.integers(-3000, 3000, mix.sum())
    keys = rng.integers(0, 3000, n).astype(np.int64)
    vals = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(size, offset), ("sum", "count"), lateness=2000,
                max_open_slices=64)
    _run_both(hip, oracle_engine, cfg, keys, ts, vals, 8192, 1000, ["sum_i64", "count"])


def test_missing_timestamp_fails(hip):
    from flink_amd import _abi
    from flink_amd.windowing import TumblingEventTimeWindows
    e = hip(_cfg(TumblingEventTimeWindows.of(1000)))
    e.push(np.array([1, 2], np.int64), np.array([5, -(1 << 63)], np.int64), np.array([1, 1], np.int64))
    with pytest.raises(_abi.FwError, match="Long.MIN_VALUE timestamp"):
        e.sync()
    e.close()


def test_foreign_key_group_fails(hip):
    from flink_amd import _abi
    from flink_amd.windowing import TumblingEventTimeWindows
    e = hip(_cfg(TumblingEventTimeWindows.of(1000), max_parallelism=128, key_group_range=(0, 0)))
    e.push(np.array([42], np.int64), np.array([5], np.int64), np.array([1], np.int64))
    with pytest.raises(_abi.FwError, match="Unexpected key group index"):
        e.sync()
    e.close()


@pytest.mark.parametrize("mode", MODES)
def test_device_resident_input(hip, oracle_engine, mode):
    """Columns already in HBM (torch tensors): no host copy on the push path."""
    import torch
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(50_000, 777, rate=1 << 14)
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000), first=True)
    eg = hip(cfg)
    dk, dt, dv = (torch.from_numpy(a).cuda() for a in (keys, ts, vals))
    out = []
    for s in range(0, len(keys), 10_000):
        eg.push(dk[s:s + 10_000], dt[s:s + 10_000], dv[s:s + 10_000])
        eg.advance_watermark(int(ts[:s + 10_000].max()) - 1)
        out.append(eg.collect())
    eg.advance_watermark(LONG_MAX)
    out.append(eg.collect())
    eo = oracle_engine(cfg)
    ro = drive(eo, keys, ts, vals, 10_000, 1, LONG_MAX)
    _compare(epochs_of(out, ["sum_i64"], True), epochs_of(ro, ["sum_i64"], True), None)
    eg.close(); eo.close()


def test_partition_by_operator_matches_key_group_routing(hip):
    """fw_partition_by_operator = KeyGroupStreamPartitioner routing, stable per destination."""
    import ctypes
    import torch
    from flink_amd.keygroups import operator_index_np
    from flink_amd.windowing import TumblingEventTimeWindows
    e = hip(_cfg(TumblingEventTimeWindows.of(1000)))
    keys, ts, vals = gen_stream(100_003, 1 << 20, rate=1 << 14)
    d = {n: torch.from_numpy(a).cuda() for n, a in (("k", keys), ("t", ts), ("v", vals))}
    ok, of1, ot, ov = (torch.empty_like(d["k"]) for _ in range(4))
    okh = torch.empty(len(keys), dtype=torch.int32, device="cuda")
    counts = torch.zeros(8, dtype=torch.int64, device="cuda")
    offs = torch.zeros(8, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = e.lib.fw_partition_by_operator(e.h, P(d["k"]), None, None, P(d["t"]), P(d["v"]), len(keys), 128, 8,
                                        P(ok), P(okh), P(of1), P(ot), P(ov), P(counts), P(offs))
    assert rc == 0
    e.sync()
    dest = operator_index_np(keys, 128, 8)
    order = np.argsort(dest, kind="stable")
    assert np.array_equal(ok.cpu().numpy(), keys[order])
    assert np.array_equal(ov.cpu().numpy(), vals[order])
    assert np.array_equal(ot.cpu().numpy(), ts[order])
    assert np.array_equal(counts.cpu().numpy(), np.bincount(dest, minlength=8))
    e.close()


@pytest.mark.parametrize("last", range(8))
def test_partition_by_operator_last_rotated_order(hip, last):
    """fw_partition_by_operator_last at parallelism 8 (the keyBy exchange's form, keyby.py): destinations in the
    rotated order last+1 .. 7, 0 .. last (keyby.py _dest_order), each stable, counts indexed by operator and
    offsets[d] the start of operator d's run; keys routed by KeyGroupStreamPartitioner (maxParallelism 128)."""
    import ctypes
    import torch
    from flink_amd.keygroups import operator_index_np
    from flink_amd.windowing import TumblingEventTimeWindows
    e = hip(_cfg(TumblingEventTimeWindows.of(1000)))
    keys, ts, vals = gen_stream(70_001 + 37 * last, 1 << 20, rate=1 << 14, seed=3 + last)
    d = {n: torch.from_numpy(a).cuda() for n, a in (("k", keys), ("t", ts), ("v", vals))}
    ok, ot, ov = (torch.empty_like(d["k"]) for _ in range(3))
    counts = torch.zeros(8, dtype=torch.int64, device="cuda")
    offs = torch.zeros(8, dtype=torch.int64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = e.lib.fw_partition_by_operator_last(e.h, P(d["k"]), None, None, P(d["t"]), P(d["v"]), len(keys), 128, 8,
                                             P(ok), None, None, P(ot), P(ov), P(counts), P(offs), last)
    assert rc == 0
    e.sync()
    dest = operator_index_np(keys, 128, 8)
    rank = (dest - (last + 1)) % 8            # position of each destination in the rotated order
    order = np.argsort(rank, kind="stable")
    assert np.array_equal(ok.cpu().numpy(), keys[order])
    assert np.array_equal(ot.cpu().numpy(), ts[order])
    assert np.array_equal(ov.cpu().numpy(), vals[order])
    cnt = np.bincount(dest, minlength=8)
    assert np.array_equal(counts.cpu().numpy(), cnt)
    rot = [(last + 1 + i) % 8 for i in range(8)]
    start, want = 0, np.zeros(8, np.int64)
    for dd in rot:
        want[dd] = start
        start += cnt[dd]
    assert np.array_equal(offs.cpu().numpy(), want)
    e.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_host_buffers_reusable_after_push(hip, oracle_engine, mode, pinned):
    """fw_push_batch(FW_MEM_HOST) returns once the columns are on the device (flink_window.h): the caller
    overwrites its arrays right after each push (as a JNI caller releasing its critical arrays would) and the
    results still equal the oracle's on the true stream."""
    import torch
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(200_000, 3000, rate=1 << 15)
    batch = 1 << 14
    cfg = _cfgm(mode, TumblingEventTimeWindows.of(1000), ("sum", "count"), first=True)
    eg = hip(cfg)
    bufs = [torch.empty(batch, dtype=torch.int64) for _ in range(3)]
    if pinned:
        bufs = [b.pin_memory() for b in bufs]
    out, max_ts = [], -(1 << 63)
    for s in range(0, len(keys), batch):
        e = min(len(keys), s + batch)
        m = e - s
        for b, src in zip(bufs, (keys, ts, vals)):
            b[:m].copy_(torch.from_numpy(src[s:e]))
        eg.push(bufs[0][:m], bufs[1][:m], bufs[2][:m])
        for b in bufs:
            b.fill_(-7)   # the caller's arrays reused at once
        max_ts = max(max_ts, int(ts[s:e].max()))
        eg.advance_watermark(max_ts - 1)
        out.append(eg.collect())
    eg.advance_watermark(LONG_MAX)
    out.append(eg.collect())
    eg.close()
    eo = oracle_engine(cfg)
    ro = drive(eo, keys, ts, vals, batch, 1, LONG_MAX)
    eo.close()
    _compare(epochs_of(out, ["sum_i64", "count"], True), epochs_of(ro, ["sum_i64", "count"], True), None)
