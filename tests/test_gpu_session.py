"""Session windows on the HIP engine (fw_session.hip): the reference's known answers (WindowOperatorTest
session tests, tests/golden/session_*.json) and bit-exact parity with the oracle on random out-of-order streams
(integer sum / min / max / count and the window start; double sums within relative 1e-9).
"""
import numpy as np
import pytest

from harness import SESSION_FIXTURES, drive, epochs_of, expected_epochs, load_golden, replay
from test_session_oracle import session_stream

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1


@pytest.fixture(scope="module")
def hip():
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    _abi.load_library()
    return WindowEngine


@pytest.fixture(scope="module")
def oracle_engine():
    from oracle.oracle import OracleEngine
    return OracleEngine


@pytest.mark.parametrize("name", SESSION_FIXTURES)
def test_session_golden_fixture(hip, name):
    fx = load_golden(name)
    got = replay(fx, hip)
    assert got == expected_epochs(fx), fx["source"]


def _cfg(gap, fields, vt="i64", lateness=0, purging=False, **kw):
    from flink_amd.windowing import (EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, ReduceFunction,
                                     make_config)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else EventTimeTrigger.create()
    args = dict(max_parallelism=128, key_capacity=4096, max_batch=1 << 14, out_capacity=1 << 20)
    args.update(kw)
    return make_config(EventTimeSessionWindows.withGap(gap), ReduceFunction(fields, vt), trig, lateness, **args)


def _both(hip, oracle_engine, cfg, keys, ts, vals, batch, lag, fields, rel=0.0):
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, batch, lag, LONG_MAX)
        st = e.stats()
        e.close()
        out.append((epochs_of(r, fields + ["win_start"]), st))
    (g, sg), (o, so) = out
    assert len(g) == len(o)
    for (wg, rg), (wo, ro) in zip(g, o):
        assert wg == wo and len(rg) == len(ro), (wg, len(rg), len(ro))
        if rel == 0.0:
            assert rg == ro, wg
        else:
            for x, y in zip(rg, ro):
                for u, v in zip(x, y):
                    if isinstance(u, float):
                        assert abs(u - v) <= rel * max(1.0, abs(v)), (wg, x, y)
                    else:
                        assert u == v, (wg, x, y)
    assert sg["records_late"] == so["records_late"] and sg["panes_fired"] == so["panes_fired"]
    assert sg["late_fires"] == so["late_fires"]
    return g


@pytest.mark.parametrize("lateness,purging", [(0, False), (0, True), (150, False), (150, True), (5000, False),
                                              (5000, True)])
def test_session_parity_int(hip, oracle_engine, lateness, purging):
    fields = ["sum_i64", "min_i64", "max_i64", "count"]
    keys, ts, vals = session_stream(60000, 500, 11 + lateness, 600000, 400)
    cfg = _cfg(100, ("sum", "min", "max", "count"), lateness=lateness, purging=purging)
    g = _both(hip, oracle_engine, cfg, keys, ts, vals, 4096, 150, fields)
    assert sum(len(r) for _, r in g) > 1000


def test_session_parity_double(hip, oracle_engine):
    fields = ["sum_f64", "min_f64", "max_f64", "count"]
    keys, ts, _ = session_stream(40000, 300, 5, 400000, 300)
    vals = np.random.default_rng(3).random(len(keys))
    vals[::97] = -0.0
    cfg = _cfg(120, ("sum", "min", "max", "count"), vt="f64", lateness=100)
    _both(hip, oracle_engine, cfg, keys, ts, vals, 4096, 100, fields, rel=1e-9)


def test_session_hot_keys_and_batches(hip, oracle_engine):
    """Few keys, large batches: long per-key runs walked in arrival order, many merges per batch."""
    fields = ["sum_i64", "count"]
    keys, ts, vals = session_stream(1 << 16, 7, 21, 200000, 2000)
    cfg = _cfg(400, ("sum", "count"), lateness=300, max_batch=1 << 16, max_open_slices=64)
    _both(hip, oracle_engine, cfg, keys, ts, vals, 1 << 15, 500, fields)


def test_session_extreme_timestamps(hip, oracle_engine):
    """Long.MIN_VALUE timestamps are legal for sessions (no assigner check); ts + gap wraps near Long.MAX_VALUE."""
    keys = np.array([1, 1, 2, 2, 3, 3], np.int64)
    ts = np.array([-(1 << 63), -(1 << 63) + 5, LONG_MAX - 3, LONG_MAX - 50, 0, 5], np.int64)
    vals = np.arange(6, dtype=np.int64) + 1
    cfg = _cfg(10, ("sum", "count"))
    _both(hip, oracle_engine, cfg, keys, ts, vals, 6, 0, ["sum_i64", "count"])


def _red_cfg(gap, red, lateness=0, purging=False, **kw):
    from flink_amd.windowing import EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, make_config
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else EventTimeTrigger.create()
    args = dict(max_parallelism=128, key_capacity=4096, max_batch=1 << 14, out_capacity=1 << 20)
    args.update(kw)
    return make_config(EventTimeSessionWindows.withGap(gap), red, trig, lateness, **args)


def _merge_heavy_stream(n, n_keys, seed, gap):
    """Out-of-order records whose sessions keep bridging earlier ones: many merges of 2+ windows (the HashSet
    order of the merged windows decides the state window, f1 and the reduce order)."""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, n_keys, n).astype(np.int64)
    base = np.sort(rng.integers(0, max(1, int(n / n_keys * gap * 0.8)), n)).astype(np.int64)   # ~0.8 gap apart per key
    ts = base - rng.integers(0, 4 * gap, n).astype(np.int64)
    vals = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    return keys, ts, vals


@pytest.mark.parametrize("lateness,purging", [(0, False), (300, False), (300, True)])
def test_session_first_arrival_f1(hip, oracle_engine, lateness, purging):
    """Tuple3.of(a.f0, a.f1, a.f2 + b.f2): f1 of the merge target's state (MergingWindowSet.addWindow takes the
    state window of the first merged window in HashSet order, MergingWindowSet.java:142-214) — bit-exact."""
    from flink_amd.windowing import ReduceFunction
    keys, ts, vals = _merge_heavy_stream(30000, 200, 5 + lateness, 40)
    f1 = np.arange(len(keys), dtype=np.int64) * 7 + 3
    cfg = _red_cfg(40, ReduceFunction(("sum", "count"), "i64", keep_first_f1=True), lateness, purging)
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, 2048, 60, LONG_MAX, f1=f1)
        out.append((epochs_of(r, ["sum_i64", "count", "win_start"], f1=True), e.stats()))
        e.close()
    (g, sg), (o, so) = out
    assert g == o
    assert sg["panes_fired"] == so["panes_fired"] > 1000


def test_session_double_sums_exact(hip, oracle_engine):
    """Double sums reduce in the reference's order (sources in HashSet order, then into the target): bit-exact."""
    from flink_amd.windowing import ReduceFunction
    keys, ts, _ = _merge_heavy_stream(30000, 150, 9, 50)
    vals = np.random.default_rng(4).random(len(keys)) * 1e6
    cfg = _red_cfg(50, ReduceFunction(("sum", "min", "max", "count"), "f64", keep_first_f1=True), 100)
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, 2048, 80, LONG_MAX)
        out.append(epochs_of(r, ["sum_f64", "min_f64", "max_f64", "count", "win_start"], f1=True))
        e.close()
    assert out[0] == out[1]


@pytest.mark.parametrize("field,first", [("maxBy", True), ("maxBy", False), ("minBy", True), ("minBy", False)])
def test_session_max_by(hip, oracle_engine, field, first):
    """maxBy / minBy over merging windows: the extremal record, ties by argument order of the reduce
    (ComparableAggregator.java:74-81) — values drawn from a small range so ties are common."""
    from flink_amd.windowing import ReduceFunction
    keys, ts, _ = _merge_heavy_stream(20000, 100, 13, 40)
    vals = np.random.default_rng(6).integers(0, 8, len(keys)).astype(np.int64)
    f1 = np.arange(len(keys), dtype=np.int64)
    cfg = _red_cfg(40, ReduceFunction((field,), "i64", first=first), 200)
    col = "max_i64" if field == "maxBy" else "min_i64"
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, 2048, 60, LONG_MAX, f1=f1)
        out.append(epochs_of(r, [col, "win_start"], f1=True))
        e.close()
    assert out[0] == out[1]


def _list_groups(results):
    """Per watermark mark: {(key, window maxTimestamp, window start): [(f1, value) in emitted order]} — the
    element order of a window is its list order (HeapListState), the order between windows unspecified."""
    ep = []
    for res in results:
        pos = 0
        for wm, mp in list(zip(res["mark_wm"], res["mark_pos"])) + [(None, res["n"])]:
            groups = {}
            for j in range(pos, int(mp)):
                g = (int(res["key"][j]), int(res["ts"][j]), int(res["win_start"][j]))
                groups.setdefault(g, []).append((int(res["f1"][j]), int(res["sum_i64"][j])))
            if wm is not None or groups:
                ep.append((None if wm is None else int(wm), groups))
            pos = int(mp)
    return ep


@pytest.mark.parametrize("lateness,purging", [(0, False), (200, False), (200, True)])
def test_session_list_state(hip, oracle_engine, lateness, purging):
    """WindowedStream.apply over EventTimeSessionWindows (the reference's testSessionWindows shape): each
    window's elements in list order — a merge appends the sources' lists to the target's in HashSet order
    (AbstractKeyedStateBackend.mergePartitionedStates :315-333) — grouped per window, bit-exact."""
    from flink_amd.windowing import ListStateDescriptor
    keys, ts, vals = _merge_heavy_stream(20000, 150, 21 + lateness, 40)
    f1 = np.arange(len(keys), dtype=np.int64) + 100
    cfg = _red_cfg(40, ListStateDescriptor("i64", list_capacity=1 << 16), lateness, purging)
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, 2048, 60, LONG_MAX, f1=f1)
        out.append((_list_groups(r), e.stats()))
        e.close()
    (g, sg), (o, so) = out
    assert len(g) == len(o)
    for (wg, xg), (wo, xo) in zip(g, o):
        assert wg == wo and xg == xo, wg
    assert sg["panes_fired"] == so["panes_fired"] > 500
    assert sg["records_late"] == so["records_late"]


def test_session_list_capacity(hip):
    """More buffered elements than list_capacity: FW_ERR_CAPACITY, not a wrong answer."""
    from flink_amd import _abi
    from flink_amd.windowing import ListStateDescriptor
    e = hip(_red_cfg(1000, ListStateDescriptor("i64", list_capacity=64)))
    n = 200   # one key, one long session: every element stays buffered
    e.push(np.ones(n, np.int64), np.arange(n, dtype=np.int64), np.ones(n, np.int64))
    with pytest.raises(_abi.FwError) as ei:
        e.collect()
    assert ei.value.code == _abi.FW_ERR_CAPACITY
    e.close()


def test_session_list_pool_reuse(hip, oracle_engine):
    """list_capacity bounds the elements buffered AT ONCE: one long session (key 0, a record every
    100 ms, gap 1 s) stays open over 40 batches while 60 new keys per batch open short sessions that the watermark
    closes a second later.  2,440 arrivals pass through a 1,024-entry pool with at most ~700 elements live; the
    pool reuses the entries of purged windows (an arrival-ordinal ring would have failed at the 1,025th arrival
    while key 0's first element is still buffered)."""
    from flink_amd.windowing import ListStateDescriptor
    keys, ts = [], []
    for b in range(40):
        keys += [0] + list(range(1 + 60 * b, 61 + 60 * b))
        ts += [100 * b] + [100 * b + 1 + j for j in range(60)]
    keys, ts = np.array(keys, np.int64), np.array(ts, np.int64)
    vals = np.arange(len(keys), dtype=np.int64) * 3 - 7
    f1 = np.arange(len(keys), dtype=np.int64) + 100
    cfg = _red_cfg(1000, ListStateDescriptor("i64", list_capacity=1024))
    out = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        r = drive(e, keys, ts, vals, 61, 0, LONG_MAX, f1=f1)
        out.append(_list_groups(r))
        e.close()
    g, o = out
    assert g == o
    assert max(len(x) for _, grp in g for x in grp.values()) == 40   # key 0's one session, every element


def test_session_rejections(hip):
    from flink_amd import _abi
    e = hip(_cfg(10, ("sum",)))
    e.push(np.array([1], np.int64), np.array([5], np.int64), np.array([1], np.int64))
    with pytest.raises(_abi.FwError, match="session"):
        e.snapshot_kg(0)
    e.close()


@pytest.mark.parametrize("slots,batch,lag", [(100, 200, 8000), (256, 500, 30_000)])
def test_session_many_in_flight(hip, oracle_engine, slots, batch, lag):
    """Far more in-flight sessions per key than one 64-bit slot mask holds (MergingWindowSet has no bound;
    the engine takes up to 256 per key): a slow watermark over hot keys with short gaps, and late records that
    bridge sessions, against the oracle."""
    rng = np.random.default_rng(slots)
    n = 6000   # ~200 ms apart per key, gap 20: nearly every record a session; at most 84 / 240 in flight per key
    keys = rng.integers(0, 6, n).astype(np.int64)
    ts = (np.sort(rng.integers(0, 200_000, n)) - rng.integers(0, 3000, n)).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    cfg = _cfg(20, ("sum", "count"), lateness=400, max_open_slices=slots, max_batch=1 << 14)
    g = _both(hip, oracle_engine, cfg, keys, ts, vals, batch, lag, ["sum_i64", "count"])
    assert sum(len(r) for _, r in g) > 1000
    if slots == 100:   # the same stream with 64 slots runs out of them: the test does exceed one mask word
        from flink_amd import _abi
        e = hip(_cfg(20, ("sum", "count"), lateness=400, max_open_slices=64, max_batch=1 << 14))
        with pytest.raises(_abi.FwError) as ei:
            drive(e, keys, ts, vals, batch, lag, LONG_MAX)
        assert ei.value.code == _abi.FW_ERR_CAPACITY
        e.close()


def test_session_capacity_error(hip):
    """More in-flight sessions for one key than the engine's slots: FW_ERR_CAPACITY, not a wrong answer."""
    from flink_amd import _abi
    e = hip(_cfg(10, ("sum",), max_open_slices=4))
    ts = np.arange(0, 1000, 100, dtype=np.int64)   # ten disjoint sessions of key 1 in flight, 4 slots
    e.push(np.ones(len(ts), np.int64), ts, np.ones(len(ts), np.int64))
    with pytest.raises(_abi.FwError) as ei:
        e.collect()
    assert ei.value.code == _abi.FW_ERR_CAPACITY
    e.close()
