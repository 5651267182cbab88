"""WindowedStream.apply(WindowFunction) over list state (FW_AGG_LIST, fw_list.hip): the reference's known answers
(WindowOperatorTest sliding / tumbling Apply tests and the list-state cleanup timer, tests/golden/list_*.json) and
parity with the oracle's HeapListState: every (key, window) group holds the same elements in the same arrival
order (bit-exact, doubles included: elements are passed through, not combined).
"""
import numpy as np
import pytest

from harness import LIST_FIXTURES, expected_epochs, gen_stream, load_golden, replay

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


@pytest.mark.parametrize("name", LIST_FIXTURES)
def test_list_golden_fixture(hip, name):
    fx = load_golden(name)
    assert replay(fx, hip) == expected_epochs(fx), fx["source"]


def _groups(res, vt):
    """Per watermark epoch: {(key, window maxTimestamp): [(f1, value) in output order]}; checks contiguity."""
    vals = res["sum_i64"] if vt == "i64" else res["sum_f64"]
    epochs, pos = [], 0
    for wm, mp in list(zip(res["mark_wm"].tolist(), res["mark_pos"].tolist())) + [(None, res["n"])]:
        g, last = {}, None
        for i in range(pos, mp):
            k = (int(res["key"][i]), int(res["ts"][i]))
            assert k == last or k not in g, "a (key, window) group split in the output"
            g.setdefault(k, []).append((int(res["f1"][i]), vals[i].item()))
            last = k
        epochs.append((wm, g))
        pos = mp
    return epochs


def _drive(eng, keys, ts, vals, batch, lag, vt):
    out = []
    mx = -(1 << 63)
    for s in range(0, len(keys), batch):
        e = min(len(keys), s + batch)
        eng.push(keys[s:e], ts[s:e], vals[s:e], f1=np.arange(s, e, dtype=np.int64))
        mx = max(mx, int(ts[s:e].max()))
        eng.advance_watermark(mx - lag)
        out += _groups(eng.collect(), vt)
    eng.advance_watermark(LONG_MAX)
    out += _groups(eng.collect(), vt)
    return out


@pytest.mark.parametrize("assigner,vt", [("tumbling", "i64"), ("sliding", "i64"), ("sliding_uneven", "f64")])
def test_list_parity(hip, oracle_engine, assigner, vt):
    from flink_amd.windowing import (ListStateDescriptor, SlidingEventTimeWindows, TumblingEventTimeWindows,
                                     make_config)
    a = {"tumbling": TumblingEventTimeWindows.of(1000), "sliding": SlidingEventTimeWindows.of(3000, 1000),
         "sliding_uneven": SlidingEventTimeWindows.of(2500, 1000, 300)}[assigner]
    keys, ts, vals = gen_stream(60000, 400, rate=1 << 13, ooo=200, value_type=vt)
    cfg = make_config(a, ListStateDescriptor(vt), max_parallelism=128, key_capacity=1 << 11, max_batch=1 << 13,
                      out_capacity=1 << 19)
    res = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        res.append(_drive(e, keys, ts, vals, 4096, 300, vt))
        st = e.stats()
        e.close()
        res[-1].append(("stats", (st["panes_fired"], st["records_late"])))
    g, o = res
    assert g == o
    assert sum(len(x) for _, x in g[:-1]) > 1000


def _fires(res, vt):
    """Per watermark epoch: the sorted list of fires (key, window maxTimestamp, ((f1, value), ...)).  A fire's
    elements come in arrival order (f1 = arrival index here), so a fire of the same (key, window) right after
    another one starts where f1 drops."""
    vals = res["sum_i64"] if vt == "i64" else res["sum_f64"]
    epochs, pos = [], 0
    for wm, mp in list(zip(res["mark_wm"].tolist(), res["mark_pos"].tolist())) + [(None, res["n"])]:
        fires, cur, last = [], None, None
        for i in range(pos, mp):
            k = (int(res["key"][i]), int(res["ts"][i]))
            f1 = int(res["f1"][i])
            if cur is None or k != cur[0] or f1 <= last:
                cur = (k, [])
                fires.append(cur)
            cur[1].append((f1, vals[i].item()))
            last = f1
        epochs.append((wm, sorted((k[0], k[1], tuple(el)) for k, el in fires)))
        pos = mp
    return epochs


@pytest.mark.parametrize("assigner", ["tumbling", "sliding", "sliding_uneven"])
def test_list_late_refires(hip, oracle_engine, assigner):
    """Allowed lateness over list state: an element for a window that already fired is added and re-fires the
    window for its key with every element so far (EventTimeTrigger.onElement FIRE, WindowOperator.java:302-333);
    later elements of the same key re-fire it again, each with the list up to itself."""
    from flink_amd.windowing import (ListStateDescriptor, SlidingEventTimeWindows, TumblingEventTimeWindows,
                                     make_config)
    a = {"tumbling": TumblingEventTimeWindows.of(1000), "sliding": SlidingEventTimeWindows.of(3000, 1000),
         "sliding_uneven": SlidingEventTimeWindows.of(2500, 1000, 300)}[assigner]
    keys, ts, vals = gen_stream(40000, 300, rate=1 << 13, t0=10_000, ooo=900)   # (no ts below offset - slide)
    cfg = make_config(a, ListStateDescriptor("i64"), None, 600, max_parallelism=128, key_capacity=1 << 11,
                      max_batch=1 << 12, out_capacity=1 << 22)
    res = []
    for f in (hip, oracle_engine):
        e = f(cfg)
        out = []
        mx = -(1 << 63)
        for s0 in range(0, len(keys), 2048):
            s1 = min(len(keys), s0 + 2048)
            e.push(keys[s0:s1], ts[s0:s1], vals[s0:s1], f1=np.arange(s0, s1, dtype=np.int64))
            mx = max(mx, int(ts[s0:s1].max()))
            e.advance_watermark(mx - 100)
            out += _fires(e.collect(), "i64")
        e.advance_watermark(LONG_MAX)
        out += _fires(e.collect(), "i64")
        st = e.stats()
        e.close()
        res.append((out, (st["panes_fired"], st["late_fires"], st["records_late"])))
    (g, sg), (o, so) = res
    assert len(g) == len(o)
    for (wg, xg), (wo, xo) in zip(g, o):
        assert wg == wo and xg == xo, wg
    assert sg == so and so[1] > 100


def test_list_operator_window_function(hip, oracle_engine):
    """The operator surface: apply(WindowFunction) receiving each key's elements of a window in arrival order
    (the reference's PassThroughFunction2 joins them into a string, WOT:1933-1940)."""
    from flink_amd.windowing import (ListStateDescriptor, StreamRecord, TumblingEventTimeWindows, Watermark,
                                     WindowOperator)

    def got(key, window, elements, out):
        out.collect("GOT: " + ",".join(f"({k},{v})" for k, v in elements))

    outs = []
    for f in (hip, oracle_engine):
        op = WindowOperator(TumblingEventTimeWindows.of(2000), ListStateDescriptor(), window_function=got,
                            engine_factory=f, max_parallelism=128, key_capacity=64, max_batch=64, out_capacity=1024)
        for v, t in [(1, 10), (2, 1500), (3, 700), (4, 2100)]:
            op.processElement(StreamRecord(("key2", v), t))
        op.processElement(StreamRecord(("key1", 9), 50))
        op.processWatermark(Watermark(1999))
        op.processWatermark(Watermark(5000))
        outs.append([(x.value, x.timestamp) if isinstance(x, StreamRecord) else ("wm", x.timestamp)
                     for x in op.getOutput()])
        op.close()
    g, o = outs
    assert sorted(g[:2]) == sorted(o[:2]) and g[2:] == o[2:]
    assert sorted(g[:2]) == [("GOT: (key1,9)", 1999), ("GOT: (key2,1),(key2,2),(key2,3)", 1999)]
    assert g[2:] == [("wm", 1999), ("GOT: (key2,4)", 3999), ("wm", 5000)]


def test_list_rejections(hip):
    from flink_amd import _abi
    from flink_amd.windowing import ListStateDescriptor, TumblingEventTimeWindows, make_config
    e = hip(make_config(TumblingEventTimeWindows.of(1000), ListStateDescriptor(), None, 500, key_capacity=64,
                        max_batch=64, out_capacity=1024))
    e.push(np.array([1], np.int64), np.array([100], np.int64), np.array([1], np.int64))
    with pytest.raises(_abi.FwError, match="list state"):
        e.snapshot_kg(0)
    e.close()
    # PurgingTrigger: a re-fire would purge one window of slices other windows share
    from flink_amd.windowing import EventTimeTrigger, PurgingTrigger
    e = hip(make_config(TumblingEventTimeWindows.of(1000), ListStateDescriptor(), PurgingTrigger.of(EventTimeTrigger.create()),
                        500, key_capacity=64, max_batch=64, out_capacity=1024))
    e.push(np.array([1], np.int64), np.array([100], np.int64), np.array([1], np.int64))
    e.advance_watermark(1200)   # window [0, 1000) fired, kept for the lateness
    e.collect()
    e.push(np.array([1], np.int64), np.array([200], np.int64), np.array([1], np.int64))   # would re-fire it
    with pytest.raises(_abi.FwError) as ei:
        e.collect()
    assert ei.value.code == _abi.FW_ERR_UNSUPPORTED
    e.close()
