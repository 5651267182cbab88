"""The operator surface: the reference's golden vectors driven through flink_amd.windowing.WindowOperator
exactly as WindowOperatorTest drives its KeyedOneInputStreamOperatorTestHarness
(SJT/runtime/operators/windowing/WindowOperatorTest.java:92-157): processElement(StreamRecord(Tuple2
("key1", 1), ts)), processWatermark(Watermark(t)), then getOutput() compared with
TestHarnessUtil.assertOutputEqualsSorted (SJT/util/TestHarnessUtil.java:80-117: watermark positions
exact, records between two watermarks as a sorted multiset).

String keys "key1"/"key2" (their Java String.hashCode() is what the fixtures' key_hash column holds);
the closed-form ITCase fixtures use Long keys.  The CPU variant puts the oracle behind the surface
(tests the host mirror); the GPU variant the HIP engine.
"""
import pytest

from harness import WINDOW_FIXTURES, fixture_events, load_golden
from flink_amd.windowing import (EventTimeTrigger, PurgingTrigger, ReduceFunction, SlidingEventTimeWindows,
                                 StreamRecord, TumblingEventTimeWindows, Watermark, WindowOperator,
                                 java_string_hash)


def _operator(fx, engine_factory):
    c = fx["config"]
    if c["assigner"] == "tumbling":
        assigner = TumblingEventTimeWindows.of(c["size"], c["offset"] or None)
    else:
        assigner = SlidingEventTimeWindows.of(c["size"], c["slide"], c["offset"] or None)
    trigger = EventTimeTrigger.create() if c["trigger"] == "event_time" else PurgingTrigger.of(EventTimeTrigger.create())
    reduce = ReduceFunction(tuple(c["agg"]), c["value_type"], c["keep_first_f1"])
    kw = dict(max_parallelism=c["max_parallelism"], key_capacity=1024, max_batch=1 << 12, out_capacity=1 << 16)
    if engine_factory is not None:
        kw["engine_factory"] = engine_factory
    return WindowOperator(assigner, reduce, trigger, c["allowed_lateness"], **kw)


def _key_of(fx, k):
    if fx.get("key_hash"):
        name = f"key{k}"
        assert java_string_hash(name) == fx["key_hash"][str(k)]
        return name
    return k


def assert_output_equals_sorted(expected, actual):
    """TestHarnessUtil.assertOutputEqualsSorted: watermarks at the same positions; the records between
    two watermarks compared as sorted lists."""
    def epochs(out):
        ep, cur = [], []
        for e in out:
            if isinstance(e, Watermark):
                ep.append((e.timestamp, sorted((r.value, r.timestamp) for r in cur)))
                cur = []
            else:
                cur.append(e)
        ep.append((None, sorted((r.value, r.timestamp) for r in cur)))
        return ep
    assert epochs(actual) == epochs(expected)


def replay_operator(fx, engine_factory):
    op = _operator(fx, engine_factory)
    for e in fixture_events(fx):
        if e[0] == "rec":
            _, k, v, ts = e
            op.processElement(StreamRecord((_key_of(fx, k), v), ts))
        else:
            op.processWatermark(Watermark(e[1]))
    expected = []
    for x in fx["expected"]:
        expected += [StreamRecord((_key_of(fx, k), v), ts) for k, v, ts in x["records"]]
        expected.append(Watermark(x["wm"]))
    out = op.getOutput()
    op.close()
    return expected, out


@pytest.mark.parametrize("name", WINDOW_FIXTURES)
def test_operator_surface_oracle(name):
    from oracle.oracle import OracleEngine
    fx = load_golden(name)
    expected, out = replay_operator(fx, OracleEngine)
    assert_output_equals_sorted(expected, out)


@pytest.mark.gpu
@pytest.mark.parametrize("name", WINDOW_FIXTURES)
def test_operator_surface_hip(name):
    from flink_amd import _abi
    _abi.load_library()
    fx = load_golden(name)
    expected, out = replay_operator(fx, None)
    assert_output_equals_sorted(expected, out)


def test_mixed_key_types_rejected():
    from oracle.oracle import OracleEngine
    op = WindowOperator(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",)), engine_factory=OracleEngine)
    op.processElement(StreamRecord(("a", 1), 5))
    with pytest.raises(TypeError):
        op.processElement(StreamRecord((7, 1), 5))
    with pytest.raises(TypeError):
        op.processElement(StreamRecord(((1, 2), 1), 5))
    op.close()
