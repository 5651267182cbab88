"""WindowedStream.reduce(ReduceFunction, WindowFunction) / apply(reduce, function) (WindowedStream.java:347-425):
the pre-aggregated window path of EventTimeWindowCheckpointingITCase.testPreAggregatedTumblingTimeWindow /
testPreAggregatedSlidingTimeWindow (FT/checkpointing/EventTimeWindowCheckpointingITCase.java:344-485).
The source emits (key, i) at event time i for i = 0..2999 and 100 keys, a watermark i after every round
(FailingSource :495-579); the window function emits Tuple4(key, window.start, window.end, sum), which the
ValidatingSink (:582-686) checks: sum = sum of i over [start, end) with i > 0, and exactly
3000 / slide windows per key.  The reduce runs in the engine (oracle on CPU, HIP on the GPU), the
window function on the host per fired pane.
"""
import pytest

from flink_amd.windowing import (ReduceFunction, SlidingEventTimeWindows, StreamRecord, TumblingEventTimeWindows,
                                 Watermark, WindowOperator)

N_KEYS, N_ELEMENTS = 100, 3000


class Tuple4WindowFunction:
    """The ITCase's RichWindowFunction: for (key, sum) in input, collect (key, start, end, sum)."""

    def apply(self, key, window, inputs, out):
        for k, total in inputs:
            out.collect((k, window.getStart(), window.getEnd(), total))


def _run(assigner, engine_factory):
    kw = dict(max_parallelism=128, key_capacity=256, max_batch=1 << 12, out_capacity=1 << 16)
    if engine_factory is not None:
        kw["engine_factory"] = engine_factory
    op = WindowOperator(assigner, ReduceFunction(("sum",)), window_function=Tuple4WindowFunction(), **kw)
    for i in range(N_ELEMENTS):
        for k in range(N_KEYS):
            op.processElement(StreamRecord((k, i), i))
        op.processWatermark(Watermark(i))
    # no final MAX_WATERMARK: the ITCase's sink ends the job once every key has its expected windows, so
    # only windows with maxTimestamp <= 2999 (the last watermark) fire
    out = op.getOutput()
    op.close()
    return out


def _validate(out, size, slide):
    """ValidatingSink.invoke / close: per-window closed-form sums, exact window count per key, each
    result timestamped with window.maxTimestamp()."""
    counts = {}
    for e in out:
        if isinstance(e, Watermark):
            continue
        k, start, end, total = e.value
        assert end - start == size
        assert e.timestamp == end - 1
        assert total == sum(i for i in range(start, end) if i > 0), (start, end)
        counts[k] = counts.get(k, 0) + 1
    # numWindowsExpected = NUM_ELEMENTS_PER_KEY / WINDOW_SLIDE (EventTimeWindowCheckpointingITCase.java:410,485)
    expected = N_ELEMENTS // slide
    assert len(counts) == N_KEYS and set(counts.values()) == {expected}


@pytest.mark.parametrize("window", ["tumbling", "sliding"])
def test_pre_aggregated_window_function_oracle(window):
    from oracle.oracle import OracleEngine
    assigner = TumblingEventTimeWindows.of(100) if window == "tumbling" else SlidingEventTimeWindows.of(1000, 100)
    _validate(_run(assigner, OracleEngine), assigner.size, assigner.slide)


@pytest.mark.gpu
@pytest.mark.parametrize("window", ["tumbling", "sliding"])
def test_pre_aggregated_window_function_hip(window):
    from flink_amd import _abi
    _abi.load_library()
    assigner = TumblingEventTimeWindows.of(100) if window == "tumbling" else SlidingEventTimeWindows.of(1000, 100)
    _validate(_run(assigner, None), assigner.size, assigner.slide)
