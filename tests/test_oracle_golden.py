"""The CPU oracle against the reference's own known answers (tests/golden/, see make_fixtures.py).

These pin the oracle; the GPU parity tests then compare the HIP engine with the pinned oracle.
"""
import ctypes

import numpy as np
import pytest

from harness import FOLD_FIXTURES, LIST_FIXTURES, SESSION_FIXTURES, WINDOW_FIXTURES, expected_epochs, load_golden, replay

oracle = pytest.importorskip("oracle.oracle")


@pytest.mark.parametrize("name", WINDOW_FIXTURES + SESSION_FIXTURES + FOLD_FIXTURES + LIST_FIXTURES)
def test_oracle_window_fixtures(name):
    fx = load_golden(name)
    got = replay(fx, oracle.OracleEngine)
    assert got == expected_epochs(fx), fx["source"]


def test_time_window_start_known_answers():
    lib = oracle.load()
    for ts, off, size, exp in load_golden("time_window_start")["cases"]:
        assert lib.fwo_window_start(ts, off, size) == exp


def test_murmur_key_group_cross_check():
    lib = oracle.load()
    for key, lh, mm, kg, op in load_golden("murmur_key_groups")["cases"]:
        assert lib.fwo_long_hash_code(key) == lh
        assert lib.fwo_murmur_hash(lh) == mm
        assert lib.fwo_key_group(lh, 128) == kg
        assert lib.fwo_operator_index(128, 8, kg) == op


def test_key_group_ranges():
    for case in load_golden("key_group_ranges")["cases"]:
        mp, p, i, s, e = case
        assert oracle.key_group_range(mp, p, i) == (s, e)


def test_oracle_rejects_missing_timestamp():
    from harness import fixture_config
    fx = load_golden("tumbling_reduce")
    cfg, _ = fixture_config(fx["config"])
    eng = oracle.OracleEngine(cfg)
    keys = np.array([1], np.int64)
    ts = np.array([-(1 << 63)], np.int64)
    with pytest.raises(RuntimeError, match="Long.MIN_VALUE timestamp"):
        eng.push(keys, ts, np.array([1], np.int64))
    eng.close()


def test_oracle_rejects_foreign_key_group():
    from harness import fixture_config
    fx = load_golden("tumbling_reduce")
    cfg, _ = fixture_config(fx["config"], max_parallelism=128, key_group_range=(0, 0))
    eng = oracle.OracleEngine(cfg)
    # key 42 -> key group 29 (Appendix B), not owned by a subtask holding [0, 0]
    with pytest.raises(RuntimeError, match="Unexpected key group index"):
        eng.push(np.array([42], np.int64), np.array([5], np.int64), np.array([1], np.int64))
    eng.close()


def test_oracle_parallel_job_matches_single_subtask():
    """The p-subtask CPU job (the timed CPU column) fires the same results as one subtask."""
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    from harness import drive, gen_stream
    keys, ts, vals = gen_stream(20000, 500, rate=4000)
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",)), key_capacity=1024)
    n4, cs4 = oracle.run_parallel(cfg, 4, keys, ts, vals, 2000, 1, (1 << 63) - 1)
    n1, cs1 = oracle.run_parallel(cfg, 1, keys, ts, vals, 2000, 1, (1 << 63) - 1)
    assert n4 == n1 and cs4 == cs1
    eng = oracle.OracleEngine(cfg)
    res = drive(eng, keys, ts, vals, 2000, 1, (1 << 63) - 1)
    tot = sum(r["n"] for r in res)
    cs = int(np.sum(np.concatenate([r["sum_i64"] for r in res]).astype(np.uint64)).astype(np.int64))
    assert tot == n1 and cs == cs1


def test_oracle_sliding_negative_remainder_known_answer():
    """SlidingEventTimeWindows.of(3 s, 1 s), one record at ts = -1500: Java's -500 % 1000 = -500 puts the first
    window start at -1000 (TimeWindow.java:239-241), so the loop of SlidingEventTimeWindows.java:64-77 assigns
    four windows (starts -1000 .. -4000), one more than contain the record (worked by hand from the source)."""
    from flink_amd.windowing import ReduceFunction, SlidingEventTimeWindows, make_config
    cfg = make_config(SlidingEventTimeWindows.of(3000, 1000), ReduceFunction(("sum",)), key_capacity=1024,
                      max_batch=1 << 12, out_capacity=1 << 16)
    e = oracle.OracleEngine(cfg)
    e.push(np.array([7], np.int64), np.array([-1500], np.int64), np.array([5], np.int64))
    e.advance_watermark((1 << 63) - 1)
    r = e.collect()
    e.close()
    assert sorted(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist())) == \
        [(7, -1001, 5), (7, -1, 5), (7, 999, 5), (7, 1999, 5)]
