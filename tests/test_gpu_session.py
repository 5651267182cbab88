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


def test_session_rejections(hip):
    from flink_amd import _abi
    from flink_amd.windowing import (EventTimeSessionWindows, ReduceFunction, make_config)
    with pytest.raises(_abi.FwError):
        hip(make_config(EventTimeSessionWindows.withGap(10), ReduceFunction(("sum",), keep_first_f1=True)))
    e = hip(_cfg(10, ("sum",)))
    e.push(np.array([1], np.int64), np.array([5], np.int64), np.array([1], np.int64))
    with pytest.raises(_abi.FwError, match="session"):
        e.snapshot_kg(0)
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
