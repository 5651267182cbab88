"""Session windows on the CPU: the C++ oracle's merging branch against an independent Python statement of
the same reference semantics (tests/session_model.py) on random out-of-order streams with lateness, both
triggers.  The reference's own known answers pin the oracle in test_oracle_golden.py (session_* fixtures).
"""
import numpy as np
import pytest

from harness import drive, epochs_of
from session_model import SessionModel

oracle = pytest.importorskip("oracle.oracle")

LONG_MAX = (1 << 63) - 1


def session_stream(n, n_keys, seed, span, ooo):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, n_keys, n).astype(np.int64)
    base = np.sort(rng.integers(0, span, n)).astype(np.int64)
    ts = base - rng.integers(0, ooo + 1, n).astype(np.int64)
    vals = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    return keys, ts, vals


def model_run(keys, ts, vals, batch, lag, gap, lateness, purging):
    m = SessionModel(gap, lateness, purging)
    max_ts = -(1 << 63)
    for s in range(0, len(keys), batch):
        e = min(len(keys), s + batch)
        for i in range(s, e):
            m.element(int(keys[i]), int(ts[i]), int(vals[i]))
        max_ts = max(max_ts, int(ts[s:e].max()))
        m.watermark(max_ts - lag)
    m.watermark(LONG_MAX)
    return m.epochs()


@pytest.mark.parametrize("lateness,purging", [(0, False), (0, True), (150, False), (150, True), (5000, False)])
def test_oracle_sessions_match_model(lateness, purging):
    from flink_amd.windowing import (EventTimeSessionWindows, EventTimeTrigger, PurgingTrigger, ReduceFunction,
                                     make_config)
    gap = 100
    keys, ts, vals = session_stream(6000, 40, 7 + lateness + purging, 60000, 300)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else EventTimeTrigger.create()
    cfg = make_config(EventTimeSessionWindows.withGap(gap), ReduceFunction(("sum", "count")), trig, lateness,
                      max_parallelism=128, key_capacity=256, max_batch=1 << 12, out_capacity=1 << 16)
    eng = oracle.OracleEngine(cfg)
    res = drive(eng, keys, ts, vals, 500, 120, LONG_MAX)
    eng.close()
    got = epochs_of(res, ["sum_i64", "count", "win_start"])
    # (key, ts, sum, count, start) -> the model's (key, sum, count, ts, start)
    got = [(w, sorted((r[0], r[2], r[3], r[1], r[4]) for r in recs)) for w, recs in got]
    want = model_run(keys, ts, vals, 500, 120, gap, lateness, purging)
    assert got == want
    assert sum(len(r) for _, r in got) > 100
