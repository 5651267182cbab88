"""Asynchronous drains (fw_collect_begin / fw_collect_end): the results and watermark marks of every drain equal
what the synchronous fw_collect returns at the same point of the same stream (two engines fed identically), with
one to three drains outstanding while later batches run, quiet watermarks (marks without results) included, and
for tumbling, sliding and session windows (the window-start column).  The operator may hand watermark j's results
downstream after batch j + 1 is pushed: results need only precede their watermark
(AbstractStreamOperator.java:803-808)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1


def _stream(n, keys, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, keys, n).astype(np.int64)
    t = (1_700_000_000_000 + np.arange(n) // 8 - rng.integers(0, 30, n)).astype(np.int64)
    v = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    return k, t, v


def _rows(r):
    cols = [r[c] for c in ("key", "ts", "f1", "sum_i64", "min_i64", "max_i64", "count")
            if r.get(c) is not None and len(r[c]) == r["n"]]
    if r.get("win_start") is not None and len(r["win_start"]) == r["n"] and r["n"]:
        cols.append(r["win_start"])
    rows = np.stack(cols, axis=1) if r["n"] else np.zeros((0, len(cols)), np.int64)
    # per watermark epoch, as a multiset (TestHarnessUtil order contract)
    out, pos = [], 0
    for wm, mp in list(zip(r["mark_wm"].tolist(), r["mark_pos"].tolist())) + [(None, r["n"])]:
        part = rows[pos:mp]
        pos = mp
        out.append((wm, sorted(map(tuple, part.tolist()))))
    return out


@pytest.mark.parametrize("kind", ["tumbling", "sliding", "session", "tumbling_all_fields"])
@pytest.mark.parametrize("lag", [0, 1, 2])   # drains left outstanding before the next begins (three at most at once)
def test_async_drain_matches_collect(kind, lag):
    from flink_amd.windowing import (EventTimeSessionWindows, ReduceFunction, SlidingEventTimeWindows,
                                     TumblingEventTimeWindows, WindowEngine, make_config)
    assigner = {"tumbling": TumblingEventTimeWindows.of(100), "sliding": SlidingEventTimeWindows.of(300, 100),
                "session": EventTimeSessionWindows.withGap(20),
                "tumbling_all_fields": TumblingEventTimeWindows.of(100)}[kind]
    # (all fields: every output column present, so the drain's packed columns are all in play)
    fields = ("sum", "min", "max", "count") if kind == "tumbling_all_fields" else ("sum", "count")
    cfg = make_config(assigner, ReduceFunction(fields, "i64", keep_first_f1=True), max_parallelism=128,
                      key_capacity=1 << 12, max_batch=1 << 12, out_capacity=1 << 18)
    k, t, v = _stream(40_000, 2000, 11)
    a, b = WindowEngine(cfg), WindowEngine(cfg)
    got, want, pending = [], [], []
    mx = -(1 << 63)
    for s in range(0, len(k), 1 << 12):
        sl = slice(s, s + (1 << 12))
        mx = max(mx, int(t[sl].max()))
        for e in (a, b):
            e.push(k[sl], t[sl], v[sl])
            e.advance_watermark(mx - 10)
            if s % 3 == 0:
                e.advance_watermark(mx - 10)   # a repeated (quiet) watermark: a mark without results
        if len(pending) > lag:
            got += _rows(a.collect_end(pending.pop(0)))
        pending.append(a.collect_begin())
        want += _rows(b.collect())
    for e in (a, b):
        e.advance_watermark(LONG_MAX)
    while len(pending) > 2:
        got += _rows(a.collect_end(pending.pop(0)))
    pending.append(a.collect_begin())
    while pending:
        got += _rows(a.collect_end(pending.pop(0)))
    want += _rows(b.collect())
    a.close()
    b.close()
    # epochs without a mark (the tail of a drain) concatenate with the next drain's first epoch
    def merged(eps):
        out, carry = [], []
        for wm, rows in eps:
            carry += rows
            if wm is not None:
                out.append((wm, sorted(carry)))
                carry = []
        return out, sorted(carry)
    assert merged(got) == merged(want)
    assert sum(len(r) for _, r in got) > 1000


def test_async_drain_limits():
    from flink_amd import _abi
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
    cfg = make_config(TumblingEventTimeWindows.of(100), ReduceFunction(("sum",), "i64"), key_capacity=1 << 10,
                      max_batch=1 << 10, out_capacity=1 << 12)
    e = WindowEngine(cfg)
    k, t, v = _stream(1 << 10, 100, 3)
    e.push(k, t, v)
    e.advance_watermark(LONG_MAX)
    t1 = e.collect_begin()
    t2 = e.collect_begin()
    t3 = e.collect_begin()
    with pytest.raises(_abi.FwError):   # a fourth drain while three are outstanding
        e.collect_begin()
    with pytest.raises(_abi.FwError):   # no such ticket
        e.collect_end(t3 + 1)
    r2, r1, r3 = e.collect_end(t2), e.collect_end(t1), e.collect_end(t3)   # any order
    assert r1["n"] > 0 and r2["n"] == 0 and r3["n"] == 0
    assert list(r1["mark_wm"]) == [LONG_MAX] and len(r2["mark_wm"]) == 0
    with pytest.raises(_abi.FwError):   # ended already
        e.collect_end(t1)
    t4 = e.collect_begin()   # the ring turns over
    assert e.collect_end(t4)["n"] == 0
    e.close()
