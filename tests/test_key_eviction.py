"""Unbounded key spaces: keys leave the engine's directory once no live slice holds a pane of them
(k_compact), as the reference drops a key's entry when its last pane is cleared (AbstractHeapState.clear,
AbstractHeapState.java:90-119) — VERDICT r1 item 6.

The stream drifts through 4x key_capacity distinct keys over time while fewer than key_capacity are live
at once: without eviction the directory (4 x key_capacity slots) overflows.  Bit-exact against the
oracle, both ingest forms; the checkpoint sections afterwards are byte-identical too (key groups whose
keys were all evicted stay "present", HeapKeyedStateBackend.java:228-233).
"""
import ctypes

import numpy as np
import pytest

from harness import drive, epochs_of, hip_engine

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
CAP = 4096


def _drifting_stream(n_windows=44, per_window=6000, span=2000, step=500, seed=3):
    """Window w (1 s) draws its keys from [w*step, w*step + span): consecutive windows share keys, and
    n_windows*step + span distinct keys pass through in total."""
    rng = np.random.default_rng(seed)
    keys, ts = [], []
    for w in range(n_windows):
        keys.append(rng.integers(w * step, w * step + span, per_window) * 7919 + 13)
        ts.append(np.sort(rng.integers(w * 1000, (w + 1) * 1000, per_window)))
    keys, ts = np.concatenate(keys).astype(np.int64), np.concatenate(ts).astype(np.int64)
    vals = rng.integers(-50, 50, len(keys)).astype(np.int64)
    return keys, ts, vals


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("window", ["tumbling", "sliding"])
def test_keys_evicted_over_time(mode, window):
    from flink_amd.windowing import (ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows,
                                     WindowEngine, make_config)
    from oracle.oracle import OracleEngine
    keys, ts, vals = _drifting_stream()
    assert len(np.unique(keys)) >= 4 * CAP
    assigner = TumblingEventTimeWindows.of(1000) if window == "tumbling" else SlidingEventTimeWindows.of(2000, 1000)
    cfg = make_config(assigner, ReduceFunction(("sum", "count"), "i64", True), None, 0, max_parallelism=128,
                      key_capacity=CAP, max_batch=1 << 13, out_capacity=1 << 20, ingest_mode=mode)
    f1 = np.arange(len(keys), dtype=np.int64)
    n = len(keys) - 6000
    res = []
    for factory in (WindowEngine, OracleEngine):
        e = factory(cfg) if factory is OracleEngine else hip_engine(cfg)
        out = drive(e, keys[:n], ts[:n], vals[:n], 6000, 1, None, f1=f1[:n])
        snap = {kg: e.snapshot_kg_flink(kg, ("key", "f1", "sum", "count")) for kg in range(128)}
        out += drive(e, keys[n:], ts[n:], vals[n:], 6000, 1, LONG_MAX, f1=f1[n:])
        st = e.stats()
        dbg = np.zeros(8, np.int64)
        if factory is WindowEngine:
            e.lib.fw_debug_counters(e.h, dbg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        e.close()
        res.append((out, snap, st, dbg))
    (rg, sg, stg, dbg), (ro, so, sto, _) = res
    assert dbg[7] == 0, f"capacity error at site {dbg[7]}"
    assert stg["compactions"] > 0
    assert stg["keys_resident"] < 4 * CAP
    assert epochs_of(rg, ["sum_i64", "count"], True) == epochs_of(ro, ["sum_i64", "count"], True)
    assert stg["panes_fired"] == sto["panes_fired"]
    for kg in range(128):
        assert sg[kg] == so[kg], f"key group {kg}: checkpoint sections differ after evictions"


def test_without_eviction_the_directory_overflows(monkeypatch):
    """The same stream with compaction disabled (FW_COMPACT_FILL=0) runs out of directory slots: the
    capacity error the eviction removes."""
    from flink_amd import _abi
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
    monkeypatch.setenv("FW_COMPACT_FILL", "0")
    keys, ts, vals = _drifting_stream()
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 0,
                      key_capacity=CAP, max_batch=1 << 13, out_capacity=1 << 20, ingest_mode=2)
    e = WindowEngine(cfg)
    with pytest.raises(_abi.FwError) as ei:
        drive(e, keys, ts, vals, 6000, 1, LONG_MAX)
    assert ei.value.code == _abi.FW_ERR_CAPACITY
    e.close()
