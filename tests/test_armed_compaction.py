"""Re-arm marks of a restored disarmed window survive key eviction.

A tumbling window that fired before the checkpoint and is kept for its allowed lateness is restored at
Long.MIN_VALUE (HeapInternalTimerService.java:72 restarts the timer service there) with its panes disarmed:
only keys a later record re-arms fire at its maxTimestamp (EventTimeTrigger.onElement, :37-45).  The marks
are kept per (slot, key id).  Here an earlier window fires and is cleaned before the disarmed one fires,
the directory is compacted in between (FW_COMPACT_FILL=1: after every firing watermark; one dense bucket,
FW_DIR_SLOTS=100), so the surviving keys change ids; the disarmed window must still fire exactly for the
re-armed keys, as the oracle restored the same way.
"""
import numpy as np
import pytest


LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
LAYOUT = ("key", "f1", "sum")


def _cfg(mode=0):
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    kw = dict(max_parallelism=128, key_capacity=512, max_batch=1 << 12, out_capacity=1 << 14)
    if mode:
        kw["ingest_mode"] = mode
    return make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 500, **kw)


def _checkpoint():
    """Oracle checkpoint at watermark 2100: window [1000, 2000) of keys 0..63 fired, kept until 2499."""
    from oracle.oracle import OracleEngine
    e = OracleEngine(_cfg())
    k = np.arange(64, dtype=np.int64)
    e.push(k, 1000 + 13 * k, k * 7 + 1, f1=k + 100)
    e.advance_watermark(2100)
    e.collect()
    blobs = {kg: e.snapshot_kg_flink(kg, LAYOUT) for kg in range(128)}
    e.close()
    return blobs


def _continue(e, blobs):
    for kg, (st, tm) in blobs.items():
        e.restore_kg_flink(kg, LAYOUT, st, tm, LONG_MIN)
    out = []
    # window [0, 1000): 200 new keys, inserted after the restored ones
    kz = np.arange(1000, 1200, dtype=np.int64)
    e.push(kz, 100 + (kz % 800), kz, f1=kz + 1)
    # the disarmed window [1000, 2000): re-arms restored keys 0..31 and adds 100 new keys (inserted last, so the
    # probe chains place them behind window [0, 1000)'s keys)
    ka = np.concatenate([np.arange(32, dtype=np.int64), np.arange(2000, 2100, dtype=np.int64)])
    e.push(ka, 1500 + (ka % 400), 3 * ka + 5, f1=ka + 7)
    out.append(e.collect())
    e.advance_watermark(1600)   # fires [0, 1000) and cleans it (999 + 500 <= 1600): its keys die, compaction
    out.append(e.collect())
    e.advance_watermark(2100)   # the disarmed window's maxTimestamp: re-armed keys only
    out.append(e.collect())
    e.advance_watermark(LONG_MAX)
    out.append(e.collect())
    return out


def test_oracle_fires_only_rearmed_keys():
    from oracle.oracle import OracleEngine
    e = OracleEngine(_cfg())
    out = _continue(e, _checkpoint())
    e.close()
    fired = {int(k) for k in out[2]["key"]}
    assert fired == set(range(32)) | set(range(2000, 2100))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_rearm_marks_move_with_compaction(mode, monkeypatch):
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    monkeypatch.setenv("FW_COMPACT_FILL", "1")
    monkeypatch.setenv("FW_DIR_SLOTS", "100")
    blobs = _checkpoint()
    res = []
    for factory in (WindowEngine, OracleEngine):
        e = factory(_cfg(mode))
        out = _continue(e, blobs)
        if factory is WindowEngine:
            assert e.stats()["compactions"] > 0, "no compaction ran between the two fires"
        e.close()
        res.append([sorted(zip(r["key"].tolist(), r["f1"].tolist(), r["sum_i64"].tolist(), r["ts"].tolist()))
                    for r in out])
    assert res[0] == res[1]
    assert {k for k, *_ in res[1][2]} == set(range(32)) | set(range(2000, 2100))
