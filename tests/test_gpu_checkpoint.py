"""Checkpoint snapshot/restore per key group (fw_snapshot_kg / fw_restore_kg).

The reference's pattern (EventTimeWindowCheckpointingITCase, RescalingITCase): a job that fails and
restores from a checkpoint must produce the same windows as an uninterrupted run.  Here: run the first
part of a seeded stream on one HIP engine, snapshot every key group (HeapKeyedStateBackend
.writeStateTableForKeyGroup + HeapInternalTimerService.snapshotTimersForKeyGroup), restore the blobs
into fresh engines — the same key-group range, or rescaled to two subtasks that each take their
KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex share (StateAssignmentOperation) — run the
rest, and compare the union of all fired windows with the oracle's uninterrupted run.

Bar: bit-exact for int64 fields and first-arrival f1; double sums within relative 1e-9.
"""
import numpy as np
import pytest

from harness import epochs_of, gen_stream

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
MP = 128


@pytest.fixture(scope="module")
def hip():
    from flink_amd import _abi
    from harness import hip_engine
    _abi.load_library()
    return hip_engine


@pytest.fixture(scope="module")
def oracle_engine():
    from oracle.oracle import OracleEngine
    return OracleEngine


def _abi_words():
    from flink_amd import _abi
    return _abi.FW_SNAP_HEADER_WORDS


def _cfg(assigner, fields, vt="i64", first=False, lateness=0, trigger=None, mode=0, kg=(0, MP - 1)):
    from flink_amd.windowing import ReduceFunction, make_config
    return make_config(assigner, ReduceFunction(fields, vt, first), trigger, lateness, max_parallelism=MP,
                       key_group_range=kg, key_capacity=1 << 14, max_batch=1 << 16, out_capacity=1 << 20,
                       ingest_mode=mode)


def _watermarks(ts, batch, lag):
    """wm after each batch = max ts seen so far - lag (BoundedOutOfOrdernessTimestampExtractor style)."""
    wms, mx = [], -(1 << 63)
    for s in range(0, len(ts), batch):
        mx = max(mx, int(ts[s:s + batch].max()))
        wms.append(mx - lag)
    return wms


def _drive(engines, route, keys, ts, vals, batches, wms, batch):
    """Push batches [b0, b1) (records split over the engines by `route`), advance every engine to the
    batch's watermark, collect.  Returns one list of collect() results per engine."""
    out = [[] for _ in engines]
    for j in batches:
        s, e = j * batch, min(len(keys), (j + 1) * batch)
        dest = route(keys[s:e])
        for r, eng in enumerate(engines):
            sel = np.nonzero(dest == r)[0] + s
            if len(sel):
                eng.push(keys[sel], ts[sel], vals[sel])
            wm = wms[j] if j < len(wms) else LONG_MAX
            eng.advance_watermark(wm)
            out[r].append(eng.collect())
    return out


def _merge(per_engine):
    """Union of the engines' epochs (every engine sees the same watermarks in the same order)."""
    merged = per_engine[0]
    for other in per_engine[1:]:
        assert [w for w, _ in merged] == [w for w, _ in other]
        merged = [(w, sorted(a + b)) for (w, a), (_, b) in zip(merged, other)]
    return merged


def _compare(a, b, rel):
    assert [w for w, _ in a] == [w for w, _ in b]
    for (w, ra), (_, rb) in zip(a, b):
        assert len(ra) == len(rb), f"wm {w}: {len(ra)} vs {len(rb)} records"
        for x, y in zip(ra, rb):
            for u, v in zip(x, y):
                if isinstance(u, float) and rel:
                    assert abs(u - v) <= rel * max(1.0, abs(v)), (w, x, y)
                else:
                    assert u == v, (w, x, y)


def _checkpoint_roundtrip(hip, oracle_engine, make_cfg, keys, ts, vals, batch, lag, fields, first, parallelism,
                          rel=0.0, cut=0.5):
    from flink_amd.keygroups import compute_key_group_range_for_operator_index, operator_index_np
    nb = (len(keys) + batch - 1) // batch
    wms = _watermarks(ts, batch, lag)
    # uninterrupted oracle run (+ the final MAX_WATERMARK)
    eo = oracle_engine(make_cfg((0, MP - 1)))
    ro = _drive([eo], lambda k: np.zeros(len(k), np.int64), keys, ts, vals, range(nb + 1), wms, batch)[0]
    eo.close()
    # part one on one HIP engine, snapshot of every key group
    cb = max(1, int(nb * cut))
    e0 = hip(make_cfg((0, MP - 1)))
    r0 = _drive([e0], lambda k: np.zeros(len(k), np.int64), keys, ts, vals, range(cb), wms, batch)[0]
    state = {kg: e0.snapshot_kg(kg) for kg in range(MP)}
    n_entries = sum((len(b) // 8 - _abi_words()) // 8 for b in state.values())
    assert n_entries > 0
    e0.close()
    # restore into `parallelism` subtasks, each taking its key-group range, and run the rest
    ranges = [compute_key_group_range_for_operator_index(MP, parallelism, i) for i in range(parallelism)]
    engines = []
    for lo, hi in ranges:
        e = hip(make_cfg((lo, hi)))
        for kg in range(lo, hi + 1):
            e.restore_kg(kg, state[kg])
        engines.append(e)
    r1 = _drive(engines, lambda k: operator_index_np(k, MP, parallelism), keys, ts, vals, range(cb, nb + 1), wms,
                batch)
    for e in engines:
        e.close()
    got = epochs_of(r0, fields, first) + _merge([epochs_of(r, fields, first) for r in r1])
    _compare(got, epochs_of(ro, fields, first), rel)
    return n_entries


MODES = [pytest.param(1, id="direct"), pytest.param(2, id="partitioned")]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("parallelism", [1, 2])
def test_tumbling_long_sum_first_arrival_restore(hip, oracle_engine, mode, parallelism):
    """C1 shape: the restored panes keep their sums and their first arrival's f1."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(120_000, 4096, rate=1 << 16)
    mk = lambda kg: _cfg(TumblingEventTimeWindows.of(1000), ("sum",), first=True, mode=mode, kg=kg)
    _checkpoint_roundtrip(hip, oracle_engine, mk, keys, ts, vals, 1 << 13, 1, ["sum_i64"], True, parallelism)


@pytest.mark.parametrize("mode", MODES)
def test_lateness_rescale_restore(hip, oracle_engine, mode):
    """C4 shape: Zipf keys, out-of-order, allowed lateness: fired-but-not-cleaned panes survive the
    checkpoint, later records re-fire them per element (WindowOperator.java:317-325)."""
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(100_000, 1 << 12, rate=1 << 16, zipf=1.2, ooo=200)
    mk = lambda kg: _cfg(TumblingEventTimeWindows.of(1000), ("sum", "count"), first=True, lateness=100, mode=mode,
                         kg=kg)
    _checkpoint_roundtrip(hip, oracle_engine, mk, keys, ts, vals, 2048, 50, ["sum_i64", "count"], True, 2)


@pytest.mark.parametrize("mode", MODES)
def test_sliding_double_rescale_restore(hip, oracle_engine, mode):
    """C3 shape: sliding 10 s / 1 s over slices; restored slices rebuild every open window."""
    from flink_amd.windowing import SlidingEventTimeWindows
    keys, ts, vals = gen_stream(100_000, 2000, rate=1 << 13, value_type="f64")
    mk = lambda kg: _cfg(SlidingEventTimeWindows.of(10_000, 1000), ("sum", "min", "max", "count"), "f64", True,
                         mode=mode, kg=kg)
    _checkpoint_roundtrip(hip, oracle_engine, mk, keys, ts, vals, 8192, 1,
                          ["sum_f64", "min_f64", "max_f64", "count"], True, 2, rel=1e-9)


def test_all_int_fields_offset_restore(hip, oracle_engine):
    from flink_amd.windowing import TumblingEventTimeWindows
    keys, ts, vals = gen_stream(80_000, 1000, rate=1 << 15, ooo=300)
    mk = lambda kg: _cfg(TumblingEventTimeWindows.of(1000, 250), ("sum", "min", "max", "count"), kg=kg)
    _checkpoint_roundtrip(hip, oracle_engine, mk, keys, ts, vals, 10_000, 1,
                          ["sum_i64", "min_i64", "max_i64", "count"], False, 2, cut=0.3)


def test_restore_errors(hip):
    """Foreign key group (HeapInternalTimerService.restoreTimersForKeyGroup's range check), restore after
    the first push, mismatched configuration, mismatched watermarks, Java key hashes."""
    from flink_amd import _abi
    from flink_amd.windowing import SlidingEventTimeWindows, TumblingEventTimeWindows
    e = hip(_cfg(TumblingEventTimeWindows.of(1000), ("sum",)))
    e.push(np.arange(100, dtype=np.int64), np.arange(100, dtype=np.int64) * 7, np.ones(100, np.int64))
    e.advance_watermark(300)
    blobs = {kg: e.snapshot_kg(kg) for kg in range(MP)}
    kg = max(blobs, key=lambda k: len(blobs[k]))
    hdr = np.frombuffer(blobs[kg], np.int64)[:_abi_words()]
    assert hdr[0] == _abi.FW_SNAP_MAGIC and hdr[2] == kg and hdr[3] > 0 and hdr[4] == 300
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg(kg, blobs[kg])           # after the first push
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    e.close()
    half = hip(_cfg(TumblingEventTimeWindows.of(1000), ("sum",), kg=(0, 63)))
    other = kg if kg >= 64 else kg + 64
    with pytest.raises(_abi.FwError) as ei:
        half.restore_kg(other, blobs[other])
    assert "does not belong to the local range" in str(ei.value)
    half.close()
    sl = hip(_cfg(SlidingEventTimeWindows.of(3000, 1000), ("sum",)))
    with pytest.raises(_abi.FwError):
        sl.restore_kg(kg, blobs[kg])          # different window configuration
    sl.close()
    lt = hip(_cfg(TumblingEventTimeWindows.of(1000), ("sum",), lateness=200))
    with pytest.raises(_abi.FwError):
        lt.restore_kg(kg, blobs[kg])          # different allowed lateness (the implicit timers would differ)
    lt.close()
    f = hip(_cfg(TumblingEventTimeWindows.of(1000), ("sum",)))
    f.restore_kg(kg, blobs[kg])
    b2 = np.frombuffer(blobs[(kg + 1) % MP], np.int64).copy()
    b2[4] = 999
    with pytest.raises(_abi.FwError):
        f.restore_kg((kg + 1) % MP, b2.tobytes())   # checkpointed at another watermark
    f.close()
    h = hip(_cfg(TumblingEventTimeWindows.of(1000), ("sum",)))
    h.push(np.arange(4, dtype=np.int64), np.arange(4, dtype=np.int64), np.ones(4, np.int64),
           key_hash=np.arange(4, dtype=np.int32))
    with pytest.raises(_abi.FwError) as ei:
        h.snapshot_kg(0)
    assert ei.value.code == _abi.FW_ERR_UNSUPPORTED
    h.close()
