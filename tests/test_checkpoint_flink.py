"""Checkpoint sections in the reference's own key-group byte layout (fw_snapshot_kg_flink /
fw_restore_kg_flink):

  state   HeapKeyedStateBackend.snapshot's section at KeyGroupRangeOffsets[kg] + writeStateTableForKeyGroup
          (RT/state/heap/HeapKeyedStateBackend.java:196-248)
  timers  HeapInternalTimerService.snapshotTimersForKeyGroup after its serializer records (:285-310)

tests/golden/checkpoint_flink.json holds, per scenario, a seeded stream, the checkpoint position and the
expected bytes of every key group, encoded by tests/golden/make_checkpoint_fixture.py — a plain-Python
model of the heap backend written from the layout's definition, independent of the oracle and of the
engine.  Parity is pinned by that hand-built fixture (no JVM here to run the reference).

CPU: the oracle's restatement reproduces the fixture bytes, and restoring them reproduces them again.
GPU: the HIP engine writes the same bytes; a restore of the fixture into the engine continues exactly as
the oracle restored from the same bytes; engine and oracle agree byte for byte on larger streams.
"""
import json
import os
import struct

import numpy as np
import pytest

from harness import epochs_of

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "checkpoint_flink.json")))
SCEN = {s["name"]: s for s in FIX["scenarios"]}
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


def _cfg(sc, kg=None, mode=0):
    from flink_amd.windowing import ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows, make_config
    c = sc["config"]
    if c["assigner"] == "tumbling":
        assigner = TumblingEventTimeWindows.of(c["size"], c["offset"])
    else:
        assigner = SlidingEventTimeWindows.of(c["size"], c["slide"], c["offset"])
    kw = dict(max_parallelism=c["mp"], key_capacity=1 << 10, max_batch=1 << 12, out_capacity=1 << 16)
    if kg is not None:
        kw["key_group_range"] = kg
    if mode:
        kw["ingest_mode"] = mode
    return make_config(assigner, ReduceFunction(tuple(c["aggs"]), c["value_type"], True), None, c["lateness"], **kw)


def _columns(sc, lo, hi):
    r = np.array(sc["records"][lo:hi], dtype=np.int64).reshape(-1, 4)
    vals = r[:, 3].copy()
    if sc["config"]["value_type"] == "f64":
        vals = vals.view(np.float64)
    return r[:, 0].copy(), r[:, 1].copy(), r[:, 2].copy(), vals


def _drive(eng, sc, lo, hi, final=False):
    """Push records [lo, hi) and the watermarks between them, in order; collect after each watermark."""
    out, pos = [], lo
    marks = [(i, w) for i, w in sc["watermarks"] if lo < i <= hi]
    if final:
        marks.append((hi, LONG_MAX))
    for i, wm in marks:
        if i > pos:
            k, f1, ts, v = _columns(sc, pos, i)
            eng.push(k, ts, v, f1=f1)
            pos = i
        eng.advance_watermark(wm)
        out.append(eng.collect())
    if pos < hi:
        k, f1, ts, v = _columns(sc, pos, hi)
        eng.push(k, ts, v, f1=f1)
        out.append(eng.collect())
    return out


def _expected(sc):
    return {int(kg): (bytes.fromhex(s), bytes.fromhex(t)) for kg, (s, t) in sc["kgs"].items()}


def _snapshot_all(eng, sc):
    return {kg: eng.snapshot_kg_flink(kg, sc["layout"]) for kg in range(sc["config"]["mp"])}


def _restore_wm(sc):
    return sc["checkpoint_wm"] if sc["restore_wm"] == "checkpoint" else LONG_MIN


def _diff(got, want):
    for kg in sorted(want):
        for part, g, w in (("state", got[kg][0], want[kg][0]), ("timers", got[kg][1], want[kg][1])):
            if g != w:
                at = next((i for i in range(min(len(g), len(w))) if g[i] != w[i]), min(len(g), len(w)))
                return f"kg {kg} {part}: {len(g)} vs {len(w)} bytes, first difference at byte {at}"
    return None


@pytest.mark.parametrize("name", list(SCEN))
def test_fixture_is_well_formed(name):
    """Every present key group's state section parses to the layout; timers section length matches."""
    sc = SCEN[name]
    nf = len(sc["layout"])
    for kg, (st, tm) in _expected(sc).items():
        k, sid, present = struct.unpack(">ihb", st[:7])
        assert (k, sid) == (kg, 0)
        pos = 7
        if present:
            (nns,) = struct.unpack(">i", st[pos:pos + 4])
            pos += 4
            for _ in range(nns):
                start, end, n = struct.unpack(">qqi", st[pos:pos + 20])
                assert end - start == sc["config"]["size"]
                pos += 20 + n * 8 * (1 + nf)
        assert pos == len(st)
        (nt,) = struct.unpack(">i", tm[:4])
        assert len(tm) == 8 + 32 * nt


@pytest.mark.parametrize("name", list(SCEN))
def test_oracle_writes_fixture_bytes(name):
    from oracle.oracle import OracleEngine
    sc = SCEN[name]
    eo = OracleEngine(_cfg(sc))
    _drive(eo, sc, 0, sc["cut"])
    got = _snapshot_all(eo, sc)
    eo.close()
    assert _diff(got, _expected(sc)) is None, _diff(got, _expected(sc))


@pytest.mark.parametrize("name", list(SCEN))
def test_oracle_restore_round_trip(name):
    """readStateTableForKeyGroup / restoreTimersForKeyGroup put in blob order: a snapshot right after the
    restore writes the same bytes."""
    from oracle.oracle import OracleEngine
    sc = SCEN[name]
    want = _expected(sc)
    eo = OracleEngine(_cfg(sc))
    for kg, (st, tm) in want.items():
        eo.restore_kg_flink(kg, sc["layout"], st, tm, _restore_wm(sc))
    got = _snapshot_all(eo, sc)
    eo.close()
    assert _diff(got, want) is None, _diff(got, want)


# ---------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", list(SCEN))
def test_engine_writes_fixture_bytes(name, mode):
    from flink_amd.windowing import WindowEngine
    sc = SCEN[name]
    eg = WindowEngine(_cfg(sc, mode=mode))
    _drive(eg, sc, 0, sc["cut"])
    got = _snapshot_all(eg, sc)
    eg.close()
    assert _diff(got, _expected(sc)) is None, _diff(got, _expected(sc))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", [n for n, s in SCEN.items() if s["restore_wm"] is not None])
def test_engine_restore_continues_like_oracle(name, mode):
    """Restore the fixture's key groups (into two subtasks, each its KeyGroupRangeAssignment share), run the
    rest of the stream and a final MAX_WATERMARK: the same output as the oracle restored from the same
    bytes at the same watermark; a snapshot right after the restore writes the fixture bytes back."""
    _restore_and_continue(SCEN[name], _restore_wm(SCEN[name]), mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_sliding_restore_into_window_panes(mode):
    """Sliding windows in the reference layout hold one state per window (namespace = TimeWindow); the engine
    restores each into that window's own pane (records after the restore go to slices, and a window fires
    slices + pane) — restored at Long.MIN_VALUE, as the reference restarts its timers."""
    _restore_and_continue(SCEN["sliding_i64"], LONG_MIN, mode)


def _restore_and_continue(sc, wm, mode):
    from flink_amd.keygroups import compute_key_group_range_for_operator_index, operator_index_np
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    mp, want = sc["config"]["mp"], _expected(sc)
    eo = OracleEngine(_cfg(sc))
    for kg, (st, tm) in want.items():
        eo.restore_kg_flink(kg, sc["layout"], st, tm, wm)
    ro = _drive(eo, sc, sc["cut"], len(sc["records"]), final=True)
    eo.close()
    fields = [f"{a}_{sc['config']['value_type']}" if a != "count" else "count" for a in sc["config"]["aggs"]]
    engines = []
    for i in range(2):
        lo, hi = compute_key_group_range_for_operator_index(mp, 2, i)
        e = WindowEngine(_cfg(sc, kg=(lo, hi), mode=mode))
        for kg in range(lo, hi + 1):
            e.restore_kg_flink(kg, sc["layout"], *want[kg], watermark=wm)
        back = {kg: e.snapshot_kg_flink(kg, sc["layout"]) for kg in range(lo, hi + 1)}
        assert _diff(back, {kg: want[kg] for kg in range(lo, hi + 1)}) is None
        engines.append((e, i))
    # split the rest of the stream by operator index, as keyBy would
    k_all = np.array([r[0] for r in sc["records"]], np.int64)
    dest = operator_index_np(k_all, mp, 2)
    per = []
    for e, i in engines:
        sub = dict(sc)
        sub["records"] = [r if d == i else None for r, d in zip(sc["records"], dest)]
        per.append(_drive_sparse(e, sub, sc["cut"], len(sc["records"])))
        e.close()
    got = _merge([epochs_of(r, fields, True) for r in per])
    exp = _canon(epochs_of(ro, fields, True))
    assert got == exp


def _drive_sparse(eng, sc, lo, hi):
    """_drive over a record list in which other subtasks' records are None."""
    out, pos = [], lo
    marks = [(i, w) for i, w in sc["watermarks"] if lo < i <= hi] + [(hi, LONG_MAX)]

    def push(a, b):
        rows = [r for r in sc["records"][a:b] if r is not None]
        if rows:
            r = np.array(rows, dtype=np.int64)
            v = r[:, 3].copy()
            if sc["config"]["value_type"] == "f64":
                v = v.view(np.float64)
            eng.push(r[:, 0].copy(), r[:, 2].copy(), v, f1=r[:, 1].copy())
    for i, wm in marks:
        push(pos, i)
        pos = i
        eng.advance_watermark(wm)
        out.append(eng.collect())
    return out


def _canon(ep):
    """Epochs with doubles as their doubleToLongBits (NaN, -0.0 compare exactly), records sorted."""
    def tok(x):
        if isinstance(x, float):
            return ("d", b"nan" if x != x else struct.pack(">d", x))
        return x
    return [(w, sorted((tuple(tok(x) for x in r) for r in recs), key=repr)) for w, recs in ep]


def _merge(per_engine):
    per_engine = [_canon(p) for p in per_engine]
    merged = per_engine[0]
    for other in per_engine[1:]:
        assert [w for w, _ in merged] == [w for w, _ in other]
        merged = [(w, sorted(a + b, key=repr)) for (w, a), (_, b) in zip(merged, other)]
    return merged


@pytest.mark.gpu
@pytest.mark.parametrize("window", ["tumbling_lateness", "sliding", "tumbling_purging"])
def test_engine_matches_oracle_bytes_random(window):
    """Zipf keys, out-of-order timestamps, 128 key groups: every key group's sections byte-identical."""
    from flink_amd.windowing import (ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows,
                                     WindowEngine, make_config)
    from harness import drive, gen_stream
    from oracle.oracle import OracleEngine
    keys, ts, vals = gen_stream(60_000, 3000, rate=1 << 14, zipf=1.1, ooo=300)
    kw = dict(max_parallelism=128, key_capacity=1 << 13, max_batch=1 << 14, out_capacity=1 << 20)
    if window == "sliding":
        cfg = make_config(SlidingEventTimeWindows.of(3000, 1000), ReduceFunction(("sum", "count"), "i64", True),
                          None, 0, **kw)
        layout = ("key", "f1", "sum", "count")
    elif window == "tumbling_purging":
        from flink_amd.windowing import EventTimeTrigger, PurgingTrigger
        cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "max"), "i64", True),
                          PurgingTrigger.of(EventTimeTrigger.create()), 0, **kw)
        layout = ("f1", "key", "max", "sum")
    else:
        cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "min", "count"), "i64", True),
                          None, 400, **kw)
        layout = ("key", "f1", "sum", "min", "count")
    f1 = np.arange(len(keys), dtype=np.int64) * 3 + 1
    n = len(keys) * 2 // 3
    res = []
    for factory in (WindowEngine, OracleEngine):
        e = factory(cfg)
        drive(e, keys[:n], ts[:n], vals[:n], 4096, 120, None, f1=f1[:n])
        res.append({kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)})
        e.close()
    assert sum(len(s) for s, _ in res[1].values()) > 128 * 8
    assert _diff(res[0], res[1]) is None, _diff(res[0], res[1])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_restore_at_long_min_keeps_records_late_at_the_checkpoint(mode):
    """The reference restarts its timer service at Long.MIN_VALUE (HeapInternalTimerService.java:72, not
    checkpointed): after a restore, records whose windows were already cleaned at the checkpoint are not
    late until the next watermark — they build fresh panes that the next watermark fires
    (WindowOperator.java:302-333).  Restored at INT64_MIN, the engine does the same as the oracle restored
    the same way (pin restore watermark semantics)."""
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    sc = SCEN["tumbling_f64_min_max"]
    want = _expected(sc)
    cw = sc["checkpoint_wm"]
    # records 1-3 s behind the checkpoint's watermark (their windows are gone), then the stream's rest
    late_ts = np.array([cw - 3000, cw - 2500, cw - 1200, cw - 1100], np.int64)
    late = dict(key=np.array([3, 5, 3, 7], np.int64), ts=late_ts, f1=np.arange(4, dtype=np.int64) + 9000,
                value=np.array([1.5, -0.0, 2.25, 7.0]))
    res = []
    for factory in (WindowEngine, OracleEngine):
        e = factory(_cfg(sc, mode=mode))
        for kg, (st, tm) in want.items():
            e.restore_kg_flink(kg, sc["layout"], st, tm, LONG_MIN)
        e.push(late["key"], late["ts"], late["value"], f1=late["f1"])
        out = [e.collect()]
        out += _drive(e, sc, sc["cut"], len(sc["records"]), final=True)
        res.append(_canon(epochs_of(out, ["sum_f64", "min_f64", "max_f64", "count"], True)))
        e.close()
    assert res[0] == res[1]
    first_wm = res[1][0]
    assert any(t < cw for _, t, *_ in first_wm[1]), "the late records fired at the first watermark"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_restore_at_long_min_with_fired_but_kept_panes(mode):
    """Allowed lateness 500: at the checkpoint some windows have fired and are kept for their lateness — their
    panes carry only cleanup timers.  Restored at Long.MIN_VALUE (the reference's timer service restarts there,
    HeapInternalTimerService.java:72), such a window fires again only for keys a record re-arms before the
    watermark passes it (EventTimeTrigger.onElement registers maxTimestamp, :37-45), with the restored contents;
    the other keys' panes wait for their cleanup.  Two subtasks by KeyGroupRangeAssignment, the same output as
    the oracle restored the same way; a snapshot right after the restore writes the fixture bytes back."""
    from flink_amd.keygroups import compute_key_group_range_for_operator_index, operator_index_np
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    sc = SCEN["tumbling_lateness_i64"]
    mp, want, cw = sc["config"]["mp"], _expected(sc), sc["checkpoint_wm"]
    # records for windows that fired before the checkpoint (and some that did not), pushed before any watermark
    pre_keys = np.array([k for k in range(12)] * 3, np.int64)
    pre_ts = np.array([cw - 450 + 37 * j for j in range(len(pre_keys))], np.int64)
    pre_f1 = np.arange(len(pre_keys), dtype=np.int64) + 50_000
    pre_v = np.arange(len(pre_keys), dtype=np.int64) * 11 + 5
    eo = OracleEngine(_cfg(sc))
    for kg, (st, tm) in want.items():
        eo.restore_kg_flink(kg, sc["layout"], st, tm, LONG_MIN)
    eo.push(pre_keys, pre_ts, pre_v, f1=pre_f1)
    ro = [eo.collect()] + _drive(eo, sc, sc["cut"], len(sc["records"]), final=True)
    eo.close()
    pre_dest = operator_index_np(pre_keys, mp, 2)
    dest = operator_index_np(np.array([r[0] for r in sc["records"]], np.int64), mp, 2)
    per = []
    for i in range(2):
        lo, hi = compute_key_group_range_for_operator_index(mp, 2, i)
        e = WindowEngine(_cfg(sc, kg=(lo, hi), mode=mode))
        for kg in range(lo, hi + 1):
            e.restore_kg_flink(kg, sc["layout"], *want[kg], watermark=LONG_MIN)
        back = {kg: e.snapshot_kg_flink(kg, sc["layout"]) for kg in range(lo, hi + 1)}
        assert _diff(back, {kg: want[kg] for kg in range(lo, hi + 1)}) is None
        sel = pre_dest == i
        e.push(pre_keys[sel], pre_ts[sel], pre_v[sel], f1=pre_f1[sel])
        sub = dict(sc)
        sub["records"] = [r if d == i else None for r, d in zip(sc["records"], dest)]
        per.append([e.collect()] + _drive_sparse(e, sub, sc["cut"], len(sc["records"])))
        e.close()
    fields = ["sum_i64"]
    got = _merge([epochs_of(r, fields, True) for r in per])
    exp = _canon(epochs_of(ro, fields, True))
    assert got == exp
    refired = [r for _, recs in exp for r in recs if r[1] <= cw]
    assert refired, "a window that fired before the checkpoint fired again after its re-arm"


@pytest.mark.gpu
def test_restore_rejections():
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    sc = SCEN["tumbling_lateness_i64"]
    want = _expected(sc)
    kg = max(want, key=lambda k: len(want[k][0]))
    st, tm = want[kg]
    e = WindowEngine(_cfg(sc))
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink(kg, sc["layout"], st[:-3], tm, sc["checkpoint_wm"])
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink(kg, ("key", "sum"), st, tm, sc["checkpoint_wm"])    # f1 is tracked: layout must name it
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink((kg + 1) % 8, sc["layout"], st, tm, sc["checkpoint_wm"])   # another key group's section
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    e.restore_kg_flink(kg, sc["layout"], st, tm, sc["checkpoint_wm"])
    with pytest.raises(_abi.FwError):
        e.restore_kg_flink((kg + 1) % 8, sc["layout"], *want[(kg + 1) % 8], sc["checkpoint_wm"] + 1)
    e.close()
    sl = dict(SCEN["sliding_i64"])
    sl["config"] = dict(sl["config"], lateness=100)   # timers of a lateness-0 checkpoint: rejected
    e = WindowEngine(_cfg(sl))
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink(0, sl["layout"], *_expected(sl)[0])
    assert ei.value.code == _abi.FW_ERR_UNSUPPORTED
    e.close()
    # no record accepted yet: no keyed state at all (HeapKeyedStateBackend.snapshot writes no stream)
    e = WindowEngine(_cfg(sc))
    st0, tm0 = e.snapshot_kg_flink(0, sc["layout"])
    assert st0 == b"" and tm0 == bytes(8)
    e.close()


def _purging_lateness_run(factory_g, mode, restore_at, sliding=False):
    """PurgingTrigger + allowed lateness 400 (tumbling 1 s): a window's fire purges its state but each key keeps its
    cleanup timer until maxTimestamp + 400 (WindowOperator.java:365-371 clears the contents only; the timer is
    deleted at cleanup, :420-428), and a per-element fire within the lateness registers one for a key that had
    none.  Snapshot at a watermark with purged windows inside their lateness; restore (at that watermark, or at
    Long.MIN_VALUE as the reference restarts its timers) and continue."""
    from flink_amd.windowing import (EventTimeTrigger, PurgingTrigger, ReduceFunction, SlidingEventTimeWindows,
                                     TumblingEventTimeWindows, make_config)
    from harness import drive, gen_stream
    from oracle.oracle import OracleEngine
    keys, ts, vals = gen_stream(48_000, 2000, rate=1 << 13, zipf=1.1, ooo=300)   # ~6 s of event time
    f1 = np.arange(len(keys), dtype=np.int64) * 3 + 1
    kw = dict(max_parallelism=128, key_capacity=1 << 13, max_batch=1 << 13, out_capacity=1 << 20)
    if mode:
        kw["ingest_mode"] = mode
    # (sliding 2 s / 1 s: window [1 s, 3 s) fired and purged at the checkpoint, within its lateness; its slices
    # also feed the unfired [2 s, 4 s))
    asg = SlidingEventTimeWindows.of(2000, 1000) if sliding else TumblingEventTimeWindows.of(1000)
    cfg = make_config(asg, ReduceFunction(("sum", "max"), "i64", True), PurgingTrigger.of(EventTimeTrigger.create()),
                      400, **kw)
    layout = ("f1", "key", "max", "sum")
    n = int(3.25 * (1 << 13)) + 17   # checkpoint watermark ~3.13 s: window [2 s, 3 s) fired, within its lateness
    wm_cut = int(ts[:n].max()) - 120
    assert 2999 < wm_cut < 3399
    blobs = {}
    for name, factory in (("g", factory_g), ("o", OracleEngine)):
        if factory is None:
            continue
        e = factory(cfg)
        drive(e, keys[:n], ts[:n], vals[:n], 2048, 120, None, f1=f1[:n])
        blobs[name] = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        e.close()
    # cleanup timers without state: (key, window) pairs in the timer section that the state section lacks
    ghosts = 0
    for kg, (st, tm) in blobs["o"].items():
        have = set()
        if st and st[6]:
            pos, (nns,) = 11, struct.unpack(">i", st[7:11])
            for _ in range(nns):
                start, end, ne = struct.unpack(">qqi", st[pos:pos + 20])
                pos += 20
                for _ in range(ne):
                    (k,) = struct.unpack(">q", st[pos:pos + 8])
                    have.add((k, start))
                    pos += 8 * (1 + len(layout))
        (nt,) = struct.unpack(">i", tm[:4])
        for j in range(nt):
            k, start, end, t = struct.unpack(">qqqq", tm[4 + 32 * j:36 + 32 * j])
            ghosts += (k, start) not in have
    assert ghosts > 50, ghosts
    wm = wm_cut if restore_at == "checkpoint" else LONG_MIN
    outs = {}
    for name, factory in (("g", factory_g), ("o", OracleEngine)):
        if factory is None:
            continue
        e = factory(cfg)
        for kg, (st, tm) in blobs["o"].items():
            e.restore_kg_flink(kg, layout, st, tm, wm)
        back = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        assert _diff(back, blobs["o"]) is None, _diff(back, blobs["o"])
        outs[name] = _canon(epochs_of(drive(e, keys[n:], ts[n:], vals[n:], 2048, 120, LONG_MAX, f1=f1[n:]),
                                      ["sum_i64", "max_i64"], True))
        e.close()
    return blobs, outs


@pytest.mark.parametrize("sliding", [False, True])
@pytest.mark.parametrize("restore_at", ["checkpoint", "long_min"])
def test_oracle_purging_lateness_round_trip(restore_at, sliding):
    _purging_lateness_run(None, 0, restore_at, sliding)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("restore_at", ["checkpoint", "long_min"])
@pytest.mark.parametrize("sliding", [False, True])
def test_purging_lateness_checkpoint(mode, restore_at, sliding):
    """The engine's sections byte-identical with the oracle's (purged windows' cleanup timers included), its
    restore writes them back, and the restored engine continues as the restored oracle.  Sliding (round 6): a fired
    window's state is purged though its slices stay for the windows that share them; its keys whose first element
    preceded the fire keep a cleanup timer without state."""
    from flink_amd.windowing import WindowEngine
    blobs, outs = _purging_lateness_run(WindowEngine, mode, restore_at, sliding)
    assert _diff(blobs["g"], blobs["o"]) is None, _diff(blobs["g"], blobs["o"])
    assert outs["g"] == outs["o"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_sliding_lateness_checkpoint(mode):
    """SlidingEventTimeWindows.of(3 s, 1 s) with allowed lateness 1.5 s, checkpointed while fired windows are kept
    for their lateness: the engine's sections equal the oracle's, restore (at the checkpoint's watermark) writes them
    back — each window's state in its own window pane — and the restored engine's per-element fires and watermark
    fires continue as the restored oracle's, restored at the checkpoint's watermark or at Long.MIN_VALUE (windows
    that fired before the checkpoint: disarmed window panes, re-armed per key by later records)."""
    from flink_amd.windowing import ReduceFunction, SlidingEventTimeWindows, WindowEngine, make_config
    from harness import drive, gen_stream
    from oracle.oracle import OracleEngine
    keys, ts, vals = gen_stream(48_000, 1500, rate=1 << 13, zipf=1.1, ooo=400)
    f1 = np.arange(len(keys), dtype=np.int64) * 5 + 2
    cfg = make_config(SlidingEventTimeWindows.of(3000, 1000), ReduceFunction(("sum", "count"), "i64", True), None, 1500,
                      max_parallelism=128, key_capacity=1 << 13, max_batch=1 << 13, out_capacity=1 << 20, ingest_mode=mode)
    layout = ("key", "f1", "sum", "count")
    n = int(3.25 * (1 << 13)) + 29
    wm_cut = int(ts[:n].max()) - 120
    blobs = {}
    for name, factory in (("g", WindowEngine), ("o", OracleEngine)):
        e = factory(cfg)
        drive(e, keys[:n], ts[:n], vals[:n], 2048, 120, None, f1=f1[:n])
        blobs[name] = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        e.close()
    assert _diff(blobs["g"], blobs["o"]) is None, _diff(blobs["g"], blobs["o"])
    outs = {}
    for name, factory in (("g", WindowEngine), ("o", OracleEngine)):
        e = factory(cfg)
        for kg, (st, tm) in blobs["o"].items():
            e.restore_kg_flink(kg, layout, st, tm, wm_cut)
        back = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        assert _diff(back, blobs["o"]) is None, _diff(back, blobs["o"])
        outs[name] = _canon(epochs_of(drive(e, keys[n:], ts[n:], vals[n:], 2048, 120, LONG_MAX, f1=f1[n:]),
                                      ["sum_i64", "count"], True))
        e.close()
    assert outs["g"] == outs["o"]
    late = [r for w, recs in outs["o"] if w != "tail" for r in recs if r[1] < wm_cut]
    assert late, "windows kept for their lateness fired again after the restore"
    # restored at Long.MIN_VALUE: a window that fired before the checkpoint (its panes carry only cleanup timers)
    # is restored with its own pane disarmed — it fires at its maxTimestamp only for the keys a later record
    # re-armed (EventTimeTrigger.onElement), the others wait for their cleanup — as the oracle restored alike
    outs = {}
    for name, factory in (("g", WindowEngine), ("o", OracleEngine)):
        e = factory(cfg)
        for kg, (st, tm) in blobs["o"].items():
            e.restore_kg_flink(kg, layout, st, tm, LONG_MIN)
        back = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        assert _diff(back, blobs["o"]) is None, _diff(back, blobs["o"])
        res = drive(e, keys[n:], ts[n:], vals[n:], 2048, 120, None, f1=f1[n:])
        mid = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        e.advance_watermark(LONG_MAX)
        res.append(e.collect())
        outs[name] = (_canon(epochs_of(res, ["sum_i64", "count"], True)), mid)
        e.close()
    assert outs["g"][0] == outs["o"][0]
    assert _diff(outs["g"][1], outs["o"][1]) is None, _diff(outs["g"][1], outs["o"][1])
    refired = [r for w, recs in outs["o"][0] if w != "tail" for r in recs if r[1] < wm_cut]
    assert refired, "a window that fired before the checkpoint fired again for re-armed keys"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_native_snapshot_purging_lateness(mode):
    """PurgingTrigger + allowed lateness through the engine's own blob (fw_snapshot_kg): refused while a purged window
    is within its lateness (its keys' cleanup timers have no place in that format, only in the reference layout);
    taken between two such periods, restored, and continued — late records, per-element fires and purges, windows
    reusing slice slots — the engine's results and reference-layout sections (purged windows' cleanup timers
    included) equal an oracle that ran through without the checkpoint.  (a slot's purged-window
    ordinals were inherited by the next window claiming the slot, and a native round trip lost the tracking.)"""
    from flink_amd import _abi
    from flink_amd.windowing import (EventTimeTrigger, PurgingTrigger, ReduceFunction, TumblingEventTimeWindows,
                                     WindowEngine, make_config)
    from harness import drive, gen_stream
    from oracle.oracle import OracleEngine
    keys, ts, vals = gen_stream(64_000, 2000, rate=1 << 13, zipf=1.1, ooo=300)   # ~7.8 s of event time
    f1 = np.arange(len(keys), dtype=np.int64) * 3 + 1
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "max"), "i64", True),
                      PurgingTrigger.of(EventTimeTrigger.create()), 400, max_parallelism=128, key_capacity=1 << 13,
                      max_batch=1 << 13, out_capacity=1 << 20, max_open_slices=4, ingest_mode=mode)
    layout = ("f1", "key", "max", "sum")
    B = 2048
    wm_after = lambda n: int(ts[:n].max()) - 120   # drive()'s watermark after the batch ending at n
    cuts = [n for n in range(B * 4, B * 20, B)]
    inside = next(n for n in cuts if 0 <= wm_after(n) % 1000 < 380)     # a fired window within its lateness
    between = next(n for n in cuts if 420 <= wm_after(n) % 1000 < 990)  # none: cleanup passed, next not fired
    e = WindowEngine(cfg)
    drive(e, keys[:inside], ts[:inside], vals[:inside], B, 120, None, f1=f1[:inside])
    with pytest.raises(_abi.FwError) as ei:
        e.snapshot_kg(0)
    assert ei.value.code == _abi.FW_ERR_UNSUPPORTED
    e.close()
    n = between
    # the engine up to the cut, its own blobs, a fresh engine restored from them
    e = WindowEngine(cfg)
    drive(e, keys[:n], ts[:n], vals[:n], B, 120, None, f1=f1[:n])
    blobs = {kg: e.snapshot_kg(kg) for kg in range(128)}
    e.close()
    g = WindowEngine(cfg)
    for kg, blob in blobs.items():
        g.restore_kg(kg, blob)
    o = OracleEngine(cfg)
    drive(o, keys[:n], ts[:n], vals[:n], B, 120, None, f1=f1[:n])
    m = len(keys) - 3 * B   # continue up to a point with purged windows within their lateness, then compare
    outs = {}
    for name, eng in (("g", g), ("o", o)):
        outs[name] = _canon(epochs_of(drive(eng, keys[n:m], ts[n:m], vals[n:m], B, 120, None, f1=f1[n:m]),
                                      ["sum_i64", "max_i64"], True))
    assert outs["g"] == outs["o"]
    assert any(r[1] < w for w, recs in outs["o"] if w != "tail" for r in recs), "per-element fires after the restore"
    sg = {kg: g.snapshot_kg_flink(kg, layout) for kg in range(128)}
    so = {kg: o.snapshot_kg_flink(kg, layout) for kg in range(128)}
    assert _diff(sg, so) is None, _diff(sg, so)
    assert any(tm != b"\x00\x00\x00\x00" and len(tm) > 4 for _, tm in so.values())
    g.close()
    o.close()


FOLD_CASES = [("sum", 123456789, "i64", "tumbling"), ("count", -7, "i64", "sliding"), ("max", 1 << 62, "i64", "tumbling"),
              ("min", 0.25, "f64", "sliding"), ("sum", 2.5, "f64", "tumbling")]


def _fold_run(factory, kind, initial, vt, assigner, mode, restore=None):
    """Drive 2/3 of a Zipf stream through a fold engine and snapshot every key group in the reference layout
    (the key and the accumulator: HeapFoldingState's value); or restore such snapshots at their watermark and
    drive the rest to a final MAX_WATERMARK."""
    from flink_amd.windowing import FoldFunction, SlidingEventTimeWindows, TumblingEventTimeWindows, make_config
    from harness import drive, gen_stream
    a = TumblingEventTimeWindows.of(1000) if assigner == "tumbling" else SlidingEventTimeWindows.of(3000, 1000)
    keys, ts, vals = gen_stream(40_000, 2000, rate=1 << 14, zipf=1.1, ooo=300, value_type=vt)
    cfg = make_config(a, FoldFunction(kind, initial, vt), None, 0, max_parallelism=128, key_capacity=1 << 13,
                      max_batch=1 << 14, out_capacity=1 << 20, ingest_mode=mode)
    layout = ("key", kind)
    n = len(keys) * 2 // 3
    wm = int(ts[:n].max()) - 120
    e = factory(cfg)
    if restore is None:
        drive(e, keys[:n], ts[:n], vals[:n], 4096, 120, None)
        snaps = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        e.close()
        return snaps, wm
    for kg, (st, tm) in restore.items():
        e.restore_kg_flink(kg, layout, st, tm, wm)
    back = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
    out = drive(e, keys[n:], ts[n:], vals[n:], 4096, 120, LONG_MAX)
    e.close()
    return back, out


@pytest.mark.parametrize("kind,initial,vt,assigner", FOLD_CASES)
def test_oracle_fold_checkpoint_round_trip(kind, initial, vt, assigner):
    """The oracle's HeapFoldingState sections restore and snapshot back byte for byte."""
    from oracle.oracle import OracleEngine
    snaps, _ = _fold_run(OracleEngine, kind, initial, vt, assigner, 0)
    assert sum(len(s) for s, _ in snaps.values()) > 128 * 8
    back, _ = _fold_run(OracleEngine, kind, initial, vt, assigner, 0, restore=snaps)
    assert _diff(back, snaps) is None


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("kind,initial,vt,assigner", FOLD_CASES)
def test_fold_checkpoint(mode, kind, initial, vt, assigner):
    """fold in the reference layout (WindowOperator's window-contents as HeapFoldingState: the initial value
    folded with the window's records).  The engine's sections are byte-identical to the oracle's, it restores
    the oracle's sections (subtracting a sum or count's initial value back out), snapshots them back unchanged
    and continues like the oracle restored from the same bytes — exactly, but for a double sum with a
    non-zero initial value (relative 1e-12: the engine adds the initial value once, at the fire)."""
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    g, _ = _fold_run(WindowEngine, kind, initial, vt, assigner, mode)
    o, _ = _fold_run(OracleEngine, kind, initial, vt, assigner, 0)
    # a double sum is associated differently (slices, then the initial value): same layout, values to 1e-12
    exact = not (vt == "f64" and kind == "sum")
    if exact:
        assert _diff(g, o) is None, _diff(g, o)
    else:
        assert {kg: (len(a), b) for kg, (a, b) in g.items()} == {kg: (len(a), b) for kg, (a, b) in o.items()}
    back, out_g = _fold_run(WindowEngine, kind, initial, vt, assigner, mode, restore=o)
    _, out_o = _fold_run(OracleEngine, kind, initial, vt, assigner, 0, restore=o)
    if exact:
        assert _diff(back, o) is None
    field = "count" if kind == "count" else f"{kind}_{vt}"
    from harness import epochs_of
    eg, eo = epochs_of(out_g, [field]), epochs_of(out_o, [field])
    assert [w for w, _ in eg] == [w for w, _ in eo] and sum(len(r) for _, r in eo) > 1000
    for (w, rg), (_, ro) in zip(eg, eo):
        if exact:
            assert rg == ro, w
        else:
            assert len(rg) == len(ro) and all(x[:2] == y[:2] and abs(x[2] - y[2]) <= 1e-12 * max(1.0, abs(y[2]))
                                              for x, y in zip(rg, ro)), w


def _list_run(factory, vt, lateness, mode, restore=None, layout=("key", "f1", "value"), restore_wm=None, pre=None,
              sliding=False, slide=1000):
    """List state (WindowedStream.apply: HeapListState "window-contents" of the input tuples), tumbling 1 s windows
    or (sliding) 3 s windows every 1 s: drive 2/3 of a Zipf stream, snapshot every key group in the reference
    layout; or restore such sections at their watermark and drive the rest to a final MAX_WATERMARK."""
    from flink_amd.windowing import ListStateDescriptor, SlidingEventTimeWindows, TumblingEventTimeWindows, make_config
    from harness import drive, gen_stream
    keys, ts, vals = gen_stream(24_000, 1200, rate=1 << 13, zipf=1.1, ooo=300, value_type=vt)
    f1 = np.arange(len(keys), dtype=np.int64) * 7 + 3
    asg = SlidingEventTimeWindows.of(3000, slide) if sliding else TumblingEventTimeWindows.of(1000)
    cfg = make_config(asg, ListStateDescriptor(vt), None, lateness, max_parallelism=128,
                      key_capacity=1 << 12, max_batch=1 << 12, out_capacity=1 << 20, ingest_mode=mode)
    n = len(keys) * 2 // 3
    wm = int(ts[:n].max()) - 100
    e = factory(cfg)
    if restore is None:
        drive(e, keys[:n], ts[:n], vals[:n], 2048, 100, None, f1=f1[:n])
        snaps = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
        e.close()
        return snaps
    for kg, (st, tm) in restore.items():
        e.restore_kg_flink(kg, layout, st, tm, wm if restore_wm is None else restore_wm)
    back = {kg: e.snapshot_kg_flink(kg, layout) for kg in range(128)}
    first = []
    if pre is not None:   # records pushed right after the restore, before any watermark
        sel = np.arange(pre)
        e.push(keys[sel].copy(), 600 + sel.astype(np.int64), vals[sel].copy(), f1=90_000 + sel.astype(np.int64))
        first = [e.collect()]
    out = first + drive(e, keys[n:], ts[n:], vals[n:], 2048, 100, LONG_MAX, f1=f1[n:])
    e.close()
    return back, out


@pytest.mark.parametrize("vt,lateness", [("i64", 0), ("f64", 400), ("i64", 900)])
def test_oracle_list_checkpoint_round_trip(vt, lateness):
    """The oracle's HeapListState sections (ListSerializer: int size, then the elements) restore and snapshot
    back byte for byte."""
    from oracle.oracle import OracleEngine
    snaps = _list_run(OracleEngine, vt, lateness, 0)
    assert sum(len(s) for s, _ in snaps.values()) > 128 * 8
    back, _ = _list_run(OracleEngine, vt, lateness, 0, restore=snaps)
    assert _diff(back, snaps) is None


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("vt,lateness", [("i64", 0), ("f64", 400), ("i64", 900)])
def test_list_checkpoint(mode, vt, lateness):
    """List state of tumbling windows in the reference layout: the engine's sections (its slices' element
    buffers grouped per window and key in arrival order) are byte-identical to the oracle's; the engine
    restores the oracle's sections (elements back into the slices, ahead of every later arrival), writes them
    back unchanged, and its fires — watermark fires and, under allowed lateness, per-element re-fires — continue
    exactly as the oracle restored from the same bytes."""
    from flink_amd.windowing import WindowEngine
    from harness import epochs_of
    from oracle.oracle import OracleEngine
    g = _list_run(WindowEngine, vt, lateness, mode)
    o = _list_run(OracleEngine, vt, lateness, 0)
    assert _diff(g, o) is None, _diff(g, o)
    back, out_g = _list_run(WindowEngine, vt, lateness, mode, restore=o)
    _, out_o = _list_run(OracleEngine, vt, lateness, 0, restore=o)
    assert _diff(back, o) is None, _diff(back, o)
    field = f"sum_{vt}"
    eg, eo = _canon(epochs_of(out_g, [field], True)), _canon(epochs_of(out_o, [field], True))
    assert eg == eo and sum(len(r) for _, r in eo) > 1000


@pytest.mark.parametrize("vt,lateness,slide", [("i64", 0, 1000), ("f64", 800, 1000), ("i64", 500, 2000)])
def test_oracle_sliding_list_checkpoint_round_trip(vt, lateness, slide):
    """Sliding windows' list state: every window's list of its elements (a record sits in each of its windows'
    lists) restores and snapshots back byte for byte in the oracle."""
    from oracle.oracle import OracleEngine
    snaps = _list_run(OracleEngine, vt, lateness, 0, sliding=True, slide=slide)
    assert sum(len(s) for s, _ in snaps.values()) > 128 * 8
    back, _ = _list_run(OracleEngine, vt, lateness, 0, restore=snaps, sliding=True, slide=slide)
    assert _diff(back, snaps) is None


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("vt,lateness,slide", [("i64", 0, 1000), ("f64", 800, 1000), ("i64", 500, 2000)])
def test_sliding_list_checkpoint(mode, vt, lateness, slide):
    """Sliding-window list state in the reference layout (round 6): the engine writes each window's list — its
    slices' elements of the key merged in arrival order — byte-identical to the oracle's; it restores the oracle's
    sections by peeling the windows newest first (a window's list less the elements of its newer slices, matched in
    order, is its oldest slice), writes them back unchanged, and continues exactly as the oracle restored from the
    same bytes.  A slide that does not divide the size (3 s every 2 s: slices of 1 s, a window starting every second
    slice): each element is identified across its windows' lists, its live windows pick its slice, and the arrival
    order is one every list agrees with."""
    from flink_amd.windowing import WindowEngine
    from harness import epochs_of
    from oracle.oracle import OracleEngine
    g = _list_run(WindowEngine, vt, lateness, mode, sliding=True, slide=slide)
    o = _list_run(OracleEngine, vt, lateness, 0, sliding=True, slide=slide)
    assert _diff(g, o) is None, _diff(g, o)
    back, out_g = _list_run(WindowEngine, vt, lateness, mode, restore=o, sliding=True, slide=slide)
    _, out_o = _list_run(OracleEngine, vt, lateness, 0, restore=o, sliding=True, slide=slide)
    assert _diff(back, o) is None, _diff(back, o)
    field = f"sum_{vt}"
    eg, eo = _canon(epochs_of(out_g, [field], True)), _canon(epochs_of(out_o, [field], True))
    assert eg == eo and sum(len(r) for _, r in eo) > 1000


@pytest.mark.gpu
def test_list_checkpoint_rejections():
    """Sliding-window list state (slide not dividing the size) whose windows' lists share no consistent slices — an
    element missing from a window between two that hold it — is refused."""
    from flink_amd import _abi
    from flink_amd.keygroups import assign_to_key_group
    from flink_amd.windowing import ListStateDescriptor, SlidingEventTimeWindows, WindowEngine, make_config
    e = WindowEngine(make_config(SlidingEventTimeWindows.of(3000, 1000 * 2), ListStateDescriptor(),
                                 max_parallelism=128))
    key = 7
    kg = assign_to_key_group(key, 128)
    el = struct.pack(">qqq", key, 11, 5)   # (key, f1, value)
    other = struct.pack(">qqq", key, 12, 6)
    body = struct.pack(">i", 3)
    for start, elems in ((0, [el]), (2000, [other]), (4000, [el])):   # el in windows 0 and 2, not in window 1
        body += struct.pack(">qqi", start, start + 3000, 1) + struct.pack(">q", key) + struct.pack(">i", len(elems))
        body += b"".join(elems)
    st = struct.pack(">ihb", kg, 0, 1) + body
    tm = b"".join(struct.pack(">qqqq", key, s0, s0 + 3000, s0 + 2999) for s0 in (0, 2000, 4000))
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink(kg, ("key", "f1", "value"), st, struct.pack(">i", 3) + tm + struct.pack(">i", 0), -1)
    assert ei.value.code in (_abi.FW_ERR_INVALID_ARG, _abi.FW_ERR_UNSUPPORTED)
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_list_restore_at_long_min(mode):
    """Tumbling list state restored at Long.MIN_VALUE while window [0, 1000) had fired and was kept for its lateness
    (its entries carry only cleanup timers): restored disarmed, it fires again at its maxTimestamp only for the keys a
    later record re-armed, with every element so far (EventTimeTrigger.onElement), the others wait for their cleanup —
    as the oracle restored from the same bytes; the sections are written back unchanged."""
    from harness import epochs_of
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    o = _list_run(OracleEngine, "i64", 900, 0)
    outs = {}
    for name, factory, md in (("g", WindowEngine, mode), ("o", OracleEngine, 0)):
        back, out = _list_run(factory, "i64", 900, md, restore=o, restore_wm=LONG_MIN, pre=40)
        assert _diff(back, o) is None, (name, _diff(back, o))
        outs[name] = _canon(epochs_of(out, ["sum_i64"], True))
    assert outs["g"] == outs["o"]
    refired = [r for w, recs in outs["o"] if w != "tail" for r in recs if r[1] < 1000]
    assert refired, "the window that fired before the checkpoint fired again for re-armed keys"
