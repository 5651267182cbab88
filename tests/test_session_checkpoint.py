"""Session windows' checkpoints in the reference's key-group byte layout.

A session job holds two keyed states (WindowOperator.java:445-460, 724-736):

  "window-contents"     the reducing state, under each in-flight window's STATE window (the window the
                        session started as: MergingWindowSet keeps the first merged window's state window)
  "merging-window-set"  ListState<Tuple2<W, W>> in VoidNamespace: per key its in-flight windows and their state
                        windows (MergingWindowSet.persist, MergingWindowSet.java:91-95), rewritten by snapshotState
                        for every key whose set was fetched since the operator opened, and read back lazily
                        (getMergingWindowSet) the first time a restored key is touched

The key-group section lists both tables in stateTables' HashMap order ("window-contents" first, id 0), then the
timers: each in-flight window's trigger timer (while pending) and cleanup timer.

CPU: the oracle's sections restore and snapshot back byte for byte, and an operator restored from them continues
exactly as the one that wrote them.  GPU: the HIP engine writes the oracle's bytes, restores them, writes them back
unchanged and continues like the oracle restored from the same bytes.

Parity of the byte order is the builder's HashMap model (tests/golden/make_checkpoint_fixture.py's rules) —
unpinned by a JVM run, as for the other checkpoint layouts.
"""
import numpy as np
import pytest

LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1
MP = 128

CASES = [
    # (value type, fields, lateness, purging)
    ("i64", ("sum", "min", "max", "count"), 0, False),
    ("f64", ("sum", "min", "max", "count"), 400, False),
    ("i64", ("sum", "count"), 0, True),
    ("i64", ("maxBy",), 250, False),
    ("i64", ("sum", "count"), 300, True),   # a purged session's cleanup timer outlives it
    ("f64", ("list",), 200, False),          # WindowedStream.apply: each session's elements (HeapListState)
]


def _layout(fields):
    return ("key", "f1") + (("value",) if fields in (("maxBy",), ("minBy",), ("list",)) else tuple(fields))


def _stream(vt):
    from harness import gen_stream
    keys, ts, vals = gen_stream(24_000, 600, rate=1 << 11, zipf=1.1, ooo=300, value_type=vt, seed=7)
    f1 = np.arange(len(keys), dtype=np.int64) * 7 + 3
    return keys, ts, vals, f1


def _config(vt, fields, lateness, purging, list_state=False):
    list_state = list_state or fields == ("list",)
    from flink_amd.windowing import (EventTimeSessionWindows, EventTimeTrigger, ListStateDescriptor, PurgingTrigger,
                                     ReduceFunction, make_config)
    trig = PurgingTrigger.of(EventTimeTrigger.create()) if purging else EventTimeTrigger.create()
    red = ListStateDescriptor(vt) if list_state else ReduceFunction(fields, vt, True)
    return make_config(EventTimeSessionWindows.withGap(150), red, trig, lateness, max_parallelism=MP,
                       key_capacity=1 << 12, max_batch=1 << 12, out_capacity=1 << 20)


def _snap(e, layout):
    return {kg: e.snapshot_kg_flink(kg, layout) for kg in range(MP)}


def _run(factory, case, restore=None, restore_wm=None, cut=(1 / 3, 2 / 3)):
    """Drive the stream to `cut[0]` (snapshot), to `cut[1]` (snapshot), then to the end and a final MAX_WATERMARK.
    With `restore`: restore those sections at `restore_wm` (default: the checkpoint's watermark), snapshot back,
    then drive from `cut[1]` on.  Returns (snapshots, outputs after the last snapshot)."""
    from harness import drive
    vt, fields, lateness, purging = case
    keys, ts, vals, f1 = _stream(vt)
    n1, n2 = int(len(keys) * cut[0]), int(len(keys) * cut[1])
    wm2 = int(ts[:n2].max()) - 100
    layout = _layout(fields)
    e = factory(_config(vt, fields, lateness, purging))
    snaps = []
    if restore is None:
        drive(e, keys[:n1], ts[:n1], vals[:n1], 2048, 100, None, f1=f1[:n1])
        snaps.append(_snap(e, layout))
        drive(e, keys[n1:n2], ts[n1:n2], vals[n1:n2], 2048, 100, None, f1=f1[n1:n2])
        e.advance_watermark(wm2)
        e.collect()
        snaps.append(_snap(e, layout))
    else:
        for kg, (st, tm) in restore.items():
            e.restore_kg_flink(kg, layout, st, tm, wm2 if restore_wm is None else restore_wm)
        snaps.append(_snap(e, layout))
    out = drive(e, keys[n2:], ts[n2:], vals[n2:], 2048, 100, LONG_MAX, f1=f1[n2:])
    e.close()
    return snaps, out


def _diff(got, want):
    for kg in sorted(want):
        for part, g, w in (("state", got[kg][0], want[kg][0]), ("timers", got[kg][1], want[kg][1])):
            if g != w:
                at = next((i for i in range(min(len(g), len(w))) if g[i] != w[i]), min(len(g), len(w)))
                return f"kg {kg} {part}: {len(g)} vs {len(w)} bytes, first difference at byte {at}"
    return None


def _epochs(out, case):
    from harness import epochs_of
    vt, fields, _, _ = case
    if fields == ("list",):
        cols = ["sum_" + vt]   # (list state: one row per element, its value in the sum column)
    elif fields == ("maxBy",):
        cols = ["max_" + vt]
    else:
        cols = [f"{f}_{vt}" if f != "count" else "count" for f in fields]
    return epochs_of(out, cols, True)   # (double sums compared exactly: the same values reduced in the same order)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{'-'.join(c[1])}-late{c[2]}-{'purging' if c[3] else 'event'}")
def test_oracle_session_checkpoint_round_trip(case):
    """The oracle's two-table sections restore and snapshot back byte for byte, and the restored operator continues
    exactly as the one that wrote them (same fires, same watermark epochs, to the last bit)."""
    from oracle.oracle import OracleEngine
    snaps, out_a = _run(OracleEngine, case)
    last = snaps[-1]
    assert sum(len(st) for st, _ in last.values()) > 8000, "the checkpoint holds in-flight sessions"
    back, out_b = _run(OracleEngine, case, restore=last)
    assert _diff(back[0], last) is None, _diff(back[0], last)
    ea, eb = _epochs(out_a, case), _epochs(out_b, case)
    assert ea == eb and sum(len(r) for _, r in ea) > 1000


@pytest.mark.parametrize("case", [CASES[1], CASES[4]], ids=["f64-late400", "purging-late300"])
def test_oracle_session_restore_at_long_min(case):
    """Restored at Long.MIN_VALUE (the reference's timer service restarts there): sessions whose trigger fired before
    the checkpoint (kept for their allowed lateness, cleanup timer only) re-arm on their next record and fire again;
    the sections are written back unchanged."""
    from oracle.oracle import OracleEngine
    snaps, _ = _run(OracleEngine, case)
    back, out = _run(OracleEngine, case, restore=snaps[-1], restore_wm=LONG_MIN)
    assert _diff(back[0], snaps[-1]) is None
    assert sum(len(r) for _, r in _epochs(out, case)) > 1000


# ---------------------------------------------------------------- GPU: the HIP engine against the oracle


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{'-'.join(c[1])}-late{c[2]}-{'purging' if c[3] else 'event'}")
def test_session_checkpoint(case):
    """The engine's session sections (both snapshots: the second rewrites every touched key's merging-window-set entry
    after the first's) are byte-identical to the oracle's; the engine restores the oracle's sections, writes them back
    unchanged, and continues exactly as the oracle restored from the same bytes."""
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    g, _ = _run(WindowEngine, case)
    o, out_direct = _run(OracleEngine, case)
    for i in range(len(o)):
        assert _diff(g[i], o[i]) is None, (i, _diff(g[i], o[i]))
    back, out_g = _run(WindowEngine, case, restore=o[-1])
    _, out_o = _run(OracleEngine, case, restore=o[-1])
    assert _diff(back[0], o[-1]) is None, _diff(back[0], o[-1])
    eg, eo = _epochs(out_g, case), _epochs(out_o, case)
    assert eg == eo and eo == _epochs(out_direct, case) and sum(len(r) for _, r in eo) > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("case", [CASES[1], CASES[3]], ids=["f64-late400", "maxBy-late250"])
def test_session_checkpoint_hot_walk(case, monkeypatch):
    """The same with FW_SESS_HOT=4: keys with >= 4 records in a batch are walked by k_sess_walk_hot (one wave per
    key), which keeps the same checkpoint bookkeeping (state windows, put / timer ordinals, namespace log)."""
    monkeypatch.setenv("FW_SESS_HOT", "4")
    test_session_checkpoint(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [CASES[1], CASES[4]], ids=["f64-late400", "purging-late300"])
def test_session_restore_at_long_min(case):
    """As the oracle: a restore at Long.MIN_VALUE re-arms fired-but-kept sessions on their next record (PurgingTrigger:
    purged sessions' restored cleanup timers fire with nothing to clean, fetching their keys' sets)."""
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    o, _ = _run(OracleEngine, case)
    back, out_g = _run(WindowEngine, case, restore=o[-1], restore_wm=LONG_MIN)
    _, out_o = _run(OracleEngine, case, restore=o[-1], restore_wm=LONG_MIN)
    assert _diff(back[0], o[-1]) is None, _diff(back[0], o[-1])
    assert _epochs(out_g, case) == _epochs(out_o, case)


@pytest.mark.gpu
def test_session_checkpoint_rejections():
    """A restored window-contents namespace that is not a session's first window [ts, ts + gap) fails loudly."""
    import struct
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    e = WindowEngine(_config("i64", ("sum",), 0, False))
    kg = 5
    st = struct.pack(">ihbi", kg, 0, 1, 1) + struct.pack(">qqi", 100, 100 + 151, 0)
    with pytest.raises(_abi.FwError) as ei:
        e.restore_kg_flink(kg, ("key", "f1", "sum"), st, struct.pack(">ii", 0, 0))
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    e.close()


@pytest.mark.gpu
def test_session_checkpoint_bookkeeping_off(monkeypatch):
    """FW_SESS_CKPT=0 drops the checkpoint bookkeeping (13-16 % of session throughput): results are
    unchanged, and a reference-layout snapshot fails loudly instead of writing wrong bytes."""
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    from harness import drive
    from oracle.oracle import OracleEngine
    monkeypatch.setenv("FW_SESS_CKPT", "0")
    case = CASES[1]
    vt, fields, lateness, purging = case
    keys, ts, vals, f1 = _stream(vt)
    outs = {}
    for name, factory in (("g", WindowEngine), ("o", OracleEngine)):
        e = factory(_config(vt, fields, lateness, purging))
        outs[name] = _epochs(drive(e, keys, ts, vals, 2048, 100, LONG_MAX, f1=f1), case)
        if name == "g":
            with pytest.raises(_abi.FwError) as ei:
                e.snapshot_kg_flink(0, _layout(fields))
            assert ei.value.code == _abi.FW_ERR_UNSUPPORTED
        e.close()
    assert outs["g"] == outs["o"] and sum(len(r) for _, r in outs["o"]) > 1000
