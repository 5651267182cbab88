"""Ingest from Flink's wire format (fw_decode): length-prefixed
StreamElementSerializer elements over a TupleSerializer tuple (SpanningRecordSerializer.java:69-92,
StreamElementSerializer.java:155-198, TupleSerializer.java:120-139) decoded into the record columns
fw_push_batch takes, plus watermarks and latency markers with their record positions.

tests/golden/wire_stream.json is encoded by tests/golden/make_wire_fixture.py from the format's definition
(no JVM here to produce buffers): it pins the oracle's decoder on CPU; the GPU decoder is checked against
the fixture and against the oracle on large random streams, cut into 32 KiB network buffers.
"""
import json
import os
import struct

import numpy as np
import pytest

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "wire_stream.json")))
SCEN = {s["name"]: s for s in FIX["scenarios"]}
LONG_MIN, LONG_MAX = -(1 << 63), (1 << 63) - 1


def _engine(factory, sc):
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    vt = "f64" if sc["fields"][sc["value"]] == "double" else "i64"
    return factory(make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), vt, True), None, 0,
                               key_capacity=1 << 12, max_batch=1 << 14, out_capacity=1 << 16))


def _decode(e, sc, data, **kw):
    return e.decode(data, sc["fields"], key=sc["key"], value=sc["value"], f1=sc["f1"], **kw)


def _check(out, sc):
    recs = np.array(sc["records"], dtype=np.int64).reshape(-1, 4)
    assert out["n_records"] == len(recs)
    assert np.array_equal(out["key"], recs[:, 0])
    assert np.array_equal(out["f1"], recs[:, 1])
    assert np.array_equal(out["ts"], recs[:, 2])
    assert np.array_equal(np.asarray(out["value"]).view(np.int64), recs[:, 3])
    if sc["fields"][sc["key"]] == "int":
        assert np.array_equal(out["key_hash"], recs[:, 0].astype(np.int32))   # Integer.hashCode
    assert [list(x) for x in zip(out["wm"].tolist(), out["wm_pos"].tolist())] == sc["watermarks"]
    lms = [[int(a), int(b), int(p)] for (a, b), p in zip(out["lm"].tolist(), out["lm_pos"].tolist())]
    assert lms == sc["latency_markers"]


@pytest.mark.parametrize("name", list(SCEN))
def test_oracle_decodes_fixture(name):
    from oracle.oracle import OracleEngine
    sc = SCEN[name]
    e = _engine(OracleEngine, sc)
    data = bytes.fromhex(sc["stream"])
    out = _decode(e, sc, data)
    e.close()
    assert out["consumed"] == len(data)
    _check(out, sc)


@pytest.mark.parametrize("name", list(SCEN))
def test_oracle_decodes_buffer_by_buffer(name):
    """32 KiB network buffers, an element spanning two of them left for the next call (consumed)."""
    from oracle.oracle import OracleEngine
    sc = SCEN[name]
    e = _engine(OracleEngine, sc)
    data = bytes.fromhex(sc["stream"])
    acc, carry = [], b""
    for s in range(0, len(data), 32 << 10):
        buf = carry + data[s:s + (32 << 10)]
        out = _decode(e, sc, buf)
        acc.append(out)
        carry = buf[out["consumed"]:]
    e.close()
    assert carry == b""
    assert sum(o["n_records"] for o in acc) == len(sc["records"])
    assert np.array_equal(np.concatenate([o["key"] for o in acc]), np.array([r[0] for r in sc["records"]], np.int64))


# ---------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("device_input", [False, True])
@pytest.mark.parametrize("name", list(SCEN))
def test_gpu_decodes_fixture(name, device_input):
    import torch
    from flink_amd.windowing import WindowEngine
    sc = SCEN[name]
    e = _engine(WindowEngine, sc)
    data = bytes.fromhex(sc["stream"])
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda() if device_input else data
    out = _decode(e, sc, src)
    assert out["consumed"] == len(data)
    _check(out, sc)
    # cut anywhere: the decoded prefix is whole elements, the rest is carried
    for cut in (len(data) // 3 + 1, len(data) - 5):
        part = _decode(e, sc, data[:cut])
        rest = _decode(e, sc, data[part["consumed"]:])
        assert part["consumed"] <= cut and part["n_records"] + rest["n_records"] == len(sc["records"])
    e.close()


def _random_stream(n, seed, fields=("long", "long", "long")):
    """Large stream: the fixture generator's element writer over seeded numpy draws."""
    rng = np.random.default_rng(seed)
    kinds = rng.choice(3, size=n, p=[0.97, 0.02, 0.01])
    parts = []
    tsv = 1_700_000_000_000 + np.cumsum(rng.integers(0, 3, n))
    keys = rng.integers(0, 1 << 40, n)
    keys[rng.random(n) < 0.3] = 33                              # looks like a record length to a misaligned scan
    vals = rng.integers(-(1 << 62), 1 << 62, n)
    for i in range(n):
        if kinds[i] == 0:
            body = struct.pack(">bqqqq", 0, int(tsv[i]), int(keys[i]), i, int(vals[i]))
        elif kinds[i] == 1:
            body = struct.pack(">bq", 2, int(tsv[i]) - 100)
        else:
            body = struct.pack(">bqii", 3, int(tsv[i]), 7, i % 64)
        parts.append(struct.pack(">i", len(body)) + body)
    return b"".join(parts)


@pytest.mark.gpu
def test_gpu_matches_oracle_on_large_stream():
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    sc = dict(fields=["long", "long", "long"], key=0, value=2, f1=1)   # Tuple3(key, i, value)
    data = _random_stream(200_000, 5, sc["fields"])
    res = []
    for factory in (WindowEngine, OracleEngine):
        from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
        e = factory(make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 0,
                                key_capacity=1 << 12, max_batch=1 << 14, out_capacity=1 << 16))
        res.append(_decode(e, sc, data, record_cap=1 << 18, marker_cap=1 << 14))
        e.close()
    g, o = res
    assert g["consumed"] == o["consumed"] == len(data)
    for k in ("key", "f1", "ts", "value", "wm", "wm_pos", "lm", "lm_pos"):
        assert np.array_equal(g[k], o[k]), k
    assert g["n_records"] > 190_000 and g["n_watermarks"] > 3000


@pytest.mark.gpu
def test_gpu_rejects_corrupt_stream():
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    sc = SCEN["tuple3_long"]
    e = _engine(WindowEngine, sc)
    data = bytearray(bytes.fromhex(sc["stream"]))
    pos = 0
    while pos < 20000:   # the element boundary at or after byte 20000
        pos += 4 + struct.unpack(">i", bytes(data[pos:pos + 4]))[0]
    data[pos:pos + 4] = struct.pack(">i", 0x7fff)   # a length no element has, mid-stream
    with pytest.raises(_abi.FwError) as ei:
        _decode(e, sc, bytes(data))
    assert ei.value.code == _abi.FW_ERR_INVALID_ARG
    e.close()


@pytest.mark.gpu
def test_decode_then_window_end_to_end():
    """Decoded device columns go straight to fw_push_batch, watermarks at their record positions: the same
    fired windows as the oracle fed the fixture's records."""
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    from harness import epochs_of
    sc = SCEN["tuple3_long"]
    data = bytes.fromhex(sc["stream"])
    recs = np.array(sc["records"], dtype=np.int64).reshape(-1, 4)
    ok = recs[:, 2] != LONG_MIN   # records without timestamp would fail the assigner: left out here
    keep = np.nonzero(ok)[0]
    results = []
    eg = _engine(WindowEngine, sc)
    d = _decode(eg, sc, data, device=True)
    import torch
    sel = torch.from_numpy(keep).cuda()
    k, f1, ts, v = (d[c].index_select(0, sel) for c in ("key", "f1", "ts", "value"))
    pos = np.searchsorted(keep, d["wm_pos"].cpu().numpy())   # watermark positions among the kept records
    start, out, top = 0, [], LONG_MIN
    for w, p in zip(d["wm"].cpu().numpy().tolist(), pos.tolist()):
        if w <= top:   # StreamInputProcessor forwards only increasing watermarks (:147-161)
            continue
        top = w
        if p > start:
            eg.push(k[start:p], ts[start:p], v[start:p], f1=f1[start:p])
            start = p
        eg.advance_watermark(w)
        out.append(eg.collect())
    eg.push(k[start:], ts[start:], v[start:], f1=f1[start:])
    eg.advance_watermark(LONG_MAX)
    out.append(eg.collect())
    eg.close()
    eo = _engine(OracleEngine, sc)
    r = recs[keep]
    start, ro, top = 0, [], LONG_MIN
    for (w, p0) in sc["watermarks"]:
        if w <= top:
            continue
        top = w
        p = int(np.searchsorted(keep, p0))
        if p > start:
            eo.push(r[start:p, 0].copy(), r[start:p, 2].copy(), r[start:p, 3].copy(), f1=r[start:p, 1].copy())
            start = p
        eo.advance_watermark(w)
        ro.append(eo.collect())
    eo.push(r[start:, 0].copy(), r[start:, 2].copy(), r[start:, 3].copy(), f1=r[start:, 1].copy())
    eo.advance_watermark(LONG_MAX)
    ro.append(eo.collect())
    eo.close()
    assert epochs_of(out, ["sum_i64"], True) == epochs_of(ro, ["sum_i64"], True)


@pytest.mark.gpu
def test_gpu_decode_begin_end_pipelined():
    """fw_decode_begin / fw_decode_end: two decodes in flight (the second enqueued before the first's counts are
    read), each equal to the synchronous fw_decode of the same bytes, ended in any order; a third outstanding
    begin and an unknown ticket are rejected."""
    from flink_amd import _abi
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
    sc = dict(fields=["long", "long", "long"], key=0, value=2, f1=1)
    streams = [_random_stream(60_000, s, sc["fields"]) for s in (7, 8, 9)]
    e = WindowEngine(make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 0,
                                 key_capacity=1 << 12, max_batch=1 << 14, out_capacity=1 << 16))
    kw = dict(key=0, value=2, f1=1, record_cap=1 << 17, marker_cap=1 << 13)
    want = [e.decode(d, sc["fields"], **kw) for d in streams]
    h0 = e.decode_begin(streams[0], sc["fields"], **kw)
    h1 = e.decode_begin(streams[1], sc["fields"], **kw)
    with pytest.raises(_abi.FwError):
        e.decode_begin(streams[2], sc["fields"], **kw)
    got0 = e.decode_end(h0)
    h2 = e.decode_begin(streams[2], sc["fields"], **kw)
    got2 = e.decode_end(h2)   # ends in any order: the newer first, then a begin takes the slot it freed
    h3 = e.decode_begin(streams[0], sc["fields"], **kw)
    got1, got3 = e.decode_end(h1), e.decode_end(h3)
    with pytest.raises(_abi.FwError):
        e.decode_end(h2)
    for g, w in zip((got0, got1, got2, got3), want + want[:1]):
        assert g["consumed"] == w["consumed"] and g["n_records"] == w["n_records"] > 50_000
        for k in ("key", "f1", "ts", "value", "wm", "wm_pos", "lm", "lm_pos"):
            assert np.array_equal(g[k], w[k]), k
    e.close()



@pytest.mark.gpu
def test_gpu_decode_all_chunks_undecided():
    """Every record's timestamp, key, f1 and value bytes read as a record header (length 33, tag 0 / 1) at the same
    offset of every record, so every chunk has false survivors whose exits disagree with the true one: every
    chunk's entry comes from the walk from the nearest decided chunk (here: chunk 0).  Same columns as the oracle."""
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
    from oracle.oracle import OracleEngine
    sc = dict(fields=["long", "long", "long"], key=0, value=2, f1=1)
    n = 12_000
    ts, key, f1, val = 0x0000002100000000, 0x0000002101000000, 0x0000002100000005, 0x0000002100000007
    data = b"".join(struct.pack(">ibqqqq", 33, 0, ts, key, f1, val) for _ in range(n))
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 0,
                      key_capacity=1 << 12, max_batch=1 << 14, out_capacity=1 << 16)
    res = []
    for factory in (WindowEngine, OracleEngine):
        e = factory(cfg)
        res.append(e.decode(data, sc["fields"], key=0, value=2, f1=1, record_cap=1 << 15, marker_cap=1 << 10))
        e.close()
    g, o = res
    assert g["n_records"] == o["n_records"] == n and g["consumed"] == o["consumed"] == len(data)
    for k in ("key", "f1", "ts", "value"):
        assert np.array_equal(g[k], o[k]), k
