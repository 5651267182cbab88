"""HIP engine vs the oracle at the geometry bench.py measures (the C1 bench shape had
only a checksum).  Bit-exact on every fired record (key, window maxTimestamp, f1 of the first arrival,
sum / count), per watermark epoch (TestHarnessUtil contract, SJT/util/TestHarnessUtil.java:80-117).

  C1  64 Ki keys, batches of 2^22 events (1024 route tiles, 256 directory buckets of 1024 slots),
      R = 2^24 events per event-time second, a watermark after every batch, 4 batches + MAX_WATERMARK
  C4  the same geometry with Zipf(1.2) keys, R = 2^25 (125-ms batches), timestamps up to 300 ms out of
      order, watermark lag 50 ms, allowed lateness 100 ms: per-element late fires and late drops
  C2  10 M key capacity (the direct ingest form: a directory bucket does not fit LDS), 16 Mi events
      over 10 M keys in batches of 2^22, one window purged and its slot reused

The streams are the bench's synthetic generator (flink_amd.synth), made on the GPU and copied to the
oracle.  Sizes are the bench's; the oracle needs tens of seconds for the largest (C2).
"""
import numpy as np
import pytest
import torch


pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1
T0 = 1_700_000_000_000


def _stream(j, batch, n_keys, rate, vt="i64", zipf=None, ooo=0):
    from flink_amd.synth import stream
    k, t, v = stream(j * batch, batch, n_keys, rate, T0, device="cuda", value_type=vt, zipf=zipf, ooo=ooo)
    return k, t, v


def _run(cfg, batches, batch, n_keys, rate, lag, zipf=None, ooo=0, fields=("sum_i64",)):
    from flink_amd.windowing import WindowEngine
    from oracle.oracle import OracleEngine
    eg, eo = WindowEngine(cfg), OracleEngine(cfg)
    rg, ro = [], []
    max_ts = -(1 << 63)
    for j in range(batches):
        k, t, v = _stream(j, batch, n_keys, rate, zipf=zipf, ooo=ooo)
        max_ts = max(max_ts, int(t.max().item()))
        wm = max_ts - lag
        eg.push(k, t, v)
        eg.advance_watermark(wm)
        rg.append(eg.collect())
        kn, tn, vn = k.cpu().numpy(), t.cpu().numpy(), v.cpu().numpy()
        eo.push(kn, tn, vn)
        eo.advance_watermark(wm)
        ro.append(eo.collect())
    for e, out in ((eg, rg), (eo, ro)):
        e.advance_watermark(LONG_MAX)
        out.append(e.collect())
    sg, so = eg.stats(), eo.stats()
    eg.close()
    eo.close()
    a, b = _epochs_np(rg, fields), _epochs_np(ro, fields)
    assert [w for w, _ in a] == [w for w, _ in b]
    for (w, x), (_, y) in zip(a, b):
        assert x.shape == y.shape, f"wm {w}: {x.shape[0]} vs {y.shape[0]} records"
        assert np.array_equal(x, y), f"wm {w}: {int((x != y).any(axis=1).sum())} records differ"
    assert sum(x.shape[0] for _, x in b) > 0
    return sg, so


def _epochs_np(results, fields):
    """Per watermark: the fired records as rows (key, ts, f1, fields...) sorted lexicographically
    (numpy: the C2 epochs hold millions of records)."""
    ep = []
    for res in results:
        cols = np.stack([res["key"], res["ts"], res["f1"]] + [res[f] for f in fields], axis=1) if res["n"] else \
            np.zeros((0, 3 + len(fields)), np.int64)
        pos = 0
        for wm, mp in list(zip(res["mark_wm"], res["mark_pos"])) + [(None, res["n"])]:
            part = cols[pos:mp]
            pos = mp
            if wm is None and part.shape[0] == 0:
                continue
            order = np.lexsort(part.T[::-1]) if part.shape[0] else np.zeros(0, np.int64)
            ep.append((None if wm is None else int(wm), part[order]))
    return ep


def test_c1_bench_geometry():
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    batch = 1 << 22
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                      max_parallelism=128, key_capacity=1 << 16, max_batch=batch, out_capacity=1 << 20)
    sg, so = _run(cfg, 5, batch, 1 << 16, 1 << 24, 1)
    assert sg["ingest_form"] == 3   # the fused form the bench runs
    assert sg["panes_fired"] == so["panes_fired"] > 0


def test_c1_bench_geometry_partitioned():
    """The same C1 stream through the two-kernel partitioned form (ingest_mode 2)."""
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    batch = 1 << 22
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                      max_parallelism=128, key_capacity=1 << 16, max_batch=batch, out_capacity=1 << 20, ingest_mode=2)
    sg, so = _run(cfg, 5, batch, 1 << 16, 1 << 24, 1)
    assert sg["ingest_form"] == 2
    assert sg["panes_fired"] == so["panes_fired"] > 0


def test_c4_zipf_lateness_bench_geometry():
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    batch = 1 << 22
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count"), "i64", keep_first_f1=True),
                      allowed_lateness=100, max_parallelism=128, key_capacity=1 << 16, max_batch=batch,
                      out_capacity=1 << 22)
    sg, so = _run(cfg, 12, batch, 1 << 16, 1 << 25, 50, zipf=1.2, ooo=300, fields=("sum_i64", "count"))
    assert sg["ingest_form"] == 2
    assert so["late_fires"] > 0 and sg["late_fires"] == so["late_fires"]
    assert sg["records_late"] == so["records_late"] > 0


def test_c2_ten_million_keys():
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    batch = 1 << 22
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                      max_parallelism=128, key_capacity=10_000_000, max_batch=batch, out_capacity=1 << 24,
                      max_open_slices=3)
    # R = 2^22 events per second: one window per batch (~3.4 M panes each); with 3 slice slots the
    # fourth window reuses the first one's slot after its purge
    sg, so = _run(cfg, 4, batch, 10_000_000, 1 << 22, 1)
    assert sg["ingest_form"] == 1   # direct: a 10 M-key directory bucket does not fit LDS
    assert sg["panes_fired"] == so["panes_fired"] > 0
