"""Diagnostic: per-phase timing of k_watermark (FW_DEBUG_AGG=16 stamps) at C3's geometry (sliding 10 s / 1 s,
double sum/min/max/count, 64 Ki keys, 4 Mi-event batches, watermark after each batch).  Phases per workgroup:
plan (slice tags, firing windows, purge list), scan (every firing window's panes, emit), purge."""
import ctypes, os, sys
os.environ["FW_DEBUG_AGG"] = "16"
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows, WindowEngine, make_config
C1 = os.environ.get("WM_CFG") == "c1"
asg = TumblingEventTimeWindows.of(1000) if C1 else SlidingEventTimeWindows.of(10_000, 1000)
red = ReduceFunction(("sum",), "i64", True) if C1 else ReduceFunction(("sum", "min", "max", "count"), "f64", True)
cfg = make_config(asg, red, None, 0, key_capacity=1 << 16, max_batch=1 << 22, out_capacity=1 << 24, ingest_mode=2)
e = WindowEngine(cfg)
B = 1 << 22
buf = np.zeros(16 << 16, dtype=np.int64)
n_fire = 0
for j in range(48):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda", value_type="i64" if C1 else "f64")
    e.push(k, t, v)
    before = e.stats()["panes_fired"]
    buf[12 << 16:] = 0
    e.advance_watermark(int(t.max().item()) - 1)
    e.sync()
    fired = e.stats()["panes_fired"] - before
    e.collect()
    if fired == 0:
        continue
    e.lib.fw_debug_stamps(e.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), buf.size)
    a = buf[12 << 16:].reshape(-1, 8)
    nb = int(np.count_nonzero(a[:, 0]))
    if nb == 0:
        continue
    a = a[:nb, :4].astype(np.float64)
    t0 = a[:, 0].min()
    d = np.diff(a, axis=1) * 10.0
    n_fire += 1
    print(f"fire {n_fire} (batch {j}, {fired} panes, {nb} workgroups): start-skew {(a[:, 0] - t0).mean() * 10:.0f} ns, "
          f"plan {d[:, 0].mean():.0f} scan {d[:, 1].mean():.0f} purge {d[:, 2].mean():.0f} | span {(a[:, 3].max() - t0) * 10:.0f} ns"
          f" | scan max {d[:, 1].max():.0f}", flush=True)
    buf[:] = 0
e.close()
