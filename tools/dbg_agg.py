"""Diagnostic: C1 batches through the partitioned ingest with FW_DEBUG_AGG=3 counters."""
import ctypes, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), key_capacity=1 << 16,
                  max_batch=1 << 22, out_capacity=1 << 21, ingest_mode=2)
e = WindowEngine(cfg)
B = 1 << 22
for j in range(8):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda")
    e.push(k, t, v)
    e.advance_watermark(int(t[-1].item()) - 1)
    e.sync()
    c = (ctypes.c_int64 * 8)()
    e.lib.fw_debug_counters(e.h, c)
    print(j, "probes", c[5], "cas", c[6], "records", c[7], "avg probe", c[5] / max(c[7], 1))
