"""Diagnostics: how often k_aggregate's branch-free 4-slot probe misses (FW_DEBUG_AGG & 8 counts slow-path waves)."""
import ctypes, os, sys
os.environ["FW_DEBUG_AGG"] = "8"
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), key_capacity=1 << 16,
                  max_batch=1 << 22, out_capacity=1 << 21, ingest_mode=2)
e = WindowEngine(cfg)
B = 1 << 22
buf = np.zeros(8, dtype=np.int64)
for j in range(4):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda")
    torch.cuda.synchronize()
    e.push(k, t, v)
    e.sync()
    e.lib.fw_debug_counters(e.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    print(f"batch {j}: slow-path waves so far {buf[5]} (of ~{B // 64 * (j + 1)} wave-records)")
    e.advance_watermark(int(t[-1].item()) - 1)
    e.collect()
