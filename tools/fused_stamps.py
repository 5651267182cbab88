"""Diagnostic: phase timing of k_fused (ingest_mode 3) from in-kernel realtime stamps (FW_DEBUG_AGG=16).

Stamps per workgroup (fw_fused.hip FU_STAMP): 0 start, 1 prologue done (directory copy, placement known),
2 producers done, 3 consumers done, 4 flushed, 5 end; 63 = xcc | one_l2 << 8.  Realtime ticks are 100 MHz.
Env: STAMP_CFG=c3 (sliding 10 s / 1 s doubles, sum/min/max/count) or c1 (default).
"""
import ctypes
import os
import sys
import time

os.environ["FW_DEBUG_AGG"] = "16"
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream  # noqa: E402
from flink_amd.windowing import (ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows,  # noqa: E402
                                 WindowEngine, make_config)

C3 = os.environ.get("STAMP_CFG") == "c3"
if C3:
    cfg = make_config(SlidingEventTimeWindows.of(10_000, 1000), ReduceFunction(("sum", "min", "max", "count"), "f64", True),
                      key_capacity=1 << 14, max_batch=1 << 22, out_capacity=1 << 22, ingest_mode=3)
else:
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True),
                      key_capacity=1 << 16, max_batch=1 << 22, out_capacity=1 << 22, ingest_mode=3)
e = WindowEngine(cfg)
B = 1 << 22
buf = np.zeros(16 << 16, dtype=np.int64)
names = ("prologue", "producers", "consumers", "flushed", "end")
for j in range(6):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda", value_type="f64" if C3 else "i64")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.push(k, t, v)
    e.sync()
    wall = (time.perf_counter() - t0) * 1e6
    e.lib.fw_debug_stamps(e.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), buf.size)
    a = buf[: 256 * 64].reshape(256, 64)
    info = a[:, 63]
    st = a[:, :6].astype(np.float64)
    t0s = st[:, 0].min()
    rel = (st - t0s) * 10.0   # ns from the first workgroup's start
    xcc = info & 255
    one = (info >> 8) & 1
    print(f"batch {j}: wall {wall:.0f} us; one_l2 groups {int(one[:8].sum())}/8; xcc==blockIdx%8: "
          f"{int((xcc == (np.arange(256) % 8)).sum())}/256; start skew max {rel[:, 0].max():.0f} ns")
    print("  " + "  ".join(f"{nm} p50 {np.median(rel[:, q + 1]):7.0f} max {rel[:, q + 1].max():7.0f}"
                           for q, nm in enumerate(names)))
    full = (a[:, :56].astype(np.float64) - t0s) * 10.0
    for r in range(8):
        p = [full[:, 8 + 3 * r + q] for q in range(3)]
        c = [full[:, 32 + 3 * r + q] for q in range(3)]
        if (a[:, 8 + 3 * r] == 0).all():
            break
        print(f"  unit {r}: P start {np.median(p[0]):7.0f} slot {np.median(p[1]):7.0f} stored {np.median(p[2]):7.0f}"
              f" | C published {np.median(c[0]):7.0f} loaded {np.median(c[1]):7.0f} reduced {np.median(c[2]):7.0f}")
