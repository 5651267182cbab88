"""Diagnostic: per-round timing of k_fused (ingest_mode 3) from in-kernel realtime stamps (FW_DEBUG_AGG=16).

Stamps per workgroup (fw_fused.hip FU_STAMP): 0 start, 1 placement known, 2 + 4k + {0 produced, 1 published,
2 round k arrived, 3 consumed}, 60 partials published, 61 fold range ready, 62 end; 63 = xcc | one_l2 << 8.
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
                      key_capacity=1 << 16, max_batch=1 << 22, out_capacity=1 << 22, ingest_mode=3)
else:
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True),
                      key_capacity=1 << 16, max_batch=1 << 22, out_capacity=1 << 22, ingest_mode=3)
e = WindowEngine(cfg)
B = 1 << 22
R = B // (256 * 2048)
buf = np.zeros(16 << 16, dtype=np.int64)
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
    st = a[:, :63].astype(np.float64)
    t0s = st[:, 0].min()
    rel = (st - t0s) * 10.0   # ns from the first workgroup's start
    xcc = info & 255
    one = (info >> 8) & 1
    print(f"batch {j}: wall {wall:.0f} us; one_l2 groups {int(one[:8].sum())}/8; xcc==blockIdx%8: "
          f"{int((xcc == (np.arange(256) % 8)).sum())}/256")
    print(f"  start skew max {rel[:, 0].max():.0f} ns, placement known p50 {np.median(rel[:, 1]):.0f} max {rel[:, 1].max():.0f}")
    for r in range(R + 1):
        cols = []
        for q, name in enumerate(("prod", "pub", "arr", "cons")):
            i = 2 + 4 * r + q
            if (r == R and q < 2) or (r == 0 and False):
                continue
            x = rel[:, i]
            if (a[:, i] == 0).all():
                continue
            cols.append(f"{name} {np.median(x):7.0f}/{x.max():7.0f}")
        print(f"  round {r}: " + "  ".join(cols))
    for i, name in ((60, "published"), (61, "fold ready"), (62, "end")):
        x = rel[:, i]
        print(f"  {name}: p50 {np.median(x):.0f} max {x.max():.0f} ns")
    e.advance_watermark(int(t.max().item()) - 1)
    e.collect()
e.close()
