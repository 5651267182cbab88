"""Diagnostic: host-side cost of the drain paths on the C1 workload (per step: push + watermark, then nothing /
fw_collect / fw_collect_begin + fw_collect_end of the previous step)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream  # noqa: E402
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config  # noqa: E402

B, R, T0 = 1 << 22, 1 << 24, 1_700_000_000_000
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                  key_capacity=1 << 16, max_batch=B, out_capacity=1 << 24)
e = WindowEngine(cfg)
cols = [stream(j * B, B, 1 << 16, R, T0, device="cuda") for j in range(48)]
torch.cuda.synchronize()
wm = lambda j: T0 + (((j + 1) * B - 1) * 1000) // R - 1
for _ in range(2):
    e.collect_end(e.collect_begin())
j = 0
for mode in ("none", "sync", "async", "none"):
    e.sync()
    torch.cuda.synchronize()
    t = time.perf_counter()
    tin = {"push": 0.0, "wm": 0.0, "begin": 0.0, "end": 0.0, "collect": 0.0}
    prev = None
    for q in range(12):
        k, ts, v = cols[j % 48]
        a = time.perf_counter(); e.push(k, ts, v); b = time.perf_counter(); tin["push"] += b - a
        e.advance_watermark(wm(j)); c = time.perf_counter(); tin["wm"] += c - b
        j += 1
        if mode == "sync":
            e.collect(); tin["collect"] += time.perf_counter() - c
        elif mode == "async":
            cur = e.collect_begin(); d = time.perf_counter(); tin["begin"] += d - c
            if prev is not None:
                e.collect_end(prev); tin["end"] += time.perf_counter() - d
            prev = cur
    if prev is not None:
        e.collect_end(prev)
    e.sync()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 12
    print(f"{mode:6s} {dt * 1e3:.3f} ms/step  " + "  ".join(f"{k} {v / 12 * 1e3:.3f}" for k, v in tin.items() if v), flush=True)
    e.collect()
