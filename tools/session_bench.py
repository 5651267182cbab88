"""Session-window throughput (no session figure existed): keyed event-time session windows
(EventTimeSessionWindows.withGap, the merging branch of WindowOperator.java:228-301) over a resident synthetic
stream, one JSON line.  Not the headline metric (BASELINE.json names tumbling / sliding configs); a measurement
of fw_session.hip's per-key walk.

Workload (env overrides): SB_KEYS keys (default 65536), SB_RATE events per event-time second (default 2^22, so
~64 events per key per second, ~16 ms apart), SB_GAP session gap in ms (default 10: mostly 1-3 record sessions
that fire as the watermark passes), SB_BATCH events per push (default 2^20), SB_ZIPF (unset: uniform keys).
Check: after the final MAX watermark the wrapping sum of the fired sums equals that of the values pushed.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream  # noqa: E402
from flink_amd.windowing import EventTimeSessionWindows, ReduceFunction, WindowEngine, make_config  # noqa: E402

LONG_MAX = (1 << 63) - 1
T0 = 1_700_000_000_000


def main():
    keys = int(os.environ.get("SB_KEYS", 1 << 16))
    rate = int(os.environ.get("SB_RATE", 1 << 22))
    gap = int(os.environ.get("SB_GAP", 10))
    batch = int(os.environ.get("SB_BATCH", 1 << 20))
    zipf = float(os.environ["SB_ZIPF"]) if os.environ.get("SB_ZIPF") else None
    steps, warmup = int(os.environ.get("SB_STEPS", 16)), int(os.environ.get("SB_WARMUP", 4))
    slots = int(os.environ.get("SB_SLOTS", 32))
    dev = "cuda"
    cfg = make_config(EventTimeSessionWindows.withGap(gap), ReduceFunction(("sum",), "i64", True),
                      max_parallelism=128, key_capacity=keys, max_batch=batch, max_open_slices=slots,
                      out_capacity=batch * (steps + warmup + 2))
    eng = WindowEngine(cfg)
    cols = [stream(j * batch, batch, keys, rate, T0, device=dev, zipf=zipf) for j in range(warmup + steps)]
    torch.cuda.synchronize()

    def wm_of(j):
        return int(T0 + (((j + 1) * batch - 1) * 1000) // rate) - 1

    for j in range(warmup):
        eng.push(*cols[j])
        eng.advance_watermark(wm_of(j))
    eng.sync()
    torch.cuda.synchronize()
    got = [eng.collect()]
    t0 = time.perf_counter()
    for j in range(warmup, warmup + steps):
        eng.push(*cols[j])
        eng.advance_watermark(wm_of(j))
    eng.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    got.append(eng.collect())
    eng.advance_watermark(LONG_MAX)
    got.append(eng.collect())
    mask = (1 << 64) - 1
    fired = sum(int(r["sum_i64"].astype("uint64").sum(dtype="uint64")) for r in got if r["n"]) & mask
    pushed = 0
    for k, t, v in cols:
        pushed = (pushed + (int(v.sum().item()) & mask)) & mask
    line = {"metric": "events/s keyed event-time session windows (sum, f1 = first arrival)",
            "value": steps * batch / dt, "unit": "events/s", "ms_per_step": dt * 1e3 / steps, "steps": steps,
            "config": {"keys": keys, "rate_per_s": rate, "gap_ms": gap, "batch": batch, "zipf": zipf,
                       "slots_per_key": slots},
            "sessions_fired": int(st["panes_fired"]), "check": "ok" if fired == pushed else "MISMATCH",
            "data": "synthetic (splitmix64 counter stream), resident in HBM"}
    print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
