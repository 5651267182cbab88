"""Diagnostics: the same 4M-record batches through a plain engine and through the keyBy exchange (one-rank
RCCL world); per watermark, the fired panes must agree.  ONLY_PLAIN=1 runs the plain engine alone."""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flink_amd.synth import stream  # noqa: E402
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config  # noqa: E402

B = 1 << 22
only = os.environ.get("ONLY_PLAIN") == "1"


def mk():
    return make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), max_parallelism=128,
                       key_group_range=(0, 127), key_capacity=1 << 16, max_batch=int(os.environ.get("MB_MUL", "1")) * B,
                       out_capacity=1 << 22)


ea = WindowEngine(mk())
if not only:
    import torch.distributed as dist
    from flink_amd.keyby import KeyByExchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29544"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    eb = WindowEngine(mk())
    ex = KeyByExchange(eb, 1, 0, 128, B, torch.device("cuda", 0))


def rows(e):
    try:
        r = e.collect()
    except Exception as err:   # noqa: BLE001
        return f"ERR {err} stats={e.stats()}"
    return sorted(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist()))


for j in range(8):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda")
    wm = int(t.max().item()) - 1
    ea.push(k, t, v)
    ea.advance_watermark(wm)
    ra = rows(ea)
    if only:
        print(j, ra if isinstance(ra, str) else len(ra), flush=True)
        continue
    ex.step(k, t, v, wm)
    rb = rows(eb)
    print(j, ra if isinstance(ra, str) else len(ra), rb if isinstance(rb, str) else len(rb), ra == rb, flush=True)
if not only:
    dist.destroy_process_group()
