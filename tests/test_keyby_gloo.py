"""The N>1 path on CPU: two processes (gloo), each a source subtask and a window subtask.

Each rank routes its source batch by key group (maxParallelism 128) through KeyByExchange (count
all-to-all, record all-to-all), aligns the watermark with a MIN all-reduce, and feeds its own
subtask (key-group range of its operator index).  The union of both subtasks' fired results must
equal one subtask over the whole stream (order-independent fields: int64 sum/count, bit-exact).
The window subtasks here are oracle engines (no GPU); on GPUs the same class drives the HIP engine
and the HIP partition kernel over RCCL.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LONG_MAX = (1 << 63) - 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd.keyby import KeyByExchange
    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    from flink_amd.synth import stream
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    from oracle.oracle import OracleEngine

    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count")), max_parallelism=128,
                      key_group_range=compute_key_group_range_for_operator_index(128, world, rank),
                      key_capacity=4096, max_batch=1 << 14, out_capacity=1 << 18)
    eng = OracleEngine(cfg)
    ex = KeyByExchange(eng, world, rank, 128, 1 << 13, "cpu")
    batch = 4096
    rows = []
    for j in range(12):
        k, t, v = stream(j * batch * world, batch * world, 3000, 1 << 13)
        k, t, v = k[rank::world].contiguous(), t[rank::world].contiguous(), v[rank::world].contiguous()
        # local watermark lags a bit differently per source: the aligned one is their min
        wm_local = int(t.max()) - 1 - 37 * rank
        rk, rt, rv = ex.exchange(k, t, v)
        if rk.numel():
            eng.push(rk.numpy(), rt.numpy(), rv.numpy())
        wm = ex.align_watermark(wm_local)
        _, tall, _ = stream(j * batch * world, batch * world, 3000, 1 << 13)
        assert wm == min(int(tall[r::world].max()) - 1 - 37 * r for r in range(world))
        eng.advance_watermark(wm)
        r = eng.collect()
        rows += list(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
    eng.advance_watermark(LONG_MAX)
    r = eng.collect()
    rows += list(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
    q.put((rank, rows))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_keyby_exchange_two_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, rows = q.get(timeout=240)
        got[rank] = rows
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    union = sorted(got[0] + got[1])
    # every key lands on exactly one subtask
    assert not ({r[0] for r in got[0]} & {r[0] for r in got[1]})

    from flink_amd.synth import stream
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    from oracle.oracle import OracleEngine
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count")), key_capacity=4096,
                      max_batch=1 << 17, out_capacity=1 << 18)
    e = OracleEngine(cfg)
    k, t, v = stream(0, 12 * 4096 * world, 3000, 1 << 13)
    e.push(k.numpy(), t.numpy(), v.numpy())
    e.advance_watermark(LONG_MAX)
    r = e.collect()
    ref = sorted(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
    assert union == ref
