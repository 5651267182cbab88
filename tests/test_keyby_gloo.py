"""The N>1 path on CPU: two processes (gloo), each a source subtask and a window subtask.

Each rank routes its source batch by key group (maxParallelism 128) through KeyByExchange (count
all-to-all, record all-to-all), aligns the watermark with a MIN all-reduce, and feeds its own
subtask (key-group range of its operator index).  The union of both subtasks' fired results must
equal one subtask over the whole stream (order-independent fields: int64 sum/count, bit-exact).
The window subtasks here are oracle engines (no GPU); on GPUs the same class drives the HIP engine
and the HIP partition kernel over RCCL.  `pipelined` runs the GPUs' own step()/_finish() code (the
depth-2 software pipeline, count all-to-all and MIN all-reduce in one meta tensor, the receive ring) on
CPU tensors; the Zipf(1.2) case makes one rank receive several times its engine's max_batch, which the
exchange pushes in pieces (the hot keys' key groups meet on one operator at p = 8).  Without
skew every rank makes exactly one engine push per step (own and received shares in one run of records).
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


def _local_wm(j, r, t_part):
    """Source r's watermark after its batch j: max ts - 1 - 37 r, with regressions (rank 1 every 5th
    step) and repeats (rank 0 every 4th step) that the channel valve must swallow."""
    wm = int(t_part.max()) - 1 - 37 * r
    if r == 1 and j % 5 == 3:
        wm -= 4000
    if r == 0 and j % 4 == 1 and j > 0:
        wm = -(1 << 63) + 5
    return wm


def _stream(j, world, zipf):
    from flink_amd.synth import stream
    return stream(j * BATCH * world, BATCH * world, 3000, 1 << 13, zipf=zipf)


def expected_forwarded(world, steps, batch, zipf=None):
    """StreamInputProcessor.java:147-161 over the world's source channels, one forward per step at most."""
    from flink_amd.keyby import ChannelWatermarks
    from flink_amd.synth import stream
    valve = ChannelWatermarks(world)
    out = []
    for j in range(steps):
        _, t, _ = stream(j * batch * world, batch * world, 3000, 1 << 13, zipf=zipf)
        fwd = None
        for r in range(world):
            x = valve.on_watermark(r, _local_wm(j, r, t[r::world]))
            fwd = x if x is not None else fwd
        out.append(fwd)
    return out


STEPS, BATCH = 12, 4096


def _worker(rank, world, port, q, pipelined=False, zipf=None):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from harness import epochs_of
    from flink_amd.keyby import KeyByExchange
    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    from flink_amd.synth import stream
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    from oracle.oracle import OracleEngine

    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count")), max_parallelism=128,
                      key_group_range=compute_key_group_range_for_operator_index(128, world, rank),
                      key_capacity=4096, max_batch=BATCH if zipf else 1 << 14, out_capacity=1 << 18)
    eng = OracleEngine(cfg)
    ex = KeyByExchange(eng, world, rank, 128, 1 << 13, "cpu", pipelined=pipelined)
    results = []
    for j in range(STEPS):
        k, t, v = _stream(j, world, zipf)
        k, t, v = k[rank::world].contiguous(), t[rank::world].contiguous(), v[rank::world].contiguous()
        ex.step(k, t, v, _local_wm(j, rank, t))
        results.append(eng.collect())
    ex.flush()
    results.append(eng.collect())
    eng.advance_watermark(LONG_MAX)
    results.append(eng.collect())
    pushes = ex.pushes
    q.put((rank, epochs_of(results, ["sum_i64", "count"]), ex.emitted, pushes))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,pipelined,zipf", [
    (2, False, None), (3, False, None), (8, False, None),   # 8: the ranks of one MI355X node
    (2, True, None), (8, True, None),                      # the GPU path's pipelined step() / _finish()
    (8, True, 1.2)])                                       # skew: shares above max_batch pushed in pieces
def test_keyby_exchange_two_ranks(world, pipelined, zipf):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, pipelined, zipf)) for r in range(world)]
    for p in procs:
        p.start()
    got, emitted, pushes = {}, {}, {}
    for _ in range(world):
        rank, ep, em, pu = q.get(timeout=240)
        got[rank], emitted[rank], pushes[rank] = ep, em, pu
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = expected_forwarded(world, STEPS, BATCH, zipf)
    if world == 2:
        assert any(e is None for e in exp), "the stream must exercise non-increasing aligned watermarks"
    if zipf:   # some rank received more than max_batch = BATCH per step: its run goes in pieces
        assert max(pushes.values()) > STEPS
    else:      # own share and received shares between two watermarks: ONE engine push per step
        assert all(pushes[r] == STEPS for r in range(world)), pushes
    forwarded = [e for e in exp if e is not None]
    # every window subtask forwards exactly the valve's watermarks (positions included)
    for r in range(world):
        assert emitted[r] == forwarded
        assert [w for w, _ in got[r]] == forwarded + [LONG_MAX]
    # every key lands on exactly one subtask
    keys = [{rec[0] for _, recs in got[r] for rec in recs} for r in range(world)]
    assert all(not (keys[a] & keys[b]) for a in range(world) for b in range(a + 1, world))

    # one subtask over the whole stream, fed the same forwarded watermarks after the same batches
    from harness import epochs_of
    from flink_amd.synth import stream
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, make_config
    from oracle.oracle import OracleEngine
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count")), key_capacity=4096,
                      max_batch=1 << 17, out_capacity=1 << 18)
    e = OracleEngine(cfg)
    res = []
    for j in range(STEPS):
        k, t, v = _stream(j, world, zipf)
        e.push(k.numpy(), t.numpy(), v.numpy())
        if exp[j] is not None:
            e.advance_watermark(exp[j])
        res.append(e.collect())
    e.advance_watermark(LONG_MAX)
    res.append(e.collect())
    ref = epochs_of(res, ["sum_i64", "count"])
    union = [(w, sorted(rec for r in range(world) for rec in got[r][i][1])) for i, (w, _) in enumerate(got[0])]
    assert union == ref
    assert sum(len(r) for _, r in ref) > 0
