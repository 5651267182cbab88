"""The keyBy exchange on the GPU path, as a one-rank RCCL world (the box has one GPU): the HIP partition
kernel (KeyGroupStreamPartitioner routing), the count all-to-all, the per-column record all-to-alls and
the watermark MIN all-reduce feed a HIP engine; its results must equal the oracle's over the same stream.
The multi-rank routing itself is covered on CPU (test_keyby_gloo.py)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LONG_MAX = (1 << 63) - 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_keyby_exchange_one_rank_rccl():
    import torch
    import torch.distributed as dist
    from flink_amd.keyby import KeyByExchange
    from flink_amd.synth import stream
    from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
    from oracle.oracle import OracleEngine

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        batch, n_keys, rate = 1 << 15, 3000, 1 << 14
        cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count")), max_parallelism=128,
                          key_group_range=(0, 127), key_capacity=4096, max_batch=2 * batch, out_capacity=1 << 18)
        eng = WindowEngine(cfg)
        ex = KeyByExchange(eng, 1, 0, 128, batch, torch.device("cuda", 0), depth=2)
        wms = []
        for j in range(10):
            k, t, v = stream(j * batch, batch, n_keys, rate, device="cuda")
            wm = int(t.max().item()) - 1 - (5000 if j % 4 == 3 else 0)   # regressions: swallowed by the valve
            wms.append(wm)
            ex.step(k, t, v, wm)
        ex.flush()
        results = [eng.collect()]
        eng.advance_watermark(LONG_MAX)
        results.append(eng.collect())
        eng.close()
    finally:
        dist.destroy_process_group()
    from harness import epochs_of
    from flink_amd.keyby import ChannelWatermarks
    valve = ChannelWatermarks(1)
    expected = [valve.on_watermark(0, w) for w in wms]
    assert any(e is None for e in expected)
    assert ex.emitted == [e for e in expected if e is not None]
    eo = OracleEngine(cfg)
    res = []
    for j in range(10):
        k, t, v = stream(j * batch, batch, n_keys, rate)
        eo.push(k.numpy(), t.numpy(), v.numpy())
        if expected[j] is not None:
            eo.advance_watermark(expected[j])
        res.append(eo.collect())
    eo.advance_watermark(LONG_MAX)
    res.append(eo.collect())
    ref = epochs_of(res, ["sum_i64", "count"])
    got = epochs_of(results, ["sum_i64", "count"])
    assert sum(len(r) for _, r in ref) > 0 and got == ref
