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
        ex = KeyByExchange(eng, 1, 0, 128, batch, torch.device("cuda", 0))
        rows = []
        for j in range(10):
            k, t, v = stream(j * batch, batch, n_keys, rate, device="cuda")
            ex.step(k, t, v, int(t.max().item()) - 1)
            r = eng.collect()
            rows += list(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
        eng.advance_watermark(LONG_MAX)
        r = eng.collect()
        rows += list(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
        eng.close()
    finally:
        dist.destroy_process_group()
    eo = OracleEngine(cfg)
    k, t, v = stream(0, 10 * batch, n_keys, rate)
    eo.push(k.numpy(), t.numpy(), v.numpy())
    eo.advance_watermark(LONG_MAX)
    r = eo.collect()
    ref = sorted(zip(r["key"].tolist(), r["ts"].tolist(), r["sum_i64"].tolist(), r["count"].tolist()))
    assert len(ref) > 0 and sorted(rows) == ref
