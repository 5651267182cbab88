"""Guard for the round-3 fault: the direct form's first-arrival fix-up (k_fix_first_f1, profile
phase FW_PHASE_FIXUP) reads the per-record list `new_list` that only the direct tumbling / sliding ingest writes.
Session and list-state engines ingest through their own kernels and never write it, so a push of theirs must never
launch the fix-up (it would read stale device memory: "an illegal memory access was encountered" in
test_list_operator_window_function, gpurun_out/list.log of round 3).  The direct form is the positive control.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fixups(cfg, keys, ts, vals, batch=1 << 12):
    from flink_amd import _abi
    from flink_amd.windowing import WindowEngine
    e = WindowEngine(cfg)
    e.lib.fw_set_profiling(e.h, 1)
    for s in range(0, len(keys), batch):
        sl = slice(s, s + batch)
        e.push(keys[sl], ts[sl], vals[sl], f1=np.arange(s, min(s + batch, len(keys)), dtype=np.int64))
        e.advance_watermark(int(ts[sl].max()) - 5)
    e.sync()
    prof = _abi.FwProfile()
    e.lib.fw_get_profile(e.h, prof)
    e.advance_watermark((1 << 63) - 1)
    e.collect()
    e.close()
    return prof.launches[_abi.FW_PHASE_FIXUP]


def _stream(n=1 << 14, keys=512, seed=7):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, keys, n).astype(np.int64)
    t = (1_700_000_000_000 + np.arange(n) // 4 - rng.integers(0, 20, n)).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    return k, t, v


def test_session_and_list_never_launch_direct_fixup():
    from flink_amd.windowing import (EventTimeSessionWindows, ListStateDescriptor, ReduceFunction,
                                     TumblingEventTimeWindows, make_config)
    k, t, v = _stream()
    common = dict(max_parallelism=128, key_capacity=1 << 11, max_batch=1 << 12, out_capacity=1 << 20)
    sess = make_config(EventTimeSessionWindows.withGap(30), ReduceFunction(("sum",), "i64", keep_first_f1=True), **common)
    assert _fixups(sess, k, t, v) == 0
    sess_list = make_config(EventTimeSessionWindows.withGap(30), ListStateDescriptor("i64", list_capacity=1 << 16), **common)
    assert _fixups(sess_list, k, t, v) == 0
    lst = make_config(TumblingEventTimeWindows.of(1000), ListStateDescriptor("i64"), **common)
    assert _fixups(lst, k, t, v) == 0
    # positive control: the direct form with a first-arrival f1 launches it once per push
    direct = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                         ingest_mode=1, **common)
    assert _fixups(direct, k, t, v) == (len(k) + (1 << 12) - 1) >> 12
