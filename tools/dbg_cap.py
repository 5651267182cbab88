import sys, torch
sys.path.insert(0, "/root/repo")
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
def run(keys, batch, first, nb=2, mode=2):
    cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=first),
                      key_capacity=keys, max_batch=batch, out_capacity=1 << 20, ingest_mode=mode)
    e = WindowEngine(cfg)
    try:
        for j in range(nb):
            k, t, v = stream(j * batch, batch, keys, 1 << 24, 1_700_000_000_000, device="cuda")
            e.push(k, t, v); e.advance_watermark(int(t.max().item()) - 1)
            e.sync()
        r = "ok"
    except Exception as ex:
        r = str(ex)[:80]
    e.close()
    print(keys, batch, first, mode, r, flush=True)
for keys, batch in [(4096, 1 << 16), (4096, 1 << 20), (4096, 1 << 22), (1 << 16, 1 << 16), (1 << 16, 1 << 20), (1 << 16, 1 << 22)]:
    run(keys, batch, True)
run(1 << 16, 1 << 22, False)
import ctypes, numpy as np
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", keep_first_f1=True),
                  key_capacity=1 << 16, max_batch=1 << 20, out_capacity=1 << 20, ingest_mode=2)
e = WindowEngine(cfg)
k, t, v = stream(0, 1 << 20, 1 << 16, 1 << 24, 1_700_000_000_000, device="cuda")
e.push(k, t, v)
torch.cuda.synchronize()
c = np.zeros(8, np.int64)
e.lib.fw_debug_counters(e.h, c.ctypes.data_as(ctypes.c_void_p))
print("counters", c.tolist(), flush=True)
