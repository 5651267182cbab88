"""Diagnostic: where the pipelined keyBy exchange's host time goes at N=1 (--force-exchange shape), per step.
Wraps KeyByExchange's phases with wall-clock timers; prints mean microseconds per step per phase."""
import collections, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from flink_amd import keyby
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config

acc = collections.defaultdict(float)
def wrap(cls, name):
    f = getattr(cls, name)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t
    setattr(cls, name, g)
for n in ("_finish", "_route_into", "_wait_read", "_push_share", "_transfer", "_forward"):
    wrap(keyby.KeyByExchange, n)
sync0 = torch.cuda.Event.synchronize
def sync(self):
    t = time.perf_counter(); sync0(self); acc["event.synchronize"] += time.perf_counter() - t
torch.cuda.Event.synchronize = sync

B = 1 << 22
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True), None, 0,
                  key_capacity=1 << 16, max_batch=B, out_capacity=1 << 22, ingest_mode=2)
e = WindowEngine(cfg)
dev = torch.device("cuda", 0)
cols = [stream(j * B, B, 1 << 16, 1 << 24, 0, device=dev) for j in range(24)]
ex = keyby.KeyByExchange(e, 1, 0, 128, B, dev)
def wm(j): return ((j + 1) * B * 1000) // (1 << 24) - 1
for j in range(4):
    ex.step(*cols[j][:3], wm(j))
ex.flush(); e.sync(); torch.cuda.synchronize()
acc.clear()
t0 = time.perf_counter()
for j in range(4, 24):
    ex.step(*cols[j][:3], wm(j))
t_loop = time.perf_counter() - t0
ex.flush(); torch.cuda.synchronize(); e.sync()
dt = time.perf_counter() - t0
print("per step us: loop %.1f  total %.1f" % (t_loop / 20 * 1e6, dt / 20 * 1e6))
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print("  %-20s %.1f" % (k, v / 20 * 1e6))
e.close()
