"""Diagnostic: fw_decode kernels on one C1-sized batch of wire bytes (run under rocprofv3 --kernel-trace --stats)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
dev = torch.device("cuda", 0)
n = 1 << 22
k, t, v = stream(0, n, 1 << 16, 1 << 24, 1_700_000_000_000, device=dev)
be = lambda x: x.view(torch.uint8).view(n, 8).flip(1)
head = torch.tensor([0, 0, 0, 33, 0], dtype=torch.uint8, device=dev).expand(n, 5)
wire = torch.cat([head, be(t), be(k), be(t), be(v)], dim=1).reshape(-1).contiguous()
e = WindowEngine(make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum",), "i64", True),
                             key_capacity=1 << 16, max_batch=n, out_capacity=1 << 20))
for i in range(6):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    out = e.decode(wire, ["long", "long", "long"], key=0, f1=1, value=2, record_cap=n, device=True)
    torch.cuda.synchronize(); print(f"decode {1e3 * (time.perf_counter() - t0):.3f} ms", out["n_records"])
e.close()
