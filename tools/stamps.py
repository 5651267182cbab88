"""Diagnostic: per-phase timing of k_route / k_aggregate from in-kernel realtime stamps (FW_DEBUG_AGG=16)."""
import ctypes, os, sys
os.environ["FW_DEBUG_AGG"] = str(16 | int(os.environ.get("FW_DEBUG_AGG_EXTRA", "0")))
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd.synth import stream
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config
C4 = os.environ.get("STAMP_CFG") == "c4"   # Zipf(1.2) keys, 300 ms out of order, lag 50, lateness 100 (bench c4)
cfg = make_config(TumblingEventTimeWindows.of(1000), ReduceFunction(("sum", "count") if C4 else ("sum",), "i64", True),
                  None, 100 if C4 else 0, key_capacity=1 << 16, max_batch=1 << 22, out_capacity=1 << 22, ingest_mode=2)
e = WindowEngine(cfg)
B = 1 << 22
buf = np.zeros(16 << 16, dtype=np.int64)
def phases(a, nblk, npts):
    a = a[: nblk * 8].reshape(nblk, 8)[:, :npts].astype(np.float64)
    t0 = a[:, 0].min()
    d = np.diff(a, axis=1) * 10.0  # ns
    if os.environ.get("STAMP_MAX"):
        end = (a[:, npts - 1] - t0) * 10
        print("      max per phase", np.round(d.max(axis=0)), "end p50/p90/max", np.percentile(end, [50, 90, 100]).round())
        if nblk == 256:
            m = d[:, 2]
            st = (a[:, 0] - t0) * 10
            slow = np.argsort(end)[-6:][::-1]
            print("      slowest blocks (blockIdx, start ns, main ns, end ns):",
                  [(int(b), round(st[b]), round(m[b]), round(end[b])) for b in slow])
            print("      main by blockIdx%8:", [round(m[i::8].mean()) for i in range(8)])
            print("      main by blockIdx//32:", [round(m[i*32:(i+1)*32].mean()) for i in range(8)])
    return (a[:, 0] - t0).mean() * 10, d.mean(axis=0), (a[:, npts - 1].max() - t0) * 10
for j in range(6):
    k, t, v = stream(j * B, B, 1 << 16, 1 << 25 if C4 else 1 << 24, 1_700_000_000_000, device="cuda",
                     zipf=1.2 if C4 else None, ooo=300 if C4 else 0)
    torch.cuda.synchronize()
    e.push(k, t, v)
    if os.environ.get("STAMP_WM"):   # the bench's watermark after each batch: max timestamp - lag (50 ms for c4)
        e.advance_watermark(int(t.max().item()) - (50 if C4 else 1))
    e.sync()
    e.lib.fw_debug_stamps(e.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), buf.size)
    sk, d, span = phases(buf, B // 4096, 5)
    print(f"batch {j} route: start-skew {sk:.0f} ns, load {d[0]:.0f} phaseB {d[1]:.0f} scan {d[2]:.0f} write {d[3]:.0f} | span {span:.0f} ns")
    rs = buf[: (B // 4096) * 8].reshape(-1, 8).astype(np.float64)
    if rs[:, 5].any():   # inside phase B (ns from stamp 1): per-record pass, slow path, bins + ranks
        print("      phaseB split: records %.0f slow %.0f bins %.0f rest %.0f" % tuple(
            (np.diff(rs[:, [1, 5, 6, 7, 2]], axis=1) * 10.0).mean(axis=0)))
    nagg = 256
    if os.environ.get("STAMP_HELPERS"):   # owners + helper shares (blocks past 256 that ran)
        a = buf[8 << 16:].reshape(-1, 8)
        nagg = int(np.nonzero(a[:, 0])[0].max()) + 1 if a[:, 0].any() else 256
        ends = (a[:nagg, 4] - a[:nagg, 0][a[:nagg, 0] > 0].min()) * 10
        top = np.argsort(ends)[-8:][::-1]
        print(f"      agg blocks {nagg}; slowest (blockIdx, end ns, main ns):",
              [(int(b), int(ends[b]), int((a[b, 3] - a[b, 2]) * 10)) for b in top])
        t0 = a[:nagg, 0][a[:nagg, 0] > 0].min()
        for b in top[:4]:   # every stamp of the block, ns from the kernel's first stamp (0 = not reached)
            print(f"        block {int(b)}:", [int((x - t0) * 10) if x else 0 for x in a[b]])
    ag = buf[8 << 16:][: nagg * 8].reshape(-1, 8).astype(np.float64)
    if ag[:, 5].any() and ag[:, 7].any():   # inside the segment-table phase (ns from stamp 1)
        print("      segtab split: decide %.0f gsl+barrier %.0f g0 %.0f rest %.0f" % tuple(
            (np.diff(ag[:, [1, 5, 6, 7, 2]], axis=1) * 10.0).mean(axis=0)))
    sk, d, span = phases(buf[8 << 16:], nagg, 5)
    print(f"        aggregate: start-skew {sk:.0f} ns, ldir {d[0]:.0f} segtab {d[1]:.0f} main {d[2]:.0f} fold {d[3]:.0f} | span {span:.0f} ns")
    e.advance_watermark(int(t.max().item()) - (50 if C4 else 1))
    e.collect()
