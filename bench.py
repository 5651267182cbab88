#!/usr/bin/env python3
"""Benchmark: keyed 1 s tumbling event-time long-sum (BASELINE.json metric), events/s whole node.

Workload.  Default config C1, the job BASELINE.json's metric is quoted on:
  keyBy(0).window(TumblingEventTimeWindows.of(1 s)).reduce((a, b) -> Tuple3(a.f0, a.f1, a.f2 + b.f2))
  over Tuple3<Long key, Long ts, Long value>; 64K uniform keys; R = 2^24 events per event-time
  second; a punctuated watermark (max ts seen - 1) after every batch of 2^22 events.
Other configs (--config): c2 = the same at 10M keys (R = 2^26); c3 = sliding 10 s / 1 s windows,
double values, sum/min/max/count; c4 = Zipf(1.2) keys, timestamps up to 300 ms out of order, watermark
lag 50 ms, allowed lateness 100 ms (per-element late fires and late drops; R = 2^25), sum/count.
A step = one batch of 2^22 events per GPU pushed through the engine + its watermark (fire/purge).
Inputs are generated on the GPU and resident in HBM before the timed region.

Multi-GPU (torchrun, one process per GPU): every rank is a source subtask producing its own 2^22
events per step (weak scaling); records are routed to the key-group owner (maxParallelism 128) by
the keyBy exchange (HIP partition kernel + RCCL all-to-all) and the watermark is the min over ranks.

Roofline: algorithmic bytes per step = 24 B x events + 96 B (112 B for C3) x fired
panes; the headline `achieved` divides them by the whole step time (ms_per_step), so every kernel of
the path and the gaps between them count.  Per-kernel device times (HIP events on the stream each runs
on, measured after the timed region) and the PMC HBM traffic of the committed rocprofv3 summary of this
library build are reported beside it.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from flink_amd import _abi  # noqa: E402
from flink_amd.synth import stream  # noqa: E402
from flink_amd.windowing import (ReduceFunction, SlidingEventTimeWindows, TumblingEventTimeWindows,  # noqa: E402
                                 WindowEngine, make_config)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
LONG_MAX = (1 << 63) - 1
LONG_MIN = -(1 << 63)
T0 = 1_700_000_000_000     # epoch ms, aligned to the window size

CONFIGS = {
    "c1": dict(keys=1 << 16, rate=1 << 24, batch=1 << 22, key_cap=1 << 16, window=("tumbling", 1000),
               reduce=(("sum",), "i64"), zipf=None, ooo=0, wm_lag=1, lateness=0, pane_bytes=96,
               desc="tumbling 1s event-time long-sum, f1 = first arrival"),
    "c2": dict(keys=10_000_000, rate=1 << 26, batch=1 << 22, key_cap=10_000_000, window=("tumbling", 1000),
               reduce=(("sum",), "i64"), zipf=None, ooo=0, wm_lag=1, lateness=0, pane_bytes=96,
               desc="tumbling 1s event-time long-sum at 10M keys, f1 = first arrival"),
    "c3": dict(keys=1 << 16, rate=1 << 24, batch=1 << 22, key_cap=1 << 16, window=("sliding", 10_000, 1000),
               reduce=(("sum", "min", "max", "count"), "f64"), zipf=None, ooo=0, wm_lag=1, lateness=0, pane_bytes=112,
               desc="sliding 10s/1s event-time windows, double sum/min/max/count, f1 = first arrival"),
    "c4": dict(keys=1 << 16, rate=1 << 25, batch=1 << 22, key_cap=1 << 16, window=("tumbling", 1000),
               reduce=(("sum", "count"), "i64"), zipf=1.2, ooo=300, wm_lag=50, lateness=100, pane_bytes=96,
               desc="Zipf(1.2) keys, ts up to 300 ms out of order, watermark lag 50 ms, allowed lateness 100 ms"),
    # BASELINE configs[4]: the keyBy shuffle over N GPUs, maxParallelism 128, 100 M uniform keys; each rank's
    # engine holds its key-group range's share of the keys (KeyGroupRangeAssignment.java:78-89)
    "c5": dict(keys=100_000_000, rate=1 << 27, batch=1 << 22, key_cap=None, window=("tumbling", 1000),
               reduce=(("sum",), "i64"), zipf=None, ooo=0, wm_lag=1, lateness=0, pane_bytes=96,
               desc="keyBy shuffle (maxParallelism 128) over 100M uniform keys, tumbling 1s long-sum, f1 = first arrival"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--ingest-mode", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 25, help="events in the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--force-exchange", action="store_true",
                    help="diagnostics: run the keyBy exchange (partition + RCCL all-to-all + MIN all-reduce) at N=1 too")
    ap.add_argument("--prof-steps", type=int, default=8,
                    help="steps after the timed region run with per-kernel device-time events (roofline); "
                         "timed events serialise kernels, so the timed region runs without them")
    ap.add_argument("--decode-steps", type=int, default=4,
                    help="wire-format decode leg (fw_decode of the batch as Flink network bytes; 0 = skip)")
    ap.add_argument("--drain-steps", type=int, default=32,
                    help="steps of the leg that collects fired results to the host after every step (0 = skip)")
    ap.add_argument("--h2d-steps", type=int, default=8,
                    help="steps after the timed region pushed from pinned host columns (PCIe-inclusive rate; 0 = skip)")
    return ap.parse_args()


def dist_init(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.force_exchange:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def cpu_baseline(cfg, C, n):
    """The oracle as a p-subtask CPU job (key-group partitioned threads) on a bounded sample.  Also returns what it
    fired on the sample — the count of results and the wrapping sum of their sums (counts for doubles) — which the
    GPU is checked against on the same sample (sample_check)."""
    from oracle import oracle
    cores = min(16, len(os.sched_getaffinity(0)))
    keys, ts, vals = (t.numpy() for t in stream(0, n, C["keys"], C["rate"], T0, device="cpu",
                                                 value_type=C["reduce"][1], zipf=C["zipf"], ooo=C["ooo"]))
    oracle.load()
    t = time.perf_counter()
    fired, csum = oracle.run_parallel(cfg, cores, keys, ts, vals, C["batch"], C["wm_lag"], LONG_MAX)
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "events/s", "cores": cores, "kind": "port",
            "sample": f"first {n} events of the same stream, {cores} key-group subtasks (oracle/fw_oracle.cpp), "
                      f"watermark every {C['batch']} events, final MAX_WATERMARK; {fired} windows fired"}, (fired, csum)


def sample_check(cfg, C, n, dev, want):
    """A fresh GPU engine over the cpu_baseline sample with the oracle job's watermarks (after every batch: the
    largest timestamp so far - lag; then MAX_WATERMARK): the number of results it fires (window fires and
    per-element late fires) and the wrapping sum of their sums (counts for doubles) equal the oracle's."""
    keys, ts, vals = stream(0, n, C["keys"], C["rate"], T0, device=dev, value_type=C["reduce"][1], zipf=C["zipf"],
                            ooo=C["ooo"])
    eng = WindowEngine(cfg)
    b = C["batch"]
    fired, csum, mask = 0, 0, (1 << 64) - 1
    col = "sum_i64" if C["reduce"][1] == "i64" else "count"

    def take(r):
        nonlocal fired, csum
        fired += int(r["n"])
        if r["n"]:
            csum = (csum + int(r[col].astype(np.uint64).sum(dtype=np.uint64))) & mask
    max_ts = LONG_MIN
    for s in range(0, n, b):
        k, t, v = keys[s:s + b], ts[s:s + b], vals[s:s + b]
        max_ts = max(max_ts, int(t.max().item()))
        eng.push(k, t, v)
        eng.advance_watermark(max_ts - C["wm_lag"])
        take(eng.collect())
    eng.advance_watermark(LONG_MAX)
    take(eng.collect())
    eng.close()
    o_fired, o_csum = want
    ok = fired == o_fired and csum == (o_csum & mask)
    return ("ok" if ok else "MISMATCH"), {"events": n, "fired": fired, "fired_oracle": o_fired,
                                          "checksum_equal": csum == (o_csum & mask)}


def pmc_traffic(config="c1"):
    """HBM bytes per launch of every engine kernel from the committed rocprofv3 PMC summary of THIS
    library build (profiles/*_pmc.json, written by tools/summarize_profiles.py from separate FETCH_SIZE /
    WRITE_SIZE passes): ({kernel name: bytes}, file), or ({}, None) when no summary matches the library's md5."""
    import glob
    import hashlib
    lib = os.path.join(ROOT, "flink_amd", "lib", "libflink_window.so")
    md5 = hashlib.md5(open(lib, "rb").read()).hexdigest()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=os.path.getmtime, reverse=True):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if d.get("library_md5") != md5 or d.get("config", "c1") != config:   # this build, this workload
            continue
        return {n: k["hbm_bytes_corrected"] for n, k in d.get("kernels", {}).items()
                if k.get("hbm_bytes_corrected")}, os.path.basename(f)
    return {}, None


def traffic_of(pmc, short):
    for name, b in pmc.items():
        if f"::{short}" in name:
            return b
    return None


def main():
    args = parse()
    world, rank, local = dist_init(args)
    dev = torch.device("cuda", local)
    C = CONFIGS[args.config]
    n_keys, rate, batch, key_cap = C["keys"], C["rate"], C["batch"], C["key_cap"]
    fields, vt = C["reduce"]
    total_steps = args.warmup + args.steps + args.prof_steps + args.h2d_steps + args.decode_steps + 2 * args.drain_steps + 2

    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    mp = 128
    kg = compute_key_group_range_for_operator_index(mp, world, rank)
    if key_cap is None:   # this rank's key groups' share of the key space, with a margin for the hash spread
        key_cap = int(n_keys * (kg[1] - kg[0] + 1) / mp * 1.05) + 4096
    reduce_fn = ReduceFunction(fields, vt, keep_first_f1=True)
    if C["window"][0] == "tumbling":
        assigner = TumblingEventTimeWindows.of(C["window"][1])
        windows_per_record = 1
    else:
        assigner = SlidingEventTimeWindows.of(C["window"][1], C["window"][2])
        windows_per_record = C["window"][1] // C["window"][2]
    windows_in_run = (total_steps * batch * world) // rate + 2
    per_window = min(key_cap, rate // max(world, 1) * (C["window"][1] // 1000 or 1))   # panes of a rank per window
    out_cap = windows_in_run * windows_per_record * per_window * 2 + 4096
    if C["lateness"]:
        out_cap += total_steps * batch // 4
    cfg = make_config(assigner, reduce_fn, allowed_lateness=C["lateness"], max_parallelism=mp, key_group_range=kg,
                      device=local, key_capacity=key_cap, max_batch=batch * (2 if world > 1 or args.force_exchange else 1),
                      out_capacity=int(min(out_cap, 1 << 29)), ingest_mode=args.ingest_mode)
    eng = WindowEngine(cfg)

    # resident synthetic input: rank r is source subtask r; its i-th event is global index i*world + r
    # (the interleaving keeps event time aligned across sources)
    cols = []
    for j in range(args.warmup + args.steps + args.prof_steps):
        k, t, v = stream(j * batch * world, batch * world, n_keys, rate, T0, device=dev, value_type=vt,
                         zipf=C["zipf"], ooo=C["ooo"])
        if world > 1:
            k, t, v = k[rank::world].contiguous(), t[rank::world].contiguous(), v[rank::world].contiguous()
        cols.append((k, t, v))
    torch.cuda.synchronize()

    exch = None
    if world > 1 or args.force_exchange:
        from flink_amd.keyby import KeyByExchange
        exch = KeyByExchange(eng, world, rank, mp, batch, dev)

    def wm_of(j):
        # source watermark after batch j: max ts seen - lag (BoundedOutOfOrdernessTimestampExtractor)
        return int(T0 + (((j + 1) * batch * world - 1) * 1000) // rate) - C["wm_lag"]

    def step(j, k, t, v):
        if exch is None:
            eng.push(k, t, v)
            eng.advance_watermark(wm_of(j))
        else:
            exch.step(k, t, v, wm_of(j))

    def drain():
        if exch is not None:
            exch.flush()   # the pipelined exchange's outstanding batches

    # the warm-up's results are collected to the host before its last step, so the timed region does not start
    # from a device left idle through that copy (the device clocks down while idle: a 20-step region lost ~10 us
    # per step to its first steps, round 6)
    collected = []
    for j in range(args.warmup):
        if j == args.warmup - 1:
            drain()
            eng.sync()
            collected.append(eng.collect())
        step(j, *cols[j])
    drain()
    eng.sync()
    torch.cuda.synchronize()
    st0 = eng.stats()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        step(j, *cols[j])
    drain()
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (host-bound if close to dt)
    torch.cuda.synchronize()      # device-wide: covers the engine's own streams
    barrier(world)
    dt = time.perf_counter() - t0
    st1 = eng.stats()
    fired_per_step = (st1["panes_fired"] - st0["panes_fired"]) / args.steps
    collected.append(eng.collect())

    # per-kernel device time on the continuation of the same stream (untimed)
    eng.lib.fw_set_profiling(eng.h, 1)
    eng.lib.fw_get_profile(eng.h, _abi.FwProfile())  # reset counters
    j0 = args.warmup + args.steps
    for j in range(j0, j0 + args.prof_steps):
        step(j, *cols[j])
        drain()
        eng.sync()   # isolate the kernels (no route/aggregate overlap across batches while timing them)
    prof = _abi.FwProfile()
    eng.lib.fw_get_profile(eng.h, prof)
    eng.lib.fw_set_profiling(eng.h, 0)
    eng.sync()
    collected.append(eng.collect())

    # PCIe-inclusive ingest: the same kind of batch pushed from pinned host columns (FW_MEM_HOST)
    h2d = None
    if args.h2d_steps > 0 and exch is None:
        j0 = args.warmup + args.steps + args.prof_steps
        host = []
        for j in range(j0, j0 + args.h2d_steps):
            k, t, v = stream(j * batch, batch, n_keys, rate, T0, device=dev, value_type=vt, zipf=C["zipf"], ooo=C["ooo"])
            host.append(tuple(x.cpu().pin_memory() for x in (k, t, v)))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for j, (k, t, v) in enumerate(host):
            eng.push(k, t, v)
            eng.advance_watermark(wm_of(j0 + j))
        eng.sync()
        dth = time.perf_counter() - t1
        h2d = {"value": args.h2d_steps * batch / dth, "unit": "events/s", "steps": args.h2d_steps,
               "note": "pinned host key/ts/value columns -> fw_push_batch(FW_MEM_HOST): hipMemcpyAsync to HBM, then "
                       "the same kernels; PCIe-inclusive, never the headline value"}
        collected.append(eng.collect())

    # wire-format ingest: the batch as Flink network bytes (length-prefixed StreamElementSerializer records of
    # Tuple3<Long key, Long f1, Long value> with timestamps), resident in HBM, decoded by fw_decode
    dec = None
    dec_sums = []   # value sums / record counts of batches pushed outside `cols` (checksum below)
    extra_n = 0
    if args.decode_steps > 0 and exch is None and vt == "i64":
        k, t, v = cols[0]
        n = k.numel()
        be = lambda x: x.view(torch.uint8).view(n, 8).flip(1)
        head = torch.tensor([0, 0, 0, 33, 0], dtype=torch.uint8, device=dev).expand(n, 5)   # length 33, tag 0
        wire = torch.cat([head, be(t), be(k), be(t), be(v)], dim=1).reshape(-1).contiguous()
        out = eng.decode(wire, ["long", "long", "long"], key=0, f1=1, value=2, record_cap=n, device=True)
        ok = out["n_records"] == n and bool(torch.equal(out["key"], k)) and bool(torch.equal(out["value"], v))
        fields3 = ["long", "long", "long"]
        bufs = [out["buffers"], eng.decode(wire, fields3, key=0, f1=1, value=2, record_cap=n, device=True)["buffers"]]
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(args.decode_steps):   # into the same output columns (allocated by the first call)
            eng.decode(wire, fields3, key=0, f1=1, value=2, record_cap=n, device=True, buffers=bufs[0])
        torch.cuda.synchronize()
        dts = (time.perf_counter() - t2) / args.decode_steps
        # fw_decode_begin / fw_decode_end: one buffer's count read-back overlaps the next buffer's kernels
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pend = []
        for q in range(args.decode_steps):
            pend.append(eng.decode_begin(wire, fields3, key=0, f1=1, value=2, record_cap=n, device=True, buffers=bufs[q % 2]))
            if len(pend) == 2:
                eng.decode_end(pend.pop(0))
        for h in pend:
            eng.decode_end(h)
        torch.cuda.synchronize()
        dtd = (time.perf_counter() - t2) / args.decode_steps
        dec = {"value": n / dtd, "unit": "records/s", "GB_s_in": wire.numel() / dtd / 1e9, "bytes_per_record": 37,
               "check": "ok" if ok else "MISMATCH",
               "note": "fw_decode_begin / fw_decode_end of one batch of Flink wire bytes in HBM after another, two in "
                       "flight (counts read back behind the next batch's kernels); the window kernels not included",
               "sync": {"value": n / dts, "unit": "records/s", "GB_s_in": wire.numel() / dts / 1e9,
                        "note": "the host-synchronous fw_decode, one call after another"}}
        del bufs
        del wire, out
        # the drop-in path end to end: wire bytes in HBM -> fw_decode -> fw_push_batch of the decoded columns ->
        # the watermark, per step (fresh batches after everything above, so their windows are live)
        jd = args.warmup + args.steps + args.prof_steps + args.h2d_steps + 2
        wires = []
        for j in range(jd, jd + args.decode_steps):
            k, t, v = stream(j * batch, batch, n_keys, rate, T0, device=dev, value_type=vt, zipf=C["zipf"], ooo=C["ooo"])
            wires.append(torch.cat([head, be(t), be(k), be(t), be(v)], dim=1).reshape(-1).contiguous())
            dec_sums.append(int(v.sum().item()))   # these batches enter the window state too (checksum below)
            extra_n += int(k.numel())
        eng.sync()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        # fresh output columns per batch (the push reads them on the engine's route stream after it returns); batch
        # q + 1's decode is enqueued before batch q's counts are read back and its columns pushed
        nxt = eng.decode_begin(wires[0], fields3, key=0, f1=1, value=2, record_cap=n, device=True)
        for q in range(len(wires)):
            cur = nxt
            if q + 1 < len(wires):
                nxt = eng.decode_begin(wires[q + 1], fields3, key=0, f1=1, value=2, record_cap=n, device=True)
            o = eng.decode_end(cur)
            m = o["n_records"]
            eng.push(o["key"][:m], o["ts"][:m], o["value"][:m], f1=o["f1"][:m])
            eng.advance_watermark(wm_of(jd + q))
        eng.sync()
        torch.cuda.synchronize()
        dtw = (time.perf_counter() - t3) / args.decode_steps
        dec["decode_window"] = {"value": n / dtw, "unit": "events/s", "GB_s_in": wires[0].numel() / dtw / 1e9,
                                "note": "wire bytes in HBM -> fw_decode_begin/end -> fw_push_batch -> fw_advance_watermark "
                                        "per batch (the drop-in path from network buffers), the next batch's decode "
                                        "enqueued before this one's counts are read back"}
        collected.append(eng.collect())
        del wires

    # results drained as they fire, the way the reference's operator hands fired windows downstream: push +
    # watermark + an asynchronous drain (fw_collect_begin / fw_collect_end) every step, results of step j landing
    # in pinned host columns while step j + 1 runs (they need only precede watermark j downstream); and the same
    # with the synchronous fw_collect for comparison.  Fresh batches after the decode leg's
    drain_leg = None

    def _digest(r):   # read every drained value once, as an operator emitting them would (for the checksum below)
        d = {"n": r["n"]}
        for c in ("sum_i64", "count"):
            a = r.get(c)
            if a is not None:
                d[c] = np.array([a.view(np.uint64).sum(dtype=np.uint64)], np.uint64).view(np.int64)
        return d

    drained = []
    if args.drain_steps > 0 and exch is None:
        jr = args.warmup + args.steps + args.prof_steps + args.h2d_steps + 2 + args.decode_steps
        legs = {}
        for mode in ("async", "sync"):
            fresh = []
            for j in range(jr, jr + args.drain_steps):
                k, t, v = stream(j * batch, batch, n_keys, rate, T0, device=dev, value_type=vt, zipf=C["zipf"], ooo=C["ooo"])
                fresh.append((k, t, v))
                if vt == "i64":
                    dec_sums.append(int(v.sum().item()))
                extra_n += int(k.numel())
            if mode == "async":   # the drains' pinned host staging (three buffers) is allocated by their first use
                for _ in range(3):
                    collected.append(eng.collect_end(eng.collect_begin()))
            eng.sync()
            torch.cuda.synchronize()
            n_out = 0
            t4 = time.perf_counter()
            pend = []
            for q, (k, t, v) in enumerate(fresh):
                eng.push(k, t, v)
                eng.advance_watermark(wm_of(jr + q))
                if mode == "sync":
                    r = eng.collect()
                    n_out += r["n"]
                    collected.append(r)
                    continue
                if len(pend) == 3:   # three drains in flight: the oldest (two batches back) has landed by now
                    r = eng.collect_end(pend.pop(0), copy=False)   # the pinned columns, read in place
                    n_out += r["n"]
                    drained.append(_digest(r))
                pend.append(eng.collect_begin())
            for tk in pend:
                r = eng.collect_end(tk, copy=False)
                n_out += r["n"]
                drained.append(_digest(r))
            torch.cuda.synchronize()
            dtr = (time.perf_counter() - t4) / args.drain_steps
            legs[mode] = {"value": batch / dtr, "unit": "events/s", "steps": args.drain_steps, "results": n_out,
                          "ms_per_step": dtr * 1e3}
            jr += args.drain_steps
            del fresh
        drain_leg = dict(legs["async"])
        drain_leg["note"] = ("push + watermark + fw_collect_begin every step, fw_collect_end of the drain begun two steps "
                             "before (pinned host columns; results of watermark j land while batches j + 1, j + 2 run); the headline "
                             "leaves them in the device output log, drained after the timed region")
        drain_leg["sync"] = dict(legs["sync"], note="the same with the host-synchronous fw_collect after every step")

    if world > 1:
        import torch.distributed as dist
        t_all = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
        dt = float(t_all.item())

    # --- correctness property (untimed).  After MAX_WATERMARK every record has fired exactly once per
    # window: C1/C2 wrapping sum of fired sums = wrapping sum of all values pushed (checksum of
    # checksums); C3 sum of fired counts = windows per record x records
    check = "skipped"
    cpu_line, cpu_fired = None, None
    if rank == 0 and args.cpu_sample > 0:   # at every N: the CPU job on the host's cores, beside the GPU line
        cpu_line, cpu_fired = cpu_baseline(cfg, C, args.cpu_sample)
    if not args.no_check and C["lateness"] == 0:
        eng.advance_watermark(LONG_MAX)
        collected.append(eng.collect())
        pushed_cols = [c for c in cols] + ([] if h2d is None else [tuple(x for x in hc) for hc in host])
        if vt == "i64":
            mask = (1 << 64) - 1
            fired = int(np.concatenate([r["sum_i64"] for r in collected + drained]).astype(np.uint64).sum(dtype=np.uint64)) & mask
            pushed = 0
            for k, t, v in pushed_cols:
                pushed = (pushed + (int(v.sum().item()) & mask)) & mask      # int64 tensor sums wrap
            for x in dec_sums:
                pushed = (pushed + (x & mask)) & mask
        else:
            fired = int(np.concatenate([r["count"] for r in collected + drained]).sum())
            pushed = windows_per_record * (sum(int(k.numel()) for k, t, v in pushed_cols) + extra_n)
        if world > 1:
            import torch.distributed as dist
            signed = lambda x: x - (1 << 64) if x >= (1 << 63) else x
            x = torch.tensor([signed(fired), signed(pushed)], dtype=torch.int64, device=dev)
            dist.all_reduce(x)
            fired, pushed = int(x[0].item()) & ((1 << 64) - 1), int(x[1].item()) & ((1 << 64) - 1)
        check = "ok" if fired == pushed else "MISMATCH"

    stats = eng.stats()
    form = stats["ingest_form"]
    events = args.steps * batch * world
    value = events / dt
    ms_step = dt * 1e3 / args.steps

    def per(ph):
        n_ = prof.launches[ph]
        return (prof.ms[ph] / n_ if n_ else 0.0), n_
    route_ms, _ = per(_abi.FW_PHASE_INGEST)
    agg_ms, _ = per(_abi.FW_PHASE_AGGREGATE)
    wm_ms, wm_n = per(_abi.FW_PHASE_FIRE)
    late_ms, late_n = per(_abi.FW_PHASE_LATE)
    wm_per_step = wm_n / max(args.prof_steps, 1)
    # algorithmic bytes: 24 B per event (key, ts, value) + per fired pane 96 B (C3:
    # 112 B); at N > 1 the keyBy exchange sends each GPU's (N-1)/N share of its events to the other GPUs (21 B/event
    # at N = 8: SURVEY.md 8(e)), which the receivers write to HBM: B_alg = 24 N + 96 P_fired + 24 (N-1)/N N
    ev_gpu = batch
    xchg_step = 24.0 * ev_gpu * (world - 1) / world if world > 1 else 0.0
    alg_step = 24.0 * ev_gpu + C["pane_bytes"] * fired_per_step / max(world, 1) + xchg_step
    achieved = alg_step / (ms_step / 1e3) / 1e9
    pmc, pmc_src = pmc_traffic(args.config)
    kernels = {}
    names = ([("k_route", route_ms, 1.0), ("k_aggregate", agg_ms, 1.0)] if form == 2 else
             [("k_ingest_direct", route_ms, 1.0)])
    names.append(("k_watermark", wm_ms, wm_per_step))
    for name, ms, per_step in names:
        tr = traffic_of(pmc, name)
        kernels[name] = {"ms": ms, "launches_per_step": per_step,
                         "achieved_GBs": (24.0 * ev_gpu / (ms / 1e3) / 1e9) if ms and name != "k_watermark" else None,
                         "traffic_bytes_per_launch": tr}
        if kernels[name]["achieved_GBs"]:
            kernels[name]["frac"] = kernels[name]["achieved_GBs"] / HBM_PEAK_GBS
    if late_n:
        kernels["late_path"] = {"ms": late_ms, "launches_per_step": late_n / max(args.prof_steps, 1)}
    ingest = [n for n, _, _ in names if n != "k_watermark"]
    dom = max(ingest, key=lambda n: kernels[n]["ms"])
    traffic_step = None
    if pmc and all(kernels[n]["traffic_bytes_per_launch"] for n in ingest):
        traffic_step = sum(kernels[n]["traffic_bytes_per_launch"] * kernels[n]["launches_per_step"] for n in kernels
                           if kernels[n].get("traffic_bytes_per_launch"))
    line = {
        "metric": "events/sec (whole node) keyed 1s tumbling sum; % of HBM roofline",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64" if vt == "i64" else "f64",
        "data": "synthetic (splitmix64 counter stream, SURVEY.md §8d), resident in HBM",
        "config": {"workload": f"{args.config}: {C['desc']}, {n_keys} keys, {rate} events/s event time, "
                               f"watermark every {batch} events per source",
                   "batch_per_gpu": batch, "keys": n_keys, "max_parallelism": mp, "parallelism": f"kg{world}",
                   "reduce": f"{'/'.join(fields)} over {vt}, f1 = first arrival"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_step,
                     "scope": "whole step: algorithmic bytes of one batch (24 B/event + pane bytes x fired panes) "
                              "over ms_per_step, every kernel and gap included",
                     "algorithmic_bytes_per_step": alg_step, "fired_panes_per_step": fired_per_step,
                     "traffic_unit": "HBM bytes per step: sum over kernels of PMC bytes per launch (FETCH_SIZE x2 + "
                                     "WRITE_SIZE, rocprofv3 --pmc) x launches per step",
                     "traffic_ratio": (traffic_step / alg_step) if traffic_step else None,
                     "traffic_source": pmc_src,
                     "dominant_kernel": dom, "kernels": kernels,
                     "device_time_source": f"HIP events around each kernel on its stream, {args.prof_steps} "
                                           "batches after the timed region, one batch at a time"},
        "check": check,
        "stats": {k: stats[k] for k in ("records_in", "records_late", "panes_fired", "late_fires", "ingest_form")},
        "host_enqueue_ms_per_step": t_enq * 1e3 / args.steps,
    }
    if world > 1:
        # xGMI: the sent share over the point-to-point links to the other N-1 GPUs (7 x ~153 GB/s per GPU at N = 8,
        # SURVEY.md 8(e)); the bound of C5
        peak_x = 153.0 * min(world - 1, 7)
        got_x = xchg_step / (ms_step / 1e3) / 1e9
        line["xgmi"] = {"bytes_sent_per_step": xchg_step, "achieved": got_x, "peak": peak_x, "unit": "GB/s",
                        "frac": got_x / peak_x, "links": min(world - 1, 7),
                        "note": "keyBy exchange payload (24 B x the (N-1)/N share of a rank's events) over ms_per_step"}
    if h2d is not None:
        line["h2d_ingest"] = h2d
    if dec is not None:
        line["wire_decode"] = dec
    if drain_leg is not None:
        line["with_drain"] = drain_leg
    if cpu_line is not None:
        line["cpu_baseline"] = cpu_line
    eng.close()
    # allowed lateness: results are per-element fires and late drops, so the checksum above does not apply; the GPU
    # is checked against the oracle on the cpu_baseline sample instead (a fresh engine, the oracle job's watermarks)
    if not args.no_check and C["lateness"] > 0 and cpu_fired is not None and world == 1:
        check, detail = sample_check(cfg, C, args.cpu_sample, dev, cpu_fired)
        line["check"] = check
        line["check_detail"] = dict(detail, note="GPU vs oracle on the cpu_baseline sample: results fired (window and "
                                                 "per-element late fires) and the wrapping sum of their sums")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1 or args.force_exchange:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
