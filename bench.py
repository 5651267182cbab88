#!/usr/bin/env python3
"""Benchmark: keyed 1 s tumbling event-time long-sum (BASELINE.json metric), events/s whole node.

Workload (SURVEY.md §8d, config C1 — BASELINE.json configs[1] asks for 10M keys on one GPU; the
metric itself is quoted on the C1 job, which is what this measures at N=1 unless --config c2):
  keyBy(0).window(TumblingEventTimeWindows.of(1 s)).reduce((a, b) -> Tuple3(a.f0, a.f1, a.f2 + b.f2))
  over Tuple3<Long key, Long ts, Long value>; 64K uniform keys; R = 2^24 events per event-time
  second; a punctuated watermark (max ts seen - 1) after every batch of 2^22 events.
A step = one batch of 2^22 events pushed through the engine + its watermark (fire/purge).
Inputs are generated on the GPU and resident in HBM before the timed region.

Multi-GPU (torchrun, one process per GPU): every rank is a source subtask producing its own 2^22
events per step (weak scaling); records are routed to the key-group owner (maxParallelism 128) by
the keyBy exchange (HIP partition kernel + RCCL all-to-all) and the watermark is the min over ranks.

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
from flink_amd.windowing import ReduceFunction, TumblingEventTimeWindows, WindowEngine, make_config  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
LONG_MAX = (1 << 63) - 1
T0 = 1_700_000_000_000     # epoch ms, aligned to the window size

CONFIGS = {
    # name: (n_keys, rate events/s of event time, batch, key_capacity)
    "c1": (1 << 16, 1 << 24, 1 << 22, 1 << 16),
    "c2": (10_000_000, 1 << 26, 1 << 22, 10_000_000),
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


def cpu_baseline(cfg, n_keys, rate, n):
    """The oracle as a p-subtask CPU job (key-group partitioned threads) on a bounded sample."""
    from oracle import oracle
    cores = min(16, len(os.sched_getaffinity(0)))
    keys, ts, vals = (t.numpy() for t in stream(0, n, n_keys, rate, T0, device="cpu"))
    oracle.load()
    t = time.perf_counter()
    fired, _ = oracle.run_parallel(cfg, cores, keys, ts, vals, 1 << 22, 1, LONG_MAX)
    dt = time.perf_counter() - t
    return {"value": n / dt, "unit": "events/s", "cores": cores, "kind": "port",
            "sample": f"first {n} events of the same stream, {cores} key-group subtasks (oracle/fw_oracle.cpp), "
                      f"watermark every 2^22 events, final MAX_WATERMARK; {fired} windows fired"}


def pmc_traffic(kernel):
    """HBM bytes per ingest launch from the committed rocprofv3 PMC summary of THIS library build
    (profiles/*_pmc.json, written by tools/summarize_profiles.py from separate FETCH_SIZE / WRITE_SIZE
    passes), or None when no summary matches the library's md5."""
    import glob
    import hashlib
    lib = os.path.join(ROOT, "flink_amd", "lib", "libflink_window.so")
    md5 = hashlib.md5(open(lib, "rb").read()).hexdigest()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=os.path.getmtime, reverse=True):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        if d.get("library_md5") != md5:
            continue
        for name, k in d.get("kernels", {}).items():
            if kernel in name and k.get("hbm_bytes_corrected"):
                return k["hbm_bytes_corrected"], os.path.basename(f)
    return None, None


def main():
    args = parse()
    world, rank, local = dist_init(args)
    dev = torch.device("cuda", local)
    n_keys, rate, batch, key_cap = CONFIGS[args.config]
    total_steps = args.warmup + args.steps + args.prof_steps

    from flink_amd.keygroups import compute_key_group_range_for_operator_index
    mp = 128
    kg = compute_key_group_range_for_operator_index(mp, world, rank)
    reduce_fn = ReduceFunction(("sum",), "i64", keep_first_f1=True)
    windows_in_run = (total_steps * batch * world) // rate + 2
    cfg = make_config(TumblingEventTimeWindows.of(1000), reduce_fn, max_parallelism=mp, key_group_range=kg,
                      device=local, key_capacity=key_cap, max_batch=batch * (2 if world > 1 or args.force_exchange else 1),
                      out_capacity=int(min(windows_in_run * key_cap // max(world, 1) * 2 + 4096, 1 << 27)),
                      ingest_mode=args.ingest_mode)
    eng = WindowEngine(cfg)

    # resident synthetic input: rank r is source subtask r; its i-th event is global index i*world + r
    # (the interleaving keeps event time aligned across sources)
    cols = []
    for j in range(total_steps):
        k, t, v = stream(j * batch * world, batch * world, n_keys, rate, T0, device=dev)
        if world > 1:
            k, t, v = k[rank::world].contiguous(), t[rank::world].contiguous(), v[rank::world].contiguous()
        cols.append((k, t, v))
    torch.cuda.synchronize()

    exch = None
    if world > 1 or args.force_exchange:
        from flink_amd.keyby import KeyByExchange
        exch = KeyByExchange(eng, world, rank, mp, batch, dev)

    def step(j):
        k, t, v = cols[j]
        wm_local = int(T0 + (((j + 1) * batch * world - 1) * 1000) // rate) - 1   # max ts seen - 1
        if exch is None:
            eng.push(k, t, v)
            eng.advance_watermark(wm_local)
        else:
            exch.step(k, t, v, wm_local)

    for j in range(args.warmup):
        step(j)
    eng.sync()
    torch.cuda.synchronize()
    warm_res = eng.collect()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        step(j)
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (host-bound if close to dt)
    torch.cuda.synchronize()      # device-wide: covers the engine's own streams
    barrier(world)
    dt = time.perf_counter() - t0

    # per-kernel device time on the continuation of the same stream (untimed)
    eng.lib.fw_set_profiling(eng.h, 1)
    eng.lib.fw_get_profile(eng.h, _abi.FwProfile())  # reset counters
    for j in range(args.warmup + args.steps, total_steps):
        step(j)
        eng.sync()   # isolate the kernels (no route/aggregate overlap across batches while timing them)
    prof = _abi.FwProfile()
    eng.lib.fw_get_profile(eng.h, prof)
    eng.lib.fw_set_profiling(eng.h, 0)
    eng.sync()

    if world > 1:
        import torch.distributed as dist
        t_all = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
        dt = float(t_all.item())

    # --- correctness property (untimed): after MAX_WATERMARK every record has fired exactly once,
    # so the wrapping sum of fired sums equals the wrapping sum of all values pushed (checksum of checksums)
    check = "skipped"
    if not args.no_check:
        mask = (1 << 64) - 1
        res = eng.collect()
        eng.advance_watermark(LONG_MAX)
        res2 = eng.collect()
        fired = int(np.concatenate([warm_res["sum_i64"], res["sum_i64"], res2["sum_i64"]]).astype(np.uint64).sum(dtype=np.uint64)) & mask
        pushed = 0
        for k, t, v in cols:
            pushed = (pushed + (int(v.sum().item()) & mask)) & mask      # int64 tensor sums wrap
        if world > 1:
            import torch.distributed as dist
            signed = lambda x: x - (1 << 64) if x >= (1 << 63) else x
            x = torch.tensor([signed(fired), signed(pushed)], dtype=torch.int64, device=dev)
            dist.all_reduce(x)
            fired, pushed = int(x[0].item()) & mask, int(x[1].item()) & mask
        check = "ok" if fired == pushed else "MISMATCH"

    form = eng.stats()["ingest_form"]
    events = args.steps * batch * world
    value = events / dt

    def per(ph):
        n_ = prof.launches[ph]
        return (prof.ms[ph] / n_ if n_ else 0.0), (prof.records[ph] / n_ if n_ else 0.0)
    route_ms, route_rec = per(_abi.FW_PHASE_INGEST)
    agg_ms, _ = per(_abi.FW_PHASE_AGGREGATE)
    wm_ms, _ = per(_abi.FW_PHASE_FIRE)
    # dominant kernel: the one taking the most device time per batch; its algorithmic bytes are SURVEY.md
    # 8(d)'s 24 B per event (key, ts, value int64) times the events one launch processes
    names = {"k_route": route_ms, "k_aggregate": agg_ms} if form == 2 else {"k_ingest_direct": route_ms}
    dom = max(names, key=names.get)
    dom_ms = names[dom]
    alg_bytes = 24.0 * route_rec
    achieved = alg_bytes / (dom_ms / 1e3) / 1e9 if dom_ms else 0.0
    path_ms = route_ms + agg_ms
    traffic, traffic_src = pmc_traffic(dom)
    line = {
        "metric": "events/sec (whole node) keyed 1s tumbling sum; % of HBM roofline",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (splitmix64 counter stream, SURVEY.md §8d), resident in HBM",
        "config": {"workload": f"{args.config}: tumbling 1s event-time long-sum, {n_keys} keys, "
                               f"{rate} events/s event time, watermark every {batch} events per source",
                   "batch_per_gpu": batch, "keys": n_keys, "max_parallelism": mp, "parallelism": f"kg{world}",
                   "reduce": "Tuple3(a.f0, a.f1, a.f2 + b.f2), f1 = first arrival"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 --pmc)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": alg_bytes, "bytes_per_event": 24,
                     "kernel_ms": {k: v for k, v in names.items()}, "watermark_ms": wm_ms,
                     "path_achieved": alg_bytes / (path_ms / 1e3) / 1e9 if path_ms else 0.0,
                     "path_note": "24 B/event over the summed device time of the ingest kernels of one batch",
                     "device_time_source": f"HIP events around each kernel on its stream, {args.prof_steps} "
                                           "batches after the timed region, one batch at a time"},
        "check": check,
        "host_enqueue_ms_per_step": t_enq * 1e3 / args.steps,
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        line["cpu_baseline"] = cpu_baseline(cfg, n_keys, rate, args.cpu_sample)
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1 or args.force_exchange:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
