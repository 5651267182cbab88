"""Turn rocprofv3 outputs under gpurun_out/ into committed summaries under profiles/.

Writes profiles/<tag>_kernel_stats.csv (the --kernel-trace --stats summary), and
profiles/<tag>_pmc.json: per-kernel FETCH_SIZE / WRITE_SIZE per dispatch (KB as reported) and the
HBM traffic per ingest launch, corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE reads half
of a wide coalesced stream on gfx950: doubled; WRITE_SIZE exact), keyed by the md5 of the library.
"""
import csv
import collections
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(tag):
    os.makedirs(PROF, exist_ok=True)
    pre = os.environ.get("PROF_SRC", "prof")   # gpurun_out/<pre>_trace, <pre>_fetch, <pre>_write, <pre>_md5.txt
    src = os.path.join(OUT, f"{pre}_trace", "run_kernel_stats.csv")
    if os.path.exists(src):
        shutil.copy(src, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    lib = os.path.join(ROOT, "flink_amd", "lib", "libflink_window.so")
    md5 = hashlib.md5(open(lib, "rb").read()).hexdigest()
    ran = open(os.path.join(OUT, f"{pre}_md5.txt")).read().strip()
    if ran != md5:
        sys.exit(f"gpurun_out/prof_* was measured on library {ran}, not the in-tree {md5}: re-run the profile")
    res = {"library_md5": md5, "config": os.environ.get("PROF_CONFIG", "c1"),   # the bench config profiled
           "units": "KB per dispatch as reported by rocprofv3", "kernels": {}}
    f = os.path.join(OUT, f"{pre}_fetch", "run_counter_collection.csv")
    w = os.path.join(OUT, f"{pre}_write", "run_counter_collection.csv")
    if os.path.exists(f) and os.path.exists(w):
        fetch, write = per_kernel(f, "FETCH_SIZE"), per_kernel(w, "WRITE_SIZE")
        ingest_bytes = 0.0
        for k in sorted(set(fetch) | set(write)):
            if "fw::" not in k:
                continue
            fb, wb = fetch.get(k, 0.0), write.get(k, 0.0)
            res["kernels"][k] = {"FETCH_SIZE_KB": fb, "WRITE_SIZE_KB": wb,
                                 "hbm_bytes_corrected": (2 * fb + wb) * 1024}
            if any(x in k for x in ("k_route", "k_aggregate", "k_ingest_direct")):
                ingest_bytes += (2 * fb + wb) * 1024
        res["ingest_traffic_bytes_per_launch"] = ingest_bytes
        res["correction"] = "FETCH_SIZE x2 (gfx950 reads half of a wide coalesced stream), WRITE_SIZE x1"
    json.dump(res, open(os.path.join(PROF, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(res, indent=1)[:2000])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
