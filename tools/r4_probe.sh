#!/bin/bash
# round 4 probe: C1 default + fused bench lines, then FETCH_SIZE / WRITE_SIZE passes of the fused form
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--cpu-sample 0 --decode-steps 0 --h2d-steps 0 --drain-steps 0 --no-check"
timeout -k 10 200 python bench.py $B > gpurun_out/p_c1.log 2>&1 || { echo c1 fail; tail gpurun_out/p_c1.log; exit 1; }
tail -1 gpurun_out/p_c1.log | cut -c1-300
timeout -k 10 200 python bench.py $B --ingest-mode 3 > gpurun_out/p_fu.log 2>&1 || { echo fu fail; tail gpurun_out/p_fu.log; exit 1; }
tail -1 gpurun_out/p_fu.log | cut -c1-300
A="--steps 8 --warmup 2 --prof-steps 0 $B --ingest-mode 3"
rm -rf gpurun_out/pf_fetch gpurun_out/pf_write
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf_fetch -o run -- python3 bench.py $A > gpurun_out/pf_fetch.log 2>&1 || { echo fetch fail; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pf_write -o run -- python3 bench.py $A > gpurun_out/pf_write.log 2>&1 || { echo write fail; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pf_fetch", "gpurun_out/pf_write"):
    f = glob.glob(d + "/**/*counter_collection*.csv", recursive=True)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "fw::" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in agg.items(): print(d, k, len(v), sum(v) / len(v))
PY
