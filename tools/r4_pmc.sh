#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, no trace domains): MODE = ingest mode, CFG = config
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
A="--config ${CFG:-c1} --steps 6 --warmup 2 --prof-steps 0 --cpu-sample 0 --no-check --decode-steps 0 --h2d-steps 0 --drain-steps 0 --ingest-mode ${MODE:-0}"
i=0
for pass in ${PASSES:-FETCH_SIZE WRITE_SIZE}; do ctrs="${pass//_SQ_/ SQ_}"; ctrs="${ctrs//_TCC_/ TCC_}";
  i=$((i+1)); rm -rf gpurun_out/pmc_$i
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_$i -o run -- python3 bench.py $A > gpurun_out/pmc_$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/pmc_*/")):
    f = glob.glob(d + "**/*counter_collection*.csv", recursive=True)
    if not f: continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "fw::" in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()): print(d, k, len(v), round(sum(v) / len(v), 1))
PY
