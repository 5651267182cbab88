#!/bin/bash
# A/B of FW_DEBUG_AGG knobs: a short bench run (throughput + per-kernel device times) and one
# FETCH_SIZE --pmc pass (no trace domains) per knob value.  Usage: KNOBS="0 32" bash tools/ab_knobs.sh
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
ARGS=${AB_ARGS:-"--steps 32 --warmup 4 --cpu-sample 0 --no-check"}
for d in ${KNOBS:-0 32}; do
  FW_DEBUG_AGG=$d timeout -k 10 180 python3 bench.py $ARGS > gpurun_out/ab_$d.log 2>&1 || { echo "bench $d failed"; tail -5 gpurun_out/ab_$d.log; exit 1; }
  python3 - gpurun_out/ab_$d.log $d <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("knob", sys.argv[2], "Gev/s %.2f" % (d["value"] / 1e9), "ms/step %.4f" % d["ms_per_step"], d["roofline"]["kernel_ms"])
PY
  if [ -z "$NO_PMC" ]; then
    FW_DEBUG_AGG=$d timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$REPO/gpurun_out/ab_fetch_$d" -o run -- python3 bench.py --steps 8 --warmup 2 --prof-steps 0 --cpu-sample 0 --no-check > gpurun_out/ab_fetch_$d.log 2>&1 || { echo "pmc $d failed"; exit 1; }
    python3 - "$REPO/gpurun_out/ab_fetch_$d/run_counter_collection.csv" $d <<'PY'
import csv, collections, sys
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "fw::" in r["Kernel_Name"]:
        agg[r["Kernel_Name"].split("(")[0][-28:]].append(float(r["Counter_Value"]))
print("knob", sys.argv[2], {k: round(sum(v) / len(v) / 1024, 1) for k, v in agg.items()}, "MB FETCH_SIZE per dispatch")
PY
  fi
done
