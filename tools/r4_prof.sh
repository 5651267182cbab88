#!/bin/bash
# kernel trace of a short bench run: NAME = output tag, BENCH_ARGS = bench.py arguments; prints the per-kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
n=${NAME:-prof}; rm -rf gpurun_out/$n
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$n -o run -- python3 bench.py ${BENCH_ARGS} > gpurun_out/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/$n.log; exit 1; }
f=$(find gpurun_out/$n -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:20]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us')
PY
