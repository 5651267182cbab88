#!/bin/bash
# k_route / k_aggregate ablations under rocprofv3 kernel trace (stats only, no counters)
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
for d in 0 1 2; do
  FW_DEBUG_AGG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/abl_$d" -o run -- python3 bench.py --steps 8 --warmup 2 --cpu-sample 0 --no-check --ingest-mode 2 > gpurun_out/abl_$d.log 2>&1 || exit $?
  python3 - "$REPO/gpurun_out/abl_$d/run_kernel_stats.csv" $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fw::' in r['Name']: print(sys.argv[2], r['Name'][:48], r['Calls'], int(float(r['AverageNs']))//1000, 'us')
PY
done
