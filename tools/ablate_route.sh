#!/bin/bash
# k_route / k_aggregate ablations (FW_DEBUG_AGG bits: 1 aggregate skips LDS work, 2 aggregate skips the
# fold, 4 route skips window math, 8 route resolves the slice once per wave); timing only
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
for d in ${DBGS:-0 1 2 4 8 12 15}; do
  FW_DEBUG_AGG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/abr_$d" -o run -- python3 bench.py --steps 8 --warmup 2 --cpu-sample 0 --no-check --ingest-mode 2 > gpurun_out/abr_$d.log 2>&1 || exit 1
  python3 - "$REPO/gpurun_out/abr_$d/run_kernel_stats.csv" $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_route' in r['Name'] or 'k_aggregate' in r['Name']: print(sys.argv[2], r['Name'][:30], int(float(r['AverageNs']))//1000, 'us')
PY
done
