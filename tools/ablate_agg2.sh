#!/bin/bash
# k_aggregate ablations (FW_DEBUG_AGG: 1 = loads only, 2 = LDS work only on synthetic records); timing only
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for d in ${DBGS:-0 1 2}; do
  FW_DEBUG_AGG=$d timeout -k 10 120 python bench.py --steps 16 --warmup 4 --cpu-sample 0 --no-check > gpurun_out/abl_$d.log 2>&1 || exit $?
  echo "dbg=$d $(tail -1 gpurun_out/abl_$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'])")"
done
