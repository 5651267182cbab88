#!/bin/bash
# A/B of FW_DEBUG_AGG ablation bits on the default bench (no check: ablations change results)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for d in ${DBG_LIST:-0 64 128 0}; do
  FW_DEBUG_AGG=$d timeout -k 10 120 python bench.py --cpu-sample 0 --no-check --h2d-steps 0 ${BENCH_ARGS} > gpurun_out/ab_$d.log 2>&1 || exit $?
  echo "dbg=$d $(tail -1 gpurun_out/ab_$d.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e9,1), 'Gev/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v['ms']*1e3,1) for k, v in r['kernels'].items()})")"
done
