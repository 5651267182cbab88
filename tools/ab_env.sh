#!/bin/bash
# A/B of engine environment knobs on the default bench: ENVS="A=1 A=2 ..." (one bench line each, "-" = none)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for kv in ${ENVS}; do
  for rep in 1 2; do
    if [ "$kv" = "-" ]; then timeout -k 10 200 python bench.py --cpu-sample 0 --decode-steps 0 --h2d-steps 0 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1
    else env $kv timeout -k 10 200 python bench.py --cpu-sample 0 --decode-steps 0 --h2d-steps 0 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1; fi
    rc=$?; [ $rc -ne 0 ] && { echo "$kv rc=$rc"; tail -3 gpurun_out/ab.log; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$kv', round(d['value']/1e9,2), 'G ev/s', round(d['ms_per_step']*1000,1), 'us/step')"
  done
done
