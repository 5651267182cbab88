#!/bin/bash
# A/B of engine builds (FW_LIBRARY) on the default bench line; LIBS="a.so b.so"
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for lib in ${LIBS}; do
  FW_LIBRARY=$lib timeout -k 10 120 python bench.py --cpu-sample 0 --no-check --h2d-steps 0 --decode-steps 0 ${BENCH_ARGS} > gpurun_out/ab_lib.log 2>&1 || exit $?
  echo "$(basename $lib) $(tail -1 gpurun_out/ab_lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e9,1), 'Gev/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v['ms']*1e3,1) for k, v in r['kernels'].items()})")"
done
