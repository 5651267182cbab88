#!/bin/bash
# One bench line per config (c1 default run incl. the CPU baseline; c2-c4 short), each under its own limit
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py ${C1_ARGS} > gpurun_out/bench_c1.log 2>&1 || { echo "c1 rc=$?"; tail -3 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c --steps 32 --warmup 4 --cpu-sample 0 > gpurun_out/bench_$c.log 2>&1 || { echo "$c rc=$?"; tail -3 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', round(d['value']/1e9,2), 'Gev/s', round(d['ms_per_step']*1e3,1), 'us/step frac', round(r['frac'],3), {k: round(v['ms']*1e3,1) for k, v in r['kernels'].items()}, d['check'], d.get('h2d_ingest',{}).get('value'))"
done
