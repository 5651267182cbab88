# C4 A/B: owner dispatch order (FW_DEBUG_AGG=128 = plain order) and share size
set -e
mkdir -p gpurun_out
[ -n "$NOTESTS" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "zipf or hot_buckets" tests/test_gpu_bench_geometry.py > gpurun_out/ab_c4_tests.log 2>&1
[ -n "$NOTESTS" ] || tail -2 gpurun_out/ab_c4_tests.log
run() {   # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --config c4 --steps 64 --drain-steps 0 --decode-steps 0 --h2d-steps 0 --cpu-sample 0 --no-check > gpurun_out/ab_c4_$n.json 2>/dev/null
  python3 -c "import json; l=json.loads(open('gpurun_out/ab_c4_$n.json').read().strip().splitlines()[-1]); k=l['roofline']['kernels']; print('$n', round(l['value']/1e9,2), round(l['ms_per_step']*1e3,1), {a:round(b['ms']*1e3,1) for a,b in k.items()})"
}
# longest-share-first owner order (default) against the plain order, interleaved A-B-A-B
run lpt FW_DEBUG_AGG=0
run plain FW_DEBUG_AGG=128
run lpt_b FW_DEBUG_AGG=0
run plain_b FW_DEBUG_AGG=128
# share size
run lpt250 FW_DEBUG_AGG=0 FW_AGG_CHUNK_PCT=250
run lpt175 FW_DEBUG_AGG=0 FW_AGG_CHUNK_PCT=175
