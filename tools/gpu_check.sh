#!/bin/bash
# GPU check: parity tests, smoke, default bench line (+ extra configs in BENCH_CONFIGS).  Each step runs under
# its own limit; the script stops at the first fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
step() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu ${T_TEST:-600} python -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS}
[ -z "$SKIP_SMOKE" ] && step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
[ -z "$SKIP_BENCH" ] && step bench 300 python bench.py ${BENCH_ARGS}
for c in ${BENCH_CONFIGS}; do step bench_$c 300 python bench.py --config $c --cpu-sample 0; done
if [ -n "$TRACE" ]; then
  export TMPDIR=/tmp; rm -rf gpurun_out/prof_trace
  md5sum flink_amd/lib/libflink_window.so | cut -d' ' -f1 > gpurun_out/prof_md5.txt
  step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_trace" -o run -- python3 bench.py --steps 16 --warmup 4 --prof-steps 0 --cpu-sample 0 --no-check --decode-steps 0 --h2d-steps 0 ${TRACE_ARGS}
fi
exit 0
