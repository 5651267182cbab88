#!/bin/bash
# GPU session: parity tests, smoke, bench of the XCD-private and partitioned ingest forms, XCD microbench.
# Every GPU step has its own time limit; the script stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
[ -z "$SKIP_TESTS" ] && run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS}
[ -z "$SKIP_SMOKE" ] && run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench_xcd 300 python bench.py --ingest-mode 3 ${BENCH_ARGS}
[ -z "$SKIP_ROUTED" ] && run bench_routed 300 python bench.py --ingest-mode 2 --cpu-sample 0 ${BENCH_ARGS}
[ -n "$MB" ] && run xcd_mb 200 ./tools/microbench/xcd_mb
exit 0
