#!/bin/bash
# GPU iteration: parity tests, then one bench line (each step under its own limit; stop at the first
# fault / abort / timeout).  PYTEST_ARGS / BENCH_ARGS / SKIP_TESTS / SKIP_BENCH tune it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${T_TEST:-500} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 ${T_BENCH:-300} python bench.py --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
  exit $rc
fi
