#!/bin/bash
# GPU: parity tests + C1 bench (auto form) + C2 (10M keys) bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in c1 c2; do
  timeout -k 10 300 python bench.py --config $cfg --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -1 gpurun_out/bench_$cfg.log | cut -c1-300
  tail -1 gpurun_out/bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['roofline']['watermark_ms'], d['check'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
