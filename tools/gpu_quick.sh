#!/bin/bash
# GPU iteration: parity tests, one bench line, phase stamps (each step under its own limit)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e9, 'Gev/s', d['ms_per_step'], 'ms/step', d['roofline']['kernel_ms'], d['roofline']['watermark_ms'], d['check'])"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log | tail -6
exit $rc
