#!/bin/bash
# Round-6 baseline on one box: a parity test, the C1 lean microbenchmark, engine phase stamps, C1 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step armtest 300 python -u -m pytest tests/test_armed_compaction.py -x -v --timeout 120 --timeout-method thread
step c1_mb 240 tools/microbench/bin/c1_mb serial
step stamps 240 python3 tools/stamps.py
step bench_c1 240 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0
step bench_c1b 240 python3 bench.py --steps 64 --warmup 8 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0
