#!/bin/bash
# round 4: fused form (ingest_mode 3) parity + bench + stamps; every GPU step under its own limit, stop at the first failure
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-5} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
B="--cpu-sample 0 --decode-steps 0 --h2d-steps 0 --drain-steps 0"
step geo 300 python -u -m pytest tests/test_gpu_bench_geometry.py -k fused -x -q --timeout 240 --timeout-method thread
step bench_fu 200 python bench.py $B --ingest-mode 3 ${BENCH_EXTRA}
step stamps 200 python tools/fused_stamps.py
[ -n "$FULL" ] && step par 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_checkpoint.py tests/test_signed_zero_sum.py tests/test_checkpoint_flink.py -k "fused or 3" -x -q --timeout 240 --timeout-method thread
exit 0
