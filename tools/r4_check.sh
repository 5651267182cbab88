#!/bin/bash
# round 4: quick GPU checks of the current build (every GPU step under its own limit; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$TESTS" ] && step tests 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"}
for c in ${CONFIGS:-}; do step bench_$c 300 python bench.py --config $c ${BENCH_ARGS}; done
[ -n "$FUSED" ] && step bench_fu 200 python bench.py --cpu-sample 0 --decode-steps 0 --h2d-steps 0 --drain-steps 0 --ingest-mode 3 && step stamps 200 python tools/fused_stamps.py
exit 0
