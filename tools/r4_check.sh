#!/bin/bash
# round 4: quick GPU checks of the current build (every GPU step under its own limit; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$TESTS" ] && step tests 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"}
for c in ${CONFIGS:-}; do step bench_$c 300 python bench.py --config $c ${BENCH_ARGS}; done

exit 0
