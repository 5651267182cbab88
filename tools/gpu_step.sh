# ad-hoc GPU step used while iterating (parity subset + bench configs); every step under its own limit
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$TESTS" ] && step parity 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"}
[ "$CONFIGS" = none ] || for c in ${CONFIGS:-c1}; do step bench_$c 300 python bench.py --config $c --cpu-sample 0 --decode-steps 0 --h2d-steps 0 ${BENCH_ARGS}; done
exit 0
