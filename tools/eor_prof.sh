# round-end measurement: rocprofv3 trace + PMC passes (tools/profile_round.sh), then the bench lines of every
# config; each GPU step under its own limit, stopping at the first failure
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/profile_round.sh || exit $?
for c in ${CONFIGS:-c1 c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c ${BENCH_ARGS} > gpurun_out/eor_bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; tail -c 400 gpurun_out/eor_bench_$c.log; echo; [ $rc -eq 0 ] || exit $rc
done
