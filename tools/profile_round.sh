#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (MI355X_MICROARCH.md §HBM: never mix --pmc with trace domains).  Outputs under
# gpurun_out/prof_*; copy the summaries to profiles/.
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$REPO"
ARGS=${PROF_ARGS:-"--steps 16 --warmup 4 --prof-steps 0 --cpu-sample 0 --no-check"}
export TMPDIR=/tmp
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write
md5sum flink_amd/lib/libflink_window.so | cut -d' ' -f1 > gpurun_out/prof_md5.txt
timeout -k 10 ${T_PROF:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_trace" -o run -- python3 bench.py $ARGS > gpurun_out/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 gpurun_out/prof_trace.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$NO_PMC" ]; then exit 0; fi
timeout -k 10 ${T_PROF:-300} rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$REPO/gpurun_out/prof_fetch" -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; tail -2 gpurun_out/prof_fetch.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 ${T_PROF:-300} rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$REPO/gpurun_out/prof_write" -o run -- python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1
rc=$?; echo "write rc=$rc"; tail -2 gpurun_out/prof_write.log
exit $rc
