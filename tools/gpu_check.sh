cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/eor_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/eor_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_u.log 2>&1 || exit $?; tail -1 gpurun_out/sess_u.log
SB_ZIPF=1.2 timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_z.log 2>&1 || exit $?; tail -1 gpurun_out/sess_z.log
timeout -k 10 300 python bench.py --cpu-sample 0 --decode-steps 0 --h2d-steps 0 > gpurun_out/drain_c1.log 2>&1 || exit $?; tail -c 420 gpurun_out/drain_c1.log
