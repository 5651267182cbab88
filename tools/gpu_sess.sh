cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_session_hot.py tests/test_gpu_session.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sess_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sess_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_u.log 2>&1 || exit $?; tail -1 gpurun_out/sess_u.log
SB_ZIPF=1.2 timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_z.log 2>&1 || exit $?; tail -1 gpurun_out/sess_z.log
