cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_session_hot.py tests/test_gpu_session.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sess_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sess_t.log; [ $rc -eq 0 ] || exit $rc
for h in 0 256; do
FW_SESS_HOT=$h timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_u_$h.log 2>&1 || exit $?; tail -1 gpurun_out/sess_u_$h.log | cut -c1-150
FW_SESS_HOT=$h SB_ZIPF=1.2 timeout -k 10 200 python tools/session_bench.py > gpurun_out/sess_z_$h.log 2>&1 || exit $?; tail -1 gpurun_out/sess_z_$h.log | cut -c1-150
done
