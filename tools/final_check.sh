cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/profile_round.sh || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/final_tests.log; exit $rc
