cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/eor_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/eor_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/eor_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/eor_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/eor_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/eor_bench.log; exit $rc
