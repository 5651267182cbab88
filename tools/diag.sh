cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/diag -o run -- python3 bench.py --steps 16 --warmup 4 --prof-steps 0 --cpu-sample 0 --no-check > gpurun_out/diag.log 2>&1
rc=$?; tail -14 gpurun_out/stamps.log; exit $rc
