cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step fused_parity 400 python -u -m pytest tests/test_gpu_parity.py -k fused -x -q --timeout 120 --timeout-method thread
step c1geo 300 python -u -m pytest tests/test_gpu_bench_geometry.py -k "c1_bench_geometry and not partitioned" -x -q --timeout 200 --timeout-method thread
step bench_fused 200 python bench.py --steps 32 --warmup 8 --cpu-sample 0 --decode-steps 0 --h2d-steps 0
step bench_routed 200 python bench.py --steps 32 --warmup 8 --cpu-sample 0 --decode-steps 0 --h2d-steps 0 --ingest-mode 2
