# decode A/B: wire-decode tests and the bench's decode leg for each library given (FW_LIBRARY)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  FW_LIBRARY=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_wire_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dect_$tag.log 2>&1 || { echo "tests $tag failed"; tail -20 gpurun_out/dect_$tag.log; exit 1; }
  FW_LIBRARY=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_dec_$tag -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-sample 0 --decode-steps 8 --h2d-steps 0 --prof-steps 0 > gpurun_out/dec_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/dec_$tag.log; exit 1; }
  echo "== $tag: $(tail -1 gpurun_out/dect_$tag.log)"; grep -o "\"wire_decode\": {[^}]*}" gpurun_out/dec_$tag.log | cut -c1-120
  grep dec_ gpurun_out/prof_dec_$tag/run_kernel_stats.csv | cut -d, -f1,4 | cut -c1-90
done
