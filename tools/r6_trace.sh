#!/bin/bash
# Round-6: rocprofv3 kernel traces of the C1 bench's timed region for each library in LIBS, then the timeline
# summary (per-kernel durations while pipelined, gaps, overlap).  Outputs under gpurun_out/tr_<lib>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${LIBS:-main base}; do
  [ "$v" = main ] && path=flink_amd/lib/libflink_window.so || path=flink_amd/lib/$v/libflink_window.so
  export FW_LIBRARY=$PWD/$path
  rm -rf gpurun_out/tr_$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/tr_$v" -o run -- python3 bench.py --config ${CFG:-c1} --steps ${STEPS:-64} --warmup 8 --prof-steps 0 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0 > gpurun_out/tr_$v.log 2>&1 || { echo "trace $v failed"; tail -5 gpurun_out/tr_$v.log; exit 1; }
  f=$(ls gpurun_out/tr_$v/*kernel_trace.csv | head -1)
  echo "== $v"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr_$v.log; python3 tools/timeline.py "$f" 40 | tail -12
done
