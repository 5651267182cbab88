#!/bin/bash
# Round-6: per-kernel times of the session bench (uniform keys) for the in-tree library and flink_amd/lib/sessbase
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in main sessbase; do
  [ "$lib" = main ] && path=flink_amd/lib/libflink_window.so || path=flink_amd/lib/$lib/libflink_window.so
  rm -rf gpurun_out/sp_$lib
  FW_LIBRARY=$PWD/$path timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/sp_$lib" -o run -- python3 tools/session_bench.py > gpurun_out/sp_$lib.log 2>&1 || { echo "prof $lib failed"; tail -5 gpurun_out/sp_$lib.log; exit 1; }
  echo "== $lib"; f=$(ls gpurun_out/sp_$lib/*kernel_stats.csv | head -1); cut -d, -f1-4 "$f" | head -12
done
