#!/bin/bash
# Round-6 same-box A/B of the session bench (tools/session_bench.py): the in-tree library against
# flink_amd/lib/sessbase (the sources before the session-checkpoint bookkeeping), uniform and Zipf(1.2) keys
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in ${SB_LIBS:-main sessbase}; do
    envl=""; case $lib in main) path=flink_amd/lib/libflink_window.so;; nockpt) path=flink_amd/lib/libflink_window.so; envl="FW_SESS_CKPT=0";; *) path=flink_amd/lib/$lib/libflink_window.so;; esac
    for z in uniform zipf; do
      envz=""; [ "$z" = zipf ] && envz="SB_ZIPF=1.2"
      env $envz $envl FW_LIBRARY=$PWD/$path timeout -k 10 300 python3 tools/session_bench.py > gpurun_out/sess_${lib}_${z}_$rep.log 2>&1 || { echo "session bench $lib $z failed"; tail -5 gpurun_out/sess_${lib}_${z}_$rep.log; exit 1; }
      echo "$lib $z $rep $(grep -o '"value": [0-9.e+]*' gpurun_out/sess_${lib}_${z}_$rep.log | head -1)"
    done
  done
done
