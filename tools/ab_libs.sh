#!/bin/bash
# A/B of two builds of the engine library in one run: bench throughput, per-kernel device time and the
# host enqueue time per step.  Usage: LIB_B=flink_amd/lib/old/libflink_window.so bash tools/ab_libs.sh
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
ARGS=${AB_ARGS:-"--steps 64 --warmup 8 --cpu-sample 0 --no-check"}
for rep in 1 2; do
  for lib in flink_amd/lib/libflink_window.so ${LIB_B}; do
    tag=$(basename $(dirname $lib))_$rep
    FW_LIBRARY=$REPO/$lib timeout -k 10 180 python3 bench.py $ARGS > gpurun_out/abl_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/abl_$tag.log; exit 1; }
    python3 - gpurun_out/abl_$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "Gev/s %.2f" % (d["value"] / 1e9), "ms/step %.4f" % d["ms_per_step"],
      "enqueue ms/step %.4f" % d.get("host_enqueue_ms_per_step", -1), d["roofline"]["kernel_ms"])
PY
  done
done
