#!/bin/bash
# Round-5 A/B of engine builds on one box: C1 bench lines (driver's command shape) for each library given in
# LIBS (paths relative to the repo; "main" = flink_amd/lib/libflink_window.so) and optional env per variant.
# Usage: LIBS="main lib/v8" CFG=c1 bash tools/r5_ab.sh
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
CFG=${CFG:-c1}
ARGS=${AB_ARGS:-"--steps 20 --warmup 5 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0 --config $CFG"}
for rep in ${REPS:-1 2}; do
  for v in ${LIBS:-main}; do
    envs=""; lib=$v
    case $v in *=*) envs=${v#*:}; lib=${v%%:*};; esac
    [ "$lib" = main ] && path=flink_amd/lib/libflink_window.so || path=flink_amd/$lib/libflink_window.so
    tag=$(echo $v | tr '/:=' '___')_$rep
    env $envs FW_LIBRARY=$REPO/$path timeout -k 10 180 python3 bench.py $ARGS > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python3 - gpurun_out/ab_$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print("%-28s Gev/s %6.2f  us/step %6.1f  frac %.3f  check %s  " % (sys.argv[2], d["value"] / 1e9, d["ms_per_step"] * 1e3,
      d["roofline"]["frac"], d["check"]), " ".join("%s %.1f" % (n, v["ms"] * 1e3) for n, v in k.items()), flush=True)
PY
  done
done
