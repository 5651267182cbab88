#!/bin/bash
# Round-6 same-box A/B: C1 bench lines (driver's command shape) alternating between libraries.
# LIBS="main base" (main = flink_amd/lib/libflink_window.so, X = flink_amd/lib/X/libflink_window.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFG=${CFG:-c1}
for rep in ${REPS:-1 2 3}; do
  for v in ${LIBS:-main base}; do
    lib=${v%%:*}; envs=""; [ "$lib" != "$v" ] && envs=${v#*:}   # "lib:VAR=value" runs lib with that variable set
    [ "$lib" = main ] && path=flink_amd/lib/libflink_window.so || path=flink_amd/lib/$lib/libflink_window.so
    v=$(echo "$v" | tr ':=/' '___')
    env $envs FW_LIBRARY=$PWD/$path timeout -k 10 180 python3 bench.py --config $CFG --steps ${STEPS:-20} --warmup 5 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0 > gpurun_out/ab_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/ab_${v}_$rep.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print("%-8s Gev/s %6.2f  us/step %6.1f  frac %.3f  check %s  enq %.1f " % (sys.argv[2], d["value"] / 1e9, d["ms_per_step"] * 1e3,
      d["roofline"]["frac"], d["check"], d["host_enqueue_ms_per_step"] * 1e3), " ".join("%s %.1f" % (n, v["ms"] * 1e3) for n, v in k.items()), flush=True)
PY
  done
done
