#!/bin/bash
# Round-6 iteration on one box: optional parity tests (TESTS), engine phase stamps, C1 bench lines (driver's shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$TESTS" ] && step tests 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread ${TEST_K:+-k "$TEST_K"}
[ -z "$NOSTAMPS" ] && step stamps 240 python3 tools/stamps.py
[ "$CONFIGS" = none ] || for c in ${CONFIGS:-c1}; do
  for rep in ${REPS:-1}; do
    step bench_${c}_$rep 240 python3 bench.py --config $c --steps ${STEPS:-20} --warmup 5 --cpu-sample 0 --decode-steps 0 --drain-steps 0 --h2d-steps 0
    python3 - gpurun_out/bench_${c}_$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print("RESULT Gev/s %6.2f  us/step %6.1f  frac %.3f  check %s  enq %.1f us " % (d["value"] / 1e9, d["ms_per_step"] * 1e3,
      d["roofline"]["frac"], d["check"], d["host_enqueue_ms_per_step"] * 1e3), " ".join("%s %.1f" % (n, v["ms"] * 1e3) for n, v in k.items()))
PY
  done
done
exit 0
