#!/bin/bash
# Round-6 bench lines at the in-tree library (C1 with the driver's --steps 20 --warmup 5, three times, and 64 steps;
# C2-C4), each under its own limit
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
b() { local tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > gpurun_out/r6_bench_$tag.log 2>&1; local rc=$?; echo "bench $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2 3; do b c1_steps20_$r --steps 20 --warmup 5; done
b c1 --steps 64 --warmup 8
for c in c2 c3 c4; do b $c --config $c --steps 32 --warmup 8 --decode-steps 0 --drain-steps 0 --h2d-steps 0; done
exit 0
