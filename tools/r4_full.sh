#!/bin/bash
# round 4: the whole GPU suite, then the bench lines of every single-GPU config (each step under its own limit)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-3} "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
md5sum flink_amd/lib/libflink_window.so > gpurun_out/full_md5.txt
[ -z "$NOTESTS" ] && step full_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for c in ${CONFIGS:-c1 c2 c3 c4}; do step full_bench_$c 300 python bench.py --config $c ${BENCH_ARGS}; done
exit 0
