#!/bin/bash
# Round-6 profiles at the in-tree library: per config a rocprofv3 kernel trace + stats of the bench (C1: 64 timed
# steps), then FETCH_SIZE and WRITE_SIZE in passes of their own (tools/profile_round.sh); outputs gpurun_out/p6<cfg>_*
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for c in ${CONFIGS:-c1 c2 c3 c4}; do
  steps=16; [ "$c" = c1 ] && steps=64
  PROF_ARGS="--config $c --steps $steps --warmup 8 --prof-steps 0 --cpu-sample 0 --no-check --decode-steps 0 --drain-steps 0 --h2d-steps 0" \
    T_PROF=240 tools/profile_round.sh || exit 1
  for x in trace fetch write; do rm -rf gpurun_out/p6${c}_$x; mv gpurun_out/prof_$x gpurun_out/p6${c}_$x; done
  for x in trace fetch write; do mv gpurun_out/prof_$x.log gpurun_out/p6${c}_$x.log; done
  cp gpurun_out/prof_md5.txt gpurun_out/p6${c}_md5.txt
  python3 tools/steady_stats.py gpurun_out/p6${c}_trace/run_kernel_trace.csv gpurun_out/p6${c}_steady.csv 8 > /dev/null
done
exit 0
